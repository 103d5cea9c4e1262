#!/bin/bash
# One parameterised GPU runner (replaces round 1-2's one-off gpu_*.sh).
# Each argument is a step "KIND:NAME:ARGS", run in order on the GPU box from
# the repo root, each under its own time limit; the first failure ends the run
# (after a fault, an abort or a time limit nothing more touches the GPU).
#   pytest:NAME:ARGS   python -m pytest ARGS        -> gpurun_out/pytest_NAME.log
#   bench:NAME:ARGS    python bench.py ARGS          -> gpurun_out/bench_NAME.json (+ .err)
#   prof:NAME:ARGS     rocprofv3 kernel trace + stats of bench.py ARGS -> gpurun_out/prof_NAME/
#   pmc:NAME:CTR:ARGS  one rocprofv3 --pmc pass (CTR) of bench.py ARGS -> gpurun_out/pmc_NAME/
#   py:NAME:ARGS       python ARGS                   -> gpurun_out/py_NAME.log
#   smoke:NAME:        __graft_entry__.smoke()       -> gpurun_out/smoke_NAME.log
#   ab:NAME:VARIANTS   config-3 pivots/s of each variant ("[LIB] [NAME=VALUE ...]", ';'-separated),
#                      interleaved twice (tools/sweep_exp.py) -> gpurun_out/ab_NAME.log
#   run:NAME:CMD       any other command (lab binaries such as tools/flush_lab,
#                      env-var sweeps: "run:x:env LPG_DEFER=32 python bench.py")
#                                                    -> gpurun_out/run_NAME.log
# Limits: T_PYTEST (900 s), T_BENCH (300 s), T_PY (300 s).
# Profiles: "prof:c3:--steps 2 --warmup 0 --no-cpu", then one pmc step per
# counter group, e.g. "pmc:fetch:FETCH_SIZE:--steps 2 --warmup 0 --no-cpu".
# KIND@VAR=VAL,VAR2=VAL:NAME:ARGS exports those variables for that step only
# (e.g. "pmc@LPG_FLUSH_XCD=0:fetch0:FETCH_SIZE:--steps 2 --warmup 0 --no-cpu").
# Example: gpurun --timeout 1200 -- bash tools/gpu.sh "pytest:all:tests -m gpu -x -q" "bench:c3:--steps 20"
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run_step() {
    case $kind in
        pytest)
            timeout -k 10 "${T_PYTEST:-900}" python -u -m pytest $args -p no:cacheprovider --timeout 300 \
                --timeout-method thread > "gpurun_out/pytest_$name.log" 2>&1 || { tail -30 "gpurun_out/pytest_$name.log"; exit 1; }
            tail -3 "gpurun_out/pytest_$name.log" ;;
        bench)
            timeout -k 10 "${T_BENCH:-300}" python -u bench.py $args > "gpurun_out/bench_$name.json" \
                2> "gpurun_out/bench_$name.err" || { tail -20 "gpurun_out/bench_$name.err"; exit 1; }
            cat "gpurun_out/bench_$name.json" ;;
        prof)
            timeout -k 10 "${T_BENCH:-300}" rocprofv3 --kernel-trace --stats --output-format csv \
                -d "gpurun_out/prof_$name" -o run -- python3 bench.py $args > "gpurun_out/prof_$name.json" \
                2> "gpurun_out/prof_$name.err" || { tail -20 "gpurun_out/prof_$name.err"; exit 1; } ;;
        pmc)
            ctr=${args%%:*}
            bargs=${args#*:}
            timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "gpurun_out/pmc_$name" -o run -- \
                python3 bench.py $bargs > "gpurun_out/pmc_$name.json" 2> "gpurun_out/pmc_$name.err" \
                || { tail -20 "gpurun_out/pmc_$name.err"; exit 1; } ;;
        py)
            timeout -k 10 "${T_PY:-300}" python -u $args > "gpurun_out/py_$name.log" 2>&1 \
                || { tail -30 "gpurun_out/py_$name.log"; exit 1; }
            tail -5 "gpurun_out/py_$name.log" ;;
        smoke)
            timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$name.log" 2>&1 \
                || { tail -20 "gpurun_out/smoke_$name.log"; exit 1; }
            tail -2 "gpurun_out/smoke_$name.log" ;;
        ab)
            # ARGS: variants separated by ';', each "[LIB] [NAME=VALUE ...]" (empty: the in-tree
            # build as it is), run twice, interleaved (tools/sweep_exp.py)
            : > "gpurun_out/ab_$name.log"
            IFS=';' read -ra vars <<< "$args"
            for rep in 1 2; do
                for v in "${vars[@]}"; do
                    timeout -k 10 "${T_PY:-300}" python -u tools/sweep_exp.py $v >> "gpurun_out/ab_$name.log" 2>&1 \
                        || { tail -30 "gpurun_out/ab_$name.log"; exit 1; }
                done
            done
            grep pivots/s "gpurun_out/ab_$name.log" ;;
        run)
            timeout -k 10 "${T_PY:-300}" $args > "gpurun_out/run_$name.log" 2>&1 \
                || { tail -30 "gpurun_out/run_$name.log"; exit 1; }
            tail -5 "gpurun_out/run_$name.log" ;;
        *)
            echo "unknown step kind: $kind" >&2
            exit 2 ;;
    esac
}
for spec in "$@"; do
    kind=${spec%%:*}
    rest=${spec#*:}
    name=${rest%%:*}
    args=${rest#*:}
    envs=""
    if [[ $kind == *@* ]]; then envs=${kind#*@}; kind=${kind%%@*}; fi
    echo "[gpu.sh] $kind $name: $args ${envs:+(env $envs)}" >&2
    ( if [ -n "$envs" ]; then IFS=',' read -ra kvs <<< "$envs"; for kv in "${kvs[@]}"; do export "$kv"; done; fi
      run_step ) || exit $?
done
