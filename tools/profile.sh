#!/bin/bash
# rocprofv3 evidence for bench.py's config (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command           -> gpurun_out/prof/trace
#   2. FETCH_SIZE pass (own run, kernel counters only)      -> gpurun_out/prof/fetch
#   3. WRITE_SIZE pass (own run)                            -> gpurun_out/prof/write
# Every step has its own time limit; the first failure ends the script.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof
CFG=${CFG:-3}
STEPS=${STEPS:-2}   # whole deferred blocks (bench.py steps), no warm-up: every flush applies a full block
mkdir -p $OUT
echo "[profile] trace" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --config $CFG --steps $STEPS --warmup 0 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
echo "[profile] fetch" >&2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --config $CFG --steps $STEPS --warmup 0 --no-cpu > $OUT/fetch_bench.json 2> $OUT/fetch.err || exit $?
echo "[profile] write" >&2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --config $CFG --steps $STEPS --warmup 0 --no-cpu > $OUT/write_bench.json 2> $OUT/write.err || exit $?
find $OUT -name "*.csv" | head -50 >&2
