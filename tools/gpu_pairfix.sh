#!/bin/bash
# After the load-serialisation fixes: tests, the pair's kernel stats, bench lines for the pair paths and config 3 / 4.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pairprof
timeout -k 10 900 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_pairfix.log 2>&1 || exit $?
bash tools/gpu_pairprof.sh || exit $?
timeout -k 10 200 python bench.py --steps 64 --no-cpu > gpurun_out/pf_c3.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --force-rccl --steps 64 --no-cpu > gpurun_out/pf_rccl1.json 2>/dev/null || exit $?
LPG_PERSIST_MR=0 timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/pf_push1_pair.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/pf_push1.json 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/pf_c4.json 2>/dev/null || exit $?
