#!/bin/bash
# 128-pivot blocks: bitwise tests (defer, block, dist), then config 4 at K = 128 (default) and K = 64.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_k128.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/k128_c4.json 2>> gpurun_out/k128.err || exit $?
LPG_DEFER=64 timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/k64_c4.json 2>> gpurun_out/k128.err || exit $?
