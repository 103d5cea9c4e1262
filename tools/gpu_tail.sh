#!/bin/bash
# After a change to the block-end kernels: the deferred / block / dist tests, then config 3 and config 4 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_tail.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 64 --no-cpu > gpurun_out/tail_c3.json 2>> gpurun_out/tail.err || exit $?
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/tail_c4.json 2>> gpurun_out/tail.err || exit $?
