#!/bin/bash
# Multi-rank path on one GPU: distributed tests, then the 1-rank RCCL stand-in at config 3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_defer.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_mr.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --force-rccl > gpurun_out/bench_rccl1.json 2> gpurun_out/bench_rccl1.err || exit $?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_nocomm.json 2> gpurun_out/bench_nocomm.err || exit $?
