#!/bin/bash
# Multi-rank k_pivot_block: the distributed tests (1-rank self-push, 2-3 processes), then the block tests.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mrp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_defer.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_mrp2.log 2>&1 || exit $?
