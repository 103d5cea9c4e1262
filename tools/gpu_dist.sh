#!/bin/bash
# The distributed GPU tests alone.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || exit $?
