#!/bin/bash
# Quick GPU check: the block-kernel tests and the parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || exit $?
