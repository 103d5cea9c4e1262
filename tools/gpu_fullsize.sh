#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_integration_cli.py -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread --durations=0 > gpurun_out/pytest_full.log 2>&1
