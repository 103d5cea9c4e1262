#!/bin/bash
# Final check at HEAD: the GPU suite, then what the driver runs (smoke, default bench).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || exit $?
bash tools/round_end_check.sh || exit $?
