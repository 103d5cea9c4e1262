#!/bin/bash
# GPU suite + probes + default bench (with the CPU baseline legs).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 ./tools/launch_floor > gpurun_out/launch_floor.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
exit $rc
