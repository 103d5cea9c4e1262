#!/bin/bash
# Round-2 evidence at HEAD: GPU suite, driver-form and sustained config-3 bench lines (CPU leg on the default run),
# configs 2/4/5, rocprofv3 trace + FETCH/WRITE passes, block-kernel phase probe.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ev/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/ev/bench_default.json 2> gpurun_out/ev/bench_default.err || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ev/bench_driver_form.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 1024 --no-cpu > gpurun_out/ev/bench_sustained.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/ev/bench_config2.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config 5 > gpurun_out/ev/bench_config5.json 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/ev/bench_config4.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --force-rccl --steps 64 --no-cpu > gpurun_out/ev/bench_config3_rccl1.json 2>/dev/null || exit $?
timeout -k 10 200 python tools/block_probe.py > gpurun_out/ev/block_probe.log 2>&1 || exit $?
rm -rf gpurun_out/prof
STEPS=4 ./tools/profile.sh || exit $?
