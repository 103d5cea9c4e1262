#!/bin/bash
# Round evidence on the GPU box: full GPU test suite, bench lines for configs
# 3 (default, with CPU baseline), 2, 5 and 4 (single GPU), then the rocprofv3
# kernel trace + PMC passes of the config-3 bench. Each GPU step has its own
# time limit; a crash / timeout ends the script (plain test failures do not).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_config3.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 1500 --no-cpu > gpurun_out/bench_config2.json 2>> gpurun_out/bench.err || exit $?
timeout -k 10 300 python bench.py --config 5 > gpurun_out/bench_config5.json 2>> gpurun_out/bench.err || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 64 --warmup 2 --no-cpu > gpurun_out/bench_config4.json 2>> gpurun_out/bench.err || exit $?
if [ -z "${NO_PROFILE:-}" ]; then ./tools/profile.sh || exit $?; fi
exit $rc
