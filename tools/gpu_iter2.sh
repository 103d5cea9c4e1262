#!/bin/bash
# Round-2 iteration on the GPU box: load orders, GPU suite, driver-form bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in lpg_first torch_first; do
  timeout -k 10 120 python tools/runtime_order.py $o >> gpurun_out/runtime_order.log 2>&1; rc=$?
  echo "$o rc=$rc" >> gpurun_out/runtime_order.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >&2; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit $?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
exit $rc
