#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench [-> profile]. Stops at
# the first crash / timeout (exit codes > 1); a plain test failure (1) still
# runs the bench.
set -u
mkdir -p gpurun_out
for o in ${ORDERS:-}; do
  timeout -k 10 120 python tools/runtime_order.py $o >> gpurun_out/runtime_order.log 2>&1 || { echo "$o rc=$?" >> gpurun_out/runtime_order.log; exit 3; }
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest ${PYTEST_FILES:-tests} -m gpu -v -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
else
  rc=0
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
for o in ${LATE_ORDERS:-}; do
  timeout -k 10 120 python tools/runtime_order.py $o >> gpurun_out/runtime_order.log 2>&1 || { echo "$o rc=$?" >> gpurun_out/runtime_order.log; exit 3; }
done
exit $rc
