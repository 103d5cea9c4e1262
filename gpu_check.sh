#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench. Stops at the first
# crash / timeout (exit codes > 1); a plain test failure (1) still benches.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_integration_cli.py tests/test_gpu_dist.py} -m gpu -v -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
exit $rc
