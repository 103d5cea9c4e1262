#!/bin/bash
# Iteration check on the GPU box: GPU tests (PYTEST_FILES, default all) then
# bench lines (BENCHES: "name:args;name:args"). Each step time-limited; the
# first crash / timeout ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || exit $?
IFS=';' read -ra BS <<< "${BENCHES:-b3:--no-cpu}"
for b in "${BS[@]}"; do
  name=${b%%:*}; args=${b#*:}
  timeout -k 10 300 python bench.py $args > gpurun_out/$name.json 2>>gpurun_out/bench_iter.err || exit $?
done
