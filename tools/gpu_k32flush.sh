#!/bin/bash
# Blocks of 32 vs 64 under k_flushw (the default flush now) at three sizes below the 512 MB default switch,
# after the deferred-path tests.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_block.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_k32.log 2>&1 || exit $?
: > gpurun_out/k32flush.log
for mn in "1024 2048" "2048 4096" "4096 8192"; do
  set -- $mn
  for k in 32 64; do
    M=$1 N=$2 LPG_DEFER=$k timeout -k 10 120 python tools/sweep_exp.py >> gpurun_out/k32flush.log 2>&1 || exit $?
  done
done
