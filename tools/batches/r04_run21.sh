#!/bin/bash
# round-4 GPU batch 21: the chains' batches fully unrolled per batch count (no runtime
# loop): phase probe, bitwise block tests, interleaved A/B against HEAD
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 200 block_probe_unroll python -u tools/block_probe.py
sed -n 3,8p gpurun_out/r04_block_probe_unroll.log | cut -c1-120
step 600 pytest_gpu_unroll python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_block.py tests/test_gpu_defer.py
tail -1 gpurun_out/r04_pytest_gpu_unroll.log
for i in 1 2 3; do
  step 200 unroll_head_$i python -u tools/sweep_exp.py tools/liblpg_head.so
  step 200 unroll_new_$i python -u tools/sweep_exp.py
done
grep -h "pivots/s" gpurun_out/r04_unroll_head_*.log gpurun_out/r04_unroll_new_*.log
