#!/bin/bash
# round-4 GPU batch 12: k_select_d two banks of 48 from 64 pending pivots, k_flush_pivot_rows<96>
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 900 pytest_gpu_sel96 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_fullsize.py tests/test_gpu_block.py tests/test_big_m.py
for i in 1 2 3; do
  step 300 ab_sel96_new_$i env M=65536 N=131072 python -u tools/sweep_exp.py
  step 300 ab_sel96_head_$i env M=65536 N=131072 python -u tools/sweep_exp.py tools/liblpg_head.so
done
grep -h pivots/s gpurun_out/r04_ab_sel96_*.log
