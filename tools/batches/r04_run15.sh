#!/bin/bash
# round-4 GPU batch 15: k_flush_pivot_rows<96> vs <128> for 96-slot blocks (config 4, 32 blocks each)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
for i in 1 2 3; do
  step 300 pr_96_$i env M=65536 N=131072 python -u tools/sweep_exp.py tools/liblpg_pr.so
  step 300 pr_128_$i env LPG_PIVROWS128=1 M=65536 N=131072 python -u tools/sweep_exp.py tools/liblpg_pr.so
done
grep -H pivots/s gpurun_out/r04_pr_*.log
