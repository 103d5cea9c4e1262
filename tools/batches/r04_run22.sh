#!/bin/bash
# round-4 GPU batch 22: config 3's persistent launch on 256 workgroups (64 rows each: the
# entering-column chain on one wave) against the default 227 (73 rows: two waves)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
for i in 1 2 3; do
  step 200 wg227_$i python -u tools/sweep_exp.py
  step 200 wg256_$i env LPG_PERSIST_WG=256 python -u tools/sweep_exp.py
done
grep -h "pivots/s" gpurun_out/r04_wg227_*.log gpurun_out/r04_wg256_*.log
