#!/bin/bash
# round-4 GPU batch 5: config 4 item height A/B (K = 96)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r04_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; exit $rc; }; }
B="python -u bench.py --config 4 --steps 4 --warmup 1 --no-cpu"
for i in 1 2; do
  step 300 c4_rows512_$i $B
  step 300 c4_rows2048_$i env LPG_FLUSH_ROWS=2048 $B
  step 300 c4_rows1024_$i env LPG_FLUSH_ROWS=1024 $B
done
