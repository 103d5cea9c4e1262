#!/bin/bash
# round-4 GPU batch 6: item height, config 4 (4096 / 8192) and config 3 (1024 / 2048)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -3 "gpurun_out/r04_$name.log"; exit $rc; }; }
B4="python -u bench.py --config 4 --steps 4 --warmup 1 --no-cpu"
B3="python -u bench.py --steps 20 --warmup 3 --no-cpu"
for i in 1 2; do
  step 300 c4_rows4096_$i env LPG_FLUSH_ROWS=4096 $B4
  step 300 c4_rows8192_$i env LPG_FLUSH_ROWS=8192 $B4
  step 300 c4_rows2048b_$i env LPG_FLUSH_ROWS=2048 $B4
  step 200 c3_rows512_$i $B3
  step 200 c3_rows1024_$i env LPG_FLUSH_ROWS=1024 $B3
  step 200 c3_rows2048_$i env LPG_FLUSH_ROWS=2048 $B3
done
for f in gpurun_out/r04_c4_rows4096_* gpurun_out/r04_c4_rows8192_* gpurun_out/r04_c4_rows2048b_* gpurun_out/r04_c3_rows*; do
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['value']), 'block', round(d['ms_per_step'],3), 'pass', round(r['update_ms_mean'],3))
"
done
