#!/bin/bash
# round-4 GPU batch 10: config-3 item height with a lower fill threshold (2048-row items)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
B3="python -u bench.py --steps 20 --warmup 3 --no-cpu"
for i in 1 2 3; do
  step 200 c3_min2048_$i $B3
  step 200 c3_min1024_$i env LPG_FLUSH_MINITEMS=1024 $B3
  step 200 c3_min512_$i env LPG_FLUSH_MINITEMS=512 $B3
done
for f in gpurun_out/r04_c3_min*; do
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['value']), 'block', round(d['ms_per_step'],4), 'pass', round(r['update_ms_mean'],4))
"
done
