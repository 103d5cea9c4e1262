#!/bin/bash
# round-4 GPU batch 18: the block pass at 72 slots (k_flushw<72>, LPG_FLUSH_K72=1) on the
# config-3 shape against 64 and 96 slots: pass time per block decides whether 72-pivot
# blocks in the persistent launch can pay
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 200 k72_soak env LPG_FLUSH_K72=1 python -u tools/soak.py 60 7272
tail -1 gpurun_out/r04_k72_soak.log
B3="python -u bench.py --steps 12 --warmup 3 --no-cpu"
for i in 1 2; do
  step 200 k72_d64_$i $B3
  step 300 k72_d72k96_$i $B3 --defer 72
  step 300 k72_d72k72_$i env LPG_FLUSH_K72=1 $B3 --defer 72
done
for f in gpurun_out/r04_k72_d*; do
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['value']), 'block', round(d['ms_per_step'],4), 'other', round(r.get('other_ms_per_block',0),4), 'achieved', round(r['achieved']), 'pass_ms', round(r['update_ms_mean'],4))
"
done
