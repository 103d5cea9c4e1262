#!/bin/bash
# round-4 GPU batch 14: k_flushw<96> with tableau bands two ahead (LPG_FLUSH_LA=2) vs one, config 4
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 300 pytest_gpu_la2 env LPG_FLUSH_LA=2 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py -k "96 or flush_kernels_block_sizes"
B4="python -u bench.py --config 4 --steps 4 --warmup 1 --no-cpu"
for i in 1 2 3; do
  step 300 la_1_$i $B4
  step 300 la_2_$i env LPG_FLUSH_LA=2 $B4
done
for f in gpurun_out/r04_la_*; do
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['value']), 'block', round(d['ms_per_step'],3), 'pass', round(r['update_ms_mean'],3))
"
done
