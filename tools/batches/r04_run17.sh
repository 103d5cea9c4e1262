#!/bin/bash
# round-4 GPU batch 17: staggered stores in the 64-slot block pass (LPG_FLUSH_STAG=1: the
# upper half of each block's waves stores band s-1 after band s's matrix ops):
# bitwise tests with it, then interleaved config-3 A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 900 pytest_gpu_stag env LPG_FLUSH_STAG=1 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_fullsize.py
B3="python -u bench.py --steps 20 --warmup 3 --no-cpu"
for i in 1 2 3; do
  step 200 stag_off_$i $B3
  step 200 stag_on_$i env LPG_FLUSH_STAG=1 $B3
done
for f in gpurun_out/r04_stag_*; do
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['value']), 'block', round(d['ms_per_step'],4), 'other', round(r['other_ms_per_block'],4), 'achieved', round(r['achieved']))
"
done
