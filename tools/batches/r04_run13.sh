#!/bin/bash
# round-4 GPU batch 13: k_prep_d<96> at 2 waves per SIMD in the owner-push form too (launch bounds)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 900 pytest_gpu_lb96 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_fullsize.py tests/test_gpu_defer.py -k "not flush_kernels"
S="python -u bench.py --shape 8192,131072 --force-push --steps 6 --warmup 1 --no-cpu"
for i in 1 2; do
  step 300 c4p8_push_new_$i $S
done
grep -h '^{' gpurun_out/r04_c4p8_push_new_*.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print(round(d['value']), round(d['ms_per_step'],3), r.get('update_ms_mean'), r.get('other_ms_per_block'))"
