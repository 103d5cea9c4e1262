#!/bin/bash
# round-4 GPU batch 19: the pivot-row rewrite on a second stream beside the block pass
# (k_flushw no longer stores the block's pivot rows): bitwise tests, soak, then
# interleaved config-3 A/B against the previous HEAD (tools/liblpg_head.so) and
# the one-stream order (LPG_ROWS_OVERLAP=0)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 900 pytest_gpu_rowsovl python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_dual.py
tail -1 gpurun_out/r04_pytest_gpu_rowsovl.log
step 200 rowsovl_soak python -u tools/soak.py 90 1919
tail -1 gpurun_out/r04_rowsovl_soak.log
for i in 1 2 3; do
  step 200 rowsovl_head_$i python -u tools/sweep_exp.py tools/liblpg_head.so
  step 200 rowsovl_on_$i python -u tools/sweep_exp.py
  step 200 rowsovl_off_$i env LPG_ROWS_OVERLAP=0 python -u tools/sweep_exp.py
done
grep -h "pivots/s" gpurun_out/r04_rowsovl_{head,on,off}_*.log
step 200 rowsovl_bench python -u bench.py --steps 20 --warmup 3 --no-cpu
grep '^{' gpurun_out/r04_rowsovl_bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', round(d['value']), 'block', round(d['ms_per_step'],4), 'pass', round(r['update_ms_mean'],4), 'other', round(r['other_ms_per_block'],4))"
