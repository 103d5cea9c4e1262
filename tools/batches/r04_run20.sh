#!/bin/bash
# round-4 GPU batch 20: k_pivot_block's chains as software-pipelined 16-slot batches
# (instead of every slot's LDS read before the first fma), the entering-column chain
# only on waves holding rows: bitwise tests (single and multi-rank), soak, then
# interleaved config-3 A/B against the previous HEAD (tools/liblpg_head.so)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 900 pytest_gpu_chainp python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_dual.py tests/test_gpu_dist.py
tail -1 gpurun_out/r04_pytest_gpu_chainp.log
step 200 chainp_soak python -u tools/soak.py 90 2020
tail -1 gpurun_out/r04_chainp_soak.log
for i in 1 2 3; do
  step 200 chainp_head_$i python -u tools/sweep_exp.py tools/liblpg_head.so
  step 200 chainp_new_$i python -u tools/sweep_exp.py
done
grep -h "pivots/s" gpurun_out/r04_chainp_head_*.log gpurun_out/r04_chainp_new_*.log
step 200 chainp_bench python -u bench.py --steps 20 --warmup 3 --no-cpu
grep '^{' gpurun_out/r04_chainp_bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench', round(d['value']), 'block', round(d['ms_per_step'],4), 'pass', round(r['update_ms_mean'],4), 'other', round(r['other_ms_per_block'],4))"
