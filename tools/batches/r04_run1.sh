#!/bin/bash
# round-4 GPU batch 1: labs, the fixes' tests, k_flushd bitwise + A/B, probes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; tail -3 "gpurun_out/r04_$name.log"; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; exit $rc; }; }
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step 170 hbm_ceiling tools/hbm_ceiling 5
step 120 flush64_lab tools/flush64_lab 5
step 400 pytest_fix $PYT tests/test_dual.py tests/test_gpu_block.py -m gpu -k "gpu_dual or inconsistent"
step 400 pytest_dist_dual $PYT tests/test_gpu_dist.py -m gpu -k dual
step 300 pytest_defer $PYT tests/test_gpu_defer.py -m gpu
step 200 bench_w python -u bench.py --steps 20 --warmup 3 --no-cpu
step 200 bench_d env LPG_FLUSH_KERNEL=d python -u bench.py --steps 20 --warmup 3 --no-cpu
step 200 bench_w2 python -u bench.py --steps 20 --warmup 3 --no-cpu
step 200 bench_d2 env LPG_FLUSH_KERNEL=d python -u bench.py --steps 20 --warmup 3 --no-cpu
step 300 dual_late_wg python -u tools/dual_late_wg.py linearprogramming_amd/liblpg.so tools/liblpg_r03.so
step 200 block_probe python -u tools/block_probe.py
step 400 pytest_c4_8ranks $PYT -s tests/test_gpu_dist_fullsize.py -m gpu -k eight
