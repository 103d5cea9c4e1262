#!/bin/bash
# round-4 GPU batch 9: pair grid changes (k_prep_d two banks of 48, k_select_d objective-row fold)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 600 pytest_gpu_pairfold python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py -k "pair_select_grid or generic_and_prefetching or wide_tableau or reordered"
step 300 bench_c4_pairfold python -u bench.py --config 4 --steps 4 --warmup 1 --no-cpu
step 300 phase_probe_c4_pairfold env M=65536 N=131072 python -u tools/phase_probe.py
step 900 pytest_gpu_pairfold_all python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_fullsize.py tests/test_big_m.py tests/test_two_phase.py tests/test_gpu_parity.py
step 300 bench_c3_pairfold python -u bench.py --steps 20 --warmup 3 --no-cpu
