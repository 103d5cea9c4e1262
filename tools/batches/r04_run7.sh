#!/bin/bash
# round-4 GPU batch 7: 2048-row items default -- flush bitwise tests, benches; sweep lab
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 120 sweep_lab ./tools/sweep_lab 4000
step 900 pytest_gpu_rows2048 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py tests/test_gpu_fullsize.py tests/test_gpu_block.py
step 300 bench_c3_rows2048 python -u bench.py --steps 20 --warmup 3 --no-cpu
step 300 bench_c4_rows2048 python -u bench.py --config 4 --steps 4 --warmup 1 --no-cpu
step 300 bench_c2_rows2048 python -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu
