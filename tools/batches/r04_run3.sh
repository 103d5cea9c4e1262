#!/bin/bash
# round-4 GPU batch 3: speculative entering-column loads (bitwise + A/B), K=96 lab
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r04_$name.log"; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; exit $rc; }; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step 600 pytest_spec $PYT tests/test_gpu_block.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu
for i in 1 2 3; do
  step 200 ab_spec_$i python -u tools/sweep_exp.py
  step 200 ab_base_$i python -u tools/sweep_exp.py tools/liblpg_base.so
done
step 200 bench_spec python -u bench.py --steps 20 --warmup 3 --no-cpu
step 200 flush96_lab env LAB_K=96 tools/flush64_lab 5
