#!/bin/bash
# round-4 GPU batch 4: single-guess speculation, per phase, A/B against the base
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r04_$name.log"; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; exit $rc; }; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step 300 pytest_spec1 $PYT tests/test_gpu_block.py tests/test_gpu_fullsize.py -m gpu -k "not config4 and not config5"
for i in 1 2; do
  step 200 ab4_both_$i python -u tools/sweep_exp.py tools/liblpg_spec1.so
  step 200 ab4_S_$i python -u tools/sweep_exp.py tools/liblpg_specS.so
  step 200 ab4_P_$i python -u tools/sweep_exp.py tools/liblpg_specP.so
  step 200 ab4_base_$i python -u tools/sweep_exp.py tools/liblpg_base.so
done
