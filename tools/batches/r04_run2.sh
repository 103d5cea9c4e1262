#!/bin/bash
# round-4 GPU batch 2: bitwise suites with the tail item map, tail A/B, per-rank shapes, rocprof
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r04_$name.log"; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; exit $rc; }; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
step 600 pytest_tail $PYT tests/test_gpu_defer.py tests/test_gpu_block.py tests/test_gpu_fullsize.py -m gpu
B="python -u bench.py --steps 20 --warmup 3 --no-cpu"
for i in 1 2 3; do
  step 200 tail_on_$i $B
  step 200 tail_off_$i env LPG_FLUSH_TAIL=0 $B
done
for P in 2 4 8; do
  M=$((16384 / P)); N=$((49152 - M))
  step 200 shape_p${P}_push $B --shape $M,$N --force-push
  step 200 shape_p${P}_single $B --shape $M,$N
done
step 300 prof_c3 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof_c3 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu
