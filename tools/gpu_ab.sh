#!/bin/bash
# A/B: config-3 pivots/s of the in-tree liblpg vs tools/sweep_libs/*.so, interleaved.
set -u
mkdir -p gpurun_out
: > gpurun_out/ab.log
for lib in "" tools/sweep_libs/*.so "" tools/sweep_libs/*.so; do
  timeout -k 10 120 python tools/sweep_exp.py $lib >> gpurun_out/ab.log 2>&1 || exit $?
done
