#!/bin/bash
# Record store / load cache-policy experiment: config-3 pivots/s per liblpg build (tools/sweep_libs).
set -u
mkdir -p gpurun_out
: > gpurun_out/sweep_exp.log
for lib in "" tools/sweep_libs/*.so ""; do
  timeout -k 10 120 python tools/sweep_exp.py $lib >> gpurun_out/sweep_exp.log 2>&1 || exit $?
done
