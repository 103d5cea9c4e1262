#!/bin/bash
# Sustained config-3 rate: long timed regions (the tableau keeps evolving;
# the block pass must not grow as columns leave the basis).
set -u
mkdir -p gpurun_out
for s in 1024 4096 16384; do
  timeout -k 10 300 python bench.py --no-cpu --steps $s --warmup 64 > gpurun_out/sustained_$s.json 2>/dev/null || exit $?
done
