#!/bin/bash
set -u
mkdir -p gpurun_out
for w in 16 32 64 128; do
LPG_PERSIST_WG=$w timeout -k 10 120 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/wg_c2_$w.json 2>/dev/null || exit $?
done
for w in 128 192; do
LPG_PERSIST_WG=$w timeout -k 10 200 python bench.py --config 5 --no-cpu > gpurun_out/wg_c5_$w.json 2>/dev/null || exit $?
LPG_PERSIST_WG=$w timeout -k 10 200 python bench.py --steps 32 --no-cpu > gpurun_out/wg_c3_$w.json 2>/dev/null || true
done
