#!/bin/bash
# Column trade on / off (LPG_NO_REORDER) at configs 2, 5 and 3.
set -u
mkdir -p gpurun_out
for r in 0 1; do
  LPG_NO_REORDER=$r timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/ro_c2_$r.json 2>/dev/null || exit $?
  LPG_NO_REORDER=$r timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/ro_c5_$r.json 2>/dev/null || exit $?
  LPG_NO_REORDER=$r timeout -k 10 200 python bench.py --steps 64 --no-cpu > gpurun_out/ro_c3_$r.json 2>/dev/null || exit $?
done
