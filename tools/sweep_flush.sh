#!/bin/bash
# Deferred-update sweep on the GPU box: block size K (LPG_DEFER) and flush
# variants (LPG_FLUSH_VARIANT) on bench config C; one JSON line each.
set -u
C=${C:-3}
STEPS=${STEPS:-192}
OUT=${OUT:-gpurun_out/sweep_flush_c$C.log}
: > $OUT
for K in ${KS:-32}; do
  for V in ${VS:-0}; do
    echo "K=$K V=$V" >> $OUT
    LPG_FLUSH_VARIANT=$V timeout -k 10 120 python bench.py --config $C --defer $K --steps $STEPS --warmup 3 --no-cpu >> $OUT 2>/dev/null || exit $?
  done
done
