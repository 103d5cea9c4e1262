#!/bin/bash
# Config-3 bench under several k_flushw forms (LPG_FLUSH_VARIANT), interleaved
# so that box drift hits every form alike; one JSON line per run, appended to
# gpurun_out/fv_<variant>.jsonl.
set -u
mkdir -p gpurun_out
rm -f gpurun_out/fv_*.jsonl
for v in ${VARIANTS:-21 25 21 25 21 25}; do
  LPG_FLUSH_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu >> gpurun_out/fv_$v.jsonl 2>/dev/null || exit $?
done
