#!/bin/bash
# Re-measure the pair-path lines (config 4, 1-rank RCCL, 1-rank push pair) twice each.
set -u
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --force-rccl --steps 64 --no-cpu > gpurun_out/rc_rccl1_$i.json 2>/dev/null || exit $?
LPG_PERSIST_MR=0 timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/rc_push1_$i.json 2>/dev/null || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/rc_c4_$i.json 2>/dev/null || exit $?
done
