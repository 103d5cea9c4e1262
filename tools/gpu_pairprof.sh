#!/bin/bash
# Kernel stats of the single-rank two-kernel pair (LPG_PERSIST=0) at config 3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pairprof
LPG_PERSIST=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pairprof -o run -- \
    python3 bench.py --steps 4 --warmup 0 --no-cpu > gpurun_out/pairprof/bench.json 2> gpurun_out/pairprof/err || exit $?
