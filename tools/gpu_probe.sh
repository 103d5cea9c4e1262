#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mfma_rate > gpurun_out/mfma_rate2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_a -o run -- \
    python3 bench.py --steps 8 --warmup 1 --no-cpu > gpurun_out/prof_a_bench.json 2> gpurun_out/prof_a.err || exit $?
