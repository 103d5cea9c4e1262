#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 64 > gpurun_out/bench_block.json 2> gpurun_out/bench_block.err || exit $?
