#!/bin/bash
# Persistent pivot kernel: its parity tests, the phase probe, a short config-3 bench (and the two-kernel pair's).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_block.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_block.log 2>&1 || exit $?
timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 64 > gpurun_out/bench_block.json 2> gpurun_out/bench_block.err || exit $?
LPG_PERSIST=0 timeout -k 10 300 python bench.py --no-cpu --steps 64 > gpurun_out/bench_pair.json 2> gpurun_out/bench_pair.err || exit $?
