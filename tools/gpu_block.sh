#!/bin/bash
# Persistent pivot kernel: its parity tests, the phase probe, config-3 bench (and the two-kernel pair's), configs 2 and 5.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_block.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_block.log 2>&1 || exit $?
timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 64 > gpurun_out/bench_block.json 2> gpurun_out/bench_block.err || exit $?
LPG_PERSIST=0 timeout -k 10 300 python bench.py --no-cpu --steps 64 > gpurun_out/bench_pair.json 2> gpurun_out/bench_pair.err || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/bench_c2.json 2>> gpurun_out/bench_cfg.err || exit $?
timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/bench_c5.json 2>> gpurun_out/bench_cfg.err || exit $?
