#!/bin/bash
# Bench lines of configs 2, 4, 5 with the persistent pivot kernel and with the two-kernel pair.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/bench_c2.json 2>> gpurun_out/bench_cfg.err || exit $?
LPG_PERSIST=0 timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/bench_c2_pair.json 2>> gpurun_out/bench_cfg.err || exit $?
timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/bench_c5.json 2>> gpurun_out/bench_cfg.err || exit $?
LPG_PERSIST=0 timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/bench_c5_pair.json 2>> gpurun_out/bench_cfg.err || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4.json 2>> gpurun_out/bench_cfg.err || exit $?
