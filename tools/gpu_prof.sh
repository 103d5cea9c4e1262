#!/bin/bash
# rocprofv3 evidence of the config-3 bench (kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes),
# then the other BASELINE configs' bench lines.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
STEPS=4 ./tools/profile.sh || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/bench_config2.json 2>> gpurun_out/bench_cfg.err || exit $?
timeout -k 10 300 python bench.py --config 5 > gpurun_out/bench_config5.json 2>> gpurun_out/bench_cfg.err || exit $?
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_config4.json 2>> gpurun_out/bench_cfg.err || exit $?
