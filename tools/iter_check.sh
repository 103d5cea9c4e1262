#!/bin/bash
# One iteration on the GPU box: GPU parity suite, default bench, kernel-trace stats of the config-3 bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_iter
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --steps 256 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter -o run -- \
    python3 bench.py --steps 8 --warmup 1 --no-cpu > gpurun_out/prof_iter/bench.json 2> gpurun_out/prof_iter/err || exit $?
