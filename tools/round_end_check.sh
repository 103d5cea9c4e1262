#!/bin/bash
# What the driver runs at round end, in its order: smoke(), then bench.py with
# no flags (N=1 defaults). Each step time-limited; the first failure ends it.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || exit $?
time timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
