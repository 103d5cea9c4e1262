#!/bin/bash
# After the column-trade default change: the GPU suite, then configs 2, 5, 3 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_trade.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/tr_c2.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config 5 > gpurun_out/tr_c5.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --steps 64 --no-cpu > gpurun_out/tr_c3.json 2>/dev/null || exit $?
