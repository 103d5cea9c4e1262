#!/bin/bash
# After a change to the block argmins: block / defer / parity tests, the phase probes, config 3 and 5 bench lines.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_defer.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_argmin.log 2>&1 || exit $?
timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe.log 2>&1 || exit $?
PHASES_LIB=liblpg_phases_nowait.so timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe_nowait.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 64 --no-cpu > gpurun_out/argmin_c3.json 2>> gpurun_out/argmin.err || exit $?
timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/argmin_c5.json 2>> gpurun_out/argmin.err || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/argmin_c2.json 2>> gpurun_out/argmin.err || exit $?
