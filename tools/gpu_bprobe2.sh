#!/bin/bash
# Block-kernel phase probe: completion stamps (liblpg_phases.so) and issue-time stamps (liblpg_phases_nowait.so).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe.log 2>&1 || exit $?
PHASES_LIB=liblpg_phases_nowait.so timeout -k 10 200 python tools/block_probe.py > gpurun_out/block_probe_nowait.log 2>&1 || exit $?
