#!/bin/bash
# flush lab on the GPU box (tools/flush_lab.hip): config-3 rows (LAB_ROWS), designs picked by LAB_ONLY
set -u
mkdir -p gpurun_out
timeout -k 10 300 ./tools/flush_lab ${LAB_ROWS:-16384} > gpurun_out/flush_lab.log 2>&1 || exit $?
