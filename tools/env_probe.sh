#!/bin/bash
# Config-3 bench under HIP runtime settings (one line per setting).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/env_base.json 2>/dev/null || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --no-cpu > gpurun_out/env_devkarg.json 2>/dev/null || exit $?
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python bench.py --no-cpu > gpurun_out/env_hostkarg.json 2>/dev/null || exit $?
