#!/bin/bash
# round-4 final check after the unrolled chain batches: whole -m gpu suite and smoke
# (part 1), then the benches of configs 3 / 4 / 2 / 5 and rocprofv3 stats (part 2)
set -u
export TMPDIR=/tmp
if [ "${1:-1}" = 1 ]; then
T_PYTEST=1100 bash tools/gpu.sh "pytest:r04_all5:tests -m gpu -x -v" && bash tools/gpu.sh "smoke:r04_5:"
else
bash tools/gpu.sh "bench:r04_default5:" "bench:r04_driver5:--steps 20 --warmup 5" \
    "bench:r04_config4_5:--config 4 --steps 4 --warmup 1 --no-cpu" \
    "bench:r04_config2_5:--config 2 --steps 20 --warmup 3 --no-cpu" "bench:r04_config5_5:--config 5 --no-cpu" \
    "prof:r04_final5:--steps 8 --warmup 2 --no-cpu"
fi
