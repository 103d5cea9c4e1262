#!/bin/bash
# round-4 final check after the pipelined chains: whole -m gpu suite and smoke
# (part 1), then the benches of configs 3 / 4 / 2 / 5 and rocprofv3 stats (part 2)
set -u
export TMPDIR=/tmp
if [ "${1:-1}" = 1 ]; then
T_PYTEST=1100 bash tools/gpu.sh "pytest:r04_all4:tests -m gpu -x -v" && bash tools/gpu.sh "smoke:r04_4:"
else
bash tools/gpu.sh "bench:r04_default4:" "bench:r04_driver4:--steps 20 --warmup 5" \
    "bench:r04_config4_4:--config 4 --steps 4 --warmup 1 --no-cpu" \
    "bench:r04_config2_4:--config 2 --steps 20 --warmup 3 --no-cpu" "bench:r04_config5_4:--config 5 --no-cpu" \
    "prof:r04_final4:--steps 8 --warmup 2 --no-cpu"
fi
