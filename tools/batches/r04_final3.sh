#!/bin/bash
# round-4 last check at HEAD: whole -m gpu suite, smoke, default bench
set -u
export TMPDIR=/tmp
T_PYTEST=1100 bash tools/gpu.sh "pytest:r04_all3:tests -m gpu -x -v" && \
bash tools/gpu.sh "smoke:r04_3:" "bench:r04_default3:" "bench:r04_config4_3:--config 4 --steps 4 --warmup 1 --no-cpu"
