#!/bin/bash
# round-4 final evidence at HEAD (after the 96-slot select / pivot-row / prep changes):
# whole -m gpu suite, smoke, default and driver-form benches, config 4, a sustained config-3 run
set -u
export TMPDIR=/tmp
T_PYTEST=1100 bash tools/gpu.sh "pytest:r04_all2:tests -m gpu -x -v" && \
bash tools/gpu.sh "smoke:r04_2:" \
    "bench:r04_default2:" \
    "bench:r04_driver_form2:--steps 20 --warmup 5" \
    "bench:r04_config4_2:--config 4 --steps 4 --warmup 1 --no-cpu" \
    "bench:r04_sustained:--steps 512 --warmup 8 --no-cpu" \
    "prof:r04_c4:--config 4 --steps 3 --warmup 1 --no-cpu"
