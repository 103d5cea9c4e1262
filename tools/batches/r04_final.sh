#!/bin/bash
# round-4 final evidence: whole -m gpu suite, smoke, benches (default + driver form + configs 2/4),
# rocprofv3 kernel stats and the two PMC passes of the default bench
set -u
export TMPDIR=/tmp
T_PYTEST=1100 bash tools/gpu.sh "pytest:r04_all:tests -m gpu -x -v" && \
bash tools/gpu.sh "smoke:r04:" \
    "bench:r04_default:" \
    "bench:r04_driver_form:--steps 20 --warmup 5" \
    "bench:r04_config2:--config 2 --steps 20 --warmup 3 --no-cpu" \
    "bench:r04_config4:--config 4 --steps 4 --warmup 1 --no-cpu" \
    "prof:r04_c3:--steps 5 --warmup 1 --no-cpu" \
    "pmc:r04_fetch:FETCH_SIZE:--steps 2 --warmup 0 --no-cpu" \
    "pmc:r04_write:WRITE_SIZE:--steps 2 --warmup 0 --no-cpu"
