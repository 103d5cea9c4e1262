#!/bin/bash
# (LPG_PIVROWS and k_flush_pivot_rows_pf existed only for this experiment; the source was
# reverted after it: DESIGN.md §8, profiles/r06_ab_pivrows_pf.log)
# Round 6: the latency-hidden pivot-row rewrite (k_flush_pivot_rows_pf,
# default) against the form before (LPG_PIVROWS=0), interleaved, config 3
# (driver's form) and config 4; then rocprofv3 kernel stats of both at config 3.
REPS=4 python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_PIVROWS=0" || exit 1
REPS=2 T_RUN=400 python -u tools/ab_bench.py "--config 4 --steps 4 --warmup 1" "" "LPG_PIVROWS=0" || exit 1
export TMPDIR=/tmp
for v in 1 0; do
    LPG_PIVROWS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pivrows_$v -o run \
        -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/prof_pivrows_$v.json 2> gpurun_out/prof_pivrows_$v.err || exit 1
    grep -h "pivot_rows" gpurun_out/prof_pivrows_$v/run_kernel_stats.csv | cut -d, -f1,2,4
done
