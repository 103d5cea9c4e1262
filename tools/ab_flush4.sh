#!/bin/bash
# Round 6: eighth-height tail pieces (LPG_FLUSH_XPIECES=8; the tail tiles per
# group unchanged) against the default quarter pieces at config 3 (driver's
# form), config 5 and config 4 (one GPU), interleaved. (Fewer tail tiles,
# LPG_FLUSH_XTAIL=4, cost config 5 -- whose live columns sit in a few low
# tiles -- a third of its rate: 47.6k vs 72.7k pivots/s.)
REPS=5 python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XPIECES=8" || exit 1
REPS=3 python -u tools/ab_bench.py "--config 5" "" "LPG_FLUSH_XPIECES=8" || exit 1
REPS=2 T_RUN=400 python -u tools/ab_bench.py "--config 4 --steps 4 --warmup 1" "" "LPG_FLUSH_XPIECES=8"
