#!/bin/bash
# Round 6: the pending-block size K at config 5 (default 64) and config 2
# (default 32), interleaved.
REPS=3 python -u tools/ab_bench.py "--config 5" "" "LPG_DEFER=48" "LPG_DEFER=96" || exit 1
REPS=3 python -u tools/ab_bench.py "--config 2" "" "LPG_DEFER=16" "LPG_DEFER=48"
