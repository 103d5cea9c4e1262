#!/bin/bash
# Round 6: the column trade (and with it region mode) below its 2 GB default
# threshold, at config 5 (1.3 GB, K = 64 all-column slices by default) and
# config 2 (25 MB, K = 32), interleaved.
REPS=3 python -u tools/ab_bench.py "--config 5" "" "LPG_NO_REORDER=0" "LPG_NO_REORDER=0 LPG_DEFER=96" || exit 1
REPS=3 python -u tools/ab_bench.py "--config 2" "" "LPG_NO_REORDER=0" "LPG_NO_REORDER=0 LPG_DEFER=64"
