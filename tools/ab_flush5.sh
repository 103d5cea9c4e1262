#!/bin/bash
# Round 6: 8 / 16 / 32 tail pieces per tail tile (LPG_FLUSH_XPIECES) against
# the default 4 at config 3 (driver's form) and config 5, interleaved.
REPS=5 python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XPIECES=8" "LPG_FLUSH_XPIECES=16" || exit 1
REPS=3 python -u tools/ab_bench.py "--config 5" "" "LPG_FLUSH_XPIECES=8" "LPG_FLUSH_XPIECES=16" "LPG_FLUSH_XPIECES=32"
