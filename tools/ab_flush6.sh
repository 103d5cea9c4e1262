#!/bin/bash
# Round 6, after eighth-height tail pieces became the default: more tail tiles
# per group (LPG_FLUSH_XTAIL; default nblocks / 16 = 16 at configs 3 and 5),
# interleaved at config 5 and config 3 (driver's form).
REPS=3 python -u tools/ab_bench.py "--config 5" "" "LPG_FLUSH_XTAIL=24" "LPG_FLUSH_XTAIL=32" || exit 1
REPS=4 python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XTAIL=24" "LPG_FLUSH_XTAIL=32"
