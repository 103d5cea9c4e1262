#!/bin/bash
# Round 6: row pieces per tail tile of the XCD item map (LPG_FLUSH_XPIECES,
# default 4) and tail tiles per group (LPG_FLUSH_XTAIL, default nblocks/16 = 16
# at config 3), interleaved A/B at config 3 in the driver's form (per-item
# timestamps: the tail after a block's last item is 3.3-4.1% of the pass with
# quarter pieces, profiles/r06_flushw_ts.log).
export REPS=${REPS:-2}
python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XPIECES=8 LPG_FLUSH_XTAIL=8" \
    "LPG_FLUSH_XPIECES=16 LPG_FLUSH_XTAIL=8" "LPG_FLUSH_XPIECES=8 LPG_FLUSH_XTAIL=4" \
    "LPG_FLUSH_XPIECES=16 LPG_FLUSH_XTAIL=4" "LPG_FLUSH_XPIECES=4 LPG_FLUSH_XTAIL=8"
