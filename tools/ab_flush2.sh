#!/bin/bash
# Round 6: the XCD item map's column classes (LPG_FLUSH_XCD = hH) and the
# global queue at its default heights, interleaved A/B at config 3
# (tools/order_lab.hip: ORD 2 -- XCD x owns tiles t = x mod 8, all rows -- streamed
# 5.16-5.29 TB/s vs 4.91 for the banded map at 2048-row items).
export REPS=${REPS:-2}
python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XCD=h8" "LPG_FLUSH_XCD=h4" "LPG_FLUSH_XCD=0" \
    "LPG_FLUSH_XCD=0 LPG_FLUSH_MINITEMS=1024"
