#!/bin/bash
# Round 6: the block pass's item order / height / block width, interleaved A/B
# at config 3 (tools/ab_bench.py; tools/order_lab.hip measured the memory path
# alone: the global queue with 64-row items streams 5.80 TB/s, the XCD-banded
# 2048-row map 4.91).
export REPS=${REPS:-2}
python -u tools/ab_bench.py "--steps 20 --warmup 5" "" "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=64" \
    "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=128" "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=256" "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=512" \
    "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=128 LPG_FLUSH_W96=4" "LPG_FLUSH_XCD=0 LPG_FLUSH_ROWS=64 LPG_FLUSH_W96=4"
