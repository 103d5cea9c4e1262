#!/bin/bash
# Config 2: k_flushm (default for 32-pivot blocks) vs k_flushw.
set -u
mkdir -p gpurun_out
for fk in m w m w; do
  LPG_FLUSH_KERNEL=$fk timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/c2f_$fk.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('gpurun_out/c2f_$fk.json')); print('$fk', round(d['value']), d['roofline'].get('update_ms_mean'))" >> gpurun_out/c2f.log || exit $?
done
