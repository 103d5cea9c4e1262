#!/bin/bash
# Config 2 block size under the persistent pivot launch.
set -u
mkdir -p gpurun_out
for k in 16 32 48 64; do
  LPG_DEFER=$k timeout -k 10 200 python bench.py --config 2 --steps 40 --no-cpu > gpurun_out/c2_k$k.json 2>> gpurun_out/c2k.err || exit $?
done
