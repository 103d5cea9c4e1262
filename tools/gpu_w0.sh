#!/bin/bash
# --warmup 0 with the push exchange: one untimed validation block, then the timed region.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --force-push --steps 4 --warmup 0 --no-cpu > gpurun_out/w0_push1.json 2> gpurun_out/w0_push1.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
    bench.py --gpus 2 --config 2 --host-comm --steps 8 --warmup 0 > gpurun_out/w0_c2_2.json 2> gpurun_out/w0_c2_2.err || exit $?
