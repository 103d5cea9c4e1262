#!/bin/bash
# Owner-push stand-ins on one MI355X: 1 rank pushing to itself with k_pivot_block's multi-rank form and with the
# two-kernel pair; 2 processes sharing the GPU with the pair (two 227-workgroup persistent launches cannot share
# 256 CUs; one process per GPU, the driver's layout, runs the persistent form).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1.json 2> gpurun_out/bench_push1.err || exit $?
LPG_PERSIST_MR=0 timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1_pair.json 2> gpurun_out/bench_push1_pair.err || exit $?
LPG_PERSIST_MR=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --host-comm --steps 16 > gpurun_out/bench_push2.json 2> gpurun_out/bench_push2.err || exit $?
