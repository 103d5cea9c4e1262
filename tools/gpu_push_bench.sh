#!/bin/bash
# Owner-push exchange stand-ins on one MI355X: 1 rank pushing to itself; 2 processes sharing the GPU (gloo setup, IPC push).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1.json 2> gpurun_out/bench_push1.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --host-comm --steps 16 > gpurun_out/bench_push2.json 2> gpurun_out/bench_push2.err || exit $?
