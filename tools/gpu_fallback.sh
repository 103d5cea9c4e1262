#!/bin/bash
# Robustness: 2 ranks on ONE GPU with the default settings. Their persistent launches (227 workgroups each) cannot
# both be resident, so the owner-push warm-up must time out (bounded waits) and bench.py must fall back to the
# collectives and still print one valid line.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
    bench.py --gpus 2 --host-comm --steps 4 --warmup 1 > gpurun_out/bench_fallback.json 2> gpurun_out/bench_fallback.err || exit $?
