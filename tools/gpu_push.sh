#!/bin/bash
# Owner-push exchange: the multi-rank GPU tests, then the 1-rank and 2-process stand-ins.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_push.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1.json 2> gpurun_out/bench_push1.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --host-comm --steps 16 > gpurun_out/bench_push2.json 2> gpurun_out/bench_push2.err || exit $?
