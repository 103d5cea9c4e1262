#!/bin/bash
# Multi-rank k_pivot_block: the distributed tests (1-rank self-push, 2-3 processes), the block tests, then the
# owner-push stand-ins on one GPU (1 rank pushing to itself: the multi-rank form and the pair; 2 processes: the pair).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mrp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_defer.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_mrp2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1.json 2> gpurun_out/bench_push1.err || exit $?
LPG_PERSIST_MR=0 timeout -k 10 200 python bench.py --force-push --steps 32 --no-cpu > gpurun_out/bench_push1_pair.json 2> gpurun_out/bench_push1_pair.err || exit $?
LPG_PERSIST_MR=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --host-comm --steps 16 > gpurun_out/bench_push2.json 2> gpurun_out/bench_push2.err || exit $?
