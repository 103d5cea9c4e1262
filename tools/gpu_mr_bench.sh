#!/bin/bash
# bench.py end to end with 2 and 3 ranks on ONE GPU at config 2 (13-workgroup persistent launches: all resident at
# once), owner push + the multi-rank persistent launch, host-comm setup; and the same with the pair.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 \
    bench.py --gpus 2 --config 2 --host-comm --steps 32 > gpurun_out/mrb_c2_2.json 2> gpurun_out/mrb_c2_2.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29552 \
    bench.py --gpus 3 --config 2 --host-comm --steps 32 > gpurun_out/mrb_c2_3.json 2> gpurun_out/mrb_c2_3.err || exit $?
LPG_PERSIST_MR=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29553 \
    bench.py --gpus 2 --config 2 --host-comm --steps 32 > gpurun_out/mrb_c2_2_pair.json 2> gpurun_out/mrb_c2_2_pair.err || exit $?
