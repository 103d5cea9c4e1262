set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --force-rccl --no-cpu > gpurun_out/mr_rccl.json 2> gpurun_out/mr.err || exit $?
LPG_GRAPH_RCCL=1 timeout -k 10 200 python bench.py --force-rccl --no-cpu > gpurun_out/mr_rccl_graph.json 2>> gpurun_out/mr.err || exit $?
timeout -k 10 200 python bench.py --no-cpu --steps 1024 > gpurun_out/c3_1024.json 2>> gpurun_out/mr.err || exit $?
