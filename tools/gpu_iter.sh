set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defer.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_defer.log 2>&1 || exit $?
for K in 64 32; do
timeout -k 10 200 python bench.py --defer $K --no-cpu > gpurun_out/b3_k$K.json 2>>gpurun_out/b.err || exit $?
timeout -k 10 200 python bench.py --config 2 --steps 1536 --defer $K --no-cpu > gpurun_out/b2_k$K.json 2>>gpurun_out/b.err || exit $?
done
