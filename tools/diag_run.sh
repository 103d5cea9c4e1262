set -u
timeout -k 10 200 python tools/diag_mr.py > gpurun_out/diag_mr.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu --force-rccl --steps 256 > gpurun_out/rccl1.json 2>gpurun_out/rccl1.err || exit $?
timeout -k 10 200 python bench.py --no-cpu --steps 256 > gpurun_out/b3.json 2>/dev/null || exit $?
