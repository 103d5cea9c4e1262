set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -k "pivot_block_sizes" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_nt.log 2>&1 || exit $?
for nt in 64 128 256; do
LPG_PIVOT_NT=$nt timeout -k 10 200 python tools/diag_c3.py > gpurun_out/diag_c3_$nt.log 2>&1 || exit $?
LPG_PIVOT_NT=$nt timeout -k 10 200 python bench.py --no-cpu --steps 256 > gpurun_out/nt_$nt.json 2>/dev/null || exit $?
done
