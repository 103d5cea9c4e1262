set -u
for S in 0 64 32; do
LAB_SCATTER=$S LAB_ONLY=w timeout -k 10 120 tools/flush_lab 64 > gpurun_out/lab64_s$S.log 2>&1 || exit $?
done
LAB_SCATTER=32 LAB_ONLY="variant 20" timeout -k 10 120 tools/flush_lab 64 >> gpurun_out/lab64_s32.log 2>&1 || exit $?
LAB_SCATTER=32 LAB_ONLY="variant 8" timeout -k 10 120 tools/flush_lab 32 > gpurun_out/lab32_s32.log 2>&1 || exit $?
