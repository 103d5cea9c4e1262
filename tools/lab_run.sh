set -u
timeout -k 10 120 tools/flush_lab 96 > gpurun_out/lab96.log 2>&1 || exit $?
timeout -k 10 120 tools/flush_lab 128 > gpurun_out/lab128.log 2>&1 || exit $?
