set -u
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pr3 -o run -- python3 bench.py --steps 512 --warmup 64 --no-cpu > gpurun_out/pr3.json 2>/dev/null || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pr5 -o run -- python3 bench.py --config 5 --no-cpu > gpurun_out/pr5.json 2>/dev/null || exit $?
