#!/bin/bash
# round-4 GPU batch 8: config-4 pair phases (K = 96) and kernel stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1 name=$2; shift 2; echo "[r04] $name" >&2; timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "[r04] $name failed rc=$rc" >&2; tail -5 "gpurun_out/r04_$name.log"; exit $rc; }; }
step 300 phase_probe_c4 env M=65536 N=131072 python -u tools/phase_probe.py
step 400 prof_c4 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 -- python3 -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu
find gpurun_out/prof_c4 -name '*stats*' > gpurun_out/r04_prof_c4_files.txt
