set -u
for nt in 256 128 64; do
  LPG_PIVOT_NT=$nt timeout -k 10 200 python bench.py --no-cpu --steps 256 > gpurun_out/nt_$nt.json 2>/dev/null || exit $?
done
