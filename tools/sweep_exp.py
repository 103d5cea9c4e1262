"""Config-3 pivots/s of one liblpg build (argv[1], default the in-tree one):
warm-up, then 32 whole blocks timed around enqueue + sync. Experiments only."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402

if len(sys.argv) > 1:
    lpg.load(sys.argv[1])
m, n = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768))
e = lpg.Engine(m, n + m + 1)
e.generate(n, 20220518, 0)
K = e.info.defer_k
e.reserve_log(40 * K)
e.solve(2 * K, 0)
torch.cuda.synchronize()
t0 = time.perf_counter()
e.enqueue(32 * K, 0)
r = e.sync()
dt = time.perf_counter() - t0
print(f"{os.path.basename(sys.argv[1]) if len(sys.argv) > 1 else 'liblpg.so'} m={m} n={n} K={K} "
      f"flush={os.environ.get('LPG_FLUSH_KERNEL', 'default')}: {32 * K / dt:.0f} pivots/s, "
      f"{dt / 32 * 1e3:.3f} ms/block, pivots {r.pivots}")
