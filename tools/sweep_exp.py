"""Config-3 pivots/s of one liblpg build (experiments only): warm-up, then
32 whole blocks timed around enqueue + sync.

    python tools/sweep_exp.py [LIB] [NAME=VALUE ...]

LIB defaults to the in-tree liblpg.so; NAME=VALUE pairs are set in the
environment before the context is created (LPG_DEFER, LPG_REGION, ...)."""
import os
import sys
import time

args = sys.argv[1:]
lib = None
for a in args:
    if "=" in a:
        k, v = a.split("=", 1)
        os.environ[k] = v
    else:
        lib = a

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402

if lib:
    lpg.load(lib)
m, n = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768))
e = lpg.Engine(m, n + m + 1)
e.generate(n, 20220518, 0)
K = e.info.defer_k
nb = int(os.environ.get("BLOCKS", 32))
e.reserve_log((nb + 4) * K)
e.solve(2 * K, 0)
torch.cuda.synchronize()
t0 = time.perf_counter()
e.enqueue(nb * K, 0)
r = e.sync()
dt = time.perf_counter() - t0
label = " ".join(a for a in args) or "liblpg.so"
print(f"{label} m={m} n={n} K={K} wg={e.info.pivot_wg} region={e.info.region}: {nb * K / dt:.0f} pivots/s, "
      f"{dt / nb * 1e3:.3f} ms/block, {dt / (nb * K) * 1e6:.2f} us/pivot, pivots {r.pivots}", flush=True)
