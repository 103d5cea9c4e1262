"""Dual-simplex pivots/s on LPG_GEN_DUAL (m = n, default 16384): the deferred
blocks (lpg_dual.hip) against eager rank-1 updates (LPG_FLAG_EAGER), the same
pivots (the logs are compared). Tools only:

    python tools/dual_rate.py [M] [PIVOTS]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402
from linearprogramming_amd import _lib  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
piv = int(sys.argv[2]) if len(sys.argv) > 2 else 640
logs = {}
for name, flags in (("deferred", 0), ("eager", _lib.FLAG_EAGER)):
    e = lpg.Engine(m, 2 * m + 1, flags=flags)
    e.generate(m, 7, lpg.GEN_DUAL)
    e.reserve_log(piv + 64)
    e.solve_dual(8)                      # warm-up (first block's kernels, the log buffer)
    e.device_sync()
    t0 = time.perf_counter()
    r = e.solve_dual(piv)
    e.device_sync()
    dt = time.perf_counter() - t0
    logs[name] = e.get_log()
    print(f"{name:9s} m=n={m} defer_k={e.info.defer_k}: {r.pivots - 8} dual pivots in {dt:.3f} s = "
          f"{(r.pivots - 8) / dt:.0f} pivots/s, status {r.status_name}, z={r.objective!r}", flush=True)
    e.close()
same = all(np.array_equal(a, b) for a, b in zip(logs["deferred"], logs["eager"]))
print("identical pivot logs:", same)
