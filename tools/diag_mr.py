"""Multi-rank (threads, host comm) deferred engine vs the oracle after n pivots."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402
from test_gpu_dist import _run_threads  # noqa: E402

m, n, seed = 96, 160, 777
for npiv in [1, 2, 3, 4, 5, 8, 16, 33, 40]:
    parts = _run_threads(lpg, 2, m, n, seed, 0, 0, npiv)
    o = Oracle(m, n + m + 1)
    o.generate(n, seed, 0)
    o.solve(npiv, 0)
    k, r = o.get_log()
    T = o.get_rows()
    rows = np.vstack([p["rows"] for p in parts])
    same_log = all(np.array_equal(p["log"][0], k) and np.array_equal(p["log"][1], r) for p in parts)
    print(npiv, "log", same_log, "obj", [bool(np.array_equal(p["obj"], T[m])) for p in parts],
          "rows", bool(np.array_equal(rows, T[:m])), "maxdiff", float(np.abs(rows - T[:m]).max()), flush=True)
    if not same_log:
        print("  gpu", list(zip(parts[0]["log"][0].tolist(), parts[0]["log"][1].tolist())))
        print("  cpu", list(zip(k.tolist(), r.tolist())))
        break
