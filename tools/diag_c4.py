"""Config-4 (65536 x 131072) first-pivot logs of the single-rank engine under
block sizes (eager, 64, 128) and optionally the C oracle (ORACLE=1: 103 GB of
host RAM, minutes): where do they first differ? Diagnostics only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import linearprogramming_amd as lpg  # noqa: E402

m, n, K = int(os.environ.get("M", 65536)), int(os.environ.get("N", 131072)), int(os.environ.get("K", 80))
logs = {}
for defer in os.environ.get("DEFERS", "0,64,128").split(","):
    os.environ["LPG_DEFER"] = defer
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, 20220518, 0)
    e.reserve_log(K + 8)
    r = e.solve(K, 0)
    k, rr = e.get_log()
    logs[defer] = (k.copy(), rr.copy(), r.objective)
    print(f"defer={defer} pivots={r.pivots} z={r.objective!r} tail={list(zip(k[60:K].tolist(), rr[60:K].tolist()))}",
          flush=True)
    e.close()
if os.environ.get("ORACLE") == "1":
    from oracle.lpo import Oracle
    o = Oracle(m, n + m + 1, nthreads=16)
    o.generate(n, 20220518, 0)
    res = o.solve(K, 0)
    k, rr = o.get_log()
    logs["oracle"] = (k, rr, res.objective)
    print(f"oracle pivots={res.pivots} z={res.objective!r} tail={list(zip(k[60:K].tolist(), rr[60:K].tolist()))}",
          flush=True)
names = list(logs)
for a in names:
    for b in names:
        if a < b:
            ka, ra, za = logs[a]
            kb, rb, zb = logs[b]
            bad = np.nonzero((ka != kb) | (ra != rb))[0]
            print(f"{a} vs {b}: first difference at pivot {bad[0] if len(bad) else None}, z equal {za == zb}", flush=True)
