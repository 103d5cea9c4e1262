"""Objective row of the deferred engine vs the oracle after each of the first pivots (config 3)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402

m, n = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768))
o = Oracle(m, n + m + 1)
o.generate(n, 20220518, 0)
e = lpg.Engine(m, n + m + 1)
e.generate(n, 20220518, 0)
for t in range(5):
    o.solve(1, 0)
    e.enqueue(1, 0)
    e.sync()
    eo = e.get_rows(m, 1)[0]
    oo = o.get_rows()[m]
    d = np.nonzero(eo != oo)[0]
    k, r = e.get_log()
    ok, orr = o.get_log()
    print(f"after pivot {t}: log gpu {(int(k[-1]), int(r[-1]))} cpu {(int(ok[-1]), int(orr[-1]))}; objective row differs at "
          f"{len(d)} columns {d[:12].tolist()}", flush=True)
    if len(d):
        j = d[:6]
        print("   gpu", eo[j].tolist(), "\n   cpu", oo[j].tolist(), flush=True)
