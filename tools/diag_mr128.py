"""Multi-rank (threads, host transport) vs single-rank vs oracle logs with
128-pivot blocks, at SIZES (m,n;...): where does the row partition first
differ? Diagnostics only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402
from test_gpu_dist import _run_threads  # noqa: E402

lpg.load()
os.environ["LPG_DEFER"] = os.environ.get("DEFER", "128")
npiv = int(os.environ.get("K", "130"))
for spec in os.environ.get("SIZES", "4096,8192;16384,32768").split(";"):
    m, n = (int(x) for x in spec.split(","))
    for world in (2,):
        parts = _run_threads(lpg, world, m, n, 20220518, 0, 0, npiv)
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, 20220518, 0)
        e.solve(npiv, 0)
        k1, r1 = e.get_log()
        if os.environ.get("ORACLE", "1") == "1":
            o = Oracle(m, n + m + 1, nthreads=16)
            o.generate(n, 20220518, 0)
            o.solve(npiv, 0)
            ko, ro = o.get_log()
        else:                       # the single-rank engine is the reference
            ko, ro = k1, r1

        def first(ka, ra, kb, rb):
            bad = np.nonzero((ka != kb) | (ra != rb))[0]
            return int(bad[0]) if len(bad) else None
        print(f"m={m} n={n} world={world}: single vs oracle {first(k1, r1, ko, ro)}; "
              + "; ".join(f"rank{q} vs oracle {first(p['log'][0], p['log'][1], ko, ro)}" for q, p in enumerate(parts)),
              flush=True)
        d = first(parts[0]["log"][0], parts[0]["log"][1], ko, ro)
        if d is not None:
            print("   oracle", list(zip(ko[d - 3:d + 3].tolist(), ro[d - 3:d + 3].tolist())))
            print("   rank0 ", list(zip(parts[0]["log"][0][d - 3:d + 3].tolist(), parts[0]["log"][1][d - 3:d + 3].tolist())))
        e.close()
        if d is not None and os.environ.get("OBJDIFF"):
            # the objective rows after d pivots: which columns differ
            parts = _run_threads(lpg, world, m, n, 20220518, 0, 0, d)
            e = lpg.Engine(m, n + m + 1)
            e.generate(n, 20220518, 0)
            e.solve(d, 0)
            ob = e.get_rows(m, 1)[0]
            for q, p in enumerate(parts):
                bad = np.nonzero(p["obj"] != ob)[0]
                print(f"   after {d}: rank{q} objective row differs in {len(bad)} columns {bad[:10].tolist()}",
                      flush=True)
            e.close()
