"""First-pivot logs (fast deferred pair) vs the oracle over sizes, to bracket a size-dependent fault."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402

K = 4
for m in [int(x) for x in os.environ.get("MS", "8192 12288 16319 16320 16383 16384").split()]:
    n = int(os.environ.get("NRATIO", 2)) * m
    o = Oracle(m, n + m + 1)
    o.generate(n, 20220518, 0)
    o.solve(K, 0)
    ok, orr = o.get_log()
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, 20220518, 0)
    e.solve(K, 0)
    k, r = e.get_log()
    eo = e.get_rows(m, 1)[0]
    oo = o.get_rows()[m]
    print(f"m={m} n={n} log_same={k.tolist() == ok.tolist() and r.tolist() == orr.tolist()} "
          f"obj_same={bool((eo == oo).all())}", flush=True)
    e.close()
    o.close()
