"""Config-3 first-pivot logs of the HIP engine under block sizes / pivot paths vs the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402

m, n, K = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768)), int(os.environ.get("K", 8))
o = Oracle(m, n + m + 1)
o.generate(n, 20220518, 0)
o.solve(K, 0)
ok, orr = o.get_log()
print("oracle", list(zip(ok.tolist(), orr.tolist())), flush=True)
for defer, slow, nt in [("64", "0", os.environ.get("LPG_PIVOT_NT", "256"))]:
        os.environ["LPG_DEFER"] = defer
        os.environ["LPG_SLOW_PIVOT"] = slow
        os.environ["LPG_PIVOT_NT"] = nt
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, 20220518, 0)
        e.solve(K, 0)
        k, r = e.get_log()
        same = k.tolist() == ok.tolist() and r.tolist() == orr.tolist()
        print(f"defer={defer} slow={slow} nt={nt} same={same}", list(zip(k.tolist(), r.tolist())), flush=True)
        e.close()
