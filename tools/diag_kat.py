"""One KAT case on the engine vs the oracle, pivot by pivot (objective row, status)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import Oracle  # noqa: E402
from util import kat_cases, kat_tableau  # noqa: E402

name = os.environ.get("CASE", "a6_decimals.txt")
rule = int(os.environ.get("RULE", 1))
case = next(c for c in kat_cases() if c["name"] == name)
T = kat_tableau(case)
m = T.shape[0] - 1
print("T=\n", T, "basis", case["basis"])
e = lpg.Engine(m, T.shape[1])
o = Oracle(m, T.shape[1])
for x in (e, o):
    x.load_tableau(T, case["basis"])
for t in range(4):
    ro = o.solve(1, rule)
    e.enqueue(1, rule)
    re = e.sync()
    print(f"pivot {t}: gpu status {re.status_name} piv {re.pivots} log {e.get_log()}  cpu status {ro.status} log {o.get_log()}")
    print("   gpu rows\n", e.get_rows(0, m + 1), "\n   cpu rows\n", o.get_rows())
