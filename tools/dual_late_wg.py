"""A/B of the deferred dual's optimality peek with late workgroups.

usage: python tools/dual_late_wg.py LIB [LIB ...]

Runs tests/test_dual.py::test_gpu_dual_optimal_with_late_workgroups's LP
(m = 32, n = 2.5M: ~4900 column blocks of k_dual_row_d) through each given
liblpg build and counts the objective-row entries that differ from the
oracle's. Used to show that the round-3 build (tools/liblpg_r03.so, from
commit 1c743e0) loses the owed update on late workgroups and the fixed one
does not (profiles/r04_dual_late_wg.log). Each LIB runs in its own process.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(lib):
    import numpy as np

    import linearprogramming_amd as lpg
    from oracle.lpo import GEN_DUAL, Oracle
    lpg.load(lib)
    m, n, seed = 32, 2_500_000, 11
    o = Oracle(m, n + m + 1, nthreads=16)
    o.generate(n, seed, GEN_DUAL)
    ro = o.solve_dual(100_000)
    oo = o.get_rows(m, 1)[0]
    for rep in range(3):
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, seed, lpg.GEN_DUAL)
        r = e.solve_dual(100_000)
        eo = e.get_rows(m, 1)[0]
        bad = np.flatnonzero(eo.view(np.uint64) != oo.view(np.uint64))
        print(f"{os.path.basename(lib)} run {rep}: status {r.status_name} pivots {r.pivots} (oracle {ro.pivots}) "
              f"objective-row mismatches {bad.size}" + (f", first {bad[:4].tolist()}" if bad.size else ""), flush=True)
        e.close()


if __name__ == "__main__":
    if len(sys.argv) > 2 or (len(sys.argv) == 2 and sys.argv[1] != "--one"):
        rc = 0
        for lib in sys.argv[1:]:
            rc |= subprocess.run([sys.executable, __file__, "--one"], env=dict(os.environ, DLW_LIB=lib)).returncode
        sys.exit(rc)
    one(os.environ["DLW_LIB"])
