"""Generate tests/golden/config5_solve.json: BASELINE config 5's whole
two-phase solve (m = n = 8192, GEN_ARTIFICIAL, splitmix64 seed 20220518,
Bland, pivot cap 20000) by the C oracle (oracle/liblpo.so, OpenMP): status,
pivot count, the objective's float.hex, the whole (entering, leaving) log,
and the digests (tests/golden/trajectory.py) of the basis, column 0, the
objective row and 67 sampled rows. Run in the build container (~10 min on 8
cores):

    python tests/golden/make_config5_golden.py

The GPU test and bench.py's config-5 parity leg compare against it instead of
re-running the oracle on the GPU box (47 s of the GPU suite before).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import trajectory as T  # noqa: E402
from oracle.lpo import GEN_ARTIFICIAL, RULE_BLAND, STATUS_NAMES, Oracle  # noqa: E402

M = N = 8192
SEED, CAP = 20220518, 20000
ART_FIRST = 1 + N + (M + 1) // 2
FIXTURE = os.path.join(HERE, "config5_solve.json")


def sample_rows():
    """The rows the GPU test compares: 64 drawn with numpy's PCG64 seed 5, the ends, and the objective row."""
    rng = np.random.default_rng(5)
    return sorted(set(rng.choice(M, 64, replace=False).tolist()) | {0, M - 1, M})


def main():
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    o = Oracle(M, N + M + 1, nthreads=threads)
    o.generate(N, SEED, GEN_ARTIFICIAL)
    t0 = time.time()
    res = o.solve_two_phase(ART_FIRST, None, CAP, RULE_BLAND)
    k, r = o.get_log()
    rows = sample_rows()
    c0 = np.concatenate([o.get_rows(i, min(1024, M - i))[:, 0] for i in range(0, M, 1024)])
    fix = {"what": "BASELINE config 5 (GEN_ARTIFICIAL m=n=8192, seed 20220518), two-phase, Bland, cap 20000, by "
                   "oracle/liblpo.so; digests per tests/golden/trajectory.py",
           "generator": "tests/golden/make_config5_golden.py", "m": M, "n": N, "seed": SEED, "cap": CAP,
           "art_first": ART_FIRST, "status": STATUS_NAMES[res.status], "pivots": int(res.pivots),
           "objective_hex": float(res.objective).hex(), "log_k": [int(x) for x in k], "log_r": [int(x) for x in r],
           "basis": T.digest(o.get_basis()), "column0": T.digest(c0), "rows": rows,
           "row_digests": [T.digest(o.get_rows(i, 1)[0]) for i in rows]}
    with open(FIXTURE, "w") as f:
        json.dump(fix, f, separators=(",", ":"))
        f.write("\n")
    print(f"wrote {FIXTURE}: {fix['status']} after {fix['pivots']} pivots, z={res.objective!r}, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
