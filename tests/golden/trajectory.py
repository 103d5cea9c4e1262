"""Config 3's pinned trajectory: the fixture format and its digests.

`config3_2400.json` (made by `make_config3_golden.py` from the C oracle,
oracle/liblpo.so, in the build container) holds the first 2,400 Dantzig pivots
of BASELINE config 3 (m = 16384, n = 32768, splitmix64 seed 20220518): the
(entering, leaving) log, and at every 96th pivot the objective's float.hex,
the basis digest and the digests of column 0, the objective row and 16 fixed
constraint rows. 2,400 = 25 blocks of 96 = bench.py's driver form
(`--warmup 5 --steps 20`); its default form (`--warmup 2 --steps 16`) ends at
1,728, also a checkpoint. The reference has no pivot loop (simplex.c:40-65),
so the restatement is the checker.

Pure numpy: the generator, `tests/test_gpu_trajectory.py` and bench.py's
parity leg share these functions; none of them touches oracle/ at run time
except the generator.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "config3_2400.json")
M, N, SEED, PIVOTS, EVERY = 16384, 32768, 20220518, 2400, 96
# fixed constraint rows whose digests are stored (ends, block edges of the
# 2- / 4- / 8-way row partitions, and a spread in between)
ROWS = (0, 1, 2047, 2048, 4095, 4096, 5000, 8191, 8192, 9999, 12287, 12288, 14336, 16381, 16382, 16383)


def digest(a) -> str:
    """sha256 of an array's little-endian float64 / int64 bytes."""
    a = np.ascontiguousarray(a)
    if a.dtype.kind == "f":
        a = a.astype("<f8", copy=False)
    else:
        a = a.astype("<i8", copy=False)
    return hashlib.sha256(a.tobytes()).hexdigest()


def snapshot(objective: float, basis, column0, objective_row, rows) -> dict:
    """The checkpoint record: rows is len(ROWS) x ncols, in ROWS order."""
    return {"objective_hex": float(objective).hex(), "basis": digest(basis), "column0": digest(column0),
            "objective_row": digest(objective_row), "rows": [digest(r) for r in rows]}


def load(path: str = FIXTURE) -> dict:
    with open(path) as f:
        return json.load(f)


def compare(fix: dict, k, r, snaps: dict) -> dict:
    """Compare a log (k, r) and {pivots: snapshot} with the fixture (a snapshot
    may hold a subset of the fields: only those are compared). Returns
    {"pivots_compared", "log_equal", "first_mismatch", "checkpoints": {p: {field: bool}}, "ok"}."""
    k = np.asarray(k, dtype=np.int64)
    r = np.asarray(r, dtype=np.int64)
    fk = np.asarray(fix["log_k"], dtype=np.int64)
    fr = np.asarray(fix["log_r"], dtype=np.int64)
    n = min(len(k), len(fk))
    bad = np.nonzero((k[:n] != fk[:n]) | (r[:n] != fr[:n]))[0]
    out = {"pivots_compared": int(n), "log_equal": bool(bad.size == 0),
           "first_mismatch": int(bad[0]) if bad.size else None, "checkpoints": {}}
    ok = out["log_equal"] and n > 0
    for p, s in snaps.items():
        ref = fix["checkpoints"].get(str(p))
        if ref is None:
            continue
        res = {key: s[key] == ref[key] for key in ("objective_hex", "basis", "column0", "objective_row", "rows")
               if key in s}
        out["checkpoints"][str(p)] = res
        ok = ok and all(res.values())
    out["ok"] = bool(ok)
    return out
