"""Randomised parity soak (test infrastructure; the oracle is the checker):
many random LPs through the engine and oracle/liblpo.so, every pivot log,
basis, status, objective and whole tableau compared (np.array_equal), under
random engine settings (block size, persistent launch on/off, column trade
on/off, flush kernel, pricing rule, generator kind, primal / two-phase /
Big-M / dual). Prints one line per case and a summary; exits 1 on the first
mismatch (the case's settings are printed so it can be replayed).

    python tools/soak.py [seconds] [seed] [big]     (big: m 1024-4097, n 2048-8192)
"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import GEN_ARTIFICIAL, GEN_DEGENERATE, GEN_DENSE, GEN_DUAL, Oracle  # noqa: E402

# per-context knobs (read at lpg_create); the process-wide ones (LPG_PIVOT_XCD1,
# LPG_FLUSH_W96, LPG_FLUSH_ROWS, ...) are read once per process: set them for a
# whole soak run instead
KNOBS = ("LPG_DEFER", "LPG_PERSIST", "LPG_NO_REORDER", "LPG_FLUSH_KERNEL", "LPG_PERSIST_WG", "LPG_REGION",
         "LPG_FLUSH_XCD", "LPG_FLUSH_TLIVE", "LPG_MOVE_UNIT")


def case(rng: random.Random, big: bool = False):
    mode = rng.choice(["primal", "primal", "primal", "two_phase", "big_m", "dual"])
    if big:    # sizes where the pass has many items and the tail, the select grid folds (m % 256 == 0)
        m = rng.choice([1024, 2047, 2048, 4095, 4096, 4097])
        n = rng.choice([2048, 6000, 8192])
    else:
        m = rng.choice([16, 33, 64, 100, 255, 256, 257, 300, 511, 512, 700, 1024, 1500])
        n = rng.choice([16, 48, 100, 257, 500, 1000, 2000, 3000])
    env = {
        "LPG_DEFER": str(rng.choice([0, 1, 2, 5, 8, 16, 31, 32, 33, 48, 63, 64, 65, 77, 96, 100, 128])),
        "LPG_PERSIST": rng.choice(["0", "1"]),
        "LPG_NO_REORDER": rng.choice(["0", "1"]),
        "LPG_FLUSH_KERNEL": rng.choice(["m", "w", "w"]),
        "LPG_REGION": rng.choice(["0", "1", "1"]),
        "LPG_FLUSH_XCD": rng.choice(["0", "1", "1", "h2", "h8"]),
        "LPG_FLUSH_TLIVE": rng.choice(["0", "1", "1"]),
        "LPG_MOVE_UNIT": rng.choice(["0", "1", "1"]),
    }
    if rng.random() < 0.3:
        env["LPG_PERSIST_WG"] = str(rng.choice([8, 16, 32, 64, 128]))
    rule = rng.choice([0, 1]) if mode != "dual" else 0
    kind = {"primal": rng.choice([GEN_DENSE, GEN_DEGENERATE]), "two_phase": GEN_ARTIFICIAL,
            "big_m": GEN_ARTIFICIAL, "dual": GEN_DUAL}[mode]
    seed = rng.randrange(1 << 30)
    cap = rng.choice([50, 200, 1000]) if big else rng.choice([50, 200, 1000, 5000])
    return dict(mode=mode, m=m, n=n, env=env, rule=rule, kind=kind, seed=seed, cap=cap)


def run(c):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(c["env"])
    m, n, mode = c["m"], c["n"], c["mode"]
    big = mode == "big_m"
    e = lpg.Engine(m, n + m + 1, flags=lpg._lib.FLAG_BIG_M if big else 0)
    for k in KNOBS:
        os.environ.pop(k, None)
    o = Oracle(m, n + m + 1, nthreads=8, nobj=2 if big else 1)
    try:
        e.generate(n, c["seed"], c["kind"])
        o.generate(n, c["seed"], c["kind"])
        art = 1 + n + (m + 1) // 2
        if mode == "primal":
            r, ro = e.solve(c["cap"], c["rule"]), o.solve(c["cap"], c["rule"])
        elif mode == "two_phase":
            r, ro = e.solve_two_phase(art, None, c["cap"], c["rule"]), o.solve_two_phase(art, None, c["cap"], c["rule"])
        elif mode == "big_m":
            r, ro = e.solve_big_m(art, None, c["cap"], c["rule"]), o.solve_big_m(art, None, c["cap"], c["rule"])
        else:
            r, ro = e.solve_dual(c["cap"]), o.solve_dual(c["cap"])
        rows = m + (2 if big else 1)
        bad = []
        if r.status != ro.status:
            bad.append(f"status {r.status} vs {ro.status}")
        if r.pivots != ro.pivots:
            bad.append(f"pivots {r.pivots} vs {ro.pivots}")
        ek, er = e.get_log()
        ok_, or_ = o.get_log()
        if not (np.array_equal(ek, ok_) and np.array_equal(er, or_)):
            bad.append("log")
        if not np.array_equal(e.get_basis(), o.get_basis()):
            bad.append("basis")
        T, To = e.get_rows(0, rows), o.get_rows()
        if not np.array_equal(T, To):
            d = np.flatnonzero(~((T == To) | (np.isnan(T) & np.isnan(To))))
            if d.size:
                i, j = np.unravel_index(d[0], T.shape)
                bad.append(f"tableau ({d.size} entries, first [{i},{j}] {T[i, j]!r} vs {To[i, j]!r})")
        return r, bad
    finally:
        e.close()
        o.close()


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20261017
    big = len(sys.argv) > 3 and sys.argv[3] == "big"
    rng = random.Random(seed)
    lpg.load()
    t0 = time.time()
    n = 0
    while time.time() - t0 < budget:
        c = case(rng, big)
        try:
            r, bad = run(c)
        except lpg.LPGError as ex:   # a refused combination: reported, not counted as parity
            print(f"     {c['mode']:9s} m={c['m']} n={c['n']} env={c['env']} -> REFUSED: {ex}", flush=True)
            continue
        n += 1
        tag = "MISMATCH " + "; ".join(bad) if bad else "ok"
        print(f"{n:4d} {c['mode']:9s} m={c['m']:5d} n={c['n']:5d} rule={c['rule']} kind={c['kind']} seed={c['seed']} "
              f"cap={c['cap']} env={c['env']} -> {r.status_name} {r.pivots} pivots: {tag}", flush=True)
        if bad:
            sys.exit(1)
    print(f"soak: {n} cases, all bitwise equal to the oracle ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
