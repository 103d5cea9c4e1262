"""Divergence hunts for the engine (diagnostics only; replaces the round-1..3
one-off tools/diag_*.py scripts).

  python tools/diag.py log  --m M --n N [--pivots K] [--ref oracle|engine]
                            [--variant "LPG_DEFER=64,LPG_SLOW_PIVOT=0" ...] [--world W]
      First K pivots of the engine under each variant (environment settings
      read at context creation; --world: W ranks as threads over the host
      transport) against the reference run: the C oracle, or for sizes the
      oracle cannot hold quickly the single-rank engine with default
      settings. Prints the first differing pivot per variant.

  python tools/diag.py step --m M --n N [--pivots K] | --kat CASE [--rule R]
      Pivot by pivot against the oracle: status, log, and the first entries
      of the objective row and the constraint rows that differ.

  python tools/diag.py state --m M --n N --pivots P [--rows i,j,..] [--world W]
      W ranks (threads, host transport) against one rank after P pivots: the
      objective row, the given rows, the log; then one more pivot from the
      materialised tableau, compared again.

Synthetic LPs: --kind 0 dense (default), 1 degenerate, 3 dual; --seed.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _env(variant: str) -> dict:
    return dict(kv.split("=", 1) for kv in variant.split(",") if kv)


def _first_diff(ka, ra, kb, rb):
    n = min(len(ka), len(kb))
    bad = np.nonzero((ka[:n] != kb[:n]) | (ra[:n] != rb[:n]))[0]
    return int(bad[0]) if len(bad) else None


def _threads(lpg, world, m, n, seed, kind, body):
    """Run body(engine, rank) on `world` ranks as threads over the host transport."""
    from test_gpu_dist import ThreadComm
    comm = ThreadComm(world)
    out = [None] * world

    def worker(rank):
        e = lpg.Engine(m, n + m + 1, world=world, rank=rank)
        e.comm_init_host(lambda b: comm.allgather(rank, b), lambda a: comm.allreduce(rank, a))
        e.generate(n, seed, kind)
        out[rank] = body(e, rank)
        e.close()
    th = [threading.Thread(target=worker, args=(q,)) for q in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


def cmd_log(a, lpg):
    from oracle.lpo import Oracle
    m, n = a.m, a.n
    if a.ref == "oracle":
        o = Oracle(m, n + m + 1, nthreads=a.threads)
        o.generate(n, a.seed, a.kind)
        o.solve(a.pivots, a.rule)
        ref = o.get_log()
    else:
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, a.seed, a.kind)
        e.solve(a.pivots, a.rule)
        ref = e.get_log()
        e.close()
    print(f"reference ({a.ref}): {len(ref[0])} pivots", flush=True)
    for v in a.variant or [""]:
        saved = dict(os.environ)
        os.environ.update(_env(v))
        try:
            if a.world > 1:
                logs = _threads(lpg, a.world, m, n, a.seed, a.kind,
                                lambda e, rank: (e.solve(a.pivots, a.rule), e.get_log())[1])
            else:
                e = lpg.Engine(m, n + m + 1)
                e.generate(n, a.seed, a.kind)
                e.solve(a.pivots, a.rule)
                logs = [e.get_log()]
                e.close()
        finally:
            os.environ.clear()
            os.environ.update(saved)
        for q, (k, r) in enumerate(logs):
            d = _first_diff(k, r, *ref)
            where = "same" if d is None else f"first difference at pivot {d}: ({k[d]}, {r[d]}) vs ({ref[0][d]}, {ref[1][d]})"
            print(f"[{v or 'default'}] rank {q}: {len(k)} pivots, {where}", flush=True)


def cmd_step(a, lpg):
    from oracle.lpo import Oracle
    if a.kat:
        from util import kat_cases, kat_tableau
        case = next(c for c in kat_cases() if c["name"] == a.kat)
        T = kat_tableau(case)
        m, ncols = T.shape[0] - 1, T.shape[1]
        e, o = lpg.Engine(m, ncols), Oracle(m, ncols)
        for x in (e, o):
            x.load_tableau(T, case["basis"])
    else:
        m, ncols = a.m, a.n + a.m + 1
        e, o = lpg.Engine(m, ncols), Oracle(m, ncols)
        for x in (e, o):
            x.generate(a.n, a.seed, a.kind)
    for t in range(a.pivots):
        ro = o.solve(1, a.rule)
        e.enqueue(1, a.rule)
        re = e.sync()
        Te, To = e.get_rows(0, m + 1), o.get_rows()
        bo = np.nonzero(Te[m].view(np.uint64) != To[m].view(np.uint64))[0]
        br = np.argwhere(Te[:m].view(np.uint64) != To[:m].view(np.uint64))
        d = _first_diff(*e.get_log(), *o.get_log())
        print(f"pivot {t}: gpu {re.status_name} {re.pivots} / oracle status {ro.status} {ro.pivots}; log "
              f"{'same' if d is None else 'differs at ' + str(d)}; objective row: {len(bo)} differ {bo[:6].tolist()}; "
              f"rows: {len(br)} differ {br[:4].tolist()}", flush=True)
        if ro.status != 4 and ro.status != 0:
            break


def cmd_state(a, lpg):
    m, n = a.m, a.n
    rows = [int(x) for x in a.rows.split(",")] if a.rows else [0, m - 1]

    def body(e, rank):
        e.solve(a.pivots, a.rule)
        info = e.info
        got = {"obj": e.get_rows(m, 1)[0]}
        for i in rows:
            if info.row0 <= i < info.row0 + info.nrows:
                got[f"row{i}"] = e.get_rows(i, 1)[0]
        e.solve(1, a.rule)
        got["log"] = e.get_log()
        got["obj+1"] = e.get_rows(m, 1)[0]
        return got
    parts = _threads(lpg, a.world, m, n, a.seed, a.kind, body)
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, a.seed, a.kind)
    one = body(e, 0)
    e.close()
    for q, p in enumerate(parts):
        for key, v in p.items():
            if key == "log":
                d = _first_diff(*v, *one["log"])
                print(f"rank {q} log: {'same' if d is None else 'first difference at ' + str(d)}", flush=True)
            else:
                bad = np.nonzero(v.view(np.uint64) != one[key].view(np.uint64))[0]
                print(f"rank {q} {key}: {len(bad)} entries differ {bad[:8].tolist()}", flush=True)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cmd", choices=["log", "step", "state"])
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--seed", type=int, default=20220518)
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--rule", type=int, default=0)
    ap.add_argument("--pivots", type=int, default=8)
    ap.add_argument("--ref", choices=["oracle", "engine"], default="oracle")
    ap.add_argument("--variant", action="append")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rows", default="")
    ap.add_argument("--kat", default="")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import linearprogramming_amd as lpg
    lpg.load()
    {"log": cmd_log, "step": cmd_step, "state": cmd_state}[a.cmd](a, lpg)


if __name__ == "__main__":
    main()
