"""Randomised parity soak of the row partition (test infrastructure; the
oracle is the checker): each case runs W = 2-4 ranks as threads of this
process on the one GPU (host collectives in-process, optionally the
owner-push exchange between the ranks' buffers), under random block sizes,
launch forms and solve modes, and compares every rank's status, pivot log,
basis, objective row(s) and its own constraint rows with the oracle
(np.array_equal). Exits 1 on the first mismatch.

    python tools/soak_dist.py [seconds] [seed]

With LPG_PUSH_SHARED_QUEUES=1 in the environment the owner push runs between
the rank threads (the multi-rank pivot launch, in region mode where LPG_REGION
allows and the column trade is on); exchange timeouts are then counted, not
compared (threads share the process's hardware queues). SOAK_DIST_FOCUS=region
draws only cases of that launch in region mode.
"""
import os
import random
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402
from oracle.lpo import GEN_ARTIFICIAL, GEN_DEGENERATE, GEN_DENSE, GEN_DUAL, Oracle  # noqa: E402

KNOBS = ("LPG_DEFER", "LPG_PERSIST_MR", "LPG_NO_REORDER", "LPG_FLUSH_XCD", "LPG_REGION")


class Comm:
    """allgather / allreduce-sum between rank threads (the engine's allreduces
    have one contributor, the other ranks send signed zeros)."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world

    def allgather(self, rank, data):
        self.slots[rank] = data
        self.bar.wait()
        out = b"".join(self.slots)
        self.bar.wait()
        return out

    def allreduce(self, rank, arr):
        self.slots[rank] = arr
        self.bar.wait()
        acc = self.slots[0].copy()
        for q in range(1, self.world):
            acc = acc + self.slots[q]
        self.bar.wait()
        return acc


def case(rng):
    mode = rng.choice(["primal", "primal", "two_phase", "big_m", "dual"])
    world = rng.choice([2, 3, 4])
    m = rng.choice([12, 40, 64, 100, 257, 300, 511, 700])
    n = rng.choice([16, 60, 200, 500, 1000])
    env = {"LPG_DEFER": str(rng.choice([0, 1, 3, 8, 16, 32, 33, 64, 77, 96, 128])),
           "LPG_PERSIST_MR": rng.choice(["0", "1"]), "LPG_NO_REORDER": rng.choice(["0", "1"]),
           "LPG_FLUSH_XCD": rng.choice(["0", "1", "h8"]), "LPG_REGION": rng.choice(["0", "1", "1"])}
    push = rng.random() < 0.6
    if os.environ.get("SOAK_DIST_FOCUS") == "region":   # the multi-rank launch in region mode only
        env.update({"LPG_DEFER": str(rng.choice([3, 8, 16, 32, 33, 64, 77, 96])), "LPG_PERSIST_MR": "1",
                    "LPG_NO_REORDER": "0", "LPG_REGION": "1"})
        mode = rng.choice(["primal", "primal", "two_phase"])
        push = True
    rule = rng.choice([0, 1]) if mode != "dual" else 0
    kind = {"primal": rng.choice([GEN_DENSE, GEN_DEGENERATE]), "two_phase": GEN_ARTIFICIAL, "big_m": GEN_ARTIFICIAL,
            "dual": GEN_DUAL}[mode]
    return dict(mode=mode, world=world, m=m, n=n, env=env, push=push, rule=rule, kind=kind,
                seed=rng.randrange(1 << 30), cap=rng.choice([40, 300, 2000]))


def run(c):
    W, m, n, mode = c["world"], c["m"], c["n"], c["mode"]
    big = mode == "big_m"
    comm = Comm(W)
    out = [None] * W
    errs = []
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(c["env"])
    engines = [lpg.Engine(m, n + m + 1, world=W, rank=r, flags=lpg._lib.FLAG_BIG_M if big else 0) for r in range(W)]
    for k in KNOBS:
        os.environ.pop(k, None)
    art = 1 + n + (m + 1) // 2

    def worker(r):
        e = engines[r]
        try:
            e.comm_init_host(lambda b: comm.allgather(r, b), lambda a: comm.allreduce(r, a))
            if c["push"]:
                # ranks as threads of one process share its hardware queues: the push is
                # refused at attach time (lpg_ctx.hip) unless LPG_PUSH_SHARED_QUEUES=1 is set
                # for this run; a refused case continues on the collectives (no pivot ran yet)
                allb = comm.allgather(r, e.push_base().to_bytes(8, "little"))
                try:
                    e.comm_init_push_local([int.from_bytes(allb[8 * q:8 * q + 8], "little") for q in range(W)])
                except lpg.LPGError as ex:
                    if "owner-push exchange refused" not in str(ex):
                        raise
                    c["push_refused"] = True
            e.generate(n, c["seed"], c["kind"])
            if mode == "primal":
                res = e.solve(c["cap"], c["rule"])
            elif mode == "two_phase":
                res = e.solve_two_phase(art, None, c["cap"], c["rule"])
            elif mode == "big_m":
                res = e.solve_big_m(art, None, c["cap"], c["rule"])
            else:
                res = e.solve_dual(c["cap"])
            info = e.info
            out[r] = dict(res=res, log=e.get_log(), basis=e.get_basis(), rows=e.get_rows(info.row0, info.nrows),
                          obj=e.get_rows(m, 2 if big else 1))
        except Exception as ex:
            errs.append(repr(ex))
            comm.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    for e in engines:
        e.close()
    if errs:   # an engine error (refused combination or a real fault): reported, the case is not compared
        return None, [f"error: {errs[0]}"]
    o = Oracle(m, n + m + 1, nthreads=8, nobj=2 if big else 1)
    o.generate(n, c["seed"], c["kind"])
    if mode == "primal":
        ro = o.solve(c["cap"], c["rule"])
    elif mode == "two_phase":
        ro = o.solve_two_phase(art, None, c["cap"], c["rule"])
    elif mode == "big_m":
        ro = o.solve_big_m(art, None, c["cap"], c["rule"])
    else:
        ro = o.solve_dual(c["cap"])
    T = o.get_rows()
    ok_, or_ = o.get_log()
    bad = []
    for r, p in enumerate(out):
        if p["res"].status != ro.status or p["res"].pivots != ro.pivots:
            bad.append(f"rank {r}: status/pivots {p['res'].status}/{p['res'].pivots} vs {ro.status}/{ro.pivots}")
        if not (np.array_equal(p["log"][0], ok_) and np.array_equal(p["log"][1], or_)):
            bad.append(f"rank {r}: log")
        if not np.array_equal(p["basis"], o.get_basis()):
            bad.append(f"rank {r}: basis")
        if not np.array_equal(p["obj"], T[m:m + (2 if big else 1)]):
            bad.append(f"rank {r}: objective row")
    if not np.array_equal(np.vstack([p["rows"] for p in out]), T[:m]):
        bad.append("constraint rows")
    o.close()
    return out[0]["res"], bad


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 4242
    rng = random.Random(seed)
    lpg.load()
    t0 = time.time()
    n = refused_attach = timeouts = 0
    while time.time() - t0 < budget:
        c = case(rng)
        res, bad = run(c)
        n += 1
        desc = (f"{n:4d} {c['mode']:9s} W={c['world']} m={c['m']:4d} n={c['n']:4d} rule={c['rule']} kind={c['kind']} "
                f"push={int(c['push'])}{' (refused at attach: collectives)' if c.get('push_refused') else ''} "
                f"seed={c['seed']} cap={c['cap']} env={c['env']}")
        refused_attach += 1 if c.get("push_refused") else 0
        timeouts += 1 if bad and res is None and "waited > 2 s" in bad[0] else 0
        if bad and res is None and "LPGError" in bad[0]:
            print(desc + " -> REFUSED " + bad[0], flush=True)
            continue
        if bad:
            print(desc + " -> MISMATCH " + "; ".join(bad), flush=True)
            sys.exit(1)
        print(desc + f" -> {res.status_name} {res.pivots} pivots: ok", flush=True)
    print(f"soak_dist: {n} cases, every rank bitwise equal to the oracle ({time.time() - t0:.0f} s); "
          f"owner push refused at attach in {refused_attach} (ran on the collectives), exchange timeouts {timeouts}")


if __name__ == "__main__":
    main()
