"""Config-4 row partition (2 ranks as threads, host transport) vs one rank:
state after P pivots (objective row, given rows), and whether continuing from
a materialised tableau changes the next pivot. Diagnostics only."""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import linearprogramming_amd as lpg  # noqa: E402
from test_gpu_dist import ThreadComm  # noqa: E402

lpg.load()
m, n = int(os.environ.get("M", 65536)), int(os.environ.get("N", 131072))
P = int(os.environ.get("P", 72))
ROWS = [int(x) for x in os.environ.get("ROWS", "65436,8457,26474").split(",")]
world = 2


def mr(steps):
    comm = ThreadComm(world)
    out = [None] * world

    def worker(rank):
        e = lpg.Engine(m, n + m + 1, world=world, rank=rank)
        e.comm_init_host(lambda b: comm.allgather(rank, b), lambda a: comm.allreduce(rank, a))
        e.generate(n, 20220518, 0)
        res = []
        for st in steps:
            if st == "read":
                res.append(("obj", e.get_rows(m, 1)[0]))
                info = e.info
                for i in ROWS:
                    if info.row0 <= i < info.row0 + info.nrows:
                        res.append((f"row{i}", e.get_rows(i, 1)[0]))
            else:
                e.solve(st, 0)
        k, r = e.get_log()
        res.append(("log", (k, r)))
        out[rank] = res
        e.close()
    th = [threading.Thread(target=worker, args=(q,)) for q in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


def single(steps):
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, 20220518, 0)
    res = []
    for st in steps:
        if st == "read":
            res.append(("obj", e.get_rows(m, 1)[0]))
            for i in ROWS:
                res.append((f"row{i}", e.get_rows(i, 1)[0]))
        else:
            e.solve(st, 0)
    k, r = e.get_log()
    res.append(("log", (k, r)))
    e.close()
    return res


SAVE = {}
for steps in ([P, "read", 1, "read"],):
    a = mr(steps)
    sb = single(steps)
    print("steps", steps, flush=True)
    dict_b = {}
    for x, y in sb:
        dict_b.setdefault(x, []).append(y)
    for q in range(world):
        cnt = {}
        for x, y in a[q]:
            c = cnt.get(x, 0)
            cnt[x] = c + 1
            yb = dict_b[x][c]
            if x != "log":
                SAVE[f"mr{q}_{x}_{c}"] = y
                SAVE[f"one_{x}_{c}"] = yb
            if x == "log":
                ka, ra = y
                kb, rb = yb
                nn = min(len(ka), len(kb))
                bad = np.nonzero((ka[:nn] != kb[:nn]) | (ra[:nn] != rb[:nn]))[0]
                print(f"  rank{q} log: first difference {bad[0] if len(bad) else None} (len {len(ka)}/{len(kb)})",
                      flush=True)
            else:
                bad = np.nonzero(y != yb)[0]
                print(f"  rank{q} {x}#{c}: {len(bad)} entries differ {bad[:8].tolist()}", flush=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "diag_mr4.npz"), **SAVE)
