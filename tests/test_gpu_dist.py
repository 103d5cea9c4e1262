"""Multi-rank HIP engine on the one-GPU box.

The engine's row-block protocol (allgather of ratio candidates, allreduce of
the owner's normalised pivot row) runs through lpg_comm_init_host:
* in one process, 2-3 ranks as threads sharing the GPU with an in-process
  host transport;
* in 2 processes with torch.distributed `gloo` collectives on host tensors
  (the RCCL transport itself needs one GPU per rank and runs in the driver's
  8-GPU bench).
Every rank's pivot log, basis and replicated objective row, and the stacked
row blocks, must equal the single-rank engine and the oracle bitwise.
"""
from __future__ import annotations

import os
import pickle
import subprocess
import tempfile
import threading

import numpy as np
import pytest

from oracle.lpo import GEN_ARTIFICIAL, GEN_DUAL, Oracle
from util import degenerate_two_phase_lp, spawn_ranks, torchrun_cmd

pytestmark = pytest.mark.gpu


class ThreadComm:
    """In-process allgather / allreduce-sum for ranks running as threads."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.violations = []

    def allgather(self, rank, data: bytes) -> bytes:
        self.slots[rank] = data
        self.bar.wait()
        out = b"".join(self.slots)
        self.bar.wait()
        return out

    def allreduce(self, rank, arr: np.ndarray) -> np.ndarray:
        self.slots[rank] = arr
        self.bar.wait()
        # The engine's allreduces are broadcasts in disguise: the
        # pivot row from its owner, every other rank sending exactly -0, and the
        # objective chain from the rank whose turn it is, the others +0. So at
        # most one rank contributes anything but zeros, every other rank's
        # buffer is one signed zero throughout, and the sum is the contributor's
        # buffer bit for bit (round 2 summed uninitialised padding here).
        bits = [np.ascontiguousarray(s).view(np.uint64) for s in self.slots]
        live = [q for q in range(self.world) if np.any(bits[q] << np.uint64(1))]
        acc = self.slots[0].copy()
        for q in range(1, self.world):
            acc = acc + self.slots[q]
        bad = None
        if len(live) > 1:
            bad = f"ranks {live} both contributed to one exchange of {len(arr)} doubles"
        for q in range(self.world):
            if q not in live and not np.all(bits[q] == bits[q][0]):
                bad = f"rank {q} sent a mix of +0 and -0"
        if live and all(bits[q][0] == np.uint64(1 << 63) for q in range(self.world) if q != live[0]):
            if not np.array_equal(acc.view(np.uint64), bits[live[0]]):
                bad = "the sum is not the owner's row"
        self.bar.wait()
        if bad:
            self.violations.append(bad)
            raise AssertionError(bad)
        return acc


def _run_threads(lpg, world, m, n, seed, kind, rule, max_pivots, push=False):
    comm = ThreadComm(world)
    out = [None] * world
    errs = []

    def worker(rank):
        try:
            e = lpg.Engine(m, n + m + 1, world=world, rank=rank)
            e.comm_init_host(lambda b: comm.allgather(rank, b), lambda a: comm.allreduce(rank, a))
            if push:                              # owner-push exchange between the threads' buffers
                mine = e.push_base().to_bytes(8, "little")
                allb = comm.allgather(rank, mine)
                e.comm_init_push_local([int.from_bytes(allb[8 * r:8 * r + 8], "little") for r in range(world)])
            e.generate(n, seed, kind)
            res = e.solve(max_pivots, rule)
            info = e.info
            out[rank] = dict(res=res, log=e.get_log(), basis=e.get_basis(),
                             rows=e.get_rows(info.row0, info.nrows), obj=e.get_rows(m, 1)[0])
            e.close()
        except Exception as ex:   # pragma: no cover
            errs.append(ex)
            comm.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not comm.violations, comm.violations[:4]
    assert not errs, errs
    return out


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    return lpg


@pytest.fixture(autouse=True)
def _acknowledge_shared_gpu(monkeypatch, request):
    """Every multi-rank case here runs on the ONE GPU of the test box, so the
    owner push would be refused at attach time (ranks sharing a process's
    queues or a GPU's CUs, lpg_ctx.hip push_shares_device): these tests keep
    exercising the protocol at sizes whose grids co-reside, and say so. The
    refusals themselves are tested below with the acknowledgements cleared."""
    if "refused" not in request.node.name:
        monkeypatch.setenv("LPG_PUSH_SHARED_QUEUES", "1")
        monkeypatch.setenv("LPG_PUSH_SHARED_DEVICE", "1")


@pytest.mark.parametrize("defer", [None, "0", "5", "64", "128"])
@pytest.mark.parametrize("world,m,n,kind,rule", [(2, 96, 160, 0, 0), (3, 101, 77, 0, 0), (2, 64, 64, 1, 1),
                                                 (4, 203, 301, 0, 0), (8, 203, 301, 0, 0)])
def test_threads_row_partition_bitwise(lpg, world, m, n, kind, rule, defer, monkeypatch):
    """Row blocks over ranks; default deferred blocks, eager (0), 5-, 64- and 128-pivot blocks."""
    if defer is not None:
        monkeypatch.setenv("LPG_DEFER", defer)
    seed = 777
    parts = _run_threads(lpg, world, m, n, seed, kind, rule, 5000)
    o = Oracle(m, n + m + 1)
    o.generate(n, seed, kind)
    ores = o.solve(5000, rule)
    k, r = o.get_log()
    T = o.get_rows()
    for p in parts:
        assert p["res"].status == ores.status and p["res"].pivots == ores.pivots
        assert np.array_equal(p["log"][0], k) and np.array_equal(p["log"][1], r)
        assert np.array_equal(p["basis"], o.get_basis())
        assert np.array_equal(p["obj"], T[m])
    assert np.array_equal(np.vstack([p["rows"] for p in parts]), T[:m])


def _gloo_worker(rank, world, init, m, n, seed, outdir, push=False, kind=0, rule=0, defer=None, mr=None, big_m=False,
                 two_phase=False, dual=False, region=None):
    if region is not None:                        # 0: the all-column slices instead of region mode
        os.environ["LPG_REGION"] = region
    if defer is not None:
        os.environ["LPG_DEFER"] = defer
    if mr is not None:                            # 0: the two-kernel pair instead of k_pivot_block's multi-rank form
        os.environ["LPG_PERSIST_MR"] = mr
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    import linearprogramming_amd as lpg

    def allgather(b: bytes) -> bytes:
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.numpy()) for o in outs)

    def allreduce(a: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(a)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    e = lpg.Engine(m, n + m + 1, world=world, rank=rank, flags=lpg._lib.FLAG_BIG_M if big_m else 0)
    e.comm_init_host(allgather, allreduce)
    if push:                                      # owner-push exchange through IPC handles
        h = allgather(e.push_handle())
        e.comm_init_push([h[64 * r:64 * r + 64] for r in range(world)])
    if big_m:                                     # two objective rows (M part, real part)
        e.generate(n, seed, lpg.GEN_ARTIFICIAL)
        res = e.solve_big_m(1 + n + (m + 1) // 2, None, 5000, rule)
    elif dual:                                    # the deferred dual over the row partition
        e.generate(n, seed, lpg.GEN_DUAL)
        res = e.solve_dual(5000)
    elif two_phase == "degenerate":               # an artificial left basic at zero: the forced drive-out
        T, basis, art_first = degenerate_two_phase_lp(m, n, seed)
        e.load_rows(0, T)
        e.set_basis(basis)
        res = e.solve_two_phase(art_first, None, 5000, rule)
    elif two_phase:
        e.generate(n, seed, lpg.GEN_ARTIFICIAL)
        res = e.solve_two_phase(1 + n + (m + 1) // 2, None, 5000, rule)
    else:
        e.generate(n, seed, kind)
        res = e.solve(5000, rule)
    info = e.info
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(dict(status=res.status, pivots=res.pivots, log=e.get_log(), basis=e.get_basis(), wg=info.pivot_wg,
                         region=info.region,
                         rows=e.get_rows(info.row0, info.nrows), obj=e.get_rows(m, 2 if big_m else 1)), f)
    e.close()
    dist.destroy_process_group()


def _processes(world, m, n, seed, push, kind=0, rule=0, defer=None, mr=None, big_m=False, two_phase=False, dual=False,
               region=None):
    with tempfile.TemporaryDirectory() as d:
        spawn_ranks(_gloo_worker, lambda init: (world, init, m, n, seed, d, push, kind, rule, defer, mr, big_m,
                                                 two_phase, dual, region), world)
        parts = [pickle.load(open(os.path.join(d, f"r{r}.pkl"), "rb")) for r in range(world)]
    if big_m:
        o = Oracle(m, n + m + 1, nobj=2)
        o.generate(n, seed, GEN_ARTIFICIAL)
        ores = o.solve_big_m(1 + n + (m + 1) // 2, None, 5000, rule)
    elif dual:
        o = Oracle(m, n + m + 1)
        o.generate(n, seed, GEN_DUAL)
        ores = o.solve_dual(5000)
        assert ores.status == 1 and ores.pivots > 0
    elif two_phase == "degenerate":
        T0, basis, art_first = degenerate_two_phase_lp(m, n, seed)
        o = Oracle(m, n + m + 1)
        o.load_tableau(T0, basis)
        ores = o.solve_two_phase(art_first, None, 5000, rule)
        assert ores.status == 1                   # OPTIMAL (after the drive-out)
    elif two_phase:
        o = Oracle(m, n + m + 1)
        o.generate(n, seed, GEN_ARTIFICIAL)
        ores = o.solve_two_phase(1 + n + (m + 1) // 2, None, 5000, rule)
    else:
        o = Oracle(m, n + m + 1)
        o.generate(n, seed, kind)
        ores = o.solve(5000, rule)
    T = o.get_rows()
    for p in parts:
        assert p["status"] == ores.status and p["pivots"] == ores.pivots
        assert np.array_equal(p["log"][0], o.get_log()[0]) and np.array_equal(p["log"][1], o.get_log()[1])
        assert np.array_equal(p["basis"], o.get_basis())
        assert np.array_equal(p["obj"], T[m:m + (2 if big_m else 1)])
    assert np.array_equal(np.vstack([p["rows"] for p in parts]), T[:m])
    return parts


def test_two_processes_gloo_bitwise(lpg):
    _processes(2, 120, 200, 31, push=False)


@pytest.mark.parametrize("push,mr", [(False, None), (True, None), (True, "0")])
@pytest.mark.parametrize("world,m,n,rule", [(2, 257, 300, 0), (3, 640, 512, 1)])
def test_processes_big_m_bitwise(lpg, world, m, n, rule, push, mr):
    """Big-M (two objective rows, lexicographic pricing) over 2-3 processes:
    the collectives, the owner push with the multi-rank pivot launch (its
    NOBJ = 2 form) and with the pair -- bitwise the oracle."""
    parts = _processes(world, m, n, 9, push=push, rule=rule, mr=mr, big_m=True)
    assert all((p["wg"] > 0) == (push and mr is None) for p in parts)


def _cross(lps, forms, full, default):
    """Every LP in the default form; the other forms only for the LPs in
    `full`, the rest `extended` (LPG_EXTENDED_TESTS=1, conftest.py)."""
    return [pytest.param(*lp, *f, marks=() if (lp in full or f == default) else pytest.mark.extended)
            for lp in lps for f in forms]


@pytest.mark.parametrize("world,m,n,rule,seed,lp,push,mr", _cross(
    [(2, 257, 300, 0, 9, "gen"), (3, 640, 512, 1, 9, "gen"), (2, 64, 80, 0, 1, "degenerate"),
     (3, 257, 300, 0, 2, "degenerate"), (2, 300, 200, 1, 3, "degenerate")],
    [(False, None), (True, None), (True, "0")],
    full=[(2, 257, 300, 0, 9, "gen"), (3, 257, 300, 0, 2, "degenerate")], default=(True, None)))
def test_processes_two_phase_bitwise(lpg, world, m, n, rule, seed, lp, push, mr):
    """Two-phase over 2-3 processes (round 3; single rank before): phase I on
    the artificial objective, the |b| test summed over ranks in global row
    order, forced pivots driving basic artificials out (each row's owner finds
    the column), phase II -- status, pivot count, log, basis, every row and the
    objective row bitwise the oracle's."""
    _processes(world, m, n, seed, push=push, rule=rule, mr=mr, two_phase=lp)


@pytest.mark.parametrize("world,m,n,seed,defer", [(2, 100, 150, 3, None), (3, 400, 300, 3, None), (2, 257, 200, 5, "5"),
                                                  (3, 700, 500, 7, "32"),
                                                  (2, 1000, 800, 3, "128")])
def test_processes_dual_bitwise(lpg, world, m, n, seed, defer):
    """The deferred dual simplex over 2-3 processes (round 3; single rank
    before): row candidates allgathered, the leaving row summed from its owner
    (-0 elsewhere), the ratio test on every rank over the replicated row, each
    rank's rows through its own chain and block pass -- status, pivot count,
    log, basis, every row and the objective row bitwise the oracle's."""
    _processes(world, m, n, seed, push=world == 2, defer=defer, dual=True)   # the push attached: unused, harmless


@pytest.mark.parametrize("world,m,n,kind,rule,defer,mr,region", _cross(
    [(2, 120, 200, 0, 0, None), (2, 96, 160, 0, 0, "5"), (3, 101, 77, 0, 0, "64"), (2, 64, 64, 1, 1, "5"),
     (3, 203, 301, 0, 0, "32"), (2, 203, 301, 0, 0, "128"), (2, 1024, 2048, 0, 0, None), (3, 700, 900, 1, 1, "64")],
    [(None, None), (None, "0"), ("0", None)],
    full=[(2, 120, 200, 0, 0, None), (3, 101, 77, 0, 0, "64"), (3, 700, 900, 1, 1, "64")], default=(None, None)))
def test_processes_owner_push_bitwise(lpg, world, m, n, kind, rule, defer, mr, region):
    """The owner-push exchange between ranks in separate processes sharing the
    GPU (IPC-mapped exchange buffers, the layout of one process per GPU): no
    collective per pivot -- the owner stores the pivot row into every rank's
    buffer, every rank its candidates -- bitwise the oracle. (Ranks as threads
    of one process are not used here: a process gets GPU_MAX_HW_QUEUES = 4
    hardware queues, and two ranks' streams on one queue would serialise a
    waiting kernel in front of the kernel it waits for.)
    By default (mr None) every rank runs k_pivot_block's multi-rank form --
    one launch per block, the leaving row and the pivot row exchanged inside
    it -- wherever its slices fit (blocks of <= 64 pivots); mr "0" keeps the
    two-kernel pair. Round 5: that launch runs in region mode on every rank
    (slices of the live columns only, a spare per pending pivot taking over
    its leaving column, decided from the global pivot rows so every rank
    agrees; a non-owner reads the spare's entry from the owner's push);
    region "0" keeps the all-column slices."""
    parts = _processes(world, m, n, 778, push=True, kind=kind, rule=rule, defer=defer, mr=mr, region=region)
    persistent = mr is None and (defer is None or int(defer) <= 64)
    assert all((p["wg"] > 0) == persistent for p in parts)
    assert all(p["region"] == (persistent and region is None) for p in parts)
    assert len({p["wg"] for p in parts}) == 1          # the same slices on every rank


@pytest.mark.parametrize("world,m,n,kind,rule,defer,push,mr", [(4, 1024, 2048, 0, 0, None, True, None),
                                                               (4, 700, 900, 1, 1, "64", True, None)])
def test_processes_4_ranks(lpg, world, m, n, kind, rule, defer, push, mr):
    """The driver's N = 4 row partition rehearsed on one GPU (config 2's
    shape: 175-256 rows per rank): 4 processes with the owner push and the
    persistent multi-rank launch on every rank (the candidate words of 4 ranks
    in xpoll_best) -- bitwise the oracle. Eight processes also ran bitwise on
    a fresh box (push, persistent launch and the pair;
    profiles/r03_pytest_gpu_4_8_ranks.log), but not inside this whole suite:
    after its earlier GPU tests, 8 processes' spinning launches on ONE GPU are
    not reliably scheduled side by side (a rank waited > 2 s for another's
    candidates), and 8 processes over the per-pivot host collectives outran
    the box's silence limit. One process per GPU, the driver's layout, shares
    no GPU between ranks."""
    parts = _processes(world, m, n, 778, push=push, kind=kind, rule=rule, defer=defer, mr=mr)
    assert all((p["wg"] > 0) == (push and mr is None) for p in parts)
    assert all(p["region"] == (push and mr is None) for p in parts)
    assert len({p["wg"] for p in parts}) == 1


@pytest.mark.parametrize("m,n,defer,graphs", [(300, 500, None, "0"), (1024, 2048, None, "0"), (1024, 2048, "64", "0"),
                                              (1024, 2048, "128", "0"), (1024, 2048, None, "1")])
def test_rccl_single_rank_communicator(lpg, m, n, defer, graphs, monkeypatch):
    """The RCCL transport on a 1-rank communicator: every per-pivot ncclAllReduce
    (pivot row) and ncclAllGather (ratio candidates) really runs, and the result
    is bitwise the engine without a communicator (and the oracle)."""
    if defer is not None:
        monkeypatch.setenv("LPG_DEFER", defer)
    monkeypatch.setenv("LPG_GRAPH_RCCL", graphs)     # 1: the collectives are captured into the replayed graphs
    e = lpg.Engine(m, n + m + 1)
    e.comm_init_rccl(lpg.Engine.rccl_unique_id())
    e.generate(n, 41, 0)
    res = e.solve(100_000, 0)
    o = Oracle(m, n + m + 1)
    o.generate(n, 41, 0)
    ores = o.solve(100_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots and res.objective == ores.objective
    assert np.array_equal(e.get_log()[0], o.get_log()[0]) and np.array_equal(e.get_log()[1], o.get_log()[1])
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


@pytest.mark.parametrize("method", ["dual", "two_phase", "two_phase_degenerate"])
def test_rccl_single_rank_dual_and_two_phase(lpg, method):
    """The dual and two-phase on a 1-rank RCCL communicator: the partition
    code path (row candidates through ncclAllGather, the leaving row and the
    |b| running sum through ncclAllReduce, the drive-out column shared) runs
    for real and equals the oracle bit for bit."""
    m, n = 400, 300
    e = lpg.Engine(m, n + m + 1)
    e.comm_init_rccl(lpg.Engine.rccl_unique_id())
    o = Oracle(m, n + m + 1)
    if method == "dual":
        e.generate(n, 3, lpg.GEN_DUAL)
        o.generate(n, 3, GEN_DUAL)
        res, ores = e.solve_dual(100_000), o.solve_dual(100_000)
    elif method == "two_phase":
        e.generate(n, 9, lpg.GEN_ARTIFICIAL)
        o.generate(n, 9, GEN_ARTIFICIAL)
        art = 1 + n + (m + 1) // 2
        res, ores = e.solve_two_phase(art, None, 100_000, 1), o.solve_two_phase(art, None, 100_000, 1)
    else:
        T, basis, art = degenerate_two_phase_lp(m, n, 2)
        e.load_rows(0, T)
        e.set_basis(basis)
        o.load_tableau(T, basis)
        res, ores = e.solve_two_phase(art, None, 100_000, 0), o.solve_two_phase(art, None, 100_000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots and res.objective == ores.objective
    assert np.array_equal(e.get_log()[0], o.get_log()[0]) and np.array_equal(e.get_log()[1], o.get_log()[1])
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())
    assert np.array_equal(e.get_basis(), o.get_basis())


def test_host_comm_single_rank(lpg):
    e = lpg.Engine(50, 50 + 70 + 1)
    e.comm_init_host(lambda b: b, lambda a: a)
    e.generate(70, 42, 0)
    res = e.solve(10_000, 0)
    o = Oracle(50, 50 + 70 + 1)
    o.generate(70, 42, 0)
    ores = o.solve(10_000, 0)
    assert res.pivots == ores.pivots and np.array_equal(e.get_rows(0, 51), o.get_rows())
    with pytest.raises(lpg.LPGError):
        e.comm_init_host(lambda b: b, lambda a: a)     # one communicator per context


@pytest.mark.parametrize("trade", [None, "1"])
@pytest.mark.parametrize("mr", ["1", "0"])
@pytest.mark.parametrize("m,n", [(300, 500), (1024, 2048)])
def test_owner_push_single_rank(lpg, m, n, mr, trade, monkeypatch):
    """The owner-push exchange on a 1-rank communicator (pushes to itself):
    k_pivot_block's multi-rank form (mr 1) and the two-kernel pair (mr 0),
    bitwise the engine without a communicator and the oracle. trade "1": the
    block-end column trade on (one rank below 2 GB keeps it off by default),
    with it region mode on the multi-rank form."""
    monkeypatch.setenv("LPG_DEFER", "64")
    monkeypatch.setenv("LPG_PERSIST_MR", mr)
    if trade is not None:
        monkeypatch.setenv("LPG_NO_REORDER", "0")
    e = lpg.Engine(m, n + m + 1)
    e.comm_init_host(lambda b: b, lambda a: a)
    e.comm_init_push([e.push_handle()])
    assert e.info.exchange in (1, 2)                # 2: the exchange buffer is uncached (hipDeviceMallocUncached)
    assert (e.info.pivot_wg > 0) == (mr == "1")
    assert e.info.region == (mr == "1" and trade == "1")   # region mode on the ranks of a push exchange (round 5)
    print(f"exchange mode {e.info.exchange}")
    e.generate(n, 43, 0)
    res = e.solve(100_000, 0)
    o = Oracle(m, n + m + 1)
    o.generate(n, 43, 0)
    ores = o.solve(100_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots and res.objective == ores.objective
    assert np.array_equal(e.get_log()[0], o.get_log()[0]) and np.array_equal(e.get_log()[1], o.get_log()[1])
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


@pytest.mark.parametrize("world,exchange", [(4, "push")])
def test_bench_torchrun_4_ranks(world, exchange):
    """bench.py as the driver launches it for N > 1 (torch.distributed.run,
    one process per rank, 127.0.0.1 rendezvous), rehearsed on one GPU at
    config 2 (host collectives for setup: RCCL refuses ranks sharing a GPU):
    exactly one JSON line on stdout, the owner push attached and the
    persistent multi-rank launch on every rank (no fallback to the
    collectives), the ranks' replicated logs agreeing after the warm-up
    (8 ranks passed on a fresh box, profiles/r03_pytest_gpu_4_8_ranks.log;
    see test_processes_4_ranks for why not in this suite)."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = torchrun_cmd(world) + ["bench.py", "--gpus", str(world), "--config", "2", "--host-comm", "--exchange",
                                 exchange, "--steps", "4", "--warmup", "1", "--no-cpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["value"] > 0 and d["status"] == "ITER_LIMIT"
    if exchange == "push":
        assert "owner push" in d["config"]["parallelism"], d["config"]
        assert d["config"]["pivot_loop"].startswith("k_pivot_block"), d["config"]
    assert d["config"]["pivots_timed"] > 0 and d["config"]["pivots_timed"] % 4 == 0
    assert "using the collectives" not in p.stderr


def test_push_between_threads_refused(lpg, monkeypatch):
    """ranks that are threads of one process share its
    hardware queues, so a spinning exchange kernel can sit in front of the
    peer kernel it waits for (tools/soak_dist.py's 2 s timeouts mid-solve).
    lpg_comm_init_push_local refuses that at attach time with a named error,
    before any pivot; the ranks keep their collectives."""
    monkeypatch.delenv("LPG_PUSH_SHARED_QUEUES", raising=False)
    es = [lpg.Engine(64, 64 + 128 + 1, world=2, rank=r) for r in range(2)]
    for e in es:
        e.comm_init_host(lambda b: b, lambda a: a)
    bases = [e.push_base() for e in es]
    for e in es:
        with pytest.raises(lpg.LPGError, match=r"owner-push exchange refused: the 2 ranks are threads of one process"):
            e.comm_init_push_local(bases)
        assert e.info.exchange == 0
        e.close()


def test_push_on_one_gpu_refused_bench_falls_back(monkeypatch):
    """two processes on ONE GPU (the same PCI bus id in
    their exchange buffers) share its CUs, so lpg_comm_init_push refuses the
    owner push at attach time ("ranks 0 and 1 share GPU ...") and bench.py
    falls back to the collectives before its first pivot -- the line reports
    the collectives and a normal run, not a mid-solve timeout."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # plain `python3 bench.py --gpus 2`: bench.py starts its own rank processes
    # (VERDICT r5 missing #3), as the driver's first 8-GPU run may call it
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--config", "2", "--host-comm", "--exchange", "push",
           "--steps", "2", "--warmup", "1", "--no-cpu"]
    env = {k: v for k, v in os.environ.items() if k not in ("LPG_PUSH_SHARED_DEVICE", "LPG_PUSH_SHARED_QUEUES")}
    env["OMP_NUM_THREADS"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "owner-push exchange refused: ranks" in p.stderr and "share GPU" in p.stderr, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0, d
    assert "owner push" not in d["config"]["parallelism"] and d["config"]["pivots_timed"] > 0, d["config"]
