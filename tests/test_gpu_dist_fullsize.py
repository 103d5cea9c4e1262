"""The row partition at BASELINE.json's full sizes, two processes on the one GPU.

BASELINE config 4 is "row-partitioned across 8 x MI355X": the multi-rank path
(lpg_create_dist + a communicator + the owner-push exchange) is
what the driver's 8-GPU run takes first. Here two ranks, one process each,
share the lease's GPU through IPC-mapped exchange buffers (the layout of one
process per GPU), at the full sizes:

* config 3 (16384 x 32768, 8192 rows per rank), 200 pivots = three whole
  64-pivot blocks (each ending in the column trade, the block pass and the
  pivot-row rewrite on every rank) and a partial block flushed by the readout;
  bitwise against the C oracle: pivot log, basis, objective row, every pivot
  row and 64 sampled rows per rank.
  - with the two-kernel pair (LPG_PERSIST_MR=0);
  - with the persistent multi-rank launch left on: two 198-workgroup grids do
    not fit one GPU's 256 CUs at once, so the launch's residency census
    (lpg_block.hip) stops it before its first pivot on BOTH ranks (one
    decision word) and the library continues on the pair by itself --
    lpg_info.residency_fallbacks counts it -- instead of waiting 2 s and
    failing (round 2).
* config 4's shape (65536 x 131072, 32768 rows and 51.5 GB per rank, blocks
  of 96 pivots, the multi-rank column trade over 196,609 columns), 320
  pivots over the collectives (the owner push's spinning prep grid needs a GPU
  per rank at this size, see the test): bitwise equal to the single-rank engine (partition invariance: log,
  basis, objective row, column 0, every pivot row and 64 sampled rows per
  rank), plus unit basic columns on those rows and b >= 0 on every row.

Reference: the loop simplex.c:40 -> :65 lacks.
"""
from __future__ import annotations

import os
import pickle
import tempfile

import numpy as np
import pytest

from oracle.lpo import Oracle
from util import spawn_ranks

pytestmark = pytest.mark.gpu
SEED = 20220518


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    assert lpg.device_count() >= 1, "no GPU visible"
    return lpg


@pytest.fixture(autouse=True)
def _acknowledge_shared_gpu(monkeypatch):
    """The ranks here are processes on the test box's ONE GPU: the owner push
    refuses that at attach time unless acknowledged (lpg_ctx.hip
    push_shares_device; the refusal is tested in test_gpu_dist.py). The
    persistent grids cannot co-reside at these sizes, so the residency census
    hands these cases to the two-kernel pair, as before."""
    monkeypatch.setenv("LPG_PUSH_SHARED_DEVICE", "1")


def _sample(m, world, rank, k, seed):
    """k sampled global rows of rank `rank`'s block (floor(m p / W) split)."""
    r0, r1 = m * rank // world, m * (rank + 1) // world
    rng = np.random.default_rng(seed + rank)
    return sorted(set(rng.choice(np.arange(r0, r1), k, replace=False).tolist()) | {r0, r1 - 1})


def _worker(rank, world, init, m, n, seed, pivots, outdir, env, push, sample_rows=None, sweep=False):
    os.environ.update(env)
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

    e = lpg.Engine(m, n + m + 1, world=world, rank=rank)
    e.comm_init_host(allgather, allreduce)
    if push:
        h = allgather(e.push_handle())
        e.comm_init_push([h[64 * r:64 * r + 64] for r in range(world)])
    wg0 = e.info.pivot_wg
    e.generate(n, seed, lpg.GEN_DENSE)
    e.reserve_log(pivots + 8)
    res = e.solve(pivots, lpg.RULE_DANTZIG)
    print(f"rank {rank}/{world}: {res.pivots} pivots", flush=True)   # progress (a long test, run with -s)
    info = e.info
    k, r = e.get_log()
    basis = e.get_basis()
    if sample_rows is not None:                  # the rows the caller read from its reference run
        rows = [i for i in sample_rows if info.row0 <= i < info.row0 + info.nrows]
    else:
        rows = sorted(set(_sample(m, world, rank, 64, seed)) | {int(x) for x in r if info.row0 <= x < info.row0 + info.nrows})
    bad = []
    if sweep:                                    # every local row: basic columns unit, b >= 0
        for i0 in range(info.row0, info.row0 + info.nrows, 256):
            nr = min(256, info.row0 + info.nrows - i0)
            blk = e.get_rows(i0, nr)
            sub = blk[:, basis]
            idx = np.arange(i0, i0 + nr)
            if not (np.array_equal(sub[np.arange(nr), idx], np.ones(nr)) and np.count_nonzero(sub) == nr):
                bad.append(f"rows {i0}..: basic columns not unit")
            if not np.all(blk[:, 0] >= 0.0):
                bad.append(f"rows {i0}..: b < 0")
    out = dict(bad=bad, status=res.status, pivots=res.pivots, objective=res.objective, log=(k, r), basis=basis,
               obj=e.get_rows(m, 1)[0], rows={i: e.get_rows(i, 1)[0] for i in rows}, x0=e.get_column0(),
               wg0=wg0, wg=info.pivot_wg, fallbacks=info.residency_fallbacks, exchange=info.exchange,
               defer=info.defer_k, row0=info.row0, nrows=info.nrows)
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(out, f)
    e.close()
    dist.destroy_process_group()


def _run(world, m, n, pivots, env, push=True, sample_rows=None, sweep=False):
    with tempfile.TemporaryDirectory() as d:
        spawn_ranks(_worker, lambda init: (world, init, m, n, SEED, pivots, d, env, push, sample_rows, sweep), world)
        return [pickle.load(open(os.path.join(d, f"r{q}.pkl"), "rb")) for q in range(world)]


def _check_against(parts, m, pivots, log, basis, obj, row_of):
    """Every rank equals the reference run (the oracle or the single-rank engine)."""
    for p in parts:
        assert p["pivots"] == pivots and p["status"] == 4              # ITER_LIMIT: the budget ran out first
        assert np.array_equal(p["log"][0], log[0]) and np.array_equal(p["log"][1], log[1])
        assert np.array_equal(p["basis"], basis)
        assert np.array_equal(p["obj"], obj), "objective row"
        pivot_rows = {int(x) for x in log[1]}
        own = {i for i in pivot_rows if p["row0"] <= i < p["row0"] + p["nrows"]}
        assert own <= set(p["rows"]), "a pivot row was not read back"
        for i, ri in p["rows"].items():
            assert np.array_equal(ri, row_of(i)), f"rank row {i}"
            assert ri[basis[i]] == 1.0 and np.count_nonzero(ri[basis]) == 1, f"row {i}: basic columns not unit"
        assert np.all(p["x0"] >= 0.0)
    assert sum(p["nrows"] for p in parts) == m


@pytest.mark.parametrize("mr", ["0", None])
def test_config3_two_processes_bitwise(lpg, mr):
    m, n, piv = 16384, 32768, 200
    env = {"LPG_PERSIST_MR": mr} if mr is not None else {}
    parts = _run(2, m, n, piv, env)
    # 3.2 GB per rank: ranks take 96-pivot blocks from 1 GB (lpg_ctx.hip, region geometry)
    assert all(p["defer"] == 96 and p["exchange"] in (1, 2) for p in parts), [p["defer"] for p in parts]
    if mr == "0":
        assert all(p["wg0"] == 0 and p["wg"] == 0 and p["fallbacks"] == 0 for p in parts)
    else:
        # the persistent form was on; two such grids cannot be resident on one GPU:
        # the census stopped the first launch on both ranks and the pair took over
        assert all(p["wg0"] > 0 for p in parts), "the persistent multi-rank form was not selected"
        assert all(p["fallbacks"] >= 1 and p["wg"] == 0 for p in parts), [(p["fallbacks"], p["wg"]) for p in parts]
    o = Oracle(m, n + m + 1, nthreads=min(16, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    o.generate(n, SEED, 0)
    ores = o.solve(piv, 0)
    assert ores.pivots == piv
    assert all(p["objective"] == ores.objective for p in parts)
    _check_against(parts, m, piv, o.get_log(), o.get_basis(), o.get_rows(m, 1)[0], lambda i: o.get_rows(i, 1)[0])
    x0 = np.concatenate([p["x0"] for p in parts])
    assert np.array_equal(x0, np.concatenate([o.get_rows(i0, 1024)[:, 0] for i0 in range(0, m, 1024)]))


def test_config4_shape_two_processes_partition_invariance(lpg):
    m, n, piv = 65536, 131072, 320
    # the collectives (host transport), not the owner push: on ONE GPU the push's
    # non-owner prep blocks spin until the owner's chunk lands, and a 385-block
    # spinning grid can hold every slot the owner's grid needs (one process per
    # GPU, the real layout, has no such coupling); config 3's 97-block grids fit
    parts = _run(2, m, n, piv, {}, push=False)
    assert all(p["defer"] == 96 and p["wg"] == 0 and p["exchange"] == 0 for p in parts)   # the pair, 96-pivot blocks
    # the same LP on one rank (run after the two processes have freed the GPU)
    e = lpg.Engine(m, n + m + 1)
    assert e.info.defer_k == 96
    e.generate(n, SEED, lpg.GEN_DENSE)
    e.reserve_log(piv + 8)
    res = e.solve(piv, lpg.RULE_DANTZIG)
    k1, r1 = e.get_log()
    for p in parts:                                  # the first divergence, if any, named before the details
        k2, r2 = p["log"]
        bad = np.nonzero((k1[:len(k2)] != k2[:len(k1)]) | (r1[:len(k2)] != r2[:len(k1)]))[0]
        assert len(bad) == 0, f"pivot {bad[0]}: single rank ({k1[bad[0]]}, {r1[bad[0]]}), rank ({k2[bad[0]]}, {r2[bad[0]]})"
    assert res.pivots == piv and all(p["objective"] == res.objective for p in parts), \
        (res.objective, [p["objective"] for p in parts])
    _check_against(parts, m, piv, e.get_log(), e.get_basis(), e.get_rows(m, 1)[0], lambda i: e.get_rows(i, 1)[0])
    assert np.array_equal(np.concatenate([p["x0"] for p in parts]), e.get_column0())
    e.close()


def test_config4_eight_processes_partition_invariance(lpg):
    """BASELINE config 4's actual split on the one GPU (VERDICT r3 missing #2):
    8 processes x 8192 rows x 196,609 columns (12.9 GB each, 103 GB in all).
    Each rank is under 16 GB, so it takes 64-pivot blocks, the two-kernel
    pair (the slices do not fit the persistent launch) and the 8-rank column
    trade; the exchange is the host collectives (gloo), as in the 2-process
    config-4 test. 200 pivots = three whole blocks and a partial one settled
    by the readout. The single-rank engine runs the same LP first (96-pivot
    blocks: the deferral is bitwise the eager chain, so the block size must
    not matter) and is released before the ranks start; every rank must equal
    it bit for bit: status, pivot count, objective, log, basis, objective
    row, column 0, every pivot row and 64 sampled rows per rank. Every row
    of every rank also has unit basic columns and b >= 0."""
    m, n, piv, world = 65536, 131072, 200, 8
    e = lpg.Engine(m, n + m + 1)
    assert e.info.defer_k == 96
    e.generate(n, SEED, lpg.GEN_DENSE)
    e.reserve_log(piv + 8)
    res = e.solve(piv, lpg.RULE_DANTZIG)
    assert res.pivots == piv and res.status == 4
    log, basis, obj, x0 = e.get_log(), e.get_basis(), e.get_rows(m, 1)[0], e.get_column0()
    rows = set(int(x) for x in log[1])
    for p in range(world):
        rows |= set(_sample(m, world, p, 64, SEED))
    rows = sorted(rows)
    ref_rows = {i: e.get_rows(i, 1)[0] for i in rows}
    e.close()
    del e
    parts = _run(world, m, n, piv, {}, push=False, sample_rows=rows, sweep=True)
    assert all(p["defer"] == 64 and p["wg"] == 0 and p["exchange"] == 0 for p in parts)   # the pair, 64-pivot blocks
    assert [p["nrows"] for p in parts] == [m // world] * world
    for p in parts:                                  # the first divergence, if any, named before the details
        k2, r2 = p["log"]
        badp = np.nonzero((log[0][:len(k2)] != k2[:len(log[0])]) | (log[1][:len(k2)] != r2[:len(log[0])]))[0]
        assert len(badp) == 0, f"pivot {badp[0]}: single rank ({log[0][badp[0]]}, {log[1][badp[0]]}), " \
                               f"rank ({k2[badp[0]]}, {r2[badp[0]]})"
        assert not p["bad"], p["bad"][:4]
        assert len(p["rows"]) >= 64
    assert all(p["objective"] == res.objective for p in parts), (res.objective, [p["objective"] for p in parts])
    _check_against(parts, m, piv, log, basis, obj, lambda i: ref_rows[i])
    assert np.array_equal(np.concatenate([p["x0"] for p in parts]), x0)
