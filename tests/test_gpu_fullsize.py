"""Parity at BASELINE.json's full sizes (configs 3, 4 and 5), on the device.

* config 3 (16384 x 32768): three whole deferred blocks of 96 (the default)
  or 64 pivots plus 8
  (each ending in the column trade k_swap_plan / k_move_cols / k_fill_cols,
  the block pass k_flushw over reordered columns and the pivot-row rewrite
  k_flush_pivot_rows; the pivots in the region-mode persistent launch)
  plus 8 pending pivots flushed by the readout; bitwise
  against the C oracle: pivot log, basis, column 0, objective row, every pivot
  row and 64 sampled rows; basic columns are unit vectors on those rows.
* config 5 (two-phase, Bland, m = n = 8192, KM-style degenerate with
  equality rows): the whole solve to optimality, bitwise against the oracle
  (status, pivot count, objective, log, basis, sampled rows).
* config 4's width (196,609 columns) at m = 2048: 308 pivots through the
  two-kernel pair with 96- and 64-pivot blocks, bitwise against the oracle.
* config 4 (65536 x 131072, 103 GB tableau, one GPU): 320 pivots (three
  whole 96-pivot blocks, then a partial one of 32); the oracle cannot hold it, so size-independent properties over the
  WHOLE tableau, read back in row chunks: every basic column is a unit vector
  in every row, b >= 0 (primal feasibility), z is nondecreasing block to block,
  and the objective row equals c_B T - c (recomputed on the host in global row
  order on ~64 sampled columns and on column 0) to 1e-9 relative to
  sum |c_B| |T| -- the device row is the result of 320 rank-1 updates, not of
  that dot product, so this one is a tolerance, not bitwise.

Reference: the pivot loop simplex.c:40 -> :65 lacks.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle.lpo import Oracle

pytestmark = pytest.mark.gpu
SEED = 20220518


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    assert lpg.device_count() >= 1, "no GPU visible"
    return lpg


def _oracle(m, ncols):
    return Oracle(m, ncols, nthreads=min(16, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def _log(x):
    k, r = x.get_log()
    return list(zip(k.tolist(), r.tolist()))


@pytest.mark.parametrize("defer", [None, 64])
def test_config3_three_blocks_bitwise(lpg, defer, monkeypatch):
    """The default (96-pivot blocks, the region-mode persistent launch) and
    64-pivot blocks: three whole blocks and a partial one of 8."""
    m, n = 16384, 32768
    if defer:
        monkeypatch.setenv("LPG_DEFER", str(defer))
    e = lpg.Engine(m, n + m + 1)
    monkeypatch.delenv("LPG_DEFER", raising=False)
    K = e.info.defer_k
    assert K == (defer or 96) and e.info.pivot_wg > 0 and e.info.region == 1
    e.generate(n, SEED, lpg.GEN_DENSE)
    e.reserve_log(3 * K + 16)
    e.enqueue(K, lpg.RULE_DANTZIG)           # block 1
    e.prepare(lpg.RULE_DANTZIG)
    e.enqueue(2 * K, lpg.RULE_DANTZIG)       # blocks 2 and 3
    mid = e.sync()
    assert mid.pivots == 3 * K
    res = e.solve(8, lpg.RULE_DANTZIG)       # 8 more: a partial block, flushed by the readout
    assert res.status_name == "ITER_LIMIT" and res.pivots == 3 * K + 8
    o = _oracle(m, n + m + 1)
    o.generate(n, SEED, 0)
    ores = o.solve(3 * K + 8, 0)
    assert ores.pivots == 3 * K + 8 and res.objective == ores.objective
    log = _log(e)
    assert log == _log(o)
    basis = e.get_basis()
    assert np.array_equal(basis, o.get_basis())
    rng = np.random.default_rng(3)
    rows = sorted(set(rng.choice(m, 64, replace=False).tolist()) | {r for _, r in log} | {0, m - 1})
    for i in rows:
        ri = e.get_rows(i, 1)
        assert np.array_equal(ri, o.get_rows(i, 1)), f"row {i}"
        assert ri[0, basis[i]] == 1.0 and np.count_nonzero(ri[0, basis]) == 1, f"row {i} basic columns"
    assert np.array_equal(e.get_rows(m, 1), o.get_rows(m, 1)), "objective row"
    x0 = e.get_column0()
    for i in rows:
        assert x0[i] == o.get_rows(i, 1)[0, 0]


def test_config5_two_phase_against_the_fixture(lpg):
    """Config 5's whole two-phase solve against tests/golden/config5_solve.json
    (the C oracle's solve, made in the build container by
    tests/golden/make_config5_golden.py): status, pivot count, objective
    bits, the whole log, basis, column 0 and 67 sampled rows (digests)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import trajectory as T
    from make_config5_golden import ART_FIRST, CAP, FIXTURE, M, N, SEED as S5
    sys.path.pop(0)
    fix = T.load(FIXTURE)
    e = lpg.Engine(M, N + M + 1)
    e.generate(N, S5, lpg.GEN_ARTIFICIAL)
    e.reserve_log(CAP + 8)
    res = e.solve_two_phase(ART_FIRST, None, CAP, lpg.RULE_BLAND)
    k, r = e.get_log()
    assert res.status_name == fix["status"] == "OPTIMAL" and res.pivots == fix["pivots"] > 4096
    assert float(res.objective).hex() == fix["objective_hex"]
    assert k.tolist() == fix["log_k"] and r.tolist() == fix["log_r"]
    assert T.digest(e.get_basis()) == fix["basis"] and T.digest(e.get_column0()) == fix["column0"]
    assert [T.digest(e.get_rows(i, 1)[0]) for i in fix["rows"]] == fix["row_digests"]


@pytest.mark.extended
def test_config5_two_phase_full_bitwise(lpg):
    """The same against the oracle run live on the GPU box's cores (~45 s)."""
    m = n = 8192
    art_first = 1 + n + (m + 1) // 2
    cap = 20000
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, SEED, lpg.GEN_ARTIFICIAL)
    e.reserve_log(cap + 8)
    res = e.solve_two_phase(art_first, None, cap, lpg.RULE_BLAND)
    o = _oracle(m, n + m + 1)
    o.generate(n, SEED, 2)
    ores = o.solve_two_phase(art_first, None, cap, lpg.RULE_BLAND)
    assert res.status_name == "OPTIMAL" and res.status == ores.status
    assert res.pivots == ores.pivots and res.pivots > 4096
    assert res.objective == ores.objective
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    rng = np.random.default_rng(5)
    for i in sorted(set(rng.choice(m, 64, replace=False).tolist()) | {0, m - 1, m}):
        assert np.array_equal(e.get_rows(i, 1), o.get_rows(i, 1)), f"row {i}"


def test_config4_full_size_properties(lpg):
    m, n = 65536, 131072
    N1 = n + m + 1
    e = lpg.Engine(m, N1)
    assert e.info.defer_k == 96                  # >= 16 GB: 96-pivot blocks
    e.generate(n, SEED, lpg.GEN_DENSE)
    c = -e.get_rows(m, 1)[0, 1:]                # slack basis: row m = [0 | -c]
    assert np.all(c[:n] > 0) and np.all(c[n:] == 0)
    e.reserve_log(512)
    zs = [0.0]
    for step in (96, 96, 96, 32):
        r = e.solve(step, lpg.RULE_DANTZIG)
        assert r.status_name == "ITER_LIMIT"
        zs.append(r.objective)
    assert r.pivots == 320
    assert all(b >= a for a, b in zip(zs, zs[1:])) and zs[-1] > 0
    basis = e.get_basis()
    assert len(set(basis.tolist())) == m
    log = _log(e)
    entered = {k for k, _ in log}
    obj = e.get_rows(m, 1)[0]
    rng = np.random.default_rng(7)
    nonbasic = np.setdiff1d(np.arange(1, N1), basis)
    cols = np.unique(np.concatenate([[0], rng.choice(nonbasic, 56, replace=False),
                                     np.array(sorted(entered))[:8]]))
    cb = np.where(basis <= n, c[basis - 1], 0.0)       # costs of the basic variables (slacks: 0)
    acc = np.zeros(len(cols))
    scale = np.zeros(len(cols))
    chunk = 256
    for i0 in range(0, m, chunk):
        blk = e.get_rows(i0, chunk)
        # basic columns are unit vectors in every row
        sub = blk[:, basis]
        idx = np.arange(i0, i0 + chunk)
        assert np.array_equal(sub[np.arange(chunk), idx], np.ones(chunk)), f"rows {i0}.."
        assert np.count_nonzero(sub) == chunk, f"rows {i0}.. basic columns not unit"
        assert np.all(blk[:, 0] >= 0.0), f"rows {i0}.. infeasible b"
        t = blk[:, cols]
        w = cb[i0:i0 + chunk]
        for q in np.nonzero(w)[0]:               # c_B T in global row order
            acc += w[q] * t[q]
        scale += np.abs(w) @ np.abs(t)
    d = acc.copy()
    d[1:] -= np.where(cols[1:] <= n, c[np.maximum(cols[1:], 1) - 1], 0.0)
    dev = obj[cols]
    tol = 1e-9 * (scale + 1.0)
    assert np.all(np.abs(d - dev) <= tol), np.max(np.abs(d - dev) / tol)
    assert abs(obj[0] - zs[-1]) <= 1e-9 * abs(zs[-1])
    # the entered columns are basic now: their reduced costs are exactly 0 in the device row
    assert np.all(obj[basis] == 0.0)


@pytest.fixture(scope="module")
def width_oracle():
    """Config 4's width (N + 1 = 196,609 columns) at m = 2048: the oracle's 308
    pivots (3.2 GB tableau), shared by the K = 96 and K = 64 runs below."""
    m, n, piv = 2048, 194560, 308
    o = _oracle(m, n + m + 1)
    o.generate(n, SEED, 0)
    ores = o.solve(piv, 0)
    assert ores.pivots == piv
    yield m, n, piv, o, ores
    o.close()


@pytest.mark.parametrize("defer", [96, 64])
def test_config4_width_bitwise(lpg, width_oracle, defer, monkeypatch):
    """config 4's exact pivot path -- the two-kernel pair
    (k_prep_d / k_select_d: 196,609 columns do not fit the persistent kernel's
    slices) with 96-pivot blocks (config 4 on one GPU) and 64-pivot blocks
    (one rank of its 8-way split) -- against the oracle at config 4's width:
    308 pivots = three whole 96-pivot blocks + 20 (four whole 64-pivot blocks +
    52), bitwise: pivot log, basis, objective row, column 0, every pivot row
    and 64 sampled rows."""
    m, n, piv, o, ores = width_oracle
    monkeypatch.setenv("LPG_DEFER", str(defer))
    e = lpg.Engine(m, n + m + 1)
    monkeypatch.delenv("LPG_DEFER")
    assert e.info.defer_k == defer and e.info.pivot_wg == 0 and e.info.column_trade == 1
    e.generate(n, SEED, lpg.GEN_DENSE)
    e.reserve_log(piv + 8)
    res = e.solve(piv, lpg.RULE_DANTZIG)
    assert res.status_name == "ITER_LIMIT" and res.pivots == piv and res.objective == ores.objective
    log = _log(e)
    assert log == _log(o)
    basis = e.get_basis()
    assert np.array_equal(basis, o.get_basis())
    assert np.array_equal(e.get_rows(m, 1), o.get_rows(m, 1)), "objective row"
    rng = np.random.default_rng(11)
    rows = sorted(set(rng.choice(m, 64, replace=False).tolist()) | {r for _, r in log} | {0, m - 1})
    x0 = e.get_column0()
    for i in rows:
        ri = e.get_rows(i, 1)
        assert np.array_equal(ri, o.get_rows(i, 1)), f"row {i}"
        assert x0[i] == ri[0, 0]
    e.close()
