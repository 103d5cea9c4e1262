"""The persistent pivot kernel (k_pivot_block, lpg_block.hip) vs the oracle
and vs the two-kernel pivot (k_prep_d / k_select_d), bitwise.

One launch runs a whole run of pivots: each workgroup keeps its slice of the
pending P rows and C columns in LDS, and the per-pivot grid decisions are
all-to-alls of write-through records inside the launch. The arithmetic and
the tie-breaks are the two-kernel pair's, so pivot logs, bases and whole
tableaus must equal the oracle's (np.array_equal) for every workgroup split
(LPG_PERSIST_WG), block size (LPG_DEFER), pricing rule, objective-row count
(Big-M keeps two) and for runs that start inside a block (lpg_solve's
growing batches, reads that flush a partial block).
Reference anchor: the loop is absent upstream (Source/simplex.c:40 -> :65).
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lpo import GEN_ARTIFICIAL, Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    assert lpg.device_count() >= 1, "no GPU visible"
    return lpg


def _log(x):
    k, r = x.get_log()
    return list(zip(k.tolist(), r.tolist()))


def _engine(lpg, monkeypatch, m, ncols, defer=None, wg=None, persist=None, **kw):
    env = {"LPG_DEFER": defer, "LPG_PERSIST_WG": wg, "LPG_PERSIST": persist}
    for k, v in env.items():
        if v is not None:
            monkeypatch.setenv(k, str(v))
    e = lpg.Engine(m, ncols, **kw)
    for k, v in env.items():
        if v is not None:
            monkeypatch.delenv(k)
    return e


def _fits(m, ncols, defer, wg):
    """block_geometry's rule (lpg_block.hip): <= 256 columns and rows per
    workgroup, the LDS slices within 150 KB."""
    if wg is None:
        return True
    ncp = (ncols + 1) & ~1
    cw, rw = -(-ncp // wg), -(-m // wg)
    s = ((defer + 15) & ~15) + 2                           # slot_stride
    return cw <= 256 and rw <= 256 and s * (cw + rw) * 8 <= 150 * 1024


def _assert_same(e, o, m):
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


def test_engaged_where_the_slices_fit(lpg, monkeypatch):
    e = _engine(lpg, monkeypatch, 600, 1701, defer=32)
    assert e.info.pivot_wg > 0
    assert _engine(lpg, monkeypatch, 600, 1701, defer=32, persist=0).info.pivot_wg == 0
    assert _engine(lpg, monkeypatch, 600, 1701, defer=0).info.pivot_wg == 0      # eager updates
    assert _engine(lpg, monkeypatch, 600, 1701, defer=65).info.pivot_wg > 0      # 65..96: two lane banks
    assert _engine(lpg, monkeypatch, 600, 1701, defer=97).info.pivot_wg == 0     # blocks of > 96 pivots: the pair
    # 256 workgroups hold at most 256 columns each: wider tableaus keep the pair
    assert _engine(lpg, monkeypatch, 8, 256 * 256 + 3, defer=8).info.pivot_wg == 0


@pytest.mark.parametrize("trade", ["0", "1"])
@pytest.mark.parametrize("wg", [None, 3, 7, 64, 256])
@pytest.mark.parametrize("defer", [8, 32, 64, 96])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(200, 300, 12, 0, 0), (48, 48, 14, 1, 1), (257, 100, 15, 1, 0)])
def test_to_optimality(lpg, monkeypatch, wg, defer, m, n, seed, kind, rule, trade):
    monkeypatch.setenv("LPG_NO_REORDER", "0" if trade == "1" else "1")
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, wg=wg)
    if e.info.pivot_wg == 0 and not _fits(m, n + m + 1, defer, wg):
        pytest.skip("this split holds neither the all-column nor the region slices")
    assert e.info.pivot_wg > 0 and e.info.region == (1 if trade == "1" else 0)
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == 1
    assert res.pivots == ores.pivots > 0 and res.objective == ores.objective
    _assert_same(e, o, m)


def _edge_cases(defers, keep_slow):
    """Every block size on the dense Dantzig LP; the KM-style Bland LP (4 s a
    case: thousands of degenerate pivots) at the bank / batch edges in
    keep_slow only, the rest `extended` (LPG_EXTENDED_TESTS=1, conftest.py)."""
    out = []
    for case in ((300, 450, 21, 0, 0), (257, 300, 22, 1, 1)):
        for d in defers:
            slow = case[0] == 257 and d not in keep_slow
            out.append(pytest.param(d, *case, marks=pytest.mark.extended) if slow else pytest.param(d, *case))
    return out


@pytest.mark.parametrize("defer,m,n,seed,kind,rule",
                         _edge_cases([15, 16, 17, 31, 33, 47, 48, 49, 63, 64, 65, 79, 80, 81, 95, 96], (16, 17, 64, 65, 96)))
def test_chain_batch_edges(lpg, monkeypatch, defer, m, n, seed, kind, rule):
    """The chains run in batches of 16 slots (lpg_block.hip chain<>): block
    sizes on either side of every batch edge, dense (Dantzig) and degenerate
    (Bland: pivot rows that recur inside a block take the restart form); from
    65 pending slots on the per-slot scalars take a second lane bank."""
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    assert e.info.pivot_wg > 0
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status and res.pivots == ores.pivots > 2 * defer
    _assert_same(e, o, m)


@pytest.mark.parametrize("xcd1", [None, "0"])
@pytest.mark.parametrize("wg", [None, 17])
def test_config2_to_optimality(lpg, monkeypatch, wg, xcd1):
    """Config 2 to optimality, bitwise the oracle; its 13 (or 17) workgroups
    run on one XCD (blocks 8 w of an 8 x nwg grid) or spread (LPG_PIVOT_XCD1=0)."""
    if xcd1 is not None:
        monkeypatch.setenv("LPG_PIVOT_XCD1", xcd1)
    m, n = 1024, 2048
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=32, wg=wg)
    assert e.info.pivot_wg > 0
    o = Oracle(m, n + m + 1, nthreads=8)
    e.generate(n, 20220518, 0)
    o.generate(n, 20220518, 0)
    res = e.solve(200_000, 0)
    ores = o.solve(200_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("defer", [64, 96])
def test_runs_that_start_inside_a_block(lpg, monkeypatch, defer):
    """Enqueue 5, 9, 17, ... pivots: every launch after the first starts at a
    pending index > 0 and reloads the earlier slots' slices from Pbuf / Cbuf
    (with 96-slot blocks also past slot 64, the second lane bank); a read in
    between flushes a partial block."""
    m, n = 600, 900
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    assert e.info.pivot_wg > 0
    o = Oracle(m, n + m + 1)
    e.generate(n, 77, 0)
    o.generate(n, 77, 0)
    e.reserve_log(4096)
    total = 0
    for step in (5, 9, 17, 1, 33, 2, 64, 7, 70, 3, 90):
        e.enqueue(step, 0)
        total += step
        if step == 17:
            e.get_rows(0, 4)                      # flushes the 31 pending pivots
    res = e.sync()
    ores = o.solve(total, 0)
    assert res.pivots == ores.pivots == total
    _assert_same(e, o, m)


@pytest.mark.parametrize("defer", [32, 96])
@pytest.mark.parametrize("m,n,rule", [(257, 300, 0), (640, 512, 1)])
def test_big_m_two_objective_rows(lpg, monkeypatch, m, n, rule, defer):
    art_first = 1 + n + (m + 1) // 2
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, flags=lpg._lib.FLAG_BIG_M)
    assert e.info.pivot_wg > 0 and e.info.nobj == 2
    o = Oracle(m, n + m + 1, nobj=2)
    e.generate(n, 9, GEN_ARTIFICIAL)
    o.generate(n, 9, GEN_ARTIFICIAL)
    r = e.solve_big_m(art_first, None, 100_000, rule)
    ro = o.solve_big_m(art_first, None, 100_000, rule)
    assert r.status == ro.status and r.pivots == ro.pivots > 0 and r.objective == ro.objective
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + 2), o.get_rows())


@pytest.mark.parametrize("defer", [64, 96])
@pytest.mark.parametrize("m,n,piv", [(4096, 8192, 200), (2048, 20000, 150)])
def test_same_as_two_kernel_pair(lpg, monkeypatch, m, n, piv, defer):
    """At sizes where the oracle is slow the persistent kernel is checked
    against the two-kernel pair: same log, same rows (sampled)."""
    a = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    b = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, persist=0)
    assert a.info.pivot_wg > 0 and b.info.pivot_wg == 0
    for e in (a, b):
        e.generate(n, 5, 0)
        e.solve(piv, 0)
    assert _log(a) == _log(b)
    assert np.array_equal(a.get_basis(), b.get_basis())
    rows = np.random.default_rng(1).choice(m, 48, replace=False)
    for i in list(rows) + [m]:
        assert np.array_equal(a.get_rows(int(i), 1), b.get_rows(int(i), 1))


@pytest.mark.parametrize("defer", [8, 64])
def test_two_kernel_pair_still_bitwise(lpg, monkeypatch, defer):
    """LPG_PERSIST=0 (and tableaus too wide for the slices, and every
    communicator) keep k_prep_d / k_select_d: still the oracle's results."""
    m, n = 200, 300
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, persist=0)
    assert e.info.pivot_wg == 0
    o = Oracle(m, n + m + 1)
    e.generate(n, 12, 0)
    o.generate(n, 12, 0)
    res = e.solve(200_000, 0)
    ores = o.solve(200_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


def test_reload_into_a_solved_context(lpg, monkeypatch):
    """Solve, load a different tableau into the same context (its pending
    block flushed and its column order restored first), solve again: both
    solves equal the oracle's (lpg_load_rows after pivoting)."""
    m, n = 220, 330
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=32)
    assert e.info.pivot_wg > 0
    o = Oracle(m, n + m + 1)
    e.generate(n, 31, 0)
    o.generate(n, 31, 0)
    e.solve(45, 0)                                  # stops inside a block: 13 pivots pending
    o.solve(45, 0)
    _assert_same(e, o, m)
    o2 = Oracle(m, n + m + 1)
    o2.generate(n, 32, 0)                           # another LP, loaded through the host path
    T = o2.get_rows()
    basis = np.arange(n + 1, n + m + 1, dtype=np.int64)
    e.load_tableau(T, basis)
    r2 = e.solve(200_000, 0)
    ro2 = o2.solve(200_000, 0)
    assert r2.status == ro2.status == 1 and r2.objective == ro2.objective
    assert np.array_equal(e.get_rows(0, m + 1), o2.get_rows())


@pytest.mark.parametrize("persist", [None, 0])
@pytest.mark.parametrize("case", ["nan_b", "inf_b", "overflowing_ratio"])
def test_numeric_rule_matches_oracle(lpg, monkeypatch, persist, case):
    """The oracle stops NUMERIC when the chosen row's pivot element or b is not
    finite (oracle/lpo.c lpo_solve) and otherwise pivots, an overflowing
    ratio b / a included: the persistent kernel and the pair agree."""
    m, n = 60, 90
    o = Oracle(m, n + m + 1)
    o.generate(n, 5, 0)
    T = o.get_rows().copy()
    basis = np.arange(n + 1, n + m + 1, dtype=np.int64)
    if case == "nan_b":
        T[7, 0] = np.nan
    elif case == "inf_b":
        T[7, 0] = -np.inf
    else:                                      # b finite, b / a overflows for the entering column
        T[7, 0] = 1e308
        T[7, 1:n + 1] = 1e-10
    o2 = Oracle(m, n + m + 1)
    o2.load_tableau(T, basis)
    ores = o2.solve(1000, 0)
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=32, persist=persist)
    e.load_tableau(T, basis)
    res = e.solve(1000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots
    assert _log(e) == _log(o2)


def _tied_lp(m, n, seed):
    """A <= LP whose objective and coefficients take few distinct values
    (quarters), so many columns share the least reduced cost exactly: the
    pricing sweep's key ties (one-granule records, resolved by j) are hit at
    the first pivots and again wherever the quantised entries repeat."""
    rng = np.random.default_rng(seed)
    T = np.zeros((m + 1, n + m + 1))
    T[:m, 0] = 4.0 + rng.integers(0, 8, m)
    T[:m, 1:n + 1] = rng.integers(1, 5, (m, n)) / 4.0
    T[np.arange(m), n + 1 + np.arange(m)] = 1.0
    T[m, 1:n + 1] = -(1.0 + rng.integers(0, 2, n) / 4.0)
    return T, n + 1 + np.arange(m, dtype=np.int64)


@pytest.mark.parametrize("wg", [None, 7])
@pytest.mark.parametrize("defer", [32, 64])
@pytest.mark.parametrize("m,n,seed", [(300, 500, 3), (97, 1500, 4)])
def test_pricing_key_ties(lpg, monkeypatch, wg, defer, m, n, seed):
    T, basis = _tied_lp(m, n, seed)
    assert _fits(m, n + m + 1, defer, wg)
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, wg=wg)
    assert e.info.pivot_wg > 0
    e.load_rows(0, T)
    e.set_basis(basis)
    o = Oracle(m, n + m + 1)
    o.load_tableau(T, basis)
    res = e.solve(3000, 0)
    ores = o.solve(3000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots > 0
    _assert_same(e, o, m)


@pytest.mark.parametrize("persist", [None, 0])
@pytest.mark.parametrize("what", ["npend", "kq", "lv", "rq", "ahead"])
def test_inconsistent_pending_block_stops_numeric(lpg, monkeypatch, what, persist):
    """k_swap_plan's guard (a stopped block left npend
    ahead of the slots it filled, and the plan indexed inv / colmap / Cbuf
    with what it found, faulting the GPU). The test-hook build
    (liblpg_testhooks.so; the product library has no hook) corrupts the
    pending block before the second flush, with the column trade on: the loop
    stops with NUMERIC, the flush applies nothing, lpg_last_error names the
    field. "ahead" leaves npend one past the slots a partial block filled:
    the slot it reaches holds the never-filled sentinels every block end
    writes back, not the previous block's in-range values, so the
    plan refuses it as well. The context then refuses every pivoting call
    until the LP is regenerated (its basis and constraint rows
    disagree), after which it solves bitwise -- and the GPU is healthy."""
    from linearprogramming_amd import _lib as L
    m, n = 600, 1100
    hooks = L.load_testhooks()
    monkeypatch.setenv("LPG_TEST_PENDING_FAULT", f"1:{what}")
    monkeypatch.setenv("LPG_NO_REORDER", "0")          # the column trade on: the plan indexes with kq / lv
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=32, persist=persist, lib=hooks)
    monkeypatch.delenv("LPG_TEST_PENDING_FAULT")
    assert e.info.column_trade == 1 and (e.info.pivot_wg > 0) == (persist is None)
    e.generate(n, 5, 0)
    # "ahead": 40 pivots = one full block, then a partial one of 8 (flush 1 at the solve's end)
    field = "kq" if what == "ahead" else what
    with pytest.raises(lpg.LPGError, match=rf"pending block inconsistent at the flush \({field}\["):
        e.solve(40 if what == "ahead" else 100_000, 0)
    with pytest.raises(lpg.LPGError, match=r"context unusable"):
        e.solve(100_000, 0)
    if what == "npend" and persist is None:
        # a partial (here one-row) reload keeps it refused; only a
        # replaced basis or a regenerated LP clears it
        e.load_rows(0, e.get_rows(0, 1))
        with pytest.raises(lpg.LPGError, match=r"context unusable"):
            e.solve(100_000, 0)
    e.generate(n, 5, 0)                                # a rewritten tableau: usable again
    res = e.solve(100_000, 0)
    o = Oracle(m, n + m + 1)
    o.generate(n, 5, 0)
    ores = o.solve(100_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots > 64
    _assert_same(e, o, m)
    e.close()


def test_product_library_has_no_test_hook(lpg, monkeypatch):
    """the fault hook is compiled into the test-hook build only --
    the product library ignores LPG_TEST_PENDING_FAULT and solves bitwise."""
    m, n = 600, 1100
    monkeypatch.setenv("LPG_TEST_PENDING_FAULT", "1:npend")
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=32)
    monkeypatch.delenv("LPG_TEST_PENDING_FAULT")
    e.generate(n, 5, 0)
    res = e.solve(100_000, 0)
    o = Oracle(m, n + m + 1)
    o.generate(n, 5, 0)
    ores = o.solve(100_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)
    e.close()
