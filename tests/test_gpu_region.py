"""Region mode of the persistent pivot kernel (k_pivot_block<.., REG>,
lpg_block.hip) vs the oracle, bitwise.

In region mode the column slices hold only the columns whose pending P
entries can be nonzero: the nonbasic columns of the block start (which the
column trade keeps in place from block to block) and one spare slot per
pending pivot that takes over the column leaving the basis at that pivot. The
arithmetic is the all-column kernel's, so pivot logs, bases and whole tableaus
must equal the oracle's (np.array_equal) -- across block sizes (32, 64, 96 and
the lane-bank edges), Dantzig and Bland, dense and degenerate LPs, workgroup
splits (a spare slot per pending pivot: several per workgroup when the grid is
small), launches that start inside a block (spares restored from Pbuf), host
reads between launches (the region rebuilt for the restored column order),
loaded tableaus (the unit-column precondition checked; a tableau that fails
it runs without region mode), two-phase with its forced drive-out pivots,
and an inconsistent block end (rbad: the region rebuilt, the pivots re-run).
Reference anchor: the loop is absent upstream (Source/simplex.c:40 -> :65).
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lpo import GEN_ARTIFICIAL, Oracle
from util import degenerate_two_phase_lp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    assert lpg.device_count() >= 1, "no GPU visible"
    return lpg


def _engine(lpg, monkeypatch, m, ncols, defer=None, wg=None, region=None, **kw):
    env = {"LPG_DEFER": defer, "LPG_PERSIST_WG": wg, "LPG_REGION": region, "LPG_NO_REORDER": "0"}
    for k, v in env.items():
        if v is not None:
            monkeypatch.setenv(k, str(v))
    e = lpg.Engine(m, ncols, **kw)
    for k, v in env.items():
        if v is not None:
            monkeypatch.delenv(k)
    return e


def _fits(m, n, defer, wg):
    """block_geometry_region's rule (lpg_block.hip) for a forced split: column
    threads (live + spares + column 0) and rows <= 256 each, LDS within 150 KB."""
    if wg is None:
        return True
    nlive, s = n, ((defer + 15) & ~15) + 2
    cw, rw, nsp = -(-nlive // wg), -(-m // wg), -(-defer // wg)
    x = cw + nsp + 1
    return x <= 256 and rw <= 256 and (x + rw) * s * 8 <= 150 * 1024


def _log(x):
    k, r = x.get_log()
    return list(zip(k.tolist(), r.tolist()))


def _assert_same(e, o, m, nobj=1):
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + nobj), o.get_rows())


def test_engaged_with_the_trade_and_one_objective_row(lpg, monkeypatch):
    e = _engine(lpg, monkeypatch, 600, 1701, defer=64)
    assert e.info.pivot_wg > 0 and e.info.region == 1 and e.info.column_trade == 1
    assert _engine(lpg, monkeypatch, 600, 1701, defer=64, region=0).info.region == 0
    monkeypatch.setenv("LPG_NO_REORDER", "1")
    assert lpg.Engine(600, 1701).info.region == 0                           # no trade: all-column slices
    monkeypatch.delenv("LPG_NO_REORDER")
    assert _engine(lpg, monkeypatch, 600, 1701, defer=64, flags=lpg._lib.FLAG_BIG_M).info.region == 0   # two rows


@pytest.mark.parametrize("wg", [None, 3, 13, 64])
@pytest.mark.parametrize("defer", [32, 64, 96])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(200, 300, 12, 0, 0), (48, 48, 14, 1, 1), (257, 100, 15, 1, 0),
                                                (300, 700, 16, 0, 1)])
def test_to_optimality(lpg, monkeypatch, wg, defer, m, n, seed, kind, rule):
    if not _fits(m, n, defer, wg):
        pytest.skip("this split does not hold the region's slices")
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, wg=wg)
    assert e.info.region == 1 and e.info.pivot_wg == (wg or e.info.pivot_wg)
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == 1
    assert res.pivots == ores.pivots > 0 and res.objective == ores.objective
    _assert_same(e, o, m)


def _edge_cases(defers, keep_slow):
    """As tests/test_gpu_block.py: the KM-style Bland LP at keep_slow only,
    the other block sizes `extended` (LPG_EXTENDED_TESTS=1)."""
    out = []
    for case in ((300, 450, 21, 0, 0), (257, 300, 22, 1, 1)):
        for d in defers:
            slow = case[0] == 257 and d not in keep_slow
            out.append(pytest.param(d, *case, marks=pytest.mark.extended) if slow else pytest.param(d, *case))
    return out


@pytest.mark.parametrize("defer,m,n,seed,kind,rule", _edge_cases([16, 17, 63, 64, 65, 80, 95, 96], (16, 64, 96)))
def test_block_size_edges(lpg, monkeypatch, defer, m, n, seed, kind, rule):
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    assert e.info.region == 1
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status and res.pivots == ores.pivots > 2 * defer
    _assert_same(e, o, m)


@pytest.mark.parametrize("defer", [64, 96])
def test_runs_that_start_inside_a_block(lpg, monkeypatch, defer):
    """Launches of 5, 9, 17, ... pivots start at pending indices inside the
    block: the spares of the earlier launches are restored from lv / kq / inv
    and Pbuf; a host read in between restores the caller's column order, after
    which the region is rebuilt for it."""
    m, n = 600, 900
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    assert e.info.region == 1
    o = Oracle(m, n + m + 1)
    e.generate(n, 77, 0)
    o.generate(n, 77, 0)
    e.reserve_log(4096)
    total = 0
    for step in (5, 9, 17, 1, 33, 2, 64, 7, 70, 3, 90):
        e.enqueue(step, 0)
        total += step
        if step in (17, 7):
            e.get_rows(0, 4)
    res = e.sync()
    ores = o.solve(total, 0)
    assert res.pivots == ores.pivots == total
    _assert_same(e, o, m)


def test_loaded_tableau_passes_the_unit_check(lpg, monkeypatch):
    """lpg_load_rows + lpg_set_basis: the basic (slack) columns are exact unit
    vectors with zero reduced costs, so region mode stays on."""
    m, n = 300, 500
    o = Oracle(m, n + m + 1)
    o.generate(n, 5, 0)
    T = o.get_rows().copy()
    basis = np.arange(n + 1, n + m + 1, dtype=np.int64)
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=64)
    e.load_tableau(T, basis)
    res = e.solve(200_000, 0)
    assert e.info.region == 1
    ores = o.solve(200_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


def test_loaded_tableau_failing_the_unit_check_leaves_region_mode(lpg, monkeypatch):
    """A basic column that is not an exact unit vector (row 7's slack scaled
    by 2, so its basic value is not 1) breaks the region's premise: the
    context leaves region mode at the bootstrap and still solves bitwise."""
    m, n = 300, 500
    o0 = Oracle(m, n + m + 1)
    o0.generate(n, 5, 0)
    T = o0.get_rows().copy()
    T[7, n + 1 + 7] = 2.0
    basis = np.arange(n + 1, n + m + 1, dtype=np.int64)
    o = Oracle(m, n + m + 1)
    o.load_tableau(T, basis)
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=64)
    assert e.info.region == 1
    e.load_tableau(T, basis)
    res = e.solve(200_000, 0)
    assert e.info.region == 0
    ores = o.solve(200_000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots
    _assert_same(e, o, m)


def test_loaded_tableau_with_negative_zero_in_a_basic_column_leaves_region_mode(lpg, monkeypatch):
    """The unit check is bit for bit: a -0 in a basic column is not the +0 the
    column trade writes for a leaving column's base data (k_move_cols writes
    the unit vector without reading it), so such a tableau leaves region mode
    and still solves bitwise the oracle."""
    m, n = 300, 500
    o0 = Oracle(m, n + m + 1)
    o0.generate(n, 5, 0)
    T = o0.get_rows().copy()
    T[11, n + 1 + 3] = -0.0
    basis = np.arange(n + 1, n + m + 1, dtype=np.int64)
    o = Oracle(m, n + m + 1)
    o.load_tableau(T, basis)
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=64)
    e.load_tableau(T, basis)
    res = e.solve(200_000, 0)
    assert e.info.region == 0
    ores = o.solve(200_000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("unit", ["0", "1"])
@pytest.mark.parametrize("defer", [64, 96])
def test_leaving_columns_written_as_unit_vectors(lpg, monkeypatch, unit, defer):
    """The column trade's move of the leaving columns (k_move_cols) with their
    base data read (LPG_MOVE_UNIT=0) or written as the unit vector of their
    row (default in region blocks): bitwise the oracle either way, over whole
    blocks with many trades."""
    monkeypatch.setenv("LPG_MOVE_UNIT", unit)
    m, n = 2048, 4096
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    o = Oracle(m, n + m + 1)
    e.generate(n, 77, 0)
    o.generate(n, 77, 0)
    res = e.solve(5 * defer + 9, 0)
    assert e.info.region == 1
    ores = o.solve(5 * defer + 9, 0)
    assert res.pivots == ores.pivots == 5 * defer + 9
    _assert_same(e, o, m)


@pytest.mark.parametrize("defer", [32, 96])
@pytest.mark.parametrize("m,n,rule", [(120, 150, 0), (257, 300, 1)])
def test_two_phase(lpg, monkeypatch, defer, m, n, rule):
    art_first = 1 + n + (m + 1) // 2
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    assert e.info.region == 1
    o = Oracle(m, n + m + 1)
    e.generate(n, 9, GEN_ARTIFICIAL)
    o.generate(n, 9, GEN_ARTIFICIAL)
    r = e.solve_two_phase(art_first, None, 100_000, rule)
    ro = o.solve_two_phase(art_first, None, 100_000, rule)
    assert r.status == ro.status and r.pivots == ro.pivots > 0 and r.objective == ro.objective
    _assert_same(e, o, m)


@pytest.mark.parametrize("defer", [32, 96])
def test_two_phase_forced_drive_out(lpg, monkeypatch, defer):
    """Phase I leaves an artificial basic at zero; the drive-out is a forced
    pivot (lpg_pivot) on a negative element, whose block's column trade is
    then incomplete (k_swap_plan sets rbad): the next launch stops, the region
    is rebuilt and the pivots re-run -- the solve stays the oracle's."""
    T, basis, art_first = degenerate_two_phase_lp(200, 260, 3)
    cost = None
    m, ncols = T.shape[0] - 1, T.shape[1]
    e = _engine(lpg, monkeypatch, m, ncols, defer=defer)
    assert e.info.region == 1
    e.load_tableau(T, basis)
    o = Oracle(m, ncols)
    o.load_tableau(T, basis)
    r = e.solve_two_phase(art_first, cost, 100_000, 0)
    ro = o.solve_two_phase(art_first, cost, 100_000, 0)
    assert r.status == ro.status and r.pivots == ro.pivots and r.objective == ro.objective
    _assert_same(e, o, m)


@pytest.mark.parametrize("flush", [0, 2])
def test_region_stall_mid_enqueue_recovers_bitwise(lpg, monkeypatch, flush):
    """the kStallRegion path itself. A forced pivot is always
    followed by a bootstrap that rebuilds the region before any launch reads
    rbad, so the drive-out test above never stalls. The test-hook build
    (liblpg_testhooks.so) sets rbad after block `flush`'s swap plan, as an
    incomplete column trade would, in the middle of ONE lpg_enqueue: the next
    region launch runs no pivot (neither does any launch after it),
    recover_region counts it, and lpg_sync re-runs the lost pivots after a
    region rebuild -- pivot count, log, basis and whole tableau the oracle's."""
    from linearprogramming_amd import _lib as L
    m, n, K = 700, 1300, 32
    hooks = L.load_testhooks()
    monkeypatch.setenv("LPG_TEST_REGION_BAD", str(flush))
    e = _engine(lpg, monkeypatch, m, n + m + 1, defer=K, lib=hooks)
    monkeypatch.delenv("LPG_TEST_REGION_BAD")
    assert e.info.region == 1 and e.info.pivot_wg > 0
    e.generate(n, 17, 0)
    e.reserve_log(6 * K + 8)
    e.enqueue(6 * K, 0)
    res = e.sync()
    assert e.info.region_recoveries == 1, "the hook's rbad must have stopped a launch"
    o = Oracle(m, n + m + 1)
    o.generate(n, 17, 0)
    ores = o.solve(6 * K, 0)
    assert res.pivots == ores.pivots == 6 * K and res.objective == ores.objective
    _assert_same(e, o, m)
    e.close()


@pytest.mark.parametrize("defer", [64, 96])
@pytest.mark.parametrize("m,n,piv", [(4096, 8192, 300), (2048, 20000, 250)])
def test_same_as_all_column_kernel(lpg, monkeypatch, m, n, piv, defer):
    """At sizes where the oracle is slow: region mode against the all-column
    slices and the two-kernel pair -- same log, same rows (sampled)."""
    a = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
    b = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer, region=0)
    assert a.info.region == 1 and b.info.region == 0
    for e in (a, b):
        e.generate(n, 5, 0)
        e.solve(piv, 0)
    assert _log(a) == _log(b)
    assert np.array_equal(a.get_basis(), b.get_basis())
    rows = np.random.default_rng(1).choice(m, 48, replace=False)
    for i in list(rows) + [m]:
        assert np.array_equal(a.get_rows(int(i), 1), b.get_rows(int(i), 1))


@pytest.mark.parametrize("xcd,m,n,seed,kind,rule,defer", [
    # the KM-style Bland LP (6-7 s a case) with the grouped queue only; its global
    # queue and H = 8 classes are `extended` (LPG_EXTENDED_TESTS=1)
    pytest.param(x, *lp, marks=pytest.mark.extended if (lp[0] == 257 and x != "1") else ())
    for lp in [(600, 900, 31, 0, 0, 64), (257, 300, 22, 1, 1, 96), (1100, 700, 33, 0, 0, 32)]
    for x in ["0", "1", "h8"]])
def test_tile_liveness_map(lpg, monkeypatch, xcd, m, n, seed, kind, rule, defer):
    """The block pass skips tiles without a block-start nonbasic column (tlive,
    built with the region) and loads only the leaving columns' P entries on
    the tiles they sit in: bitwise the oracle, and the pass reads and writes
    exactly the bytes it does with the map off (LPG_FLUSH_TLIVE=0), i.e. the
    map skips only all-zero column pairs."""
    monkeypatch.setenv("LPG_FLUSH_XCD", xcd)
    runs = {}
    for tl in ("1", "0"):
        monkeypatch.setenv("LPG_FLUSH_TLIVE", tl)
        e = _engine(lpg, monkeypatch, m, n + m + 1, defer=defer)
        assert e.info.region == 1
        e.generate(n, seed, kind)
        e.set_timing(True)
        e.get_timing()
        res = e.solve(200_000, rule)
        runs[tl] = (e, res, e.get_timing().update_bytes)
    o = Oracle(m, n + m + 1)
    o.generate(n, seed, kind)
    ores = o.solve(200_000, rule)
    for tl, (e, res, _) in runs.items():
        assert res.status == ores.status and res.pivots == ores.pivots
        _assert_same(e, o, m)
    assert runs["1"][2] == runs["0"][2] > 0
