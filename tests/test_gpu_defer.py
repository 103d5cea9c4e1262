"""Deferred (blocked) updates vs eager updates and the oracle, bitwise.

In deferred mode the constraint rows lag behind by up to K pending pivots;
prep / select evaluate the pending chain x = (i == r_q) ? P_q[j] :
fma(-C_q[i], P_q[j], x) for the entries they need and k_flush applies the
block in one pass. The operations per tableau entry are exactly the eager
ones, so every pivot log, basis, objective and whole tableau must equal the
oracle's (np.array_equal) for any block size K, including blocks cut short by
a read (lpg_get_rows), by the end of a solve, or by an early stop.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lpo import Oracle

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


def _assert_same(e, o, m):
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


def _engine(lpg, monkeypatch, k, m, ncols, **kw):
    monkeypatch.setenv("LPG_DEFER", str(k))
    e = lpg.Engine(m, ncols, **kw)
    monkeypatch.delenv("LPG_DEFER")
    return e


@pytest.mark.parametrize("trade", ["0", "1"])
@pytest.mark.parametrize("k", [0, 1, 2, 3, 8, 16, 31, 32, 64, 65, 100, 128])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(200, 300, 12, 0, 0), (48, 48, 14, 1, 1), (257, 100, 15, 1, 0)])
def test_block_sizes_to_optimality(lpg, monkeypatch, k, m, n, seed, kind, rule, trade):
    """Every block size, with the block-end column trade (trade 1, forced on
    for these small tableaus) and without it (their default)."""
    monkeypatch.setenv("LPG_NO_REORDER", "0" if trade == "1" else "1")
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    assert e.info.column_trade == (1 if trade == "1" and k > 0 else 0)
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == 1
    assert res.pivots == ores.pivots > 0 and res.objective == ores.objective
    _assert_same(e, o, m)


@pytest.mark.parametrize("k", [8, 32, 64, 128])
def test_config2_to_optimality(lpg, monkeypatch, k):
    m, n = 1024, 2048
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1, nthreads=8)
    e.generate(n, 20220518, 0)
    o.generate(n, 20220518, 0)
    res = e.solve(200_000, 0)
    ores = o.solve(200_000, 0)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("k", [32, 128])
def test_reads_inside_a_block(lpg, monkeypatch, k):
    """Reads in the middle of a block flush it; the loop then continues from the
    flushed tableau and stays on the oracle's path."""
    m, n = 150, 220
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1)
    e.generate(n, 71, 0)
    o.generate(n, 71, 0)
    for step in (5, 1, 13, 32, 40, 3, 70, 90):
        e.enqueue(step, 0)
        assert e.get_column0().shape == (m,)           # flushes
        o.solve(step, 0)
        _assert_same(e, o, m)
    res, ores = e.solve(100_000, 0), o.solve(100_000, 0)
    assert res.pivots == ores.pivots and res.objective == ores.objective
    _assert_same(e, o, m)


def test_enqueue_past_optimal_partial_block(lpg, monkeypatch):
    """The LP finishes inside a block: the later pivots are device no-ops and the
    flush applies only the pivots actually taken."""
    m, n = 40, 60
    e = _engine(lpg, monkeypatch, 32, m, n + m + 1)
    o = Oracle(m, n + m + 1)
    e.generate(n, 21, 0)
    o.generate(n, 21, 0)
    ores = o.solve(100_000, 0)
    e.enqueue(ores.pivots + 45, 0)
    res = e.sync()
    assert res.status_name == "OPTIMAL" and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("kernel,k", [("m", 8), ("m", 16), ("m", 32), ("w", 8), ("w", 32), ("w", 64), ("w", 96), ("w", 128)])
def test_flush_kernels_identical(lpg, monkeypatch, kernel, k):
    """k_flushm and k_flushw at their block sizes (LPG_FLUSH_KERNEL forces one)."""
    monkeypatch.setenv("LPG_FLUSH_KERNEL", kernel)
    m, n = 300, 700
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1)
    e.generate(n, 24, 0)
    o.generate(n, 24, 0)
    res = e.solve(100, 0)
    o.solve(100, 0)
    assert res.pivots == 100
    _assert_same(e, o, m)


def test_flush_accounting(lpg, monkeypatch):
    """Without column skipping a flush reads and writes every constraint-row entry
    once: 16 B x m x ncols per flush, one flush per K pivots."""
    m, n, k = 256, 512, 8
    monkeypatch.setenv("LPG_NO_SKIP", "1")
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    e.generate(n, 81, 0)
    e.set_timing(True)
    e.get_timing()
    e.enqueue(32, 0)
    e.sync()
    t = e.get_timing()
    assert t.update_count == 32 // k
    assert t.update_bytes == t.update_count * 16 * m * (n + m + 1)
    assert t.update_ms > 0 and t.select_ms == 0      # deferred mode times the flushes only


def test_eager_flag(lpg):
    e = lpg.Engine(64, 64 + 96 + 1, flags=lpg._lib.FLAG_EAGER)
    o = Oracle(64, 64 + 96 + 1)
    e.generate(96, 5, 0)
    o.generate(96, 5, 0)
    assert e.solve(10_000, 0).pivots == o.solve(10_000, 0).pivots
    _assert_same(e, o, 64)


def test_bad_block_size(lpg, monkeypatch):
    monkeypatch.setenv("LPG_DEFER", "129")
    with pytest.raises(lpg.LPGError):
        lpg.Engine(8, 20)


@pytest.mark.parametrize("kernel,k", [("m", 3), ("m", 8), ("m", 32), ("w", 3), ("w", 32), ("w", 64), ("w", 77), ("w", 96), ("w", 100), ("w", 128)])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(203, 301, 16, 0, 0), (48, 48, 14, 1, 1)])
def test_flush_kernels_block_sizes(lpg, monkeypatch, kernel, k, m, n, seed, kind, rule):
    """k_flushm (strip-staged C) and k_flushw (tall banded items) at every
    compiled block bound, to optimality, against the oracle (odd shapes: ragged
    column tiles, strips and bands)."""
    monkeypatch.setenv("LPG_FLUSH_KERNEL", kernel)
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("xcd,k,m,n,seed,kind,rule", [
    # the 1100 x 1300 Bland LP at 3-pivot blocks (2.4-9 s a case) with the middle
    # class counts h1 / h2 / h4 is `extended` (LPG_EXTENDED_TESTS=1): h8 and the
    # global / grouped queues keep that shape, every other case keeps them all
    pytest.param(x, k, *lp, marks=pytest.mark.extended if (lp[0] == 1100 and k == 3 and x in ("h1", "h2", "h4")) else ())
    for lp in [(203, 301, 16, 0, 0), (48, 48, 14, 1, 1), (1100, 1300, 17, 0, 1)]
    for k in [3, 32, 64, 96, 128] for x in ["0", "1", "h1", "h2", "h4", "h8"]])
def test_flush_item_maps_agree(lpg, monkeypatch, xcd, k, m, n, seed, kind, rule):
    """k_flushw's global item queue (LPG_FLUSH_XCD=0) and the XCD-grouped
    queues (FlushX: row bands x H column classes, sub-bands, short tail
    pieces, stealing between groups) at any size and H, to optimality,
    against the oracle. Host-side coverage of the map: tests/test_item_map.py."""
    monkeypatch.setenv("LPG_FLUSH_KERNEL", "w")
    monkeypatch.setenv("LPG_FLUSH_XCD", xcd)
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    key = (m, n, seed, kind, rule)
    if key not in _SOLVED:
        o = Oracle(m, n + m + 1, nthreads=8)
        o.generate(n, seed, kind)
        _SOLVED[key] = (o, o.solve(200_000, rule))
    o, ores = _SOLVED[key]
    e.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


_SOLVED: dict = {}


@pytest.mark.parametrize("k", [5, 32, 40, 64, 96, 128])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(203, 301, 16, 0, 0), (48, 48, 14, 1, 1)])
def test_generic_and_prefetching_pivot_kernels_agree(lpg, monkeypatch, k, m, n, seed, kind, rule):
    """The deferred single-rank pivot runs through k_prep_d / k_select_d; the generic
    k_prep / k_select pair (LPG_SLOW_PIVOT=1, also the multi-rank path) must give the
    same bits."""
    monkeypatch.setenv("LPG_SLOW_PIVOT", "1")
    f = _engine(lpg, monkeypatch, k, m, n + m + 1)
    monkeypatch.delenv("LPG_SLOW_PIVOT")
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1)
    for x in (e, f, o):
        x.generate(n, seed, kind)
    res, fres, ores = e.solve(200_000, rule), f.solve(200_000, rule), o.solve(200_000, rule)
    assert res.pivots == fres.pivots == ores.pivots
    _assert_same(e, o, m)
    _assert_same(f, o, m)


@pytest.mark.parametrize("k", [32, 64, 128])
@pytest.mark.parametrize("m,n,seed,kind,rule", [(203, 301, 16, 0, 0), (48, 48, 14, 1, 1), (600, 1100, 3, 0, 0)])
def test_reordered_columns_to_optimality(lpg, monkeypatch, k, m, n, seed, kind, rule):
    """Whole solves over many blocks: after every block the columns are reordered
    (forced on, these tableaus are below its 2 GB default),
    the entering column's physical index travels in PricePart.pad through
    every reduction, and everything must stay bitwise the oracle's."""
    monkeypatch.setenv("LPG_NO_REORDER", "0")
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    assert e.info.column_trade == 1
    o = Oracle(m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == 1 and res.pivots == ores.pivots
    _assert_same(e, o, m)


@pytest.mark.parametrize("k", [32, 64, 128])
@pytest.mark.parametrize("rule,cap", [(0, 200_000), (1, 3000)])
def test_wide_tableau_more_partials_than_threads(lpg, monkeypatch, k, rule, cap):
    """ncols > 131072: k_prep_d leaves more pricing partials (two columns per
    thread, 256 threads per block) than k_select_d has threads, so select
    reduces them in a loop and reads the entering column's physical index
    through inv (config 4's shape). Bland's rule needs ~41k
    pivots here, so it stops at an iteration limit."""
    m, n = 96, 140_000
    monkeypatch.setenv("LPG_NO_REORDER", "0")      # the physical column through inv (only with the trade)
    e = _engine(lpg, monkeypatch, k, m, n + m + 1)
    o = Oracle(m, n + m + 1, nthreads=8)
    e.generate(n, 7, 0)
    o.generate(n, 7, 0)
    res = e.solve(cap, rule)
    ores = o.solve(cap, rule)
    assert res.status == ores.status and res.pivots == ores.pivots > k
    assert res.status == (1 if rule == 0 else 4)
    assert res.objective == ores.objective
    _assert_same(e, o, m)


@pytest.mark.parametrize("k", [64, 96, 128])
@pytest.mark.parametrize("m,n,seed,kind,rule,big_m", [(512, 700, 5, 0, 0, False), (768, 500, 6, 1, 1, False),
                                                      (767, 600, 9, 2, 0, True)])
def test_pair_select_grid_folds_objective_rows(lpg, monkeypatch, k, m, n, seed, kind, rule, big_m):
    """The single-rank pair (LPG_PERSIST=0) launches k_select_d over the
    constraint rows only; block 0 writes the objective rows' C entries and a
    'none' candidate for each block the grid left out (m = 512, 768: every
    objective row folded; m = 767 with the big-M row: the second one only).
    Blocks of 64 / 96 / 128 also run k_prep_d's two-bank forms (48 + 48 slots
    from 48 pending pivots, 64 + 64 from 96). Bitwise the oracle throughout."""
    monkeypatch.setenv("LPG_PERSIST", "0")
    flags = lpg._lib.FLAG_BIG_M if big_m else 0
    monkeypatch.setenv("LPG_DEFER", str(k))
    e = lpg.Engine(m, n + m + 1, flags=flags)
    monkeypatch.delenv("LPG_DEFER")
    o = Oracle(m, n + m + 1, nobj=2 if big_m else 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    cap = 3000
    if big_m:
        art_first = 1 + n + (m + 1) // 2
        res, ores = e.solve_big_m(art_first, None, cap, rule), o.solve_big_m(art_first, None, cap, rule)
    else:
        res, ores = e.solve(cap, rule), o.solve(cap, rule)
    assert res.status == ores.status and res.pivots == ores.pivots > 48
    assert res.objective == ores.objective
    rows = m + (2 if big_m else 1)
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, rows), o.get_rows())



def test_96_slot_pass_many_items(lpg, monkeypatch):
    """The 96-slot block pass over many items and the short tail items
    (4096 x 12289, 2048-row items halved to fill the chip), bitwise the oracle
    after 3 whole blocks and a partial one."""
    m, n = 4096, 8192
    e = _engine(lpg, monkeypatch, 96, m, n + m + 1)
    o = Oracle(m, n + m + 1, nthreads=8)
    e.generate(n, 20220518, 0)
    o.generate(n, 20220518, 0)
    res = e.solve(3 * 96 + 17, 0)
    ores = o.solve(3 * 96 + 17, 0)
    assert res.status == ores.status and res.pivots == ores.pivots == 3 * 96 + 17
    _assert_same(e, o, m)
