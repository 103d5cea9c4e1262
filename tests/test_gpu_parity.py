"""HIP engine (liblpg.so, gfx950) vs the oracles, through the C-ABI.

Bar: bit-exact. The engine's arithmetic contract (P = row/pivot, fma(-C, P, T))
is the oracle's, so pivot logs, bases, objectives and whole tableaus must be
identical (np.array_equal, i.e. +0 == -0), not merely close. The exact
(fractions) fixtures are met to 1e-9 relative on the objective and exactly on
the pivot sequence and basis.
"""
from __future__ import annotations

import os
from fractions import Fraction

import numpy as np
import pytest

from oracle.lpo import Oracle
from util import STATUS, frac, kat_cases, kat_costs, kat_tableau, pivots_of, synthetic_cases

pytestmark = pytest.mark.gpu

RULES = {"dantzig": 0, "bland": 1}


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    assert lpg.device_count() >= 1, "no GPU visible"
    return lpg


def _pair(lpg, m, ncols, **kw):
    return lpg.Engine(m, ncols, **kw), Oracle(m, ncols, nthreads=int(os.environ.get("OMP_NUM_THREADS", "8")))


def _log(x):
    k, r = x.get_log()
    return list(zip(k.tolist(), r.tolist()))


def _assert_same(e, o, m):
    assert _log(e) == _log(o)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


@pytest.mark.parametrize("rule", ["dantzig", "bland"])
@pytest.mark.parametrize("case", kat_cases(), ids=lambda c: c["name"])
def test_kat_cases(lpg, case, rule):
    T = kat_tableau(case)
    m = T.shape[0] - 1
    exp = case[rule]
    budget = len(exp["pivots"]) if exp["status"] == "ITER_LIMIT" else 10_000
    e, o = _pair(lpg, m, T.shape[1])
    for x in (e, o):
        x.load_tableau(T, case["basis"])
    res = e.solve(budget, RULES[rule])
    ores = o.solve(budget, RULES[rule])
    assert _log(e) == pivots_of(exp)
    assert res.status == STATUS[exp["status"]] == ores.status
    assert res.objective == ores.objective
    if exp["status"] != "UNBOUNDED":
        assert abs(res.objective - float(frac(exp["objective"]))) <= 1e-9 * max(1, abs(float(frac(exp["objective"]))))
    _assert_same(e, o, m)


def test_testdata_known_answer(lpg):
    """Source/testdata.txt (max:) -> z* = 12 with basis {x2, x4}."""
    case = next(c for c in kat_cases() if c["name"] == "testdata_max.txt")
    e = lpg.Engine(2, 5)
    e.load_tableau(kat_tableau(case), case["basis"])
    res = e.solve(100)
    assert res.status_name == "OPTIMAL" and res.pivots == 3
    assert abs(res.objective + float(frac(case["constant"])) - 12.0) < 1e-12
    assert e.get_basis().tolist() == [2, 4]
    np.testing.assert_allclose(e.get_column0(), [17 / 3, 6.0], rtol=0, atol=1e-14)


@pytest.mark.parametrize("m,n,seed,kind", [(7, 5, 1, 0), (64, 96, 2, 0), (65, 130, 3, 0), (300, 257, 4, 0),
                                          (129, 129, 5, 1), (1024, 2048, 20220518, 0)])
def test_generator_bitwise(lpg, m, n, seed, kind):
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())
    assert np.array_equal(e.get_basis(), o.get_basis())


@pytest.mark.parametrize("case", synthetic_cases(), ids=lambda c: f"{c['m']}x{c['n']}k{c['kind']}")
def test_synthetic_exact_fixtures(lpg, case):
    m, n = case["m"], case["n"]
    for rule in ("dantzig", "bland"):
        if rule not in case:
            continue
        exp = case[rule]
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, case["seed"], case["kind"])
        res = e.solve(10_000, RULES[rule])
        assert res.status == STATUS[exp["status"]]
        assert _log(e) == pivots_of(exp)
        z = float(Fraction(exp["objective"]))
        assert abs(res.objective - z) <= 1e-9 * max(1.0, abs(z))


@pytest.mark.parametrize("m,n,seed,kind,rule", [
    (64, 96, 11, 0, 0), (200, 300, 12, 0, 0), (333, 517, 13, 0, 0), (48, 48, 14, 1, 1), (257, 100, 15, 1, 0),
    (1024, 2048, 20220518, 0, 0),   # BASELINE config 2, to optimality
])
def test_to_optimality_bitwise(lpg, m, n, seed, kind, rule):
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, seed, kind)
    o.generate(n, seed, kind)
    res = e.solve(200_000, rule)
    ores = o.solve(200_000, rule)
    assert res.status == ores.status == STATUS["OPTIMAL"]
    assert res.pivots == ores.pivots > 0
    assert res.objective == ores.objective
    _assert_same(e, o, m)


@pytest.mark.parametrize("m,cap", [(512, 3000), (2048, 400)])
def test_bland_degenerate_capped(lpg, m, cap):
    """KM-style degenerate LP (b_i = 0 on even rows) under Bland: the pivot count grows
    exponentially with m (config 5 is pivot-capped); the capped runs agree bitwise."""
    e, o = _pair(lpg, m, 2 * m + 1)
    e.generate(m, 14, 1)
    o.generate(m, 14, 1)
    res = e.solve(cap, 1)
    ores = o.solve(cap, 1)
    assert res.status == ores.status and res.pivots == ores.pivots
    assert res.objective == ores.objective
    _assert_same(e, o, m)


def test_config3_first_pivots(lpg):
    """BASELINE config 3 (16384 x 32768, 6.44 GB tableau): the first pivots agree bitwise;
    at full size the invariant 'basic columns are unit vectors' is checked on sampled rows."""
    m, n, K = 16384, 32768, 6
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, 20220518, 0)
    o.generate(n, 20220518, 0)
    res = e.solve(K, 0)
    o.solve(K, 0)
    assert res.status_name == "ITER_LIMIT" and res.pivots == K
    assert _log(e) == _log(o)
    basis = e.get_basis()
    assert np.array_equal(basis, o.get_basis())
    rows = sorted(set([0, 1, m - 1] + [r for _, r in _log(e)]))
    for i in rows:
        assert np.array_equal(e.get_rows(i, 1), o.get_rows(i, 1)), i
        ri = e.get_rows(i, 1)[0]
        assert ri[basis[i]] == 1.0 and np.count_nonzero(ri[basis]) == 1
    assert np.array_equal(e.get_rows(m, 1), o.get_rows(m, 1))
    del o


def test_enqueue_sync_and_noop_after_optimal(lpg):
    m, n = 40, 60
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, 21, 0)
    o.generate(n, 21, 0)
    ores = o.solve(100_000, 0)
    e.enqueue(ores.pivots + 50, 0)      # more pivots than needed: the extra ones are device no-ops
    res = e.sync()
    assert res.status_name == "OPTIMAL" and res.pivots == ores.pivots
    _assert_same(e, o, m)
    again = e.solve(10, 0)               # already optimal: nothing more happens
    assert again.pivots == ores.pivots


def test_iteration_limit_then_resume(lpg):
    m, n = 50, 80
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, 22, 0)
    o.generate(n, 22, 0)
    first = e.solve(5, 0)
    assert first.status_name == "ITER_LIMIT" and first.pivots == 5
    res = e.solve(100_000, 0)
    ores = o.solve(100_000, 0)
    assert res.status == ores.status and res.pivots == ores.pivots
    _assert_same(e, o, m)


def test_unbounded_and_immediately_optimal(lpg):
    e = lpg.Engine(1, 4)
    e.load_tableau(np.array([[1.0, -1.0, 1.0, 1.0], [0.0, -1.0, 0.0, 0.0]]), [3])
    assert e.solve(10).status_name == "UNBOUNDED"
    e = lpg.Engine(1, 3)
    e.load_tableau(np.array([[1.0, 1.0, 1.0], [0.0, 1.0, 0.0]]), [2])
    res = e.solve(10)
    assert res.status_name == "OPTIMAL" and res.pivots == 0


def test_set_objective_general_basis(lpg):
    """Objective row from costs and a non-slack basis (fma chain in row order) == oracle, bitwise."""
    m, n = 30, 45
    e, o = _pair(lpg, m, n + m + 1)
    o.generate(n, 23, 0)
    o.solve(7, 0)                                  # move to a non-trivial basis
    T = o.get_rows()
    basis = o.get_basis()
    rng = np.random.default_rng(0)
    c = rng.uniform(0.5, 2.0, n + m)
    o.set_objective(c)
    e.load_tableau(T, basis)
    e.set_objective(c)
    assert np.array_equal(e.get_rows(m, 1)[0], o.get_rows()[m])
    res = e.solve(10_000, 0)
    ores = o.solve(10_000, 0)
    assert res.status == ores.status and res.objective == ores.objective


@pytest.mark.parametrize("variant", [0, 1])
def test_update_variants_identical(lpg, variant, monkeypatch):
    monkeypatch.setenv("LPG_DEFER", "0")            # the per-pivot update kernel runs in eager mode
    monkeypatch.setenv("LPG_UPDATE_VARIANT", str(variant))
    m, n = 300, 700
    e, o = _pair(lpg, m, n + m + 1)
    e.generate(n, 24, 0)
    o.generate(n, 24, 0)
    res = e.solve(40, 0)
    o.solve(40, 0)
    assert res.pivots == 40
    _assert_same(e, o, m)


@pytest.mark.parametrize("m,n,kind,rule,piv", [(500, 900, 0, 0, 300), (300, 300, 1, 1, 2000)])
def test_column_skipping_is_value_identical(lpg, m, n, kind, rule, piv, monkeypatch):
    """Skipping slices whose pivot-row entries are zero changes no value (np.array_equal;
    only the sign of a zero may differ) and no decision; the touched-bytes counter is
    exact without skipping and smaller with it (eager per-pivot update)."""
    monkeypatch.setenv("LPG_DEFER", "0")
    e = lpg.Engine(m, n + m + 1)
    monkeypatch.setenv("LPG_NO_SKIP", "1")
    f = lpg.Engine(m, n + m + 1)
    monkeypatch.delenv("LPG_NO_SKIP")
    for x in (e, f):
        x.generate(n, 51, kind)
        x.set_timing(True)
        x.get_timing()
        x.solve(piv, rule)
    te, tf = e.get_timing(), f.get_timing()
    assert _log(e) == _log(f)
    assert np.array_equal(e.get_rows(0, m + 1), f.get_rows(0, m + 1))
    # 16-byte slices: an odd N+1 rounds up to one padding double per row
    assert tf.update_bytes == tf.update_count * 32 * (m + 1) * ((n + m + 2) // 2)
    assert 0 < te.update_bytes < tf.update_bytes


@pytest.mark.parametrize("defer", ["0", "32", "8"])
def test_graph_replay_identical(lpg, defer, monkeypatch):
    """Batches of >= 2 graph lengths replay a captured hipGraph (32 pivots eager, one
    block of K pivots + its flush deferred); the result must be bitwise the eager
    launches (LPG_NO_GRAPH=1) and the oracle."""
    monkeypatch.setenv("LPG_DEFER", defer)
    m, n = 200, 300
    e = lpg.Engine(m, n + m + 1)
    monkeypatch.setenv("LPG_NO_GRAPH", "1")
    f = lpg.Engine(m, n + m + 1)
    monkeypatch.delenv("LPG_NO_GRAPH")
    o = Oracle(m, n + m + 1)
    for x in (e, f, o):
        x.generate(n, 61, 0)
    e.enqueue(1, 0)            # odd start: a graph per parity; deferred: finish the open block first
    e.enqueue(150, 0)
    r = e.sync()
    f.solve(151, 0)
    o.solve(151, 0)
    assert r.pivots == o.get_log()[0].size
    _assert_same(e, o, m)
    _assert_same(f, o, m)


@pytest.mark.parametrize("defer", ["0", "32", "64"])
def test_prepare_then_replay(lpg, defer, monkeypatch):
    """lpg_prepare builds the replayed graph ahead of time (here after an odd
    number of pivots, with a block open); the pivots that follow replay it and
    stay bitwise on the oracle's path, and a prepare under the other rule is a
    rebuild, not an error."""
    monkeypatch.setenv("LPG_DEFER", defer)
    m, n = 200, 300
    e = lpg.Engine(m, n + m + 1)
    o = Oracle(m, n + m + 1)
    e.generate(n, 62, 0)
    o.generate(n, 62, 0)
    e.enqueue(3, 0)
    e.prepare(0)
    e.prepare(0)               # already built: no-op
    e.enqueue(200, 0)
    r = e.sync()
    o.solve(203, 0)
    assert r.pivots == o.get_log()[0].size
    _assert_same(e, o, m)
    e.prepare(1)
    res, ores = e.solve(100_000, 1), o.solve(100_000, 1)
    assert res.status == ores.status and res.pivots == ores.pivots
    _assert_same(e, o, m)


def test_timing_counters(lpg, monkeypatch):
    monkeypatch.setenv("LPG_DEFER", "0")
    e = lpg.Engine(512, 512 + 1024 + 1)
    e.generate(1024, 25, 0)
    e.set_timing(True)
    e.reserve_log(64)
    e.enqueue(32, 0)
    e.sync()
    t = e.get_timing()
    assert t.update_count == 32 and t.update_ms > 0 and t.select_ms > 0


def test_bad_arguments_are_errors(lpg):
    e = lpg.Engine(4, 10)
    with pytest.raises(lpg.LPGError):
        e.generate(100)                       # ncols != n + m + 1
    with pytest.raises(lpg.LPGError):
        e.set_basis([0, 1, 2, 3])             # column 0 is b, not a variable
    with pytest.raises(lpg.LPGError):
        e.solve(10, rule=7)
