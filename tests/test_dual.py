"""Dual simplex (reference: router option 2, Source/router.c:32-34, prints the
wrong label and does nothing; LPStandardize(model, 1) flips every >= row so the
slack basis is dual feasible, Source/simplex.c:178-179)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle.lpo import GEN_DUAL, Oracle
from tests.golden.make_golden import synthetic
from util import STATUS


@pytest.mark.parametrize("m,n", [(5, 7), (30, 20), (100, 150)])
def test_dual_matches_highs(m, n):
    so = pytest.importorskip("scipy.optimize")
    o = Oracle(m, n + m + 1)
    o.generate(n, 3, GEN_DUAL)
    T = np.array(synthetic(m, n, 3, 3)[0])
    assert np.array_equal(o.get_rows(), T)
    r = o.solve_dual(100_000)
    hs = so.linprog(T[m, 1:n + 1], A_ub=T[:m, 1:n + 1], b_ub=T[:m, 0], bounds=(0, None), method="highs")
    assert r.status == STATUS["OPTIMAL"] and hs.status == 0
    assert abs(-r.objective - hs.fun) <= 1e-9 * abs(hs.fun)
    assert (o.get_rows()[:m, 0] >= -1e-9).all()              # primal feasible at the end


def test_dual_infeasible_and_not_dual_feasible():
    # x1 + x2 >= 2 and x1 + x2 <= 1 (as -x1 - x2 <= -2): primal infeasible
    T = np.array([[-2.0, -1, -1, 1, 0], [1.0, 1, 1, 0, 1], [0, 1, 1, 0, 0]])
    o = Oracle(2, 5)
    o.load_tableau(T, [3, 4])
    assert o.solve_dual(100).status == STATUS["INFEASIBLE"]
    bad = T.copy()
    bad[2, 1] = -1.0                                          # d_1 < 0: not dual feasible
    o = Oracle(2, 5)
    o.load_tableau(bad, [3, 4])
    with pytest.raises(RuntimeError):
        o.solve_dual(100)


@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    return lpg


def _flags(lpg, path):
    from linearprogramming_amd import _lib
    return _lib.FLAG_EAGER if path == "eager" else 0


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["eager", "deferred"])
@pytest.mark.parametrize("m,n", [(5, 7), (100, 150), (400, 300), (2000, 1500)])
def test_gpu_dual_bitwise(lpg, m, n, path):
    """Both device forms of the dual: rank-1 updates every pivot (eager) and
    the deferred blocks (lpg_dual.hip: two kernels per pivot, the block pass
    every defer_k pivots)."""
    e = lpg.Engine(m, n + m + 1, flags=_flags(lpg, path))
    assert (e.info.defer_k == 0) == (path == "eager")
    e.generate(n, 3, lpg.GEN_DUAL)
    o = Oracle(m, n + m + 1)
    o.generate(n, 3, GEN_DUAL)
    r = e.solve_dual(100_000)
    ro = o.solve_dual(100_000)
    assert r.status == ro.status == STATUS["OPTIMAL"] and r.pivots == ro.pivots and r.objective == ro.objective
    ek, er = e.get_log()
    ok, orr = o.get_log()
    assert np.array_equal(ek, ok) and np.array_equal(er, orr)
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())
    assert np.array_equal(e.get_basis(), o.get_basis())


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["eager", "deferred"])
def test_gpu_dual_budget_and_resume(lpg, path):
    """ITER_LIMIT when the budget runs out first, OPTIMAL when the last pivot of
    the budget reaches optimality (the final peek, as the oracle), and a second
    call that resumes where the first stopped (mid-block on the deferred path:
    the objective row's owed update and the pending pivots are settled first)."""
    m, n = 400, 300
    o = Oracle(m, n + m + 1)
    o.generate(n, 3, GEN_DUAL)
    total = o.solve_dual(100_000).pivots
    assert total > 40
    for cut in (total - 1, total, 37):
        e = lpg.Engine(m, n + m + 1, flags=_flags(lpg, path))
        e.generate(n, 3, lpg.GEN_DUAL)
        oc = Oracle(m, n + m + 1)
        oc.generate(n, 3, GEN_DUAL)
        r, rc = e.solve_dual(cut), oc.solve_dual(cut)
        assert r.status == rc.status == STATUS["OPTIMAL" if cut == total else "ITER_LIMIT"]
        assert r.pivots == rc.pivots == cut and r.objective == rc.objective
        assert np.array_equal(e.get_rows(0, m + 1), oc.get_rows())
        r2, rc2 = e.solve_dual(100_000), oc.solve_dual(100_000)
        assert r2.status == rc2.status == STATUS["OPTIMAL"] and r2.pivots == rc2.pivots == total
        assert r2.objective == rc2.objective
        assert np.array_equal(e.get_rows(0, m + 1), oc.get_rows())


@pytest.mark.gpu
def test_gpu_dual_deferred_full_size(lpg):
    """LPG_GEN_DUAL at 16384 x 16384 (4.3 GB, the default blocks: 96 pivots
    since round 5): three whole blocks and a partial one of 8 settled by the
    readout, bitwise against the C oracle (log, basis, objective row, column 0,
    every pivot row and 64 sampled rows)."""
    m = n = 16384
    e = lpg.Engine(m, n + m + 1)
    assert e.info.defer_k in (64, 96)
    piv = 3 * e.info.defer_k + 8
    e.generate(n, 7, lpg.GEN_DUAL)
    e.reserve_log(piv + 8)
    r = e.solve_dual(piv)
    o = Oracle(m, n + m + 1, nthreads=min(16, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    o.generate(n, 7, GEN_DUAL)
    ro = o.solve_dual(piv)
    assert r.status == ro.status == STATUS["ITER_LIMIT"] and r.pivots == ro.pivots == piv
    assert r.objective == ro.objective
    ek, er = e.get_log()
    ok, orr = o.get_log()
    assert np.array_equal(ek, ok) and np.array_equal(er, orr)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(m, 1), o.get_rows(m, 1))
    assert np.array_equal(e.get_column0(), np.concatenate([o.get_rows(i0, 1024)[:, 0] for i0 in range(0, m, 1024)]))
    rng = np.random.default_rng(1)
    for i in sorted(set(int(x) for x in orr) | set(rng.choice(m, 64, replace=False).tolist())):
        assert np.array_equal(e.get_rows(i, 1), o.get_rows(i, 1)), f"row {i}"
    e.close()


@pytest.mark.gpu
def test_gpu_dual_optimal_with_late_workgroups(lpg):
    """A dual LP whose rows span ~4900 column blocks of k_dual_row_d, far more
    workgroups than the chip holds at once, so most start after workgroup 0
    has finished. The round-3 kernel let workgroup 0 publish OPTIMAL into the
    status word every workgroup reads on entry, and a late one then skipped
    the objective row's owed update. This LP (230
    pivots) reaches optimality mid-block with that update owed: status,
    pivots, log, basis, the whole objective row and column 0 bitwise the
    oracle's."""
    m, n, seed = 32, 2_500_000, 11
    e = lpg.Engine(m, n + m + 1)
    assert e.info.defer_k == 64
    e.generate(n, seed, lpg.GEN_DUAL)
    r = e.solve_dual(100_000)
    o = Oracle(m, n + m + 1, nthreads=min(16, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    o.generate(n, seed, GEN_DUAL)
    ro = o.solve_dual(100_000)
    assert r.status == ro.status == STATUS["OPTIMAL"] and r.pivots == ro.pivots and r.objective == ro.objective
    assert 0 < ro.pivots % 64, "optimality must come mid-block (an owed update pending)"
    ek, er = e.get_log()
    ok, orr = o.get_log()
    assert np.array_equal(ek, ok) and np.array_equal(er, orr)
    assert np.array_equal(e.get_basis(), o.get_basis())
    eo, oo = e.get_rows(m, 1)[0], o.get_rows(m, 1)[0]
    bad = np.flatnonzero(eo.view(np.uint64) != oo.view(np.uint64))
    assert bad.size == 0, f"objective row differs in {bad.size} columns, first {bad[:8].tolist()}"
    assert np.array_equal(e.get_column0(), o.get_rows(0, m)[:, 0])
    e.close()


@pytest.mark.gpu
def test_gpu_dual_infeasible_and_errors(lpg):
    T = np.array([[-2.0, -1, -1, 1, 0], [1.0, 1, 1, 0, 1], [0, 1, 1, 0, 0]])
    e = lpg.Engine(2, 5)
    e.load_tableau(T, [3, 4])
    assert e.solve_dual(100).status_name == "INFEASIBLE"
    bad = T.copy()
    bad[2, 1] = -1.0
    e = lpg.Engine(2, 5)
    e.load_tableau(bad, [3, 4])
    with pytest.raises(lpg.LPGError):
        e.solve_dual(100)
