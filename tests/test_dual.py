"""Dual simplex (reference: router option 2, Source/router.c:32-34, prints the
wrong label and does nothing; LPStandardize(model, 1) flips every >= row so the
slack basis is dual feasible, Source/simplex.c:178-179)."""
from __future__ import annotations

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


@pytest.mark.gpu
@pytest.mark.parametrize("m,n", [(5, 7), (100, 150), (400, 300), (2000, 1500)])
def test_gpu_dual_bitwise(lpg, m, n):
    e = lpg.Engine(m, n + m + 1)
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
