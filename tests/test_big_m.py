"""Big-M method with a symbolic M (two objective rows, lexicographic pricing).

The reference's Number carries a symbolic constant M (Source/numOprts.h:15-37,
constant declared at dataReader.c:165-173) and its menu offers "1. Big M
Method." (simplex.c:47-48) with an empty handler (simplex.c:58-60). The
engine keeps the M part as its own objective row (LPG_FLAG_BIG_M): d_j =
dM_j M + dR_j is compared lexicographically, never as a floating product.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lpo import GEN_ARTIFICIAL, RULE_BLAND, RULE_DANTZIG, Oracle
from util import STATUS

# A5: max x1 + 2 x2; x1 + x2 = 3; x1 - x2 <= 1
A5 = np.array([[3.0, 1, 1, 0, 1], [1.0, 1, -1, 1, 0], [0, 0, 0, 0, 0], [0, 0, 0, 0, 0]])
INF = np.array([[2.0, 1, 1, 0, 1], [1.0, 1, 1, 1, 0], [0, 0, 0, 0, 0], [0, 0, 0, 0, 0]])
# max x1; x2 = 1, x2 = 2 (artificials a1, a2): infeasible, and x1's column (0, 0)
# is a ray of the real objective once the M part is optimal (a2 = 1 left)
INF_RAY = np.array([[1.0, 0, 1, 1, 0], [2.0, 0, 1, 0, 1], [0, 0, 0, 0, 0], [0, 0, 0, 0, 0]])


def _oracle(T, basis):
    o = Oracle(T.shape[0] - 2, T.shape[1], nobj=2)
    o.load_tableau(T, basis)
    return o


@pytest.mark.parametrize("rule", [RULE_DANTZIG, RULE_BLAND])
def test_a5_big_m(rule):
    o = _oracle(A5, [4, 3])
    r = o.solve_big_m(4, [1.0, 2.0, 0.0, 0.0], 100, rule)
    assert r.status == STATUS["OPTIMAL"] and abs(r.objective - 6.0) < 1e-12
    T = o.get_rows()
    assert T[2, 0] == 0.0                         # M part of z is zero: no artificial left positive


def test_big_m_infeasible():
    o = _oracle(INF, [4, 3])
    assert o.solve_big_m(4, [1.0, 1.0, 0.0, 0.0], 100).status == STATUS["INFEASIBLE"]


def test_big_m_infeasible_with_a_ray():
    """A ray found while an artificial is still positive is INFEASIBLE, not UNBOUNDED."""
    o = _oracle(INF_RAY, [3, 4])
    assert o.solve_big_m(3, [1.0, 0.0, 0.0, 0.0], 100).status == STATUS["INFEASIBLE"]


@pytest.mark.parametrize("m,n,rule", [(8, 8, RULE_BLAND), (33, 33, RULE_DANTZIG), (64, 64, RULE_BLAND)])
def test_big_m_agrees_with_two_phase(m, n, rule):
    art_first = 1 + n + (m + 1) // 2
    bm = Oracle(m, n + m + 1, nobj=2)
    bm.generate(n, 9, GEN_ARTIFICIAL)
    rb = bm.solve_big_m(art_first, None, 100_000, rule)
    tp = Oracle(m, n + m + 1)
    tp.generate(n, 9, GEN_ARTIFICIAL)
    rt = tp.solve_two_phase(art_first, None, 100_000, rule)
    assert rb.status == rt.status == STATUS["OPTIMAL"]
    assert abs(rb.objective - rt.objective) <= 1e-9 * max(1.0, abs(rt.objective))


# ---------------------------------------------------------------- GPU ----

@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    return lpg


def _same(e, o, rows):
    ek, er = e.get_log()
    ok, orr = o.get_log()
    assert np.array_equal(ek, ok) and np.array_equal(er, orr)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, rows), o.get_rows())


@pytest.mark.gpu
@pytest.mark.parametrize("rule", [RULE_DANTZIG, RULE_BLAND])
def test_gpu_big_m_small(lpg, rule):
    e = lpg.Engine(2, 5, flags=lpg._lib.FLAG_BIG_M)
    e.load_tableau(A5, [4, 3])
    r = e.solve_big_m(4, [1.0, 2.0, 0.0, 0.0], 100, rule)
    o = _oracle(A5, [4, 3])
    ro = o.solve_big_m(4, [1.0, 2.0, 0.0, 0.0], 100, rule)
    assert r.status == ro.status == STATUS["OPTIMAL"] and r.objective == ro.objective == 6.0
    _same(e, o, 4)
    e = lpg.Engine(2, 5, flags=lpg._lib.FLAG_BIG_M)
    e.load_tableau(INF, [4, 3])
    assert e.solve_big_m(4, [1.0, 1.0, 0.0, 0.0], 100).status_name == "INFEASIBLE"


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,rule", [(64, 64, RULE_BLAND), (257, 300, RULE_DANTZIG), (1024, 1024, RULE_BLAND)])
def test_gpu_big_m_bitwise(lpg, m, n, rule):
    art_first = 1 + n + (m + 1) // 2
    e = lpg.Engine(m, n + m + 1, flags=lpg._lib.FLAG_BIG_M)
    e.generate(n, 9, GEN_ARTIFICIAL)
    o = Oracle(m, n + m + 1, nobj=2)
    o.generate(n, 9, GEN_ARTIFICIAL)
    assert np.array_equal(e.get_rows(0, m + 2), o.get_rows())
    r = e.solve_big_m(art_first, None, 100_000, rule)
    ro = o.solve_big_m(art_first, None, 100_000, rule)
    assert r.status == ro.status and r.pivots == ro.pivots and r.objective == ro.objective
    _same(e, o, m + 2)


@pytest.mark.gpu
def test_big_m_infeasible_with_a_ray_on_device(lpg):
    e = lpg.Engine(2, 5, flags=lpg._lib.FLAG_BIG_M)
    e.load_tableau(INF_RAY, [3, 4])
    assert e.solve_big_m(3, [1.0, 0.0, 0.0, 0.0], 100).status == STATUS["INFEASIBLE"]
    e.close()
