"""Two-phase method (artificial variables).

The reference offers "1. Big M Method. / 2. Two-phase Method." when
CreateSMatrix finds rows without an identity column (Source/simplex.c:41-55)
and then does nothing in either case (simplex.c:57-63). Here: the oracle's
two-phase restatement is checked against HiGHS and hand answers on CPU, and
the engine against the oracle bitwise on the GPU.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle.lpo import GEN_ARTIFICIAL, RULE_BLAND, RULE_DANTZIG, Oracle
from tests.golden.make_golden import synthetic
from util import STATUS, degenerate_two_phase_lp

# A5 of SURVEY.md Appendix A (lack row 0): max x1 + 2 x2; x1 + x2 = 3; x1 - x2 <= 1.
# Columns [b | x1 x2 x3(slack) | a1(artificial for row 0)]
A5 = np.array([[3.0, 1, 1, 0, 1], [1.0, 1, -1, 1, 0], [0, 0, 0, 0, 0]])
A5_BASIS, A5_COST, A5_ART = [4, 3], [1.0, 2.0, 0.0, 0.0], 4
# infeasible: x1 + x2 = 2 (artificial) and x1 + x2 <= 1
INF = np.array([[2.0, 1, 1, 0, 1], [1.0, 1, 1, 1, 0], [0, 0, 0, 0, 0]])


def _oracle(T, basis):
    o = Oracle(T.shape[0] - 1, T.shape[1])
    o.load_tableau(T, basis)
    return o


@pytest.mark.parametrize("rule", [RULE_DANTZIG, RULE_BLAND])
def test_a5_two_phase_known_answer(rule):
    o = _oracle(A5, A5_BASIS)
    r = o.solve_two_phase(A5_ART, A5_COST, 100, rule)
    assert r.status == STATUS["OPTIMAL"] and abs(r.objective - 6.0) < 1e-12
    assert 4 not in o.get_basis().tolist()           # the artificial left the basis


def test_infeasible_detected():
    o = _oracle(INF, [4, 3])
    assert o.solve_two_phase(4, [1.0, 1.0, 0.0, 0.0], 100).status == STATUS["INFEASIBLE"]


@pytest.mark.parametrize("m,n,rule", [(8, 8, RULE_BLAND), (33, 33, RULE_DANTZIG), (64, 64, RULE_BLAND), (120, 150, RULE_DANTZIG)])
def test_config5_family_matches_highs(m, n, rule):
    so = pytest.importorskip("scipy.optimize")
    o = Oracle(m, n + m + 1)
    o.generate(n, 9, GEN_ARTIFICIAL)
    T, basis = synthetic(m, n, 9, 2)
    assert np.array_equal(o.get_rows(), np.array(T)) and o.get_basis().tolist() == basis
    art_first = 1 + n + (m + 1) // 2
    r = o.solve_two_phase(art_first, None, 100_000, rule)
    Ta = np.array(T)
    hs = so.linprog(Ta[m, 1:art_first], A_eq=Ta[:m, 1:art_first], b_eq=Ta[:m, 0], bounds=(0, None), method="highs")
    if hs.status == 3:
        assert r.status == STATUS["UNBOUNDED"]
    else:
        assert r.status == STATUS["OPTIMAL"]
        assert abs(r.objective - (-hs.fun)) <= 1e-9 * abs(hs.fun)
        assert all(b < art_first for b in o.get_basis())



@pytest.mark.parametrize("m,n,seed,rule", [(64, 80, 1, RULE_DANTZIG), (257, 300, 2, RULE_DANTZIG), (300, 200, 3, RULE_BLAND)])
def test_degenerate_lp_needs_the_drive_out(m, n, seed, rule):
    """The fixture of the multi-rank drive-out tests does what it says: phase I
    stops OPTIMAL with E2's artificial basic at zero and a usable (negative)
    original entry in its row; the two-phase solve then ends OPTIMAL with no
    artificial basic, and its optimum equals HiGHS on the same LP."""
    T, basis, art = degenerate_two_phase_lp(m, n, seed)
    N = n + m
    o = _oracle(T, basis)
    c1 = np.zeros(N)
    c1[art - 1:] = -1.0
    o.set_active_columns(N)
    o.set_objective(c1)
    r1 = o.solve(5000, rule)
    b = o.get_basis()
    assert r1.status == STATUS["OPTIMAL"] and r1.objective == 0.0
    assert [i for i in range(m) if b[i] >= art] == [m - 1]
    assert o.get_rows(m - 1, 1)[0, 3] == -1.0
    o = _oracle(T, basis)
    r = o.solve_two_phase(art, None, 5000, rule)
    assert r.status == STATUS["OPTIMAL"] and all(x < art for x in o.get_basis())
    from scipy.optimize import linprog
    A, bb = T[:m, 1:art], T[:m, 0]
    eq = np.zeros(m, dtype=bool)
    eq[[1, m - 1]] = True
    hs = linprog(-(-T[m, 1:art]), A_ub=A[~eq], b_ub=bb[~eq], A_eq=A[eq], b_eq=bb[eq], bounds=(0, None), method="highs")
    assert hs.status == 0 and abs(r.objective - (-hs.fun)) <= 1e-9 * abs(hs.fun)

# ---------------------------------------------------------------- GPU ----

@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    return lpg


def _same(e, o, m):
    ek, er = e.get_log()
    ok, orr = o.get_log()
    assert np.array_equal(ek, ok) and np.array_equal(er, orr)
    assert np.array_equal(e.get_basis(), o.get_basis())
    assert np.array_equal(e.get_rows(0, m + 1), o.get_rows())


@pytest.mark.gpu
@pytest.mark.parametrize("rule", [RULE_DANTZIG, RULE_BLAND])
def test_gpu_a5_and_infeasible(lpg, rule):
    e = lpg.Engine(2, 5)
    e.load_tableau(A5, A5_BASIS)
    r = e.solve_two_phase(A5_ART, A5_COST, 100, rule)
    o = _oracle(A5, A5_BASIS)
    ro = o.solve_two_phase(A5_ART, A5_COST, 100, rule)
    assert r.status == ro.status == STATUS["OPTIMAL"] and r.objective == ro.objective == 6.0
    _same(e, o, 2)
    e = lpg.Engine(2, 5)
    e.load_tableau(INF, [4, 3])
    assert e.solve_two_phase(4, [1.0, 1.0, 0.0, 0.0], 100).status_name == "INFEASIBLE"


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,rule", [(64, 64, RULE_BLAND), (257, 300, RULE_DANTZIG), (1024, 1024, RULE_BLAND)])
def test_gpu_config5_family_bitwise(lpg, m, n, rule):
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, 9, GEN_ARTIFICIAL)
    o = Oracle(m, n + m + 1)
    o.generate(n, 9, GEN_ARTIFICIAL)
    art_first = 1 + n + (m + 1) // 2
    r = e.solve_two_phase(art_first, None, 100_000, rule)
    ro = o.solve_two_phase(art_first, None, 100_000, rule)
    assert r.status == ro.status and r.pivots == ro.pivots and r.objective == ro.objective
    _same(e, o, m)


@pytest.mark.gpu
def test_gpu_forced_pivot_matches_oracle(lpg):
    m, n = 40, 60
    e = lpg.Engine(m, n + m + 1)
    e.generate(n, 3, 0)
    o = Oracle(m, n + m + 1)
    o.generate(n, 3, 0)
    for (k, r) in [(5, 7), (17, 0), (n + 3, 11)]:     # arbitrary pivots, one on a slack column
        T = o.get_rows()
        if abs(T[r, k]) > 1e-9:
            e.pivot(k, r)
            o.pivot(k, r)
    _same(e, o, m)
    with pytest.raises(lpg.LPGError):
        e.pivot(1 + n + 30, 2)            # slack of row 30: zero in row 2 -> refused, nothing applied
    _same(e, o, m)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,seed,rule", [(64, 80, 1, RULE_DANTZIG), (300, 200, 3, RULE_BLAND)])
def test_gpu_two_phase_drive_out_bitwise(lpg, m, n, seed, rule):
    """An artificial left basic at zero after phase I, driven out by a forced
    (negative) pivot, on one rank: bitwise the oracle."""
    T, basis, art = degenerate_two_phase_lp(m, n, seed)
    e = lpg.Engine(m, n + m + 1)
    e.load_tableau(T, basis)
    r = e.solve_two_phase(art, None, 5000, rule)
    o = _oracle(T, basis)
    ro = o.solve_two_phase(art, None, 5000, rule)
    assert r.status == ro.status == STATUS["OPTIMAL"] and r.pivots == ro.pivots and r.objective == ro.objective
    _same(e, o, m)
