"""CPU oracle (oracle/liblpo.so) pinned against the golden fixtures.

* kat_cases.json: tableaus read back from the REFERENCE binary's own aligned
  printout (Source/simplex.c:238-260 -> matrix.c:19-91) and solved exactly;
* synthetic_cases.json: splitmix64 LPs solved exactly (fractions);
* scipy/HiGHS optima as an independent cross-check.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np
import pytest

from oracle.lpo import GEN_DEGENERATE, GEN_DENSE, RULE_BLAND, RULE_DANTZIG, Oracle
from tests.golden.make_golden import synthetic
from util import STATUS, frac, kat_cases, kat_costs, kat_tableau, pivots_of, synthetic_cases

RULES = {"dantzig": RULE_DANTZIG, "bland": RULE_BLAND}


def _solve_case(case, rule, max_pivots=None):
    T = kat_tableau(case)
    m = T.shape[0] - 1
    o = Oracle(m, T.shape[1])
    o.load_tableau(T, case["basis"])
    exp = case[rule]
    budget = max_pivots if max_pivots is not None else (len(exp["pivots"]) if exp["status"] == "ITER_LIMIT" else 10_000)
    res = o.solve(budget, RULES[rule])
    return o, res, exp


@pytest.mark.parametrize("rule", ["dantzig", "bland"])
@pytest.mark.parametrize("case", kat_cases(), ids=lambda c: c["name"])
def test_kat_matches_exact_oracle(case, rule):
    o, res, exp = _solve_case(case, rule)
    k, r = o.get_log()
    assert list(zip(k.tolist(), r.tolist())) == pivots_of(exp)
    assert res.status == STATUS[exp["status"]]
    if exp["status"] in ("OPTIMAL", "ITER_LIMIT"):
        z = float(frac(exp["objective"]))
        assert abs(res.objective - z) <= 1e-9 * max(1.0, abs(z))
        assert o.get_basis().tolist() == exp["basis"]


def test_testdata_known_answer():
    """Source/testdata.txt with max: -> z* = 12 at x = (0, 17/3), x4 = 6."""
    case = next(c for c in kat_cases() if c["name"] == "testdata_max.txt")
    o, res, exp = _solve_case(case, "dantzig")
    assert res.status == STATUS["OPTIMAL"] and res.pivots == 3
    assert list(zip(*[a.tolist() for a in o.get_log()])) == [(1, 1), (2, 0), (4, 1)]
    z = res.objective + float(frac(case["constant"]))
    assert abs(z - 12.0) < 1e-12
    T = o.get_rows()
    assert o.get_basis().tolist() == [2, 4]
    np.testing.assert_allclose(T[0], [17 / 3, 14 / 9, 1, 14 / 9, 0], rtol=0, atol=1e-14)
    np.testing.assert_allclose(T[1], [6, 32 / 9, 0, 14 / 9, 1], rtol=0, atol=1e-14)
    np.testing.assert_allclose(T[2], [17 / 3, 5 / 9, 0, 14 / 9, 0], rtol=0, atol=1e-14)


def test_beale_cycles_under_dantzig_and_bland_terminates():
    case = next(c for c in kat_cases() if c["name"] == "kat_beale_cycling.txt")
    o, res, _ = _solve_case(case, "dantzig", max_pivots=24)
    k, r = o.get_log()
    assert res.status == STATUS["ITER_LIMIT"]
    assert list(zip(k[:6], r[:6])) == list(zip(k[6:12], r[6:12]))      # period-6 cycle
    o, res, exp = _solve_case(case, "bland")
    assert res.status == STATUS["OPTIMAL"] and abs(res.objective - 1.25) < 1e-12


def test_min_problem_sign():
    """min problems are solved as max(-z) (simplex.c:99-106): zcoef = -1 flips the optimum back."""
    case = next(c for c in kat_cases() if c["name"] == "kat_min_ge.txt")
    assert frac(case["zcoef"]) == -1
    _, res, _ = _solve_case(case, "dantzig")
    assert abs(res.objective * float(frac(case["zcoef"])) - (-20.0)) < 1e-12


def test_generator_matches_python_restatement():
    for (m, n, seed, kind) in [(5, 7, 1, GEN_DENSE), (9, 4, 20220518, GEN_DENSE), (6, 6, 3, GEN_DEGENERATE)]:
        o = Oracle(m, n + m + 1)
        o.generate(n, seed, kind)
        T, basis = synthetic(m, n, seed, kind)
        assert np.array_equal(o.get_rows(), np.array(T))
        assert o.get_basis().tolist() == basis


@pytest.mark.parametrize("case", synthetic_cases(), ids=lambda c: f"{c['m']}x{c['n']}k{c['kind']}")
def test_synthetic_matches_exact_oracle(case):
    m, n = case["m"], case["n"]
    T, _ = synthetic(m, n, case["seed"], case["kind"])
    assert [float.hex(r[0]) for r in T[:m]] == case["b_hex"]
    for rule in ("dantzig", "bland"):
        if rule not in case:
            continue
        exp = case[rule]
        o = Oracle(m, n + m + 1)
        o.generate(n, case["seed"], case["kind"])
        res = o.solve(10_000, RULES[rule])
        assert res.status == STATUS[exp["status"]]
        assert list(zip(*[a.tolist() for a in o.get_log()])) == pivots_of(exp)
        z = float(Fraction(exp["objective"]))
        assert abs(res.objective - z) <= 1e-9 * max(1.0, abs(z))
        assert o.get_basis().tolist() == exp["basis"]


@pytest.mark.parametrize("m,n,seed", [(20, 30, 1), (40, 60, 2), (64, 96, 3)])
def test_dense_optimum_matches_highs(m, n, seed):
    scipy_opt = pytest.importorskip("scipy.optimize")
    o = Oracle(m, n + m + 1)
    o.generate(n, seed, GEN_DENSE)
    T0 = o.get_rows()
    res = o.solve(100_000, RULE_DANTZIG)
    assert res.status == STATUS["OPTIMAL"]
    A, b, c = T0[:m, 1:n + 1], T0[:m, 0], -T0[m, 1:n + 1]
    hs = scipy_opt.linprog(-c, A_ub=A, b_ub=b, bounds=(0, None), method="highs")
    assert hs.status == 0
    assert abs(res.objective - (-hs.fun)) <= 1e-9 * abs(hs.fun)


def test_kat_optima_match_highs():
    scipy_opt = pytest.importorskip("scipy.optimize")
    for case in kat_cases():
        T = kat_tableau(case)
        m = T.shape[0] - 1
        o = Oracle(m, T.shape[1])
        o.load_tableau(T, case["basis"])
        res = o.solve(10_000, RULE_BLAND)
        c = kat_costs(case)
        hs = scipy_opt.linprog(-c, A_eq=T[:m, 1:], b_eq=T[:m, 0], bounds=(0, None), method="highs")
        if hs.status == 3:
            assert res.status == STATUS["UNBOUNDED"], case["name"]
        else:
            assert res.status == STATUS["OPTIMAL"], case["name"]
            assert abs(res.objective - (-hs.fun)) <= 1e-9 * max(1, abs(hs.fun)), case["name"]


@pytest.mark.parametrize("rule", [RULE_DANTZIG, RULE_BLAND])
def test_partition_invariance(rule):
    """Row-block partition (loopback allgather of ratio candidates) never changes a decision."""
    logs = []
    for parts in (1, 2, 3, 4, 8):
        o = Oracle(48, 48 + 80 + 1)
        o.generate(80, 99, GEN_DENSE if rule == RULE_DANTZIG else GEN_DEGENERATE)
        o.solve(5000, rule, parts)
        logs.append((o.get_log()[0].tolist(), o.get_log()[1].tolist(), o.get_rows().tobytes()))
    assert all(l == logs[0] for l in logs[1:])


def test_set_objective_matches_slack_form():
    o = Oracle(16, 16 + 24 + 1)
    o.generate(24, 5, GEN_DENSE)
    T = o.get_rows()
    c = np.concatenate([-T[16, 1:25], np.zeros(16)])
    o.set_objective(c)
    assert np.array_equal(o.get_rows()[16], T[16])


def test_unbounded_and_immediately_optimal():
    # max x1 s.t. -x1 + x2 <= 1: unbounded in x1
    o = Oracle(1, 4)
    o.load_tableau(np.array([[1.0, -1.0, 1.0, 1.0], [0.0, -1.0, 0.0, 0.0]]), [3])
    assert o.solve(10).status == STATUS["UNBOUNDED"]
    # max -x1: optimal at the slack basis, zero pivots
    o = Oracle(1, 3)
    o.load_tableau(np.array([[1.0, 1.0, 1.0], [0.0, 1.0, 0.0]]), [2])
    res = o.solve(10)
    assert res.status == STATUS["OPTIMAL"] and res.pivots == 0
