"""The host front end (linearprogramming_amd/frontend.py): LP text -> the
reference's SimplexMatrix, checked against the reference itself.

* the 12 fixture LPs: equal to tests/golden/kat_cases.json, the tableaus read
  back from the reference binary's transcripts (tests/golden/make_golden.py);
* 200 random LPs in the reference's format (free and x <= 0 variables, min and
  max, objective constants, decimals, fractions, negative right-hand sides,
  terms on either side, =, >=, <= rows): equal to what the reference binary
  (oracle/_ref/lp, compiled from /root/reference by oracle/Makefile) prints
  after LPAlign -- or rejected by both. Skipped where that binary is absent
  (the GPU box builds nothing; the CPU suite runs here);
* on the GPU: the device solve of the fixture LPs (known optima, Appendix A)
  and of random LPs against HiGHS on the same SimplexMatrix.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
from fractions import Fraction

import numpy as np
import pytest

from conftest import ROOT
import refparse

from linearprogramming_amd import frontend as F

LP = os.path.join(ROOT, "tests", "golden", "lp")
REF = os.path.join(ROOT, "oracle", "_ref", "lp")
needs_ref = pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref/lp not built (needs /root/reference)")


def _fx(s):
    return Fraction(s)


def _as_case(sm: F.SMatrix):
    return {"names": sm.display_names, "basis": sm.basis, "lacking": sm.lacking, "costs": sm.costs,
            "constant": sm.constant, "zcoef": sm.zcoef, "rows": sm.rows}


def _same(sm: F.SMatrix, names, basis, lacking, costs, constant, zcoef, rows):
    got = _as_case(sm)
    exp = {"names": names, "basis": basis, "lacking": lacking, "costs": costs, "constant": constant,
           "zcoef": zcoef, "rows": rows}
    return got == exp, got, exp


@pytest.mark.parametrize("case", json.load(open(os.path.join(ROOT, "tests", "golden", "kat_cases.json"))),
                         ids=lambda c: c["name"])
def test_fixture_lps_build_the_reference_smatrix(case):
    sm = F.build_smatrix(open(os.path.join(LP, case["name"])).read())
    ok, got, exp = _same(sm, case["names"], case["basis"], case["lacking"], [_fx(c) for c in case["costs"]],
                         _fx(case["constant"]), _fx(case["zcoef"]), [[_fx(x) for x in r] for r in case["rows"]])
    assert ok, (got, exp)


def test_shipped_testdata_is_rejected_like_the_reference():
    """The reference's own testdata.txt writes `ma:` (dataReader.c:455): not a model."""
    with pytest.raises(F.FrontendError, match="Objective function invalid"):
        F.build_smatrix(open(os.path.join(LP, "testdata_shipped.txt")).read())


def test_decimal_truncation_and_gcd_quirks():
    """Fractionize's (long)(d * 10^k) truncation (basicFuncs.c:264) and
    FormulaSimplify's separate numerator / denominator GCDs (dataReader.c:409-428)."""
    assert F.fractionize("0.29").value() == Fraction(28, 100)  # 0.29 * 100 = 28.999...
    assert F.fractionize("-2.45").value() == Fraction(-49, 20)
    assert not F.fractionize("0/5").valid and not F.fractionize(".5").valid
    f = F._formula("2x1+4x2<=6")
    assert [t.coef.value() for t in f.left] == [1, 2] and f.right[0].coef.value() == 3
    f = F._formula("1/2x1+1/4x2<=1/2")
    assert [t.coef.value() for t in f.left] == [1, Fraction(1, 2)] and f.right[0].coef.value() == 1


def test_sign_constraint_before_use_makes_the_variable_free():
    """PutVarItem replaces (hashTable.c): a later constraint re-registers x1 as
    unrestricted, so `x1>=0` written first is lost: x1 = x3 - x4 (the reference
    binary prints the same columns x2 x3 x4 x5)."""
    sm = F.build_smatrix("OF {\n max:z=x1+x2\n}\nST {\n x1>=0;\n x1+x2<=4;\n x2>=0\n}\n")
    assert sm.names == ["x2", "x3", "x4", "x5"]
    it = sm.vars.items["x1"]
    assert it.relation == 0 and (it.former, it.latter) == ("x3", "x4")


def _rand_coef(rng, v):
    return rng.choice([str(v), f"{v}/{rng.integers(2, 9)}", f"{v}.{rng.integers(1, 99)}"])


def _random_lp_rich(rng):
    """A random model in the reference's format, exercising its standardisation."""
    n = int(rng.integers(1, 6))
    m = int(rng.integers(1, 5))
    signs = [rng.choice(["ge", "le", "free"], p=[0.6, 0.2, 0.2]) for _ in range(n)]
    if not any(s != "free" for s in signs):
        signs[0] = "ge"

    def expr(allow_const=False):
        terms = []
        for j in range(1, n + 1):
            if rng.random() < 0.75:
                v = int(rng.integers(1, 9))
                terms.append(("-" if rng.random() < 0.25 else "+") + _rand_coef(rng, v) + f"x{j}")
        if not terms:
            terms = [f"+x{int(rng.integers(1, n + 1))}"]
        if allow_const and rng.random() < 0.3:
            terms.append("+" + _rand_coef(rng, int(rng.integers(1, 9))))
        e = "".join(terms)
        return e[1:] if e[0] == "+" else e

    rows = []
    for _ in range(m):
        rel = rng.choice(["<=", ">=", "="], p=[0.6, 0.25, 0.15])
        rhs = int(rng.integers(-5, 40))
        if rng.random() < 0.15:                       # a variable moved to the right-hand side
            rows.append(f"{expr()}{rel}{rhs}+x{int(rng.integers(1, n + 1))}")
        else:
            rows.append(f"{expr()}{rel}{rhs}")
    used = set(int(v) for r in rows for v in re.findall(r"x(\d+)", r))
    for j in range(1, n + 1):                          # every variable appears in a constraint
        if j not in used:
            rows.append(f"x{j}<=30")
    for j, s in enumerate(signs, 1):
        if s == "ge":
            rows.append(f"x{j}>=0")
        elif s == "le":
            rows.append(f"x{j}<=0")
    obj_terms = "+".join(f"{_rand_coef(rng, int(rng.integers(1, 9)))}x{j}" for j in range(1, n + 1))
    if rng.random() < 0.3:
        obj_terms += "+" + _rand_coef(rng, int(rng.integers(1, 9)))
    obj = f"{rng.choice(['max', 'min'])}:z={obj_terms}"
    return "OF {\n\t" + obj + "\n}\nST {\n\t" + ";\n\t".join(rows) + "\n}\n"


def _reference_aligned(path):
    """The reference binary's tableau after LPAlign; None if it rejected the
    model, "crash" if it died first (CreateSMatrix writes its lack list through
    `*lack[lackPtr++]`, matrix.c:86, a wild pointer once two rows lack a unit
    column; on some models with free variables heap corruption in its term
    arrays: `realloc(): invalid next size`)."""
    p = subprocess.run([REF, path], input="\n1\n\n\n1\n\n\nq\n", capture_output=True, text=True, timeout=20,
                       cwd=ROOT, env={"TERM": "dumb", "PATH": "/usr/bin:/bin"})
    models = refparse.parse_models(p.stdout)
    if len(models) < 3:
        return "crash" if p.returncode < 0 else None
    return refparse.tableau_from_aligned(models[2])


@needs_ref
def test_random_lps_match_the_reference_binary(tmp_path):
    rng = np.random.default_rng(20220607)
    compared = rejected = crashed = 0
    for t in range(200):
        text = _random_lp_rich(rng)
        f = tmp_path / f"r{t}.txt"
        f.write_text(text)
        rt = _reference_aligned(str(f))
        if rt == "crash":                 # nothing to compare with
            crashed += 1
            continue
        if rt is None:
            with pytest.raises(F.FrontendError):
                F.build_smatrix(text)
            rejected += 1
            continue
        sm = F.build_smatrix(text)
        ok, got, exp = _same(sm, rt.names, rt.basis, rt.lacking, rt.costs, rt.constant, rt.zcoef, rt.T)
        assert ok, (text, got, exp)
        compared += 1
    assert compared >= 150, (compared, rejected, crashed)


DUAL_LP = "OF {\n\tmin:z=2x1+3x2\n}\nST {\n\tx1+x2>=4;\n\tx1+3x2>=6;\n\tx1>=0;\n\tx2>=0\n}\n"


def test_dual_form():
    """LPStandardize's dual branch (simplex.c:178-179): >= rows negated into <= with a
    +1 slack each, b negative allowed, the slacks a complete basis. (The reference's
    router never reaches it, router.c:32-34: parity unpinned, structure checked.)"""
    sm = F.build_smatrix(DUAL_LP, dual=True)
    assert sm.names == ["x1", "x2", "x3", "x4"] and sm.basis == [3, 4] and sm.lacking == []
    assert sm.rows == [[-4, -1, -1, 1, 0], [-6, -1, -3, 0, 1]]
    assert sm.costs == [-2, -3, 0, 0] and sm.zcoef == -1
    primal = F.build_smatrix(DUAL_LP)
    assert primal.lacking == [0, 1]                     # the primal form needs artificials instead
    with pytest.raises(F.FrontendError, match="dual feasible"):
        F.solve(F.build_smatrix("OF {\n max:z=x1\n}\nST {\n x1<=3;\n x1>=0\n}\n", dual=True), method="dual")


def _random_dual_lp(rng):
    n, m = int(rng.integers(1, 6)), int(rng.integers(1, 6))
    rows = []
    for _ in range(m):
        terms = "+".join(f"{_rand_coef(rng, int(rng.integers(1, 9)))}x{j}" for j in range(1, n + 1))
        rows.append(f"{terms}{rng.choice(['>=', '<='], p=[0.7, 0.3])}{int(rng.integers(1, 30))}")
    rows += [f"x{j}>=0" for j in range(1, n + 1)]
    obj = "+".join(f"{_rand_coef(rng, int(rng.integers(1, 9)))}x{j}" for j in range(1, n + 1))
    return "OF {\n\tmin:z=" + obj + "\n}\nST {\n\t" + ";\n\t".join(rows) + "\n}\n"


# ---- the C restatement (host/lpfront.c, behind host/lpgcli --lp) ----------------

CLI = os.path.join(ROOT, "host", "lpgcli")
SAN_CLI = os.path.join(ROOT, "integration", "_san", "lpgcli")
needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="host/lpgcli not built")


def _c_dump(path, cli=CLI, dual=False):
    p = subprocess.run([cli, "--lp-dump", path] + (["--dual"] if dual else []), capture_output=True, text=True,
                       timeout=30)
    return p.returncode, json.loads(p.stdout)


def _py_dump(text, dual=False):
    sm = F.build_smatrix(text, dual=dual)
    return {"names": sm.display_names, "basis": sm.basis, "costs": [f"{c.numerator}/{c.denominator}" for c in sm.costs],
            "constant": f"{sm.constant.numerator}/{sm.constant.denominator}",
            "zcoef": f"{sm.zcoef.numerator}/{sm.zcoef.denominator}",
            "rows": [[f"{x.numerator}/{x.denominator}" for x in r] for r in sm.rows],
            "vars": [[it.name, it.relation, it.former, it.latter] for it in sm.vars.ordered()]}


@needs_cli
def test_c_front_end_equals_the_python_one(tmp_path):
    """lpfront.c and frontend.py build the same SimplexMatrix and variable table
    (or reject the same models) on every fixture and 200 random models; the
    Python one is pinned to the reference binary above."""
    files = [os.path.join(LP, f) for f in sorted(os.listdir(LP))]
    rng = np.random.default_rng(99)
    for t in range(200):
        f = tmp_path / f"c{t}.txt"
        f.write_text(_random_lp_rich(rng))
        files.append(str(f))
    for f in files:
        text = open(f).read()
        rc, got = _c_dump(f)
        try:
            exp = _py_dump(text)
        except F.FrontendError as ex:
            assert rc == 3 and "error" in got, (f, got, str(ex))
            continue
        assert rc == 0 and got == exp, (text, got, exp)


@needs_cli
def test_c_front_end_dual_form_equals_the_python_one(tmp_path):
    """LPStandardize's dual form (simplex.c:178-179, lpgcli --lp-dump MODEL --dual)
    in both restatements: the fixtures, 100 random dual-feasible models and 100
    general ones."""
    files = [os.path.join(LP, f) for f in sorted(os.listdir(LP))]
    rng = np.random.default_rng(17)
    for t in range(200):
        f = tmp_path / f"d{t}.txt"
        f.write_text(_random_dual_lp(rng) if t < 100 else _random_lp_rich(rng))
        files.append(str(f))
    for f in files:
        text = open(f).read()
        rc, got = _c_dump(f, dual=True)
        try:
            exp = _py_dump(text, dual=True)
        except F.FrontendError as ex:
            assert rc == 3 and "error" in got, (f, got, str(ex))
            continue
        assert rc == 0 and got == exp, (text, got, exp)


@needs_cli
@pytest.mark.parametrize("bad", ['max:z=3x1+5"x2', 'max:z=3x1+5\\x2', 'max:z=3x1+5\x01x2'])
def test_c_front_end_error_is_valid_json(tmp_path, bad):
    """Error text quotes the model's own bytes ("Invalid variable name: ..."):
    quotes, backslashes and control characters are escaped, so the line stays
    one valid JSON object."""
    f = tmp_path / "bad.txt"
    f.write_bytes(("OF {\n\t" + bad + "\n}\nST {\n\tx1<=4;\n\tx1>=0\n}\n").encode())
    rc, got = _c_dump(str(f))
    assert rc == 3 and got["error"].startswith("ERROR:")


OVERFLOW = json.load(open(os.path.join(ROOT, "tests", "golden", "overflow_cases.json")))


def _overflow_expectation(case, sm_or_error):
    """Check one front end's result on one overflow fixture against the
    reference binary's outcome (tests/golden/make_overflow_golden.py):
    accepted -> the same aligned tableau; rejected, or SIGFPE (8: its
    FormulaSimplify / NMul divide by 0 or LONG_MIN by -1) -> rejected here.
    SIGSEGV (11) is the reference's CreateSMatrix writing `*lack[lackPtr++]`
    (matrix.c:86; `*(lack[k])`, a wild stack pointer once k >= 1): it dies on
    models with two or more rows lacking a unit column. The front ends keep the
    intended lack list instead, so for those the check is that it has >= 2 rows."""
    if case["outcome"] == "accepted":
        assert not isinstance(sm_or_error, Exception), (case["name"], sm_or_error)
        return
    if case["outcome"] == "crash" and case["signal"] == 11:
        assert not isinstance(sm_or_error, Exception), (case["name"], sm_or_error)
        return
    assert isinstance(sm_or_error, Exception), (case["name"], case["outcome"])


@pytest.mark.parametrize("case", OVERFLOW, ids=lambda c: c["name"])
def test_long_overflow_matches_the_reference(case):
    """The reference's `long` arithmetic past its limits:
    wrap-around guarded sums and products, LCM overflow, strtol saturation,
    (long) casts of out-of-range doubles, NInv's unchecked LONG_MIN, traps."""
    try:
        sm = F.build_smatrix(case["text"])
    except F.FrontendError as ex:
        sm = ex
    _overflow_expectation(case, sm)
    if case["outcome"] == "crash" and case["signal"] == 11:
        assert len(sm.lacking) >= 2
    if case["outcome"] == "accepted":
        ok, got, exp = _same(sm, case["names"], case["basis"], case["lacking"], [_fx(c) for c in case["costs"]],
                             _fx(case["constant"]), _fx(case["zcoef"]), [[_fx(x) for x in r] for r in case["rows"]])
        assert ok, (case["text"], got, exp)
    elif case["outcome"] == "rejected" and "Invalid coefficient appeared after combining" in case["message"]:
        assert "Invalid coefficient appeared after combining" in str(sm)


@needs_cli
def test_c_front_end_long_overflow_matches_the_reference(tmp_path):
    """lpfront.c on the same overflow fixtures: accepted models dump the
    reference's tableau; rejected and trapping ones exit 3 with an error line."""
    for case in OVERFLOW:
        f = tmp_path / "o.txt"
        f.write_text(case["text"])
        rc, got = _c_dump(str(f))
        _overflow_expectation(case, RuntimeError(got["error"]) if rc == 3 else got)
        assert rc in (0, 3), (case["name"], rc)
        if case["outcome"] == "accepted":
            exp = {k: case[k] for k in ("names", "basis", "costs", "constant", "zcoef", "rows")}
            assert {k: got[k] for k in exp} == exp, (case["text"], got, exp)
        if case["outcome"] == "crash" and case["signal"] == 8:
            assert "arithmetic trap" in got["error"], (case["name"], got)


@pytest.mark.skipif(not os.path.exists(SAN_CLI), reason="integration/_san/lpgcli not built")
def test_c_front_end_under_asan_ubsan(tmp_path):
    """The ASan + UBSan build of lpgcli on the fixtures, the overflow fixtures
    (its `long` emulation wraps in unsigned arithmetic: no UB on overflow) and
    40 random models, incl. rejected ones."""
    files = [os.path.join(LP, f) for f in sorted(os.listdir(LP))]
    for t, case in enumerate(OVERFLOW):
        f = tmp_path / f"o{t}.txt"
        f.write_text(case["text"])
        files.append(str(f))
    rng = np.random.default_rng(7)
    for t in range(40):
        f = tmp_path / f"s{t}.txt"
        f.write_text(_random_lp_rich(rng))
        files.append(str(f))
    for f in files:
        p = subprocess.run([SAN_CLI, "--lp-dump", f], capture_output=True, text=True, timeout=60)
        assert p.returncode in (0, 3) and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
            (f, p.stderr[-2000:])


# ---- device solve ------------------------------------------------------------

@pytest.fixture(scope="module")
def lpg():
    import linearprogramming_amd as lpg
    lpg.load()
    return lpg


KNOWN = [("testdata_max.txt", 12.0), ("kat_wyndor.txt", 36.0), ("kat_min_ge.txt", -20.0),
         ("a6_decimals.txt", 194 / 25), ("kat_negative_rhs.txt", 18.0), ("a5_lack_row.txt", 6.0),
         ("a7_identity_quirk.txt", 2.0), ("a3_min_eq_neg.txt", 31 / 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["two_phase", "big_m"])
@pytest.mark.parametrize("name,z", KNOWN)
def test_device_solve_of_fixture_lps(lpg, name, z, method):
    sol = F.solve_text(open(os.path.join(LP, name)).read(), method=method)
    assert sol.status == "OPTIMAL"
    assert abs(sol.z - z) < 1e-9 * max(1.0, abs(z))


@pytest.mark.gpu
def test_device_solve_readout(lpg):
    """Appendix A2 (x1 = 0, x2 = 17/3, slack x4 = 6); A3 (x3 <= 0 un-substituted)."""
    sol = F.solve_text(open(os.path.join(LP, "testdata_max.txt")).read())
    assert sol.variables["x1"] == 0.0 and abs(sol.variables["x2"] - 17 / 3) < 1e-12
    assert abs(sol.columns["x4"] - 6.0) < 1e-12
    sol = F.solve_text(open(os.path.join(LP, "a3_min_eq_neg.txt")).read())
    assert abs(sol.variables["x1"] - 5 / 3) < 1e-12 and abs(sol.variables["x2"] - 7 / 3) < 1e-12
    assert sol.variables["x3"] == 0.0
    assert F.solve_text(open(os.path.join(LP, "kat_unbounded.txt")).read()).status == "UNBOUNDED"
    assert F.solve_text(open(os.path.join(LP, "a4_free_var.txt")).read()).status == "UNBOUNDED"


@pytest.mark.gpu
def test_device_solve_of_random_lps_matches_highs(lpg, tmp_path):
    from scipy.optimize import linprog
    rng = np.random.default_rng(31)
    solved = 0
    for t in range(60):
        text = _random_lp_rich(rng)
        try:
            sm = F.build_smatrix(text)
        except F.FrontendError:
            continue
        A = np.array([[F._dec(x) for x in r[1:]] for r in sm.rows])
        b = np.array([F._dec(r[0]) for r in sm.rows])
        c = np.array([F._dec(x) for x in sm.costs])
        ref = linprog(-c, A_eq=A, b_eq=b, bounds=[(0, None)] * len(c), method="highs")
        for method in ("two_phase", "big_m"):
            sol = F.solve(sm, method=method)
            if ref.status == 2:
                assert sol.status == "INFEASIBLE", (text, method, sol)
            elif ref.status == 3:
                assert sol.status == "UNBOUNDED", (text, method, sol)
            else:
                assert ref.status == 0 and sol.status == "OPTIMAL", (text, method, sol, ref.status)
                zref = (-ref.fun + F._dec(sm.constant)) / F._dec(sm.zcoef)
                assert abs(sol.z - zref) < 1e-7 * max(1.0, abs(zref)), (text, method, sol.z, zref)
        solved += 1
    assert solved >= 40


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("method", ["", "--big-m"])
def test_c_front_end_device_solve(lpg, method):
    """host/lpgcli --lp: the reference's model files solved on the device from plain C."""
    for name, z in KNOWN:
        args = [CLI, "--lp", os.path.join(LP, name)] + ([method] if method else [])
        p = subprocess.run(args, capture_output=True, text=True, timeout=120)
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert out["status"] == "OPTIMAL" and abs(out["z"] - z) < 1e-9 * max(1.0, abs(z)), (name, out)
    p = subprocess.run([CLI, "--lp", os.path.join(LP, "a3_min_eq_neg.txt")], capture_output=True, text=True, timeout=120)
    v = json.loads(p.stdout.strip().splitlines()[-1])["variables"]
    assert abs(v["x1"] - 5 / 3) < 1e-12 and abs(v["x2"] - 7 / 3) < 1e-12 and v["x3"] == 0.0


@pytest.mark.gpu
def test_dual_simplex_from_the_front_end(lpg):
    """The dual form solved by the device's dual simplex equals the primal
    (two-phase) optimum: the fixture-style model and 30 random dual-feasible ones."""
    sol = F.solve_text(DUAL_LP, method="dual")
    assert sol.status == "OPTIMAL" and sol.method == "dual" and abs(sol.z - 9.0) < 1e-12
    assert abs(sol.variables["x1"] - 3.0) < 1e-12 and abs(sol.variables["x2"] - 1.0) < 1e-12
    rng = np.random.default_rng(5)
    for _ in range(30):
        text = _random_dual_lp(rng)
        d = F.solve_text(text, method="dual")
        p = F.solve_text(text, method="two_phase")
        assert d.status == p.status, (text, d, p)
        if p.status == "OPTIMAL":
            assert abs(d.z - p.z) < 1e-9 * max(1.0, abs(p.z)), (text, d.z, p.z)
