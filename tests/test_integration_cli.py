"""Drop-in check: the reference's own CLI, unmodified, linked with the lpg
bridge (integration/lpg_bridge.c, --wrap=CreateSMatrix). Built in the build
container from /root/reference/Source (integration/Makefile); the binary
travels to the GPU box with the snapshot. Skipped where it was not built.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT
from util import transcripts

BIN = os.path.join(ROOT, "integration", "_ref", "lp_lpg")
MSPLIT = os.path.join(ROOT, "integration", "_ref", "msplit_check")
LP = os.path.join(ROOT, "tests", "golden", "lp")

needs_bin = pytest.mark.skipif(not os.path.exists(BIN), reason="integration/_ref/lp_lpg not built")
needs_msplit = pytest.mark.skipif(not os.path.exists(MSPLIT), reason="integration/_ref/msplit_check not built")


def _run(name, stdin):
    p = subprocess.run([BIN, os.path.join("tests", "golden", "lp", name)], input=stdin, capture_output=True,
                       text=True, timeout=120, cwd=ROOT, env={**os.environ, "TERM": "dumb"})
    return p


def _strip_timing(text):
    return "\n".join(ln for ln in text.split("\n") if not ln.startswith("> LPModel Successfully Parsed in"))


@needs_bin
@pytest.mark.parametrize("name", ["testdata_max.txt", "kat_wyndor.txt", "a6_decimals.txt", "a3_min_eq_neg.txt"])
def test_front_end_unchanged_by_the_bridge(name):
    """Up to CreateSMatrix (parse, standard form, aligned form: three PAUSEs) the
    wrapped CLI prints exactly what the reference printed."""
    ref = transcripts()[name]
    exp = _strip_timing(ref["stdout"])
    cut = 0
    for _ in range(3):
        cut = exp.index("Press Enter to continue.", cut) + len("Press Enter to continue.")
    out = _strip_timing(_run(name, ref["stdin"]).stdout)
    assert out[:cut] == exp[:cut]


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("name,z", [("testdata_max.txt", 12.0), ("kat_wyndor.txt", 36.0), ("kat_min_ge.txt", -20.0),
                                    ("a6_decimals.txt", 194 / 25), ("kat_negative_rhs.txt", 18.0)])
def test_reference_cli_solves_on_device(name, z):
    ref = transcripts()[name]
    out = _run(name, ref["stdin"]).stdout
    assert "> Device Simplex (gfx950, lpg)" in out
    line = next(ln for ln in out.splitlines() if ln.strip().startswith("z = "))
    assert abs(float(line.split("=")[1]) - z) < 1e-9 * max(1, abs(z))


@needs_bin
@pytest.mark.gpu
def test_reference_cli_testdata_readout():
    """Appendix A2: x1 = 0, x2 = 17/3 (and the slack x4 = 6)."""
    out = _run("testdata_max.txt", transcripts()["testdata_max.txt"]["stdin"]).stdout
    assert "x2=5.66666666667" in out and "x4=6" in out and "x1=0" in out


@needs_bin
@pytest.mark.gpu
def test_reference_cli_unbounded_and_free_variable():
    out = _run("kat_unbounded.txt", transcripts()["kat_unbounded.txt"]["stdin"]).stdout
    assert "UNBOUNDED" in out
    out = _run("a4_free_var.txt", transcripts()["a4_free_var.txt"]["stdin"]).stdout
    assert "UNBOUNDED" in out


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("method", ["twophase", "bigm"])
@pytest.mark.parametrize("name,z", [("a5_lack_row.txt", 6.0), ("a7_identity_quirk.txt", 2.0)])
def test_reference_cli_artificial_rows(name, z, method):
    """Rows without a unit column (CreateSMatrix's lack list; the (3/2, 1/2) quirk of
    matrix.c:67-78) are solved with artificials: the reference's menu choices."""
    ref = transcripts()[name]
    env = {**os.environ, "TERM": "dumb", "LPG_ARTIFICIAL": method}
    out = subprocess.run([BIN, os.path.join("tests", "golden", "lp", name)], input=ref["stdin"], capture_output=True,
                         text=True, timeout=120, cwd=ROOT, env=env).stdout
    assert ("Big-M" if method == "bigm" else "two-phase") in out
    line = next(ln for ln in out.splitlines() if ln.strip().startswith("z = "))
    assert abs(float(line.split("=")[1]) - z) < 1e-9


def _random_lp(rng, m, n, extra_rows):
    """A small LP file in the reference's format: <= rows with a slack each,
    plus `extra_rows` (= or >=) rows that lack a unit column."""
    def coef(v):
        return rng.choice([str(v), f"{v}/{rng.integers(2, 9)}", f"{v}.{rng.integers(1, 99)}"])

    def expr():
        terms = []
        for j in range(1, n + 1):
            if rng.random() < 0.8:
                v = int(rng.integers(1, 9))
                terms.append(("-" if rng.random() < 0.2 else "+") + coef(v) + f"x{j}")
        if not terms:
            terms = ["+x1"]
        e = "".join(terms)
        return e[1:] if e[0] == "+" else e
    rows = [f"{expr()}<={int(rng.integers(5, 60))}" for _ in range(m)]
    for _ in range(extra_rows):
        rows.insert(int(rng.integers(0, len(rows) + 1)), f"{expr()}{rng.choice(['=', '>='])}{int(rng.integers(1, 5))}")
    rows += [f"x{j}>=0" for j in range(1, n + 1)]
    obj = f"{rng.choice(['max', 'min'])}:z={expr()}"
    return "OF {\n\t" + obj + "\n}\nST {\n\t" + ";\n\t".join(rows) + "\n}\n"


@needs_msplit
def test_create_smatrix_restatement_matches_reference(tmp_path):
    """lpg_bridge.c LPGCreateSMatrix builds exactly the reference's SimplexMatrix
    (matrix.c:19-91: every cell Number, names, costs, the identity heuristic's
    basis, lack list, valid) on every fixture LP and 60 random ones (those the parser accepts) with at most
    one lacking row (two or more crash the reference at matrix.c:86)."""
    import numpy as np
    rng = np.random.default_rng(20220524)
    files = [os.path.join(LP, f) for f in sorted(os.listdir(LP)) if f not in ("a3_min_eq_neg.txt", "testdata_shipped.txt")]
    for t in range(60):
        f = tmp_path / f"r{t}.txt"
        f.write_text(_random_lp(rng, int(rng.integers(1, 5)), int(rng.integers(1, 5)), int(rng.integers(0, 2))))
        files.append(str(f))
    checked = 0
    for f in files:
        p = subprocess.run([MSPLIT, f, "compare"], capture_output=True, text=True, timeout=60, cwd=ROOT)
        if p.returncode == 3:          # the reference's parser rejected it (e.g. GCD quirks): nothing to compare
            continue
        assert p.returncode == 0 and "mismatches=0" in p.stdout, (f, p.stdout[-500:], open(f).read())
        checked += 1
    assert checked >= 50


@needs_bin
def test_two_lacking_rows_no_longer_crash():
    """the reference dies at matrix.c:86 (two rows lack a
    unit column); through the restated CreateSMatrix the CLI reaches the engine
    and then the reference's own artificial-variable menu, and exits normally."""
    ref = transcripts()["a3_min_eq_neg.txt"]
    assert ref["returncode"] != 0                   # the reference binary crashed on it
    p = _run("a3_min_eq_neg.txt", ref["stdin"])
    assert p.returncode == 0
    assert "Artificial variables are needed" in p.stdout and "Freed CONSTANT(s): M" in p.stdout


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("method", ["twophase", "bigm"])
def test_a3_min_equality_ge_nonpositive_solves(method):
    """A3: min z = 2x1 + 3x2 - x3, x1+x2+x3 >= 4, 2x1-x2 = 1, x1+3x3 <= 9, x3 <= 0:
    z* = 31/3 at x1 = 5/3, x2 = 7/3, x3 = 0 (two lacking rows -> two artificials)."""
    ref = transcripts()["a3_min_eq_neg.txt"]
    env = {**os.environ, "TERM": "dumb", "LPG_ARTIFICIAL": method}
    out = subprocess.run([BIN, os.path.join("tests", "golden", "lp", "a3_min_eq_neg.txt")], input=ref["stdin"],
                         capture_output=True, text=True, timeout=120, cwd=ROOT, env=env).stdout
    line = next(ln for ln in out.splitlines() if ln.strip().startswith("z = "))
    assert abs(float(line.split("=")[1]) - 31 / 3) < 1e-9
    assert "x1=1.66666666667" in out and "x2=2.33333333333" in out


@needs_msplit
@pytest.mark.gpu
def test_m_valued_cost_is_kept_symbolic():
    """Wyndor with cost(x1) = 1M + 0 instead of 3: lexicographic optimum first
    maximises x1 (= 4), then 5 x2 under it (x2 = 3): z = 4M + 15. Decimalize
    would have turned the cost into 0 (basicFuncs.c:298-313) and printed z = 30."""
    p = subprocess.run([MSPLIT, os.path.join(LP, "kat_wyndor.txt"), "cost", "x1", "1", "1", "0"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    assert "Big-M (symbolic M)" in p.stdout and "z = 4M + 15" in p.stdout and "valid=1" in p.stdout
    assert "Decimalize Failed" not in p.stdout


@needs_msplit
@pytest.mark.gpu
def test_m_valued_cost_with_real_part():
    """cost(x2) = -(1/2)M + 7 on Wyndor: M part first drives x2 to 0, then max 3 x1 = 12: z = 0M + 12."""
    p = subprocess.run([MSPLIT, os.path.join(LP, "kat_wyndor.txt"), "cost", "x2", "-1", "2", "7"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    line = next(ln for ln in p.stdout.splitlines() if ln.strip().startswith("z = "))
    assert abs(float(line.split("=")[1]) - 12.0) < 1e-9 and "valid=1" in p.stdout


@needs_msplit
@pytest.mark.gpu
def test_m_valued_cost_ray_with_infeasible_rows():
    """cost(x1) = M on `x2 >= 3, x2 <= 1` (no feasible point), x1 in no row: the
    M row prices x1 first (ties with x2 go to the smaller column), whose column
    is a ray while the artificial of `x2 >= 3` is still 3. A ray found with an
    artificial left positive means INFEASIBLE, as lpg_solve_big_m reports it,
    not UNBOUNDED."""
    p = subprocess.run([MSPLIT, os.path.join(LP + "_extra", "m_ray_infeasible.txt"), "cost", "x1", "1", "1", "0"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    assert "Big-M (symbolic M)" in p.stdout and "The LP is INFEASIBLE" in p.stdout and "valid=1" in p.stdout
    assert "UNBOUNDED" not in p.stdout


@needs_msplit
@pytest.mark.parametrize("args", [["cell", "0", "x1"], ["cost-denominator", "x1"]])
def test_m_where_it_cannot_be_kept_is_refused(args):
    """M in a constraint cell, or 1/M in a cost, cannot be held by the two
    objective rows: the bridge prints an ERROR and returns valid = 0 before
    touching a device (no silent Decimalize -> 0)."""
    p = subprocess.run([MSPLIT, os.path.join(LP, "kat_wyndor.txt")] + args, capture_output=True, text=True,
                       timeout=60, cwd=ROOT)
    assert p.returncode == 0
    assert "ERROR: device simplex:" in p.stdout and "valid=0" in p.stdout and "Decimalize Failed" not in p.stdout
