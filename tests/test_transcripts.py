"""Reference-binary transcripts (tests/golden/ref_transcripts.json) — the
behaviour the tableau the engine receives must agree with.

These fixtures were produced by the reference CLI itself (built from
/root/reference/Source by `make -C oracle ref`; script tests/golden/make_golden.py).
"""
from __future__ import annotations

from fractions import Fraction

import refparse
from util import kat_cases, load_json, transcripts


def _models(name):
    return refparse.parse_models(transcripts()[name]["stdout"])


def test_shipped_testdata_fails_to_parse():
    """Source/testdata.txt:2 says `ma:` — WriteIn rejects it (dataReader.c:452-487)."""
    out = transcripts()["testdata_shipped.txt"]["stdout"]
    for line in ("Objective function invalid.", "MISSING DATA: Objective Function not found.",
                 "MISSING DATA: Constraints not found.", "Error occurred when parsing the model."):
        assert line in out
    assert "Freed CONSTANT(s): M" in out


def test_testdata_max_forms():
    parsed, standard, aligned = _models("testdata_max.txt")[:3]
    assert parsed.sense == "max"
    assert [(c, v) for c, v, _ in standard.objective] == [(Fraction(19, 3), ""), (1, "x1"), (1, "x2"), (0, "x3"), (0, "x4")]
    rt = refparse.tableau_from_aligned(aligned)
    assert rt.T == [[Fraction(51, 14), 1, Fraction(9, 14), 1, 0], [Fraction(1, 3), 2, -1, 0, 1]]
    assert rt.basis == [3, 4] and rt.constant == Fraction(19, 3)


def test_decimal_truncation():
    """Fractionize truncates (long)(d*10^k) (basicFuncs.c:264): 0.29 -> 7/25, 0.57 -> 14/25."""
    parsed = _models("a6_decimals.txt")[0]
    coefs = {v: c for c, v, _ in parsed.objective}
    assert coefs["x1"] == Fraction(7, 25) and coefs["x2"] == Fraction(14, 25)
    assert coefs["x3"] == Fraction(11, 10) and coefs["x4"] == Fraction(-49, 20)


def test_row_gcd_simplification():
    parsed = _models("a8_gcd.txt")[0]
    lhs, rel, rhs = parsed.rows[0]
    assert [(c, v) for c, v, _ in lhs] == [(1, "x1"), (2, "x2")] and rel == "<=" and rhs == 4


def test_free_variable_split_and_min_inversion():
    std = _models("a4_free_var.txt")[1]
    assert [v for _, v, _ in std.objective] == ["x1", "x3", "x4", "x5", "x6"]
    assert "x2(unr)=x3-x4" in std.variables
    a3 = _models("a3_min_eq_neg.txt")[1]
    assert a3.zcoef == -1 and any(inv for _, _, inv in a3.objective)   # x3' for x3 <= 0


def test_identity_heuristic_quirk():
    """(3/2, 1/2) is accepted as a basic column in row 0 (matrix.c:67-78): no prompt, not canonical."""
    t = transcripts()["a7_identity_quirk.txt"]
    assert "Artificial variables are needed" not in t["stdout"]
    case = next(c for c in load_json("kat_cases.json") if c["name"] == "a7_identity_quirk.txt")
    assert case["basis"] == [1, 3] and not case["canonical"]


def test_artificial_prompt_and_reference_crash():
    t5 = transcripts()["a5_lack_row.txt"]
    assert "Artificial variables are needed due to the lack of Identity Matrix." in t5["stdout"]
    assert "1. Big M Method." in t5["stdout"] and "2. Two-phase Method." in t5["stdout"]
    # two lacking rows hit the out-of-bounds store at matrix.c:86 (`*lack[lackPtr++] = i`)
    t3 = transcripts()["a3_min_eq_neg.txt"]
    assert t3["returncode"] == -11 or t3["returncode"] == 139


def test_every_canonical_case_has_exact_answers():
    names = {c["name"] for c in kat_cases()}
    assert {"testdata_max.txt", "kat_wyndor.txt", "kat_beale_cycling.txt", "kat_unbounded.txt"} <= names
