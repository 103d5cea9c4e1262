"""Read the reference CLI's model printout back into a dense tableau (test helper).

The reference prints models with PrintModel/PrintTerms
(Source/basicFuncs.c:416-512): terms ``<num>[/<den>][<var>[']]`` joined by
`` + `` / `` - ``, one constraint per line. After LPAlign
(Source/simplex.c:238-260) every constraint lists exactly the objective's
variables in the same order, so the "aligned" printout *is* the tableau that
CreateSMatrix (Source/matrix.c:19-91) builds: column 0 = b, columns 1..N =
a_ij, the objective constant dropped (matrix.c:23-28).

The basis is detected with CreateSMatrix's own heuristic (matrix.c:59-78): a
column is taken as basic if the sum over its entries of (x >= 0 ? floor(x) : 6)
equals 1, in the row of its last entry equal to 1 (row 0 if none) — including
the reference's quirk that accepts a non-unit column such as (3/2, 1/2).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from fractions import Fraction

_TERM = re.compile(r"(-?\d+)(M?)(?:/(-?\d+)(M?))?(?:\[([^\]]*)\])?")


def parse_terms(s: str):
    """'1[x1] + 9/14[x2] - 1/3' -> [(Fraction, var, inverted)]; var '' for constants."""
    s = s.strip()
    out = []
    pos = 0
    sign = 1
    while pos < len(s):
        mt = _TERM.match(s, pos)
        if not mt:
            raise ValueError(f"cannot parse terms at {s[pos:]!r} in {s!r}")
        num, m1, den, m2, var = mt.groups()
        if m1 or m2:
            raise ValueError("Big-M coefficients are not representable as fp64")
        # PrintTerms prints a later term as " - labs(n)", and labs(LONG_MIN) is
        # LONG_MIN: " - -9223372036854775808" means the numerator LONG_MIN itself
        n = int(num)
        val = Fraction(n if (sign < 0 and n < 0) else n * sign, int(den) if den else 1)
        var = var or ""
        inverted = var.endswith("'")
        out.append((val, var.rstrip("'"), inverted))
        pos = mt.end()
        rest = s[pos:]
        if not rest:
            break
        if rest.startswith(" + "):
            sign = 1
        elif rest.startswith(" - "):
            sign = -1
        else:
            raise ValueError(f"unexpected separator {rest[:3]!r} in {s!r}")
        pos += 3
    return out


@dataclass
class PrintedModel:
    sense: str                 # 'max' / 'min'
    zcoef: Fraction            # coefficient of z on the left (-1 after min->max)
    objective: list            # [(coef, var, inverted)]
    rows: list                 # [(lhs terms, relation, rhs Fraction)]
    variables: str = ""


def parse_models(text: str):
    """All PrintModel blocks in a transcript, in order."""
    models = []
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        if ln.endswith("Objective Function:"):   # may follow "Press Enter to continue."
            head = lines[i + 1].strip()
            mt = re.match(r"(max|min):(.*?) = (.*)$", head)
            sense = mt.group(1)
            left = parse_terms(mt.group(2))
            obj = parse_terms(mt.group(3))
            assert lines[i + 2].startswith("Subject to:"), lines[i + 2]
            rows = []
            j = i + 3
            while j < len(lines) and lines[j].startswith("\t"):
                mr = re.match(r"\t(.*) (<=|<|>=|>|=) (.*)$", lines[j])
                lhs = parse_terms(mr.group(1))
                rhs = parse_terms(mr.group(3))
                rows.append((lhs, mr.group(2), rhs[0][0]))
                j += 1
            variables = ""
            if j + 2 < len(lines) and lines[j + 1].startswith("Variables:"):
                variables = lines[j + 2].strip()
            models.append(PrintedModel(sense, left[0][0], obj, rows, variables))
            i = j
        else:
            i += 1
    return models


@dataclass
class RefTableau:
    names: list                # column names 1..N (inverted vars keep the ')
    T: list                    # (m+1) x (N+1) Fractions; objective row = -c (slack basis form)
    costs: list                # c_1..c_N
    basis: list                # 1-based basic column per row (0 = lacking)
    constant: Fraction         # objective constant dropped by CreateSMatrix
    zcoef: Fraction            # -1 when the original problem was a min
    lacking: list = field(default_factory=list)


def tableau_from_aligned(model: PrintedModel) -> RefTableau:
    """CreateSMatrix (matrix.c:19-91) on an aligned, standardised model."""
    constant = sum((c for c, v, _ in model.objective if v == ""), Fraction(0))
    ofterms = [(c, v, inv) for c, v, inv in model.objective if v != ""]
    names = [v + ("'" if inv else "") for _, v, inv in ofterms]
    costs = [c for c, _, _ in ofterms]
    m = len(model.rows)
    T = []
    for lhs, rel, rhs in model.rows:
        assert rel == "=", "tableau needs the standard form"
        assert [v for _, v, _ in lhs] == [v for _, v, _ in ofterms], "row is not aligned"
        T.append([rhs] + [c for c, _, _ in lhs])
    basis = [0] * m
    for j in range(len(names)):
        ident = 0
        pos = 0
        for i in range(m):
            x = T[i][j + 1]
            d = float(x.numerator) / float(x.denominator)       # Decimalize
            if d == 1.0:
                pos = i
            di = int(d) if -2147483648.0 <= d < 2147483648.0 else -(1 << 31)   # (int) d on x86-64
            ident = ((ident + (di if d >= 0 else 6) + (1 << 31)) % (1 << 32)) - (1 << 31)   # int, wrapping
        if ident == 1:
            basis[pos] = j + 1
    lacking = [i for i in range(m) if basis[i] == 0]
    return RefTableau(names, T, costs, basis, constant, model.zcoef, lacking)


def canonical(rt: RefTableau) -> bool:
    """Every basic column is a true unit column (the quirk of matrix.c:67-78 can violate this)."""
    if rt.lacking:
        return False
    m = len(rt.T)
    for i, col in enumerate(rt.basis):
        for q in range(m):
            if rt.T[q][col] != (1 if q == i else 0):
                return False
    return True


def full_tableau(rt: RefTableau):
    """(m+1) x (N+1) with the objective row d_j = c_B B^-1 a_j - c_j for the detected basis."""
    m = len(rt.T)
    ncols = len(rt.T[0])
    obj = [Fraction(0)] * ncols
    for j in range(ncols):
        acc = sum((rt.costs[rt.basis[i] - 1] * rt.T[i][j] for i in range(m)), Fraction(0))
        obj[j] = acc if j == 0 else acc - rt.costs[j - 1]
    return [list(r) for r in rt.T] + [obj]
