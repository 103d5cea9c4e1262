"""Host front end: the reference's LP text -> SimplexMatrix -> the device engine.

A clean-room restatement of the reference's front end
for callers that do not link the reference CLI (integration/ does that): the
same input format, the same standard form and the same SimplexMatrix, quirks
included, so that ``build_smatrix(text)`` equals what the reference's
``CreateSMatrix`` builds from the same file (tests/test_frontend.py pins it to
the reference binary's transcripts). Stages, each citing what it restates:

* ``parse``        Parser / WriteIn / FormulaParser / FormulaSimplify
                   (Source/dataReader.c:148-235, 444-498, 301-386, 395-432),
                   numbers through Fractionize (basicFuncs.c:165-291)
* ``lp_trans``     LPTrans (dataReader.c:45-140), CmbSmlTerms (basicFuncs.c:338-366)
* ``standardize``  LPStandardize (simplex.c:91-230), CreateSlack / TermsSort /
                   VarCmp / InvertNegVars (simplex.c:269-354)
* ``align``        LPAlign (simplex.c:238-260)
* ``smatrix``      CreateSMatrix (matrix.c:19-91) -- the lack list written
                   correctly (the reference writes it through ``*lack[p++]`` and
                   crashes on two or more lacking rows, matrix.c:86)
* ``solve``        the device solve and readout the bridge performs
                   (integration/lpg_bridge.c LPGSolveSMatrix): rows without a
                   true unit column get artificials (two-phase or Big-M)

The variable table mirrors hashTable.c (PutVarItem replaces an existing key in
place; GetVarItems walks buckets in hash order, VarHash hashTable.c:148-167).
Numbers follow the reference's ``long`` arithmetic step for step (RNum:
Fractionize, FractionAdd / NAdd, NInv, GCD / LCM with their wrap-around
overflow checks, numOprts.c / basicFuncs.c), so exactly the models whose
arithmetic the reference rejects are rejected; the SimplexMatrix is then
handed on as exact rationals.
The symbolic constant M is refused: user input may not carry it
(dataReader.c:413-417).

Nothing here computes on the host what the engine computes: the pivots run in
liblpg (``Engine``); this module only turns text into the tableau and the
engine's column 0 back into variable values.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from fractions import Fraction
from math import gcd

import numpy as np

_I64 = 1 << 63


class FrontendError(ValueError):
    """The reference would mark the model invalid (or crash) here."""


# ---- the reference's `long` arithmetic, operation for operation -------------
# Every coefficient of the reference is a pair of C longs, and its sums and
# products are guarded by checks that rely on wrap-around (numOprts.c:19-26,
# 37-129; basicFuncs.c:123-158; the reference is built -O0 -fwrapv). RNum
# redoes each step with explicit 64-bit wrap, so a value the reference's
# checks reject (an intermediate that wraps, though the reduced result would
# fit) is rejected here too, and an invalid value keeps the numerator and
# denominator the reference keeps (a later sum may use them). Where the
# reference's own arithmetic traps (x / 0, LONG_MIN / -1: SIGFPE on x86-64)
# the model is refused instead (tests/test_frontend.py records these).
# host/lpfront.c carries the same restatement in C.
_I64MIN, _I64MAX = -_I64, _I64 - 1


def _w64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= _I64 else x


def _cdiv(a: int, b: int) -> int:
    """C division (truncating); the trapping cases of x86-64 idiv refuse the model."""
    if b == 0 or (a == _I64MIN and b == -1):
        raise FrontendError("ERROR: arithmetic trap (the reference dies with SIGFPE here)")
    q = abs(a) // abs(b)
    return q if (a < 0) == (b < 0) else -q


def _cmod(a: int, b: int) -> int:
    return a - b * _cdiv(a, b)


def _labs(a: int) -> int:
    return _w64(-a) if a < 0 else a               # labs(LONG_MIN) == LONG_MIN


def _rgcd(a: int, b: int) -> int:
    """GCD, basicFuncs.c:123-137."""
    a, b = _labs(a), _labs(b)
    if b > a:
        a, b = b, a
    while b:
        a, b = b, _cmod(a, b)
    return a


def _rlcm(a: int, b: int) -> int:
    """LCM, basicFuncs.c:145-158: -1 when the product wraps."""
    d = _rgcd(a, b)
    a, b = _labs(a), _labs(b)
    q = _cdiv(a, d)
    r = _w64(q * b)
    if q != 0 and _cdiv(r, q) != b:
        return -1
    return r


def _d2l(x: float) -> int:
    """(long) of a double as x86-64 converts it: out of range or NaN -> LONG_MIN."""
    if not (-9223372036854775808.0 <= x < 9223372036854775808.0):
        return _I64MIN
    return int(x)


def _w32(x: int) -> int:
    x &= (1 << 32) - 1
    return x - (1 << 32) if x >= 1 << 31 else x


def _d2i(x: float) -> int:
    """(int) of a double as x86-64 converts it: out of range or NaN -> INT_MIN."""
    if not (-2147483648.0 <= x < 2147483648.0):
        return -(1 << 31)
    return int(x)


class RNum:
    """A reference Number without a constant: (numerator, denominator, valid)."""
    __slots__ = ("num", "den", "valid")

    def __init__(self, num: int, den: int, valid: bool = True):
        self.num, self.den, self.valid = num, den, valid

    def __neg__(self):                            # NInv, numOprts.c:290-294: no check
        return RNum(_w64(-self.num), self.den, self.valid)

    def __add__(self, o):                         # NAdd -> FractionAdd, numOprts.c:77-196
        pn, pd, nn, nd = self.num, self.den, o.num, o.den
        if pd == 0 or nd == 0:
            return RNum(0, 0, False)
        valid = True
        cm = _rlcm(pd, nd)
        if cm == -1:
            valid = False
        pf = _cdiv(cm, pd)
        pa = _w64(pn * pf)
        nf = _cdiv(cm, nd)
        na = _w64(nn * nf)
        if (pn != 0 and _cdiv(pa, pn) != pf) or (nn != 0 and _cdiv(na, nn) != nf):
            valid = False
        if (pa > 0 and na > _I64MAX - pa) or (pa < 0 and na < _I64MIN - pa):   # OFAdd
            return RNum(0, 0, False)
        s, den = pa + na, cm
        g = _rgcd(s, den)
        return RNum(_cdiv(s, g), _cdiv(den, g), valid)

    def mul_m1(self):
        """NMul(Fractionize("-1"), x) = FractionMul(-1, 1, n, d) (numOprts.c:37-66; the
        free-variable split, simplex.c:131, 154): its check divides -n by -1, which
        traps for n = LONG_MIN."""
        if self.den == 0:
            return RNum(0, 0, False)
        p = _w64(-self.num)
        _cdiv(p, -1)
        return RNum(p, self.den)

    def value(self) -> Fraction:
        return Fraction(self.num, self.den)

    def __repr__(self):
        return f"RNum({self.num}/{self.den}{'' if self.valid else ' invalid'})"


def _strtol(s: str):
    """C strtol(s, &end, 10): (value, fully consumed)."""
    i, n = 0, len(s)
    while i < n and s[i] in " \t\n\v\f\r":
        i += 1
    j = i
    if j < n and s[j] in "+-":
        j += 1
    k = j
    while k < n and s[k] in "0123456789":
        k += 1
    if k == j:
        return 0, n == 0
    v = int(s[i:k])
    return max(-_I64, min(_I64 - 1, v)), k == n


def _tokens(s: str, d: str):
    return [t for t in s.split(d) if t]          # strtok: empty tokens skipped


def fractionize(s: str) -> RNum:
    """Fractionize (basicFuncs.c:165-291) without constants."""
    bad = RNum(0, 0, False)
    if "M" in s:
        raise FrontendError("Simplification Failed: Manual added CONSTANTs are not allowed.")
    if "/" in s:
        tk = _tokens(s, "/")
        if not tk:
            return bad
        num, ok = _strtol(tk[0])
        if not ok or len(tk) < 2:
            return bad
        den, ok2 = _strtol(tk[1])
        if not ok2 or num == 0:
            return bad
        g = _labs(_rgcd(num, den))
        den = _cdiv(den, g)
        num = _cdiv(num, g)
        return RNum(num, den, den > 0)            # basicFuncs.c:219-220: a denominator <= 0 is invalid
    if s == "" or s in ("+", "-"):
        s = s + "1"
    if "." in s:
        try:
            dec = float(s)
        except ValueError:
            return bad
        tk = _tokens(s, ".")
        if len(tk) < 2:
            return bad
        den = _d2l(10.0 ** len(tk[1]))
        num = _d2l(dec * float(den))              # (long)(decimal * denominator): truncation (basicFuncs.c:264)
        g = _labs(_rgcd(num, den))
        return RNum(_cdiv(num, g), _cdiv(den, g))  # no denominator check on this path (basicFuncs.c:262-270)
    v, ok = _strtol(s)
    return RNum(v, 1) if ok else bad


def _dec(x) -> float:
    """Decimalize (basicFuncs.c:298-313): (double) n / d; 0 for an invalid number or d = 0.
    Takes an RNum, or a Fraction of the SimplexMatrix handed on."""
    if isinstance(x, Fraction):
        return float(x.numerator) / float(x.denominator)
    return float(x.num) / float(x.den) if (x is not None and x.valid and x.den) else 0.0


@dataclass
class Term:
    coef: object                 # RNum (the reference's Number, valid or not)
    var: str = ""
    inverted: bool = False

    def copy(self):
        return Term(self.coef, self.var, self.inverted)


@dataclass
class Formula:
    left: list = field(default_factory=list)
    right: list = field(default_factory=list)
    relation: int = 0            # -2 <=, -1 <, 1 >, 2 >=, 3 =


@dataclass
class VarItem:
    name: str
    relation: int                # 0 unrestricted, +-2 sign constraint / slack
    number: int = 0
    former: str = ""             # x = former - latter for an unrestricted x
    latter: str = ""


def _valid_var(s: str) -> bool:
    """ValidVar (basicFuncs.c:374-377): a letter, then digits only."""
    return len(s) > 0 and s[0].isascii() and s[0].isalpha() and all(c in "0123456789" for c in s[1:])


def _var_hash(s: str) -> int:
    """VarHash (hashTable.c:148-167); 0 = not storable."""
    if not s or not _valid_var(s):
        return 0
    h = ord(s[0]) + sum(ord(ch) - 48 for ch in s[1:]) - 65
    return h if h > 0 else 0


class VarTable:
    """The reference's variable hash table (hashTable.c)."""

    def __init__(self):
        self.items: dict = {}    # name -> VarItem, in insertion order (replacement keeps the slot)
        self.max_x = 0

    def put(self, item: VarItem) -> bool:
        h = _var_hash(item.name)
        if not h:
            return False
        sub, _ = _strtol(item.name[1:])
        if item.name[0] == "x" and sub > self.max_x:
            self.max_x = sub
        self.items[item.name] = item
        return True

    def get(self, name: str):
        return self.items.get(name) if _var_hash(name) else None

    def ordered(self):
        """GetVarItems order: by bucket (hash), then chain (insertion) order."""
        return sorted(self.items.values(), key=lambda it: _var_hash(it.name))


@dataclass
class Model:
    otype: int = 0               # 1 max, -1 min
    zcoef: object = None
    objective: list = field(default_factory=list)   # right-hand terms of the objective
    rows: list = field(default_factory=list)        # Formula per constraint
    vars: VarTable = field(default_factory=VarTable)


def _formula(s: str) -> Formula:
    """FormulaParser + FormulaSimplify (dataReader.c:301-432)."""
    f = Formula()
    side = 0
    cfc = False
    coef = None
    buf = ""
    i, n = 0, len(s)
    while i < n + 1:
        ch = s[i] if i < n else "+"
        if ch in "+->=<":
            if buf or (coef is not None and coef.valid):
                t = Term(coef if coef is not None else RNum(0, 0, False))
                if not buf and coef is not None and coef.valid:
                    t.var = ""
                elif all(c in "0123456789/+-.M" for c in buf):   # IsConstTerm
                    t.coef, t.var = fractionize(buf), ""
                else:
                    t.var = buf[:3]
                    if not _valid_var(t.var):
                        raise FrontendError(f"ERROR: Invalid variable name: {t.var}")
                cfc = False
                (f.left if side == 0 else f.right).append(t)
                buf, coef = "", None
            if ch in "+-":
                buf += ch
            elif ch in "<>":
                mark = -1 if ch == "<" else 1
                if i + 1 < n and s[i + 1] == "=":
                    mark *= 2
                    i += 1
                f.relation, side = mark, 1
            else:
                f.relation, side = 3, 1
        else:
            if not cfc and ch not in "0123456789./":
                coef = fractionize(buf) if buf else RNum(1, 1)
                buf, cfc = "", True
            buf += ch
        i += 1
    if not f.left or not f.right or not f.relation:
        raise FrontendError("Simplification Failed: Formula invalid.")
    # FormulaSimplify: the common divisors of every numerator and every
    # denominator, valid or not, from the first term's own values; each one
    # divided in place (C division, no reduction)
    joined = f.left + f.right
    gn, gd = joined[0].coef.num, joined[0].coef.den
    for t in joined[1:]:
        gn, gd = _rgcd(gn, t.coef.num), _rgcd(gd, t.coef.den)
    for t in joined:
        t.coef = RNum(_cdiv(t.coef.num, gn), _cdiv(t.coef.den, gd), t.coef.valid)
    return f


def parse(text: str) -> Model:
    """Parser (dataReader.c:148-235) with WriteIn (dataReader.c:444-498)."""
    if isinstance(text, bytes):
        text = text.decode("utf-8", "surrogateescape")
    m = Model()
    flag = 0
    bracket = False
    buf = ""
    have_of = False
    for ch in text + "\0":                         # the trailing char stands for the EOF step
        if ch == "{":
            stop, bracket = True, True
        elif ch == "}":
            stop, bracket = True, False
        else:
            stop = (not bracket and ch in " \t\n\v\f\r") or ch == ";"
        if not stop:
            if ch in " \t\n\v\f\r" or ch == "\0":
                continue
            buf += ch
        elif buf:
            if buf == "OF":
                flag = 1
            elif buf == "ST":
                flag = 2
            elif flag == 1:
                sp = buf.split(":")
                if len(sp) < 2 or sp[0] not in ("max", "min"):
                    raise FrontendError("Objective function invalid.")
                if have_of:
                    raise FrontendError("There can be only ONE Objective function!")
                f = _formula(sp[1])
                if f.relation != 3:
                    raise FrontendError("Wrong relational operator in Objective function!")
                if len(f.left) != 1 or _dec(f.left[0].coef) != 1:
                    raise FrontendError("Non-standard Objective function!")
                m.otype = 1 if sp[0] == "max" else -1
                m.zcoef = f.left[0].coef
                m.objective = f.right
                have_of = True
            elif flag == 2:
                m.rows.append(_formula(buf))
            buf = ""
        if ch == "}":
            flag = 0
    if not have_of:
        raise FrontendError("MISSING DATA: Objective Function not found.")
    if not m.rows:
        raise FrontendError("MISSING DATA: Constraints not found.")
    return m


def _combine(terms: list, table: VarTable, record: bool) -> None:
    """CmbSmlTerms (basicFuncs.c:338-366); record: register the variables (constraints)."""
    j = 0
    while j < len(terms):
        k = j + 1
        while k < len(terms):
            if terms[j].var == terms[k].var:
                terms[j].coef = terms[j].coef + terms[k].coef
                del terms[k]
                k -= 1
            k += 1
        if not terms[j].coef.valid:
            raise FrontendError("CMB ERROR: Invalid coefficient appeared after combining.")
        if terms[j].coef.num == 0:
            del terms[j]
            j -= 1
        elif record:
            table.put(VarItem(terms[j].var, 0))
        j += 1


def lp_trans(m: Model) -> Model:
    """LPTrans (dataReader.c:45-140): constants right, variables left, like terms
    combined, sign constraints x >= 0 / x <= 0 moved into the variable table."""
    _combine(m.objective, m.vars, record=False)
    i = 0
    while i < len(m.rows):
        st = m.rows[i]
        j = 0
        while j < len(st.left):                    # j advances past the shifted term (the reference's loop)
            if st.left[j].var == "":
                t = st.left.pop(j)
                t.coef = -t.coef
                st.right.append(t)
            j += 1
        j = 0
        while j < len(st.right):
            if st.right[j].var != "":
                t = st.right.pop(j)
                t.coef = -t.coef
                st.left.append(t)
            j += 1
        if not st.left or not st.right:
            raise FrontendError(f"ERROR: LPModel invalid due to the incomplete CONSTRAINT (ST Line: {i + 1}).")
        _combine(st.left, m.vars, record=True)
        for j in range(len(st.right) - 1, 0, -1):
            st.right[0].coef = st.right[0].coef + st.right[j].coef
            del st.right[j]
        if not st.left:
            raise FrontendError(f"ERROR: No term left in the left hand side of the CONSTRAINT (ST Line: {i + 1}) "
                                "after combining similar terms.")
        if not st.right[0].coef.valid:
            raise FrontendError(f"ERROR: Division by zero appeared in the right hand side of the CONSTRAINT "
                                f"(ST Line: {i + 1}).")
        if (len(st.left) == 1 and len(st.right) == 1 and _dec(st.left[0].coef) == 1
                and _dec(st.right[0].coef) == 0 and abs(st.relation) == 2):
            m.vars.put(VarItem(st.left[0].var, st.relation))
            del m.rows[i]
            continue
        i += 1
    nof = sum(1 for t in m.objective if t.var)
    if len(m.vars.items) != nof:
        raise FrontendError("ERROR: Mismatch in the number of variables in the Objective Function and Constraints.")
    return m


def _varcmp(a: str, b: str) -> int:
    """VarCmp (simplex.c:316-325)."""
    ca, cb = (a[:1] or "\0"), (b[:1] or "\0")
    if ca != cb:
        return 1 if ca > cb else -1
    sa = _strtol(a[1:])[0] if len(a) > 1 else 0
    sb = _strtol(b[1:])[0] if len(b) > 1 else 0
    return sa - sb


def _sort(terms: list) -> None:
    """TermsSort (simplex.c:288-305): selection sort, swaps as the reference's."""
    for i in range(len(terms)):
        mi = i
        for j in range(i + 1, len(terms)):
            if _varcmp(terms[mi].var, terms[j].var) > 0:
                mi = j
        if mi != i:
            terms[i], terms[mi] = terms[mi], terms[i]


def _invert_neg(terms: list, table: VarTable) -> None:
    """InvertNegVars (simplex.c:343-354): x <= 0 becomes x' = -x >= 0."""
    for t in terms:
        it = table.get(t.var)
        if it is not None and it.relation < 0 and it.number == 0:
            t.coef = -t.coef
            t.inverted = True


def standardize(m: Model, dual: bool = False) -> Model:
    """LPStandardize (simplex.c:91-230). Primal form (dual = 0): rows with a
    negative right-hand side are negated. Dual form (dual = 1, simplex.c:178-179):
    every > / >= row is negated into < / <= instead, whatever the sign of b, so
    each inequality gets a +1 slack (the dual simplex's starting basis; the
    reference's router never reaches this branch, router.c:32-34)."""
    sub = [m.vars.max_x]

    def slack():
        sub[0] += 1
        name = f"x{sub[0]}"
        m.vars.put(VarItem(name, 2))
        return Term(RNum(0, 1), name)

    if m.otype != 1:
        m.otype = 1
        m.zcoef = -m.zcoef
        for t in m.objective:
            t.coef = -t.coef
    i = 0
    while i < len(m.objective):
        t = m.objective[i]
        it = m.vars.get(t.var)
        if it is not None and it.relation == 0:    # unrestricted: x = x'' - x'
            target, c = t.var, t.coef
            former = slack()
            former.coef = c
            m.objective[i] = former
            latter = slack()
            latter.coef = c.mul_m1()
            m.objective.insert(i + 1, latter)
            it.former, it.latter = former.var, latter.var
            i += 1
            for st in m.rows:
                k = 0
                while k < len(st.left):
                    if st.left[k].var == target:
                        ck = st.left[k].coef
                        st.left[k] = Term(ck, former.var, former.inverted)
                        st.left.insert(k + 1, Term(ck.mul_m1(), latter.var, latter.inverted))
                        k += 1
                    k += 1
        i += 1
    for st in m.rows:
        b = st.right[0]
        if (not dual and _dec(b.coef) < 0) or (dual and st.relation > 0 and st.relation != 3):
            b.coef = -b.coef
            for t in st.left:
                t.coef = -t.coef
            if st.relation != 3:
                st.relation = -st.relation
        if st.relation != 3:
            s = slack()
            m.objective.append(s)
            s = s.copy()
            s.coef = RNum(-1, 1) if st.relation > 0 else RNum(1, 1)
            st.relation = 3
            st.left.append(s)
        _sort(st.left)
        _invert_neg(st.left, m.vars)
    _sort(m.objective)
    _invert_neg(m.objective, m.vars)
    return m


def align(m: Model) -> Model:
    """LPAlign (simplex.c:238-260): every row lists the objective's variables, 0 where absent."""
    for st in m.rows:
        k = 0
        for t in m.objective:
            if t.var:
                if k >= len(st.left) or st.left[k].var != t.var:
                    z = t.copy()
                    z.coef = RNum(0, 1)
                    st.left.insert(k, z)
                k += 1
    return m


@dataclass
class SMatrix:
    """CreateSMatrix's SimplexMatrix (matrix.c:19-91) as exact rationals."""
    names: list                  # column variables 1..N (no prime)
    inverted: list               # x <= 0 columns (printed with a prime)
    costs: list                  # c_j (max form)
    rows: list                   # m x (N+1): b, a_i1 .. a_iN
    basis: list                  # 1-based basic column per row, 0 = lacking (the identity heuristic)
    lacking: list
    constant: Fraction           # the objective constant CreateSMatrix drops
    zcoef: Fraction              # -1 when the model was a min
    vars: VarTable = None

    @property
    def display_names(self):
        return [v + ("'" if inv else "") for v, inv in zip(self.names, self.inverted)]


def smatrix(m: Model) -> SMatrix:
    """CreateSMatrix (matrix.c:19-91), the lack list written correctly."""
    constant = sum((t.coef.value() for t in m.objective if not t.var), Fraction(0))
    of = [t for t in m.objective if t.var]
    rows = []
    for st in m.rows:
        if len(st.left) < len(of):
            raise FrontendError("ERROR occurred during the Standardization and the Alignment :( ")
        rows.append([st.right[0].coef] + [st.left[j].coef for j in range(len(of))])
    basis = [0] * len(rows)
    for j in range(len(of)):
        ident, pos = 0, 0
        for i, r in enumerate(rows):
            d = _dec(r[j + 1])
            if d == 1:
                pos = i
            ident = _w32(ident + (_d2i(d) if d >= 0 else 6))   # int identityPart, (int) decimalized
        if ident == 1:
            basis[pos] = j + 1
    rows = [[x.value() for x in r] for r in rows]
    return SMatrix([t.var for t in of], [t.inverted for t in of], [t.coef.value() for t in of], rows, basis,
                   [i for i, b in enumerate(basis) if b == 0], constant, m.zcoef.value(), m.vars)


def build_smatrix(text: str, dual: bool = False) -> SMatrix:
    """LP text -> the reference's SimplexMatrix (Parser, LPTrans, LPStandardize, LPAlign, CreateSMatrix);
    ``dual``: LPStandardize's dual form (for ``solve(method="dual")``)."""
    return smatrix(align(standardize(lp_trans(parse(text)), dual=dual)))


@dataclass
class LPSolution:
    status: str                  # OPTIMAL / UNBOUNDED / INFEASIBLE / ITER_LIMIT / NUMERIC
    pivots: int
    z: float = float("nan")      # the original objective (constant added, min sign restored)
    columns: dict = field(default_factory=dict)    # standard-form column -> value
    variables: dict = field(default_factory=dict)  # the user's variables, un-substituted
    method: str = "primal"


def solve(sm: SMatrix, method: str = "two_phase", rule=None, device: int = 0) -> LPSolution:
    """The bridge's device solve (integration/lpg_bridge.c LPGSolveSMatrix) on liblpg:
    rows without a true unit basic column get artificials (two-phase by default,
    ``method="big_m"`` for Big-M; ``method="dual"``: the dual simplex from the
    slack basis of a dual-form SimplexMatrix, which must be complete and dual
    feasible); the readout un-substitutes x <= 0 and free variables as the
    reference's variable table records them."""
    from . import _lib as L
    from .engine import Engine
    if rule is None:
        rule = L.RULE_DANTZIG
    m, nc0 = len(sm.rows), len(sm.names) + 1
    basis = list(sm.basis)
    for i in range(m):                              # keep a basic column only if it is a true unit column
        j = basis[i]
        if j and any(sm.rows[q][j] != (1 if q == i else 0) for q in range(m)):
            basis[i] = 0
    nlack = sum(1 for b in basis if b == 0)
    if method == "dual":
        if nlack:
            raise FrontendError("dual simplex: rows without a slack basis (equality rows); use build_smatrix(text, dual=True)")
        if any(_dec(c) > 0 for c in sm.costs):
            raise FrontendError("dual simplex: the slack basis is not dual feasible (a positive max-form cost)")
    nc = nc0 + nlack
    rows = np.zeros((m, nc), dtype=np.float64)
    for i, r in enumerate(sm.rows):
        rows[i, :nc0] = [_dec(x) for x in r]
    a = nc0
    for i in range(m):
        if not basis[i]:
            rows[i, a] = 1.0
            basis[i] = a
            a += 1
    cost = np.zeros(nc, dtype=np.float64)
    cost[:nc0 - 1] = [_dec(c) for c in sm.costs]
    bigm = method == "big_m" and nlack > 0
    with Engine(m, nc, device=device, flags=L.FLAG_BIG_M if bigm else 0) as e:
        e.load_rows(0, rows)
        e.set_basis(np.asarray(basis, dtype=np.int64))
        if method == "dual":
            e.set_objective(cost)
            r = e.solve_dual()
            used = "dual"
        elif nlack == 0:
            e.set_objective(cost)
            r = e.solve(rule=rule)
            used = "primal"
        elif bigm:
            r = e.solve_big_m(nc0, cost, rule=rule)
            used = "big_m"
        else:
            r = e.solve_two_phase(nc0, cost, rule=rule)
            used = "two_phase"
        sol = LPSolution(r.status_name, int(r.pivots), method=used)
        if r.status != L.OPTIMAL:
            return sol
        xb = e.get_column0()
        bas = e.get_basis()
    x = np.zeros(nc, dtype=np.float64)
    for i in range(m):
        x[bas[i] - 1] = xb[i]
    sol.z = (r.objective + _dec(sm.constant)) / _dec(sm.zcoef)
    sol.columns = {v: float(x[j]) for j, v in enumerate(sm.display_names)}
    val = {v: float(x[j]) for j, v in enumerate(sm.names)}
    for it in sm.vars.ordered():
        if it.relation == 0 and it.former:
            sol.variables[it.name] = val.get(it.former, 0.0) - val.get(it.latter, 0.0)
        elif it.relation < 0 and it.number == 0:
            sol.variables[it.name] = -val.get(it.name, 0.0)
        else:
            sol.variables[it.name] = val.get(it.name, 0.0)
    return sol


def solve_text(text: str, method: str = "two_phase", rule=None, device: int = 0) -> LPSolution:
    """LP text (the reference's input format) -> the optimum on the device."""
    return solve(build_smatrix(text, dual=method == "dual"), method=method, rule=rule, device=device)


def main(argv=None) -> int:
    """``python -m linearprogramming_amd.frontend model.txt [--big-m] [--bland]``:
    the reference's input file solved on the device, non-interactively."""
    import argparse
    from . import _lib as L
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("path")
    ap.add_argument("--big-m", action="store_true", help="artificials by Big-M instead of two-phase")
    ap.add_argument("--dual", action="store_true", help="dual form and the dual simplex (dual-feasible models)")
    ap.add_argument("--bland", action="store_true", help="Bland's rule instead of Dantzig's")
    a = ap.parse_args(argv)
    method = "dual" if a.dual else ("big_m" if a.big_m else "two_phase")
    try:
        sm = build_smatrix(open(a.path, "rb").read(), dual=a.dual)
        sol = solve(sm, method=method, rule=L.RULE_BLAND if a.bland else L.RULE_DANTZIG)
    except FrontendError as ex:
        print(ex)
        return 2
    print(f"{sol.status} after {sol.pivots} pivots ({sol.method})")
    if sol.status == "OPTIMAL":
        print(f"\tz = {sol.z:.12g}")
        print("\t" + "".join(f"{k}={v:.12g} | " for k, v in sol.columns.items()))
        print("Variables:\n\t" + "".join(f"{k}={v:.12g} | " for k, v in sol.variables.items()))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
