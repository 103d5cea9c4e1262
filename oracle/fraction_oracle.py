"""Exact-rational restatement of the pivot loop — TEST INFRASTRUCTURE ONLY.

Pure-Python ``fractions.Fraction`` tableau simplex with the same rules as
oracle/lpo.c and the device engine: Dantzig pricing
(argmin d_j, ties -> smallest j) or Bland (first j with d_j < 0), min-ratio
over a_ik > 0 with ties -> smallest row (Dantzig) / smallest basic column
(Bland), Gauss-Jordan update. In exact arithmetic the tolerances are zero.

It plays the role the reference's Number arithmetic (Source/numOprts.c:137-294,
long num/den with GCD reduction) would have played had the reference's pivot
loop existed (it does not: Source/simplex.c:40 -> :65): exact rationals, but
with unbounded integers so it cannot overflow the way `long` fractions do
after ~16 chained updates. Small cases only (pure Python).
"""
from __future__ import annotations

from fractions import Fraction


def solve(T, basis, rule="dantzig", max_pivots=10_000, nact=None):
    """T: list of m+1 rows (objective row last) of numbers; basis: m 1-based columns.

    Returns dict(status, pivots=[(k, r), ...], basis, objective (Fraction), tableau).
    """
    T = [[Fraction(x) for x in row] for row in T]
    basis = list(basis)
    m = len(T) - 1
    ncols = len(T[0])
    nact = ncols - 1 if nact is None else nact
    pivots = []
    status = "ITER_LIMIT"
    for _ in range(max_pivots):
        d = T[m]
        if rule == "bland":
            k = next((j for j in range(1, nact + 1) if d[j] < 0), None)
        else:
            k = min(range(1, nact + 1), key=lambda j: (d[j], j))
            if not d[k] < 0:
                k = None
        if k is None:
            status = "OPTIMAL"
            break
        best = None
        for i in range(m):
            a = T[i][k]
            if a > 0:
                b = T[i][0]
                theta = b / a if b > 0 else Fraction(0)
                key = (theta, basis[i] if rule == "bland" else i)
                if best is None or key < best[0]:
                    best = (key, i)
        if best is None:
            status = "UNBOUNDED"
            break
        r = best[1]
        piv = T[r][k]
        P = [x / piv for x in T[r]]
        for i in range(m + 1):
            if i == r:
                continue
            c = T[i][k]
            if c != 0:
                T[i] = [t - c * p for t, p in zip(T[i], P)]
        T[r] = P
        basis[r] = k
        pivots.append((k, r))
    else:
        # budget exhausted: report OPTIMAL if the final tableau is optimal
        d = T[m]
        if rule == "bland":
            done = all(not d[j] < 0 for j in range(1, nact + 1))
        else:
            done = not min(d[1:nact + 1]) < 0
        if done:
            status = "OPTIMAL"
    return {"status": status, "pivots": pivots, "basis": basis, "objective": T[m][0], "tableau": T}
