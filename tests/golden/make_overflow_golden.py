"""Overflow fixtures: LP models whose coefficients drive the reference's `long`
arithmetic past its limits, and what the reference binary does with each.

The reference guards sums and products of its rationals with checks that rely
on wrap-around (Source/numOprts.c:52-53 FractionMul, :106-107 FractionAdd,
:19-26 OFAdd, basicFuncs.c:145-158 LCM), converts decimals with
(long) pow(10, k) and (long)(d * 10^k) (basicFuncs.c:262-264), negates without
a check (NInv, numOprts.c:290-294) and divides in FormulaSimplify
(dataReader.c:420-428). Run with oracle/_ref/lp (built -O0 -fwrapv by
oracle/Makefile from /root/reference) in the build container:

    python tests/golden/make_overflow_golden.py    -> tests/golden/overflow_cases.json

Each case records the model text and the reference's outcome: "accepted" with
its aligned tableau as printed (numerators / denominators as the reference
holds them), "rejected" with the reference's first error line, or "crash"
(the process died: SIGFPE where its arithmetic divides by zero or LONG_MIN by
-1). Data only: the model texts are generated here, the outcomes are the
reference's output.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import refparse  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "lp")
STDIN = "\n1\n\n\n1\n\n\nq\n"
L = (1 << 63) - 1


def lp(obj, rows):
    return "OF {\n\t" + obj + "\n}\nST {\n\t" + ";\n\t".join(rows) + "\n}\n"


NAMED = [
    ("obj_like_terms_overflow", lp(f"max:z={L}x1+1x1", ["x1<=4", "x1>=0"])),
    ("lcm_overflow_like_terms", lp("max:z=x1+x2", ["1/3037000499x1+1/3037000507x1+x2<=4", "x1>=0", "x2>=0"])),
    ("min_with_long_max", lp(f"min:z={L}x1+x2", ["x1+x2>=4", "x1>=0", "x2>=0"])),
    ("decimal_19_digits", lp("max:z=x1+x2", ["0.1234567890123456789x1+x2<=4", "x1>=0", "x2>=0"])),
    ("decimal_25_digits", lp("max:z=x1+x2", ["0.1234567890123456789012345x1+x2<=4", "x1>=0", "x2>=0"])),
    ("sum_of_two_2_62", lp("max:z=x1+x2", [f"{1 << 62}x1+{1 << 62}x1+x2<=4", "x1>=0", "x2>=0"])),
    ("huge_rhs_flip", lp("max:z=x1+x2", [f"x1+x2<={1 << 62}", f"x1-3x2>=-{L}", "x1>=0", "x2>=0"])),
    # the reduced sum (2^62 + 1) fits in a long, the intermediate 2^63 + 2 does not: rejected
    ("intermediate_sum_overflow", lp("max:z=x1+x2", [f"{(1 << 62) + 1}/2x1+{(1 << 62) + 1}/2x1+x2<=4", "x1>=0",
                                                     "x2>=0"])),
    # LONG_MIN negated by NInv stays LONG_MIN (no check): min -> max keeps its sign
    ("min_with_long_min", lp(f"min:z=-{1 << 63}x1+x2", ["x1+x2<=4", "x1>=0", "x2>=0"])),
    # ... and NMul(-1, LONG_MIN) of the free-variable split traps (SIGFPE)
    ("free_var_long_min", lp(f"max:z=-{1 << 63}x1+x2", ["x1+x2<=4", "x2>=0"])),
    # FormulaSimplify divides by the GCD of all numerators: 0 for an all-zero formula (SIGFPE)
    ("all_zero_formula", lp("max:z=x1+x2", ["0x1<=0", "x1+x2<=4", "x1>=0", "x2>=0"])),
    ("big_decimal_value", lp("max:z=x1+x2", ["12345678901234567.5x1+x2<=40", "x1>=0", "x2>=0"])),
    # right-hand sides combined in reverse order: an LCM overflow's invalid sum 0/-1 made valid again by + 0
    ("rhs_validity_restored", lp("max:z=x1+x2", ["x1+x2<=1/3037000499+0+1/3037000507", "x1>=0", "x2>=0"])),
    ("rhs_sum_overflow", lp("max:z=x1+x2", [f"x1+x2<={1 << 62}+{1 << 62}", "x1>=0", "x2>=0"])),
    ("strtol_saturates", lp("max:z=x1+x2", ["99999999999999999999x1+x2<=4", "x1>=0", "x2>=0"])),
    ("fraction_saturates", lp("max:z=x1+x2", ["1/99999999999999999999x1+x2<=4", "x1>=0", "x2>=0"])),
    ("moved_term_overflow", lp("max:z=x1+x2", [f"{L}x1<=4-1x1", "x2<=3", "x1>=0", "x2>=0"])),
]

BIG = [str(v) for v in (L, L - 1, 1 << 62, (1 << 62) + 1, 3037000499, 3037000507, 2147483647, 2147483648,
                        4294967296, 999999999999, 1 << 40)]


def random_big(rng):
    """A small model mixing ordinary and near-limit coefficients."""
    n = int(rng.integers(1, 4))

    def coef():
        k = rng.random()
        if k < 0.3:
            return rng.choice(BIG)
        if k < 0.45:
            return f"1/{rng.choice(BIG)}"
        if k < 0.55:
            return f"{rng.choice(BIG)}/{rng.integers(2, 9)}"
        if k < 0.65:
            return f"0.{''.join(str(d) for d in rng.integers(0, 10, int(rng.integers(12, 22))))}"
        return str(int(rng.integers(1, 9)))

    def expr():
        terms = []
        for j in range(1, n + 1):
            for _ in range(int(rng.integers(1, 3))):       # like terms get combined
                terms.append(("-" if rng.random() < 0.3 else "+") + coef() + f"x{j}")
        e = "".join(terms)
        return e[1:] if e[0] == "+" else e
    rows = [f"{expr()}{rng.choice(['<=', '>=', '='])}{rng.choice(['4', '40', rng.choice(BIG)])}"
            for _ in range(int(rng.integers(1, 4)))]
    rows += [f"x{j}>=0" for j in range(1, n + 1)]
    obj = f"{rng.choice(['max', 'min'])}:z=" + "+".join(f"{coef()}x{j}" for j in range(1, n + 1))
    return lp(obj, rows)


def outcome(text, path):
    with open(path, "w") as f:
        f.write(text)
    p = subprocess.run([REF, path], input=STDIN, capture_output=True, text=True, timeout=20, cwd=ROOT,
                       env={"TERM": "dumb", "PATH": "/usr/bin:/bin"})
    if p.returncode < 0:
        return {"outcome": "crash", "signal": -p.returncode}
    models = refparse.parse_models(p.stdout)
    if len(models) < 3:
        err = next((ln.strip() for ln in p.stdout.splitlines() if "ERROR" in ln or "Failed" in ln or "invalid" in ln),
                   "")
        return {"outcome": "rejected", "message": err}
    rt = refparse.tableau_from_aligned(models[2])
    fs = lambda x: f"{x.numerator}/{x.denominator}"   # noqa: E731
    return {"outcome": "accepted", "names": rt.names, "basis": rt.basis, "lacking": rt.lacking,
            "costs": [fs(c) for c in rt.costs], "constant": fs(rt.constant), "zcoef": fs(rt.zcoef),
            "rows": [[fs(x) for x in r] for r in rt.T]}


def main():
    if not os.path.exists(REF):
        sys.exit("oracle/_ref/lp not built (make -C oracle ref)")
    rng = np.random.default_rng(20221017)
    cases = [(name, text) for name, text in NAMED] + [(f"random_{t}", random_big(rng)) for t in range(120)]
    out = []
    tmp = os.path.join("/tmp", "lpg_overflow_case.txt")
    for name, text in cases:
        rec = {"name": name, "text": text}
        rec.update(outcome(text, tmp))
        out.append(rec)
    with open(os.path.join(HERE, "overflow_cases.json"), "w") as f:
        json.dump(out, f, indent=1)
    counts = {k: sum(1 for r in out if r["outcome"] == k) for k in ("accepted", "rejected", "crash")}
    print("wrote overflow_cases.json", counts)


if __name__ == "__main__":
    main()
