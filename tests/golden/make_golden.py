"""Regenerate the golden fixtures under tests/golden/ (run in the build container).

1. ref_transcripts.json — stdout + exit code of the REFERENCE CLI (built from
   /root/reference/Source by `make -C oracle ref` into oracle/_ref/lp) on each
   LP file in tests/golden/lp/, with the menu answers given on stdin. These pin
   the front end and the tableau the reference's CreateSMatrix builds
   (parse -> LPTrans -> LPStandardize -> LPAlign).
2. kat_cases.json — for every transcript whose aligned model yields a canonical
   identity basis: the tableau read back from the transcript and the exact
   (fractions) pivot sequence, basis and objective under Dantzig and Bland
   (oracle/fraction_oracle.py).
3. synthetic_cases.json — small splitmix64 LPs (the device generator's
   definition, restated here in Python) solved exactly by the fraction oracle.

Usage: python tests/golden/make_golden.py   (needs oracle/_ref/lp)
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
from fractions import Fraction

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import fraction_oracle  # noqa: E402
import refparse  # noqa: E402

REF_BIN = os.path.join(ROOT, "oracle", "_ref", "lp")

# menu answers: <Enter> after the parse, '1' primal simplex, <Enter> x2 for the
# standard/aligned PAUSEs, ['1' Big-M when the artificial prompt appears], 'q'.
STDIN_PLAIN = "\n1\n\n\nq\n"
STDIN_ARTIFICIAL = "\n1\n\n\n1\nq\n"
ARTIFICIAL = {"a3_min_eq_neg.txt", "a5_lack_row.txt"}
PARSE_FAIL = {"testdata_shipped.txt"}

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def subkey(seed: int, which: int) -> int:
    return splitmix64(seed ^ ((which * 0xD1B54A32D192ED03) & M64))


def uniform(key: int, idx: int) -> float:
    return (splitmix64(key ^ ((idx * 0x9E3779B97F4A7C15) & M64)) >> 11) * 2.0 ** -53


def synthetic(m: int, n: int, seed: int, kind: int):
    """Python restatement of lpo_generate / k_generate (float64 values)."""
    kA, kB, kC = subkey(seed, 1), subkey(seed, 2), subkey(seed, 3)
    bscale = n / 8.0
    T = []
    for i in range(m):
        row = [0.0] * (n + m + 1)
        if kind in (0, 3):
            sg = -1.0 if kind == 3 else 1.0          # kind 3 (dual): rows [-b | -A | I]
            row[0] = sg * (bscale * (1.0 + uniform(kB, i)))
            for j in range(n):
                row[1 + j] = sg * uniform(kA, i * n + j)
        else:
            row[0] = bscale * (1.0 + uniform(kB, i)) if i & 1 else 0.0
            sgn = -1.0 if (kind == 2 and not i & 1) else 1.0
            for j in range(n):
                row[1 + j] = sgn * (uniform(kA, i * n + j) / float(i + 1)) if j < i else (1.0 if j == i else 0.0)
        row[unit_column(m, n, i, kind)] = 1.0
        T.append(row)
    obj = [0.0] * (n + m + 1)
    for j in range(n):
        cj = 1.0 + uniform(kC, j)
        obj[1 + j] = cj if kind == 3 else -cj
    T.append(obj)
    basis = [unit_column(m, n, i, kind) for i in range(m)]
    return T, basis


def unit_column(m: int, n: int, i: int, kind: int) -> int:
    """Initial unit column of row i (kind 2: even-row slacks, then odd-row artificials)."""
    if kind != 2:
        return 1 + n + i
    return 1 + n + (m + 1) // 2 + i // 2 if i & 1 else 1 + n + i // 2


def frac_str(x: Fraction) -> str:
    return f"{x.numerator}/{x.denominator}"


def exact_case(T, basis, rule, max_pivots=5000):
    res = fraction_oracle.solve(T, basis, rule=rule, max_pivots=max_pivots)
    return {"status": res["status"], "pivots": res["pivots"], "basis": res["basis"],
            "objective": frac_str(res["objective"]), "objective_f64": float(res["objective"])}


def transcripts():
    out = {}
    lpdir = os.path.join(HERE, "lp")
    for name in sorted(os.listdir(lpdir)):
        stdin = STDIN_ARTIFICIAL if name in ARTIFICIAL else STDIN_PLAIN
        if name in PARSE_FAIL:
            stdin = "\n"
        p = subprocess.run([REF_BIN, os.path.join("tests", "golden", "lp", name)], input=stdin,
                           capture_output=True, text=True, timeout=20, cwd=ROOT, env={"TERM": "dumb", "PATH": "/usr/bin:/bin"})
        # the parse timer (main.c:20-23) is the only non-deterministic line
        stdout = re.sub(r"Parsed in [0-9.]+s\.", "Parsed in 0.000000s.", p.stdout)
        out[name] = {"stdin": stdin, "stdout": stdout, "returncode": p.returncode}
    return out


def kat_cases(trans):
    cases = []
    for name, t in trans.items():
        models = refparse.parse_models(t["stdout"])
        if len(models) < 3:
            continue
        aligned = models[2]
        rt = refparse.tableau_from_aligned(aligned)
        entry = {"name": name, "names": rt.names, "basis": rt.basis, "lacking": rt.lacking,
                 "costs": [frac_str(c) for c in rt.costs], "constant": frac_str(rt.constant),
                 "zcoef": frac_str(rt.zcoef), "canonical": refparse.canonical(rt),
                 "rows": [[frac_str(x) for x in r] for r in rt.T]}
        if entry["canonical"]:
            full = refparse.full_tableau(rt)
            entry["tableau"] = [[frac_str(x) for x in r] for r in full]
            for rule in ("dantzig", "bland"):
                entry[rule] = exact_case(full, rt.basis, rule, max_pivots=60)
        cases.append(entry)
    return cases


def synthetic_cases():
    cases = []
    for (m, n, seed, kind, rules) in [(3, 4, 1, 0, ("dantzig", "bland")), (6, 8, 2, 0, ("dantzig", "bland")),
                                      (8, 12, 20220518, 0, ("dantzig", "bland")), (12, 16, 7, 0, ("dantzig",)),
                                      (16, 20, 11, 0, ("dantzig",)), (6, 6, 3, 1, ("bland", "dantzig")),
                                      (10, 10, 5, 1, ("bland",))]:
        T, basis = synthetic(m, n, seed, kind)
        entry = {"m": m, "n": n, "seed": seed, "kind": kind,
                 "b_hex": [float.hex(r[0]) for r in T[:m]],
                 "a00_hex": float.hex(T[0][1])}
        for rule in rules:
            entry[rule] = exact_case(T, basis, rule)
        cases.append(entry)
    return cases


def main():
    if not os.path.exists(REF_BIN):
        sys.exit(f"{REF_BIN} missing: run `make -C oracle ref` (needs /root/reference)")
    trans = transcripts()
    with open(os.path.join(HERE, "ref_transcripts.json"), "w") as f:
        json.dump(trans, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "kat_cases.json"), "w") as f:
        json.dump(kat_cases(trans), f, indent=1)
    with open(os.path.join(HERE, "synthetic_cases.json"), "w") as f:
        json.dump(synthetic_cases(), f, indent=1)
    print("wrote", ", ".join(sorted(os.listdir(HERE))))


if __name__ == "__main__":
    main()
