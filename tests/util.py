"""Shared test helpers: golden fixtures as float64 tableaus."""
from __future__ import annotations

import json
import os
from fractions import Fraction

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STATUS = {"RUNNING": 0, "OPTIMAL": 1, "UNBOUNDED": 2, "INFEASIBLE": 3, "ITER_LIMIT": 4, "NUMERIC": 5}


def frac(s: str) -> Fraction:
    return Fraction(s)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def kat_cases():
    """Canonical cases read back from the reference transcripts."""
    return [c for c in load_json("kat_cases.json") if c.get("canonical")]


def kat_tableau(case):
    """float64 (m+1) x ncols tableau (values are exactly the fp64 rounding of the rationals)."""
    return np.array([[float(frac(x)) for x in row] for row in case["tableau"]], dtype=np.float64)


def kat_costs(case):
    return np.array([float(frac(x)) for x in case["costs"]], dtype=np.float64)


def synthetic_cases():
    return load_json("synthetic_cases.json")


def transcripts():
    return load_json("ref_transcripts.json")


def pivots_of(case_rule):
    return [tuple(p) for p in case_rule["pivots"]]
