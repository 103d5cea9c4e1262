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
LP = os.path.join(ROOT, "tests", "golden", "lp")

needs_bin = pytest.mark.skipif(not os.path.exists(BIN), reason="integration/_ref/lp_lpg not built")


def _run(name, stdin):
    p = subprocess.run([BIN, os.path.join("tests", "golden", "lp", name)], input=stdin, capture_output=True,
                       text=True, timeout=120, cwd=ROOT, env={**os.environ, "TERM": "dumb"})
    return p


def _strip_timing(text):
    return "\n".join(ln for ln in text.split("\n") if not ln.startswith("> LPModel Successfully Parsed in"))


@needs_bin
@pytest.mark.parametrize("name", ["testdata_max.txt", "kat_wyndor.txt", "a6_decimals.txt"])
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
