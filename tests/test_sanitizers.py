"""ASan + UBSan builds of the host-side C (SURVEY.md §4 "Sanitizers", §5): the
oracle (oracle/lpo.c, driven by oracle/lpo_selftest.c), the reference front
end with the lpg bridge (integration/lpg_bridge.c) and the C host driver
(host/lpgcli.c). Built by __graft_entry__.build() (`make -C oracle sanitize`,
`make -C integration sanitize`); CPU only: without a GPU the bridge run covers
parsing, standardisation, the restated CreateSMatrix and the fp64 conversion
and stops at lpg_create, and lpgcli covers its tableau-file parser.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from test_integration_cli import _random_lp
from util import transcripts

SELFTEST = os.path.join(ROOT, "oracle", "_san", "lpo_selftest")
BRIDGE = os.path.join(ROOT, "integration", "_san", "lp_lpg")
CLI = os.path.join(ROOT, "integration", "_san", "lpgcli")
LP = os.path.join(ROOT, "tests", "golden", "lp")
ENV = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1",
       "TERM": "dumb"}


def _clean(p):
    text = p.stdout + p.stderr
    assert "Sanitizer" not in text and "runtime error" not in text, text[-3000:]


@pytest.mark.skipif(not os.path.exists(SELFTEST), reason="oracle sanitizer build absent")
def test_oracle_under_asan_ubsan():
    p = subprocess.run([SELFTEST], capture_output=True, text=True, timeout=300, env=ENV)
    _clean(p)
    assert p.returncode == 0 and "lpo_selftest: ok" in p.stdout


@pytest.mark.skipif(not os.path.exists(BRIDGE), reason="bridge sanitizer build absent")
def test_bridge_front_end_under_asan_ubsan(tmp_path):
    tr = transcripts()
    runs = [(os.path.join(LP, f), tr[f]["stdin"]) for f in sorted(os.listdir(LP))]
    rng = np.random.default_rng(11)
    # random LPs, including ones with several lacking rows (the matrix.c:86 case). Menus read with
    # ReadChar, which spins on EOF (basicFuncs.c:458-462), so the input answers every prompt either
    # flow can show: the artificial-variable menu ("1") if it appears, else the algorithm menu
    # runs the method again, and a later "q" exits
    for t in range(20):
        f = tmp_path / f"r{t}.txt"
        f.write_text(_random_lp(rng, int(rng.integers(1, 6)), int(rng.integers(1, 6)), int(rng.integers(0, 4))))
        runs.append((str(f), "\n1\n\n\n1\n" + "q\n" * 8))
    for f, stdin in runs:
        p = subprocess.run([BRIDGE, f], input=stdin, capture_output=True, text=True, timeout=120, env=ENV, cwd=ROOT)
        _clean(p)
        assert p.returncode == 0, (f, p.stdout[-2000:])


@pytest.mark.skipif(not os.path.exists(CLI), reason="lpgcli sanitizer build absent")
@pytest.mark.parametrize("content", ["", "1 3\n", "2 4\n1 1 0 1\n", "x y\n", "1 3\n4 1 1\n-1 0 0\n2\n",
                                     "1 3\n4 1 1\n-1 0 0\n9\n"])
def test_lpgcli_parser_under_asan_ubsan(tmp_path, content):
    f = tmp_path / "t.txt"
    f.write_text(content)
    p = subprocess.run([CLI, "--tableau", str(f)], capture_output=True, text=True, timeout=60, env=ENV)
    _clean(p)
    assert p.returncode in (0, 1)
