"""pytest configuration: the markers and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, transcript
fixtures, the C-ABI export check and the gloo multi-rank protocol model.
`-m gpu` runs on the MI355X box and calls the HIP engine through the C-ABI.
`extended`: redundant parametrisations of a GPU case whose BASELINE-config
oracle comparison is already covered by another case (other block sizes,
launch forms, soak-style repeats); they run only with LPG_EXTENDED_TESTS=1 so
that `pytest -m gpu` stays inside the driver's step limit.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through include/lpg.h)")
    config.addinivalue_line("markers", "slow_cpu: a CPU test of tens of seconds (oracle at a BASELINE size)")
    config.addinivalue_line("markers", "extended: redundant GPU parametrisation, runs with LPG_EXTENDED_TESTS=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("LPG_EXTENDED_TESTS") == "1":
        return
    skip = pytest.mark.skip(reason="extended case (set LPG_EXTENDED_TESTS=1)")
    for it in items:
        if "extended" in it.keywords:
            it.add_marker(skip)
