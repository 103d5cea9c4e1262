"""linearprogramming_amd — MI355X-native dense-tableau simplex pivot engine.

The product is ``liblpg.so`` (HIP kernels for gfx950 behind the C-ABI in
include/lpg.h); this package is the Python plumbing used by tests/, bench.py
and __graft_entry__.py. See DESIGN.md.
"""
from ._lib import (GEN_ARTIFICIAL, GEN_DEGENERATE, GEN_DENSE, GEN_DUAL, ITER_LIMIT, NUMERIC, OPTIMAL, RULE_BLAND, RULE_DANTZIG, RUNNING,
                   STATUS_NAMES, UNBOUNDED, LIB_PATH, load)
from ._lib import bind_runtime, mapped_runtimes
from .engine import Engine, LPGError, SolveResult, device_count, flush_kernel_for

bind_runtime()   # one HIP runtime per process, whatever is imported next (see _lib.bind_runtime)

__all__ = ["bind_runtime", "mapped_runtimes", "Engine", "LPGError", "SolveResult", "device_count", "flush_kernel_for", "load", "LIB_PATH", "RULE_DANTZIG", "RULE_BLAND",
           "GEN_DENSE", "GEN_DEGENERATE", "GEN_ARTIFICIAL", "GEN_DUAL", "RUNNING", "OPTIMAL", "UNBOUNDED", "ITER_LIMIT", "NUMERIC", "STATUS_NAMES"]
