"""Diagnostic: one HIP runtime per process, and a clean exit, for each load order.

usage: python tools/runtime_order.py {lpg_only|torch_first|lpg_first}

Runs a tiny solve through the C-ABI, then lists every libamdhip64 mapped into
the process and every library family mapped from two different files (torch's
bundled copy next to the system ROCm's). Exits 1 if any is duplicated; the
caller checks the exit status as well (an abort at interpreter exit is 134).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
order = sys.argv[1]
if order == "torch_first":
    import torch  # noqa: F401
import linearprogramming_amd as lpg  # noqa: E402  (binds the runtime: see _lib.bind_runtime)

lib = lpg.load()
ctx = ctypes.c_void_p()
if lpg.device_count() == 0:   # build container: loading and exit only
    ctx = None
else:
  assert lib.lpg_create(ctypes.byref(ctx), 0, ctypes.c_int64(8), ctypes.c_int64(8 + 12 + 1), 0) == 0
  assert lib.lpg_generate(ctx, ctypes.c_int64(12), ctypes.c_uint64(1), 0) == 0
  res = lpg._lib.Result()
  assert lib.lpg_solve(ctx, ctypes.c_int64(1000), 0, ctypes.byref(res)) == 0
  assert res.status == lpg.OPTIMAL, res.status
  lib.lpg_destroy(ctx)
if order == "lpg_first":
    import torch  # noqa: F401,F811
dups = lpg._lib.duplicated_libraries()
print(order, "runtime:", lpg._lib.bind_runtime(), "libamdhip64:", lpg.mapped_runtimes(), "duplicated:", dups, flush=True)
sys.exit(1 if dups or len(lpg.mapped_runtimes()) != 1 else 0)
