"""Diagnostic: does process exit stay clean for each load order of liblpg and torch?

usage: python tools/runtime_order.py {lpg_only|torch_first|lpg_first}
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
order = sys.argv[1]
if order == "torch_first":
    import torch  # noqa: F401
lib = ctypes.CDLL(os.path.join(ROOT, "linearprogramming_amd", "liblpg.so"), mode=ctypes.RTLD_GLOBAL)
ctx = ctypes.c_void_p()
assert lib.lpg_create(ctypes.byref(ctx), 0, ctypes.c_int64(8), ctypes.c_int64(8 + 12 + 1), 0) == 0
assert lib.lpg_generate(ctx, ctypes.c_int64(12), ctypes.c_uint64(1), 0) == 0
res = (ctypes.c_char * 64)()
assert lib.lpg_solve(ctx, ctypes.c_int64(1000), 0, res) == 0
lib.lpg_destroy(ctx)
if order == "lpg_first":
    import torch  # noqa: F401,F811
print(order, "ok", flush=True)
