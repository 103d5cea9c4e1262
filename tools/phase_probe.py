"""Phase timing of the deferred pivot kernels (k_prep_d, k_select_d) on config 3.

Needs tools/probe/liblpg_phases.so (liblpg built with -DLPG_PHASES). For each pivot
position q in a block: s_memrealtime (10 ns) stamps of block 0 at the phase
boundaries, relative to the earliest block start; plus the latest stamp over
all blocks (~ kernel end).
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402

lib = lpg.load(os.path.join(ROOT, "tools", "probe", "liblpg_phases.so"))
lib.lpg_debug_phases.restype = ctypes.c_int
lib.lpg_debug_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
m, n = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768))
e = lpg.Engine(m, n + m + 1)
e.generate(n, 20220518, 0)
K = e.info.defer_k
e.reserve_log(3 * K + 8)
e.solve(K + 1, 0)                    # warm: bootstrap + one block, flushed
buf = (ctypes.c_ulonglong * 32)()
names = {0: ["start", "status", "cand-reduce", "row2-staged", "chain+P+price", "pp-reduce"],
         1: ["start", "status", "pp-reduce", "staged", "chain", "cand-reduce"]}
for q in range(K):
    lib.lpg_debug_phases(buf, 1)
    e.enqueue(1, 0)
    torch.cuda.synchronize()
    lib.lpg_debug_phases(buf, 0)
    if q in (0, 1, 16, K // 2 - 1, K // 2, 63, 64, 3 * K // 4, K - 1):
        for kern in (0, 1):
            ph = [buf[kern * 16 + j] for j in range(16)]
            t0 = ph[14]
            rel = [(ph[j] - t0) * 10 / 1000 for j in range(6)]
            print(f"q={q:2d} {'prep' if kern == 0 else 'sel '}: " +
                  " ".join(f"{names[kern][j]}={rel[j]:.2f}" for j in range(6)) + f"  last={(ph[15] - t0) * 10 / 1000:.2f} us")
