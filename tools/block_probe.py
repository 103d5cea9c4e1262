"""Phase timing of the persistent pivot kernel (k_pivot_block) on config 3.

Needs tools/liblpg_phases.so (make phases). One launch of a whole block; for
every pivot t the s_memrealtime (10 ns) stamps of thread 0 of workgroups 0
and nwg/2: loop top, ratio decision known, row loads in, pricing record
published, pricing decision known, ratio record published.
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402

lib = lpg.load(os.path.join(ROOT, "tools", os.environ.get("PHASES_LIB", "liblpg_phases.so")))
lib.lpg_debug_block_phases.restype = ctypes.c_int
lib.lpg_debug_block_phases.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
m, n = int(os.environ.get("M", 16384)), int(os.environ.get("N", 32768))
e = lpg.Engine(m, n + m + 1)
e.generate(n, 20220518, 0)
K = e.info.defer_k
print(f"m={m} n={n} K={K} workgroups={e.info.pivot_wg}")
e.reserve_log(4 * K + 8)
e.solve(2 * K, 0)                    # warm: bootstrap + two blocks, flushed
e.enqueue(K, 0)                      # one launch of K pivots
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (2 * 64 * 8 + 2 * 64 * 256))()
assert lib.lpg_debug_block_phases(buf) == 0
names = ["P-sweep", "row-load+chain", "P-publish", "S-sweep", "S-load", "S-chain", "S-publish", "->next"]
for w in (0, 1):
    st = [[buf[(w * 64 + t) * 8 + k] for k in range(8)] for t in range(K)]
    print(f"workgroup {'0' if w == 0 else 'nwg/2'}: us per phase (10 ns ticks), by pivot range")
    for lo, hi in ((0, 1), (1, 16), (16, 32), (32, 48), (48, K)):
        acc = [0.0] * 8
        cnt = 0
        for t in range(lo, min(hi, K)):
            nxt = st[t + 1][0] if t + 1 < K else st[t][5]
            d = [st[t][1] - st[t][0], st[t][2] - st[t][1], st[t][3] - st[t][2], st[t][4] - st[t][3],
                 st[t][6] - st[t][4], st[t][7] - st[t][6], st[t][5] - st[t][7], nxt - st[t][5]]
            acc = [a + x * 0.01 for a, x in zip(acc, d)]
            cnt += 1
        print(f"  t in [{lo:2d},{hi:2d}): " + " ".join(f"{nm}={a / cnt:.2f}" for nm, a in zip(names, acc)) +
              f"  total={sum(acc) / cnt:.2f}")
    print(f"  launch span (wg stamps) {(st[K - 1][5] - st[0][0]) * 0.01:.1f} us for {K} pivots")

# publish skew: per pivot, every workgroup's record-store stamp (phase P and S)
nwg = e.info.pivot_wg
base = 2 * 64 * 8
for ph, nm in ((0, "P"), (1, "S")):
    spread, late = [], {}
    for t in range(1, K):
        v = [buf[base + (ph * 64 + t) * 256 + w] for w in range(nwg)]
        srt = sorted(v)
        med = srt[len(srt) // 2]
        spread.append(((srt[-1] - med) * 0.01, (med - srt[0]) * 0.01))
        w = v.index(srt[-1])
        late[w] = late.get(w, 0) + 1
    import statistics
    print(f"phase {nm} publish: max-median {statistics.mean(a for a, _ in spread):.2f} us, "
          f"median-min {statistics.mean(b for _, b in spread):.2f} us; latest workgroups: "
          + ", ".join(f"{w}x{c}" for w, c in sorted(late.items(), key=lambda x: -x[1])[:8]))
