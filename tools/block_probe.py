"""Phase timing of the persistent pivot kernel (k_pivot_block) on config 3.

Needs tools/probe/liblpg_phases.so (make phases). One launch of a whole block; for
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

lib = lpg.load(os.path.join(ROOT, "tools", "probe", os.environ.get("PHASES_LIB", "liblpg_phases.so")))
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
NS = 16                              # stamp slots per pivot (lpg_block.hip g_bph)
# + workgroup 0's clock64 beside stamp 0, + every workgroup's decision-seen stamps
buf = (ctypes.c_ulonglong * (2 * 64 * NS + 2 * 64 * 256 + 64 + 2 * 64 * 256))()
assert lib.lpg_debug_block_phases(buf) == 0
# stamp ids in time order within a pivot: 0 top, 1 ratio decision known, 15 pivot row loaded, 2 its chain,
# 8 bookkeeping done, 9 drain, 10 P / d / pricing computed, 11 slice argmin, 3 pricing record published,
# 4 pricing decision known, 6 column loads in, 7 column chain, 12 drain, 13 C / ratio candidate,
# 14 slice argmin, 5 ratio record published; then the next pivot's 0
# (15: the pivot row's loads landed and the barrier passed, before its chain)
order = [0, 1, 15, 2, 8, 9, 10, 11, 3, 4, 6, 7, 12, 13, 14, 5]
names = ["P-sweep", "row-load", "row-chain", "bookkeeping", "P-drain", "P/d/price", "P-argmin", "P-store",
         "S-sweep", "S-load", "S-chain", "S-drain", "C/cand", "S-argmin", "S-store", "->next"]
for w in ((0, 1) if any(buf[k] for k in range(2 * 64 * NS)) else ()):   # (none in the publish-only build)
    st = [[buf[(w * 64 + t) * NS + k] for k in range(NS)] for t in range(K)]
    print(f"workgroup {'0' if w == 0 else 'nwg/2'}: us per phase (10 ns ticks), by pivot range")
    for lo, hi in ((0, 1), (1, 16), (16, 32), (32, 48), (48, K)):
        acc = [0.0] * len(names)
        cnt = 0
        for t in range(lo, min(hi, K)):
            nxt = st[t + 1][0] if t + 1 < K else st[t][5]
            d = [st[t][order[i + 1]] - st[t][order[i]] for i in range(len(order) - 1)] + [nxt - st[t][5]]
            acc = [a + x * 0.01 for a, x in zip(acc, d)]
            cnt += 1
        print(f"  t in [{lo:2d},{hi:2d}): " + " ".join(f"{nm}={a / cnt:.2f}" for nm, a in zip(names, acc)) +
              f"  total={sum(acc) / cnt:.2f}")
    print(f"  launch span (wg stamps) {(st[K - 1][5] - st[0][0]) * 0.01:.1f} us for {K} pivots")

# publish skew: per pivot, every workgroup's record-store stamp (phase P and S)
nwg = e.info.pivot_wg
base = 2 * 64 * NS
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

# shader clock over the launch: clock64 ticks / s_memrealtime (100 MHz) ticks
clk = [buf[2 * 64 * NS + 2 * 64 * 256 + t] for t in range(K)]
st0 = [buf[t * NS] for t in range(K)]
if K > 2 and st0[K - 1] > st0[1]:
    print(f"shader clock over pivots 1..{K - 1}: {(clk[K - 1] - clk[1]) / ((st0[K - 1] - st0[1]) * 10.0):.3f} GHz (clock64 / s_memrealtime)")

# the hops: per pivot, the last workgroup's publish -> each workgroup's sweep
# returning the decision (pricing: phase P of t -> phase S of t; ratio: phase
# S of t -> phase P of t + 1), and each workgroup's own work between seeing
# one decision and publishing the next record; the workgroups that publish
# late most often, and by how much on average (us behind the median)
seen0 = 2 * 64 * NS + 2 * 64 * 256 + 64
if any(buf[seen0 + k] for k in range(2 * 64 * 256)):
    import statistics as S
    pub = lambda ph, t, w: buf[base + (ph * 64 + t) * 256 + w]
    seen = lambda ph, t, w: buf[seen0 + (ph * 64 + t) * 256 + w]
    T = min(K, 64)
    for nm, ph, nxt in (("pricing (P record -> S sweep)", 0, 0), ("ratio (S record -> next P sweep)", 1, 1)):
        hop_min, hop_med, hop_max = [], [], []
        for t in range(1, T - 1):
            mp = max(pub(ph, t, w) for w in range(nwg))
            ss = sorted(seen(ph, t + nxt, w) - mp for w in range(nwg))
            hop_min.append(ss[0] * 0.01)
            hop_med.append(ss[len(ss) // 2] * 0.01)
            hop_max.append(ss[-1] * 0.01)
        print(f"hop {nm}: last publish -> decision seen: min {S.mean(hop_min):.2f} median {S.mean(hop_med):.2f} "
              f"max {S.mean(hop_max):.2f} us (mean over pivots)")
    for nm, a, b, da in (("phase P work (ratio seen -> pricing published)", (1, 0), (0, 0), 0),
                         ("phase S work (pricing seen -> ratio published)", (0, 0), (1, 0), 0)):
        med, mx = [], []
        for t in range(1, T - 1):
            d = sorted((pub(b[0], t, w) - seen(a[0], t, w)) * 0.01 for w in range(nwg))
            med.append(d[len(d) // 2])
            mx.append(d[-1])
        print(f"{nm}: median {S.mean(med):.2f} us, slowest workgroup {S.mean(mx):.2f} us")
    for ph, nm in ((0, "P"), (1, "S")):
        lag = [0.0] * nwg
        for t in range(1, T - 1):
            v = [pub(ph, t, w) for w in range(nwg)]
            md = sorted(v)[nwg // 2]
            for w in range(nwg):
                lag[w] += (v[w] - md) * 0.01 / (T - 2)
        top = sorted(range(nwg), key=lambda w: -lag[w])[:8]
        print(f"phase {nm}: mean lag behind the median publish: " + ", ".join(f"wg{w} {lag[w]:.2f}" for w in top)
              + f"; xcd of the top 32: {[w % 8 for w in sorted(range(nwg), key=lambda w: -lag[w])[:32]]}")
    print(f"pivots/s of this launch (stamps): {K / ((max(pub(1, T - 2, w) for w in range(nwg)) - min(seen(1, 1, w) for w in range(nwg))) * 1e-8 / (T - 3)):.0f}")
