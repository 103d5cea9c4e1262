"""Time every k_update variant (LPG_UPDATE_VARIANT) on one config, in one process.

  python tools/sweep_update.py [--config 3] [--steps 30] [--rounds 2] [--variants 0,6,7]

Variants are interleaved over rounds (cdna_hip_programming.md §5.4 rule 24)
and must produce identical pivot logs. Prints a table and writes
gpurun_out/sweep_config<C>.json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import linearprogramming_amd as lpg  # noqa: E402

CONFIGS = {2: (1024, 2048), 3: (16384, 32768), 4: (65536, 131072)}

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--variants", default="")
ap.add_argument("--m", type=int, default=0, help="custom shape (overrides --config)")
ap.add_argument("--n", type=int, default=0)
a = ap.parse_args()
m, n = (a.m, a.n) if a.m else CONFIGS[a.config]
lib = lpg.load()
nvar = 25
variants = [int(v) for v in a.variants.split(",")] if a.variants else list(range(nvar))
res = {v: [] for v in variants}
logs = {}
for rnd in range(a.rounds):
    for v in variants:
        os.environ["LPG_UPDATE_VARIANT"] = str(v)
        e = lpg.Engine(m, n + m + 1)
        e.generate(n, 20220518, 0)
        e.reserve_log(a.steps + 8)
        e.enqueue(3, 0)
        e.sync()
        e.set_timing(True)
        e.get_timing()
        e.enqueue(a.steps, 0)
        e.sync()
        t = e.get_timing()
        ms = t.update_ms / t.update_count
        gbs = e.info.bytes_per_pivot / (ms * 1e-3) / 1e9
        res[v].append({"update_ms": ms, "GBps": gbs, "other_ms": t.select_ms / t.update_count})
        k, r = e.get_log()
        logs.setdefault("ref", (k.tolist(), r.tolist()))
        assert (k.tolist(), r.tolist()) == logs["ref"], f"variant {v} changed the pivot sequence"
        e.close()
        print(f"round {rnd} variant {v:2d}: update {ms:8.4f} ms  {gbs:8.1f} GB/s  frac {gbs / 8000:.3f}", flush=True)
summary = {v: {"best_ms": min(x["update_ms"] for x in res[v]), "best_GBps": max(x["GBps"] for x in res[v]),
               "runs": res[v]} for v in variants}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"sweep_{m}x{n}.json"), "w") as f:
    json.dump(summary, f, indent=1)
for v in sorted(variants, key=lambda v: summary[v]["best_ms"]):
    print(f"variant {v:2d}: best {summary[v]['best_ms']:.4f} ms {summary[v]['best_GBps']:.1f} GB/s")
