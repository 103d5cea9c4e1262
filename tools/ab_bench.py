"""Interleaved A/B of bench.py under environment variants (experiments only).

    python tools/ab_bench.py "ARGS" "NAME=VAL NAME=VAL" "NAME=VAL" ...   (an empty string = the default build)

Runs `python bench.py ARGS --no-cpu` once per variant, REPS (env, default 2)
rounds interleaved, each in a fresh process, and prints per run: pivots/s,
ms per block, the pass's HIP-event mean, its TFLOP/s, and whether the
trajectory parity held. Each run is limited to T_RUN seconds (default 200).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1].split()
    variants = sys.argv[2:] or [""]
    reps = int(os.environ.get("REPS", 2))
    for rep in range(reps):
        for v in variants:
            env = dict(os.environ)
            for kv in v.split():
                k, val = kv.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, "bench.py"] + args + ["--no-cpu"], cwd=ROOT, env=env,
                               capture_output=True, text=True, timeout=int(os.environ.get("T_RUN", 200)))
            if p.returncode != 0:
                print(f"[{v or 'default'}] rc={p.returncode}: {p.stderr[-1500:]}", flush=True)
                raise SystemExit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            roof = d["roofline"]
            tr = d.get("parity_trajectory") or {}
            mf = (roof.get("mfma") or {}).get("achieved", float("nan"))
            hb = (roof.get("hbm") or {}).get("achieved", float("nan"))
            fx = (d.get("parity_fixture") or {}).get("ok")
            print(f"rep {rep} [{v or 'default'}] {d['value']:.0f} pivots/s  {d['ms_per_step']:.3f} ms/block  "
                  f"pass {roof.get('update_ms_mean', float('nan')):.3f} ms  {mf:.1f} TFLOP/s  "
                  f"HBM {hb:.0f} GB/s  trajectory_ok={tr.get('ok')} fixture_ok={fx}", flush=True)


if __name__ == "__main__":
    main()
