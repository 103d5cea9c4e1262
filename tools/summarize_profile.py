"""Turn the rocprofv3 output of tools/gpu.sh's prof / pmc steps into committed evidence.

  gpurun -- bash tools/gpu.sh "prof:rNN:ARGS" "pmc:rNN_fetch:FETCH_SIZE:ARGS" "pmc:rNN_write:WRITE_SIZE:ARGS"
  python tools/summarize_profile.py ROUND [CONFIG] [TAG]   (reads gpurun_out/prof_TAG, pmc_TAG_fetch, pmc_TAG_write;
                                                          TAG defaults to rNN)

writes
  profiles/rNN_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/rNN_pmc.json             per-kernel FETCH_SIZE / WRITE_SIZE means and HBM bytes
  profiles/pmc_configC.json         dominant kernel's HBM bytes per launch, read by bench.py

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B
stores. The two counters come from separate passes (TCC slots).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def _one(d, pattern):
    hits = sorted(glob.glob(os.path.join(OUT, d, "**", pattern), recursive=True))
    return hits[0] if hits else None


def short(name: str) -> str:
    for key in ("k_flush_pivot_rows", "k_swap_plan", "k_move_cols", "k_fill_cols", "k_flushw", "k_flushm", "k_update", "k_select_d", "k_prep_d", "k_select", "k_prep", "k_price", "k_generate", "k_basis_slack", "k_objective"):
        if key in name:
            return key
    return name[:60]


def counter_means(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            per[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: {"mean_KB": sum(v) / len(v), "dispatches": len(v)} for k, v in per.items()}


def main():
    rnd = int(sys.argv[1])
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    tag = sys.argv[3] if len(sys.argv) > 3 else f"r{rnd:02d}"
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = _one(f"prof_{tag}", "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
        with open(stats) as f:
            rows = list(csv.DictReader(f))
        for r in rows:
            print(f"{short(r['Name']):>16s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
                  f"pct={float(r['Percentage']):6.2f}")
    fetch = _one(f"pmc_{tag}_fetch", "*counter_collection.csv")
    write = _one(f"pmc_{tag}_write", "*counter_collection.csv")
    out = {"config": cfg, "units": "KB per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE)",
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half "
                         "of a 16-B/lane streaming read; MI355X_MICROARCH.md §HBM)"}
    if fetch:
        out["FETCH_SIZE"] = counter_means(fetch, "FETCH_SIZE")
    if write:
        out["WRITE_SIZE"] = counter_means(write, "WRITE_SIZE")
    # dominant kernel: the deferred block pass if it ran (k_flushw for 64-pivot blocks), else the eager update
    fk = out.get("FETCH_SIZE", {})
    kern = "k_flushw" if "k_flushw" in fk else ("k_flushm" if "k_flushm" in fk else "k_update")
    # FETCH_SIZE correction: x2 for 16-B/lane streaming reads (guide); other widths
    # are calibrated with tools/hbm_calib3 (--fetch-factor F)
    ff = float(os.environ.get("FETCH_FACTOR", "2.0"))
    out["dominant_kernel"] = kern
    out["fetch_factor"] = ff
    upd = None
    if fetch and write and kern in out["FETCH_SIZE"] and kern in out["WRITE_SIZE"]:
        f_kb = out["FETCH_SIZE"][kern]["mean_KB"]
        w_kb = out["WRITE_SIZE"][kern]["mean_KB"]
        upd = (ff * f_kb + w_kb) * 1024
        out[f"{kern}_hbm_bytes_per_launch"] = upd
        out[f"{kern}_read_bytes"] = ff * f_kb * 1024
        out[f"{kern}_write_bytes"] = w_kb * 1024
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    # the stamp, shape and pending count of the build the passes measured: from
    # the bench lines those passes printed (bench.py attaches the traffic only
    # to a line with the same stamp, kernel, pending count and m / n)
    lines = []
    for d in (f"pmc_{tag}_fetch", f"pmc_{tag}_write"):
        try:
            with open(os.path.join(OUT, d + ".json")) as f:
                lines += [json.loads(x) for x in f if x.strip().startswith("{")]
        except OSError:
            pass
    stamps = {x["roofline"].get("source_stamp") for x in lines}
    shapes = {(x["config"]["m"], x["config"]["n"], x["roofline"].get("pending_pivots_per_launch")) for x in lines}
    if upd is not None and len(lines) == 2 and len(stamps) == 1 and len(shapes) == 1 and None not in stamps:
        (m, n, pend), = shapes
        with open(os.path.join(ROOT, "profiles", f"pmc_config{cfg}.json"), "w") as f:
            json.dump({"hbm_bytes_per_launch": upd, "source": f"profiles/{tag}_pmc.json",
                       "kernel": kern, "pending_pivots": pend, "m": m, "n": n, "source_stamp": stamps.pop(),
                       "fetch_factor": ff,
                       "how": "tools/gpu.sh pmc steps: separate rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes "
                              "of bench.py (whole blocks, no warm-up), means over the block passes"}, f, indent=1)
    elif upd is not None:
        print(f"not writing pmc_config{cfg}.json: the two passes' bench lines disagree or are missing "
              f"(stamps {stamps}, shapes {shapes})", file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
