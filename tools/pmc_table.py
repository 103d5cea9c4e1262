"""Per-kernel means of any rocprofv3 --pmc counters from tools/gpu.sh pmc steps.

  python tools/pmc_table.py TAG [TAG ...]      (reads gpurun_out/pmc_TAG/**/*counter_collection.csv)

Prints one line per kernel: {counter: mean per dispatch} over every pass given,
then, for k_flushw / k_pivot_block, the derived attribution (MI355X_MICROARCH.md
"rocprofv3 PMC slots": SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles and are disjoint, WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~=
WAVE_CYCLES; SQ_VALU_MFMA_BUSY_CYCLES counts cycles; GRBM_GUI_ACTIVE is summed
over the 8 XCDs).
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from summarize_profile import short  # noqa: E402


def means(tags):
    per = defaultdict(lambda: defaultdict(list))
    for tag in tags:
        for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}", "**", "*counter_collection.csv"),
                              recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    kn = row["Kernel_Name"][:80] if os.environ.get("FULLNAME") else short(row["Kernel_Name"])
                    per[kn][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in d.items()} for k, d in per.items()}


def derived(d):
    g = lambda c: d.get(c, (None, 0))[0]
    out = {}
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA"):
            if g(c) is not None:
                out[c + "/WAVE_CYCLES"] = g(c) / wc
    mb, gui = g("SQ_VALU_MFMA_BUSY_CYCLES"), g("GRBM_GUI_ACTIVE")
    if mb is not None and gui:
        # busy cycles summed over every SIMD vs the kernel's GPU-active cycles per XCD x 32 CUs x 4 SIMDs
        out["MFMA_BUSY / (GUI_ACTIVE/8 x 1024 SIMDs)"] = mb / (gui / 8 * 1024)
    if g("SQ_BUSY_CU_CYCLES") is not None and gui:
        out["SQ_BUSY_CU_CYCLES / (GUI_ACTIVE/8 x 256)"] = g("SQ_BUSY_CU_CYCLES") / (gui / 8 * 256)
    return out


def main():
    tags = sys.argv[1:]
    m = means(tags)
    for k in sorted(m, key=lambda k: -max((v[0] for v in m[k].values()), default=0)):
        print(k, {c: round(v[0], 1) for c, v in sorted(m[k].items())}, "dispatches",
              max(v[1] for v in m[k].values()))
        if k in ("k_flushw", "k_pivot_block") or "flushw" in k:
            for c, v in derived(m[k]).items():
                print(f"    {c}: {v:.3f}")


if __name__ == "__main__":
    main()
