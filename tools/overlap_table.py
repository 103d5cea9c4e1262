"""Per-kernel durations of tools/overlap_p8 runs from rocprofv3's database.

  python tools/overlap_table.py gpurun_out/ovprof_alone/run_results.db gpurun_out/ovprof_beside/run_results.db

For every database: each kernel's dispatch count, mean and median duration;
and for the library's pivot launch (k_pivot_block) and its own pass
(k_flushw<K, 2, 3, 4> / <64, 2, 2, 8>), the share of each dispatch's time that
a pass of the lab's instance (k_flushw<K, 2, 2, 4> / <64, 2, 1, 8>, the CU-masked
stream) covered -- the "beside" numbers are the dispatches covered >= 90%.
"""
from __future__ import annotations

import sqlite3
import statistics
import sys


def short(name: str) -> str:
    base = name.split("(")[0].replace("void ", "").replace("lpg::", "")
    return base.replace(" ", "")


def load(path):
    db = sqlite3.connect(path)
    return [(short(n), s, e) for n, s, e in db.execute("select name, start, end from kernels order by start")]


def covered(s, e, bg):
    tot = 0
    for bs, be in bg:
        if be <= s or bs >= e:
            continue
        tot += min(e, be) - max(s, bs)
    return tot / max(e - s, 1)


def main():
    for path in sys.argv[1:]:
        rows = load(path)
        bgname = {"k_flushw<32,2,2,4>", "k_flushw<64,2,1,8>"}
        bg = [(s, e) for n, s, e in rows if n in bgname]
        print(path)
        names = sorted({n for n, _, _ in rows}, key=lambda n: -sum(e - s for m, s, e in rows if m == n))
        for n in names:
            d = [(e - s) / 1e3 for m, s, e in rows if m == n]
            if sum(d) < 100:
                continue
            line = f"  {n:34s} n {len(d):5d}  mean {statistics.mean(d):9.1f} us  median {statistics.median(d):9.1f} us"
            if bg and n not in bgname and n.startswith(("k_pivot_block", "k_flushw")):
                cov = [(e - s) / 1e3 for m, s, e in rows if m == n and covered(s, e, bg) >= 0.9]
                if cov:
                    line += f"  | covered >= 90% by the lab's pass: n {len(cov)} median {statistics.median(cov):.1f} us"
            print(line)


if __name__ == "__main__":
    main()
