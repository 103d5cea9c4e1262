"""Kernel statistics from a rocprofv3 SQLite result (rocpd *.db, the default
output format when --output-format is not given), in the column layout of
rocprofv3's kernel_stats.csv. Experiments only.

    python tools/rocpd_stats.py RESULTS.db [OUT.csv]
"""
import csv
import sqlite3
import sys


def stats(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, duration from kernels").fetchall()
    by = {}
    for name, dur in rows:
        by.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in by.values()) or 1
    out = []
    for name, v in by.items():
        n = len(v)
        mean = sum(v) / n
        sd = (sum((x - mean) ** 2 for x in v) / n) ** 0.5
        out.append([name, n, sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd])
    out.sort(key=lambda r: -r[2])
    return out


def main():
    res = stats(sys.argv[1])
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(hdr)
    for r in res:
        w.writerow(r)


if __name__ == "__main__":
    main()
