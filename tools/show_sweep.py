"""Print the bench lines of tools/sweep_flush.sh logs compactly."""
import json
import sys

for path in sys.argv[1:]:
    tag = None
    for line in open(path):
        if line.startswith("K="):
            tag = line.strip()
            continue
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            print(f"{path.split('/')[-1]:24s} {tag:10s} pivots/s {d['value']:9.1f}  flush {r['update_ms_mean']:7.3f} ms "
                  f"{r['achieved']:6.0f} GB/s  other/pivot {r['other_ms_per_pivot'] * 1e3:6.1f} us  n={r['launches_timed']}")
