#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --kernel-trace --stats run: name, calls, total and average time.

    python tools/prof_top.py <rocprofv3 output dir> [N]"""
import csv
import glob
import sys

root = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = []
for f in glob.glob(f"{root}/**/*kernel_stats.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
            name = name[5:] if name.startswith("void ") else name
            rows.append((float(r["TotalDurationNs"]), int(r["Calls"]), float(r["AverageNs"]), name[:100]))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows) or 1.0
for t, c, a, name in rows[:n]:
    print(f"{t / 1e6:10.3f} ms  {100 * t / tot:5.1f}%  calls {c:6d}  avg {a / 1e3:10.1f} us  {name}")
