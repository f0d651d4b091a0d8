#!/usr/bin/env python3
"""Average PMC counter values per kernel over rocprofv3 --pmc passes (tools/pmc_run.sh)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"]
            if flt and flt not in k:
                continue
            # "void tsdb::(anonymous namespace)::k_x<...>(args)" -> "tsdb::k_x<...>"
            name = k.replace("(anonymous namespace)::", "").split("(")[0]
            name = name[5:] if name.startswith("void ") else name
            acc[name[:90]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:22s} {sum(v) / len(v):16.4g}   (n={len(v)})")
