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
    # derived (MI355X: 256 CUs x 4 SIMDs; a wave64 VALU instruction issues over 4 cycles; GRBM_GUI_ACTIVE
    # sums the 8 XCDs' busy cycles, so / 8 is the kernel's cycle count)
    m = {c: sum(v) / len(v) for c, v in d.items()}
    if "SQ_INSTS_VALU" in m and m.get("GRBM_GUI_ACTIVE"):
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        print(f"   => VALU issue utilisation {m['SQ_INSTS_VALU'] * 4 / (1024 * cyc):.3f} "
              f"(SQ_INSTS_VALU x 4 / (1024 SIMDs x {cyc:.4g} cycles))")
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_LDS"):
            if c in m:
                print(f"   => {c} / SQ_WAVE_CYCLES {m[c] / m['SQ_WAVE_CYCLES']:.3f}")
    if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
        print(f"   => SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_INSTS_LDS']:.3f} cycles")
