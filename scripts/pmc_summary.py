#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per mihvd kernel from the CSVs written by pmc_bench.sh."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "").split("(")[0]
        grid = r.get("Grid_Size") or r.get("Grid_Size_X")
        if grid:
            name += "/g" + grid
        if "mihvd" not in name:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sys.argv[2:] or ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_LDS_BANK_CONFLICT", "FETCH_SIZE", "TCC_HIT_sum", "GRBM_GUI_ACTIVE"]
print("%-28s" % "kernel" + "".join("%14s" % c.replace("SQ_", "")[:13] for c in cols))
for k, d in sorted(acc.items()):
    print("%-28s" % k.replace("mihvd::", "")[:28] + "".join(
        "%14.0f" % (sum(d[c]) / len(d[c])) if d.get(c) else "%14s" % "-" for c in cols))
