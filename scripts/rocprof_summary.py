#!/usr/bin/env python3
"""Compact per-kernel table from a rocprofv3 --kernel-trace --stats --output-format csv directory.

    python scripts/rocprof_summary.py gpurun_out/prof_f32 "title" > profiles/x.txt
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else d
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    print(f"# {title}")
    print(f"# {'calls':>6} {'avg us':>8} {'min us':>8} {'max us':>8} {'%':>6}  kernel")
    for r in rows:
        name = r["Name"].split("(")[0]
        print(f"  {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f} {float(r['MinNs']) / 1e3:8.2f} "
              f"{float(r['MaxNs']) / 1e3:8.2f} {float(r['Percentage']):6.2f}  {name}")


if __name__ == "__main__":
    main()
