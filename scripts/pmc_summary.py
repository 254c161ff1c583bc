#!/usr/bin/env python3
"""Median per-dispatch PMC values per kernel (and study variant) from rocprofv3 --pmc CSV dirs.

    python scripts/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB ...
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mihvd::", "mihvd:")
            key = (name[-64:] if "mihvd" not in name else name[name.index("mihvd"):][:64], r["Grid_Size"])
            out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    agg = collections.defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in load(d).items():
            for c, v in cs.items():
                agg[k][c] = sorted(v)[len(v) // 2]
    for (name, grid), cs in sorted(agg.items()):
        if "mihvd" not in name and "f32" not in name:
            continue
        wc = cs.get("SQ_WAVE_CYCLES")
        line = f"{name:64s} grid {grid:>7s}"
        if wc:
            line += (f" | wait {cs['SQ_WAIT_ANY'] / wc:.2f} waitInst {cs['SQ_WAIT_INST_ANY'] / wc:.2f}"
                     f" active {cs['SQ_ACTIVE_INST_ANY'] / wc:.2f} waitLDS {cs['SQ_WAIT_INST_LDS'] / wc:.2f}")
        rest = {c: v for c, v in cs.items() if c not in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                          "SQ_WAIT_INST_LDS")}
        line += " | " + " ".join(f"{c.replace('SQ_', '')}={v:.3g}" for c, v in sorted(rest.items()))
        print(line)


if __name__ == "__main__":
    main()
