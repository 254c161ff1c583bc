#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace: for the steady-state steps (each starts at the
first kernel whose name contains ``--start``, default the fp32 conv1), every kernel's median start
and end offset from the step start, its queue, and the median step period.

    python scripts/step_timeline.py <dir with *kernel_trace.csv> [--start f32_conv1] [--last 0.5]
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("mihvd::", "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--start", default="f32_conv1_kernel")
    ap.add_argument("--last", type=float, default=0.5, help="fraction of the steps (the tail) to use")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.start in r["Kernel_Name"]]
    steps = []
    for j in range(len(starts) - 1):
        t0 = int(rows[starts[j]]["Start_Timestamp"])
        t1 = int(rows[starts[j + 1]]["Start_Timestamp"])
        ks = []
        for r in rows:
            s = int(r["Start_Timestamp"])
            if t0 <= s < t1:
                ks.append((short(r["Kernel_Name"]), r["Queue_Id"], s - t0, int(r["End_Timestamp"]) - t0))
        steps.append((t1 - t0, ks))
    keep = steps[int(len(steps) * (1 - a.last)):]
    # the most common kernel sequence among kept steps
    seqs = collections.Counter(tuple((k[0], k[1]) for k in ks) for _, ks in keep)
    seq, cnt = seqs.most_common(1)[0]
    sel = [ks for _, ks in keep if tuple((k[0], k[1]) for k in ks) == seq]
    print(f"steps {len(steps)}, kept {len(keep)}, modal sequence in {cnt}; median period "
          f"{statistics.median(p for p, _ in keep) / 1e3:.2f} us")
    print(f"{'kernel':<62}{'queue':>6}{'start':>9}{'end':>9}{'dur':>8}")
    for i, (name, q) in enumerate(seq):
        st = statistics.median(ks[i][2] for ks in sel) / 1e3
        en = statistics.median(ks[i][3] for ks in sel) / 1e3
        print(f"{name:<62}{q:>6}{st:9.2f}{en:9.2f}{en - st:8.2f}")


if __name__ == "__main__":
    main()
