#!/usr/bin/env python3
"""Where do the non-mihvd kernels of a rocprofv3 kernel trace sit in the step?

    python scripts/trace_neighbors.py <dir with *kernel_trace.csv> [substring ...]

For every kernel whose name contains one of the substrings (default: the HIP runtime's
``__amd_rocclr`` copy / fill kernels), counts the (previous kernel, next kernel) pairs around it on
the same queue, and prints the median gap between consecutive kernels of the steady state.
"""
import collections
import csv
import glob
import statistics
import sys


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("mihvd::", "")[:48]


def main():
    d = sys.argv[1]
    keys = sys.argv[2:] or ["__amd_rocclr"]
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    pairs = collections.Counter()
    for i, n in enumerate(names):
        if any(k in rows[i]["Kernel_Name"] for k in keys):
            prev = names[i - 1] if i else "-"
            nxt = names[i + 1] if i + 1 < len(names) else "-"
            pairs[(prev, n, nxt)] += 1
    print("%6s  %-48s %-34s %-48s" % ("count", "previous", "kernel", "next"))
    for (p, n, x), c in pairs.most_common(30):
        print("%6d  %-48s %-34s %-48s" % (c, p, n, x))
    gaps = collections.defaultdict(list)
    for i in range(1, len(rows)):
        g = (int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3
        gaps[(names[i - 1], names[i])].append(g)
    print("\nmedian gap (us) between consecutive kernels, pairs seen >= 50 times")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        if len(v) >= 50:
            print("%8.2f  %5d  %s -> %s" % (statistics.median(v), len(v), a, b))


if __name__ == "__main__":
    main()
