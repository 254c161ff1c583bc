#!/bin/bash
# Kernel-level profile of the fused training step (rocprofv3 kernel trace + stats, no PMC).
set -eu
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/prof_fused}
shift || true
export TMPDIR=/tmp
rm -rf "$out"
rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 bench.py --steps 200 --warmup 20 "$@"
find "$out" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$out/kernel_stats.csv"
python3 - "$out" <<'PY'
import csv, glob, statistics, sys
out = sys.argv[1]
f = glob.glob(out + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in by.values())
# median: the graph-replayed steady state (the mean also counts the eager warm-up launches)
print("%-60s %7s %10s %10s %7s" % ("kernel", "calls", "median_us", "mean_us", "pct"))
for name, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1]))[:25]:
    print("%-60s %7d %10.2f %10.2f %6.1f%%" % (name[:60], len(v), statistics.median(v), sum(v) / len(v),
                                            100 * sum(v) / tot))
PY
