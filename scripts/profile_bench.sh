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
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(out + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("%-60s %8s %10s %8s" % ("kernel", "calls", "avg_us", "pct"))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%-60s %8s %10.2f %7.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
PY
