#!/bin/bash
# rocprofv3 kernel statistics of one stress configuration (default: BERT-base, 1 GPU).
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=${OUT:-gpurun_out/prof_stress}
rm -rf "$out"
rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 benchmarks/stress_models.py "$@" --steps 10 --warmup 3
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("%-90s %6s %10s %6s" % ("kernel", "calls", "total_ms", "pct"))
for r in rows[:30]:
    print("%-90s %6s %10.3f %5.1f%%" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                       100 * float(r["TotalDurationNs"]) / tot))
PY
