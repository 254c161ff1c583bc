#!/usr/bin/env python3
"""Roofline of the exact-fp32 headline step (B = 100, one MI355X) from a rocprofv3 kernel trace of
``bench.py`` (scripts/profile_bench.sh): per-kernel median time over the graph-replayed steady state,
achieved TFLOP/s against the measured fp32-MFMA rate (155 TF/s, v_mfma_f32_16x16x4_f32; the xf32 /
sparsity headline figures do not apply) and TB/s against HBM3E's ~8 TB/s.

    python scripts/roofline_f32.py <run_kernel_trace.csv> [bench.log] > profiles/roofline_f32_latest.md

Start-up is filtered out: only kernels launched at least once per step over the trace's last
``--tail`` fraction count (the eager warm-up, torch's init kernels, copies and fills drop out), and
each kernel's time is the median over that window. FLOPs count 2 per multiply-add; bytes are the
compulsory HBM traffic (operands read once, outputs written once), so a kernel near neither roof is
latency- or issue-bound.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics

PEAK_TFLOPS = 155.0  # measured fp32 MFMA rate (bench_native/mfma_f32_rate.hip)
# split-bf16 kernels (csrc/kernels/f32_common.h, f32_products = 6): six bf16 part products per fp32
# product on the bf16 MFMAs (~2.5 PF dense): an fp32-equivalent ceiling of 2500 / 6 TF/s
PEAK_SPLIT = 2500.0 / 6
PEAK_TBS = 8.0
B = 100
W3 = 3136 * 1024
F = 4  # bytes per fp32

CONV1_GF = 2 * B * 784 * 32 * 25 / 1e9
CONV2_GF = 2 * B * 196 * 64 * 800 / 1e9
FC1_GF = 2 * B * W3 / 1e9
MB = 1e6

# kernel-name regex -> (label, GFLOP, MB, what)
WORK = [
    (r"f32x9_conv2_fwd_kernel", "conv2_fwd [split x6]", CONV2_GF,
     (B * 6272 * F + B * 3136 * (F + 1) + 51200 * F) / MB, "conv2 forward on split-bf16 products, bias/ReLU/pool fused"),
    (r"f32x_fc1_fwd_kernel", "fc1_fwd [split x6]", FC1_GF, (W3 * F + B * 3136 * F + 14 * B * 1024 * F) / MB,
     "fc1 split-K x14 on split-bf16 products"),
    (r"f32x_conv2_bwd_kernel", "conv2_bwd [split x6]", 2 * CONV2_GF + CONV1_GF,
     (B * 3136 * F * 2 + B * 6272 * (F + 1) + B * 784 * F + 25 * 51200 * F + 245 * 832 * F) / MB,
     "conv2 dgrad (+ conv1 wgrad epilogue) + conv2 wgrad slabs, both on split-bf16 products"),
    (r"f32_conv2_fwd_kernel<\d+, false, true, true", "conv12_fwd", CONV1_GF + CONV2_GF,
     (B * 784 * F + B * 6272 * (F + 1) + B * 3136 * (F + 1) + 51200 * F + 800 * F) / MB,
     "conv1 + conv2 forward, bias/ReLU/pool/argmax fused (one launch)"),
    (r"f32_conv2_fwd8?_kernel", "conv2_fwd", CONV2_GF,
     (B * 6272 * F + B * 3136 * (F + 1) + 51200 * F) / MB, "conv2 forward, bias/ReLU/pool/argmax fused"),
    (r"f32_conv1_kernel", "conv1_fwd", CONV1_GF, (B * 784 * F + B * 6272 * (F + 1) + 3 * 51200 * F) / MB,
     "conv1 forward (+ the two W2 fragment copies)"),
    (r"f32_fc1_fwd\d?_kernel<\d+, true>", "fc1_fwd+W3 adam", FC1_GF,
     (W3 * F * 7 + B * 3136 * F + 14 * B * 1024 * F) / MB, "fc1 split-K x14 + the deferred W3 Adam (p,g,m,v)"),
    (r"f32_fc1_fwd\d?_kernel", "fc1_fwd", FC1_GF, (W3 * F + B * 3136 * F + 14 * B * 1024 * F) / MB, "fc1 split-K x14"),
    (r"f32_head1?k?_kernel", "head", 2 * 2 * B * 1024 * 10 / 1e9, (14 * B * 1024 * F + 3 * B * 1024 * F) / MB,
     "slab sum, bias, ReLU, dropout, fc2, softmax-xent, dz"),
    (r"f32_fc1_bwd_rows_kernel<\d+, true", "fc1_bwd+W3 adam", 2 * FC1_GF,
     (W3 * F * 5 + B * 3136 * F * 2 + B * 1024 * F) / MB, "dgrad + dW3 + fused W3 Adam (W3 once; m, v in/out)"),
    (r"f32_fc1_bwd", "fc1_bwd", 2 * FC1_GF, (W3 * F * 2 + B * 3136 * F * 2 + B * 1024 * F) / MB,
     "dgrad + dW3 (+ db3, dW4, db4)"),
    (r"f32_conv2_bwd_kernel", "conv2_bwd", 2 * CONV2_GF + CONV1_GF,
     (B * 3136 * F * 2 + B * 6272 * (F + 1) + B * 784 * F + 25 * 51200 * F + 245 * 832 * F) / MB,
     "conv2 dgrad (+ conv1 wgrad epilogue) + conv2 wgrad slabs"),
    (r"f32_conv_reduce_kernel", "conv_reduce+adam", 0.0, (25 * 51200 * F + 245 * 832 * F + 58000 * F * 7) / MB,
     "dW2/dW1/db sums + Adam of the conv and small fc params"),
]


def classify(name):
    for rx, label, gf, mb, what in WORK:
        if re.search(rx, name):
            return label, gf, mb, what
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench", nargs="?", help="bench.py stdout (its JSON line gives ms_per_step)")
    ap.add_argument("--tail", type=float, default=0.5, help="fraction of the trace taken as steady state")
    ap.add_argument("--stats", help="also write the filtered per-kernel stats table to this file")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    # the window: the tail of the span of the step's own kernels (start-up and teardown work -- fills,
    # copies, communicator setup after the timed region -- lies outside it)
    step_rows = [r for r in rows if classify(r["Kernel_Name"])] or rows
    t0, t1 = int(step_rows[0]["Start_Timestamp"]), int(step_rows[-1]["End_Timestamp"])
    cut = t1 - a.tail * (t1 - t0)
    win = [r for r in rows if cut <= int(r["Start_Timestamp"]) <= t1]
    by = {}
    for r in win:
        by.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    steps = max(len(v) for n, v in by.items() if classify(n)) if any(classify(n) for n in by) else \
        max(len(v) for v in by.values())
    step_ms, bench_line = None, None
    if a.bench:
        for line in open(a.bench):
            if line.startswith("{"):
                step_ms, bench_line = json.loads(line).get("ms_per_step"), line.strip()
    if a.stats:  # the filtered per-kernel table (profiles/rocprof_f32_kernel_stats_latest.txt)
        keep = {n: v for n, v in by.items() if len(v) >= 0.8 * steps}
        tot = sum(statistics.median(v) for v in keep.values())
        with open(a.stats, "w") as f:
            if bench_line:
                f.write(bench_line + "\n")
            f.write(f"# steady state: last {int(a.tail * 100)}% of {a.trace} (graph-replayed bench.py under "
                    "rocprofv3 --kernel-trace --stats);\n")
            f.write(f"# only kernels launched about once per step ({steps} launches) are listed: start-up "
                    "fills/copies and warm-up kernels are dropped\n")
            f.write(f"{'kernel':<62s} {'calls':>6s} {'median_us':>10s} {'mean_us':>10s} {'pct':>7s}\n")
            for n, v in sorted(keep.items(), key=lambda kv: -statistics.median(kv[1])):
                m = statistics.median(v)
                f.write(f"{n[:62]:<62s} {len(v):>6d} {m:>10.2f} {statistics.mean(v):>10.2f} "
                        f"{100 * m / tot:>6.1f}%\n")
            f.write(f"{'sum of medians':<62s} {'':>6s} {tot:>10.2f}\n")
    print("# Roofline of the exact-fp32 headline step (B = 100, one MI355X)\n")
    print(f"Kernel times: median per kernel over the last {int(a.tail * 100)}% of `{a.trace}` "
          f"(graph-replayed steady state, {steps} launches of the most frequent kernel); start-up and warm-up "
          f"kernels are filtered out (a kernel counts only if it runs about once per step in that window). "
          f"Peaks: fp32 MFMA {PEAK_TFLOPS:.0f} TF/s (measured); the split-bf16 kernels ([split x6]) against "
          f"{PEAK_SPLIT:.0f} TF/s fp32-equivalent (six bf16 part products per fp32 product at ~2.5 PF); HBM3E "
          f"{PEAK_TBS:.0f} TB/s.\n")
    print("| kernel | work | µs | GFLOP | MB | TFLOP/s | % of peak (155, or 417 for split) | TB/s | % of 8 TB/s | floor µs |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    tot_us = tot_gf = tot_mb = floor_sum = 0.0
    skipped = []
    for name, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1])):
        c = classify(name)
        if c is None or len(v) < 0.8 * steps:
            skipped.append((name[:70], len(v)))
            continue
        label, gf, mb, what = c
        us = statistics.median(v)
        tf, tbs = gf / us * 1e3, mb / us
        pk = PEAK_SPLIT if "[split" in label else PEAK_TFLOPS
        floor = max(gf / pk * 1e3, mb / PEAK_TBS)
        tot_us += us
        tot_gf += gf
        tot_mb += mb
        floor_sum += floor
        print(f"| `{label}` | {what} | {us:.2f} | {gf:.3f} | {mb:.1f} | {tf:.1f} | {100 * tf / pk:.0f}% | "
              f"{tbs:.2f} | {100 * tbs / PEAK_TBS:.0f}% | {floor:.1f} |")
    print(f"| **kernel sum** | | {tot_us:.2f} | {tot_gf:.2f} | {tot_mb:.0f} | {tot_gf / tot_us * 1e3:.1f} | "
          f"{100 * tot_gf / tot_us * 1e3 / PEAK_TFLOPS:.0f}% | {tot_mb / tot_us:.2f} | "
          f"{100 * tot_mb / tot_us / PEAK_TBS:.0f}% | {floor_sum:.1f} |")
    if step_ms:
        us = step_ms * 1e3
        print(f"\nMeasured step (bench.py, graph-replayed, barrier + synchronize around the timed loop): "
              f"**{us:.1f} µs**; kernel sum {tot_us:.1f} µs, so {max(0.0, us - tot_us):.1f} µs of launch gaps. "
              f"Sum of per-kernel floors {floor_sum:.1f} µs ({100 * floor_sum / us:.0f}% of the step).")
    # launch gaps of the graph-replayed steady state: start of each kernel minus the end of the
    # kernel before it (same queue), by boundary
    seq = [r for r in win if classify(r["Kernel_Name"]) is not None]
    gaps = {}
    for a, b in zip(seq, seq[1:]):
        la, lb = classify(a["Kernel_Name"])[0], classify(b["Kernel_Name"])[0]
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if g < 50:  # (a replay boundary or a host gap is not a launch gap)
            gaps.setdefault((la, lb), []).append(g)
    if gaps:
        print("\nLaunch gaps between consecutive kernels (median µs, start of the next minus end of the previous):\n")
        print("| boundary | gap µs | count |")
        print("|---|---|---|")
        tot = 0.0
        for (la, lb), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
            if len(v) < 0.5 * steps:
                continue
            m = statistics.median(v)
            tot += m
            print(f"| `{la}` -> `{lb}` | {m:.2f} | {len(v)} |")
        print(f"| **per step** | {tot:.2f} | |")
    if skipped:
        print("\nFiltered out (start-up / warm-up / not once per step): " +
              ", ".join(f"`{n}` ×{k}" for n, k in skipped[:12]))


if __name__ == "__main__":
    main()
