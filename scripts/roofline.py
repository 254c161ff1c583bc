#!/usr/bin/env python3
"""Roofline view of the fused MNIST step: per-kernel FLOPs and HBM bytes (analytic, B = 100) against
the kernel times measured by scripts/kbench.py, as achieved TFLOP/s and TB/s and as a fraction of the
MI355X dense peaks (bf16 MFMA ~2.5 PFLOP/s without sparsity, HBM3E ~8 TB/s).

    python scripts/roofline.py profiles/kbench_latest.txt > profiles/roofline_latest.md

The bytes are the compulsory traffic of each kernel (operands read once, outputs written once); the
FLOPs count 2 per multiply-add. A kernel far below both roofs is latency-bound: at B = 100 most of
the step is, which is why the design fuses launches rather than chasing per-kernel FLOP rates.
"""
import re
import sys

PEAK_TFLOPS = 2500.0  # bf16 dense MFMA
PEAK_TBS = 8.0
B = 100
W3 = 3136 * 1024
PARAMS = 3274634

# name -> (GFLOP, MB of compulsory HBM traffic, what)
WORK = {
    "conv12_fwd": (2 * B * 784 * 32 * 25 / 1e9 + 2 * B * 196 * 64 * 800 / 1e9,
                   (B * 784 * 4 + B * 6272 * 3 + B * 3136 * 3 + 51200 * 2) / 1e6, "conv1 + conv2 fwd, pool/argmax"),
    "conv1_fwd": (2 * B * 784 * 32 * 25 / 1e9, (B * 784 * 4 + B * 6272 * 3) / 1e6, "conv1 fwd (VALU fp32)"),
    "conv2_fwd": (2 * B * 196 * 64 * 800 / 1e9, (B * 6272 * 2 + B * 3136 * 3 + 51200 * 2) / 1e6, "conv2 fwd"),
    "fc1_fwd": (2 * B * W3 / 1e9, (W3 * 2 + B * 3136 * 2 + 14 * B * 1024 * 4) / 1e6, "fc1 split-K x14"),
    "head": (2 * B * 1024 * 10 * 2 / 1e9, (14 * B * 1024 * 4 + B * 1024 * 4) / 1e6, "slab sum, dropout, fc2, xent, dz"),
    "fc1_bwd": (4 * B * W3 / 1e9, (W3 * 2 + W3 * 4 + B * 3136 * 4 + B * 1024 * 6) / 1e6, "fc1 dgrad + dW3/db3/dW4/db4"),
    "fc1_wgrad": (2 * B * W3 / 1e9, (W3 * 4 + B * 3136 * 2 + B * 1024 * 6) / 1e6, "dW3 (+ small grads)"),
    "fc1_dgrad": (2 * B * W3 / 1e9, (W3 * 2 + B * 3136 * 4 + B * 1024 * 2) / 1e6, "dz W3^T"),
    "conv2_bwd": (2 * 2 * B * 196 * 64 * 800 / 1e9 + 2 * B * 784 * 32 * 25 / 1e9,
                  (B * 3136 * 3 + B * 6272 * 3 + B * 784 * 4 + 25 * 51200 * 4 + B * 896 * 4) / 1e6,
                  "conv2 dgrad + wgrad slabs + conv1 wgrad"),
    "conv2_wgrad_reduce": (0.0, (25 * 51200 * 4 + B * 896 * 4) / 1e6, "dW2 = sum of slabs"),
    "adam": (0.0, PARAMS * (7 * 4 + 2) / 1e6, "TF1 Adam, 3.27 M params + bf16 shadow"),
    "adam_w3": (0.0, W3 * (7 * 4 + 2) / 1e6, "Adam, dense/kernel"),
    "conv2_bwd_adam+reduce_adam": (2 * 2 * B * 196 * 64 * 800 / 1e9 + 2 * B * 784 * 32 * 25 / 1e9,
                                   (B * 3136 * 3 + B * 6272 * 3 + B * 784 * 4 + 2 * 25 * 51200 * 4 + PARAMS * 30) / 1e6,
                                   "conv backward + all of Adam (tail + reduce)"),
}
STEP = ["conv12_fwd", "fc1_fwd", "head", "fc1_bwd", "conv2_bwd_adam+reduce_adam"]


def main(path):
    t = {}
    for line in open(path):
        m = re.match(r"^(\S+)\s+([0-9.]+) us", line)
        if m:
            t[m.group(1)] = float(m.group(2))
    print("# Roofline of the fused MNIST step (B = 100, one MI355X)\n")
    print(f"Kernel times: `{path}` (scripts/kbench.py, graph-replayed medians). Peaks: bf16 MFMA "
          f"{PEAK_TFLOPS / 1000:.1f} PFLOP/s dense, HBM3E {PEAK_TBS:.0f} TB/s.\n")
    print("| kernel | work | µs | GFLOP | MB | TFLOP/s | % MFMA peak | TB/s | % HBM peak |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, (gf, mb, what) in WORK.items():
        if name not in t:
            continue
        us = t[name]
        tf = gf / us * 1e3  # GFLOP / us = PFLOP/s
        tbs = mb / us  # MB / us = TB/s
        print(f"| `{name}` | {what} | {us:.2f} | {gf:.3f} | {mb:.1f} | {tf:.0f} | {100 * tf / PEAK_TFLOPS:.1f}% "
              f"| {tbs:.2f} | {100 * tbs / PEAK_TBS:.0f}% |")
    if "step" in t:
        gf = sum(WORK[k][0] for k in STEP)
        mb = sum(WORK[k][1] for k in STEP)
        us = t["step"]
        print(f"| **step** | six launches | {us:.2f} | {gf:.2f} | {mb:.0f} | {gf / us * 1e3:.0f} | "
              f"{100 * gf / us * 1e3 / PEAK_TFLOPS:.1f}% | {mb / us:.2f} | {100 * mb / us / PEAK_TBS:.0f}% |")
        floor = max(gf / PEAK_TFLOPS * 1e3, mb / PEAK_TBS)  # us
        print(f"\nRoofline floor of the step (max of compute and HBM time at peak): {floor:.1f} µs; "
              f"measured {us:.1f} µs ({floor / us * 100:.0f}% of the roof). The optimizer's HBM traffic "
              f"(~{PARAMS * 30 / 1e6:.0f} MB) is the largest single term; the rest of the step is bound by "
              f"launch ramps and dependent-latency chains at B = 100.")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/kbench_latest.txt")
