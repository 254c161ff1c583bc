#!/usr/bin/env python3
"""Per-kernel times of the exact-fp32 step (csrc/kernels/f32_*.hip) at one batch size.

Each kernel of the step is captured alone N times in a HIP graph and replayed, so the figure is the
kernel's own time in a back-to-back stream (no host launch gaps); the whole step is timed the same
way. Prints a table and writes JSON (``--json``).

    python scripts/kbench_f32.py [--batch 100] [--reps 50] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1000.0 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="comma-separated entries: run each --eager times, eagerly "
                    "(for counter collection), and exit")
    ap.add_argument("--eager", type=int, default=20)
    ap.add_argument("--products", type=int, default=6, help="the trainer's fp32 product form (whole-step entry)")
    ap.add_argument("--match", default=None, help="'|'-separated substrings: time only the entries whose name "
                    "contains one of them")
    args = ap.parse_args()

    def want(name):
        return not args.match or any(m in name for m in args.match.split("|"))
    from mihvd.models.fused_mnist import FC_START, FLAT_NUMEL, SEGMENTS, W3_START, FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    B = args.batch
    (x, y), _ = synthetic_mnist(n_train=B * 20, n_test=10, seed=1)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=B, lr=1e-3, seed=0, device="cuda", precision="fp32",
                           f32_products=args.products)
    tr.set_device_dataset(X, Y)
    for _ in range(3):
        tr.device_step()
    torch.cuda.synchronize()
    o, st, P, G = tr.ops, tr.state, tr.pview, tr.gview
    b1, b2 = tr.betas
    s3 = slice(W3_START, FLAT_NUMEL)
    gconv = (G("conv_layer2/conv2d/kernel"), G("conv_layer1/conv2d/kernel"), G("conv_layer1/conv2d/bias"),
             G("conv_layer2/conv2d/bias"))
    w2, w3 = P("conv_layer2/conv2d/kernel"), P("dense/kernel")
    w2frag = torch.empty(2, 51200, device="cuda")
    o.f32_conv1_fwd(tr.X, tr.rows, st, P("conv_layer1/conv2d/kernel"), P("conv_layer1/conv2d/bias"), tr.a1, tr.idx1,
                    w2, w2frag)
    fa8, fz8, fo8 = (torch.randn(8 * B, 392, device="cuda"), torch.randn(8 * B, 1024, device="cuda"),
                     torch.empty(392, 1024, device="cuda"))
    fa1, fz1, fo1 = (torch.randn(B, 3136, device="cuda"), torch.randn(B, 1024, device="cuda"),
                     torch.empty(3136, 1024, device="cuda"))
    fa2, fz2 = torch.randn(2 * B, 3136, device="cuda"), torch.randn(2 * B, 1024, device="cuda")
    fa4, fz4 = torch.randn(4 * B, 3136, device="cuda"), torch.randn(4 * B, 1024, device="cuda")
    fp8, fm8, fv8 = (torch.zeros(392, 1024, device="cuda") for _ in range(3))
    fp1, fm1, fv1 = (torch.zeros(3136, 1024, device="cuda") for _ in range(3))
    slab0 = torch.empty(int(o.f32_wgrad_groups(B, 0)), 51200, device="cuda")
    cpart0 = torch.empty(int(o.f32_dgrad_blocks(B, 0)), 832, device="cuda")
    slab6 = torch.empty(int(o.f32_wgrad_groups(B, 6)), 51200, device="cuda")
    cpart6 = torch.empty(int(o.f32_dgrad_blocks(B, 6)), 832, device="cuda")
    # lr 0 keeps the weights fixed while the optimizer kernels are timed
    ks = {
        "conv1_fwd": lambda: o.f32_conv1_fwd(tr.X, tr.rows, st, P("conv_layer1/conv2d/kernel"),
                                             P("conv_layer1/conv2d/bias"), tr.a1, tr.idx1),
        "conv2_fwd": lambda: o.f32_conv2_fwd(tr.a1, w2, P("conv_layer2/conv2d/bias"), tr.a2, tr.idx2),
        "fc1_fwd": lambda: o.f32_fc1_fwd(tr.a2, w3, tr.zpart),
        "fc1_fwd [split-bf16 x6]": lambda: o.f32_fc1_fwd(tr.a2, w3, tr.zpart, products=6),
        "head": lambda: o.f32_head_fwd_bwd(tr.zpart, P("dense/bias"), P("dense_1/kernel"), P("dense_1/bias"), tr.Y,
                                           tr.rows, st, tr.seed, tr.dropout, tr.h, tr.dz, tr.dlog, tr.stats),
        "fc1_bwd": lambda: o.f32_fc1_bwd(tr.dz, tr.a2, tr.idx2, tr.h, tr.dlog, w3, tr.dY2, tr.db2p, G("dense/kernel"),
                                         G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias")),
        "fc1_bwd+W3 adam": lambda: o.f32_fc1_bwd(tr.dz, tr.a2, tr.idx2, tr.h, tr.dlog, w3, tr.dY2, tr.db2p,
                                                 G("dense/kernel"), G("dense/bias"), G("dense_1/kernel"),
                                                 G("dense_1/bias"), tr.m[s3], tr.v[s3], st, 0.0, b1, b2, tr.eps, 1.0,
                                                 tr.rule, False),
        "conv1_fwd [+ W2 fragment copies]": lambda: o.f32_conv1_fwd(
            tr.X, tr.rows, st, P("conv_layer1/conv2d/kernel"), P("conv_layer1/conv2d/bias"), tr.a1, tr.idx1, w2, w2frag),
        "conv1_fwd [+ W2 fragments, batch gathered ahead]": lambda: o.f32_conv1_fwd(
            tr.X, tr.rows, st, P("conv_layer1/conv2d/kernel"), P("conv_layer1/conv2d/bias"), tr.a1, tr.idx1, w2, w2frag,
            xpre=tr.xpre),
        "head [labels gathered ahead]": lambda: o.f32_head_fwd_bwd(
            tr.zpart, P("dense/bias"), P("dense_1/kernel"), P("dense_1/bias"), tr.Y, tr.rows, st, tr.seed, tr.dropout,
            tr.h, tr.dz, tr.dlog, tr.stats, ypre=tr.ypre),
        "fc1_bwd+W3 adam [+ next batch gathered]": lambda: o.f32_fc1_bwd(
            tr.dz, tr.a2, tr.idx2, tr.h, tr.dlog, w3, tr.dY2, tr.db2p, G("dense/kernel"), G("dense/bias"),
            G("dense_1/kernel"), G("dense_1/bias"), tr.m[s3], tr.v[s3], st, 0.0, b1, b2, tr.eps, 1.0, tr.rule, False,
            px=tr.X, plabels=tr.Y, prows=tr.rows, pstate=st, xpre=tr.xpre, ypre=tr.ypre),
        "conv2_fwd [W2 fragment copy]": lambda: o.f32_conv2_fwd(tr.a1, w2, P("conv_layer2/conv2d/bias"), tr.a2, tr.idx2,
                                                                w2frag=w2frag[0]),
        "conv2_fwd [split-bf16 x9]": lambda: o.f32_conv2_fwd(tr.a1, w2, P("conv_layer2/conv2d/bias"), tr.a2, tr.idx2,
                                                             w2frag=w2frag[0], products=9),
        "conv2_fwd [split-bf16 x6]": lambda: o.f32_conv2_fwd(tr.a1, w2, P("conv_layer2/conv2d/bias"), tr.a2, tr.idx2,
                                                             w2frag=w2frag[0], products=6),
        "conv2_bwd [split-bf16 x6 dgrad]": lambda: o.f32_conv2_bwd(tr.dY2, w2, tr.a1, tr.idx1, tr.X, tr.rows, st, cpart6,
                                                                   slab6, products=6),
        "conv2_bwd [W2 fragment copy]": lambda: o.f32_conv2_bwd(tr.dY2, w2, tr.a1, tr.idx1, tr.X, tr.rows, st, cpart0,
                                                                slab0, w2frag=w2frag[1]),
        "fc1_bwd [dgrad only: fp32 factor plane]": lambda: o.f32_fc1_bwd(
            tr.dz, tr.a2, tr.idx2, tr.h, tr.dlog, w3, tr.dY2, tr.db2p, G("dense/kernel"), G("dense/bias"),
            G("dense_1/kernel"), G("dense_1/bias"), store_w3=False),
        # the factor plane's dW3-row GEMM at N = 8 (392 rows x 800 samples x 1024) and N = 1: the vendor
        # GEMM as a comparison point for the hand-written row kernel (the trainer runs only the latter)
        "factor GEMM N=8 (392x800x1024)": lambda: torch.mm(fa8.t(), fz8, out=fo8),
        "factor GEMM N=1 (3136x100x1024)": lambda: torch.mm(fa1.t(), fz1, out=fo1),
        "factor rows + Adam N=8 (HIP)": lambda: o.f32_factor_rows(fa8, fz8, None, fp8, fm8, fv8, st, 0.0, b1, b2,
                                                                  tr.eps, 0.125, tr.rule),
        "factor rows + Adam N=1 (HIP)": lambda: o.f32_factor_rows(fa1, fz1, None, fp1, fm1, fv1, st, 0.0, b1, b2,
                                                                  tr.eps, 1.0, tr.rule),
        # the replicated factor plane's dW3 (every row, N segments of B samples) + Adam
        "factor full + Adam N=1 (HIP)": lambda: o.f32_factor_full(fa1, fz1, B, None, fp1, fm1, fv1, st, 0.0, b1, b2,
                                                                  tr.eps, 1.0, tr.rule),
        "factor full + Adam N=2 (HIP)": lambda: o.f32_factor_full(fa2, fz2, B, None, fp1, fm1, fv1, st, 0.0, b1, b2,
                                                                  tr.eps, 0.5, tr.rule),
        "factor full + Adam N=4 (HIP)": lambda: o.f32_factor_full(fa4, fz4, B, None, fp1, fm1, fv1, st, 0.0, b1, b2,
                                                                  tr.eps, 0.25, tr.rule),
        "conv2_bwd": lambda: o.f32_conv2_bwd(tr.dY2, w2, tr.a1, tr.idx1, tr.X, tr.rows, st, cpart0, slab0),
        "conv_reduce": lambda: o.f32_conv_reduce(tr.slab, tr.cpart, tr.db2p, *gconv),
        "conv_reduce+adam": lambda: o.f32_conv_reduce(
            tr.slab, tr.cpart, tr.db2p, *gconv, tr.params, tr.grads, tr.m, tr.v, st,
            SEGMENTS["conv_layer1/conv2d/kernel"][0], SEGMENTS["conv_layer1/conv2d/bias"][0],
            SEGMENTS["conv_layer2/conv2d/kernel"][0], SEGMENTS["conv_layer2/conv2d/bias"][0], FC_START, W3_START, 0.0,
            b1, b2, tr.eps, 1.0, tr.rule),
        "adam_step (all)": lambda: o.adam_step(tr.params, tr.grads, tr.m, tr.v, None, st, 0, 0.0, b1, b2, tr.eps, 1.0,
                                               tr.rule, 0),
        "adam_step (W3)": lambda: o.adam_step(tr.params[s3], tr.grads[s3], tr.m[s3], tr.v[s3], None, st, 0, 0.0, b1,
                                              b2, tr.eps, 1.0, tr.rule, 0),
    }
    if args.only:
        for name in args.only.split(","):
            for _ in range(args.eager):
                ks[name]()
            torch.cuda.synchronize()
        return
    res = {}
    for name, fn in ks.items():
        if want(name):
            res[name] = timed(fn, args.reps)
    saved = tr.lr
    tr.lr = 0.0
    if want("whole step (graph, 20 steps/replay)"):
        res["whole step (graph, 20 steps/replay)"] = timed(lambda: tr._launch_step(tr.X, tr.rows, tr.Y), 20)
        tr._join()
    tr.lr = saved
    width = max(len(k) for k in res)
    for k, v in res.items():
        print(f"{k:<{width}}  {v:8.2f} us")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"batch": B, "us": res, "device": torch.cuda.get_device_name()}, f, indent=1)


if __name__ == "__main__":
    main()
