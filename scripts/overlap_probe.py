#!/usr/bin/env python3
"""Concurrency probe: can the memory-bound dense/kernel Adam update run *beside* the compute-bound
conv backward instead of in its launch tail? Times (graph-replayed, events) the two kernels
alone, back to back on one stream, forked onto two streams inside one HIP graph (Adam grid
capped at several sizes), the fused tail launch, and the bare cost of a fork/join in a graph.
Usage: python scripts/overlap_probe.py [--iters 100]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    args = ap.parse_args()
    from mihvd.models.fused_mnist import FC_START as FC, W3_START as W3, FusedMNISTTrainer

    B = 100
    tr = FusedMNISTTrainer(batch_size=B, seed=0, device="cuda", precision="bf16")
    x = torch.rand(B, 784, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    tr.train_step(x, y)
    torch.cuda.synchronize()
    o, st, sh = tr.ops, tr.state, tr.shadow
    w2 = tr.pview("conv_layer2/conv2d/kernel", sh)

    def conv():
        o.conv2_bwd(tr.g2, tr.idx2, tr.a1, w2, tr.x_buf, None, st, tr.idx1, tr.slab, tr.cpart)

    def reduce_adam():
        o.conv2_wgrad_reduce_adam(tr.slab, tr.cpart, B, tr.gview("conv_layer2/conv2d/kernel"),
                                  tr.gview("conv_layer1/conv2d/kernel"), tr.gview("conv_layer1/conv2d/bias"),
                                  tr.gview("conv_layer2/conv2d/bias"), tr.grads, tr.params, tr.m, tr.v, sh, st, FC, W3,
                                  0.0, 0.9, 0.999, 1e-8, 1.0, 0)

    def adam(blocks=0):
        o.adam_step(tr.params[W3:], tr.grads[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], st, 0, 0.0, 0.9, 0.999, 1e-8, 1.0,
                    0, 0, None, blocks)

    def tail():
        o.conv2_bwd_adam(tr.g2, tr.idx2, tr.a1, w2, tr.x_buf, None, st, tr.idx1, tr.slab, tr.cpart, tr.params[W3:],
                         tr.grads[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], 0.0, 0.9, 0.999, 1e-8, 1.0, 0)

    side = torch.cuda.Stream()

    def forked(blocks, with_reduce=False, tiny=False):
        def fn():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if tiny:
                    st[3:4].add_(0)
                else:
                    adam(blocks)
            if tiny:
                st[2:3].add_(0)
            else:
                conv()
                if with_reduce:
                    reduce_adam()
            main.wait_stream(side)
        return fn

    jobs = {
        "conv2_bwd": conv,
        "adam_w3": lambda: adam(0),
        "adam_w3[512 blk]": lambda: adam(512),
        "serial conv2_bwd; adam_w3": lambda: (conv(), adam(0)),
        "tail conv2_bwd_adam": tail,
        "tail conv2_bwd_adam + reduce_adam": lambda: (tail(), reduce_adam()),
        "serial conv2_bwd; reduce_adam; adam_w3": lambda: (conv(), reduce_adam(), adam(0)),
        "tiny kernel": lambda: st[2:3].add_(0),
        "fork/join of two tiny kernels": forked(0, tiny=True),
    }
    for blocks in (0, 256, 512, 1024):
        jobs[f"fork conv2_bwd | adam_w3[{blocks or 'all'}]"] = forked(blocks)
        jobs[f"fork conv2_bwd+reduce_adam | adam_w3[{blocks or 'all'}]"] = forked(blocks, with_reduce=True)

    def streams(n, blocks, main_fn):
        # one fork/join around n kernels per stream: the concurrent throughput without the fork cost
        def fn():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for _ in range(n):
                    adam(blocks)
            for _ in range(n):
                main_fn()
            main.wait_stream(side)
        return fn

    conv12 = lambda: o.conv12_fwd(tr.x_buf, None, st, tr.pview("conv_layer1/conv2d/kernel", sh),  # noqa: E731
                                  tr.pview("conv_layer1/conv2d/bias"), w2, tr.pview("conv_layer2/conv2d/bias"), tr.a1,
                                  tr.idx1, tr.a2, tr.idx2)
    jobs["conv12_fwd"] = conv12
    jobs["conv2_bwd; reduce_adam; conv12_fwd"] = lambda: (conv(), reduce_adam(), conv12())
    for blocks in (128, 256, 512, 2048):
        jobs[f"20x[conv2_bwd] | 20x[adam_w3[{blocks}]] /20"] = streams(20, blocks, conv)
        jobs[f"20x[conv2_bwd;reduce;conv12] | 20x[adam_w3[{blocks}]] /20"] = streams(
            20, blocks, lambda: (conv(), reduce_adam(), conv12()))

    def tiny_streams():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for _ in range(20):
                st[3:4].add_(0)
        for _ in range(20):
            st[2:3].add_(0)
        main.wait_stream(side)
    jobs["20x[tiny] | 20x[tiny] /20"] = tiny_streams
    div = {k: (20 if k.startswith("20x") else 1) for k in jobs}
    s = torch.cuda.Stream()
    only = os.environ.get("PROBE_ONLY")
    for name, fn in jobs.items():
        if only and only not in name:
            continue
        iters = max(1, args.iters // div[name])
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / (3 * iters * div[name])
        print(f"{name:56s} {us:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
