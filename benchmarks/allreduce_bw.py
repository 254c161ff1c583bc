#!/usr/bin/env python3
"""RCCL collective bandwidth sweep (SURVEY.md §7.1 "allreduce_bw"): allreduce, all-gather and
reduce-scatter of 4 KB .. 256 MB through ``torch.distributed`` (RCCL over xGMI), eager and
HIP-graph-captured, reporting algorithm and bus bandwidth like rccl-tests. Sizes that matter for
the MNIST data plane are marked: 13.1 MB (the fp32 gradient allreduce) and 0.63 / 0.2 MB per rank
(the bf16 factor all-gathers).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/allreduce_bw.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, iters, graph):
    if graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        run = g.replay
    else:
        def run():
            for _ in range(iters):
                fn()
    run()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--max-mib", type=float, default=256)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    import mihvd.torch as hvd

    hvd.init()
    n, dev = hvd.size(), hvd.device()
    sizes = []
    s = 4096
    while s <= args.max_mib * 2 ** 20:
        sizes.append(s)
        s *= 4
    sizes += [13_098_536, 627_200, 204_800]
    rows = []
    for nbytes in sorted(set(sizes)):
        numel = max(n, nbytes // 4 // n * n)
        x = torch.ones(numel, device=dev)
        shard = torch.empty(numel // n, device=dev)
        res = {"bytes": numel * 4}
        t = timed(lambda: dist.all_reduce(x), args.iters, args.graph)
        res["allreduce_us"] = t * 1e6
        res["allreduce_busbw_GBs"] = numel * 4 / t * 2 * (n - 1) / n / 1e9 if n > 1 else None
        t = timed(lambda: dist.all_gather_into_tensor(x, shard), args.iters, args.graph)
        res["allgather_us"] = t * 1e6
        res["allgather_busbw_GBs"] = numel * 4 / t * (n - 1) / n / 1e9 if n > 1 else None
        t = timed(lambda: dist.reduce_scatter_tensor(shard, x), args.iters, args.graph)
        res["reducescatter_us"] = t * 1e6
        res["reducescatter_busbw_GBs"] = numel * 4 / t * (n - 1) / n / 1e9 if n > 1 else None
        rows.append(res)
        if hvd.rank() == 0:
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
