#!/usr/bin/env python3
"""Collective bandwidth benchmark (RCCL over xGMI on MI355X; gloo on CPU for plumbing).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29600 scripts/allreduce_bw.py [--ops allreduce,allgather,reduce_scatter,broadcast]
        [--sizes 4K,64K,1M,13M,64M,256M] [--dtype bf16|fp32] [--graph] [--engine] [--xgmi]

Per op and message size: time per call (median over --iters after --warmup), algorithm bandwidth
(bytes / time) and bus bandwidth (the nccl-tests convention: allreduce x 2(n-1)/n, allgather and
reduce-scatter x (n-1)/n, broadcast x 1), the numbers that decide bucket sizes on a point-to-point
xGMI mesh (13.1 MB is the MNIST gradient bucket). --graph replays the calls from a
HIP graph (how the fused trainer issues them); --engine also times mihvd's allreduce entry point
(hvd.allreduce: negotiation/fusion bookkeeping + the same RCCL call); --xgmi also times the direct
xGMI one-shot allreduce (mihvd.parallel.xgmi, fp32 sizes). Rank 0 prints one JSON line
per (op, size) and a table.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

UNITS = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}


def parse_size(s: str) -> int:
    s = s.strip().upper()
    return int(float(s[:-1]) * UNITS[s[-1]]) if s[-1] in UNITS else int(s)


def bus_factor(op: str, n: int) -> float:
    if n == 1:
        return 1.0
    return {"allreduce": 2 * (n - 1) / n, "allgather": (n - 1) / n, "reduce_scatter": (n - 1) / n}.get(op, 1.0)


def make_call(op, buf, out, world):
    if op == "allreduce":
        return lambda: dist.all_reduce(buf)
    if op == "allgather":
        return lambda: dist.all_gather_into_tensor(out, buf)
    if op == "reduce_scatter":
        return lambda: dist.reduce_scatter_tensor(buf, out)
    if op == "broadcast":
        return lambda: dist.broadcast(buf, src=0)
    raise ValueError(op)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="allreduce,allgather,reduce_scatter,broadcast")
    ap.add_argument("--sizes", default="4K,64K,1M,4M,13M,64M,256M", help="bytes per rank (input)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", action="store_true", help="replay the calls from a HIP graph")
    ap.add_argument("--engine", action="store_true", help="also time hvd.allreduce (mihvd entry point)")
    ap.add_argument("--xgmi", action="store_true",
                    help="also time the direct xGMI one-shot allreduce (mihvd.parallel.xgmi, fp32)")
    args = ap.parse_args()

    import mihvd.torch as hvd

    hvd.init()
    world, rank, dev = hvd.size(), hvd.rank(), hvd.device()
    dtype = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    esize = torch.tensor([], dtype=dtype).element_size()
    on_gpu = dev.type == "cuda"
    sync = (lambda: torch.cuda.synchronize(dev)) if on_gpu else (lambda: None)
    rows = []
    xgmi = None
    if args.xgmi and on_gpu and world > 1:
        from mihvd.parallel.xgmi import XGMIAllreduce

        cap = max(parse_size(sz) for sz in args.sizes.split(",")) // 4 + world
        xgmi = XGMIAllreduce(cap)
    for op in args.ops.split(","):
        for sz in args.sizes.split(","):
            nbytes = parse_size(sz)
            n = max(world, nbytes // esize // world * world)
            buf = torch.ones(n, dtype=dtype, device=dev)
            out = None
            if op == "allgather":
                out = torch.empty(n * world, dtype=dtype, device=dev)
            elif op == "reduce_scatter":
                out = torch.empty(n // world, dtype=dtype, device=dev)
            call = make_call(op, buf, out, world)
            try:
                call()
            except (RuntimeError, NotImplementedError) as e:  # e.g. gloo has no reduce_scatter_tensor
                if rank == 0:
                    print(json.dumps({"op": op, "bytes": n * esize, "unsupported": str(e).splitlines()[0][:120]}))
                break
            for _ in range(args.warmup):
                call()
            sync()
            times = []
            if args.graph and on_gpu:
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                    call()
                torch.cuda.current_stream(dev).wait_stream(s)
                call = g.replay
                call()
                sync()
            for _ in range(args.iters):
                dist.barrier()
                sync()
                t0 = time.perf_counter()
                call()
                sync()
                times.append(time.perf_counter() - t0)
            t = torch.tensor([statistics.median(times)], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            sec = float(t.item())
            row = {"op": op, "bytes": n * esize, "world": world, "dtype": args.dtype, "graph": bool(args.graph and on_gpu),
                   "us": sec * 1e6, "algbw_GBs": n * esize / sec / 1e9,
                   "busbw_GBs": n * esize / sec / 1e9 * bus_factor(op, world), "backend": dist.get_backend()}
            rows.append(row)
            if args.engine and op == "allreduce":
                for _ in range(args.warmup):
                    hvd.allreduce(buf, op=hvd.Sum, name=f"bw.{n}")
                sync()
                et = []
                for _ in range(args.iters):
                    dist.barrier()
                    sync()
                    t0 = time.perf_counter()
                    hvd.allreduce(buf, op=hvd.Sum, name=f"bw.{n}")
                    sync()
                    et.append(time.perf_counter() - t0)
                t = torch.tensor([statistics.median(et)], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                rows.append(dict(row, op="hvd.allreduce", us=float(t.item()) * 1e6,
                                 algbw_GBs=n * esize / float(t.item()) / 1e9,
                                 busbw_GBs=n * esize / float(t.item()) / 1e9 * bus_factor("allreduce", world)))
            if xgmi is not None and op == "allreduce" and dtype == torch.float32 and n <= xgmi.capacity:
                xcall = lambda: xgmi.allreduce_(buf)  # noqa: E731
                for _ in range(args.warmup):
                    xcall()
                sync()
                xgmi.check()
                if args.graph:
                    g = torch.cuda.CUDAGraph()
                    s = torch.cuda.Stream(device=dev)
                    s.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                        xcall()
                    torch.cuda.current_stream(dev).wait_stream(s)
                    xcall = g.replay
                xt = []
                for _ in range(args.iters):
                    dist.barrier()
                    sync()
                    t0 = time.perf_counter()
                    xcall()
                    sync()
                    xt.append(time.perf_counter() - t0)
                xgmi.check()
                t = torch.tensor([statistics.median(xt)], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                xs = float(t.item())
                rows.append(dict(row, op="xgmi_oneshot", us=xs * 1e6, algbw_GBs=n * esize / xs / 1e9,
                                 busbw_GBs=n * esize / xs / 1e9 * bus_factor("allreduce", world)))
    if xgmi is not None:
        xgmi.close()
    if rank == 0:
        for r in rows:
            print(json.dumps(r))
        print(f"{'op':16s} {'bytes':>12s} {'us':>10s} {'algbw GB/s':>11s} {'busbw GB/s':>11s}", file=sys.stderr)
        for r in rows:
            print(f"{r['op']:16s} {r['bytes']:12d} {r['us']:10.1f} {r['algbw_GBs']:11.2f} {r['busbw_GBs']:11.2f}",
                  file=sys.stderr)
    hvd.shutdown()


if __name__ == "__main__":
    main()
