#!/usr/bin/env python3
"""Data-parallel stress benchmarks of BASELINE.json's stretch configurations:

  * ResNet-50 synthetic ImageNet, bf16 autocast (25.6 M params: allreduce bandwidth stress)
  * BERT-base MLM, synthetic seq=512, bf16 autocast, fp16 allreduce compression (110 M params:
    large-gradient fusion + compression stress)

    python benchmarks/stress_models.py --model resnet50 [--batch-size 128] [--steps 30 --warmup 10]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        benchmarks/stress_models.py --model bert-base --compression fp16

Compute is stock PyTorch-ROCm (MIOpen / hipBLASLt) — these configs exercise mihvd's DP engine:
``DistributedOptimizer`` fusion buckets whose RCCL allreduces are issued from gradient hooks while
backward is still running, in-order release, optional compression. Timing follows bench.py (barrier +
synchronize on both sides, max over ranks); rank 0 prints one JSON line with whole-job throughput.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["resnet50", "bert-base"], default="resnet50")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=0, help="per GPU (default: 128 images / 16 sequences)")
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--compression", choices=["none", "fp16", "bf16"], default="")
    ap.add_argument("--fusion-mib", type=float, default=0, help="fusion threshold (0 = engine default)")
    ap.add_argument("--optimizer", choices=["torch", "fused"], default="fused",
                    help="fused: mihvd multi-tensor HIP optimizer (FusedSGD / FusedAdam(adamw))")
    ap.add_argument("--graph", action="store_true", help="capture the whole step in one HIP graph")
    ap.add_argument("--no-dp", action="store_true",
                    help="plain optimizer without mihvd's DistributedOptimizer (world size 1: engine overhead)")
    ap.add_argument("--mlm-all-positions", action="store_true",
                    help="bert-base: MLM head on every position (default: the masked positions only)")
    return ap.parse_args()


def main():
    args = parse()
    import mihvd.torch as hvd

    hvd.init()
    dev = hvd.device()
    n = hvd.size()
    comp_name = args.compression or ("fp16" if args.model == "bert-base" else "none")
    comp = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16, "bf16": hvd.Compression.bf16}[comp_name]
    g = torch.Generator(device=dev).manual_seed(1234 + hvd.rank())
    # autocast's weight-cast cache stays off for captured steps (PyTorch's CUDA-graph guidance)
    cache = not args.graph if os.environ.get("MIHVD_STRESS_AUTOCAST_CACHE") is None else \
        os.environ["MIHVD_STRESS_AUTOCAST_CACHE"] == "1"
    if args.model == "resnet50":
        from mihvd.models.resnet import ResNet50, num_params

        B = args.batch_size or 128
        model = ResNet50().to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(B, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev, generator=g)
        if args.optimizer == "fused":
            from mihvd.optim import FusedSGD

            base = FusedSGD(model.parameters(), lr=0.1 * n, momentum=0.9, weight_decay=5e-5)
        else:
            base = torch.optim.SGD(model.parameters(), lr=0.1 * n, momentum=0.9, weight_decay=5e-5)

        def loss_fn():
            with torch.autocast(dev.type, dtype=torch.bfloat16, cache_enabled=cache):
                return torch.nn.functional.cross_entropy(model(x), y)
        unit, per_sample = "images/sec", 1
        metric = "images/sec (whole node) ResNet-50 synthetic ImageNet bf16"
        cfg = {"model": "ResNet-50 v1.5", "global_batch": B * n, "seq_len": None, "image_shape": [224, 224, 3]}
    else:
        from mihvd.models.bert import BertConfig, BertForMaskedLM, synthetic_mlm_batch

        B = args.batch_size or 16
        c = BertConfig(max_len=max(512, args.seq_len), attn_impl=os.environ.get("MIHVD_BERT_ATTN", "sdpa"),
                       embedding_impl=os.environ.get("MIHVD_BERT_EMBEDDING", "gather"))
        model = BertForMaskedLM(c).to(dev)
        ids, labels = synthetic_mlm_batch(B, args.seq_len, c.vocab_size, dev, generator=g)
        from mihvd.models.bert import masked_positions

        mpos = None if args.mlm_all_positions else masked_positions(labels)
        if args.optimizer == "fused":
            from mihvd.optim import FusedAdam

            base = FusedAdam(model.parameters(), lr=1e-4 * n, weight_decay=0.01, adamw=True)
        else:
            base = torch.optim.AdamW(model.parameters(), lr=1e-4 * n, weight_decay=0.01,
                                     **({"capturable": True} if args.graph else {}))

        def loss_fn():
            with torch.autocast(dev.type, dtype=torch.bfloat16, cache_enabled=cache):
                return model(ids, labels, masked_positions=mpos)
        unit, per_sample = "tokens/sec", args.seq_len
        metric = "tokens/sec (whole node) BERT-base MLM synthetic seq=%d bf16" % args.seq_len
        cfg = {"model": "BERT-base (12x768, 110M)", "global_batch": B * n, "seq_len": args.seq_len}
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    if args.no_dp:
        if n > 1:
            raise SystemExit("--no-dp is a world-size-1 measurement")
        opt = base
        opt.buckets = []
    else:
        opt = hvd.DistributedOptimizer(base, named_parameters=model.named_parameters(), compression=comp,
                                       fusion_threshold=int(args.fusion_mib * 2 ** 20) if args.fusion_mib else None)

    def step():
        opt.zero_grad(set_to_none=False)
        loss = loss_fn()
        loss.backward()
        opt.step()
        return loss

    if args.graph:
        from mihvd.graphs import CapturedStep

        step = CapturedStep(step, warmup=max(3, args.warmup))
    for _ in range(args.warmup):
        step()
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    sync()
    hvd.barrier()
    sync()
    t0 = time.perf_counter()
    trace = [] if os.environ.get("MIHVD_STRESS_TRACE") else None
    each = os.environ.get("MIHVD_STRESS_SYNC_EACH") == "1"
    for _ in range(args.steps):
        loss = step()
        if each:
            sync()
        if trace is not None:
            st = [loss.detach().float().reshape(1)]
            if not args.no_dp:  # after the step: the buckets hold the (wire round-tripped) gradients
                fl = [b.flat for b in opt._buckets]
                st += [sum((~f.isfinite()).sum() for f in fl).float().reshape(1),
                       torch.stack([f.nan_to_num(0, 0, 0).abs().max() for f in fl]).max().reshape(1),
                       sum((~p.isfinite()).sum() for p in model.parameters()).float().reshape(1)]
            trace.append(torch.cat(st))
    sync()
    hvd.barrier()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if n > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el)
    if trace is not None:
        print("per-step loss / non-finite grads / max|grad| / non-finite params:",
              " ".join("/".join("%.4g" % x for x in v.tolist()) for v in trace), flush=True)
    if hvd.rank() == 0:
        params = sum(p.numel() for p in model.parameters())
        cfg.update({"parallelism": f"dp{n}", "per_gpu_batch": B, "params": params,
                    "grad_bytes_fp32": params * 4, "buckets": len(opt.buckets), "compression": comp_name,
                    "optimizer": args.optimizer, "hip_graph": bool(args.graph), "final_loss": float(loss),
                    "distributed_optimizer": not args.no_dp})
        if args.model == "bert-base":
            cfg["mlm_head"] = "all positions" if args.mlm_all_positions else "masked positions"
        print(json.dumps({"metric": metric, "value": round(args.steps * B * per_sample * n / el, 1), "unit": unit,
                          "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
                          "config": cfg}), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
