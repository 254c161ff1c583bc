#!/usr/bin/env python3
"""Probe: DistributedOptimizer compression inside a CapturedStep vs eager (world size 1).

Runs the same small BERT (or a given stress model) eagerly and graph-replayed with each
compression and prints the loss per step plus the largest |gradient| of every step, so a
graph-only divergence (vs a real fp16 overflow) is visible."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(comp_name, graph, steps=8, layers=2, B=4, S=128):
    import mihvd.torch as hvd
    from mihvd.graphs import CapturedStep
    from mihvd.models.bert import BertConfig, BertForMaskedLM, masked_positions, synthetic_mlm_batch
    from mihvd.optim import FusedAdam

    hvd.init()
    dev = hvd.device()
    if os.environ.get("PROBE_SEED", "1") == "1":
        torch.manual_seed(0)
    g = torch.Generator(device=dev).manual_seed(1234)
    c = BertConfig(max_len=512, layers=layers,
                   attn_dropout=float(os.environ["PROBE_ATTN_P"]) if os.environ.get("PROBE_ATTN_P") else None)
    model = BertForMaskedLM(c).to(dev)
    ids, labels = synthetic_mlm_batch(B, S, c.vocab_size, dev, generator=g)
    mpos = masked_positions(labels)
    if os.environ.get("PROBE_BCAST", "0") == "1":
        hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    comp = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16, "bf16": hvd.Compression.bf16}[comp_name]
    opt = hvd.DistributedOptimizer(FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01, adamw=True),
                                   named_parameters=model.named_parameters(), compression=comp)
    gmax = torch.zeros((), device=dev)

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast(dev.type, dtype=torch.bfloat16):
            loss = model(ids, labels, masked_positions=mpos)
        loss.backward()
        if os.environ.get("PROBE_GMAX", "1") == "1":
            gmax.copy_(torch.stack([b.flat.abs().max() for b in opt._buckets]).max())
        opt.step()
        return loss

    if os.environ.get("PROBE_STREAMS"):  # which stream do the bucket packs run on during capture?
        import mihvd.parallel.compression as cm
        import mihvd.parallel.collectives as cl
        orig = cm.hip_pack

        def traced(*a, **k):
            s = torch.cuda.current_stream()
            print("pack on stream %#x capturing=%s thread=%s" % (s.cuda_stream, torch.cuda.is_current_stream_capturing(),
                                                                  __import__("threading").current_thread().name))
            return orig(*a, **k)
        cl.hip_pack = traced
        orig_sync = opt.synchronize

        def sync_traced():
            s = torch.cuda.current_stream()
            print("synchronize on stream %#x capturing=%s" % (s.cuda_stream, torch.cuda.is_current_stream_capturing()))
            return orig_sync()
        opt.synchronize = sync_traced
    f = CapturedStep(step, warmup=3) if graph else step
    out = []
    if os.environ.get("PROBE_DEVSYNC"):  # the stress bench's order: k replays, device sync, replays
        k = int(os.environ["PROBE_DEVSYNC"])
        for _ in range(k):
            f()
        torch.cuda.synchronize()
        for i in range(steps):
            l = f()
            st = opt.state[next(iter(model.parameters()))]
            bad = {"params": sum(int(p.isnan().sum()) for p in model.parameters()),
                   "buckets": sum(int(b.flat.isnan().sum()) for b in opt._buckets),
                   "m": sum(int(opt.state[p]["exp_avg"].isnan().sum()) for p in model.parameters()),
                   "v": sum(int(opt.state[p]["exp_avg_sq"].isnan().sum()) for p in model.parameters())}
            out.append("%.4f%s" % (float(l), "" if not any(bad.values()) else str(bad)))
    if os.environ.get("PROBE_NOSYNC", "0") == "1":  # replays queued back to back, read at the end
        ls = [(f().detach().clone(), gmax.clone()) for _ in range(steps)]
        out = ["%.4f/%.3g" % (float(l), float(m)) for l, m in ls]
    for _ in range(0 if out else steps):
        l = f()
        out.append("%.4f/%.3g" % (float(l), float(gmax)))
    print(comp_name, "graph" if graph else "eager", "buckets=%d" % len(opt.buckets), file=sys.stdout)
    print(comp_name, "graph" if graph else "eager", " ".join(out), flush=True)


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[3:]]
    run(sys.argv[1], sys.argv[2] == "graph", *a)
