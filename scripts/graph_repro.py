#!/usr/bin/env python3
"""Bisect the BERT-base HIP-graph NaN (docs/ARCHITECTURE.md, "Generic models") down to stock
PyTorch-ROCm ops, with no mihvd code on the path.

Each variant trains a small model K steps eagerly and K steps as replays of one captured step
(torch.cuda.graph, AdamW(capturable=True), bf16 autocast like benchmarks/stress_models.py), from the
same initial weights on the same fixed batch, and reports the loss curves and whether the graph
run produced non-finite values or diverged from the eager one.

    python scripts/graph_repro.py [--steps 6] [--variants emb,emb_tied,...]
"""
from __future__ import annotations

import argparse
import json
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

V, H, S, B = 30522, 256, 128, 8


class Emb(nn.Module):
    """Embedding lookup + linear head (embedding backward: sort/segment kernels)."""

    def __init__(self, tied=False):
        super().__init__()
        self.tok = nn.Embedding(V, H)
        self.lin = nn.Linear(H, H)
        self.tied = tied
        if not tied:
            self.out = nn.Linear(H, V)

    def forward(self, ids, labels):
        x = torch.tanh(self.lin(self.tok(ids)))
        logits = x @ self.tok.weight.t() if self.tied else self.out(x)
        return F.cross_entropy(logits.float().view(-1, V), labels.view(-1), ignore_index=-100)


class LnGelu(nn.Module):
    def __init__(self):
        super().__init__()
        self.tok = nn.Embedding(V, H)
        self.l1, self.l2 = nn.Linear(H, 4 * H), nn.Linear(4 * H, H)
        self.ln = nn.LayerNorm(H, eps=1e-12)
        self.out = nn.Linear(H, 16)

    def forward(self, ids, labels):
        x = self.tok(ids)
        x = self.ln(x + self.l2(F.gelu(self.l1(x))))
        return F.cross_entropy(self.out(x).float().view(-1, 16), labels.view(-1) % 16)


class Attn(nn.Module):
    def __init__(self, sdpa=True, dropout=0.0):
        super().__init__()
        self.tok = nn.Embedding(V, H)
        self.qkv, self.proj = nn.Linear(H, 3 * H), nn.Linear(H, H)
        self.out = nn.Linear(H, 16)
        self.sdpa, self.p = sdpa, dropout

    def forward(self, ids, labels):
        x = self.tok(ids)
        q, k, v = self.qkv(x).view(B, S, 3, 4, H // 4).permute(2, 0, 3, 1, 4)
        if self.sdpa:
            a = F.scaled_dot_product_attention(q, k, v, dropout_p=self.p if self.training else 0.0)
        else:
            a = F.dropout((q @ k.transpose(-2, -1) / math.sqrt(H // 4)).softmax(-1), self.p, self.training) @ v
        x = x + self.proj(a.transpose(1, 2).reshape(B, S, H))
        return F.cross_entropy(self.out(x).float().view(-1, 16), labels.view(-1) % 16)


class Dropout(nn.Module):
    """Dropout's Philox offsets advance per replay through the graph-safe generator state."""

    def __init__(self):
        super().__init__()
        self.tok = nn.Embedding(V, H)
        self.out = nn.Linear(H, 16)

    def forward(self, ids, labels):
        return F.cross_entropy(self.out(F.dropout(self.tok(ids), 0.1, self.training)).float().view(-1, 16),
                               labels.view(-1) % 16)


def bert_tiny():
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mihvd.models.bert import BertConfig, BertForMaskedLM  # stock torch ops only

    class W(nn.Module):
        def __init__(self):
            super().__init__()
            self.m = BertForMaskedLM(BertConfig(hidden=H, layers=2, heads=4, ffn=4 * H, max_len=S))

        def forward(self, ids, labels):
            return self.m(ids, labels)

    return W()


def bert_base(mpos=False):
    """The stress config's model (BERT-base 12x768) at this script's B and S; mpos: the MLM head on
    the masked positions only, index list computed outside the capture (as benchmarks/stress_models.py)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mihvd.models.bert import BertConfig, BertForMaskedLM, masked_positions

    class W(nn.Module):
        def __init__(self):
            super().__init__()
            self.m = BertForMaskedLM(BertConfig(max_len=512))
            self.mp = None

        def forward(self, ids, labels):
            if mpos and self.mp is None:
                self.mp = masked_positions(labels)
            return self.m(ids, labels, masked_positions=self.mp if mpos else None)

    return W()


VARIANTS = {
    "emb": lambda: Emb(False), "emb_tied": lambda: Emb(True), "ln_gelu": LnGelu, "sdpa": lambda: Attn(True),
    "math_attn": lambda: Attn(False), "sdpa_dropout": lambda: Attn(True, 0.1), "dropout": Dropout,
    "bert_tiny": bert_tiny, "bert_base": lambda: bert_base(False), "bert_base_mpos": lambda: bert_base(True),
}


OPTS = {"lr": 1e-3, "wd": 0.0, "captured_step": False}


def run(name, steps, graph, dropout_eval=False, sync_each=True):
    torch.manual_seed(0)
    model = VARIANTS[name]().cuda()
    if dropout_eval:
        model.eval()
    opt = torch.optim.AdamW(model.parameters(), lr=OPTS["lr"], weight_decay=OPTS["wd"], capturable=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(0, V, (B, S), device="cuda", generator=g)
    labels = torch.where(torch.rand(B, S, device="cuda", generator=g) < 0.15, ids, torch.full_like(ids, -100))
    labels[0, 0] = ids[0, 0]  # at least one label

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = model(ids, labels)
        loss.backward()
        opt.step()
        return loss

    losses = []
    if not graph:
        for _ in range(steps):
            losses.append(float(step()))
        return losses, model
    if OPTS["captured_step"]:  # mihvd.graphs.CapturedStep (the stress bench's capture path)
        import os
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mihvd.graphs import CapturedStep

        cs = CapturedStep(step, warmup=3)
        losses += [None] * 3  # its warm-up losses are not returned
        outs = [cs().clone() for _ in range(steps - 3)]
        losses += [float(o) for o in outs]
        return losses, model
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):  # warm-up (also creates the optimizer state)
            losses.append(float(step()))
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = step()
    if sync_each:
        for _ in range(steps - 3):
            gr.replay()
            losses.append(float(out))
        return losses, model
    # back-to-back replays (the stress bench's pattern): each loss is cloned on the stream behind
    # its replay, read only at the end
    outs = []
    for _ in range(steps - 3):
        gr.replay()
        outs.append(out.detach().clone())
    losses += [float(o) for o in outs]
    return losses, model


def main():
    global B, S
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--batch", type=int, default=B)
    ap.add_argument("--seq", type=int, default=S)
    ap.add_argument("--no-sync", action="store_true", help="replays back to back, losses read at the end")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--wd", type=float, default=0.0)
    ap.add_argument("--captured-step", action="store_true", help="capture with mihvd.graphs.CapturedStep")
    ap.add_argument("--hvd-init", action="store_true", help="mihvd.init() first (health monitor, observability)")
    args = ap.parse_args()
    OPTS.update(lr=args.lr, wd=args.wd, captured_step=args.captured_step)
    if args.hvd_init:
        import os
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import mihvd

        mihvd.init()
    B, S = args.batch, args.seq
    res = {}
    for name in args.variants.split(","):
        le, me = run(name, args.steps, graph=False)
        lg, mg = run(name, args.steps, graph=True, sync_each=not args.no_sync)
        finite = all(math.isfinite(v) for v in lg if v is not None) and all(torch.isfinite(p).all() for p in mg.parameters())
        pd = max(((a - b).norm() / (b.norm() + 1e-12)).item() for a, b in zip(mg.parameters(), me.parameters()))
        rel = max(abs(a - b) / max(abs(b), 1e-6) for a, b in zip(lg, le) if a is not None)
        res[name] = {"finite": finite, "loss_rel_diff": rel, "param_rel_diff": pd, "eager": le, "graph": lg}
        print(json.dumps({name: {k: v for k, v in res[name].items() if k not in ("eager", "graph")}}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
