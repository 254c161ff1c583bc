#!/usr/bin/env python3
"""Dump the HIP graph of a captured BERT training step (CapturedStep + DistributedOptimizer) as DOT
and report its topology: node count, root and sink nodes (a sink other than the last node is a
branch that the next replay is ordered after only through the graph launch itself)."""
import collections
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(layers=2, comp="fp16", out="gpurun_out/bert_graph.dot"):
    import mihvd.torch as hvd
    from mihvd.graphs import CapturedStep
    from mihvd.models.bert import BertConfig, BertForMaskedLM, masked_positions, synthetic_mlm_batch
    from mihvd.optim import FusedAdam

    hvd.init()
    dev = hvd.device()
    g = torch.Generator(device=dev).manual_seed(1234)
    c = BertConfig(max_len=512, layers=layers)
    model = BertForMaskedLM(c).to(dev)
    ids, labels = synthetic_mlm_batch(4, 128, c.vocab_size, dev, generator=g)
    mpos = masked_positions(labels)
    C = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16, "bf16": hvd.Compression.bf16}[comp]
    opt = hvd.DistributedOptimizer(FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01, adamw=True),
                                   named_parameters=model.named_parameters(), compression=C)

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast(dev.type, dtype=torch.bfloat16):
            loss = model(ids, labels, masked_positions=mpos)
        loss.backward()
        opt.step()
        return loss

    torch.cuda.graphs.CUDAGraph.enable_debug_mode = getattr(torch.cuda.graphs.CUDAGraph, "enable_debug_mode", None)
    orig = torch.cuda.CUDAGraph.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.enable_debug_mode()
    torch.cuda.CUDAGraph.__init__ = init
    cs = CapturedStep(step, warmup=3)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cs.graph.debug_dump(out)
    txt = open(out).read()
    nodes = set(re.findall(r'^\s*"?(\w+)"?\s*\[', txt, re.M))
    edges = re.findall(r'"?(\w+)"?\s*->\s*"?(\w+)"?', txt)
    succ = collections.defaultdict(set)
    pred = collections.defaultdict(set)
    for a, b in edges:
        succ[a].add(b)
        pred[b].add(a)
    nodes |= set(succ) | set(pred)
    roots = [n for n in nodes if not pred[n]]
    sinks = [n for n in nodes if not succ[n]]
    print("nodes", len(nodes), "edges", len(edges), "roots", len(roots), "sinks", len(sinks))
    labels = dict(re.findall(r'"?(\w+)"?\s*\[[^\]]*label="([^"]{0,160})', txt))
    for s in sinks[:20]:
        print("sink", s, labels.get(s, "")[:160].replace("\\n", " | "))
    for r in roots[:10]:
        print("root", r, labels.get(r, "")[:160].replace("\\n", " | "))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2, sys.argv[2] if len(sys.argv) > 2 else "fp16")
