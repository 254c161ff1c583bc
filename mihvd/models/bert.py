"""BERT-base encoder + masked-LM head for the "BERT-base synthetic seq=512 on 8×MI355X (large-grad
fusion + fp16 allreduce compression)" stretch configuration of BASELINE.json: 110 M parameters,
440 MB of fp32 gradients per step, one embedding matrix of 94 MB — a fusion-buffer and
compression stress test of the DP engine.

Built from stock PyTorch-ROCm ops (``scaled_dot_product_attention``, hipBLASLt GEMMs) under bf16
autocast. Not part of the reference repo (whose only model is the MNIST CNN).
"""
from __future__ import annotations

import dataclasses
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclasses.dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_len: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    attn_dropout: float | None = None  # attention-probability dropout (None: ``dropout``)
    attn_impl: str = "sdpa"  # "sdpa" (F.scaled_dot_product_attention) | "math" (matmul/softmax ops)
    eps: float = 1e-12
    # "gather": lookups as index_select, whose backward is a scatter-add (index_add_); "embedding":
    # F.embedding, whose backward sorts the ids and segments them with rocprim's unique_by_key —
    # that partition kernel faults (memory aperture violation) when a whole BERT step is replayed
    # from a HIP graph on this ROCm build with MLM data (many repeated [MASK] ids)
    embedding_impl: str = "gather"


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.c = c
        self.qkv = nn.Linear(c.hidden, 3 * c.hidden)
        self.proj = nn.Linear(c.hidden, c.hidden)
        self.ln1 = nn.LayerNorm(c.hidden, eps=c.eps)
        self.fc1 = nn.Linear(c.hidden, c.ffn)
        self.fc2 = nn.Linear(c.ffn, c.hidden)
        self.ln2 = nn.LayerNorm(c.hidden, eps=c.eps)
        self.drop = nn.Dropout(c.dropout)

    def _attn_p(self):
        return self.c.dropout if self.c.attn_dropout is None else self.c.attn_dropout

    def forward(self, x, mask=None):
        B, S, H = x.shape
        nh = self.c.heads
        q, k, v = self.qkv(x).view(B, S, 3, nh, H // nh).permute(2, 0, 3, 1, 4)
        p = self._attn_p() if self.training else 0.0
        if self.c.attn_impl == "math":
            w = (q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(q.size(-1)))
            if mask is not None:
                w = w + mask
            a = F.dropout(w.softmax(-1), p=p, training=p > 0) @ v
        else:
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=p)
        a = a.transpose(1, 2).reshape(B, S, H)
        x = self.ln1(x + self.drop(self.proj(a)))  # post-LN, as in BERT
        return self.ln2(x + self.drop(self.fc2(F.gelu(self.fc1(x)))))


class BertForMaskedLM(nn.Module):
    def __init__(self, c: BertConfig | None = None):
        super().__init__()
        c = c or BertConfig()
        self.c = c
        self.tok = nn.Embedding(c.vocab_size, c.hidden)
        self.pos = nn.Embedding(c.max_len, c.hidden)
        self.typ = nn.Embedding(c.type_vocab, c.hidden)
        self.ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.drop = nn.Dropout(c.dropout)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.head_dense = nn.Linear(c.hidden, c.hidden)
        self.head_ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.head_bias = nn.Parameter(torch.zeros(c.vocab_size))  # decoder weight tied to self.tok
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def _lookup(self, emb: nn.Embedding, ids: torch.Tensor) -> torch.Tensor:
        if self.c.embedding_impl == "embedding":
            return emb(ids)
        return emb.weight.index_select(0, ids.reshape(-1)).view(*ids.shape, emb.weight.shape[1])

    def forward(self, ids, labels=None, masked_positions=None):
        """``masked_positions`` (flat indices into B*S, e.g. from :func:`masked_positions`): apply the
        MLM head only at those positions, as BERT pretraining implementations do — the vocabulary
        projection and its softmax then cost ~15 % of the all-position form. Fixed-size, so the step
        stays free of host synchronisation (HIP-graph capturable)."""
        B, S = ids.shape
        pos = torch.arange(S, device=ids.device)
        x = self._lookup(self.tok, ids) + self._lookup(self.pos, pos)[None] + self._lookup(self.typ, torch.zeros_like(ids))
        x = self.drop(self.ln(x))
        for layer in self.layers:
            x = layer(x)
        if masked_positions is not None:
            x = x.reshape(B * S, -1).index_select(0, masked_positions)
            if labels is not None:
                labels = labels.reshape(-1).index_select(0, masked_positions)
        h = self.head_ln(F.gelu(self.head_dense(x)))
        logits = h @ self.tok.weight.t() + self.head_bias
        if labels is None:
            return logits
        return F.cross_entropy(logits.float().view(-1, logits.size(-1)), labels.reshape(-1), ignore_index=-100)


def masked_positions(labels: torch.Tensor) -> torch.Tensor:
    """Flat indices of the positions that carry an MLM label (one host sync: call once per batch
    layout, not per step)."""
    return (labels.reshape(-1) != -100).nonzero().squeeze(1)


def synthetic_mlm_batch(batch: int, seq: int, vocab: int, device, generator=None, mask_prob: float = 0.15):
    ids = torch.randint(0, vocab, (batch, seq), device=device, generator=generator)
    labels = torch.full_like(ids, -100)
    m = torch.rand(batch, seq, device=device, generator=generator) < mask_prob
    labels[m] = ids[m]
    ids = ids.masked_fill(m, 103)  # [MASK]
    return ids, labels


def flops_per_token(c: BertConfig, seq: int) -> float:
    """Training FLOPs per token (6·params for the dense parts + attention scores)."""
    dense = c.layers * (4 * c.hidden * c.hidden + 2 * c.hidden * c.ffn) + c.hidden * c.vocab_size
    attn = c.layers * 2 * seq * c.hidden
    return 6.0 * dense + 6.0 * attn if math.isfinite(seq) else float("nan")
