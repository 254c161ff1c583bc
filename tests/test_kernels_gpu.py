"""Numerics of the hand-written CDNA4 kernels against plain PyTorch fp32 references (run on MI355X).

Every kernel consumes bf16 MFMA operands, so references are evaluated on the same bf16-rounded
inputs where that isolates the kernel's own error (fp32 accumulation) from input quantisation.
Batch sizes include non-multiples of 16 (7, 100) to catch tiling bugs.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
 conv1_wgrad feeds the MFMAif not torch.cuda.is_available():
 conv1_wgrad feeds the MFMA    pytest.skip("needs a GPU")
 conv1_wgrad feeds the MFMAfrom mihvd import _native

 conv1_wgrad feeds the MFMA_native.require_kernels()
 conv1_wgrad feeds the MFMAreturn torch.ops.mihvd


def bf(x):
 conv1_wgrad feeds the MFMAreturn x.to(torch.bfloat16).float()


def rel_err(a, b):
 conv1_wgrad feeds the MFMAreturn ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def ref_conv_pool(x_nhwc, w_hwio, b):
 conv1_wgrad feeds the MFMA"""conv SAME + bias + ReLU + maxpool 2x2 -> (pooled NHWC, argmax 0..3)."""
 conv1_wgrad feeds the MFMAx = x_nhwc.permute(0, 3, 1, 2)
 conv1_wgrad feeds the MFMAy = F.conv2d(x, w_hwio.permute(3, 2, 0, 1), b, padding=2)
 conv1_wgrad feeds the MFMAy = F.relu(y)
 conv1_wgrad feeds the MFMApooled, ind = F.max_pool2d(y, 2, 2, return_indices=True)
 conv1_wgrad feeds the MFMAW = y.shape[-1]
 conv1_wgrad feeds the MFMAr, c = ind // W, ind % W
 conv1_wgrad feeds the MFMAd = (r % 2) * 2 + (c % 2)
 conv1_wgrad feeds the MFMAreturn pooled.permute(0, 2, 3, 1), d.permute(0, 2, 3, 1), y


@pytest.mark.parametrize("B", [7, 100])
def test_conv1_fwd(ops, B):
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(1)
 conv1_wgrad feeds the MFMAx = torch.rand(B, 784, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAw = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
 conv1_wgrad feeds the MFMAb = torch.randn(32, device="cuda", generator=g) * 0.1
 conv1_wgrad feeds the MFMAa1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAidx = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8)
 conv1_wgrad feeds the MFMAops.conv1_fwd(x, None, None, w.reshape(800), b, a1, idx)
 conv1_wgrad feeds the MFMAref, rd, _ = ref_conv_pool(x.view(B, 28, 28, 1), w, b)
 conv1_wgrad feeds the MFMAassert rel_err(a1, ref) < 5e-3
 conv1_wgrad feeds the MFMApos = ref > 1e-3
 conv1_wgrad feeds the MFMAassert (idx.long()[pos] == rd[pos]).float().mean() > 0.995


@pytest.mark.parametrize("B", [7, 100])
def test_conv2_fwd(ops, B):
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(2)
 conv1_wgrad feeds the MFMAa1 = bf(torch.rand(B, 14, 14, 32, device="cuda", generator=g))
 conv1_wgrad feeds the MFMAw = bf(torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05)
 conv1_wgrad feeds the MFMAb = torch.randn(64, device="cuda", generator=g) * 0.1
 conv1_wgrad feeds the MFMAa2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAidx = torch.empty(B, 3136, device="cuda", dtype=torch.uint8)
 conv1_wgrad feeds the MFMAops.conv2_fwd(a1.to(torch.bfloat16), w.to(torch.bfloat16).reshape(-1), b, a2, idx)
 conv1_wgrad feeds the MFMAref, rd, _ = ref_conv_pool(a1, w, b)
 conv1_wgrad feeds the MFMAassert rel_err(a2, ref.reshape(B, 3136)) < 5e-3
 conv1_wgrad feeds the MFMApos = ref.reshape(B, 3136) > 1e-2
 conv1_wgrad feeds the MFMAassert (idx.long()[pos] == rd.reshape(B, 3136)[pos]).float().mean() > 0.99


@pytest.mark.parametrize("B", [7, 100, 128])
def test_fc1_fwd(ops, B):
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(3)
 conv1_wgrad feeds the MFMAa2 = bf(torch.rand(B, 3136, device="cuda", generator=g))
 conv1_wgrad feeds the MFMAw = bf(torch.randn(3136, 1024, device="cuda", generator=g) * 0.02)
 conv1_wgrad feeds the MFMAzp = torch.empty(14, B, 1024, device="cuda")
 conv1_wgrad feeds the MFMAops.fc1_fwd(a2.to(torch.bfloat16), w.to(torch.bfloat16), zp)
 conv1_wgrad feeds the MFMAassert rel_err(zp.sum(0), a2 @ w) < 1e-4


def test_head_no_dropout(ops):
 conv1_wgrad feeds the MFMAB = 100
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(4)
 conv1_wgrad feeds the MFMAzp = torch.randn(14, B, 1024, device="cuda", generator=g) * 0.1
 conv1_wgrad feeds the MFMAb3 = torch.randn(1024, device="cuda", generator=g) * 0.1
 conv1_wgrad feeds the MFMAw4 = torch.randn(1024, 10, device="cuda", generator=g) * 0.05
 conv1_wgrad feeds the MFMAb4 = torch.randn(10, device="cuda", generator=g) * 0.1
 conv1_wgrad feeds the MFMAy = torch.randint(0, 10, (B,), device="cuda", generator=g)
 conv1_wgrad feeds the MFMAh = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAdz = torch.empty_like(h)
 conv1_wgrad feeds the MFMAdlog = torch.empty(B, 10, device="cuda")
 conv1_wgrad feeds the MFMAstats = torch.empty(B, 2, device="cuda")
 conv1_wgrad feeds the MFMAops.head_fwd_bwd(zp, b3, w4, b4, y, None, None, 0, 0.0, h, dz, dlog, stats)
 conv1_wgrad feeds the MFMAz = (zp.sum(0) + b3).requires_grad_(True)
 conv1_wgrad feeds the MFMAhr = F.relu(z)
 conv1_wgrad feeds the MFMAlogits = bf(hr) @ w4 + b4
 conv1_wgrad feeds the MFMAloss = F.cross_entropy(logits, y)
 conv1_wgrad feeds the MFMAloss.backward()
 conv1_wgrad feeds the MFMAassert rel_err(h, hr) < 5e-3
 conv1_wgrad feeds the MFMAassert abs(stats[:, 0].mean().item() - loss.item()) < 1e-3
 conv1_wgrad feeds the MFMAassert rel_err(dz, z.grad) < 1e-2
 conv1_wgrad feeds the MFMAassert stats[:, 1].mean().item() == pytest.approx((logits.argmax(1) == y).float().mean().item(), abs=0.02)


def test_head_dropout_rate(ops):
 conv1_wgrad feeds the MFMAB = 100
 conv1_wgrad feeds the MFMAzp = torch.ones(14, B, 1024, device="cuda")
 conv1_wgrad feeds the MFMAh = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAdz, dlog, stats = torch.empty_like(h), torch.empty(B, 10, device="cuda"), torch.empty(B, 2, device="cuda")
 conv1_wgrad feeds the MFMAst = torch.zeros(4, device="cuda", dtype=torch.int64)
 conv1_wgrad feeds the MFMAargs = (torch.zeros(1024, device="cuda"), torch.zeros(1024, 10, device="cuda"), torch.zeros(10, device="cuda"),
 conv1_wgrad feeds the MFMA        torch.zeros(B, device="cuda", dtype=torch.int64), None, st, 123, 0.5)
 conv1_wgrad feeds the MFMAops.head_fwd_bwd(zp, *args, h, dz, dlog, stats)
 conv1_wgrad feeds the MFMAkeep = (h.float() > 0).float()
 conv1_wgrad feeds the MFMAassert abs(keep.mean().item() - 0.5) < 0.01
 conv1_wgrad feeds the MFMAassert torch.allclose(h.float()[h.float() > 0], torch.full_like(h.float()[h.float() > 0], 28.0))  # 14*1*2
 conv1_wgrad feeds the MFMAh2 = torch.empty_like(h)
 conv1_wgrad feeds the MFMAops.head_fwd_bwd(zp, *args, h2, dz, dlog, stats)
 conv1_wgrad feeds the MFMA# head advances only the optimizer counter (state[1]); the mask is keyed on state[0]
 conv1_wgrad feeds the MFMAassert torch.equal(h, h2) and int(st[1]) == 2 and int(st[0]) == 0


def test_dropout_mask_depends_on_forward_step(ops):
 conv1_wgrad feeds the MFMAB = 16
 conv1_wgrad feeds the MFMAzp = torch.ones(14, B, 1024, device="cuda")
 conv1_wgrad feeds the MFMAst = torch.zeros(4, device="cuda", dtype=torch.int64)
 conv1_wgrad feeds the MFMAouts = []
 conv1_wgrad feeds the MFMAfor step in (0, 0, 1):
 conv1_wgrad feeds the MFMA    st[0] = step
 conv1_wgrad feeds the MFMA    h = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMA    ops.head_fwd_bwd(zp, torch.zeros(1024, device="cuda"), torch.zeros(1024, 10, device="cuda"),
 conv1_wgrad feeds the MFMA                     torch.zeros(10, device="cuda"), torch.zeros(B, device="cuda", dtype=torch.int64), None, st, 5, 0.5,
 conv1_wgrad feeds the MFMA                     h, torch.empty_like(h), torch.empty(B, 10, device="cuda"), torch.empty(B, 2, device="cuda"))
 conv1_wgrad feeds the MFMA    outs.append(h)
 conv1_wgrad feeds the MFMAassert torch.equal(outs[0], outs[1]) and not torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("B", [7, 100])
def test_fc1_bwd(ops, B):
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(5)
 conv1_wgrad feeds the MFMAdz = bf(torch.randn(B, 1024, device="cuda", generator=g) * 0.01)
 conv1_wgrad feeds the MFMAw3 = bf(torch.randn(3136, 1024, device="cuda", generator=g) * 0.02)
 conv1_wgrad feeds the MFMAa2 = bf(F.relu(torch.randn(B, 3136, device="cuda", generator=g)))
 conv1_wgrad feeds the MFMAh = bf(F.relu(torch.randn(B, 1024, device="cuda", generator=g)))
 conv1_wgrad feeds the MFMAdlog = torch.randn(B, 10, device="cuda", generator=g) * 0.01
 conv1_wgrad feeds the MFMAgW3 = torch.empty(3136, 1024, device="cuda")
 conv1_wgrad feeds the MFMAgb3, gW4, gb4 = torch.empty(1024, device="cuda"), torch.empty(1024, 10, device="cuda"), torch.empty(10, device="cuda")
 conv1_wgrad feeds the MFMAgb2, gW1, gb1 = (torch.full((64,), 3.0, device="cuda"), torch.full((800,), 3.0, device="cuda"),
 conv1_wgrad feeds the MFMA                 torch.full((32,), 3.0, device="cuda"))
 conv1_wgrad feeds the MFMAops.fc1_wgrad(dz.to(torch.bfloat16), a2.to(torch.bfloat16), h.to(torch.bfloat16), dlog, gW3, gb3, gW4, gb4, gb2,
 conv1_wgrad feeds the MFMA              gW1, gb1)
 conv1_wgrad feeds the MFMAg2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAops.fc1_dgrad(dz.to(torch.bfloat16), w3.to(torch.bfloat16), a2.to(torch.bfloat16), g2)
 conv1_wgrad feeds the MFMAassert rel_err(g2, (dz @ w3.t()) * (a2 > 0)) < 5e-3
 conv1_wgrad feeds the MFMAassert rel_err(gW3, a2.t() @ dz) < 1e-4
 conv1_wgrad feeds the MFMAassert rel_err(gb3, dz.sum(0)) < 1e-4
 conv1_wgrad feeds the MFMAassert rel_err(gW4, h.t() @ dlog) < 1e-4
 conv1_wgrad feeds the MFMAassert rel_err(gb4, dlog.sum(0)) < 1e-4
 conv1_wgrad feeds the MFMAassert gb2.abs().sum() == 0 and gW1.abs().sum() == 0 and gb1.abs().sum() == 0


@pytest.mark.parametrize("B", [7, 100])
def test_conv2_bwd_fused_conv1_wgrad(ops, B):
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(6)
 conv1_wgrad feeds the MFMA# Build consistent forward state with the kernels themselves, then compare the backward.
 conv1_wgrad feeds the MFMAx = torch.rand(B, 784, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAw1 = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
 conv1_wgrad feeds the MFMAb1 = torch.randn(32, device="cuda", generator=g) * 0.05
 conv1_wgrad feeds the MFMAw2 = bf(torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05)
 conv1_wgrad feeds the MFMAb2 = torch.randn(64, device="cuda", generator=g) * 0.05
 conv1_wgrad feeds the MFMAa1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAidx1 = torch.empty_like(a1, dtype=torch.uint8)
 conv1_wgrad feeds the MFMAops.conv1_fwd(x, None, None, w1.reshape(800), b1, a1, idx1)
 conv1_wgrad feeds the MFMAa2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMAidx2 = torch.empty_like(a2, dtype=torch.uint8)
 conv1_wgrad feeds the MFMAops.conv2_fwd(a1, w2.to(torch.bfloat16).reshape(-1), b2, a2, idx2)
 conv1_wgrad feeds the MFMAdA2 = torch.randn(B, 3136, device="cuda", generator=g) * 0.01
 conv1_wgrad feeds the MFMAg2 = (dA2 * (a2.float() > 0)).to(torch.bfloat16)  # what fc1_dgrad hands to conv2_bwd
 conv1_wgrad feeds the MFMAG = int(ops.conv2_wgrad_groups(B))
 conv1_wgrad feeds the MFMAg1 = torch.empty_like(a1)
 conv1_wgrad feeds the MFMAslab = torch.empty(G, 51200, device="cuda")
 conv1_wgrad feeds the MFMAgb2, gW1, gb1, gW2 = (torch.zeros(64, device="cuda"), torch.zeros(800, device="cuda"),
 conv1_wgrad feeds the MFMA                      torch.zeros(32, device="cuda"), torch.empty(51200, device="cuda"))
 conv1_wgrad feeds the MFMAops.conv2_bwd(g2, idx2, a1, w2.to(torch.bfloat16).reshape(-1), x, None, None, idx1, slab, gb2, gW1, gb1, g1)
 conv1_wgrad feeds the MFMAops.conv2_wgrad_reduce(slab, B, gW2)
 conv1_wgrad feeds the MFMA# Reference: autograd through conv2 (+relu+pool) on the same bf16 a1, and conv1 on fp32 x.
 conv1_wgrad feeds the MFMAa1r = a1.float().requires_grad_(True)
 conv1_wgrad feeds the MFMAw2r = w2.clone().requires_grad_(True)
 conv1_wgrad feeds the MFMAb2r = b2.clone().requires_grad_(True)
 conv1_wgrad feeds the MFMAp2, _, _ = ref_conv_pool(a1r, w2r, b2r)
 conv1_wgrad feeds the MFMAp2.reshape(B, 3136).backward(g2.float())
 conv1_wgrad feeds the MFMAassert rel_err(gW2.view(5, 5, 32, 64), w2r.grad) < 1e-2
 conv1_wgrad feeds the MFMAassert rel_err(gb2, b2r.grad) < 1e-3
 conv1_wgrad feeds the MFMAg1_ref = a1r.grad * (a1.float() > 0)
 conv1_wgrad feeds the MFMAassert rel_err(g1, g1_ref) < 1e-2
 conv1_wgrad feeds the MFMAw1r = w1.clone().requires_grad_(True)
 conv1_wgrad feeds the MFMAb1r = b1.clone().requires_grad_(True)
 conv1_wgrad feeds the MFMAp1, _, _ = ref_conv_pool(x.view(B, 28, 28, 1), w1r, b1r)
 conv1_wgrad feeds the MFMAp1.backward(g1.float())
 conv1_wgrad feeds the MFMA# conv1_wgrad feeds the MFMA with the input image in bf16 (rel. rounding 2^-9), the reference
 conv1_wgrad feeds the MFMA# keeps fp32 x: a few 1e-3 of relative difference
 conv1_wgrad feeds the MFMAassert rel_err(gW1.view(5, 5, 1, 32), w1r.grad) < 5e-3
 conv1_wgrad feeds the MFMAassert rel_err(gb1, b1r.grad) < 1e-3


def test_adam_matches_tf_rule(ops):
 conv1_wgrad feeds the MFMAfrom mihvd.optim import TFAdam

 conv1_wgrad feeds the MFMAn = 4096
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(7)
 conv1_wgrad feeds the MFMAp0 = torch.randn(n, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAp, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
 conv1_wgrad feeds the MFMAsh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
 conv1_wgrad feeds the MFMApr = torch.nn.Parameter(p0.clone())
 conv1_wgrad feeds the MFMAopt = TFAdam([pr], lr=1e-2)
 conv1_wgrad feeds the MFMAfor t in range(1, 4):
 conv1_wgrad feeds the MFMA    grad = torch.randn(n, device="cuda", generator=g)
 conv1_wgrad feeds the MFMA    ops.adam_step(p, grad * 2, m, v, sh, None, t, 1e-2, 0.9, 0.999, 1e-8, 0.5, 0)
 conv1_wgrad feeds the MFMA    pr.grad = grad.clone()
 conv1_wgrad feeds the MFMA    opt.step()
 conv1_wgrad feeds the MFMAassert torch.allclose(p, pr.detach(), atol=1e-6, rtol=1e-5)
 conv1_wgrad feeds the MFMAassert torch.equal(sh, p.to(torch.bfloat16))


class _RoundBF(torch.autograd.Function):
 conv1_wgrad feeds the MFMA"""bf16 storage point: round the value forward and the gradient backward."""

 conv1_wgrad feeds the MFMA@staticmethod
 conv1_wgrad feeds the MFMAdef forward(ctx, x):
 conv1_wgrad feeds the MFMA    return x.to(torch.bfloat16).float()

 conv1_wgrad feeds the MFMA@staticmethod
 conv1_wgrad feeds the MFMAdef backward(ctx, g):
 conv1_wgrad feeds the MFMA    return g.to(torch.bfloat16).float()


class _RoundFwd(torch.autograd.Function):
 conv1_wgrad feeds the MFMA"""bf16 weight shadow: rounded forward, fp32 (master) gradient backward."""

 conv1_wgrad feeds the MFMA@staticmethod
 conv1_wgrad feeds the MFMAdef forward(ctx, x):
 conv1_wgrad feeds the MFMA    return x.to(torch.bfloat16).float()

 conv1_wgrad feeds the MFMA@staticmethod
 conv1_wgrad feeds the MFMAdef backward(ctx, g):
 conv1_wgrad feeds the MFMA    return g


def _pool_by_index(y_nhwc, idx):
 conv1_wgrad feeds the MFMA"""Max-pool routed by the kernel's argmax (d = 2*dy + dx), differentiable."""
 conv1_wgrad feeds the MFMAB, H, W, C = y_nhwc.shape
 conv1_wgrad feeds the MFMAy = y_nhwc.reshape(B, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(B, H // 2, W // 2, C, 4)
 conv1_wgrad feeds the MFMAreturn y.gather(-1, idx.long().unsqueeze(-1)).squeeze(-1)


def _emulated_reference(params, x, y, idx1, idx2):
 conv1_wgrad feeds the MFMA"""The fused step's exact math in fp32 autograd: same bf16 rounding points, same pool routing."""
 conv1_wgrad feeds the MFMAP = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
 conv1_wgrad feeds the MFMAB = x.shape[0]
 conv1_wgrad feeds the MFMAy1 = F.conv2d(x.view(B, 1, 28, 28), P["conv_layer1/conv2d/kernel"].permute(3, 2, 0, 1),
 conv1_wgrad feeds the MFMA              P["conv_layer1/conv2d/bias"], padding=2).permute(0, 2, 3, 1)
 conv1_wgrad feeds the MFMAa1 = _RoundBF.apply(F.relu(_pool_by_index(y1, idx1)))
 conv1_wgrad feeds the MFMAw2 = _RoundFwd.apply(P["conv_layer2/conv2d/kernel"])
 conv1_wgrad feeds the MFMAy2 = F.conv2d(a1.permute(0, 3, 1, 2), w2.permute(3, 2, 0, 1), P["conv_layer2/conv2d/bias"], padding=2)
 conv1_wgrad feeds the MFMAa2 = _RoundBF.apply(F.relu(_pool_by_index(y2.permute(0, 2, 3, 1), idx2.view(B, 7, 7, 64)))).reshape(B, 3136)
 conv1_wgrad feeds the MFMAz = a2 @ _RoundFwd.apply(P["dense/kernel"]) + P["dense/bias"]
 conv1_wgrad feeds the MFMAh = _RoundBF.apply(F.relu(z))
 conv1_wgrad feeds the MFMAlogits = h @ P["dense_1/kernel"] + P["dense_1/bias"]
 conv1_wgrad feeds the MFMAloss = F.cross_entropy(logits, y)
 conv1_wgrad feeds the MFMAloss.backward()
 conv1_wgrad feeds the MFMAreturn loss.detach(), {k: v.grad for k, v in P.items()}


@pytest.mark.parametrize("B", [8, 100])
def test_fused_step_matches_emulated_reference(ops, B):
 conv1_wgrad feeds the MFMA"""One fused step (dropout off, lr 0): loss and every gradient equal an fp32 autograd
 conv1_wgrad feeds the MFMAreference with the same bf16 storage points and pool routing; the loss is also within
 conv1_wgrad feeds the MFMAmixed-precision distance of the pure fp32 model."""
 conv1_wgrad feeds the MFMAfrom mihvd.models.fused_mnist import FusedMNISTTrainer
 conv1_wgrad feeds the MFMAfrom mihvd.models.mnist import MNISTConvNet, TF_PARAM_ORDER

 conv1_wgrad feeds the MFMAtr = FusedMNISTTrainer(batch_size=B, lr=0.0, dropout=0.0, seed=3, device="cuda")
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(8)
 conv1_wgrad feeds the MFMAx = torch.rand(B, 784, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAy = torch.randint(0, 10, (B,), device="cuda", generator=g)
 conv1_wgrad feeds the MFMAparams = {n: tr.pview(n).clone() for n in TF_PARAM_ORDER}
 conv1_wgrad feeds the MFMAout = tr.train_step(x, y)
 conv1_wgrad feeds the MFMAtorch.cuda.synchronize()
 conv1_wgrad feeds the MFMAloss, grads = _emulated_reference(params, x, y, tr.idx1, tr.idx2)
 conv1_wgrad feeds the MFMAassert abs(out["loss"].item() - loss.item()) < 1e-3 * max(1.0, loss.item())
 conv1_wgrad feeds the MFMAfor name in TF_PARAM_ORDER:
 conv1_wgrad feeds the MFMA    e = rel_err(tr.gview(name), grads[name])
 conv1_wgrad feeds the MFMA    assert e < 1e-2, (name, e)
 conv1_wgrad feeds the MFMAref = MNISTConvNet(impl="torch", seed=3).cuda().eval()
 conv1_wgrad feeds the MFMAassert abs(F.cross_entropy(ref(x), y).item() - loss.item()) < 2e-2 * max(1.0, loss.item())


def test_fused_training_converges_and_graph_replays(ops):
 conv1_wgrad feeds the MFMAfrom mihvd.models.fused_mnist import FusedMNISTTrainer
 conv1_wgrad feeds the MFMAfrom mihvd.utils.data import synthetic_mnist

 conv1_wgrad feeds the MFMA(x, y), _ = synthetic_mnist(n_train=3000, n_test=10, seed=5)
 conv1_wgrad feeds the MFMAX = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
 conv1_wgrad feeds the MFMAY = torch.from_numpy(y.astype("int64")).cuda()
 conv1_wgrad feeds the MFMAtr = FusedMNISTTrainer(batch_size=100, lr=1e-3, seed=0, device="cuda")
 conv1_wgrad feeds the MFMAtr.set_device_dataset(X, Y)
 conv1_wgrad feeds the MFMAassert tr.build_graph(steps_per_replay=10)
 conv1_wgrad feeds the MFMAfirst = None
 conv1_wgrad feeds the MFMAfor i in range(30):
 conv1_wgrad feeds the MFMA    tr.run_graph()
 conv1_wgrad feeds the MFMA    if first is None:
 conv1_wgrad feeds the MFMA        first = tr.last_loss()
 conv1_wgrad feeds the MFMAtorch.cuda.synchronize()
 conv1_wgrad feeds the MFMAassert tr.global_step == 2 + 300
 conv1_wgrad feeds the MFMAassert int(tr.state[0].item()) == tr.global_step and int(tr.state[1].item()) == tr.global_step
 conv1_wgrad feeds the MFMAassert tr.last_loss() < first * 0.5, (first, tr.last_loss())
 conv1_wgrad feeds the MFMAassert tr.last_accuracy() > 0.8


def test_fused_loss_autograd_matches_trainer(ops):
 conv1_wgrad feeds the MFMA"""ops.functional.fused_mnist_loss (one autograd node) gives the trainer's gradients, and the
 conv1_wgrad feeds the MFMAHIP inference logits agree with the torch model."""
 conv1_wgrad feeds the MFMAfrom mihvd.models.fused_mnist import FusedMNISTTrainer
 conv1_wgrad feeds the MFMAfrom mihvd.models.mnist import MNISTConvNet
 conv1_wgrad feeds the MFMAfrom mihvd.ops.functional import fused_mnist_loss, mnist_logits

 conv1_wgrad feeds the MFMAB = 64
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(9)
 conv1_wgrad feeds the MFMAx = torch.rand(B, 784, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAy = torch.randint(0, 10, (B,), device="cuda", generator=g)
 conv1_wgrad feeds the MFMAmodel = MNISTConvNet(impl="hip", seed=3).cuda()
 conv1_wgrad feeds the MFMAloss, acc = fused_mnist_loss(model, x, y, training=False, return_accuracy=True)
 conv1_wgrad feeds the MFMAloss.backward()
 conv1_wgrad feeds the MFMAtr = FusedMNISTTrainer(batch_size=B, lr=0.0, dropout=0.0, seed=3, device="cuda")
 conv1_wgrad feeds the MFMAout = tr.train_step(x, y)
 conv1_wgrad feeds the MFMAtorch.cuda.synchronize()
 conv1_wgrad feeds the MFMAassert abs(loss.item() - out["loss"].item()) < 1e-5
 conv1_wgrad feeds the MFMAfor name, p in model.ordered_parameters():
 conv1_wgrad feeds the MFMA    assert rel_err(p.grad, tr.gview(name)) < 1e-3, name
 conv1_wgrad feeds the MFMAref = MNISTConvNet(impl="torch", seed=3).cuda().eval()
 conv1_wgrad feeds the MFMAwith torch.no_grad():
 conv1_wgrad feeds the MFMA    assert rel_err(mnist_logits(model, x), ref(x)) < 2e-2


def test_adasum_hip_matches_torch(ops):
 conv1_wgrad feeds the MFMA"""dp_kernels.hip segment_dots + adasum_combine vs the fp64 torch formulation (incl. gaps and
 conv1_wgrad feeds the MFMAsegments that are not float4-aligned)."""
 conv1_wgrad feeds the MFMAfrom mihvd.parallel import adasum

 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(11)
 conv1_wgrad feeds the MFMAn = 3 * 8192 + 37
 conv1_wgrad feeds the MFMAa = torch.randn(n, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAb = torch.randn(n, device="cuda", generator=g) * 0.3 + 0.5 * a
 conv1_wgrad feeds the MFMAsegs = [(0, 5), (5, 9000), (9003, 20001), (20001, n - 10)]  # gaps at 9000..9003 and the tail
 conv1_wgrad feeds the MFMAa[9000:9003] = 0
 conv1_wgrad feeds the MFMAb[9000:9003] = 0
 conv1_wgrad feeds the MFMAout = adasum.adasum_pair(a, b, segs)
 conv1_wgrad feeds the MFMAref = adasum.adasum_pair(a.cpu(), b.cpu(), segs)
 conv1_wgrad feeds the MFMAassert rel_err(out.cpu(), ref) < 1e-6
 conv1_wgrad feeds the MFMA# zero-norm rules: |a| = 0 -> b
 conv1_wgrad feeds the MFMAz = torch.zeros_like(a)
 conv1_wgrad feeds the MFMAassert torch.equal(adasum.adasum_pair(z, b), b)
 conv1_wgrad feeds the MFMA# misaligned views take the scalar paths
 conv1_wgrad feeds the MFMAout2 = adasum.adasum_pair(a[1:], b[1:])
 conv1_wgrad feeds the MFMAassert rel_err(out2.cpu(), adasum.adasum_pair(a[1:].cpu(), b[1:].cpu())) < 1e-6


def test_loss_scale_kernels(ops):
 conv1_wgrad feeds the MFMAgrads = [torch.full((1000,), 8.0, device="cuda"), torch.full((33,), -4.0, device="cuda")]
 conv1_wgrad feeds the MFMAls = torch.tensor([4.0, 0.0], device="cuda")
 conv1_wgrad feeds the MFMAtracker = torch.zeros(1, dtype=torch.int32, device="cuda")
 conv1_wgrad feeds the MFMAops.grad_check_(grads, ls, True)
 conv1_wgrad feeds the MFMAassert float(ls[1]) == 0.0 and torch.all(grads[0] == 2.0) and torch.all(grads[1] == -1.0)
 conv1_wgrad feeds the MFMAops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
 conv1_wgrad feeds the MFMAassert float(ls[0]) == 4.0 and int(tracker) == 1
 conv1_wgrad feeds the MFMAops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
 conv1_wgrad feeds the MFMAassert float(ls[0]) == 8.0 and int(tracker) == 0
 conv1_wgrad feeds the MFMAgrads[1][7] = float("inf")
 conv1_wgrad feeds the MFMAops.grad_check_(grads, ls, False)
 conv1_wgrad feeds the MFMAassert float(ls[1]) == 1.0
 conv1_wgrad feeds the MFMAops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
 conv1_wgrad feeds the MFMAassert float(ls[0]) == 4.0 and float(ls[1]) == 0.0


def test_adam_loss_scale_fused(ops):
 conv1_wgrad feeds the MFMAn = 4096
 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(12)
 conv1_wgrad feeds the MFMAp0 = torch.randn(n, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAgr = torch.randn(n, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAouts = []
 conv1_wgrad feeds the MFMAfor scale, found in ((1.0, 0.0), (8.0, 0.0), (8.0, 1.0)):
 conv1_wgrad feeds the MFMA    p, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
 conv1_wgrad feeds the MFMA    ls = torch.tensor([scale, found], device="cuda")
 conv1_wgrad feeds the MFMA    ops.adam_step(p, gr * scale, m, v, None, None, 1, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0, 0, ls)
 conv1_wgrad feeds the MFMA    outs.append(p)
 conv1_wgrad feeds the MFMAassert torch.allclose(outs[0], outs[1], atol=1e-7)
 conv1_wgrad feeds the MFMAassert torch.equal(outs[2], p0)  # overflow step skipped


def test_adam_pipeline_matches_serial(ops, monkeypatch):
 conv1_wgrad feeds the MFMA"""MIHVD_ADAM_PIPELINE=1 (fc Adam on a side stream, overlapping the conv backward and the next
 conv1_wgrad feeds the MFMAstep's convolutions, graph-captured) trains like the serial step."""
 conv1_wgrad feeds the MFMAfrom mihvd.models.fused_mnist import FusedMNISTTrainer

 conv1_wgrad feeds the MFMAg = torch.Generator(device="cuda").manual_seed(21)
 conv1_wgrad feeds the MFMAX = torch.rand(400, 784, device="cuda", generator=g)
 conv1_wgrad feeds the MFMAY = torch.randint(0, 10, (400,), device="cuda", generator=g)
 conv1_wgrad feeds the MFMAout = []
 conv1_wgrad feeds the MFMAp_init = None
 conv1_wgrad feeds the MFMAfor pipe in ("0", "1"):
 conv1_wgrad feeds the MFMA    monkeypatch.setenv("MIHVD_ADAM_PIPELINE", pipe)
 conv1_wgrad feeds the MFMA    monkeypatch.setenv("MIHVD_ADAM_BLOCKS", "128" if pipe == "1" else "0")
 conv1_wgrad feeds the MFMA    tr = FusedMNISTTrainer(batch_size=100, seed=4, device="cuda", dropout=0.0)
 conv1_wgrad feeds the MFMA    assert tr.pipeline == (pipe == "1")
 conv1_wgrad feeds the MFMA    if p_init is None:
 conv1_wgrad feeds the MFMA        p_init = tr.params.clone()
 conv1_wgrad feeds the MFMA    tr.set_device_dataset(X, Y, shuffle=False)
 conv1_wgrad feeds the MFMA    tr.build_graph(steps_per_replay=4, warmup=2)
 conv1_wgrad feeds the MFMA    tr.run_graph()
 conv1_wgrad feeds the MFMA    torch.cuda.synchronize()
 conv1_wgrad feeds the MFMA    out.append((tr.params.clone(), tr.last_loss(), int(tr.state[0]), int(tr.state[1])))
 conv1_wgrad feeds the MFMA(p0, l0, f0, t0), (p1, l1, f1, t1) = out
 conv1_wgrad feeds the MFMAassert (f0, t0) == (f1, t1) == (6, 6)
 conv1_wgrad feeds the MFMAassert abs(l0 - l1) < 1e-3 * max(1.0, abs(l0))
 conv1_wgrad feeds the MFMA# conv1_wgrad's atomics make runs differ in the last bits, which Adam's normalisation turns into
 conv1_wgrad feeds the MFMA# O(lr) steps on near-zero-gradient weights: compare the updates, not the bits
 conv1_wgrad feeds the MFMAassert rel_err(p1 - p_init, p0 - p_init) < 0.05
