"""Numerics of the hand-written CDNA4 kernels against plain PyTorch fp32 references (run on MI355X).

Every kernel consumes bf16 MFMA operands, so references are evaluated on the same bf16-rounded
inputs where that isolates the kernel's own error (fp32 accumulation) from input quantisation.
Batch sizes include non-multiples of 16 (7, 100) to catch tiling bugs.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from mihvd.models.mnist import FC1_KS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mihvd import _native

    _native.require_kernels()
    return torch.ops.mihvd


def bf(x):
    return x.to(torch.bfloat16).float()


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def ref_conv_pool(x_nhwc, w_hwio, b):
    """conv SAME + bias + ReLU + maxpool 2x2 -> (pooled NHWC, argmax 0..3)."""
    x = x_nhwc.permute(0, 3, 1, 2)
    y = F.conv2d(x, w_hwio.permute(3, 2, 0, 1), b, padding=2)
    y = F.relu(y)
    pooled, ind = F.max_pool2d(y, 2, 2, return_indices=True)
    W = y.shape[-1]
    r, c = ind // W, ind % W
    d = (r % 2) * 2 + (c % 2)
    return pooled.permute(0, 2, 3, 1), d.permute(0, 2, 3, 1), y


@pytest.mark.parametrize("B", [7, 100])
def test_conv1_fwd(ops, B):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(B, 784, device="cuda", generator=g)
    w = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
    b = torch.randn(32, device="cuda", generator=g) * 0.1
    a1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.bfloat16)
    idx = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8)
    ops.conv1_fwd(x, None, None, w.reshape(800), b, a1, idx)
    ref, rd, _ = ref_conv_pool(x.view(B, 28, 28, 1), w, b)
    assert rel_err(a1, ref) < 5e-3
    pos = ref > 1e-3
    assert (idx.long()[pos] == rd[pos]).float().mean() > 0.995


@pytest.mark.parametrize("B", [7, 100])
def test_conv2_fwd(ops, B):
    g = torch.Generator(device="cuda").manual_seed(2)
    a1 = bf(torch.rand(B, 14, 14, 32, device="cuda", generator=g))
    w = bf(torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05)
    b = torch.randn(64, device="cuda", generator=g) * 0.1
    a2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
    idx = torch.empty(B, 3136, device="cuda", dtype=torch.uint8)
    ops.conv2_fwd(a1.to(torch.bfloat16), w.to(torch.bfloat16).reshape(-1), b, a2, idx)
    ref, rd, _ = ref_conv_pool(a1, w, b)
    assert rel_err(a2, ref.reshape(B, 3136)) < 5e-3
    pos = ref.reshape(B, 3136) > 1e-2
    assert (idx.long()[pos] == rd.reshape(B, 3136)[pos]).float().mean() > 0.99


@pytest.mark.parametrize("B", [7, 100])
def test_conv12_fwd(ops, B):
    """conv1 on MFMA (bf16 operands) feeding conv2 through LDS in one launch: a1 matches the fp32
    reference on bf16-rounded inputs, a2/idx2 are bitwise those of conv2_fwd on the same a1, and the
    data gather (rows + device step) picks the same images as conv1_fwd."""
    g = torch.Generator(device="cuda").manual_seed(12)
    n_pool = 300
    xs = torch.rand(n_pool, 784, device="cuda", generator=g)
    rows = torch.randperm(n_pool, device="cuda", generator=g).to(torch.int32)
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    st[0] = 2
    w1 = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
    b1 = torch.randn(32, device="cuda", generator=g) * 0.1
    w2 = bf(torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    b2 = torch.randn(64, device="cuda", generator=g) * 0.1
    a1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.bfloat16)
    idx1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8)
    a2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
    idx2 = torch.empty(B, 3136, device="cuda", dtype=torch.uint8)
    ops.conv12_fwd(xs, rows, st, w1.reshape(800).to(torch.bfloat16), b1, w2.reshape(-1), b2, a1, idx1, a2, idx2)
    xb = xs[rows[(2 * B + torch.arange(B, device="cuda")) % n_pool].long()]
    ref, rd, _ = ref_conv_pool(bf(xb).view(B, 28, 28, 1), bf(w1), b1)
    assert rel_err(a1, ref) < 5e-3
    pos = ref > 1e-2
    assert (idx1.long()[pos] == rd[pos]).float().mean() > 0.99
    a2r = torch.empty_like(a2)
    idx2r = torch.empty_like(idx2)
    ops.conv2_fwd(a1, w2.reshape(-1), b2, a2r, idx2r)
    assert torch.equal(a2, a2r) and torch.equal(idx2, idx2r)
    # same images as the fp32 VALU conv1 with the same gather
    a1v = torch.empty_like(a1)
    ops.conv1_fwd(xs, rows, st, w1.reshape(800), b1, a1v, torch.empty_like(idx1))
    assert rel_err(a1, a1v) < 1e-2


@pytest.mark.parametrize("B", [7, 100, 128])
def test_fc1_fwd(ops, B):
    g = torch.Generator(device="cuda").manual_seed(3)
    a2 = bf(torch.rand(B, 3136, device="cuda", generator=g))
    w = bf(torch.randn(3136, 1024, device="cuda", generator=g) * 0.02)
    zp = torch.empty(FC1_KS, B, 1024, device="cuda")
    ops.fc1_fwd(a2.to(torch.bfloat16), w.to(torch.bfloat16), zp)
    assert rel_err(zp.sum(0), a2 @ w) < 1e-4


def test_head_no_dropout(ops):
    B = 100
    g = torch.Generator(device="cuda").manual_seed(4)
    zp = torch.randn(FC1_KS, B, 1024, device="cuda", generator=g) * 0.1
    b3 = torch.randn(1024, device="cuda", generator=g) * 0.1
    w4 = torch.randn(1024, 10, device="cuda", generator=g) * 0.05
    b4 = torch.randn(10, device="cuda", generator=g) * 0.1
    y = torch.randint(0, 10, (B,), device="cuda", generator=g)
    h = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
    dz = torch.empty_like(h)
    dlog = torch.empty(B, 10, device="cuda")
    stats = torch.empty(B, 2, device="cuda")
    ops.head_fwd_bwd(zp, b3, w4, b4, y, None, None, 0, 0.0, h, dz, dlog, stats)
    z = (zp.sum(0) + b3).requires_grad_(True)
    hr = F.relu(z)
    logits = bf(hr) @ w4 + b4
    loss = F.cross_entropy(logits, y)
    loss.backward()
    assert rel_err(h, hr) < 5e-3
    assert abs(stats[:, 0].mean().item() - loss.item()) < 1e-3
    assert rel_err(dz, z.grad) < 1e-2
    assert stats[:, 1].mean().item() == pytest.approx((logits.argmax(1) == y).float().mean().item(), abs=0.02)
    # stats_acc (Keras fit's epoch metrics): each launch adds its per-sample (loss, correct) in place
    acc = torch.zeros(B, 2, device="cuda")
    for _ in range(2):
        ops.head_fwd_bwd(zp, b3, w4, b4, y, None, None, 0, 0.0, h, dz, dlog, stats, stats_acc=acc)
    assert torch.allclose(acc, 2 * stats, rtol=1e-6, atol=1e-6)


def test_head_dropout_rate(ops):
    B = 100
    zp = torch.ones(FC1_KS, B, 1024, device="cuda")
    h = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
    dz, dlog, stats = torch.empty_like(h), torch.empty(B, 10, device="cuda"), torch.empty(B, 2, device="cuda")
    st = torch.zeros(4, device="cuda", dtype=torch.int64)
    args = (torch.zeros(1024, device="cuda"), torch.zeros(1024, 10, device="cuda"), torch.zeros(10, device="cuda"),
            torch.zeros(B, device="cuda", dtype=torch.int64), None, st, 123, 0.5)
    ops.head_fwd_bwd(zp, *args, h, dz, dlog, stats)
    keep = (h.float() > 0).float()
    assert abs(keep.mean().item() - 0.5) < 0.01
    assert torch.allclose(h.float()[h.float() > 0], torch.full_like(h.float()[h.float() > 0], 2.0 * FC1_KS))  # slabs of 1, x2 (dropout)
    h2 = torch.empty_like(h)
    ops.head_fwd_bwd(zp, *args, h2, dz, dlog, stats)
    # head advances only the optimizer counter (state[1]); the mask is keyed on state[0]
    assert torch.equal(h, h2) and int(st[1]) == 2 and int(st[0]) == 0


def test_dropout_mask_depends_on_forward_step(ops):
    B = 16
    zp = torch.ones(FC1_KS, B, 1024, device="cuda")
    st = torch.zeros(4, device="cuda", dtype=torch.int64)
    outs = []
    for step in (0, 0, 1):
        st[0] = step
        h = torch.empty(B, 1024, device="cuda", dtype=torch.bfloat16)
        ops.head_fwd_bwd(zp, torch.zeros(1024, device="cuda"), torch.zeros(1024, 10, device="cuda"),
                         torch.zeros(10, device="cuda"), torch.zeros(B, device="cuda", dtype=torch.int64), None, st, 5, 0.5,
                         h, torch.empty_like(h), torch.empty(B, 10, device="cuda"), torch.empty(B, 2, device="cuda"))
        outs.append(h)
    assert torch.equal(outs[0], outs[1]) and not torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("B", [7, 100])
def test_fc1_bwd(ops, B):
    g = torch.Generator(device="cuda").manual_seed(5)
    dz = bf(torch.randn(B, 1024, device="cuda", generator=g) * 0.01)
    w3 = bf(torch.randn(3136, 1024, device="cuda", generator=g) * 0.02)
    a2 = bf(F.relu(torch.randn(B, 3136, device="cuda", generator=g)))
    h = bf(F.relu(torch.randn(B, 1024, device="cuda", generator=g)))
    dlog = torch.randn(B, 10, device="cuda", generator=g) * 0.01
    gW3 = torch.empty(3136, 1024, device="cuda")
    gb3, gW4, gb4 = torch.empty(1024, device="cuda"), torch.empty(1024, 10, device="cuda"), torch.empty(10, device="cuda")
    ops.fc1_wgrad(dz.to(torch.bfloat16), a2.to(torch.bfloat16), h.to(torch.bfloat16), dlog, gW3, gb3, gW4, gb4)
    g2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
    ops.fc1_dgrad(dz.to(torch.bfloat16), w3.to(torch.bfloat16), a2.to(torch.bfloat16), g2)
    assert rel_err(g2, (dz @ w3.t()) * (a2 > 0)) < 5e-3
    assert rel_err(gW3, a2.t() @ dz) < 1e-4
    # dW3 over gathered factors (K = 3 ranks x B rows, streamed through LDS in 128-row chunks)
    K = 3 * B
    dzk = bf(torch.randn(K, 1024, device="cuda", generator=g) * 0.01)
    a2k = bf(F.relu(torch.randn(K, 3136, device="cuda", generator=g)))
    gW3k = torch.empty_like(gW3)
    ops.fc1_wgrad(dz.to(torch.bfloat16), a2.to(torch.bfloat16), h.to(torch.bfloat16), dlog, gW3k, gb3, gW4, gb4, 1,
                  dzk.to(torch.bfloat16), a2k.to(torch.bfloat16))
    assert rel_err(gW3k, a2k.t() @ dzk) < 1e-4
    assert rel_err(gb3, dz.sum(0)) < 1e-4
    assert rel_err(gW4, h.t() @ dlog) < 1e-4
    assert rel_err(gb4, dlog.sum(0)) < 1e-4
    # the one-launch fc1_bwd runs the same block code: bitwise equal to the two launches
    ops.fc1_wgrad(dz.to(torch.bfloat16), a2.to(torch.bfloat16), h.to(torch.bfloat16), dlog, gW3, gb3, gW4, gb4)
    outs = [torch.full_like(t, float("nan")) for t in (gW3, gb3, gW4, gb4)]
    g2m = torch.empty_like(g2)
    ops.fc1_bwd(dz.to(torch.bfloat16), a2.to(torch.bfloat16), h.to(torch.bfloat16), dlog, w3.to(torch.bfloat16),
                *outs, g2m, 3)
    assert torch.equal(g2m, g2)
    for a, b in zip(outs, (gW3, gb3, gW4, gb4)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [7, 100])
def test_conv2_bwd_fused_conv1_wgrad(ops, B):
    g = torch.Generator(device="cuda").manual_seed(6)
    # Build consistent forward state with the kernels themselves, then compare the backward.
    x = torch.rand(B, 784, device="cuda", generator=g)
    w1 = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
    b1 = torch.randn(32, device="cuda", generator=g) * 0.05
    w2 = bf(torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05)
    b2 = torch.randn(64, device="cuda", generator=g) * 0.05
    a1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.bfloat16)
    idx1 = torch.empty_like(a1, dtype=torch.uint8)
    ops.conv1_fwd(x, None, None, w1.reshape(800), b1, a1, idx1)
    a2 = torch.empty(B, 3136, device="cuda", dtype=torch.bfloat16)
    idx2 = torch.empty_like(a2, dtype=torch.uint8)
    ops.conv2_fwd(a1, w2.to(torch.bfloat16).reshape(-1), b2, a2, idx2)
    dA2 = torch.randn(B, 3136, device="cuda", generator=g) * 0.01
    g2 = (dA2 * (a2.float() > 0)).to(torch.bfloat16)  # what fc1_dgrad hands to conv2_bwd
    G = int(ops.conv2_wgrad_groups(B))
    g1 = torch.empty_like(a1)
    slab = torch.empty(G, 51200, device="cuda")
    gb2, gW1, gb1, gW2 = (torch.empty(64, device="cuda"), torch.empty(800, device="cuda"),
                          torch.empty(32, device="cuda"), torch.empty(51200, device="cuda"))
    cpart = torch.full((B, 896), float("nan"), device="cuda")  # every entry must be written
    ops.conv2_bwd(g2, idx2, a1, w2.to(torch.bfloat16).reshape(-1), x, None, None, idx1, slab, cpart, g1)
    ops.conv2_wgrad_reduce(slab, cpart, B, gW2, gW1, gb1, gb2)
    # Reference: autograd through conv2 (+relu+pool) on the same bf16 a1, and conv1 on fp32 x.
    a1r = a1.float().requires_grad_(True)
    w2r = w2.clone().requires_grad_(True)
    b2r = b2.clone().requires_grad_(True)
    p2, _, _ = ref_conv_pool(a1r, w2r, b2r)
    p2.reshape(B, 3136).backward(g2.float())
    assert rel_err(gW2.view(5, 5, 32, 64), w2r.grad) < 1e-2
    assert rel_err(gb2, b2r.grad) < 1e-3
    g1_ref = a1r.grad * (a1.float() > 0)
    assert rel_err(g1, g1_ref) < 1e-2
    w1r = w1.clone().requires_grad_(True)
    b1r = b1.clone().requires_grad_(True)
    p1, _, _ = ref_conv_pool(x.view(B, 28, 28, 1), w1r, b1r)
    p1.backward(g1.float())
    # the fused conv1 wgrad feeds the MFMA with the input image in bf16 (rel. rounding 2^-9), the reference
    # keeps fp32 x: a few 1e-3 of relative difference
    assert rel_err(gW1.view(5, 5, 1, 32), w1r.grad) < 5e-3
    assert rel_err(gb1, b1r.grad) < 1e-3


def test_adam_matches_tf_rule(ops):
    from mihvd.optim import TFAdam

    n = 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    p0 = torch.randn(n, device="cuda", generator=g)
    p, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    pr = torch.nn.Parameter(p0.clone())
    opt = TFAdam([pr], lr=1e-2)
    for t in range(1, 4):
        grad = torch.randn(n, device="cuda", generator=g)
        ops.adam_step(p, grad * 2, m, v, sh, None, t, 1e-2, 0.9, 0.999, 1e-8, 0.5, 0)
        pr.grad = grad.clone()
        opt.step()
    assert torch.allclose(p, pr.detach(), atol=1e-6, rtol=1e-5)
    assert torch.equal(sh, p.to(torch.bfloat16))


class _RoundBF(torch.autograd.Function):
    """bf16 storage point: round the value forward and the gradient backward."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


class _RoundFwd(torch.autograd.Function):
    """bf16 weight shadow: rounded forward, fp32 (master) gradient backward."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g


def _pool_by_index(y_nhwc, idx):
    """Max-pool routed by the kernel's argmax (d = 2*dy + dx), differentiable."""
    B, H, W, C = y_nhwc.shape
    y = y_nhwc.reshape(B, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(B, H // 2, W // 2, C, 4)
    return y.gather(-1, idx.long().unsqueeze(-1)).squeeze(-1)


def _emulated_reference(params, x, y, idx1, idx2, conv1_bf16=False):
    """The fused step's exact math in fp32 autograd: same bf16 rounding points, same pool routing
    (conv1_bf16: conv1 reads bf16-rounded images and weights, as the one-launch conv12 does)."""
    P = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    B = x.shape[0]
    w1 = P["conv_layer1/conv2d/kernel"]
    if conv1_bf16:
        x, w1 = bf(x), _RoundFwd.apply(w1)
    y1 = F.conv2d(x.view(B, 1, 28, 28), w1.permute(3, 2, 0, 1), P["conv_layer1/conv2d/bias"],
                  padding=2).permute(0, 2, 3, 1)
    a1 = _RoundBF.apply(F.relu(_pool_by_index(y1, idx1)))
    w2 = _RoundFwd.apply(P["conv_layer2/conv2d/kernel"])
    y2 = F.conv2d(a1.permute(0, 3, 1, 2), w2.permute(3, 2, 0, 1), P["conv_layer2/conv2d/bias"], padding=2)
    a2 = _RoundBF.apply(F.relu(_pool_by_index(y2.permute(0, 2, 3, 1), idx2.view(B, 7, 7, 64)))).reshape(B, 3136)
    z = a2 @ _RoundFwd.apply(P["dense/kernel"]) + P["dense/bias"]
    h = _RoundBF.apply(F.relu(z))
    logits = h @ P["dense_1/kernel"] + P["dense_1/bias"]
    loss = F.cross_entropy(logits, y)
    loss.backward()
    return loss.detach(), {k: v.grad for k, v in P.items()}


@pytest.mark.parametrize("B", [8, 100])
def test_fused_step_matches_emulated_reference(ops, B):
    """One fused step (dropout off, lr 0): loss and every gradient equal an fp32 autograd
    reference with the same bf16 storage points and pool routing; the loss is also within
    mixed-precision distance of the pure fp32 model."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.models.mnist import MNISTConvNet, TF_PARAM_ORDER

    tr = FusedMNISTTrainer(batch_size=B, lr=0.0, dropout=0.0, seed=3, device="cuda", precision="bf16")
    tr.keep_w3_grad = True  # dW3 is consumed by the fused W3 Adam; also store it for the comparison
    g = torch.Generator(device="cuda").manual_seed(8)
    x = torch.rand(B, 784, device="cuda", generator=g)
    y = torch.randint(0, 10, (B,), device="cuda", generator=g)
    params = {n: tr.pview(n).clone() for n in TF_PARAM_ORDER}
    out = tr.train_step(x, y)
    torch.cuda.synchronize()
    loss, grads = _emulated_reference(params, x, y, tr.idx1, tr.idx2, conv1_bf16=True)
    assert abs(out["loss"].item() - loss.item()) < 1e-3 * max(1.0, loss.item())
    for name in TF_PARAM_ORDER:
        e = rel_err(tr.gview(name), grads[name])
        assert e < 1e-2, (name, e)
    ref = MNISTConvNet(impl="torch", seed=3).cuda().eval()
    assert abs(F.cross_entropy(ref(x), y).item() - loss.item()) < 2e-2 * max(1.0, loss.item())


def test_fused_training_converges_and_graph_replays(ops):
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    (x, y), _ = synthetic_mnist(n_train=3000, n_test=10, seed=5)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=100, lr=1e-3, seed=0, device="cuda", precision="bf16")
    tr.set_device_dataset(X, Y)
    assert tr.build_graph(steps_per_replay=10)
    first = None
    for i in range(30):
        tr.run_graph()
        if first is None:
            first = tr.last_loss()
    torch.cuda.synchronize()
    assert tr.global_step == 2 + 300
    assert int(tr.state[0].item()) == tr.global_step and int(tr.state[1].item()) == tr.global_step
    assert tr.last_loss() < first * 0.5, (first, tr.last_loss())
    assert tr.last_accuracy() > 0.8


def test_fused_loss_autograd_matches_trainer(ops):
    """ops.functional.fused_mnist_loss (one autograd node) gives the trainer's gradients, and the
    HIP inference logits agree with the torch model."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.models.mnist import MNISTConvNet
    from mihvd.ops.functional import fused_mnist_loss, mnist_logits

    B = 64
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.rand(B, 784, device="cuda", generator=g)
    y = torch.randint(0, 10, (B,), device="cuda", generator=g)
    model = MNISTConvNet(impl="hip", seed=3).cuda()
    loss, acc = fused_mnist_loss(model, x, y, training=False, return_accuracy=True)
    loss.backward()
    tr = FusedMNISTTrainer(batch_size=B, lr=0.0, dropout=0.0, seed=3, device="cuda", precision="bf16")
    tr.keep_w3_grad = True
    out = tr.train_step(x, y)
    torch.cuda.synchronize()
    assert abs(loss.item() - out["loss"].item()) < 1e-5
    for name, p in model.ordered_parameters():
        assert rel_err(p.grad, tr.gview(name)) < 1e-3, name
    ref = MNISTConvNet(impl="torch", seed=3).cuda().eval()
    with torch.no_grad():
        assert rel_err(mnist_logits(model, x), ref(x)) < 2e-2


def test_adasum_hip_matches_torch(ops):
    """dp_kernels.hip segment_dots + adasum_combine vs the fp64 torch formulation (incl. gaps and
    segments that are not float4-aligned)."""
    from mihvd.parallel import adasum

    g = torch.Generator(device="cuda").manual_seed(11)
    n = 3 * 8192 + 37
    a = torch.randn(n, device="cuda", generator=g)
    b = torch.randn(n, device="cuda", generator=g) * 0.3 + 0.5 * a
    segs = [(0, 5), (5, 9000), (9003, 20001), (20001, n - 10)]  # gaps at 9000..9003 and the tail
    a[9000:9003] = 0
    b[9000:9003] = 0
    out = adasum.adasum_pair(a, b, segs)
    ref = adasum.adasum_pair(a.cpu(), b.cpu(), segs)
    assert rel_err(out.cpu(), ref) < 1e-6
    # zero-norm rules: |a| = 0 -> b
    z = torch.zeros_like(a)
    assert torch.equal(adasum.adasum_pair(z, b), b)
    # misaligned views take the scalar paths
    out2 = adasum.adasum_pair(a[1:], b[1:])
    assert rel_err(out2.cpu(), adasum.adasum_pair(a[1:].cpu(), b[1:].cpu())) < 1e-6


def test_loss_scale_kernels(ops):
    grads = [torch.full((1000,), 8.0, device="cuda"), torch.full((33,), -4.0, device="cuda")]
    ls = torch.tensor([4.0, 0.0], device="cuda")
    tracker = torch.zeros(1, dtype=torch.int32, device="cuda")
    ops.grad_check_(grads, ls, True)
    assert float(ls[1]) == 0.0 and torch.all(grads[0] == 2.0) and torch.all(grads[1] == -1.0)
    ops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
    assert float(ls[0]) == 4.0 and int(tracker) == 1
    ops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
    assert float(ls[0]) == 8.0 and int(tracker) == 0
    grads[1][7] = float("inf")
    ops.grad_check_(grads, ls, False)
    assert float(ls[1]) == 1.0
    ops.update_scale_(ls, tracker, 2.0, 0.5, 2, 1.0)
    assert float(ls[0]) == 4.0 and float(ls[1]) == 0.0


def test_adam_loss_scale_fused(ops):
    n = 4096
    g = torch.Generator(device="cuda").manual_seed(12)
    p0 = torch.randn(n, device="cuda", generator=g)
    gr = torch.randn(n, device="cuda", generator=g)
    outs = []
    for scale, found in ((1.0, 0.0), (8.0, 0.0), (8.0, 1.0)):
        p, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        ls = torch.tensor([scale, found], device="cuda")
        ops.adam_step(p, gr * scale, m, v, None, None, 1, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0, 0, ls)
        outs.append(p)
    assert torch.allclose(outs[0], outs[1], atol=1e-7)
    assert torch.equal(outs[2], p0)  # overflow step skipped


@pytest.mark.parametrize("K", [200, 237, 400, 513, 800])
def test_fc1_wgrad_long_k_two_group_tiles(ops, K):
    """dW3 over a long K (the all-gathered factors of N ranks: Kw = N*B > 128) runs as K-split group
    tiles (K chunks split between two — or, from five chunks on, four — 4-wave groups, partial tiles
    combined in a fixed order):
    close to the fp32 product, a row slice [lo, hi) reproduces those rows of the full range bit for
    bit (sharded and replicated optimizers agree), and the fused Adam epilogue equals adam_step on
    the stored gradient bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(K)
    B = 100
    bf = torch.bfloat16
    dz = torch.randn(B, 1024, device="cuda", generator=g).to(bf)
    a2 = torch.rand(B, 3136, device="cuda", generator=g).to(bf)
    h = torch.rand(B, 1024, device="cuda", generator=g).to(bf)
    dlog = torch.randn(B, 10, device="cuda", generator=g)
    dzw = torch.randn(K, 1024, device="cuda", generator=g).to(bf)
    a2w = torch.rand(K, 3136, device="cuda", generator=g).to(bf)
    small = [torch.zeros(n, device="cuda") for n in (1024, 10240, 10)]

    def wgrad(lo=0, hi=49):
        out = torch.zeros(3136 * 1024, device="cuda")
        ops.fc1_wgrad(dz, a2, h, dlog, out, *small, 1, dzw, a2w, lo, hi)
        return out.view(3136, 1024)

    full = wgrad()
    ref = a2w.float().t() @ dzw.float()
    assert ((full - ref).norm() / ref.norm()).item() < 1e-5
    part = wgrad(7, 14)
    assert not part[:448].any() and not part[896:].any()
    # a 13-row-tile slice (the 4-rank shard: 208 64-feature tiles) takes the 64-feature group tiles
    sl = wgrad(21, 34)
    assert ((sl[1344:2176] - ref[1344:2176]).norm() / ref[1344:2176].norm()).item() < 1e-5
    assert not sl[:1344].any() and not sl[2176:].any()
    if K <= 3 * 128:
        assert torch.equal(part[448:896], full[448:896])  # same group count: bit for bit
        assert torch.equal(sl[1344:2176], full[1344:2176])
    else:
        # a slice of at most one tile per CU runs four K groups from four chunks on (the sharded
        # optimizer's rows), all 784 tiles two: same rows, last bits may differ; both close to fp32
        assert ((part[448:896] - ref[448:896]).norm() / ref[448:896].norm()).item() < 1e-5
        assert torch.equal(part[448:896], wgrad(7, 14)[448:896])  # deterministic
    # fused Adam on a row slice == adam_step on that slice's stored gradient, bit for bit
    n3 = 3136 * 1024
    ps = torch.randn(n3, device="cuda", generator=g)
    ms = torch.randn(n3, device="cuda", generator=g).abs() * 1e-3
    vs = torch.rand(n3, device="cuda", generator=g) * 1e-4
    sts = torch.tensor([0, 2, 0, 0], device="cuda", dtype=torch.int64)
    ps2, ms2, vs2 = ps.clone(), ms.clone(), vs.clone()
    shs, shs2 = torch.zeros(n3, device="cuda", dtype=bf), torch.zeros(n3, device="cuda", dtype=bf)
    gs = torch.zeros(n3, device="cuda")
    ops.fc1_wgrad_adam(dz, a2, h, dlog, gs, *small, 1, dzw, a2w, ps, ms, vs, shs, sts, 1e-3, 0.9, 0.999, 1e-8, 0.125,
                       0, True, 7, 14)
    r0, r1 = 448 * 1024, 896 * 1024
    assert torch.equal(gs[r0:r1], part.reshape(-1)[r0:r1])
    ops.adam_step(ps2[r0:r1], gs[r0:r1], ms2[r0:r1], vs2[r0:r1], shs2[r0:r1], sts, 0, 1e-3, 0.9, 0.999, 1e-8, 0.125,
                  0, 0)
    torch.cuda.synchronize()
    assert torch.equal(ps, ps2) and torch.equal(ms, ms2) and torch.equal(vs, vs2)
    assert torch.equal(shs[r0:r1], shs2[r0:r1])
    n = 3136 * 1024
    p = torch.randn(n, device="cuda", generator=g)
    m = torch.randn(n, device="cuda", generator=g).abs() * 1e-3
    v = torch.rand(n, device="cuda", generator=g) * 1e-4
    st = torch.tensor([0, 3, 0, 0], device="cuda", dtype=torch.int64)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    sh = torch.empty(n, device="cuda", dtype=bf)
    sh2 = torch.empty_like(sh)
    gst = torch.zeros(n, device="cuda")
    ops.fc1_wgrad_adam(dz, a2, h, dlog, gst, *small, 1, dzw, a2w, p, m, v, sh, st, 1e-3, 0.9, 0.999, 1e-8, 0.125, 0,
                       True)
    ops.adam_step(p2, full.reshape(-1), m2, v2, sh2, st, 0, 1e-3, 0.9, 0.999, 1e-8, 0.125, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(gst, full.reshape(-1))
    assert torch.equal(p, p2) and torch.equal(m, m2) and torch.equal(v, v2) and torch.equal(sh, sh2)


@pytest.mark.parametrize("B", [8, 100])
def test_conv2_bwd_adam_tail_covers_slice(ops, B):
    """The tail covers every float4 of the slice exactly once (any B, any grid), including a slice
    length that is not a multiple of the 1024-element wave group."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer

    tr = FusedMNISTTrainer(batch_size=B, seed=2, device="cuda", precision="bf16", dropout=0.0)
    x = torch.rand(B, 784, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    tr.train_step(x, y)
    torch.cuda.synchronize()
    n = 1024 * 37 + 12
    gen = torch.Generator(device="cuda").manual_seed(3)
    p = torch.randn(n, device="cuda", generator=gen)
    gr = torch.randn(n, device="cuda", generator=gen)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    st = tr.state.clone()
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    ops.adam_step(pr, gr, mr, vr, None, st, 0, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0, 0)
    ops.conv2_bwd_adam(tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", tr.shadow), tr.x_buf, None, st,
                       tr.idx1, tr.slab, tr.cpart, p, gr, m, v, sh, 1e-3, 0.9, 0.999, 1e-8, 1.0, 0)
    torch.cuda.synchronize()
    assert torch.equal(p, pr) and torch.equal(m, mr) and torch.equal(v, vr)
    assert torch.equal(sh, p.to(torch.bfloat16))


def test_debug_sync_mode_matches_graph(ops, monkeypatch):
    """MIHVD_DEBUG_SYNC=1 (serialized bisection mode): eager steps with a synchronize after every
    kernel; same results as the graph-replayed step."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer

    g = torch.Generator(device="cuda").manual_seed(41)
    X = torch.rand(300, 784, device="cuda", generator=g)
    Y = torch.randint(0, 10, (300,), device="cuda", generator=g)
    out = []
    for dbg in ("0", "1"):
        monkeypatch.setenv("MIHVD_DEBUG_SYNC", dbg)
        tr = FusedMNISTTrainer(batch_size=100, seed=6, device="cuda", precision="bf16")
        tr.set_device_dataset(X, Y, shuffle=False)
        assert tr.build_graph(steps_per_replay=3, warmup=1) == (dbg == "0")
        tr.run_graph()
        torch.cuda.synchronize()
        out.append(tr.params.clone())
    assert torch.equal(out[0], out[1])


def test_gather_cols_and_column_slice_wgrad(ops):
    """gather_cols_bf16 (column slices with zero padding past K) and fc1_wgrad reading a [K][C]
    column slice of a2 for a row-tile range: equal to the full-width computation on those rows."""
    g = torch.Generator(device="cuda").manual_seed(51)
    B, N = 40, 3
    a2 = torch.randn(N * B, 3136, device="cuda", generator=g).to(torch.bfloat16)
    dz = torch.randn(N * B, 1024, device="cuda", generator=g).to(torch.bfloat16)
    T64 = 17 * 64                              # ceil(49 / 3) tiles per rank
    out = torch.empty(N, N * B, T64, device="cuda", dtype=torch.bfloat16)
    ops.gather_cols_bf16(a2, 0, out)
    for q in range(N):
        lo, hi = q * T64, min((q + 1) * T64, 3136)
        assert torch.equal(out[q, :, :hi - lo], a2[:, lo:hi])
        assert not out[q, :, hi - lo:].any()
    h = torch.zeros(B, 1024, device="cuda", dtype=torch.bfloat16)
    dlog = torch.zeros(B, 10, device="cuda")
    full = torch.zeros(3136, 1024, device="cuda")
    part = torch.zeros(3136, 1024, device="cuda")
    small = [torch.zeros(n, device="cuda") for n in (1024, 10240, 10)]
    ops.fc1_wgrad(dz[:B], a2[:B], h, dlog, full, *small, 1, dz, a2, 0, 49)
    ops.fc1_wgrad(dz[:B], a2[:B], h, dlog, part, *small, 1, dz, out[1].contiguous(), 17, 34)
    torch.cuda.synchronize()
    assert torch.equal(part[17 * 64:34 * 64], full[17 * 64:34 * 64])
    assert not part[:17 * 64].any() and not part[34 * 64:].any()
    ref = a2.float().t() @ dz.float()
    assert rel_err(full, ref) < 1e-4


@pytest.mark.parametrize("kind", ["adam", "adamw", "tf", "sgd", "nesterov"])
def test_multi_tensor_optimizers_match_torch(ops, kind):
    """multi_tensor_adam / multi_tensor_sgd (via FusedAdam / FusedSGD) vs torch.optim on GPU
    tensors of awkward sizes (not multiples of 4, > 1 chunk, > 24 tensors per launch), including a
    channels_last parameter whose gradient shares its layout."""
    from mihvd.optim import FusedAdam, FusedSGD, TFAdam

    g = torch.Generator(device="cuda").manual_seed(61)
    shapes = [(70001,), (3,), (1031, 7), (64, 32, 3, 3)] + [(257,)] * 30
    a = [torch.randn(s, device="cuda", generator=g) for s in shapes]
    a[3] = a[3].to(memory_format=torch.channels_last)
    a = [x.requires_grad_(True) for x in a]
    b = [x.detach().clone().requires_grad_(True) for x in a]
    mk = {"adam": (lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.01), lambda ps: torch.optim.Adam(ps, lr=1e-2, weight_decay=0.01)),
          "adamw": (lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.1, adamw=True), lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.1)),
          "tf": (lambda ps: FusedAdam(ps, lr=1e-2, rule="tf"), lambda ps: TFAdam(ps, lr=1e-2)),
          "sgd": (lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-3), lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-3)),
          "nesterov": (lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9, nesterov=True), lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, nesterov=True))}[kind]
    oa, ob = mk[0](a), mk[1](b)
    if kind == "tf":  # reference: TFAdam's torch foreach path, on CPU copies
        b = [x.detach().cpu().clone().requires_grad_(True) for x in b]
        ob = TFAdam(b, lr=1e-2)
    for step in range(3):
        for ps, o in ((a, oa), (b, ob)):
            o.zero_grad()
            sum((x.float() * (i + 1 + step)).cos().sum() for i, x in enumerate(ps)).backward()
            o.step()
    for x, y in zip(a, b):
        assert rel_err(x.detach().cpu(), y.detach().cpu()) < 1e-5, kind


def test_captured_step_matches_eager(ops):
    """mihvd.graphs.CapturedStep: forward + backward + DistributedOptimizer (bucketed) + FusedAdam
    captured in one HIP graph and replayed == the same steps run eagerly."""
    import mihvd.torch as hvd
    from mihvd.graphs import CapturedStep
    from mihvd.optim import FusedAdam

    hvd.init()
    try:
        torch.manual_seed(5)
        X = torch.randn(12, 64, 32, device="cuda")
        Y = torch.randn(12, 64, 4, device="cuda")

        def build():
            torch.manual_seed(1)
            m = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 4)).cuda()
            o = hvd.DistributedOptimizer(FusedAdam(m.parameters(), lr=1e-2, rule="tf"),
                                         named_parameters=m.named_parameters())
            return m, o

        m1, o1 = build()
        x = torch.zeros(64, 32, device="cuda")
        y = torch.zeros(64, 4, device="cuda")
        ctr = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step():
            i = ctr % 12
            x.copy_(X.index_select(0, i).squeeze(0))
            y.copy_(Y.index_select(0, i).squeeze(0))
            o1.zero_grad(set_to_none=False)
            loss = torch.nn.functional.mse_loss(m1(x), y)
            loss.backward()
            o1.step()
            ctr.add_(1)
            return loss

        graphed = CapturedStep(step, warmup=3)
        for _ in range(9):
            graphed()
        torch.cuda.synchronize()
        m2, o2 = build()
        for i in range(12):  # 3 warm-up steps + 9 replays (capture itself does not execute)
            o2.zero_grad(set_to_none=False)
            torch.nn.functional.mse_loss(m2(X[i % 12]), Y[i % 12]).backward()
            o2.step()
        torch.cuda.synchronize()
        assert int(ctr) == 12
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            assert torch.equal(p1, p2)
    finally:
        hvd.shutdown()


@pytest.mark.parametrize("comp", ["none", "fp16", "bf16"])
def test_captured_step_compression_survives_device_sync(ops, comp):
    """CapturedStep + DistributedOptimizer with several compressed buckets (persistent wire
    buffers, HIP pack/unpack at world size 1 too): replays, a device-wide synchronize and barrier
    (the benches' timing fence), more replays == the same steps eagerly, bitwise."""
    import mihvd.torch as hvd
    from mihvd.graphs import CapturedStep
    from mihvd.optim import FusedAdam

    hvd.init()
    try:
        C = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16, "bf16": hvd.Compression.bf16}[comp]
        torch.manual_seed(5)
        X = torch.randn(64, 128, device="cuda")
        Y = torch.randn(64, 8, device="cuda")

        def build():
            torch.manual_seed(1)
            m = torch.nn.Sequential(torch.nn.Linear(128, 256), torch.nn.GELU(), torch.nn.Linear(256, 256),
                                    torch.nn.GELU(), torch.nn.Linear(256, 8)).cuda()
            o = hvd.DistributedOptimizer(FusedAdam(m.parameters(), lr=1e-3), named_parameters=m.named_parameters(),
                                         compression=C, fusion_threshold=64 * 1024)
            return m, o

        m1, o1 = build()
        assert len(o1.buckets) >= 3

        def step():
            o1.zero_grad(set_to_none=False)
            loss = torch.nn.functional.mse_loss(m1(X), Y)
            loss.backward()
            o1.step()
            return loss

        graphed = CapturedStep(step, warmup=2)
        for _ in range(3):
            graphed()
        torch.cuda.synchronize()
        hvd.barrier()
        torch.cuda.synchronize()
        for _ in range(3):
            graphed()
        torch.cuda.synchronize()
        m2, o2 = build()
        for _ in range(8):  # 2 warm-up steps + 6 replays
            o2.zero_grad(set_to_none=False)
            torch.nn.functional.mse_loss(m2(X), Y).backward()
            o2.step()
        torch.cuda.synchronize()
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            assert torch.isfinite(p1).all()
            assert torch.equal(p1, p2)
    finally:
        hvd.shutdown()


@pytest.mark.parametrize("wire", [torch.bfloat16, torch.float16])
def test_hip_pack_unpack_matches_torch_casts(ops, wire):
    """Compression pack/unpack kernels (cast + scale fused) == torch casts then scale."""
    from mihvd.parallel.compression import Compression, hip_pack, hip_unpack

    comp = Compression.bf16 if wire == torch.bfloat16 else Compression.fp16
    g = torch.Generator(device="cuda").manual_seed(71)
    x = torch.randn(4 * 9999, device="cuda", generator=g)
    w = hip_pack(comp, x, 0.5)
    assert w.dtype == wire and torch.equal(w, (x * 0.5).to(wire))
    out = torch.empty_like(x)
    hip_unpack(w, out, 0.25)
    assert torch.equal(out, w.float() * 0.25)
