"""fp16-operand build of the MFMA kernels (csrc/kernels/common.h -DMIHVD_F16: conv_fwd / conv_bwd /
fc compiled a second time in namespace mihvd::f16 with v_mfma_f32_16x16x32_f16) — the Keras
``mixed_float16`` policy of the reference (tensorflow_mnist_gpu.py:26-28) on the HIP path.

Numerics are checked against a plain fp32 torch autograd reference of the same network (dropout
off): the fp16 kernels must land within 5 % of it and at least 2x closer than the bf16 build (3 more
mantissa bits), for any loss scale in the normal range; an oversized scale must surface as
non-finite gradients (what the dynamic loss scaler skips on), never as silently wrong ones.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mihvd import _native

    _native.require_kernels()
    assert hasattr(torch.ops.mihvd, "conv2_bwd_f16"), "kernel library built without the fp16 set"
    return torch.ops.mihvd


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _batch(B=64, seed=9):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand(B, 784, device="cuda", generator=g)
    y = torch.randint(0, 10, (B,), device="cuda", generator=g)
    return x, y


def _ref_grads(x, y, seed=3):
    from mihvd.models.mnist import MNISTConvNet

    ref = MNISTConvNet(impl="torch", seed=seed).cuda().eval()
    loss = torch.nn.functional.cross_entropy(ref(x), y)
    loss.backward()
    return loss.item(), {n: p.grad.clone() for n, p in ref.ordered_parameters()}


def _hip_grads(x, y, precision, loss_scale=None, seed=3):
    from mihvd.models.mnist import MNISTConvNet
    from mihvd.ops.functional import fused_mnist_loss

    model = MNISTConvNet(impl="hip", seed=seed).cuda()
    loss = fused_mnist_loss(model, x, y, training=False, precision=precision, loss_scale=loss_scale)
    loss.backward()
    return loss.item(), {n: p.grad.clone() for n, p in model.ordered_parameters()}


def test_f16_grads_match_fp32_reference(ops):
    x, y = _batch()
    l_ref, g_ref = _ref_grads(x, y)
    l16, g16 = _hip_grads(x, y, "fp16")
    lbf, gbf = _hip_grads(x, y, "bf16")
    assert abs(l16 - l_ref) < 2e-3 * max(1.0, abs(l_ref)), (l16, l_ref)
    e16 = {n: rel_err(g16[n], g_ref[n]) for n in g_ref}
    ebf = {n: rel_err(gbf[n], g_ref[n]) for n in g_ref}
    print("rel err fp16 / bf16 vs fp32:", {n: (round(e16[n], 5), round(ebf[n], 5)) for n in g_ref})
    # Both 16-bit builds differ from fp32 mostly through ReLU masks that flip where a pre-activation
    # sits within operand rounding of 0 (each flip moves a whole gradient row), so the relative
    # errors are percent-level; fp16's 10 mantissa bits (bf16: 7) cut them ~4x (MI355X: 1.6-3.1 %
    # against 6.5-10.6 %; the fc2 gradients, from the fp32 dlog, 0.01-0.06 %).
    for n in g_ref:
        assert torch.isfinite(g16[n]).all(), n
        assert e16[n] < 5e-2, (n, e16[n])
        assert e16[n] <= 0.5 * ebf[n] + 1e-4, (n, e16[n], ebf[n])


@pytest.mark.parametrize("S", [2.0 ** 8, 2.0 ** 15])
def test_f16_loss_scale_is_transparent(ops, S):
    """The kernels scale dz by S and the node divides it back out: the gradients do not depend on
    S (beyond fp16 rounding) and the loss not at all."""
    x, y = _batch(seed=21)
    l_ref, g_ref = _ref_grads(x, y)
    l16, g16 = _hip_grads(x, y, "fp16", loss_scale=S)
    assert abs(l16 - l_ref) < 2e-3 * max(1.0, abs(l_ref))
    for n in g_ref:
        assert rel_err(g16[n], g_ref[n]) < 5e-2, (n, S)


def test_f16_overflow_surfaces_as_nonfinite(ops):
    """dz x S past fp16's 65504 becomes inf in the kernels' 16-bit intermediates: every gradient
    derived from dz turns non-finite (what the loss scaler checks), dW4/db4 (fp32 dlog) stay finite."""
    x, y = _batch(seed=5)
    _, g = _hip_grads(x, y, "fp16", loss_scale=2.0 ** 40)
    bad = [n for n in g if not torch.isfinite(g[n]).all()]
    assert any(n.startswith("dense/kernel") for n in bad), bad
    assert torch.isfinite(g["dense_1/kernel"]).all() and torch.isfinite(g["dense_1/bias"]).all()


def test_keras_mixed_float16_trains_on_f16_kernels(ops):
    """hvd.Model(policy="mixed_float16") on an impl="hip" module: fp16 kernels + dynamic loss scaler;
    an overflowing first scale is halved and the step skipped, then training converges."""
    import mihvd.keras as K
    from mihvd.models.mnist import MNISTConvNet

    torch.manual_seed(0)
    module = MNISTConvNet(impl="hip", seed=1).cuda()
    m = K.Model(module, policy="mixed_float16")
    assert module.hip_precision == "fp16"
    opt = torch.optim.Adam(module.parameters(), lr=1e-3)
    opt.synchronize = lambda: None
    import contextlib

    opt.skip_synchronize = contextlib.nullcontext
    m.compile(opt, torch.nn.functional.cross_entropy)
    m._scaler = K._LossScaler(init_scale=2.0 ** 40, growth_interval=10 ** 6)
    x, y = _batch(B=100, seed=4)
    before = [p.detach().clone() for p in module.parameters()]
    m.train_on_batch(x, y)  # overflows: skipped, scale halved
    assert all(torch.equal(a, p) for a, p in zip(before, module.parameters()))
    assert float(m._scaler.scale) == 2.0 ** 39
    m._scaler._ls[0] = 2.0 ** 15
    first = None
    for _ in range(60):
        loss, acc = m.train_on_batch(x, y)
        first = first if first is not None else float(loss)
    assert float(loss) < 0.5 * first, (first, float(loss))
    assert all(torch.isfinite(p).all() for p in module.parameters())


def test_fused_trainer_fp16_matches_the_autograd_path_and_replays(ops):
    """FusedMNISTTrainer(precision="fp16"): the mixed_float16 step with the loss scaler on the device.
    One eager step lands where the per-batch fp16 autograd path + TF1 Adam lands (same kernels, same
    scale; only where the 1/S is applied differs), then 5 x 10-step graph replays train on."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.models.mnist import MNISTConvNet
    from mihvd.ops.functional import fused_mnist_loss
    from mihvd.optim import TFAdam

    x, y = _batch(B=100, seed=4)
    tr = FusedMNISTTrainer(batch_size=100, lr=1e-3, seed=1, dropout=0.0, device="cuda", precision="fp16")
    assert tr.f16 and tr.shadow.dtype == torch.float16 and float(tr.loss_scale[0]) == 2.0 ** 15
    ref = MNISTConvNet(impl="hip", seed=1).cuda()
    ref.dropout_rate = 0.0
    p0 = torch.cat([p.detach().reshape(-1).clone() for _, p in ref.ordered_parameters()])
    opt = TFAdam(ref.parameters(), lr=1e-3)
    loss = fused_mnist_loss(ref, x, y, training=True, precision="fp16", loss_scale=2.0 ** 15)
    loss.backward()
    opt.step()
    out = tr.train_step(x, y)
    assert abs(float(out["loss"]) - float(loss)) < 1e-3 * max(1.0, abs(float(loss)))
    got = torch.cat([tr.pview(n).reshape(-1) for n, _ in ref.ordered_parameters()])
    want = torch.cat([p.detach().reshape(-1) for _, p in ref.ordered_parameters()])
    # one TF1-Adam step is ~ -lr * sign(g): only near-zero gradients (rounding-order differences of
    # the two wgrad reductions) can move differently
    assert rel_err(got - p0, want - p0) < 1e-2, rel_err(got - p0, want - p0)
    assert int(tr.state[1]) == 1 and float(tr.loss_scale[1]) == 0.0
    X = torch.rand(2000, 784, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7))
    Y = (X[:, :392].sum(1) > X[:, 392:].sum(1)).long() * 3  # a learnable two-class labelling
    tr.set_device_dataset(X, Y)
    assert tr.build_graph(steps_per_replay=10, warmup=1)
    first = tr.last_loss()
    for _ in range(5):
        tr.run_graph()
    last = tr.last_loss()
    assert last == last and last < first, (first, last)
    assert torch.isfinite(tr.params).all() and 2.0 ** 10 <= float(tr.loss_scale[0]) <= 2.0 ** 15


def test_fused_trainer_fp16_skips_overflowing_steps_on_the_device(ops):
    """An oversized loss scale overflows the fp16 backward: the step is skipped (parameters and Adam
    slots untouched, the optimizer step taken back), the scale halves -- all inside the step's
    launches, so a graph replay does the same -- and training then proceeds."""
    from mihvd.models.fused_mnist import FusedMNISTTrainer

    x, y = _batch(B=100, seed=5)
    tr = FusedMNISTTrainer(batch_size=100, lr=1e-3, seed=2, device="cuda", precision="fp16")
    tr.loss_scale[0] = 2.0 ** 60
    p0, m0 = tr.params.clone(), tr.m.clone()
    tr.train_step(x, y)
    torch.cuda.synchronize()
    assert torch.equal(tr.params, p0) and torch.equal(tr.m, m0)
    assert float(tr.loss_scale[0]) == 2.0 ** 59 and float(tr.loss_scale[1]) == 0.0
    assert int(tr.state[1]) == 0 and int(tr.state[0]) == 1  # no optimizer step; the forward step advanced
    tr.loss_scale[0] = 2.0 ** 15
    tr.train_step(x, y)
    torch.cuda.synchronize()
    assert not torch.equal(tr.params, p0) and int(tr.state[1]) == 1


def test_keras_mixed_float16_fit_is_graph_replayed(ops):
    """hvd.Model.fit under mixed_float16 drives the fused fp16 trainer (no per-batch autograd node):
    the loss falls over the epochs and the device loss scale comes back into the model's scaler."""
    import mihvd.keras as K
    from mihvd.models.mnist import MNISTConvNet
    from mihvd.optim import TFAdam

    module = MNISTConvNet(impl="hip", seed=1).cuda()
    m = K.Model(module, policy="mixed_float16")
    m.compile(TFAdam(module.parameters(), lr=1e-3), torch.nn.functional.cross_entropy)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(3000, 784, generator=g)
    y = (x[:, :392].sum(1) > x[:, 392:].sum(1)).long() * 7
    m.fit(x.numpy(), y.numpy(), batch_size=100, epochs=3, verbose=0)
    assert getattr(m, "fused_trainer", None) is not None and m.fused_trainer.f16
    assert m.history["loss"][-1] < m.history["loss"][0], m.history
    import math

    assert math.isfinite(float(m._scaler.scale)) and float(m._scaler.scale) >= 1.0
