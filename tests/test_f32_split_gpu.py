"""Split-bf16 products of the fp32 step (f32_common.h "x9"; f32_products(1)).

Every fp32 operand is split EXACTLY into three bf16 parts and the nine part products accumulate in
fp32 on v_mfma_f32_16x16x32_bf16, so each product is exact, as on the fp32-input MFMA; only the
summation order differs. The check is against a float64 reference: the split kernels' error must be
of the fp32 kernels' size (fp32 accumulation), never of bf16's (2^-8)."""
import pytest
import torch

from test_f32_gpu import ref_conv_pool, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from mihvd import _native

    _native.require_kernels()
    return torch.ops.mihvd


def _frag(ops, B, w):
    frag = torch.empty(2, 51200, device="cuda")
    ops.f32_conv1_fwd(torch.zeros(B, 784, device="cuda"), None, None, torch.zeros(800, device="cuda"),
                      torch.zeros(32, device="cuda"), torch.empty(B, 14, 14, 32, device="cuda"),
                      torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8), w.view(-1), frag)
    return frag


@pytest.mark.parametrize("nprod", [9, 6])
@pytest.mark.parametrize("B", [7, 100, 128])
def test_split_conv2_fwd_is_fp32_accurate(ops, B, nprod):
    g = torch.Generator(device="cuda").manual_seed(12)
    a1 = torch.rand(B, 14, 14, 32, device="cuda", generator=g)
    w = torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05
    b = torch.randn(64, device="cuda", generator=g) * 0.1
    frag = _frag(ops, B, w)
    out = {}
    for mode in (0, nprod):
        a2 = torch.full((B, 3136), float("nan"), device="cuda")
        idx = torch.empty(B, 3136, device="cuda", dtype=torch.uint8)
        ops.f32_conv2_fwd(a1, w, b, a2, idx, w2frag=frag[0], products=mode)
        out[mode] = (a2, idx)
    ref, rd = ref_conv_pool(a1.double(), w.double(), b.double())
    ref, rd = ref.reshape(B, 3136), rd.reshape(B, 3136)
    e_native, e_split = rel_err(out[0][0], ref), rel_err(out[nprod][0], ref)
    print(f"B={B} rel err vs fp64: fp32 MFMA {e_native:.3e}, split-bf16 x{nprod} {e_split:.3e}")
    assert torch.isfinite(out[nprod][0]).all()
    assert e_split < 1e-6 and e_split <= 2.0 * e_native + 1e-8, (e_native, e_split)
    pos = ref > 1e-4
    assert (out[nprod][1].long()[pos] == rd[pos]).float().mean() > 0.999


@pytest.mark.parametrize("nprod", [6, 9])
@pytest.mark.parametrize("B", [7, 100, 128])
def test_split_conv2_bwd_dgrad_is_fp32_accurate(ops, B, nprod):
    """conv2_bwd with the split-bf16 dgrad role (its own block counts: up to 12-tile dgrad blocks, the
    wgrad role on the CUs left): dW1 / db1 from the routed dA1 and dW2 / db2, against float64 autograd
    of conv1 -> pool -> conv2; errors of the fp32-input MFMA launch's size or smaller."""
    import torch.nn.functional as F

    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(B, 784, device="cuda", generator=g)
    w1 = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
    b1 = torch.randn(32, device="cuda", generator=g) * 0.1
    w2 = torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05
    a1 = torch.empty(B, 14, 14, 32, device="cuda")
    idx1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8)
    ops.f32_conv1_fwd(x, None, None, w1.reshape(800), b1, a1, idx1)
    dY2 = torch.randn(B, 14, 14, 64, device="cuda", generator=g)
    db2p = torch.randn(int(ops.f32_db2_rows(B)), 64, device="cuda", generator=g)
    got = {}
    for mode in (0, nprod):
        cpart = torch.full((int(ops.f32_dgrad_blocks(B, mode)), 832), float("nan"), device="cuda")
        slab = torch.full((int(ops.f32_wgrad_groups(B, mode)), 51200), float("nan"), device="cuda")
        ops.f32_conv2_bwd(dY2, w2, a1, idx1, x, None, None, cpart, slab, products=mode)
        outs = (torch.empty(51200, device="cuda"), torch.empty(800, device="cuda"), torch.empty(32, device="cuda"),
                torch.empty(64, device="cuda"))
        ops.f32_conv_reduce(slab, cpart, db2p, *outs)
        got[mode] = outs
    xd, w1r, b1r, w2r = (t.double().clone().requires_grad_(True) for t in (x, w1, b1, w2))
    y1 = F.conv2d(xd.view(B, 1, 28, 28), w1r.permute(3, 2, 0, 1), b1r, padding=2)
    p1 = F.max_pool2d(F.relu(y1), 2, 2)
    y2 = F.conv2d(p1, w2r.permute(3, 2, 0, 1), None, padding=2)
    y2.backward(dY2.double().permute(0, 3, 1, 2))
    refs = (w2r.grad.reshape(-1), w1r.grad.reshape(-1), b1r.grad, db2p.double().sum(0))
    for k, name in enumerate(("dW2", "dW1", "db1", "db2")):
        e0, e1 = rel_err(got[0][k], refs[k]), rel_err(got[nprod][k], refs[k])
        print(f"B={B} x{nprod} {name}: fp32 MFMA {e0:.3e}, split {e1:.3e}")
        assert torch.isfinite(got[nprod][k]).all(), name
        assert e1 <= 2.0 * e0 + 1e-7, (name, e0, e1)


@pytest.mark.parametrize("nprod", [6, 9])
@pytest.mark.parametrize("B", [7, 100, 112, 128])
def test_split_fc1_fwd_is_fp32_accurate(ops, B, nprod):
    """fc1 forward partial slabs on split-bf16 products (B <= 112; B = 128 runs the fp32-input form):
    the slab sum against float64 a2 @ W3."""
    g = torch.Generator(device="cuda").manual_seed(8)
    a2 = torch.relu(torch.randn(B, 3136, device="cuda", generator=g))
    w3 = torch.randn(3136, 1024, device="cuda", generator=g) * 0.02
    ref = a2.double() @ w3.double()
    got = {}
    for mode in (0, nprod):
        zp = torch.full((14, B, 1024), float("nan"), device="cuda")
        ops.f32_fc1_fwd(a2, w3, zp, products=mode)
        got[mode] = zp.sum(0)
    e0, e1 = rel_err(got[0], ref), rel_err(got[nprod], ref)
    print(f"B={B} x{nprod} fc1_fwd: fp32 MFMA {e0:.3e}, split {e1:.3e}")
    assert torch.isfinite(got[nprod]).all()
    assert e1 <= 2.0 * e0 + 1e-8, (e0, e1)
