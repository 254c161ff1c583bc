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
