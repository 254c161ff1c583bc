"""Where the split-bf16 conv2_bwd dgrad role's dW1 / db1 error sits (per tap, per channel)."""
import sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mihvd import _native
_native.require_kernels()
ops = torch.ops.mihvd
B = int(sys.argv[1]) if len(sys.argv) > 1 else 100
g = torch.Generator(device="cuda").manual_seed(5)
x = torch.rand(B, 784, device="cuda", generator=g)
w1 = torch.randn(5, 5, 1, 32, device="cuda", generator=g) * 0.2
b1 = torch.randn(32, device="cuda", generator=g) * 0.1
w2 = torch.randn(5, 5, 32, 64, device="cuda", generator=g) * 0.05
a1 = torch.empty(B, 14, 14, 32, device="cuda")
idx1 = torch.empty(B, 14, 14, 32, device="cuda", dtype=torch.uint8)
ops.f32_conv1_fwd(x, None, None, w1.reshape(800), b1, a1, idx1)
dY2 = torch.randn(B, 14, 14, 64, device="cuda", generator=g)
db2p = torch.zeros(int(ops.f32_db2_rows(B)), 64, device="cuda")
res = {}
for mode in (0, 6):
    cpart = torch.full((int(ops.f32_dgrad_blocks(B, mode)), 832), float("nan"), device="cuda")
    slab = torch.full((int(ops.f32_wgrad_groups(B, mode)), 51200), float("nan"), device="cuda")
    ops.f32_conv2_bwd(dY2, w2, a1, idx1, x, None, None, cpart, slab, products=mode)
    outs = [torch.empty(51200, device="cuda"), torch.empty(800, device="cuda"), torch.empty(32, device="cuda"),
            torch.empty(64, device="cuda")]
    ops.f32_conv_reduce(slab, cpart, db2p, *outs)
    res[mode] = outs
# fp64 dA1 and the routed g1 -> dW1 reference
xd, w1r, b1r, w2r = (t.double().clone().requires_grad_(True) for t in (x, w1, b1, w2))
y1 = F.conv2d(xd.view(B, 1, 28, 28), w1r.permute(3, 2, 0, 1), b1r, padding=2)
p1 = F.max_pool2d(F.relu(y1), 2, 2)
y2 = F.conv2d(p1, w2r.permute(3, 2, 0, 1), None, padding=2)
y2.backward(dY2.double().permute(0, 3, 1, 2))
ref = w1r.grad.reshape(25, 32)
for mode in (0, 6):
    e = (res[mode][1].double().view(25, 32) - ref)
    print("mode", mode, "dW1 rel", (e.norm() / ref.norm()).item())
    print("  per tap  :", " ".join(f"{(e[t].norm() / ref[t].norm()).item():.1e}" for t in range(25)))
    print("  per ci   :", " ".join(f"{(e[:, c].norm() / ref[:, c].norm()).item():.1e}" for c in range(32)))
d = (res[6][1] - res[0][1]).view(25, 32).double()
print("split - native, max abs", d.abs().max().item(), "ref max", ref.abs().max().item())
print("db1 diff per ci:", " ".join(f"{v:.1e}" for v in (res[6][2] - res[0][2]).tolist()))
print("db1 ref:", " ".join(f"{v:.1e}" for v in b1r.grad.tolist()))
