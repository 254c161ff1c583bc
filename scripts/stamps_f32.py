#!/usr/bin/env python3
"""Phase timing of f32_conv2_bwd blocks from in-kernel shader-clock stamps (f32_stamps_enable).

Prints, per role, the median and max cycles of each phase and when blocks start relative to the
first block (second-round blocks start late), plus the kernel's event-timed duration for scale.
Needs the study build of the kernels (the stamps are compiled out of production builds):
``MIHVD_F32_STAMPS=1 python -m mihvd._build kernels --force``.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    B = 100
    (x, y), _ = synthetic_mnist(n_train=B * 20, n_test=10, seed=1)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=B, lr=1e-3, seed=0, device="cuda", precision="fp32")
    tr.set_device_dataset(X, Y)
    for _ in range(3):
        tr.device_step()
    torch.cuda.synchronize()
    o, st, P = tr.ops, tr.state, tr.pview
    n_dg = int(o.f32_dgrad_blocks(B))
    n_wg = 10 * int(o.f32_wgrad_groups(B))
    w2 = P("conv_layer2/conv2d/kernel")
    # the production launch: W2 from the fragment copy the step's conv1 launch wrote
    wfb = tr.w2frag[1] if tr.w2frag is not None else None
    run = lambda: o.f32_conv2_bwd(tr.dY2, w2, tr.a1, tr.idx1, tr.X, tr.rows, st, tr.cpart, tr.slab, w2frag=wfb)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000
    buf = o.f32_stamps_enable(n_dg + n_wg)
    run()
    torch.cuda.synchronize()
    s = buf.view(-1, 16).cpu().double()
    o.f32_stamps_enable(0)
    t0 = s[:, 0].min()
    span = (torch.maximum(s[:n_dg, 3], torch.zeros(1)).max().item(), s[n_dg:, 6].max().item())
    total = max(span) - t0.item()
    print(f"conv2_bwd B={B}: {us:.1f} us (event), {total:.0f} cycles first start -> last end "
          f"({total / us:.0f} cycles/us)")

    def show(name, rows, marks):
        print(f"  {name}: {rows.shape[0]} blocks")
        st_ = rows[:, 0] - t0
        print(f"    start offset   median {st_.median():8.0f}  max {st_.max():8.0f}")
        for a, b, label in marks:
            d = rows[:, b] - rows[:, a]
            print(f"    {label:14s} median {d.median():8.0f}  max {d.max():8.0f}")

    show("dgrad", s[:n_dg], [(0, 1, "staging"), (1, 2, "tap loop w0"), (2, 7, "loop skew"), (7, 3, "epilogue"),
                             (0, 3, "block total")])
    d = s[:n_dg, 8:16] - s[:n_dg, 1:2]
    print("    tap loop per wave (median over blocks): " + " ".join(f"{v:.0f}" for v in d.median(0).values))
    show("wgrad", s[n_dg:], [(0, 4, "first image"), (4, 5, "image loop"), (5, 6, "reduction"), (0, 6, "block total")])
    # wgrad slots 8 + n: wave 0's end of image n (after the image's barrier), full 8-image groups
    wg = s[n_dg:]
    full = wg[(wg[:, 15] > 0)]
    if full.shape[0]:
        per = torch.cat([full[:, 8:9] - full[:, 4:5], full[:, 9:16] - full[:, 8:15]], 1)
        print("    per image (median over full groups): " + " ".join(f"{v:.0f}" for v in per.median(0).values))

    # conv2_fwd: staging, then one stamp per tile pair (the 4-wave form carries the stamps)
    os.environ["MIHVD_F32_C2F_W8"] = "0"
    a2, idx2 = tr.a2, tr.idx2
    runf = lambda: o.f32_conv2_fwd(tr.a1, w2, P("conv_layer2/conv2d/bias"), a2, idx2)
    nblk = -(-((49 * B + 3) // 4) // 5)
    buf = o.f32_stamps_enable(nblk, 1)
    runf()
    torch.cuda.synchronize()
    f = buf.view(-1, 16).cpu().double()
    o.f32_stamps_enable(0, 1)
    print(f"conv2_fwd: {nblk} blocks")
    for a, b, label in [(0, 1, "staging"), (1, 2, "tile pair 1"), (2, 3, "tile pair 2"), (3, 4, "tile 5"),
                        (0, 4, "block total")]:
        d = f[:, b] - f[:, a]
        print(f"    {label:14s} median {d.median():8.0f}  max {d.max():8.0f}")

    # fc1_bwd row form with the fused dense/kernel Adam (as the trainer runs it at world size 1)
    from mihvd.models.fused_mnist import FLAT_NUMEL, W3_START

    G = tr.gview
    s3 = slice(W3_START, FLAT_NUMEL)
    m3, v3 = tr.m[s3], tr.v[s3]
    w3 = P("dense/kernel")
    run1 = lambda: o.f32_fc1_bwd(tr.dz, tr.a2, tr.idx2, tr.h, tr.dlog, w3, tr.dY2, tr.db2p, G("dense/kernel"),
                                 G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), m3, v3, st, 0.0, 0.9,
                                 0.999, tr.eps, 1.0, tr.rule, False)
    run1()
    torch.cuda.synchronize()
    buf = o.f32_stamps_enable(196, 2)
    run1()
    torch.cuda.synchronize()
    f = buf.view(-1, 16).cpu().double()
    o.f32_stamps_enable(0, 2)
    print("fc1_bwd rows (+W3 Adam): 196 blocks")
    marks = [(0, 1, "chunk 0")] + [(c, c + 1, f"chunk {c}") for c in range(1, 8)] + [(8, 9, "exchange"),
                                                                                    (9, 10, "epilogue"),
                                                                                    (0, 10, "block total")]
    for a, b, label in marks:
        d = f[:, b] - f[:, a]
        print(f"    {label:14s} median {d.median():8.0f}  max {d.max():8.0f}")
    st0 = f[:, 0] - f[:, 0].min()
    print(f"    start offset   median {st0.median():8.0f}  max {st0.max():8.0f}")


if __name__ == "__main__":
    main()
