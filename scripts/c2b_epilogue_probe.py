#!/usr/bin/env python3
"""conv2_bwd at HEAD (W2 fragment copy) in two forms selected by an env knob (argv[1], default
MIHVD_F32_C2B_MEPI: the conv1 weight-gradient epilogue on VALU = 0 or on MFMA = 1;
MIHVD_F32_C2B_ADMA: the wgrad role's LDS-DMA by builtin = 0 or inline asm = 1): whole launch and
each role alone (MIHVD_F32_C2B_ROLE=1 dgrad, 2 wgrad), event-timed medians of back-to-back
launches, alternating the forms."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    w2 = P("conv_layer2/conv2d/kernel")
    run = lambda: o.f32_conv2_bwd(tr.dY2, w2, tr.a1, tr.idx1, tr.X, tr.rows, st, tr.cpart, tr.slab, w2frag=tr.w2frag[1])
    knob = sys.argv[1] if len(sys.argv) > 1 else "MIHVD_F32_C2B_MEPI"
    res = {}
    for rnd in range(3):
        for mepi in ("0", "1"):
            for role in ("0", "1", "2"):
                os.environ[knob], os.environ["MIHVD_F32_C2B_ROLE"] = mepi, role
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(30):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    run()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1000)
                res.setdefault((mepi, role), []).append(statistics.median(ts))
    os.environ.pop(knob), os.environ.pop("MIHVD_F32_C2B_ROLE")
    names = {"0": "whole launch", "1": "dgrad role only", "2": "wgrad role only"}
    for (mepi, role), v in sorted(res.items()):
        print(f"conv2_bwd {knob}={mepi}, {names[role]:<16s} "
              + " ".join(f"{t:7.2f}" for t in v) + f"   median {statistics.median(v):7.2f} us")


if __name__ == "__main__":
    main()
