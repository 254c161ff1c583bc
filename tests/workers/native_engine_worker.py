"""Worker of tests/test_native_comm_gpu.py::test_native_engine_one_gpu: the C++ collective engine
(csrc/kernels/engine.cpp, MIHVD_ENGINE=native) on one GPU. At world size 1 the engine still runs
its whole path — GPU negotiation cycles (the control-vector allreduce), fusion into the persistent
buffer, RCCL allreduce, copy-out, completion events — so every result must equal its input, and a
DistributedOptimizer training run through it must match plain training bit for bit."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def train(model, opt, X, Y, steps):
    from mihvd.models.mnist import softmax_cross_entropy

    for i in range(steps):
        opt.zero_grad()
        loss = softmax_cross_entropy(model(X[i]), Y[i])
        loss.backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def main(out):
    import mihvd.torch as hvd
    from mihvd import basics
    from mihvd.parallel.native_engine import NativeEngine

    hvd.init()
    eng = basics._ctx.engine
    res = {"engine": type(eng).__name__, "world": hvd.size()}
    assert isinstance(eng, NativeEngine), type(eng)
    dev = hvd.device()
    g = torch.Generator(device="cpu").manual_seed(5)

    # 1. stream ordering: each tensor is produced by kernels queued right before its enqueue
    base = [torch.randn(n, generator=g).to(dev) for n in (7, 1000, 4096, 33, 250_000)]
    outs, hs = [], []
    for i, b in enumerate(base):
        t = (b * 3.0 + 1.0).sin_()  # the engine must read this, not an earlier value
        outs.append(t)
        hs.append(hvd.allreduce_async_(t, name=f"t{i}", op=hvd.Sum))
    exp = [(b * 3.0 + 1.0).sin_() for b in base]
    for h in hs:
        hvd.synchronize(h)
    res["values_exact"] = all(bool(torch.equal(o, e)) for o, e in zip(outs, exp))

    # 2. fusion: many small tensors enqueued together are reduced in fewer collectives
    st0 = eng.stats()
    small = [torch.full((100 + i,), float(i), device=dev) for i in range(24)]
    hs = [hvd.allreduce_async_(t, name=f"s{i}", op=hvd.Average) for i, t in enumerate(small)]
    for h in hs:
        hvd.synchronize(h)
    st1 = eng.stats()
    res["small_exact"] = all(bool(torch.equal(t, torch.full_like(t, float(i)))) for i, t in enumerate(small))
    res["small_tensors"] = st1["tensors"] - st0["tensors"]
    res["small_collectives"] = st1["collectives"] - st0["collectives"]

    # 3. a tensor above the fusion threshold is reduced in place
    big = torch.randn(3_000_000, generator=g).to(dev)
    ref = big.clone()
    hvd.synchronize(hvd.allreduce_async_(big, name="big", op=hvd.Sum))
    res["big_exact"] = bool(torch.equal(big, ref))

    # 4. DistributedOptimizer through the engine vs plain training (world 1: identical arithmetic).
    #    An MLP (deterministic GEMMs): bit for bit; the CNN (MIOpen's weight-gradient convolutions
    #    are not run-to-run deterministic): to fp32 rounding.
    from mihvd.models.mnist import MNISTConvNet

    X = torch.randn(6, 32, 784, generator=g).to(dev)
    Y = torch.randint(0, 10, (6, 32), generator=g).to(dev)

    def mlp():
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10)).to(dev)

    st2 = eng.stats()
    m1, m2 = mlp(), mlp()
    o1 = hvd.DistributedOptimizer(torch.optim.Adam(m1.parameters(), lr=1e-3), named_parameters=m1.named_parameters())
    p1 = train(m1, o1, X, Y, 6)
    p2 = train(m2, torch.optim.Adam(m2.parameters(), lr=1e-3), X, Y, 6)
    res["optimizer_bitwise"] = bool(torch.equal(p1, p2))
    c1 = MNISTConvNet(impl="torch", seed=1).to(dev).eval()  # dropout off: the same function twice
    c2 = MNISTConvNet(impl="torch", seed=1).to(dev).eval()
    oc = hvd.DistributedOptimizer(torch.optim.Adam(c1.parameters(), lr=1e-3), named_parameters=c1.named_parameters(),
                                  backward_passes_per_step=1)
    q1 = train(c1, oc, X, Y, 6)
    q2 = train(c2, torch.optim.Adam(c2.parameters(), lr=1e-3), X, Y, 6)
    res["cnn_rel_diff"] = float((q1 - q2).norm() / q2.norm())
    torch.cuda.synchronize()
    st3 = eng.stats()
    res["optimizer_collectives"] = st3["collectives"] - st2["collectives"]
    res["stats"] = st3
    hvd.shutdown()
    res["stopped"] = not bool(torch.ops.mihvd.engine_running())
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main(sys.argv[1])
