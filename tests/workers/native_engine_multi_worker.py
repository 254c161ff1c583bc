"""Worker of tests/test_native_comm_gpu.py::test_native_engine_ranks_out_of_order: the C++ engine
(csrc/kernels/engine.cpp, MIHVD_ENGINE=native) across several GPUs, one rank per GPU. Every rank
enqueues the same 80 named allreduces (more than one announce round of 64 new signatures) in a
different order (rank r rotates the list by 13 r and reverses it on odd ranks), with values that
depend on the rank, plus a few tensors above the fusion threshold; every result must equal the
closed-form sum, and a second wave of the same names (now cached signatures) must too."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(out):
    import mihvd.torch as hvd
    from mihvd import basics
    from mihvd.parallel.native_engine import NativeEngine

    hvd.init()
    eng = basics._ctx.engine
    assert isinstance(eng, NativeEngine), type(eng)
    W, r, dev = hvd.size(), hvd.rank(), hvd.device()
    n_small, sizes = 80, [17 + 5 * i for i in range(80)]
    res = {"world": W, "rank": r, "ok": []}
    for wave in range(2):
        order = list(range(n_small))
        order = order[(13 * r) % n_small:] + order[:(13 * r) % n_small]
        if r % 2:
            order.reverse()
        ts, hs = {}, []
        for i in order:
            t = torch.full((sizes[i],), float((r + 1) * (i + 1) + wave), device=dev)
            ts[i] = t
            hs.append(hvd.allreduce_async_(t, name=f"g{i}", op=hvd.Sum))
        big = [torch.full((2_000_000 + 1000 * k,), float(r + k), device=dev) for k in range(3)]
        for k in ([0, 1, 2] if r % 2 == 0 else [2, 0, 1]):
            hs.append(hvd.allreduce_async_(big[k], name=f"big{k}", op=hvd.Sum))
        for h in hs:
            hvd.synchronize(h)
        s = W * (W + 1) // 2
        ok = all(bool(torch.equal(ts[i], torch.full_like(ts[i], float(s * (i + 1) + W * wave)))) for i in range(n_small))
        ok &= all(bool(torch.equal(big[k], torch.full_like(big[k], float(s - W + W * k)))) for k in range(3))
        res["ok"].append(ok)
    res["stats"] = eng.stats()
    hvd.shutdown()
    res["stopped"] = not bool(torch.ops.mihvd.engine_running())
    with open(f"{out}.{r}", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main(sys.argv[1])
