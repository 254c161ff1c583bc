"""Worker of tests/test_native_comm_gpu.py: the framework-owned RCCL communicator
(mihvd/parallel/rccl.py) on one GPU (RCCL refuses two ranks per GPU; the collectives at world size
1 still run through ncclCommInitRank and the RCCL kernels), eagerly and captured in a HIP graph,
and the fused fp32 trainer's collective path on it against the same trainer without collectives."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(out):
    import mihvd

    mihvd.init()
    assert dist.get_backend() == "nccl"
    from mihvd.parallel.rccl import NativeComm

    dev = torch.device("cuda", 0)
    comm = NativeComm(device=dev)
    res = {"world": comm.world}
    g = torch.Generator(device="cpu").manual_seed(3)
    a = torch.randn(1000, generator=g).to(dev)
    ref = a.clone()
    comm.all_reduce_(a)
    res["allreduce_sum"] = bool(torch.equal(a, ref))
    comm.all_reduce_(a, "avg")
    res["allreduce_avg"] = bool(torch.equal(a, ref))
    b = torch.randn(64, generator=g).to(torch.bfloat16).to(dev)
    bref = b.clone()
    comm.all_reduce_(b)
    res["allreduce_bf16"] = bool(torch.equal(b, bref))
    full = torch.zeros(4, 8, device=dev)
    full[0].copy_(torch.arange(8.0))
    ag = torch.zeros(8, device=dev)
    comm.all_gather_into(ag, full[0])
    res["all_gather"] = bool(torch.equal(ag, full[0]))
    out_rs = torch.zeros(8, device=dev)
    comm.reduce_scatter(out_rs, full[0])
    res["reduce_scatter"] = bool(torch.equal(out_rs, full[0]))
    a2a_in = torch.arange(4096, device="cuda", dtype=torch.float32)
    a2a_out = torch.full_like(a2a_in, float("nan"))
    comm.all_to_all(a2a_out, a2a_in)
    res["all_to_all"] = bool(torch.equal(a2a_out, a2a_in))
    comm.broadcast_(a, 0)
    res["broadcast"] = bool(torch.equal(a, ref))
    comm.all_reduce_many_([a, b])
    res["many"] = bool(torch.equal(a, ref) and torch.equal(b, bref))
    # captured: 10 in-place sums of x2 scaling in a graph (world 1: sum is identity, scaling shows replay)
    s = torch.cuda.Stream()
    c = torch.ones(256, device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.all_reduce_(c)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(10):
            c.mul_(2.0)
            comm.all_reduce_(c)
    gr.replay()
    torch.cuda.synchronize()
    res["graph"] = float(c[0].item())
    res["async_error"] = comm.async_error()

    # fused fp32 trainer over the native communicator vs the same trainer without collectives
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    (x, y), _ = synthetic_mnist(n_train=1000, n_test=10, seed=2)
    X = torch.from_numpy(x.reshape(-1, 784)).float().to(dev) / 255.0
    Y = torch.from_numpy(y.astype("int64")).to(dev)
    trs = {}
    for mode in ("native", "none"):
        if mode == "native":
            os.environ["MIHVD_FORCE_COLLECTIVES"] = "1"
            os.environ["MIHVD_COMM"] = "native"
        else:
            os.environ.pop("MIHVD_FORCE_COLLECTIVES", None)
            os.environ.pop("MIHVD_COMM", None)
        tr = FusedMNISTTrainer(batch_size=100, lr=1e-3, seed=1, device=dev, precision="fp32")
        tr.set_device_dataset(X, Y, seed=4)
        tr.build_graph(steps_per_replay=5, warmup=1)
        for _ in range(4):
            tr.run_graph()
        tr.sync()
        trs[mode] = tr
    res["trainer_native_comm"] = trs["native"].ncomm is not None
    pa, pb = trs["native"].params, trs["none"].params
    res["trainer_rel_diff"] = float(((pa - pb).norm() / pb.norm()).item())
    res["trainer_loss"] = float(trs["native"].last_loss())
    trs["native"].close()
    comm.close()
    with open(out, "w") as f:
        json.dump(res, f)
    mihvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
