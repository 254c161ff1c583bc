"""Worker of tests/test_native_comm_gpu.py::test_bucket_plane_carries_distributed_optimizer:
DistributedOptimizer's gradient buckets on the framework-owned RCCL bucket plane
(mihvd.parallel.collectives.BucketPlane; MIHVD_FORCE_COLLECTIVES=1 keeps the collectives at world
size 1), eagerly and with the whole step captured in a HIP graph, against the same model trained
with the plain optimizer (a world-1 allreduce is the identity; stock conv backward on MIOpen is not
bitwise deterministic run to run even with its deterministic algorithms requested, so the plane's
distance from the plain optimizer is compared with the plain optimizer's distance from itself)."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(out):
    import mihvd.torch as hvd
    from mihvd import basics
    from mihvd.graphs import CapturedStep
    from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy
    from mihvd.optim import FusedAdam

    hvd.init()
    assert dist.get_backend() == "nccl"
    torch.backends.cudnn.deterministic = True  # MIOpen's deterministic convolution algorithms
    torch.backends.cudnn.benchmark = False
    dev = hvd.device()
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.rand(8, 100, 784, generator=g).to(dev)
    Y = torch.randint(0, 10, (8, 100), generator=g).to(dev)

    def make(dist_opt):
        model = MNISTConvNet(impl="torch", seed=11).to(dev)
        opt = FusedAdam(model.parameters(), lr=1e-3, rule="tf")
        if dist_opt:
            opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters())
        return model, opt

    def train(model, opt, steps, graph):
        torch.manual_seed(123)  # the same dropout masks for both optimizers
        ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        xb = torch.empty(100, 784, device=dev)
        yb = torch.empty(100, dtype=torch.int64, device=dev)

        def step():
            i = ctr % 8
            xb.copy_(X.index_select(0, i).squeeze(0))
            yb.copy_(Y.index_select(0, i).squeeze(0))
            opt.zero_grad(set_to_none=False)
            loss = softmax_cross_entropy(model(xb), yb)
            loss.backward()
            opt.step()
            ctr.add_(1)
            return loss

        run = CapturedStep(step, warmup=3) if graph else step
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        return torch.cat([p.detach().reshape(-1) for p in model.parameters()])

    res = {}
    for graph in (False, True):
        m, o = make(True)
        plane = basics._ctx.plane
        n0 = plane.launched if plane is not None else -1
        a = train(m, o, 12, graph)
        m2, o2 = make(False)
        b = train(m2, o2, 12, graph)
        m3, o3 = make(False)
        c = train(m3, o3, 12, graph)  # the plain optimizer again: the run-to-run noise floor
        key = "graph" if graph else "eager"
        res[key] = {"plane": plane is not None, "launched": (plane.launched - n0) if plane is not None else 0,
                    "buckets": len(o._buckets), "bitwise": bool(torch.equal(a, b)),
                    "rel": float((a - b).norm() / b.norm()), "noise": float((c - b).norm() / b.norm()),
                    "nranks": plane.comm.nranks() if plane is not None else None}
    # the public collective API on the same framework-owned communicator (world 1, collectives forced
    # on: every result is the identity), counted per kind by the plane
    plane = basics._ctx.plane
    c0 = dict(plane.counts) if plane is not None else {}
    t = torch.arange(12, dtype=torch.float32, device=dev)
    api = {
        "allreduce": torch.equal(hvd.allreduce(t, op=hvd.Sum), t) and torch.equal(hvd.allreduce(t), t),
        "allreduce_async": torch.equal(hvd.synchronize(hvd.allreduce_async(t.clone(), op=hvd.Sum)), t),
        "broadcast": torch.equal(hvd.broadcast(t, 0), t),
        "allgather": torch.equal(hvd.allgather(t.view(3, 4)), t.view(3, 4)),
        "reducescatter": torch.equal(hvd.reducescatter(t.view(3, 4), op=hvd.Sum), t.view(3, 4)),
        "alltoall": torch.equal(hvd.alltoall(t.view(6, 2))[0], t.view(6, 2)),
    }
    m0, _ = make(False)
    hvd.broadcast_parameters(m0.state_dict(), 0)
    c1 = dict(plane.counts) if plane is not None else {}
    res["api"] = api
    res["api_counts"] = {k: c1.get(k, 0) - c0.get(k, 0) for k in set(c1) | set(c0)}
    # an elastic reset (mihvd.elastic: shutdown + init, then State.sync -> _elastic_reset) must move a
    # DistributedOptimizer onto the new world's bucket plane
    m1, o1 = make(True)
    old = o1._plane
    hvd.shutdown()
    hvd.init()
    o1._elastic_reset()
    new_plane = basics._ctx.plane
    train(m1, o1, 2, False)
    res["elastic"] = {"had_plane": old is not None, "new_plane": new_plane is not None and new_plane is not old,
                      "uses_new": o1._plane is new_plane,
                      "launched_after": new_plane.launched if new_plane is not None else 0}
    with open(out, "w") as f:
        json.dump(res, f)
    hvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
