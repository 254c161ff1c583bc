"""Worker for tests/test_xgmi_gpu.py: the direct xGMI one-shot allreduce between ranks that share
the GPU of a one-GPU box (gloo only for the handle exchange; the data plane is hipIpc + the
device-side barrier of csrc/kernels/xgmi.hip). Launched by torch.distributed.run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(outdir):
    dist.init_process_group("gloo", init_method="env://")
    r, w = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from mihvd.parallel.xgmi import XGMIAllreduce

    ar = XGMIAllreduce(1 << 18)
    out = {"rank": r, "world": w, "eager": [], "graph": []}
    # eager: sizes with and without a float4 tail, back to back (exercises both slots)
    for it, n in enumerate([1, 7, 1024, 4099, 250_001, 1 << 18]):
        g = torch.Generator().manual_seed(1000 + it)
        xs = [torch.randn(n, generator=g) for _ in range(w)]
        ref = xs[0].clone()
        for x in xs[1:]:
            ref += x  # rank order, as the kernel sums
        t = xs[r].cuda()
        ar.allreduce_(t, average=(it % 2 == 1))
        if it == 0:
            ar.check()  # fail fast if the device barrier cannot see the peer
        exp = ref / w if it % 2 == 1 else ref
        got = t.cpu()
        out["eager"].append({"n": n, "bitwise": bool(torch.equal(got, exp)),
                             "max_err": float((got - exp).abs().max())})
    # HIP graph: one captured call replayed with new inputs every time (device-resident epoch)
    buf = torch.zeros(4096, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            ar.allreduce_(buf, average=True)
    torch.cuda.current_stream().wait_stream(s)
    for k in range(6):
        base = torch.arange(4096, dtype=torch.float32)
        buf.copy_(base * (r + 1) + k)
        graph.replay()
        exp = sum(base * (q + 1) + k for q in range(w)) / w
        got = buf.cpu()
        out["graph"].append({"k": k, "max_err": float((got - exp).abs().max())})
    ar.check()
    ar.close()
    with open(os.path.join(outdir, f"xgmi.{r}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
