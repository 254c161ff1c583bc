"""Worker for tests/test_xgmi_gpu.py: the direct xGMI collectives between ranks that share the GPU
of a one-GPU box (gloo only for the handle exchange and the references; the data plane is hipIpc +
the device-side phase barriers of csrc/kernels/xgmi.hip). Launched by torch.distributed.run.

usage: xgmi_worker.py <scenario> <outdir>
  allreduce : XGMIAllreduce (staged, double-buffered) eager over several sizes + HIP graph replay
  region    : XGMIRegion gather_rows (whole rows and a column range, row cap) and reduce, repeated
              (both epoch parities), eager and from a HIP graph
  timeout   : rank 1 arrives late (past MIHVD_XGMI_TIMEOUT_MS): rank 0's collective must produce
              NaN, check() must raise, and every later collective on rank 0 must be NaN too
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def sc_allreduce(r, w):
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
    dist.barrier()
    ar.close()
    return out


def sc_region(r, w):
    from mihvd.parallel.xgmi import XGMIRegion

    R, C = 37, 3136            # rows per rank, bf16 columns (a2-shaped rows: 6272 bytes)
    N = 4099                   # fp32 elements reduced
    reg = XGMIRegion({"rows": (w * R * C, torch.bfloat16), "vec": (N, torch.float32)})
    rows = reg.view("rows").view(w * R, C)
    vec = reg.view("vec")
    out_red = torch.empty(N, device="cuda")
    res = {"rank": r, "checks": []}

    def fill(it):
        # every peer has finished reading this rank's rows of the previous round (each synchronised
        # its gather before reaching this barrier) before they are overwritten
        dist.barrier()
        g = torch.Generator().manual_seed(77 + 13 * it + r)
        rows.zero_()
        rows[r * R:(r + 1) * R].copy_(torch.randn(R, C, generator=g).to(torch.bfloat16))
        vec.copy_(torch.randn(N, generator=g))
        torch.cuda.synchronize()
        allrows = [torch.zeros(R, C, dtype=torch.bfloat16) for _ in range(w)]
        dist.all_gather(allrows, rows[r * R:(r + 1) * R].cpu())
        vecs = [torch.zeros(N) for _ in range(w)]
        dist.all_gather(vecs, vec.cpu())
        ref = vecs[0].clone()
        for v in vecs[1:]:
            ref += v
        return torch.cat(allrows), ref

    def compare(tag, full, ref_sum, lo, hi, cap):
        got = rows.cpu()
        ok = True
        for q in range(w):
            for i in range(R):
                row = q * R + i
                if q == r:
                    continue
                if row >= cap:
                    ok &= bool((got[row] == 0).all())  # rows past the cap stay untouched
                    continue
                ok &= torch.equal(got[row, lo:hi], full[row, lo:hi])
                ok &= bool((got[row, :lo] == 0).all()) and bool((got[row, hi:] == 0).all())
        red = out_red.cpu()
        res["checks"].append({"tag": tag, "rows_ok": bool(ok), "sum_bitwise": bool(torch.equal(red, ref_sum)),
                              "sum_err": float((red - ref_sum).abs().max())})

    # eager: whole rows, then a 16-byte aligned column range with a row cap (4 rounds: both parities)
    specs = [(0, C, w * R), (128, 1024, w * R - 5), (0, C, w * R), (2048, 2048 + 16, w * R)]
    for it, (lo_b, hi_b, cap) in enumerate(specs):
        full, ref_sum = fill(it)
        reg.gather_rows("rows", 0, C * 2, R, total_rows=cap, col_lo=lo_b, col_hi=hi_b)
        reg.reduce("vec", 1, out_red)
        torch.cuda.synchronize()
        compare(f"eager{it}", full, ref_sum, lo_b // 2, hi_b // 2, cap)
    # graph: capture one gather + one reduce, replay with fresh data
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            reg.gather_rows("rows", 0, C * 2, R)
            reg.reduce("vec", 1, out_red, scale=0.5)
    torch.cuda.current_stream().wait_stream(s)
    for k in range(3):
        full, ref_sum = fill(10 + k)
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        compare(f"graph{k}", full, ref_sum * 0.5, 0, C, w * R)
    reg.check()
    dist.barrier()
    reg.close()
    return res


def sc_timeout(r, w):
    from mihvd.parallel.xgmi import XGMIRegion

    N = 1024
    reg = XGMIRegion({"vec": (N, torch.float32)})
    reg.view("vec").fill_(1.0)
    out = torch.zeros(N, device="cuda")
    torch.cuda.synchronize()
    dist.barrier()
    res = {"rank": r}
    if r == 1:
        time.sleep(3.0)  # well past rank 0's timeout
    t0 = time.perf_counter()
    reg.reduce("vec", 0, out)
    torch.cuda.synchronize()
    res["first_s"] = time.perf_counter() - t0
    res["first_nan"] = bool(torch.isnan(out).all())
    # the host-coherent mirror of the error word, and the health monitor's view of it
    import ctypes

    from mihvd._native import runtime

    addr = int(reg._o.xgmi_error_word(reg.ctx))
    res["mirror"] = ctypes.c_uint32.from_address(addr).value if addr else -1
    mon = runtime().HealthMonitor(r, 0.05, 134)
    mon.set_abort_process(False)
    mon.watch_word(addr, "xgmi test")
    res["monitor"] = list(mon.poll_once())
    mon.unwatch_word(addr)
    try:
        reg.check()
        res["raised"] = False
    except RuntimeError as e:
        res["raised"] = True
        res["msg"] = str(e)
    # a later collective after the failure: no wait, NaN again on the failed rank
    out.zero_()
    t0 = time.perf_counter()
    reg.reduce("vec", 1, out)
    torch.cuda.synchronize()
    res["second_s"] = time.perf_counter() - t0
    res["second_nan"] = bool(torch.isnan(out).all())
    dist.barrier()
    reg.close()
    return res


def main(scenario, outdir):
    dist.init_process_group("gloo", init_method="env://")
    r, w = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    out = globals()["sc_" + scenario](r, w)
    with open(os.path.join(outdir, f"{scenario}.{r}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
