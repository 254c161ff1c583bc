"""Multi-process scenarios, launched by tests through ``mihvdrun -np N`` (gloo on CPU).

Usage: python dist_worker.py <scenario> <outdir>. Each rank writes <outdir>/<scenario>.<rank>.json.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mihvd.torch as hvd  # noqa: E402


def out(outdir, name, payload):
    with open(os.path.join(outdir, f"{name}.{hvd.rank()}.json"), "w") as f:
        json.dump(payload, f)


def sc_collectives(outdir):
    r, n = hvd.rank(), hvd.size()
    res = {}
    t = torch.arange(6, dtype=torch.float32) + r
    res["sum"] = hvd.allreduce(t, op=hvd.Sum).tolist()
    res["avg"] = hvd.allreduce(t).tolist()
    res["min"] = hvd.allreduce(t, op=hvd.Min).tolist()
    res["max"] = hvd.allreduce(t, op=hvd.Max).tolist()
    res["bf16"] = hvd.allreduce(t, op=hvd.Sum, compression=hvd.Compression.bf16).tolist()
    res["fp16"] = hvd.allreduce(t, compression=hvd.Compression.fp16).tolist()
    x = torch.full((r + 1, 2), float(r))
    res["allgather"] = hvd.allgather(x).tolist()
    b = torch.full((3,), float(r))
    res["broadcast"] = hvd.broadcast(b, root_rank=n - 1).tolist()
    hvd.broadcast_(b, root_rank=0)
    res["broadcast_"] = b.tolist()
    a2a_in = torch.arange(n * 2, dtype=torch.float32) + 100 * r
    o, splits = hvd.alltoall(a2a_in)
    res["alltoall"] = o.tolist()
    res["reducescatter"] = hvd.reducescatter(torch.ones(n * 2, 3) * (r + 1), op=hvd.Sum).tolist()
    res["object"] = hvd.broadcast_object({"rank": r, "msg": "hi"}, root_rank=0)
    res["allgather_object"] = hvd.allgather_object(r * 10)
    g = hvd.grouped_allreduce([torch.ones(3) * r, torch.ones(2, 2) * (r + 1)], op=hvd.Sum)
    res["grouped"] = [x.tolist() for x in g]
    h = hvd.allreduce_async(torch.ones(4) * r, op=hvd.Sum, name="async")
    while not hvd.poll(h):
        time.sleep(0.001)
    res["async"] = hvd.synchronize(h).tolist()
    res["join"] = hvd.join()
    out(outdir, "collectives", res)


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))


def sc_dp_equivalence(outdir):
    """N ranks × B samples == 1 process × N·B samples (Average)."""
    r, n = hvd.rank(), hvd.size()
    gen = torch.Generator().manual_seed(7)
    X = torch.randn(n * 5, 8, generator=gen)
    Y = torch.randn(n * 5, 4, generator=gen)
    res = {}
    for thresh in (0, 64 * 1024 * 1024):
        m = _model(seed=100 + r)  # different init on purpose: broadcast must fix it
        hvd.broadcast_parameters(m.state_dict(), root_rank=0)
        opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), named_parameters=m.named_parameters(),
                                       fusion_threshold=thresh if thresh else 64)
        ref = _model(seed=100)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
        for step in range(3):
            opt.zero_grad()
            xs, ys = X[r * 5:(r + 1) * 5], Y[r * 5:(r + 1) * 5]
            torch.nn.functional.mse_loss(m(xs), ys).backward()
            opt.step()
            ropt.zero_grad()
            # mean of per-rank means == global mean (equal shard sizes)
            torch.nn.functional.mse_loss(ref(X), Y).backward()
            ropt.step()
        diff = max((a - b).abs().max().item() for a, b in zip(m.parameters(), ref.parameters()))
        res[f"maxdiff_{thresh}"] = diff
        res[f"nbuckets_{thresh}"] = len(opt.buckets)
    out(outdir, "dp_equivalence", res)


def sc_negotiated_fusion(outdir):
    """MIHVD_NEGOTIATE=1: groups of small allreduces submitted together are fused by the engine
    into its persistent fusion buffer — allocated once, reused every step."""
    from mihvd import basics

    r, n = hvd.rank(), hvd.size()
    eng = basics._ctx.engine
    allocs, ok = [], True
    for step in range(6):
        ts = [torch.full((k + 3,), float(r + step + k)) for k in range(6)]
        hs = [hvd.allreduce_async(t, name=f"fz{k}", op=hvd.Sum) for k, t in enumerate(ts)]
        outs = [hvd.synchronize(h) for h in hs]
        for k, o in enumerate(outs):
            ok &= bool(torch.allclose(o, torch.full((k + 3,), float(sum(q + step + k for q in range(n))))))
        allocs.append(eng.fusion_allocs)
    neg = eng.neg
    out(outdir, "negotiated_fusion", {"ok": ok, "allocs": allocs, "fused": eng.fused_launches,
                                      "submitted": neg.submitted, "cache_hits": neg.cache_hits,
                                      "records": neg.records_posted})


def sc_autotune(outdir):
    """MIHVD_AUTOTUNE=1: the optimizer tries each fusion threshold, every rank settles on the same
    one, re-plans its buckets once, and training still equals the single-process reference."""
    r, n = hvd.rank(), hvd.size()
    gen = torch.Generator().manual_seed(9)
    X = torch.randn(n * 4, 8, generator=gen)
    Y = torch.randn(n * 4, 4, generator=gen)
    m = _model(seed=3)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.05), named_parameters=m.named_parameters())
    ref = _model(seed=3)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
    seen = set()
    for step in range(20):
        opt.zero_grad()
        torch.nn.functional.mse_loss(m(X[r * 4:(r + 1) * 4]), Y[r * 4:(r + 1) * 4]).backward()
        opt.step()
        seen.add(opt.fusion_threshold)
        ropt.zero_grad()
        torch.nn.functional.mse_loss(ref(X), Y).backward()
        ropt.step()
    diff = max((a - b).abs().max().item() for a, b in zip(m.parameters(), ref.parameters()))
    out(outdir, "autotune", {"done": opt._tuner.done, "best": opt._tuner.best, "final": opt.fusion_threshold,
                             "seen": sorted(seen), "maxdiff": diff, "nbuckets": len(opt.buckets)})


def sc_bpps(outdir):
    """backward_passes_per_step=2 accumulates locally, then one allreduce."""
    r, n = hvd.rank(), hvd.size()
    m = _model(seed=5)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.0), named_parameters=m.named_parameters(),
                                   backward_passes_per_step=2, op=hvd.Sum)
    opt.zero_grad()
    for k in range(2):
        m(torch.ones(2, 8) * (r + 1 + k)).sum().backward()
    opt.step()
    g = m[2].bias.grad.clone()
    m2 = _model(seed=5)
    for rr in range(n):
        for k in range(2):
            m2(torch.ones(2, 8) * (rr + 1 + k)).sum().backward()
    out(outdir, "bpps", {"diff": (g - m2[2].bias.grad).abs().max().item()})


def sc_adasum(outdir):
    from mihvd.parallel.adasum import adasum_reference

    r, n = hvd.rank(), hvd.size()
    vecs = [torch.tensor([1.0 + i, -2.0 * i, 0.5, 3.0 - i, 1.0, 2.0], dtype=torch.float64) for i in range(n)]
    segs = [(0, 3), (3, 6)]
    got = hvd.grouped_allreduce([vecs[r][:3].clone(), vecs[r][3:].clone()], op=hvd.Adasum)
    ref = adasum_reference(vecs, segs)
    d = max((torch.cat([got[0], got[1]]) - ref).abs().max().item(), 0)
    # Optimizer path with Adasum
    m = _model(seed=1)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.01), op=hvd.Adasum)
    opt.zero_grad()
    m(torch.randn(3, 8) * (r + 1)).sum().backward()
    opt.step()
    ps = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allp = hvd.allgather(ps.view(1, -1))
    out(outdir, "adasum", {"diff": d, "param_spread": (allp - allp[0]).abs().max().item()})


def sc_adasum_vhdd(outdir):
    """Vector-halving / distance-doubling Adasum (adasum.adasum_vhdd_ over the process group) on a
    vector of several tensors with gaps, against the single-process oracle of the same pairing tree,
    and this rank's sent bytes."""
    from mihvd.parallel import adasum as A

    r, n = hvd.rank(), hvd.size()
    g = torch.Generator().manual_seed(11)
    N = 10_000
    segs = [(0, 3200), (3264, 3296), (3328, 8128), (8192, 8256), (8320, 9990)]
    vecs = []
    for i in range(n):
        v = torch.randn(N, generator=g) * (1.0 + 0.3 * i)
        for (s0, e0), (s1, _) in zip(segs, segs[1:] + [(N, N)]):
            v[e0:s1] = 0.0  # the gaps (alignment padding of a fusion buffer) are zero
        vecs.append(v)
    ref = A.adasum_reference(vecs, segs)
    got = vecs[r].clone()
    A.adasum_allreduce_(got, segs)
    rel = ((got - ref).norm() / ref.norm()).item()
    out(outdir, "adasum_vhdd", {"rel": rel, "bytes": A.last_bytes_sent, "numel": N, "elem": 4})


def sc_engine_slots(outdir):
    """The native engine's negotiation (csrc/runtime/slot_agreement.h, the code engine.cpp runs over
    its RCCL control communicator) over the TCP store: three phases of enqueues in rank-dependent
    orders -- 80 new signatures at once (more than one 64-hash announce block per rank), 40 new ones
    staggered by rank (slots pending on some ranks only), the first 80 again from the slot cache --
    then the stop protocol. Records the order in which this rank saw collectives become ready."""
    import numpy as np

    from mihvd import _native

    rt = _native.runtime()
    r, n = hvd.rank(), hvd.size()
    host, port = os.environ["MIHVD_STORE_ADDR"].rsplit(":", 1)
    neg = rt.EngineNegotiation(host, int(port), r, n, "mihvd/test/engine_slots", 256, 64)
    rng = np.random.default_rng(100 + r)
    numel = {i: 1000 + 37 * i for i in range(120)}
    hsh = {i: rt.engine_signature_hash(f"grad.{i}|6|{numel[i]}|0") for i in range(120)}
    by_hash = {h: i for i, h in hsh.items()}
    # the enqueue schedule: cycle -> names this rank enqueues at the start of that cycle
    sched = {0: list(rng.permutation(80))}
    late = list(rng.permutation(np.arange(80, 120)))
    for k in range(4):  # phase B: 10 per cycle, starting later on higher ranks
        sched.setdefault(2 + r + k, []).extend(late[10 * k:10 * (k + 1)])
    phase_c = 8 + n  # after every rank's phase B
    sched.setdefault(phase_c, []).extend(rng.permutation(80))
    last = max(sched)
    pending: dict = {}
    ready_log, partial_seen, cycles = [], 0, 0
    while True:
        for i in sched.get(cycles, []):
            h = hsh[int(i)]
            pending[h] = pending.get(h, 0) + 1
            neg.want(h)
        mine = sorted(neg.slot(h) for h, c in pending.items() if c > 0 and neg.slot(h) >= 0)
        stop = cycles > last and not any(c > 0 for c in pending.values())
        summed = neg.negotiate(mine, stop)
        cycles += 1
        if summed[0] == n:
            break
        if summed[1] > 0:
            neg.announce_round()
        nb = neg.num_slots()
        bytes_ = [4 * numel[by_hash[h]] for h in (neg_slot_hashes(neg, by_hash, hsh, nb))]
        groups, partial = neg.plan(summed, bytes_, [0] * nb, 1 << 20)
        partial_seen += len(partial)
        for s in groups:
            if s < 0:
                continue
            h = neg_slot_hashes(neg, by_hash, hsh, nb)[s]
            pending[h] -= 1
            ready_log.append(by_hash[h])
        if cycles > 400:
            raise RuntimeError("negotiation did not finish")
    out(outdir, "engine_slots", {"ready": ready_log, "announces": neg.announces, "max_fresh": neg.max_fresh,
                                 "partial_seen": partial_seen, "slots": neg.num_slots(), "cycles": cycles,
                                 "rounds": neg.rounds})


def neg_slot_hashes(neg, by_hash, hsh, nb):
    """slot -> hash for the slots [0, nb) (via the known signatures)."""
    inv = {}
    for h in hsh.values():
        s = neg.slot(h)
        if 0 <= s < nb:
            inv[s] = h
    return [inv[s] for s in range(nb)]


def sc_optimizer_state(outdir):
    r = hvd.rank()
    m = _model(seed=r)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3 * (r + 1))
    if r == 0:  # only the root has optimizer state
        m(torch.ones(1, 8)).sum().backward()
        opt.step()
    hvd.broadcast_parameters(m.state_dict(), 0)
    hvd.broadcast_optimizer_state(opt, 0)
    st = opt.state_dict()
    sig = {
        "lr": st["param_groups"][0]["lr"],
        "nstate": len(st["state"]),
        "m0": float(st["state"][0]["exp_avg"].sum()) if st["state"] else None,
        "w": float(sum(p.sum() for p in m.parameters())),
    }
    out(outdir, "optimizer_state", sig)


def sc_metric_average(outdir):
    import mihvd.keras as khvd

    cb = khvd.callbacks.MetricAverageCallback()
    logs = {"loss": float(hvd.rank()), "accuracy": 0.5 + hvd.rank(), "name": "x"}
    cb.on_epoch_end(0, logs)
    out(outdir, "metric_average", logs)


def sc_stall(outdir):
    # rank 0 issues a collective rank 1 never joins -> stall inspector warns then aborts (134).
    if hvd.rank() == 0:
        hvd.allreduce(torch.ones(1), name="lonely")
    else:
        time.sleep(30)
    out(outdir, "stall", {"unexpected": True})


def sc_fault(outdir):
    from mihvd.utils import faults

    for step in range(10):
        faults.maybe_inject(step)
        hvd.allreduce(torch.ones(1), name=f"s{step}")
    out(outdir, "fault", {"completed": True})


def sc_negotiated_order(outdir):
    """MIHVD_NEGOTIATE=1: every rank enqueues the same named collectives in a different order
    (allreduces of different shapes, a broadcast and an allgather interleaved). Without negotiation
    gloo would pair mismatched calls; the coordinator's order makes every rank agree."""
    import random

    from mihvd import basics

    r, n = hvd.rank(), hvd.size()
    eng = basics._ctx.engine
    assert eng is not None and basics._ctx.store is not None
    names = [f"t{i}" for i in range(12)]
    order = names[:]
    random.Random(100 + r).shuffle(order)
    handles = {}
    for i, nm in enumerate(order):
        k = int(nm[1:])
        handles[nm] = hvd.allreduce_async(torch.full((k + 1, 3), float(r + k)), name=nm, op=hvd.Sum)
        if i == 3 + r:  # the broadcast / allgather land at different positions on each rank
            handles["bc"] = hvd.broadcast_async(torch.full((5,), float(r)), root_rank=n - 1, name="bc")
        if i == 7 - r:
            handles["ag"] = hvd.allgather_async(torch.full((r + 1, 2), float(r)), name="ag")
    res = {nm: hvd.synchronize(h).tolist() for nm, h in handles.items()}
    ok = all(res[f"t{k}"] == torch.full((k + 1, 3), float(sum(q + k for q in range(n)))).tolist() for k in range(12))
    out(outdir, "negotiated_order", {"ok": ok, "bc": res["bc"], "ag": res["ag"], "launches": eng.launches,
                                     "fused": eng.fused_launches, "submitted": eng.neg.submitted})


def sc_negotiated_stall(outdir):
    """Rank 1 submits 'late' 3 s after rank 0: the coordinator names the missing rank, then the
    collective completes once rank 1 arrives."""
    r = hvd.rank()
    if r == 1:
        time.sleep(3.0)
    v = hvd.allreduce(torch.ones(2) * (r + 1), name="late", op=hvd.Sum)
    from mihvd import basics

    st = basics._ctx.engine.neg
    out(outdir, "negotiated_stall", {"value": v.tolist(), "warnings": st.warnings})


def sc_negotiated_mismatch(outdir):
    """Same name, different shapes on the two ranks: the coordinator refuses to launch it and
    every rank gets the error instead of a corrupted or hung collective."""
    r = hvd.rank()
    err = None
    try:
        hvd.allreduce(torch.ones(4 + r), name="shape_mismatch")
    except RuntimeError as e:
        err = str(e)
    ok = hvd.allreduce(torch.ones(3), name="after", op=hvd.Sum).tolist()
    out(outdir, "negotiated_mismatch", {"error": err, "after": ok})


def sc_torch_ops(outdir):
    """torch.ops.mihvd_dist.* custom ops: values and Horovod's autograd rules across ranks."""
    from mihvd.ops import collective_ops  # noqa: F401  (registers torch.ops.mihvd_dist)

    ops = torch.ops.mihvd_dist
    r, n = hvd.rank(), hvd.size()
    w = torch.full((3,), float(r + 1), requires_grad=True)
    y = ops.allreduce(w * 2.0, int(hvd.Average), "w")
    y.sum().backward()
    x = torch.full((r + 1, 2), float(r), requires_grad=True)
    g = ops.allgather(x, "x")
    (g * torch.arange(g.shape[0], dtype=torch.float32).unsqueeze(1)).sum().backward()
    b = torch.full((2,), float(r), requires_grad=True)
    bb = ops.broadcast(b, 0, "b")
    (bb * (r + 1)).sum().backward()
    t = torch.ones(4) * (r + 1)
    ops.allreduce_(t, int(hvd.Sum), "inplace")
    out(outdir, "torch_ops", {"y": y.tolist(), "wgrad": w.grad.tolist(), "g": g.tolist(), "xgrad": x.grad.tolist(),
                              "bb": bb.tolist(), "bgrad": b.grad.tolist(), "t": t.tolist()})


def sc_process_sets(outdir):
    """Horovod process sets on 3 ranks: {0, 2} registered through add_process_set, {1, 2} through
    init(process_sets=...) in main()."""
    r = hvd.rank()
    ps = hvd.add_process_set([0, 2])
    res = {"ids": {str(k): v for k, v in hvd.get_process_set_ids_and_ranks().items()}, "included": ps.included(),
           "set_rank": ps.rank(), "set_size": ps.size()}
    if ps.included():
        res["avg"] = hvd.allreduce(torch.full((3,), float(r)), process_set=ps).tolist()
        res["bcast"] = hvd.broadcast(torch.full((2,), float(r)), root_rank=2, process_set=ps).tolist()
        res["gather"] = hvd.allgather(torch.full((1, 2), float(r)), process_set=ps).tolist()
        o, _ = hvd.alltoall(torch.arange(4, dtype=torch.float32) + 10 * r, process_set=ps)
        res["alltoall"] = o.tolist()
    else:
        try:
            hvd.allreduce(torch.ones(1), process_set=ps)
        except ValueError as e:
            res["error"] = str(e)
    ps2 = PS_INIT[0]
    if ps2.included():
        res["sum2"] = hvd.allreduce(torch.ones(2) * (r + 1), op=hvd.Sum, process_set=ps2).tolist()
    res["world"] = hvd.allreduce(torch.ones(1), op=hvd.Sum).tolist()
    out(outdir, "process_sets", res)


def sc_api_extras(outdir):
    """Grouped / async / in-place / sparse forms of the collectives and PartialDistributedOptimizer."""
    r, n = hvd.rank(), hvd.size()
    res = {}
    ts = [torch.ones(3) * (r + 1), torch.full((2, 2), float(r)), torch.arange(4, dtype=torch.float64) * (r + 1)]
    h = hvd.grouped_allreduce_async(ts, op=hvd.Sum, name="ga")
    while not hvd.poll(h):
        time.sleep(0.001)
    res["grouped_async"] = [x.tolist() for x in hvd.synchronize(h)]
    res["grouped_unchanged"] = ts[0].tolist()
    hvd.grouped_allreduce_(ts, op=hvd.Average)
    res["grouped_inplace"] = [x.tolist() for x in ts]
    h = hvd.alltoall_async(torch.arange(n * 2, dtype=torch.float32) + 100 * r)
    o, splits = hvd.synchronize(h)
    res["alltoall_async"] = o.tolist()
    res["alltoall_splits"] = splits.tolist()
    h = hvd.reducescatter_async(torch.ones(n * 2, 3) * (r + 1), op=hvd.Sum)
    res["reducescatter_async"] = hvd.synchronize(h).tolist()
    g = hvd.grouped_reducescatter([torch.ones(n, 2) * (r + 1), torch.ones(n * 3) * r], op=hvd.Average)
    res["grouped_reducescatter"] = [x.tolist() for x in g]
    h = hvd.grouped_reducescatter_async([torch.ones(n) * (r + 1)], op=hvd.Sum)
    res["grouped_reducescatter_async"] = [x.tolist() for x in hvd.synchronize(h)]
    # grouped allgather: uneven first dims per rank (r+1 rows), two dtypes
    h = hvd.grouped_allgather_async([torch.full((r + 1, 2), float(r)), torch.arange(r + 1, dtype=torch.int64)])
    while not hvd.poll(h):
        time.sleep(0.001)
    res["grouped_allgather"] = [x.tolist() for x in hvd.synchronize(h)]
    res["grouped_allgather_sync"] = [x.tolist() for x in hvd.grouped_allgather([torch.ones(1) * r])]
    res["built"] = [hvd.ccl_built(), hvd.ddl_built(), hvd.mpi_built()]
    # sparse: rank r holds value (r+1) at row r and 1.0 at row 0 of a (n+1)x2 tensor
    idx = torch.tensor([[0, r], [0, 1]])
    sp = torch.sparse_coo_tensor(idx, torch.tensor([1.0, float(r + 1)]), (n + 1, 2))
    h = hvd.sparse_allreduce_async(sp, name="emb", op=hvd.Sum)
    res["sparse_sum"] = hvd.synchronize(h).to_dense().tolist()
    res["sparse_avg"] = hvd.synchronize(hvd.sparse_allreduce_async(sp, name="emb2")).to_dense().tolist()
    # PartialDistributedOptimizer: the head stays rank-local, the body is averaged
    torch.manual_seed(0)
    body, head = torch.nn.Linear(4, 4), torch.nn.Linear(4, 1)
    model = torch.nn.Sequential(body, torch.nn.Tanh(), head)
    opt = hvd.PartialDistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.0),
                                          named_parameters=model.named_parameters(), local_layers=[head], op=hvd.Sum)
    for _ in range(2):
        opt.zero_grad()
        model(torch.ones(2, 4) * (r + 1)).sum().backward()
        opt.step()
    res["head_grad"] = head.weight.grad.flatten().tolist()
    res["body_grad"] = body.bias.grad.tolist()
    ref_body = []
    for rr in range(n):
        torch.manual_seed(0)
        b2, h2 = torch.nn.Linear(4, 4), torch.nn.Linear(4, 1)
        torch.nn.Sequential(b2, torch.nn.Tanh(), h2)(torch.ones(2, 4) * (rr + 1)).sum().backward()
        ref_body.append(b2.bias.grad)
        if rr == r:
            res["head_ref"] = h2.weight.grad.flatten().tolist()
    res["body_ref"] = torch.stack(ref_body).sum(0).tolist()
    res["reduced_params"] = len(opt._params)
    out(outdir, "api_extras", res)


def sc_keras_tf_api(outdir):
    """Module-level functions of horovod.tensorflow.keras / horovod.tensorflow."""
    import mihvd.keras as hk
    import mihvd.tensorflow as htf

    r = hvd.rank()
    res = {"allreduce_scalar": hk.allreduce(float(r + 1)),
           "allreduce_sum": hk.allreduce(np.ones(2) * r, average=False).tolist(),
           "allgather": hk.allgather(np.full((1, 2), r)).tolist(),
           "broadcast": hk.broadcast(np.arange(3) + 10 * r, 1).tolist()}
    # broadcast_global_variables(root, model): weights and optimizer state of a compiled Model
    torch.manual_seed(r)
    mod = torch.nn.Linear(3, 2)
    m = hk.Model(mod)
    m.compile(hvd.DistributedOptimizer(torch.optim.Adam(mod.parameters(), lr=0.1),
                                       named_parameters=mod.named_parameters()), torch.nn.functional.cross_entropy)
    m.train_on_batch(torch.ones(4, 3) * (r + 1), torch.tensor([0, 1, 0, 1]))
    hk.broadcast_global_variables(0, m)
    res["weights"] = mod.weight.detach().flatten().tolist()
    res["exp_avg"] = m.optimizer.state[mod.weight]["exp_avg"].flatten().tolist()
    # load_model: every rank reads rank 0's file into a fresh module, optimizer wrapped for DP
    path = os.path.join(outdir, "km")
    if r == 0:
        m.save(path)
    hvd.barrier()
    m2 = hk.load_model(path, torch.nn.Linear(3, 2), optimizer=lambda ps: torch.optim.SGD(ps, lr=0.0))
    res["loaded"] = m2.module.weight.detach().flatten().tolist()
    res["loaded_dp"] = hasattr(m2.optimizer, "synchronize") and len(m2.optimizer._params) == 2
    # horovod.tensorflow: broadcast_variables of a dict / a list
    v = {"a": torch.ones(2) * r, "b": torch.zeros(1) + r}
    htf.broadcast_variables(v, 1)
    lst = [torch.full((2,), float(r))]
    htf.broadcast_variables(lst, 0)
    res["tf_bcast"] = [v["a"].tolist(), v["b"].tolist(), lst[0].tolist()]
    out(outdir, "keras_tf_api", res)


def sc_factor_rows(outdir):
    """fp32 factor gather (mihvd/parallel/factor.py) over gloo: each rank's rows of dW3 formed from
    the gathered factors equal those rows of the sum over ranks of a2_q^T dz_q."""
    from mihvd.parallel.factor import factor_rows_

    r, n = hvd.rank(), hvd.size()
    B, R = 24, 3136 // n

    def factors(q):
        g = torch.Generator().manual_seed(100 + q)
        return torch.randn(B, 3136, generator=g), torch.randn(B, 1024, generator=g)

    a2, dz0 = factors(r)
    dz_all = torch.empty(n, B, 1024)
    dz = dz0.clone()  # a buffer of its own (the trainer's layout: dz never aliases dz_all)
    a2_send, a2_recv = torch.empty(n, B, R), torch.empty(n, B, R)
    out_rows = torch.empty(R, 1024)
    factor_rows_(out_rows, a2, dz, dz_all, a2_send, a2_recv, r, n)
    ref = sum(f[0].double().t() @ f[1].double() for f in map(factors, range(n)))[r * R:(r + 1) * R]
    rel = ((out_rows.double() - ref).norm() / ref.norm()).item()
    out(outdir, "factor_rows", {"rel": rel, "R": R, "dz_gathered": bool(torch.equal(dz_all[(r + 1) % n],
                                                                                     factors((r + 1) % n)[1]))})


def sc_factor_full(outdir):
    """The replicated fp32 factor plane's exchange + GEMM (mihvd/parallel/factor.py) over gloo: every
    rank's dW3 from the in-place all-gathered a2 / dz equals the sum over ranks of a2_q^T dz_q, on
    every rank, also where 3136 rows do not split evenly over the ranks."""
    from mihvd.parallel.factor import factor_full_

    r, n = hvd.rank(), hvd.size()
    B = 24

    def factors(q):
        g = torch.Generator().manual_seed(200 + q)
        return torch.randn(B, 3136, generator=g), torch.randn(B, 1024, generator=g)

    a2_all, dz_all = torch.full((n, B, 3136), float("nan")), torch.full((n, B, 1024), float("nan"))
    a2_all[r], dz_all[r] = factors(r)  # this rank's slices: written by conv2_fwd / the head in the trainer
    out_full = torch.empty(3136, 1024)
    factor_full_(out_full, a2_all, dz_all, r, n)
    ref = sum(f[0].double().t() @ f[1].double() for f in map(factors, range(n)))
    rel = ((out_full.double() - ref).norm() / ref.norm()).item()
    out(outdir, "factor_full", {"rel": rel, "gathered": all(torch.equal(a2_all[q], factors(q)[0]) and
                                                            torch.equal(dz_all[q], factors(q)[1]) for q in range(n))})


PS_INIT = []


def main():
    scenario, outdir = sys.argv[1], sys.argv[2]
    if scenario == "process_sets":
        PS_INIT.append(hvd.ProcessSet([1, 2]))
        hvd.init(process_sets=PS_INIT)
    else:
        hvd.init()
    globals()["sc_" + scenario](outdir)
    hvd.shutdown()


if __name__ == "__main__":
    main()
