"""GPU multi-process scenarios for the fused trainer (launched by tests/test_fused_distributed_gpu.py).

usage: python fused_worker.py <scenario> <outdir>
  rccl_graph : world 1 over RCCL with MIHVD_FORCE_COLLECTIVES=1 — the allreduce is captured in the
               HIP graph; results must equal a trainer without collectives.
  dp_gloo    : 2 ranks (gloo, both on cuda:0), B=50 each == one trainer with B=100 (dropout off).
  dp_gloo_shard : 2 ranks, sharded dense/kernel optimizer == the unsharded factor-gather step.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import mihvd.torch as hvd  # noqa: E402
from mihvd.models.fused_mnist import W3_START as FLAT_W3, FusedMNISTTrainer  # noqa: E402
from mihvd.utils.data import synthetic_mnist  # noqa: E402


def data(n, seed=3):
    (x, y), _ = synthetic_mnist(n_train=n, n_test=10, seed=seed)
    return torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0, torch.from_numpy(y.astype("int64")).cuda()


def sc_rccl_graph(outdir):
    # 50 steps per epoch: no reshuffle inside the (up to 44) steps, so eager and graph-replayed
    # schedules of different lengths see the same batches
    X, Y = data(5000)
    prec = os.environ.get("MIHVD_TEST_PRECISION", "bf16")
    op = hvd.Adasum if os.environ.get("MIHVD_TEST_OP") == "adasum" else None
    a = FusedMNISTTrainer(batch_size=100, seed=1, device="cuda", precision=prec, op=op,
                          shard_optimizer=os.environ.get("MIHVD_SHARD_W3") == "1")
    assert a.collectives, "MIHVD_FORCE_COLLECTIVES should enable the allreduce path"
    a.set_device_dataset(X, Y, seed=4)
    p0 = a.params.clone()
    select = None
    if os.environ.get("MIHVD_XGMI") == "auto":
        # plane selection: validation against the process group + timed graph replays of both planes
        select = a.select_data_plane(steps=10, steps_per_replay=5)
    pre = a.global_step
    captured = a.build_graph(steps_per_replay=5)
    for _ in range(4):
        a.run_graph()
    os.environ["MIHVD_FORCE_COLLECTIVES"] = "0"
    b = FusedMNISTTrainer(batch_size=100, seed=1, device="cuda", precision=prec)
    b.set_device_dataset(X, Y, seed=4)
    for _ in range(pre):
        b.device_step()
    b.build_graph(steps_per_replay=5)
    for _ in range(4):
        b.run_graph()
    torch.cuda.synchronize()
    # the step has no atomics: with a world of one, the collective data plane (factor gather + RCCL
    # allreduce, captured in the graph) must reproduce the local step bit for bit
    a.gather_full_state()
    rel = ((a.params - b.params).norm() / (b.params - p0).norm()).item()
    bitwise = bool(torch.equal(a.params, b.params))
    with open(os.path.join(outdir, "rccl_graph.json"), "w") as f:
        json.dump({"captured": captured, "bitwise": bitwise, "rel_update_diff": rel, "steps": a.global_step,
                   "pre_steps": pre, "select": select,
                   "shard": a.shard_w3, "plane": a.data_plane(), "loss": a.last_loss(),
                   "native_comm": a.ncomm is not None, "precision": a.precision,
                   "engine_running": hvd.engine_running() if hasattr(hvd, "engine_running") else None,
                   "loss_ref": b.last_loss()}, f)
    a.close()


def sc_dp_gloo(outdir):
    r = hvd.rank()
    X, Y = data(600)
    prec = os.environ.get("MIHVD_TEST_PRECISION", "bf16")
    tr = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision=prec,
                           shard_optimizer=os.environ.get("MIHVD_SHARD_W3") == "1" if prec == "fp32" else None)
    assert tr.gather or prec == "fp32"
    tr.keep_w3_grad = True  # gradients are compared below
    tr.broadcast(0)
    ref = FusedMNISTTrainer(batch_size=100, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision=prec, world_size=1)
    ref.keep_w3_grad = True
    p0 = ref.params.clone()
    grel = None
    for step in range(3):
        xb = X[step * 100:(step + 1) * 100]
        yb = Y[step * 100:(step + 1) * 100]
        tr.train_step(xb[r * 50:(r + 1) * 50], yb[r * 50:(r + 1) * 50])
        ref.train_step(xb, yb)
        torch.cuda.synchronize()
        if step == 0:
            # allreduced SUM of the two per-rank batch means == 2 x the 100-sample batch mean
            red, want = tr.reduced_grads() / 2, ref.grads
            if tr.f32 and tr.shard_w3:  # the sharded fp32 planes reduce this rank's dense/kernel rows only
                R = tr._f32_R
                rows = slice(FLAT_W3 + r * R * 1024, FLAT_W3 + (r + 1) * R * 1024)
                red, want = torch.cat([red[:FLAT_W3], red[rows]]), torch.cat([want[:FLAT_W3], want[rows]])
            grel = ((red - want).norm() / want.norm()).item()
    tr.gather_full_state()
    rel = ((tr.params - ref.params).norm() / (ref.params - p0).norm()).item()
    mx = (tr.params - ref.params).abs().max().item()
    spread = hvd.allgather(tr.params[:4096].cpu().view(1, -1))
    tr.check_xgmi()
    w3 = tr.params[FLAT_W3:].view(3136, 1024)
    w3_spread = hvd.allgather(w3[::97].cpu().reshape(1, -1))  # every rank's copy of dense/kernel (sampled)
    rec = {"gather": tr.gather, "xgmi": tr.data_plane() == "xgmi", "grad_rel": grel, "rel_update_diff": rel, "max": mx,
           "rank_spread": (spread - spread[0]).abs().max().item(),
           "w3_rank_spread": (w3_spread - w3_spread[0]).abs().max().item(),
           "colaunched": getattr(tr.xplane, "colaunched", 0) if tr.xplane is not None else 0,
           "shared_device": bool(getattr(tr.xplane, "shared_device", False)),
           "xgmi_error": int(tr.ops.xgmi_error(tr.xplane.ctx)) if tr.xplane is not None else None}
    tr.close()
    with open(os.path.join(outdir, f"dp_gloo.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_dp_gloo_shard(outdir):
    """Sharded dense/kernel optimizer == unsharded factor-gather step, bit for bit (2 ranks)."""
    r = hvd.rank()
    X, Y = data(600)
    trs = [FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision="bf16", shard_optimizer=sh)
           for sh in (False, True)]
    for tr in trs:
        tr.broadcast(0)
    assert not trs[0].shard_w3 and trs[1].shard_w3
    for step in range(3):
        xb = X[step * 100:(step + 1) * 100]
        yb = Y[step * 100:(step + 1) * 100]
        for tr in trs:
            tr.train_step(xb[r * 50:(r + 1) * 50], yb[r * 50:(r + 1) * 50])
    torch.cuda.synchronize()
    trs[1].gather_full_state()
    same = {name: bool(torch.equal(getattr(trs[0], name), getattr(trs[1], name))) for name in ("params", "m", "v")}
    same["shadow_w3"] = bool(torch.equal(trs[0].w3_shadow(), trs[1].w3_shadow()))
    rec = {"same": same, "loss": trs[1].last_loss(), "loss_ref": trs[0].last_loss(),
           "planes": [tr.data_plane() for tr in trs]}
    for tr in trs:
        tr.close()
    with open(os.path.join(outdir, f"dp_gloo_shard.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_dp_gloo_switch(outdir):
    """Plane / sharding switches between steps (xGMI sharded -> RCCL replicated -> xGMI replicated
    -> xGMI sharded -> RCCL sharded) == a trainer that stays on the process group, unsharded, bit for
    bit (2 ranks: the two-term sums commute exactly)."""
    r = hvd.rank()
    X, Y = data(1200)
    a = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision="bf16", shard_optimizer=True)
    ref = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision="bf16", shard_optimizer=False)
    for tr in (a, ref):
        tr.broadcast(0)
    ref._set_plane(False, False)
    plan = [(True, True), (False, False), (True, False), (True, True), (False, True)]
    step, planes = 0, []
    for xg, sh in plan:
        a._set_plane(xg, sh)
        planes.append(a.data_plane() + ("-shard" if a.shard_w3 else "-replicated"))
        for _ in range(2):
            xb = X[step * 100:(step + 1) * 100]
            yb = Y[step * 100:(step + 1) * 100]
            for tr in (a, ref):
                tr.train_step(xb[r * 50:(r + 1) * 50], yb[r * 50:(r + 1) * 50])
            step += 1
    torch.cuda.synchronize()
    a.gather_full_state()
    same = {name: bool(torch.equal(getattr(a, name), getattr(ref, name))) for name in ("params", "m", "v")}
    same["shadow_w3"] = bool(torch.equal(a.w3_shadow(), ref.w3_shadow()))
    rec = {"same": same, "planes": planes, "loss": a.last_loss(), "loss_ref": ref.last_loss()}
    for tr in (a, ref):
        tr.close()
    with open(os.path.join(outdir, f"dp_gloo_switch.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_dp_gloo_switch_f32(outdir):
    """fp32 plane switches between steps, into and out of the replicated factor plane (whose
    conv2_fwd / head write a2 / dz into the gather buffers: the views are rebound at every switch):
    reduce-scatter sharded -> factor replicated -> RCCL replicated -> factor sharded -> factor
    replicated, against a trainer that stays on the replicated allreduce. The planes sum dW3 in
    different orders, so the match is to fp32 rounding of the update, and every rank stays equal."""
    r = hvd.rank()
    X, Y = data(1200)
    a = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision="fp32",
                          shard_optimizer=True)
    ref = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", precision="fp32",
                            shard_optimizer=False)
    for tr in (a, ref):
        tr.broadcast(0)
    p0 = ref.params.clone()
    ref._set_plane(False, False)
    plan = [(True, False), (False, True), (False, False), (True, True), (False, True)]  # (shard, factor)
    step, planes = 0, []
    for sh, fac in plan:
        a._set_plane(False, sh, fac)
        planes.append(a.data_plane() + ("-shard" if a.shard_w3 else "-replicated"))
        for _ in range(2):
            xb = X[step * 100:(step + 1) * 100]
            yb = Y[step * 100:(step + 1) * 100]
            for tr in (a, ref):
                tr.train_step(xb[r * 50:(r + 1) * 50], yb[r * 50:(r + 1) * 50])
            step += 1
    torch.cuda.synchronize()
    a.gather_full_state()
    rel = ((a.params - ref.params).norm() / (ref.params - p0).norm()).item()
    spread = hvd.allgather(a.params.cpu().view(1, -1))
    rec = {"rel": rel, "planes": planes, "loss": a.last_loss(), "loss_ref": ref.last_loss(),
           "rank_spread": (spread - spread[0]).abs().max().item()}
    for tr in (a, ref):
        tr.close()
    with open(os.path.join(outdir, f"dp_gloo_switch_f32.{r}.json"), "w") as f:
        json.dump(rec, f)


def _tf_adam_host(p, g, t, lr, b1=0.9, b2=0.999, eps=1e-8):
    """One TF1 Adam step from zero slots, float64 (tensorflow_mnist.py:130)."""
    m = (1 - b1) * g
    v = (1 - b2) * g * g
    lr_t = lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)
    return p - lr_t * m / (v.sqrt() + eps)


def sc_dp_gloo_n(outdir):
    """N ranks (gloo, all on cuda:0) x B=MIHVD_TEST_B samples: the first step's reduced gradient
    equals the sum of N single-process gradients on the same per-rank batches (each from a world-1
    trainer with the same weights), its update equals TF1 Adam on their average, and 10 more steps
    keep every rank identical and the loss falling. Precision / data plane / sharding from env."""
    r, n = hvd.rank(), hvd.size()
    B = int(os.environ.get("MIHVD_TEST_B", "50"))
    prec = os.environ.get("MIHVD_TEST_PRECISION", "bf16")
    shard = os.environ.get("MIHVD_SHARD_W3", "0") == "1"
    lr = 1e-3 * n
    X, Y = data(n * B * 12, seed=7)
    tr = FusedMNISTTrainer(batch_size=B, lr=lr, dropout=0.0, seed=1, device="cuda", precision=prec,
                           shard_optimizer=shard)
    tr.keep_w3_grad = True
    tr.broadcast(0)
    if os.environ.get("MIHVD_XGMI", "off") != "off" and tr.xplane is not None:
        tr._set_plane(True, tr.shard_w3)
    p0 = tr.params.clone()
    ref = FusedMNISTTrainer(batch_size=B, lr=lr, dropout=0.0, seed=1, device="cuda", world_size=1, precision=prec)
    ref.keep_w3_grad = True
    snap = ref._snapshot()
    gsum = torch.zeros_like(ref.grads)
    for q in range(n):
        ref._restore(snap)
        ref.train_step(X[q * B:(q + 1) * B], Y[q * B:(q + 1) * B])
        torch.cuda.synchronize()
        gsum += ref.grads
    tr.train_step(X[r * B:(r + 1) * B], Y[r * B:(r + 1) * B])
    torch.cuda.synchronize()
    red = tr.reduced_grads()
    if tr.gather or (tr.f32 and tr.shard_w3):
        # the factor-gather plane forms dW3 only for the rows whose optimizer this rank owns; the
        # fp32 sharded optimizer reduce-scatters them (or forms them from the gathered fp32 factors)
        if tr.f32:
            R = tr._f32_R
            rows = slice(FLAT_W3 + r * R * 1024, FLAT_W3 + (r + 1) * R * 1024)
        else:
            lo, hi = tr._w3_tiles
            rows = slice(FLAT_W3 + lo * 64 * 1024, FLAT_W3 + min(hi * 64, 3136) * 1024)
        red = torch.cat([red[:FLAT_W3], red[rows]])
        gsum_c = torch.cat([gsum[:FLAT_W3], gsum[rows]])
    else:
        gsum_c = gsum
    grel = ((red - gsum_c).norm() / gsum_c.norm()).item()
    tr.gather_full_state()
    upd = tr.params.double() - p0.double()
    upd_ref = _tf_adam_host(p0.double(), gsum.double() / n, 1, lr) - p0.double()
    urel = ((upd - upd_ref).norm() / upd_ref.norm()).item()
    losses = []
    for step in range(1, 11):
        i = (step * n + r) * B
        tr.train_step(X[i:i + B], Y[i:i + B])
        losses.append(tr.last_loss())
    tr.gather_full_state()
    spread = hvd.allgather(tr.params.cpu().view(1, -1))
    rec = {"grad_rel": grel, "upd_rel": urel, "losses": losses, "plane": tr.data_plane(), "shard": tr.shard_w3,
           "gather": tr.gather, "rank_spread": (spread - spread[0]).abs().max().item(), "n": n}
    tr.close()
    with open(os.path.join(outdir, f"dp_gloo_n.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_bench_flow(outdir):
    """bench.py's fused flow at N ranks without bench.py: per-rank synthetic shards (shared class
    templates), lr 1e-3 x N, dropout 0.5, select_data_plane, 20-step graphs, 2 replays."""
    from mihvd.utils.data import synthetic_mnist

    r, n = hvd.rank(), hvd.size()
    prec = os.environ.get("MIHVD_TEST_PRECISION", "fp32")
    (x, y), _ = synthetic_mnist(n_train=60 * 100, n_test=10, seed=1234, sample_seed=r)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=100, lr=1e-3 * n, seed=42, device="cuda", precision=prec)
    tr.set_device_dataset(X, Y)
    rep = tr.select_data_plane() if tr.collectives else {"plane": "none"}
    tr.build_graph(steps_per_replay=20)
    losses = []
    for _ in range(3):
        tr.run_graph()
        losses.append(tr.last_loss())
    rec = {"losses": losses, "plane": rep.get("plane"), "shard": tr.shard_w3, "n": n}
    tr.close()
    with open(os.path.join(outdir, f"bench_flow.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_ckpt_shard(outdir):
    """2 ranks, sharded dense/kernel optimizer: MonitoredTrainingSession checkpoints (collective
    gather on every rank, rank 0 writes), a fresh session restores on rank 0 and broadcasts; the
    restored state equals the trained full state bit for bit on every rank."""
    import mihvd.tensorflow as tfh

    r = hvd.rank()
    X, Y = data(1200, seed=9)
    ck = os.path.join(outdir, "ckpt")
    prec = os.environ.get("MIHVD_TEST_PRECISION", "bf16")

    def session(tr, last):
        hooks = [tfh.BroadcastGlobalVariablesHook(0), tfh.StopAtStepHook(last_step=last)]
        with tfh.MonitoredTrainingSession(checkpoint_dir=ck if r == 0 else None, hooks=hooks, state=tr,
                                          save_checkpoint_steps=2) as sess:
            while not sess.should_stop():
                s = tr.global_step
                sess.run(lambda: tr.train_step(X[(2 * s + r) * 50:(2 * s + r + 1) * 50],
                                               Y[(2 * s + r) * 50:(2 * s + r + 1) * 50]))
        return sess

    a = FusedMNISTTrainer(batch_size=50, lr=2e-3, dropout=0.0, seed=1, device="cuda", shard_optimizer=True,
                          precision=prec)
    sharded = a.shard_w3
    session(a, 5)
    a.gather_full_state()
    full = {k: getattr(a, k).clone() for k in ("params", "m", "v")}
    saved = sorted(os.listdir(ck)) if r == 0 else []
    hvd.barrier()
    b = FusedMNISTTrainer(batch_size=50, lr=2e-3, dropout=0.0, seed=2, device="cuda", shard_optimizer=True,
                          precision=prec)
    sess = session(b, 5)  # restores step 5 on rank 0, broadcasts, runs no step
    b.gather_full_state()
    same = {k: bool(torch.equal(getattr(b, k), full[k])) for k in full}
    rec = {"sharded": sharded, "same": same, "restored": sess.restored_from, "step": b.global_step, "saved": saved}
    a.close()
    b.close()
    with open(os.path.join(outdir, f"ckpt_shard.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_select_check(outdir):
    """2 ranks: plane selection's end-to-end consistency check (xGMI vs RCCL steps from one snapshot)."""
    r = hvd.rank()
    X, Y = data(2000, seed=5)
    tr = FusedMNISTTrainer(batch_size=50, lr=2e-3, seed=1, device="cuda", precision="bf16", shard_optimizer=True)
    tr.broadcast(0)
    tr.set_device_dataset(X, Y, seed=3 + r)
    rep = tr.select_data_plane(steps=6, steps_per_replay=3, shard_options=[True])
    rep["final_plane"] = tr.data_plane()
    tr.close()
    with open(os.path.join(outdir, f"select_check.{r}.json"), "w") as f:
        json.dump(rep, f)


def main():
    scenario, outdir = sys.argv[1], sys.argv[2]
    hvd.init()
    globals()["sc_" + scenario](outdir)
    hvd.shutdown()


if __name__ == "__main__":
    main()
