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
from mihvd.models.fused_mnist import FusedMNISTTrainer  # noqa: E402
from mihvd.utils.data import synthetic_mnist  # noqa: E402


def data(n, seed=3):
    (x, y), _ = synthetic_mnist(n_train=n, n_test=10, seed=seed)
    return torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0, torch.from_numpy(y.astype("int64")).cuda()


def sc_rccl_graph(outdir):
    # 50 steps per epoch: no reshuffle inside the (up to 44) steps, so eager and graph-replayed
    # schedules of different lengths see the same batches
    X, Y = data(5000)
    a = FusedMNISTTrainer(batch_size=100, seed=1, device="cuda",
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
    b = FusedMNISTTrainer(batch_size=100, seed=1, device="cuda")
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
                   "loss_ref": b.last_loss()}, f)
    a.close()


def sc_dp_gloo(outdir):
    r = hvd.rank()
    X, Y = data(600)
    tr = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda")
    assert tr.gather == (os.environ.get("MIHVD_FC_GATHER", "1") != "0")
    tr.keep_w3_grad = True  # gradients are compared below
    tr.broadcast(0)
    ref = FusedMNISTTrainer(batch_size=100, lr=1e-3, dropout=0.0, seed=1, device="cuda", world_size=1)
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
            grel = ((tr.reduced_grads() / 2 - ref.grads).norm() / ref.grads.norm()).item()
    rel = ((tr.params - ref.params).norm() / (ref.params - p0).norm()).item()
    mx = (tr.params - ref.params).abs().max().item()
    spread = hvd.allgather(tr.params[:4096].cpu().view(1, -1))
    tr.check_xgmi()
    rec = {"gather": tr.gather, "xgmi": tr.data_plane() == "xgmi", "grad_rel": grel, "rel_update_diff": rel, "max": mx,
           "rank_spread": (spread - spread[0]).abs().max().item()}
    tr.close()
    with open(os.path.join(outdir, f"dp_gloo.{r}.json"), "w") as f:
        json.dump(rec, f)


def sc_dp_gloo_shard(outdir):
    """Sharded dense/kernel optimizer == unsharded factor-gather step, bit for bit (2 ranks)."""
    r = hvd.rank()
    X, Y = data(600)
    trs = [FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", shard_optimizer=sh)
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
    a = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", shard_optimizer=True)
    ref = FusedMNISTTrainer(batch_size=50, lr=1e-3, dropout=0.0, seed=1, device="cuda", shard_optimizer=False)
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


def main():
    scenario, outdir = sys.argv[1], sys.argv[2]
    hvd.init()
    globals()["sc_" + scenario](outdir)
    hvd.shutdown()


if __name__ == "__main__":
    main()
