"""Framework-owned RCCL communicator (csrc/kernels/rccl_comm.cpp, mihvd/parallel/rccl.py) on the
box's one GPU: every collective eagerly and replayed from a HIP graph, and the fused fp32 trainer's
collective path over it (MIHVD_COMM=native, MIHVD_FORCE_COLLECTIVES=1) against the trainer with no
collectives. Multi-GPU runs of it are the driver's (RCCL refuses two ranks on one GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_rccl_comm_one_gpu(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = tmp_path / "res.json"
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "tests", "workers", "native_comm_worker.py"),
           str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads(out.read_text())
    assert r["world"] == 1
    for k in ("allreduce_sum", "allreduce_avg", "allreduce_bf16", "all_gather", "reduce_scatter", "all_to_all",
              "broadcast", "many"):
        assert r[k], (k, r)
    assert r["graph"] == 1024.0, r
    assert r["async_error"] == 0
    assert r["trainer_native_comm"]
    # the same collective-free arithmetic (world-1 sums are exact): the updates agree to fp32
    # summation order (the collective path applies the dense/kernel update in a different launch)
    assert r["trainer_rel_diff"] < 1e-5, r


def test_native_engine_one_gpu(tmp_path):
    """The C++ engine thread (csrc/kernels/engine.cpp) at world size 1: negotiation cycles, fusion,
    in-place big tensors, stream ordering, DistributedOptimizer bit-equality, clean shutdown."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = tmp_path / "eng.json"
    env = dict(os.environ, PYTHONPATH=ROOT, MIHVD_ENGINE="native", MIHVD_FUSION_THRESHOLD=str(1 << 20))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", "29563", os.path.join(ROOT, "tests", "workers", "native_engine_worker.py"),
           str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads(out.read_text())
    assert r["engine"] == "NativeEngine" and r["world"] == 1, r
    assert r["values_exact"] and r["small_exact"] and r["big_exact"], r
    assert r["small_tensors"] == 24 and r["small_collectives"] < 24, r  # fused
    assert r["optimizer_bitwise"] and r["optimizer_collectives"] >= 12, r
    assert r["cnn_rel_diff"] < 1e-5, r
    assert r["stats"]["cycles"] > 0 and r["stopped"], r


@pytest.mark.parametrize("nranks", [2, 8])
def test_native_engine_ranks_out_of_order(tmp_path, nranks):
    """The C++ engine across GPUs (one rank per GPU; RCCL refuses two ranks on one device): the
    same 80 names enqueued in a different order on every rank (more than one 64-signature announce
    round), big tensors above the fusion threshold in rank-dependent order, then the same names
    again from the signature cache; every result equals the closed-form sum, and every rank stops
    cleanly. Needs ``nranks`` GPUs: skipped on a one-GPU box."""
    import torch

    if torch.cuda.device_count() < nranks:
        pytest.skip(f"needs {nranks} GPUs (RCCL runs one rank per device)")
    out = tmp_path / "eng"
    env = dict(os.environ, PYTHONPATH=ROOT, MIHVD_ENGINE="native", MIHVD_FUSION_THRESHOLD=str(1 << 20))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
           "--master-addr", "127.0.0.1", "--master-port", "29567",
           os.path.join(ROOT, "tests", "workers", "native_engine_multi_worker.py"), str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    for r in range(nranks):
        res = json.loads((tmp_path / f"eng.{r}").read_text())
        assert res["world"] == nranks and res["ok"] == [True, True] and res["stopped"], res


def test_bucket_plane_carries_distributed_optimizer(tmp_path):
    """DistributedOptimizer's buckets -- and the public collective API (allreduce, broadcast,
    allgather, reducescatter, alltoall, broadcast_parameters) -- go through the framework-owned RCCL
    bucket plane
    (collectives.BucketPlane: NativeComm on a high-priority side stream), eagerly and inside a
    captured whole-step HIP graph, and bench.py --impl torch / torch-graph report it as the
    communicator (config.rccl_comm, RCCL's own count in config.rccl_nranks). World size 1 with the
    collectives forced on: the parameters must equal the plain optimizer's within its own run-to-run
    noise (MIOpen's conv backward need not be bitwise reproducible)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, PYTHONPATH=ROOT, MIHVD_FORCE_COLLECTIVES="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    out = tmp_path / "plane.json"
    run = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port"]
    p = subprocess.run(run + ["29565", os.path.join(ROOT, "tests", "workers", "plane_worker.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads(out.read_text())
    for key in ("eager", "graph"):
        assert r[key]["plane"] and r[key]["nranks"] == 1, r
        assert r[key]["launched"] >= r[key]["buckets"] * 3, r  # every bucket of every step (eager warm-up too)
        assert r[key]["rel"] <= max(10 * r[key]["noise"], 1e-6), r
    # the public API outside DistributedOptimizer goes through the same plane (a launch per call)
    assert all(r["api"].values()), r["api"]
    c = r["api_counts"]
    # (broadcast_parameters is a no-op at world size 1: only hvd.broadcast counts here)
    assert c.get("allreduce", 0) >= 3 and c.get("broadcast", 0) >= 1 and c.get("allgather", 0) >= 2, c
    assert c.get("reducescatter", 0) >= 1 and c.get("alltoall", 0) >= 2, c
    # after an elastic reset the optimizer's buckets run on the new world's plane
    e = r["elastic"]
    assert e["had_plane"] and e["new_plane"] and e["uses_new"] and e["launched_after"] >= 2, e
    for i, impl in enumerate(("torch", "torch-graph")):
        p = subprocess.run(run + [str(29567 + i), os.path.join(ROOT, "bench.py"), "--impl", impl, "--steps", "10",
                                  "--warmup", "3"], env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        rec = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")][-1]
        assert rec["config"]["rccl_comm"] == "bucket plane" and rec["config"]["rccl_nranks"] == 1, rec


def test_bench_reports_rccl_rank_count(tmp_path):
    """bench.py's default (fused) step at one GPU prints RCCL's own rank count (ncclCommCount of a
    witness communicator; the trainer's own with forced collectives)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "2"], env=env,
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    rec = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")][-1]
    assert rec["config"]["rccl_nranks"] == 1 and rec["config"]["rccl_user_rank"] == 0, rec
    assert rec["config"]["rccl_nranks_agree"] is True, rec
