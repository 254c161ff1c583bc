"""Multi-process CPU tests: ranks are separate processes launched by ``mihvdrun`` (gloo backend),
rendezvousing over 127.0.0.1 — the "multi-node without a cluster" strategy of SURVEY.md §4."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "workers", "dist_worker.py")

pytestmark = pytest.mark.slow


def run_scenario(tmp_path, scenario, np_=2, env=None, timeout=120, expect_ok=True):
    e = dict(os.environ)
    e.update({"MIHVD_BACKEND": "gloo", "PYTHONPATH": ROOT, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    cmd = [sys.executable, "-m", "mihvd.runner", "-np", str(np_), "--allow-run-as-root", "-bind-to", "none",
           "-map-by", "slot", "-x", "PATH", "-mca", "pml", "ob1", "-mca", "btl", "^openib",
           sys.executable, WORKER, scenario, str(tmp_path)]
    p = subprocess.run(cmd, env=e, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    if expect_ok:
        assert p.returncode == 0, p.stdout + p.stderr
    outs = []
    for r in range(np_):
        f = tmp_path / f"{scenario}.{r}.json"
        outs.append(json.loads(f.read_text()) if f.exists() else None)
    return p, outs


def test_collectives_two_ranks(tmp_path):
    _, (a, b) = run_scenario(tmp_path, "collectives")
    base = [float(i) for i in range(6)]
    assert a["sum"] == [2 * x + 1 for x in base] == b["sum"]
    assert a["avg"] == [x + 0.5 for x in base]
    assert a["min"] == base and a["max"] == [x + 1 for x in base]
    assert a["bf16"] == a["sum"]
    assert a["fp16"] == a["avg"]
    assert a["allgather"] == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]] == b["allgather"]
    assert a["broadcast"] == [1.0] * 3 and b["broadcast_"] == [0.0] * 3
    # alltoall: rank r receives slice r from every rank
    assert a["alltoall"] == [0.0, 1.0, 100.0, 101.0] and b["alltoall"] == [2.0, 3.0, 102.0, 103.0]
    assert a["reducescatter"] == [[3.0] * 3] * 2
    assert a["object"] == {"rank": 0, "msg": "hi"} == b["object"]
    assert a["allgather_object"] == [0, 10]
    assert a["grouped"] == [[1.0] * 3, [[3.0, 3.0], [3.0, 3.0]]]
    assert a["async"] == [1.0] * 4
    assert a["join"] == 1


@pytest.mark.parametrize("np_", [2, 4])
def test_f32_factor_rows_gather(tmp_path, np_):
    """The fp32 factor-gather plane's exchange + GEMM (mihvd/parallel/factor.py) on the host
    collectives: rank r's dW3 rows from every rank's dz (all-gather) and a2 columns (all-to-all)."""
    _, outs = run_scenario(tmp_path, "factor_rows", np_=np_)
    for o in outs:
        assert o["R"] == 3136 // np_ and o["dz_gathered"], o
        assert o["rel"] < 1e-6, o


@pytest.mark.parametrize("np_", [2, 3])
def test_f32_factor_full_gather(tmp_path, np_):
    """The replicated fp32 factor plane's in-place exchange + GEMM (mihvd/parallel/factor.py) on the
    host collectives: every rank forms all of dW3 from every rank's a2 and dz (3 ranks: 3136 rows do
    not split evenly, which this plane does not need)."""
    _, outs = run_scenario(tmp_path, "factor_full", np_=np_)
    for o in outs:
        assert o["gathered"], o
        assert o["rel"] < 1e-6, o


def test_dp_equivalence(tmp_path):
    _, outs = run_scenario(tmp_path, "dp_equivalence")
    for o in outs:
        assert o["maxdiff_0"] < 1e-5 and o["maxdiff_67108864"] < 1e-5
        assert o["nbuckets_0"] > 1 and o["nbuckets_67108864"] == 1


def test_dp_equivalence_four_ranks(tmp_path):
    _, outs = run_scenario(tmp_path, "dp_equivalence", np_=4)
    assert all(o["maxdiff_0"] < 1e-5 for o in outs)


def test_fusion_autotune(tmp_path):
    env = {"MIHVD_AUTOTUNE": "1", "MIHVD_AUTOTUNE_CANDIDATES": "0.0001,64", "MIHVD_AUTOTUNE_WARMUP_STEPS": "1",
           "MIHVD_AUTOTUNE_TRIAL_STEPS": "3"}
    _, (a, b) = run_scenario(tmp_path, "autotune", env=env)
    for o in (a, b):
        assert o["done"] and o["final"] == o["best"] and o["maxdiff"] < 1e-5
        assert len(o["seen"]) == 2  # both candidates were tried
    assert a["best"] == b["best"]  # every rank chose the same threshold


def test_backward_passes_per_step(tmp_path):
    _, outs = run_scenario(tmp_path, "bpps")
    assert all(o["diff"] < 1e-4 for o in outs)


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_adasum(tmp_path, np_):
    _, outs = run_scenario(tmp_path, "adasum", np_=np_)
    for o in outs:
        assert o["diff"] < 1e-9
        assert o["param_spread"] < 1e-6


@pytest.mark.parametrize("np_", [2, 3, 4, 8])
def test_adasum_vector_halving(tmp_path, np_):
    """Adasum by vector halving / distance doubling (mihvd/parallel/adasum.py adasum_vhdd_; the
    same code runs over the framework-owned RCCL communicator on GPUs) matches the single-process
    oracle of the pairing tree at 2, 3 (one folded rank), 4 and 8 ranks, and a power-of-two rank
    sends about 2 S (N - 1) / N bytes (whole-vector doubling: log2(N) S)."""
    _, outs = run_scenario(tmp_path, "adasum_vhdd", np_=np_, timeout=240)
    p2 = 1 << (np_.bit_length() - 1)
    for pos, o in enumerate(outs):
        assert o["rel"] < 1e-5, o
        S = o["numel"] * o["elem"]
        if pos < p2 and p2 == np_:
            assert o["bytes"] <= 2 * S * (np_ - 1) / np_ + 64 * 4 * 2 * np_, (o, S)
            assert o["bytes"] < S * max(1, (np_ - 1).bit_length()) or np_ == 2


@pytest.mark.parametrize("np_", [2, 8])
def test_engine_slot_agreement_over_store(tmp_path, np_):
    """The C++ engine's slot agreement (csrc/runtime/slot_agreement.h: the code csrc/kernels/engine.cpp
    runs over its RCCL control communicator) over the TCP store transport, at 2 and 8 CPU ranks:
    every rank enqueues the same 120 collectives in its own order -- 80 at once (more than one
    64-hash announce block: over 64 new slots agreed in one cycle), 40 staggered by rank (slots
    pending on some ranks only), the first 80 again from the slot cache -- and every rank must see
    the same ready sequence, each collective exactly once per enqueue, then stop together."""
    _, outs = run_scenario(tmp_path, "engine_slots", np_=np_, timeout=240)
    ref = outs[0]
    assert sorted(ref["ready"]) == sorted(list(range(120)) + list(range(80))), ref
    for o in outs:
        assert o["ready"] == ref["ready"], "ranks derived different collective orders"
        assert o["slots"] == 120 and o["max_fresh"] > 64 and o["announces"] >= 2, o
        assert o["partial_seen"] > 0, o  # some slots were pending on part of the ranks only


def test_broadcast_optimizer_state(tmp_path):
    _, (a, b) = run_scenario(tmp_path, "optimizer_state")
    assert a == b and a["nstate"] > 0 and a["lr"] == pytest.approx(1e-3)


def test_metric_average(tmp_path):
    _, (a, b) = run_scenario(tmp_path, "metric_average")
    assert a["loss"] == b["loss"] == 0.5 and a["accuracy"] == 1.0 and a["name"] == "x"


def test_stall_inspector_aborts_job(tmp_path):
    env = {"MIHVD_STALL_CHECK_TIME_SECONDS": "1", "MIHVD_STALL_SHUTDOWN_TIME_SECONDS": "3"}
    p, outs = run_scenario(tmp_path, "stall", env=env, expect_ok=False, timeout=120)
    assert p.returncode != 0
    assert "stall inspector" in p.stderr
    assert outs[0] is None


def test_fault_kill_tears_down_job(tmp_path):
    p, outs = run_scenario(tmp_path, "fault", env={"MIHVD_FAULT": "kill:rank=1:step=3:code=7"}, expect_ok=False)
    assert p.returncode == 7
    assert "rank 1 exited with code 7" in p.stderr
    assert outs == [None, None]


def test_collective_async_error_aborts_every_rank(tmp_path):
    """An asynchronous communicator error on rank 1 (injected into the native health monitor, as
    RCCL's ncclCommGetAsyncError would report it) makes that rank abort its communicator and exit
    134; the launcher then tears down rank 0, which is blocked in the next collective (mpirun
    semantics, tensorflow-mnist.yaml:17-38). Both exit promptly, not at the collective timeout."""
    import time

    t0 = time.time()
    p, outs = run_scenario(tmp_path, "fault", env={"MIHVD_FAULT": "collerr:rank=1:step=3",
                                                   "MIHVD_HEALTH_POLL_S": "0.2"}, expect_ok=False, timeout=120)
    el = time.time() - t0
    assert p.returncode == 134, p.stderr[-2000:]
    assert "mihvd health: collective error 6" in p.stderr
    assert "rank 1 exited with code 134" in p.stderr
    assert outs == [None, None]
    assert el < 60, el


def test_health_monitor_watches_error_words():
    """The xGMI plane mirrors a phase-barrier timeout into a host-coherent word that the native
    health monitor polls (csrc/runtime/health.cc watch_word): zero is healthy, any nonzero value is
    a collective failure reported like RCCL's remote error (6), naming the word's label; an
    unwatched word is ignored (here the word is host memory written by the test instead of a kernel)."""
    import numpy as np

    from mihvd._native import runtime

    mon = runtime().HealthMonitor(0, 0.05, 134)
    mon.set_abort_process(False)
    word = np.zeros(16, dtype=np.uint32)
    addr = word.ctypes.data
    mon.watch_word(addr, "xGMI phase barrier (test)")
    mon.watch_word(addr, "again")  # idempotent
    assert mon.num_words == 1
    assert mon.poll_once() == (0, "")
    word[0] = 0x80000002
    code, what = mon.poll_once()
    assert code == 6 and "xGMI phase barrier (test)" in what and "0x80000002" in what
    mon.unwatch_word(addr)
    assert mon.num_words == 0 and mon.poll_once() == (0, "")
    # the background thread reports it too (report-only mode: no exit)
    mon.watch_word(addr, "bg")
    mon.start()
    import time

    t0 = time.time()
    while mon.error == 0 and time.time() - t0 < 10:
        time.sleep(0.02)
    mon.stop()
    mon.unwatch_word(addr)
    assert mon.error == 6


NEG = {"MIHVD_NEGOTIATE": "1"}


@pytest.mark.parametrize("np_", [2, 3])
def test_negotiated_collectives_any_order(tmp_path, np_):
    """Native negotiation engine (csrc/runtime/negotiator.cc) over mihvdrun's C++ store: ranks
    enqueue named collectives in different orders and still all agree; compatible allreduces are
    fused within a coordinator record."""
    _, outs = run_scenario(tmp_path, "negotiated_order", np_=np_, env=NEG)
    for o in outs:
        assert o["ok"], o
        assert o["bc"] == [float(np_ - 1)] * 5
        assert o["ag"] == [[float(q)] * 2 for q in range(np_) for _ in range(q + 1)]
        assert o["submitted"] == 14
    assert len({o["launches"] for o in outs}) == 1  # identical launch sequence on every rank
    assert len({o["fused"] for o in outs}) == 1


def test_negotiation_stall_report_names_missing_rank(tmp_path):
    env = dict(NEG, MIHVD_STALL_CHECK_TIME_SECONDS="1")
    p, (a, b) = run_scenario(tmp_path, "negotiated_stall", env=env)
    assert a["value"] == [3.0, 3.0] == b["value"]
    assert "collective 'allreduce.late' (generation 0) was submitted by ranks [0] but not by ranks [1]" in p.stderr
    assert a["warnings"] >= 1


def test_negotiation_rejects_mismatched_shapes(tmp_path):
    _, (a, b) = run_scenario(tmp_path, "negotiated_mismatch", env=NEG)
    for o in (a, b):
        assert o["error"] and "mismatched collective 'allreduce.shape_mismatch'" in o["error"]
        assert o["after"] == [2.0] * 3


def test_negotiated_fusion_buffer_is_persistent(tmp_path):
    """The negotiated path fuses ready allreduces into one persistent buffer: no allocation per step."""
    _, outs = run_scenario(tmp_path, "negotiated_fusion", env=NEG)
    for o in outs:
        assert o["ok"], o
        assert o["fused"] > 0, o
        # grown only when a fused group outgrows the buffer (readiness timing decides the groups);
        # geometric growth from a 64 K-element floor: these groups (at most 33 elements) fit the
        # first allocation, so once in total, never once per step
        al = o["allocs"]
        assert all(x <= y for x, y in zip(al, al[1:])) and al[-1] == 1, o
        # response cache: after the first step the same 6 names are posted as cached slots, several
        # per bit-vector record
        assert o["cache_hits"] >= o["submitted"] - 2 * 6, o
        assert o["records"] < o["submitted"], o


def test_dp_equivalence_negotiated(tmp_path):
    """DistributedOptimizer bucket allreduces through the negotiation engine."""
    _, outs = run_scenario(tmp_path, "dp_equivalence", env=NEG)
    for o in outs:
        assert o["maxdiff_0"] < 1e-5 and o["maxdiff_67108864"] < 1e-5


def test_torch_store_fallback(tmp_path):
    """MIHVD_STORE=torch: the launcher does not start its store; init uses torch's TCPStore."""
    _, (a, b) = run_scenario(tmp_path, "collectives", env={"MIHVD_STORE": "torch"})
    assert a["sum"] == b["sum"]


def test_collective_custom_ops_autograd(tmp_path):
    """torch.ops.mihvd_dist: allreduce grad = allreduce(grad); allgather grad = this rank's slice of
    the summed grad; broadcast grad = sum on the root, zero elsewhere (Horovod's rules)."""
    _, (a, b) = run_scenario(tmp_path, "torch_ops")
    assert a["y"] == [3.0] * 3                      # mean of 2*1 and 2*2
    assert a["wgrad"] == b["wgrad"] == [2.0] * 3    # d/dw sum(avg(2w)) over both ranks' losses
    assert a["g"] == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]]
    # loss_r = sum_i i * g_i on both ranks -> d/dx = 2 * i for this rank's rows
    assert a["xgrad"] == [[0.0, 0.0]] and b["xgrad"] == [[2.0, 2.0], [4.0, 4.0]]
    assert a["bb"] == b["bb"] == [0.0, 0.0]
    assert a["bgrad"] == [3.0, 3.0] and b["bgrad"] == [0.0, 0.0]
    assert a["t"] == [3.0] * 4


def test_collectives_debug_sync_mode(tmp_path):
    """MIHVD_DEBUG_SYNC=1: every collective completes inside the call (bisection mode)."""
    _, (a, b) = run_scenario(tmp_path, "collectives", env={"MIHVD_DEBUG_SYNC": "1"})
    assert a["sum"] == b["sum"] and a["async"] == [1.0] * 4


def test_process_sets_three_ranks(tmp_path):
    _, (a, b, c) = run_scenario(tmp_path, "process_sets", np_=3)
    assert a["ids"] == {"0": [0, 1, 2], "1": [1, 2], "2": [0, 2]}
    assert (a["included"], b["included"], c["included"]) == (True, False, True)
    assert (a["set_rank"], c["set_rank"], a["set_size"]) == (0, 1, 2)
    assert a["avg"] == c["avg"] == [1.0] * 3               # mean of ranks 0 and 2
    assert a["bcast"] == c["bcast"] == [2.0, 2.0]
    assert a["gather"] == [[0.0, 0.0], [2.0, 2.0]]
    assert a["alltoall"] == [0.0, 1.0, 20.0, 21.0] and c["alltoall"] == [2.0, 3.0, 22.0, 23.0]
    assert "not part of" in b["error"]
    assert b["sum2"] == c["sum2"] == [5.0, 5.0] and "sum2" not in a
    assert a["world"] == b["world"] == [3.0]


def test_collective_bandwidth_benchmark_two_ranks(tmp_path):
    """scripts/allreduce_bw.py under torch.distributed.run (gloo, 2 ranks): one JSON row per op and
    size from rank 0, bus bandwidth = algbw x the nccl-tests factor, unsupported ops reported."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, MIHVD_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29641", os.path.join(root, "scripts", "allreduce_bw.py"), "--sizes", "4K,64K",
           "--iters", "3", "--warmup", "1", "--engine"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=tmp_path)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    timed = [r for r in rows if "us" in r]
    assert {r["op"] for r in timed} >= {"allreduce", "hvd.allreduce", "allgather", "broadcast"}
    for r in timed:
        assert r["world"] == 2 and r["us"] > 0
        f = {"allreduce": 1.0, "hvd.allreduce": 1.0, "allgather": 0.5, "broadcast": 1.0}.get(r["op"])
        if f is not None:
            assert abs(r["busbw_GBs"] - f * r["algbw_GBs"]) < 1e-9 * max(1.0, r["algbw_GBs"])


def test_api_extras_two_ranks(tmp_path):
    """Grouped / async / in-place / sparse collectives and PartialDistributedOptimizer."""
    _, (a, b) = run_scenario(tmp_path, "api_extras")
    assert a["grouped_async"] == b["grouped_async"] == [[3.0] * 3, [[1.0, 1.0], [1.0, 1.0]], [0.0, 3.0, 6.0, 9.0]]
    assert a["grouped_unchanged"] == [1.0] * 3                      # the non-in-place form leaves inputs alone
    assert a["grouped_inplace"] == b["grouped_inplace"] == [[1.5] * 3, [[0.5, 0.5], [0.5, 0.5]], [0.0, 1.5, 3.0, 4.5]]
    assert a["alltoall_async"] == [0.0, 1.0, 100.0, 101.0] and b["alltoall_async"] == [2.0, 3.0, 102.0, 103.0]
    assert a["alltoall_splits"] == [2, 2]
    assert a["reducescatter_async"] == b["reducescatter_async"] == [[3.0] * 3] * 2
    assert a["grouped_reducescatter"] == b["grouped_reducescatter"] == [[[1.5, 1.5]], [0.5] * 3]
    assert a["grouped_reducescatter_async"] == [[3.0]]
    assert a["grouped_allgather"] == b["grouped_allgather"] == [[[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]], [0, 0, 1]]
    assert a["grouped_allgather_sync"] == [[0.0, 1.0]]
    assert a["built"] == [False, False, False]
    assert a["sparse_sum"] == b["sparse_sum"] == [[2.0, 1.0], [0.0, 2.0], [0.0, 0.0]]
    assert a["sparse_avg"] == [[1.0, 0.5], [0.0, 1.0], [0.0, 0.0]]
    for r in (a, b):
        assert r["reduced_params"] == 2                              # body weight + bias only
        assert r["head_grad"] == pytest.approx(r["head_ref"])        # local: this rank's own gradient
        assert r["body_grad"] == pytest.approx(r["body_ref"], rel=1e-5)
    assert a["head_grad"] != b["head_grad"]


def test_api_extras_debug_sync_mode(tmp_path):
    """Composite handles (grouped / sparse) stay pollable when every collective completes eagerly."""
    _, (a, b) = run_scenario(tmp_path, "api_extras", env={"MIHVD_DEBUG_SYNC": "1"})
    assert a["grouped_async"] == b["grouped_async"] and a["sparse_sum"] == [[2.0, 1.0], [0.0, 2.0], [0.0, 0.0]]


def test_keras_and_tf_module_functions_two_ranks(tmp_path):
    """hvd.allreduce / allgather / broadcast / broadcast_global_variables / load_model of the Keras
    API and broadcast_variables of the TF1 API over two gloo ranks."""
    _, (a, b) = run_scenario(tmp_path, "keras_tf_api")
    for r in (a, b):
        assert r["allreduce_scalar"] == 1.5 and r["allreduce_sum"] == [1.0, 1.0]
        assert r["allgather"] == [[0, 0], [1, 1]] and r["broadcast"] == [10, 11, 12]
        assert r["tf_bcast"] == [[1.0, 1.0], [1.0], [0.0, 0.0]]
        assert r["loaded"] == a["weights"] and r["loaded_dp"] is True
    assert a["weights"] == b["weights"] and a["exp_avg"] == b["exp_avg"]

