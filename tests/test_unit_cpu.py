"""CPU unit tests: native runtime (planner, controller, timeline, stall inspector, faults), env
discovery, launcher argv compatibility, checkpoint layout, TF1-session and Keras-fit plumbing."""
import json
import os
import sys
import time

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from mihvd import _native
from mihvd.runner import launch as L
from mihvd.utils import checkpoint as ckpt
from mihvd.utils import env as envmod

rt = _native.runtime()

REFERENCE_ARGV = ("-np 2 --allow-run-as-root -bind-to none -map-by slot -x LD_LIBRARY_PATH -x PATH "
                  "-mca pml ob1 -mca btl ^openib python /examples/tensorflow_mnist.py").split()


# ------------------------------------------------------------------------------ planner
@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(1, 5000), st.integers(0, 1)), min_size=1, max_size=30),
       st.integers(0, 40000), st.sampled_from([4, 16, 256]))
def test_plan_buckets_properties(raw, threshold, align):
    tensors = [(n, 4 if dt == 0 else 2, dt) for n, dt in raw]  # dtype code fixes the element size
    specs = [rt.TensorSpec(n, es, dt, 0) for n, es, dt in tensors]
    order = list(range(len(specs)))[::-1]
    plan = rt.plan_buckets(specs, order, threshold, align)
    seen = set()
    for b, (mem, offs) in enumerate(zip(plan.members, plan.offsets)):
        dts = {tensors[i][2] for i in mem}
        assert len(dts) == 1  # never mixes dtypes
        esz = tensors[mem[0]][1]
        ends = []
        for i, o in zip(mem, offs):
            assert (o * esz) % align == 0
            assert o >= (ends[-1] if ends else 0)  # no overlap, pack order preserved
            ends.append(o + tensors[i][0])
            seen.add(i)
            assert plan.tensor_bucket[i] == b and plan.tensor_offset[i] == o
        assert plan.numel[b] >= ends[-1]
        if threshold > 0 and len(mem) > 1:
            assert ends[-1] * esz <= threshold
    assert seen == set(range(len(specs)))
    # deterministic
    plan2 = rt.plan_buckets(specs, order, threshold, align)
    assert list(plan2.members) == list(plan.members)


def test_controller_releases_buckets_in_order():
    c = rt.Controller([0, 0, 1, 2], 3, 1)
    assert c.mark_ready(2) == []          # bucket 1 complete but bucket 0 not launched yet
    assert c.mark_ready(0) == []
    assert c.mark_ready(1) == [0, 1]      # releases 0 then the already-complete 1
    assert c.mark_ready(3) == [2]
    with pytest.raises(RuntimeError):
        c.mark_ready(3)
    c.reset()
    assert c.flush() == [0, 1, 2]


def test_controller_backward_passes():
    c = rt.Controller([0, 0], 1, 2)
    assert c.mark_ready(0) == [] and c.mark_ready(1) == []
    assert c.mark_ready(0) == [] and c.mark_ready(1) == [0]


def test_signature_sensitivity():
    s1 = rt.tensor_signature(["a", "b"], [[2, 3], [4]], ["float32", "float32"])
    assert s1 == rt.tensor_signature(["a", "b"], [[2, 3], [4]], ["float32", "float32"])
    assert s1 != rt.tensor_signature(["a", "b"], [[3, 2], [4]], ["float32", "float32"])
    assert s1 != rt.tensor_signature(["a", "c"], [[2, 3], [4]], ["float32", "float32"])


# ------------------------------------------------------------------------------ timeline / stall / faults
def test_timeline_writes_valid_chrome_trace(tmp_path):
    p = tmp_path / "tl.json"
    tl = rt.Timeline(str(p), 3)
    tl.begin("allreduce.bucket0", "ALLREDUCE", 1)
    tl.end("allreduce.bucket0", "ALLREDUCE", 1)
    tl.complete("fc1_fwd", "COMPUTE", 0, 10.0, 5.5)
    tl.instant("step", "STEP", 0)
    tl.counter("loss", 0.25)
    tl.close()
    ev = json.loads(p.read_text())
    names = [e["name"] for e in ev]
    assert "process_name" in names and "allreduce.bucket0" in names and "loss" in names
    assert all(e["pid"] == 3 for e in ev)
    x = [e for e in ev if e["ph"] == "X"][0]
    assert x["dur"] == pytest.approx(5.5)


def test_stall_inspector_reports_old_ops():
    si = rt.StallInspector(0.2, 0.0, 0.05, 0)
    si.set_hard_abort(False)
    si.start()
    a = si.submit("allreduce.bucket0")
    b = si.submit("allreduce.bucket1")
    si.complete(b)
    time.sleep(0.5)
    out = si.outstanding(0.1)
    assert [r.name for r in out] == ["allreduce.bucket0"]
    assert si.stalled and si.warnings_emitted == 1
    si.complete(a)
    assert si.num_outstanding() == 0
    si.stop()


def test_fault_plan_parsing():
    fp = rt.FaultPlan("kill:rank=1:step=50:code=3;delay:step=2:ms=10")
    assert [a.kind for a in fp.due(1, 50)] == ["kill"]
    assert fp.due(1, 50)[0].args["code"] == "3"
    assert [a.kind for a in fp.due(0, 2)] == ["delay"]
    assert fp.due(0, 3) == []
    with pytest.raises(Exception):
        rt.FaultPlan("explode:rank=0")


def test_step_stats():
    s = rt.StepStats(4)
    for v in (1, 2, 3, 4, 100):
        s.add(v)
    assert s.count == 5 and s.mean() == pytest.approx((2 + 3 + 4 + 100) / 4)
    assert s.percentile(50) == pytest.approx(3.5)


# ------------------------------------------------------------------------------ env / launcher
def test_env_discovery_sources():
    t = envmod.discover({"OMPI_COMM_WORLD_RANK": "3", "OMPI_COMM_WORLD_SIZE": "8", "OMPI_COMM_WORLD_LOCAL_RANK": "1",
                         "OMPI_COMM_WORLD_LOCAL_SIZE": "2"})
    assert (t.rank, t.size, t.local_rank, t.local_size, t.cross_rank, t.cross_size, t.source) == (3, 8, 1, 2, 1, 4, "ompi")
    t = envmod.discover({"RANK": "1", "WORLD_SIZE": "2", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "2",
                         "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "1234"})
    assert (t.rank, t.master_addr, t.master_port, t.source) == (1, "10.0.0.1", 1234, "native")
    t = envmod.discover({"PMI_RANK": "2", "PMI_SIZE": "4"})
    assert (t.rank, t.size, t.source) == (2, 4, "pmi")
    assert envmod.discover({}).source == "single"
    with pytest.raises(ValueError):
        envmod.discover({"RANK": "5", "WORLD_SIZE": "2"})


def test_launcher_accepts_reference_mpirun_argv():
    spec = L.parse_args(REFERENCE_ARGV)
    assert spec.np == 2 and spec.map_by == "slot"
    assert spec.command == ["python", "/examples/tensorflow_mnist.py"]
    assert set(spec.env_forward) == {"LD_LIBRARY_PATH", "PATH"}
    assert ("pml", "ob1") in spec.mca and ("btl", "^openib") in spec.mca
    assert "--allow-run-as-root" in spec.ignored


def test_launcher_hosts_and_layout(tmp_path):
    spec = L.parse_args(["-np", "4", "-H", "a:2,b:2", "python", "x.py"])
    lay = L.assign_ranks(spec.hosts, spec.np, "slot")
    assert [(r, h, lr, ls, n) for r, h, lr, ls, n in lay] == [(0, "a", 0, 2, 0), (1, "a", 1, 2, 0), (2, "b", 0, 2, 1),
                                                              (3, "b", 1, 2, 1)]
    lay = L.assign_ranks(spec.hosts, spec.np, "node")
    assert [(r, h) for r, h, *_ in lay] == [(0, "a"), (1, "b"), (2, "a"), (3, "b")]
    hf = tmp_path / "hostfile"
    hf.write_text("worker-0.svc slots=8\nworker-1.svc slots=8\n# comment\n")
    spec = L.parse_args(["--hostfile", str(hf), "python", "t.py"])
    assert spec.hosts == [("worker-0.svc", 8), ("worker-1.svc", 8)] and spec.np == 16
    with pytest.raises(SystemExit):
        L.assign_ranks([("a", 1)], 2)


def test_launcher_rank_env():
    spec = L.parse_args(["-np", "2", "-x", "FOO=bar", "-x", "HOME", "--fusion-threshold-mb", "16", "python", "t.py"])
    e = L.build_rank_env(spec, 1, 1, 2, 0, "127.0.0.1", 29501, base_env={"HOME": "/h"})
    assert e["RANK"] == "1" and e["OMPI_COMM_WORLD_LOCAL_RANK"] == "1" and e["MASTER_PORT"] == "29501"
    assert e["FOO"] == "bar" and e["HOME"] == "/h" and e["MIHVD_FUSION_THRESHOLD"] == str(16 * 1024 * 1024)


def test_launcher_horovodrun_knobs(tmp_path):
    """horovodrun's tuning/diagnostic flags map onto the engine's MIHVD_* knobs; --output-filename
    writes every rank's output under <dir>/1/rank.<r>/ (Open MPI's layout); --check-build lists
    what this installation runs."""
    spec = L.parse_args(["-np", "1", "--autotune", "--autotune-log-file", "at.csv", "--log-level", "debug",
                         "--output-filename", str(tmp_path / "logs"), "--network-interface", "eth0", "--disable-cache",
                         sys.executable, "-c", "import os,sys; print('hello', os.environ['MIHVD_LOG_LEVEL']); "
                         "print('err', file=sys.stderr)"])
    assert spec.extra_env == {"MIHVD_AUTOTUNE": "1", "MIHVD_AUTOTUNE_LOG": "at.csv", "MIHVD_LOG_LEVEL": "DEBUG"}
    assert "--disable-cache" in spec.ignored and "--network-interface eth0" in spec.ignored
    assert L.launch(spec) == 0
    assert (tmp_path / "logs" / "1" / "rank.0" / "stdout").read_text() == "hello DEBUG\n"
    assert (tmp_path / "logs" / "1" / "rank.0" / "stderr").read_text() == "err\n"
    text = L.check_build()
    assert "[X] PyTorch" in text and "Available Tensor Operations:" in text and "RCCL" in text


def test_autotuner_writes_log_file(monkeypatch, hvd_single, tmp_path):
    from mihvd.parallel.autotune import FusionAutotuner

    log = tmp_path / "autotune.csv"
    tu = FusionAutotuner(["1", "2"], warmup_steps=0, trial_steps=1, log_file=str(log))
    clock = [0.0]
    monkeypatch.setattr(tu, "_now", lambda: clock[0])
    cur = tu.first()
    for _ in range(20):
        clock[0] += 1.0 if cur == 2 ** 21 else 2.0
        new = tu.on_step()
        if new is not None:
            cur = new
            if tu.done:
                break
    rows = log.read_text().splitlines()
    assert rows[0] == "fusion_threshold_bytes,median_step_ms,trial_steps,chosen" and len(rows) == 3
    assert rows[2].startswith(str(2 ** 21)) and rows[2].endswith(",1")


# ------------------------------------------------------------------------------ checkpoints
def test_checkpoint_layout_and_rotation(tmp_path):
    s = ckpt.Saver(max_to_keep=3)
    for step in (10, 20, 30, 40):
        s.save(str(tmp_path), {"w": torch.full((2,), float(step)), "global_step": torch.tensor(step)}, step)
    latest, allp = ckpt.read_index(str(tmp_path))
    assert latest == "model.ckpt-40" and allp == ["model.ckpt-20", "model.ckpt-30", "model.ckpt-40"]
    assert sorted(os.listdir(tmp_path)) == ["checkpoint", "model.ckpt-20.pt", "model.ckpt-30.pt", "model.ckpt-40.pt"]
    v = ckpt.Saver.restore(ckpt.latest_checkpoint(str(tmp_path)))
    assert float(v["w"][0]) == 40.0 and int(v["global_step"]) == 40


def test_tf_variable_mapping_roundtrip():
    from mihvd.models.mnist import NUM_PARAMS, MNISTConvNet
    from mihvd.optim import TFAdam

    m = MNISTConvNet(seed=0)
    assert sum(p.numel() for p in m.parameters()) == NUM_PARAMS == 3274634
    opt = TFAdam(m.parameters(), lr=1e-3)
    m(torch.rand(2, 784)).sum().backward()
    opt.step()
    v = ckpt.adam_to_tf_vars(m.ordered_parameters(), opt, 7)
    assert v["dense/kernel"].shape == (3136, 1024) and "dense/kernel/Adam_1" in v
    assert int(v["global_step"]) == 7 and float(v["beta1_power"]) == pytest.approx(0.9 ** 2)
    m2 = MNISTConvNet(seed=1)
    opt2 = TFAdam(m2.parameters(), lr=1e-3)
    step = ckpt.tf_vars_to_adam(v, m2.ordered_parameters(), opt2)
    assert step == 7
    for (n, a), (_, b) in zip(m.ordered_parameters(), m2.ordered_parameters()):
        assert torch.equal(a, b)
    assert float(opt2.state[m2.dense.kernel]["step"]) == 1.0


def test_tfadam_matches_tf1_formula():
    from mihvd.optim import TFAdam

    p = torch.nn.Parameter(torch.tensor([1.0, -2.0]))
    opt = TFAdam([p], lr=0.1)
    g = torch.tensor([0.5, -1.0])
    m = v = torch.zeros(2)
    ref = p.detach().clone()
    for t in (1, 2):
        p.grad = g.clone()
        opt.step()
        m = 0.9 * m + 0.1 * g
        v = 0.999 * v + 0.001 * g * g
        lr_t = 0.1 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        ref = ref - lr_t * m / (v.sqrt() + 1e-8)
    assert torch.allclose(p.detach(), ref, atol=1e-6)


# ------------------------------------------------------------------------------ session / keras (single process)
def test_monitored_session_single_rank(tmp_path, hvd_single):
    import mihvd.tensorflow as htf
    from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy
    from mihvd.optim import TFAdam

    model = MNISTConvNet(seed=0)
    opt = hvd_single.DistributedOptimizer(TFAdam(model.parameters(), lr=1e-3), named_parameters=model.named_parameters())
    state = htf.TorchTrainState(model, opt)
    log = htf.LoggingTensorHook({"step": "global_step", "loss": "loss"}, every_n_iter=2)

    def train_op(image, label):
        opt.zero_grad()
        loss = softmax_cross_entropy(model(image), label)
        loss.backward()
        opt.step()
        return {"loss": loss.detach()}

    hooks = [htf.BroadcastGlobalVariablesHook(0), htf.StopAtStepHook(last_step=5), log]
    with htf.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=hooks, state=state) as s:
        while not s.should_stop():
            s.run(train_op, feed_dict={"image": torch.rand(4, 784), "label": torch.randint(0, 10, (4,))})
    assert state.global_step == 5 and len(log.lines) == 3
    assert ckpt.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-5")
    # restart resumes at 5 and stops immediately
    state2 = htf.TorchTrainState(MNISTConvNet(seed=9), None)
    with htf.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=[htf.StopAtStepHook(last_step=5)],
                                      state=state2) as s:
        assert s.should_stop() and s.restored_from is not None
    assert state2.global_step == 5
    assert torch.equal(state2.model.dense.kernel, model.dense.kernel)


def test_session_multi_step_runs_keep_step_cadence(tmp_path, hvd_single):
    """A run that advances several steps (the fused trainer's graph replay) keeps the hooks'
    step-based semantics: LoggingTensorHook logs once per 10 steps, StopAtStepHook stops exactly at
    the last step, step-triggered checkpoints land on the run boundaries that cross them."""
    import mihvd.tensorflow as htf

    class State:
        def __init__(self):
            self.global_step = 0
            self.w = torch.zeros(3)

        def variables(self):
            return {"w": self.w.clone(), "global_step": torch.tensor(self.global_step)}

        def load_variables(self, v):
            self.w.copy_(v["w"])
            self.global_step = int(v["global_step"])

        def broadcast(self, root):
            pass

    st = State()
    last = 47
    log = htf.LoggingTensorHook({"step": "global_step", "loss": "loss"}, every_n_iter=10)

    def train_op():
        k = min(10, last - st.global_step)  # graph-replayed run of up to 10 steps
        st.global_step += k
        st.w += k
        return {"loss": torch.tensor(1.0 / st.global_step)}

    hooks = [htf.BroadcastGlobalVariablesHook(0), htf.StopAtStepHook(last_step=last), log]
    with htf.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=hooks, state=st,
                                      save_checkpoint_steps=20) as s:
        while not s.should_stop():
            s.run(train_op)
    assert st.global_step == last
    steps = [int(line.split("step=")[1].split()[0]) for line in log.lines]
    assert steps == [10, 20, 30, 40, 47], log.lines  # one line per 10 steps (iterations 0, 10, 20, ...)
    saved = sorted(f for f in os.listdir(tmp_path) if f.endswith(".pt"))
    assert saved == ["model.ckpt-20.pt", "model.ckpt-40.pt", "model.ckpt-47.pt"], saved


def test_keras_fit_single_rank(tmp_path, hvd_single):
    import mihvd.keras as hk
    from mihvd.models.mnist import MNISTConvNet
    from mihvd.optim import TFAdam
    from mihvd.utils.data import synthetic_mnist

    (x, y), (xt, yt) = synthetic_mnist(n_train=600, n_test=200, seed=3)
    x = x.reshape(-1, 784).astype(np.float32) / 255
    xt = xt.reshape(-1, 784).astype(np.float32) / 255
    model = hk.Model(MNISTConvNet(seed=0))
    opt = hk.DistributedOptimizer(TFAdam(model.module.parameters(), lr=1e-3), named_parameters=model.module.named_parameters())
    model.compile(opt, torch.nn.functional.cross_entropy, ["accuracy"])
    cbs = [hk.callbacks.BroadcastGlobalVariablesCallback(0), hk.callbacks.MetricAverageCallback(),
           hk.callbacks.TensorBoard(str(tmp_path / "logs")),
           hk.callbacks.ModelCheckpoint(str(tmp_path / "ckpt" / "mnist-{epoch}.h5"), save_best_only=True)]
    model.fit(x, y, batch_size=50, epochs=2, steps_per_epoch=6, validation_data=(xt, yt), validation_steps=2,
              callbacks=cbs, verbose=0)
    assert cbs[0].broadcast_done and len(model.history["loss"]) == 2
    assert os.path.exists(tmp_path / "ckpt" / "mnist-1.h5")
    assert (tmp_path / "logs" / "metrics.jsonl").exists()
    path = model.save(str(tmp_path / "final_model"))
    assert path.endswith("model.pt")
    m2 = hk.Model.load_weights(MNISTConvNet(seed=5), str(tmp_path / "final_model"))
    assert torch.equal(m2.dense.bias, model.module.dense.bias)


def test_lr_scaler_rule(hvd_single):
    # tensorflow_mnist.py:123-127
    hvd = hvd_single
    scaler = hvd.size()
    assert scaler == 1
    adasum_scaler = hvd.local_size() if hvd.nccl_built() else 1
    assert adasum_scaler == 1


def test_synthetic_data_and_generator():
    from mihvd.utils.data import synthetic_mnist, train_input_generator

    (x, y), (xt, yt) = synthetic_mnist(n_train=1000, n_test=100)
    assert x.shape == (1000, 28, 28) and x.dtype == np.uint8 and set(np.unique(y)) <= set(range(10))
    gen = train_input_generator(x.reshape(-1, 784), y, batch_size=300, rng=np.random.default_rng(0))
    batches = [next(gen) for _ in range(4)]
    assert all(b[0].shape == (300, 784) for b in batches)  # tail of 100 dropped each pass


def test_adasum_covering_offsets():
    from mihvd.parallel.adasum import _covering_offsets

    assert _covering_offsets([(0, 5), (8, 10)], 12) == ([0, 5, 8, 10, 12], [0, 1, 0, 1])
    assert _covering_offsets([(0, 12)], 12) == ([0, 12], [0])
    assert _covering_offsets([(2, 4)], 4) == ([0, 2, 4], [1, 0])


def test_autotuner_picks_fastest(monkeypatch, hvd_single):
    from mihvd.parallel.autotune import FusionAutotuner

    tu = FusionAutotuner(["1", "4", "16"], warmup_steps=1, trial_steps=2)
    cost = {1: 3.0, 4: 1.0, 16: 2.0}
    clock = [0.0]
    cur = [tu.first()]
    monkeypatch.setattr(tu, "_now", lambda: clock[0])
    decided = None
    for _ in range(40):
        clock[0] += cost[cur[0] // 2 ** 20]
        new = tu.on_step()
        if new is not None:
            cur[0] = new
            if tu.done:
                decided = new
                break
    assert tu.done and decided == 4 * 2 ** 20


def test_trace_range_noop_without_roctx():
    from mihvd.utils.tracing import trace_range

    with trace_range("x"):
        pass


# ---------------------------------------------------------------------------------------------
# control plane: C++ key-value store + negotiation engine (csrc/runtime/store.cc, negotiator.cc)
# ---------------------------------------------------------------------------------------------
def test_native_store_semantics():
    import threading
    import time

    from mihvd._native import runtime

    rt = runtime()
    srv = rt.StoreServer("127.0.0.1", 0)
    try:
        c = rt.StoreClient("127.0.0.1", srv.port)
        c.set("bin", b"a\x00b")
        assert c.get("bin") == b"a\x00b"
        assert c.add("ctr", 5) == 5 and c.add("ctr", -7) == -2
        assert c.try_get("nope", 0.05) is None
        with pytest.raises(RuntimeError, match="timeout"):
            c.get("nope", 0.05)
        # a blocking get is parked on the server until another client sets the key
        t0 = time.time()
        threading.Timer(0.2, lambda: rt.StoreClient("127.0.0.1", srv.port).set("late", b"v")).start()
        assert c.get("late", 5.0) == b"v" and time.time() - t0 >= 0.15
        # torch.distributed compare_set semantics
        assert c.compare_set("cs", "", "x") == b"x"
        assert c.compare_set("cs", "wrong", "y") == b"x"
        assert c.compare_set("cs", "x", "y") == b"y"
        assert c.check(["bin", "ctr"]) and not c.check(["bin", "zz"])
        assert not c.wait(["zz"], 0.05)
        c.append("ap", b"12")
        c.append("ap", b"34")
        assert c.get("ap") == b"1234"
        assert c.delete("bin") and not c.delete("bin")
        assert c.num_keys() == srv.num_keys() == 4  # ctr, late, cs, ap
        # a corrupt frame (length past the limit) drops that connection, not the server
        import socket
        import struct

        raw = socket.create_connection(("127.0.0.1", srv.port))
        raw.sendall(struct.pack("<I", 0xFFFFFFF0) + b"\x01")
        raw.settimeout(5.0)
        assert raw.recv(16) == b""  # closed by the server
        raw.close()
        assert c.get("ap") == b"1234"
    finally:
        srv.stop()


def test_native_store_backs_torch_process_group():
    import datetime

    import torch
    import torch.distributed as dist

    from mihvd.runner.store import NativeStore, start_server

    srv = start_server("127.0.0.1", 0)
    try:
        st = NativeStore("127.0.0.1", srv.port, datetime.timedelta(seconds=30))
        dist.init_process_group("gloo", store=dist.PrefixStore("t", st), rank=0, world_size=1)
        try:
            t = torch.ones(3)
            dist.all_reduce(t)
            assert t.tolist() == [1.0] * 3
        finally:
            dist.destroy_process_group()
    finally:
        srv.stop()


def test_negotiator_orders_and_validates():
    import random
    import time

    from mihvd._native import runtime

    rt = runtime()
    srv = rt.StoreServer("127.0.0.1", 0)
    W = 3
    negs = [rt.Negotiator("127.0.0.1", srv.port, r, W, "u", 0.001, 0.3, 0.0) for r in range(W)]
    try:
        names = [f"n{i}" for i in range(25)]
        for r in range(W):
            order = names[:]
            random.Random(r).shuffle(order)
            for nm in order:
                negs[r].submit(nm, "sig")
            negs[r].submit("n0", "sig")  # generation 1 of a reused name
        got = [[] for _ in range(W)]
        deadline = time.time() + 20
        while any(len(g) < 26 for g in got) and time.time() < deadline:
            for r in range(W):
                got[r] += [(x.name, x.generation, x.batch) for x in negs[r].wait(0.05)]
        assert all(g == got[0] for g in got)            # same order AND same batches on all ranks
        assert sorted(n for n, gen, _ in got[0] if gen == 0) == sorted(names)
        assert [n for n, gen, _ in got[0] if gen == 1] == ["n0"]
        # stall view: only ranks 0 and 2 submit
        negs[0].submit("stuck", "s")
        negs[2].submit("stuck", "s")
        time.sleep(0.8)
        st = negs[0].stalled(0.0)
        assert [(e.name, e.ready_ranks, e.missing_ranks) for e in st] == [("stuck", [0, 2], [1])]
        assert negs[0].warnings >= 1
        negs[1].submit("stuck", "other")  # signature mismatch is reported on every rank
        errs = []
        while not errs and time.time() < deadline:
            errs = [x.error for x in negs[1].wait(0.1)]
        assert "mismatched collective 'stuck'" in errs[0]
    finally:
        for n in negs:
            n.stop()
        srv.stop()


def test_collective_custom_ops_trace_single_rank(hvd_single):
    """torch.ops.mihvd_dist ops run at world size 1 and trace through make_fx as single nodes."""
    import torch
    from torch.fx.experimental.proxy_tensor import make_fx

    from mihvd.ops import collective_ops  # noqa: F401

    ops = torch.ops.mihvd_dist
    x = torch.randn(4, 3, requires_grad=True)
    y = ops.allreduce(x, 0, "x")
    y.sum().backward()
    assert torch.equal(y, x) and torch.equal(x.grad, torch.ones(4, 3))
    gm = make_fx(lambda t: ops.allreduce(t * 2, 1, "t") + 1)(torch.randn(5))
    assert "mihvd_dist.allreduce" in gm.code
    assert ops.allgather(torch.ones(2, 2), "g").shape == (2, 2)


def test_monitored_session_counts_self_advancing_state_once(tmp_path, hvd_single):
    """A train state that advances its own global_step (FusedMNISTTrainer.train_step) is not
    advanced a second time by the session: StopAtStepHook(last_step=N) runs exactly N steps."""
    import mihvd.tensorflow as tfh

    class SelfCounting:
        def __init__(self):
            self.global_step = 0
            self.calls = 0

        def step(self):
            self.calls += 1
            self.global_step += 1
            return {"loss": 0.0}

    st = SelfCounting()
    with tfh.MonitoredTrainingSession(state=st, hooks=[tfh.StopAtStepHook(last_step=25)]) as sess:
        while not sess.should_stop():
            sess.run(st.step)
    assert st.calls == 25 and st.global_step == 25


def test_keras_lr_schedule_callback():
    import mihvd.keras as khvd

    class _Opt:
        param_groups = [{"lr": 0.0}]

    class _M:
        optimizer = _Opt()
        _steps_per_epoch = 10

    cb = khvd.callbacks.LearningRateScheduleCallback(0.1, lambda e: 0.5 ** e, start_epoch=1, end_epoch=3)
    cb.set_model(_M())
    lrs = []
    for epoch in range(4):
        cb.on_epoch_begin(epoch)
        lrs.append(_M.optimizer.param_groups[0]["lr"])
    assert lrs == [0.0, 0.05, 0.025, 0.025]  # inactive before 1 and from 3 on
    smooth = khvd.callbacks.LearningRateScheduleCallback(1.0, lambda e: e, staircase=False)
    smooth.set_model(_M())
    smooth.on_epoch_begin(2)
    smooth.on_batch_begin(5)
    assert _M.optimizer.param_groups[0]["lr"] == 2.5


def test_fused_optimizers_torch_path_match_torch_optim():
    """FusedAdam / FusedSGD on CPU tensors (torch fallback) follow torch.optim semantics."""
    import torch

    from mihvd.optim import FusedAdam, FusedSGD

    torch.manual_seed(0)
    cases = [
        (lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.1), lambda ps: torch.optim.Adam(ps, lr=1e-2, weight_decay=0.1)),
        (lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.1, adamw=True),
         lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.1)),
        (lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True),
         lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)),
        (lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9, dampening=0.1),
         lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, dampening=0.1)),
    ]
    for mk, mk_ref in cases:
        a = [torch.randn(7, 5, requires_grad=True), torch.randn(3, requires_grad=True)]
        b = [x.detach().clone().requires_grad_(True) for x in a]
        oa, ob = mk(a), mk_ref(b)
        for _ in range(4):
            for ps, o in ((a, oa), (b, ob)):
                o.zero_grad()
                (ps[0].sin().sum() + (ps[1] ** 2).sum()).backward()
                o.step()
        for x, y in zip(a, b):
            assert torch.allclose(x, y, atol=1e-6, rtol=1e-5)


def test_synthetic_shards_share_class_templates():
    """Data-parallel shards of the synthetic set (sample_seed = rank) share the class templates: the
    per-class mean images of two shards match; independently seeded sets (the old per-rank seed)
    do not."""
    import numpy as np

    from mihvd.utils.data import synthetic_mnist

    def class_means(x, y):
        return np.stack([x[y == c].astype(np.float64).mean(0) for c in range(10)])

    (a, ya), _ = synthetic_mnist(3000, 10, seed=1234, sample_seed=0)
    (b, yb), _ = synthetic_mnist(3000, 10, seed=1234, sample_seed=1)
    (c, yc), _ = synthetic_mnist(3000, 10, seed=1)
    assert not np.array_equal(a, b)
    ma, mb, mc = class_means(a, ya), class_means(b, yb), class_means(c, yc)
    same = np.corrcoef(ma.reshape(10, -1), mb.reshape(10, -1))[np.arange(10), 10 + np.arange(10)]
    other = np.corrcoef(ma.reshape(10, -1), mc.reshape(10, -1))[np.arange(10), 10 + np.arange(10)]
    assert same.min() > 0.95, same
    assert other.mean() < 0.5, other


def _engine_ctrl(world, counts, hashes_by_rank):
    """Summed control vector of the native engine (csrc/kernels/engine.cpp) for S slots."""
    S = len(counts)
    v = np.zeros(2 + 2 * S, dtype=np.int64)
    v[2:2 + S] = counts
    v[2 + S:] = np.sum(hashes_by_rank, axis=0)
    return ((v + 2 ** 31) % 2 ** 32 - 2 ** 31).astype(np.int32)  # int32 wrap-around, as RCCL's sum


def test_native_engine_plan_fusion_and_stalls():
    """The engine's planning step (the same C++ function the engine thread runs on the summed
    control vector): ready slots fused in slot order by (dtype, op) up to the threshold, tensors
    above the threshold alone, slots pending on some ranks reported, signature mismatch fatal."""
    if not _native.load_kernels():
        pytest.skip("kernel library not built")
    from mihvd.parallel.native_engine import plan, signature_hash

    world = 4
    h = [signature_hash(f"g{i}", 6, 100, 0) for i in range(7)]
    nbytes = [400, 400, 400, 5000, 400, 400, 400]
    keys = [1, 1, 1, 1, 1, 2, 1]
    counts = [4, 4, 0, 4, 4, 4, 2]
    per_rank = [[h[s] if (counts[s] == world or (counts[s] and r < counts[s])) else 0 for s in range(7)]
                for r in range(world)]
    groups, partial = plan(_engine_ctrl(world, counts, per_rank), world, h, nbytes, keys, threshold=1000)
    # slot 2 has nothing pending; slot 3 exceeds the threshold (alone); slot 5 differs in key; slot 6 is partial
    assert groups == [[0, 1], [3], [4], [5]], groups
    assert partial == [6]
    # a rank that put a different signature in a full slot: every rank detects it
    bad = [list(r) for r in per_rank]
    bad[2][1] = signature_hash("other", 6, 100, 0)
    with pytest.raises(RuntimeError, match="different collectives"):
        plan(_engine_ctrl(world, counts, bad), world, h, nbytes, keys, threshold=1000)
    # the fused groups never exceed the threshold
    many = [signature_hash(f"m{i}", 6, 64, 0) for i in range(10)]
    groups, _ = plan(_engine_ctrl(2, [2] * 10, [many, many]), 2, many, [300] * 10, [0] * 10, threshold=1000)
    assert groups == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9]]


def test_native_engine_slot_agreement_is_order_independent():
    """Slot numbering of the native engine (engine_new_slot_order, the function the engine thread
    runs on the all-gathered announce blocks): two ranks that first enqueue the same tensors in
    OPPOSITE orders, and in different cycles, derive the same slot table — so the summed control
    vector lines the same signature up on every rank (round 3's engine numbered slots in each rank's
    local first-enqueue order, which broke exactly this case)."""
    if not _native.load_kernels():
        pytest.skip("kernel library not built")
    from mihvd.parallel.native_engine import assign, signature_hash

    K = 64
    a, b, c, d = (signature_hash(n, 6, 100, 0) for n in ("A", "B", "C", "D"))

    def block(hashes):
        return list(hashes) + [0] * (K - len(hashes))

    # cycle 1: rank 0 announces A, B; rank 1 announces B, A (opposite order) and D
    g1 = block([a, b]) + block([b, a, d])
    slots0 = assign(g1, 2)   # what rank 0 appends
    slots1 = assign(g1, 2)   # what rank 1 appends (same gathered data)
    assert slots0 == slots1 == sorted({a, b, d})
    table = list(slots0)
    # cycle 2: rank 1 announces C; rank 0 (first use of D now, already assigned) announces nothing
    g2 = block([]) + block([c])
    new = assign(g2, 2, assigned=table)
    assert new == [c]
    table += new
    # every rank's slot of a signature is its index in the common table
    assert {h: i for i, h in enumerate(table)} == {a: table.index(a), b: table.index(b), c: 3, d: table.index(d)}
    # already-assigned hashes announced again (a rank that enqueued them late) add nothing
    assert assign(block([a, d]) + block([]), 2, assigned=table) == []


def test_native_engine_wrapper_routing():
    """mihvd.parallel.native_engine.NativeEngine's Python side (no GPU): allreduces on the world go
    to the engine op, sub-groups / unsupported ops / non-contiguous tensors are declined (the caller
    launches them on the process group), flush() waits every outstanding handle once."""
    import torch.distributed as dist

    from mihvd.parallel import native_engine as ne

    class Ops:
        def __init__(self):
            self.enq, self.waited, self.n = [], [], 0

        def engine_allreduce_async(self, t, name, op):
            self.n += 1
            self.enq.append((name, op))
            return self.n

        def engine_wait(self, h):
            self.waited.append(h)

        def engine_poll(self, h):
            return h in self.waited

    eng = ne.NativeEngine.__new__(ne.NativeEngine)
    eng._o = Ops()
    import threading

    eng._lock = threading.Lock()
    eng._outstanding = set()
    t = torch.zeros(8)
    w1 = eng.allreduce("a", t, dist.ReduceOp.SUM, None)
    w2 = eng.allreduce("b", t, dist.ReduceOp.MAX, dist.group.WORLD)
    assert isinstance(w1, ne.NativeWork) and isinstance(w2, ne.NativeWork)
    assert eng._o.enq == [("a", 0), ("b", 2)]
    assert eng.allreduce("c", t, dist.ReduceOp.SUM, object()) is None            # a sub-group
    assert eng.allreduce("d", t, dist.ReduceOp.BAND, None) is None              # not an engine op
    assert eng.allreduce("e", torch.zeros(4, 4).t(), dist.ReduceOp.SUM, None) is None  # not contiguous
    assert not w1.is_completed()
    w1.wait()
    w1.wait()  # idempotent
    assert w1.is_completed() and eng._o.waited == [1]
    eng.flush()
    assert sorted(eng._o.waited) == [1, 2] and not eng._outstanding
    assert eng.collective("x", "broadcast", "sig", lambda: "launched") == "launched"


def test_captured_step_holds_the_parameters_accumulate_grad_nodes():
    """mihvd.graphs.accumulate_grad_nodes finds one AccumulateGrad node per parameter behind a
    loss whose backward already ran, and holding them keeps autograd from building new ones for the
    next forward (the capture): the node the next step uses is the held one (CapturedStep's fix of
    the BERT-base capture NaN, scripts/bert_graph_bisect.py variant A0)."""
    from mihvd.graphs import accumulate_grad_nodes

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    loss = m(torch.randn(5, 8)).square().mean()
    loss.backward()
    nodes = accumulate_grad_nodes({"loss": loss, "aux": [loss * 2]})
    assert len(nodes) == len(list(m.parameters()))
    assert {id(n.variable) for n in nodes} == {id(p) for p in m.parameters()}
    del loss
    loss2 = m(torch.randn(5, 8)).sum()
    used = {id(n) for n in accumulate_grad_nodes(loss2)}
    assert used == {id(n) for n in nodes}  # the held nodes, not new ones


def test_every_python_source_compiles():
    """Byte-compile every Python file of the package, the examples, the scripts and the tests: GPU-only
    modules (the fused trainer, the kernel wrappers) are not imported by the CPU suite, so a syntax
    error there would otherwise surface only on the GPU box."""
    import glob

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = [f for d in ("mihvd", "examples", "scripts", "tests") for f in glob.glob(os.path.join(root, d, "**", "*.py"),
                                                                                      recursive=True)]
    files += [os.path.join(root, f) for f in ("bench.py", "__graft_entry__.py")]
    bad = []
    for f in files:
        try:
            with open(f, encoding="utf-8") as fh:
                compile(fh.read(), f, "exec")
        except SyntaxError as e:
            bad.append(f"{f}: {e}")
    assert len(files) > 50 and not bad, bad


def test_roofline_f32_filters_startup_and_classifies(tmp_path):
    """scripts/roofline_f32.py on a synthetic trace: start-up kernels (fills, copies, one-off torch
    kernels) drop out, the fragment-copy conv2 instantiations are not mistaken for the fused conv12
    launch, and the per-kernel times are medians over the steady-state window."""
    import csv
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = ["mihvd::f32_conv1_kernel(float const*)", "void mihvd::f32_conv2_fwd8_kernel<5, true, 2>(x)",
             "void mihvd::f32_fc1_fwd2_kernel<7, false, false>(x)", "mihvd::f32_head_kernel(x)",
             "void mihvd::f32_fc1_bwd_rows_kernel<7, true, false, 2, false, 25>(x)",
             "void mihvd::f32_conv2_bwd_kernel<10, true, false, 2, true>(x)", "void mihvd::f32_conv_reduce_kernel<false>(x)"]
    us = [7.0, 21.0, 12.0, 5.0, 28.0, 44.0, 5.0]
    rows, t = [], 0
    for _ in range(3):  # start-up noise
        rows.append({"Kernel_Name": "__amd_rocclr_fillBufferAligned", "Start_Timestamp": t, "End_Timestamp": t + 500})
        t += 1000
    for _ in range(40):
        for n, d in zip(names, us):
            rows.append({"Kernel_Name": n, "Start_Timestamp": t, "End_Timestamp": t + int(d * 1000)})
            t += int(d * 1000)
    trace = tmp_path / "run_kernel_trace.csv"
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "roofline_f32.py"), str(trace)],
                         capture_output=True, text=True, check=True).stdout
    assert "`conv2_fwd`" in out and "conv12_fwd" not in out and "fillBuffer" not in out.split("Filtered")[0]
    assert "| `conv2_bwd` |" in out and "44.00" in out and "| **kernel sum** | | 122.00" in out


def _vendor_gemm_sites(path, only_funcs=None):
    """(line, text) of every GEMM-shaped torch call in a module (or only inside the named functions):
    ``torch.mm``/``matmul``/``bmm``/``addmm``/``einsum``/``F.linear``/... and the ``@`` operator."""
    import ast

    tree = ast.parse(open(path).read())
    roots = [n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name in only_funcs] \
        if only_funcs else [tree]
    gemm = {"mm", "matmul", "bmm", "addmm", "baddbmm", "addbmm", "einsum", "linear", "tensordot", "mv", "addmv",
            "chain_matmul", "bilinear"}
    hits = []
    for root in roots:
        for n in ast.walk(root):
            if isinstance(n, ast.BinOp) and isinstance(n.op, ast.MatMult):
                hits.append((n.lineno, "@"))
            elif isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and n.func.attr in gemm:
                hits.append((n.lineno, n.func.attr))
    return hits


def test_fused_step_reaches_no_vendor_gemm():
    """every GEMM-shaped op of the fused step, at any world size and on every data
    plane, is a hand-written HIP kernel. The step's Python (fused_mnist.py), the xGMI and RCCL planes
    it drives, and the factor exchange it imports contain no torch GEMM; the host-reference GEMM of the
    factor plane (factor_rows_, used by the CPU tests) is not imported by the trainer."""
    import mihvd.models.fused_mnist as fm
    from mihvd.parallel import factor, rccl, xgmi

    for mod in (fm, xgmi, rccl):
        assert _vendor_gemm_sites(mod.__file__) == [], mod.__name__
    assert _vendor_gemm_sites(factor.__file__, {"factor_exchange_"}) == []
    assert _vendor_gemm_sites(factor.__file__, {"factor_rows_"}) != []  # the checker does see one
    src = open(fm.__file__).read()
    assert "factor_rows_" not in src and "torch.mm" not in src and "torch.matmul" not in src


def test_fused_trainer_knob_count():
    """the flagship module reads at most 12 MIHVD_* environment knobs (kernel-study
    switches live in the C++ launch wrappers and scripts/kbench_f32.py, not in the trainer)."""
    import re

    import mihvd.models.fused_mnist as fm

    knobs = set(re.findall(r"MIHVD_[A-Z0-9_]+", open(fm.__file__).read()))
    assert len(knobs) <= 12, sorted(knobs)


@given(n=st.integers(0, 500), k=st.integers(1, 40), lead=st.integers(0, 5))
@settings(max_examples=200, deadline=None)
def test_bench_replay_schedule_covers_exactly_n_steps(n, k, lead):
    """bench.py's timed region replays graphs of these lengths: exactly n steps in total, a short
    lead graph first when n exceeds it, whole k-step graphs, then one remainder (the bench contract:
    time EXACTLY --steps steps)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    s = bench.replay_schedule(n, k, lead)
    assert sum(s) == n and all(x > 0 for x in s)
    if lead > 0 and n > lead:
        assert s[0] == lead and all(x == k for x in s[1:-1]) and 0 < s[-1] <= k
    else:
        assert all(x == k for x in s[:-1]) and (not s or 0 < s[-1] <= k)


def _bench_line(out: str) -> dict:
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(recs) == 1, out[-2000:]  # rank 0 prints ONE line
    return recs[0]


def _check_bench_contract(r: dict, n: int, steps: int, warmup: int):
    for key, typ in (("metric", str), ("unit", str), ("dtype", str), ("data", str), ("scaling", str),
                     ("config", dict)):
        assert isinstance(r[key], typ), (key, r)
    assert r["n_gpus"] == n and r["steps"] == steps and r["warmup"] == warmup
    assert r["higher_is_better"] is True and r["scaling"] in ("weak", "strong")
    assert r["value"] > 0 and r["ms_per_step"] > 0
    assert r["vs_baseline"] is None or r["vs_baseline"] > 0
    c = r["config"]
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(c), c
    assert c["parallelism"] == f"dp{n}" and c["global_batch"] == 100 * n
    # value is the whole-job aggregate: global batch / step time
    assert abs(r["value"] - c["global_batch"] / (r["ms_per_step"] / 1000.0)) <= 0.01 * r["value"] + 1.0, r


def test_bench_json_contract_one_process_cpu():
    """bench.py prints the driver's one-line JSON contract (CPU: the stock-PyTorch DistributedOptimizer
    step on gloo; the flagship fused step needs the GPU, where the GPU tests check its line)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--impl", "torch", "--steps", "2",
                        "--warmup", "1"], env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    _check_bench_contract(_bench_line(p.stdout), 1, 2, 1)


def test_bench_json_contract_two_ranks_cpu():
    """The driver's multi-rank launch form (torch.distributed.run, 127.0.0.1) at two CPU ranks over
    gloo: one JSON line from rank 0 with n_gpus = 2, dp2 and the whole-job images/s."""
    import socket
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "2", "--impl", "torch",
           "--steps", "2", "--warmup", "1"]
    p = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    _check_bench_contract(_bench_line(p.stdout), 2, 2, 1)


def test_bench_gpus_flag_launches_its_ranks_cpu():
    """``python3 bench.py --gpus 2`` with no outer launcher starts the two ranks itself (the
    framework's launcher, gloo on the CPU): one JSON line with n_gpus = 2 — the flag is never
    silently ignored."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "MIHVD_LAUNCHED"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--impl", "torch", "--steps",
                        "2", "--warmup", "1"], env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    _check_bench_contract(_bench_line(p.stdout), 2, 2, 1)


def test_bench_gpus_flag_mismatch_exits_nonzero_cpu():
    """Under a launcher whose world size differs from ``--gpus`` the bench refuses to run."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--impl", "torch", "--steps",
                        "2", "--warmup", "1"], env=env, cwd=root, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr and not any(ln.startswith("{") for ln in p.stdout.splitlines())


def test_lr_callbacks_momentum_correction(hvd_single):
    """LearningRateWarmupCallback / LearningRateScheduleCallback with ``momentum_correction``
    (Horovod's default): while the LR changes, an optimizer with momentum (SGD) has its momentum
    scaled by new_lr / old_lr for that batch and restored at the batch end; without it the momentum
    is untouched."""
    from mihvd import keras as K
    from mihvd.models.mnist import MNISTConvNet

    model = K.Model(MNISTConvNet(impl="torch", seed=1))
    opt = torch.optim.SGD(model.module.parameters(), lr=0.1, momentum=0.9)
    model.compile(opt, loss=None)
    model._steps_per_epoch = 10
    cb = K.callbacks.LearningRateScheduleCallback(initial_lr=0.1, multiplier=0.5, staircase=False)
    cb.set_model(model)
    cb.on_epoch_begin(0)
    cb.on_batch_begin(0)
    g = opt.param_groups[0]
    assert g["lr"] == pytest.approx(0.05) and g["momentum"] == pytest.approx(0.45)
    cb.on_batch_end(0)
    assert g["momentum"] == pytest.approx(0.9) and g["lr"] == pytest.approx(0.05)
    cb2 = K.callbacks.LearningRateScheduleCallback(initial_lr=0.1, multiplier=0.25, staircase=False,
                                                    momentum_correction=False)
    cb2.set_model(model)
    cb2.on_epoch_begin(0)
    cb2.on_batch_begin(1)
    assert g["lr"] == pytest.approx(0.025) and g["momentum"] == pytest.approx(0.9)
    w = K.callbacks.LearningRateWarmupCallback(initial_lr=0.2, warmup_epochs=2)
    w.set_model(model)
    w.on_epoch_begin(0)
    w.on_batch_begin(0)  # size 1: the warmup target from the first batch
    assert g["lr"] == pytest.approx(0.2) and g["momentum"] == pytest.approx(0.9 * 0.2 / 0.025)
    w.on_batch_end(0)
    assert g["momentum"] == pytest.approx(0.9)


def test_distributed_optimizer_elastic_reset_resolves_the_new_plane(hvd_single, monkeypatch):
    """After an elastic reset (shutdown closed the old world's bucket plane) DistributedOptimizer
    must not keep the destroyed communicator: _elastic_reset resolves the new world's plane."""
    from mihvd.parallel import collectives as C
    from mihvd.models.mnist import MNISTConvNet

    model = MNISTConvNet(impl="torch", seed=1)
    opt = hvd_single.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.1),
                                          named_parameters=model.named_parameters())
    opt._plane = "old world's plane"
    calls = []
    monkeypatch.setattr(C, "bucket_plane", lambda: calls.append(1) or "new plane")
    opt._elastic_reset()
    # host parameters: no plane at all (gloo); the stale one is dropped either way
    assert opt._plane is None and calls == []
