#!/usr/bin/env python3
"""Headline benchmark: MNIST CNN training images/sec for the whole node (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W [--impl fused|torch|ddp]

For N>1 the driver launches one rank per GPU with ``torch.distributed.run``; ranks read
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the environment (``--gpus`` must equal WORLD_SIZE). Run
without an outer launcher, ``--gpus N`` starts the N ranks itself (mihvd.runner, 127.0.0.1). Model: the reference's 2-conv CNN
(horovod/tensorflow_mnist.py:38-73, 3,274,634 params, random init), per-GPU batch 100
(:160-161), TF1 Adam (:130) with LR × size (:123), gradients averaged across ranks every step
(:133). Data: synthetic 28×28 images resident on the device (no network for MNIST).

Implementations:
  fused  — mihvd's hand-written CDNA4 HIP kernels, gradients written straight into the fusion
           buffer, RCCL collectives on it, TF1-Adam; the whole step (incl. the collectives) replayed
           as one HIP graph. --precision fp32 (default, the reference's precision): exact fp32
           operands on the fp32-input MFMAs (v_mfma_f32_16x16x4_f32 / 32x32x2_f32); --precision
           bf16: bf16 MFMA operands with fp32 accumulation, master weights and optimizer state;
           --precision fp16: the Keras mixed_float16 step (tensorflow_mnist_gpu.py:26-28) — fp16
           MFMA operands, fp32 master state, dynamic loss scaling held on the device.
  torch  — stock PyTorch-ROCm ops (fp32) + mihvd DistributedOptimizer (bucketed RCCL allreduce) +
           TF1 Adam on the multi-tensor HIP kernel.
  torch-graph — the same step (data gather, forward, backward, bucket allreduces, FusedAdam with a
           device step count) captured in one HIP graph (mihvd.graphs.CapturedStep).
  ddp    — stock PyTorch-ROCm ops (fp32) + torch DDP + torch Adam: the measured comparator
           (the reference publishes no images/sec).

Timing: W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize on both
sides; the max elapsed over ranks is used. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) MNIST CNN at 1/2/4/8 MI355X; scaling efficiency"
PER_GPU_BATCH = 100


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--impl", choices=["fused", "torch", "torch-graph", "ddp"],
                    default=os.environ.get("MIHVD_BENCH_IMPL", "fused"))
    ap.add_argument("--batch-size", type=int, default=PER_GPU_BATCH)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--graph-steps", type=int, default=0, help="fused: steps captured per HIP graph (0=auto)")
    ap.add_argument("--lead-steps", type=int, default=2, help="fused: steps of the short graph that starts every "
                    "run (0: none)")
    ap.add_argument("--pool-batches", type=int, default=600,
                    help="synthetic batches resident on device per rank (600 x 100 = the 60,000 images of MNIST's "
                         "training set the reference's ranks each iterate over: an epoch of 600 steps, reshuffled "
                         "at its boundary)")
    ap.add_argument("--compression", choices=["none", "bf16"], default="none")
    ap.add_argument("--device-span", action="store_true", default=False,
                    help="also report device_ms_per_step: the device time between events recorded around the "
                         "timed steps (host bracket minus launch / wait latency)")
    ap.add_argument("--use-adasum", action="store_true", default=False,
                    help="fused: Adasum instead of the average (the reference's --use-adasum, "
                         "horovod/tensorflow_mnist.py:31-32,126-133: lr x local_size over NCCL/RCCL, else x 1)")
    ap.add_argument("--precision", choices=["fp32", "bf16", "fp16"], default=os.environ.get("MIHVD_PRECISION", "fp32"),
                    help="fused: operand precision of the hand-written step. fp32 (default) = the reference's "
                         "launched config (fp32 placeholders + AdamOptimizer, tensorflow_mnist.py:118-130) on the "
                         "fp32-input MFMAs; bf16 = bf16 MFMA operands, fp32 accumulation/master weights; fp16 = the "
                         "mixed_float16 step with the device loss scaler")
    return ap.parse_args()


def synthetic_pool(n_batches, batch, device, seed=0):
    """This rank's resident batches: the class templates are shared by every rank (one dataset),
    the samples are drawn per rank (``seed`` = rank), like shards of MNIST."""
    from mihvd.utils.data import synthetic_mnist

    (x, y), _ = synthetic_mnist(n_train=n_batches * batch, n_test=10, seed=1234, sample_seed=seed)
    xt = torch.from_numpy(x.reshape(-1, 784)).to(device=device, dtype=torch.float32).div_(255.0)
    yt = torch.from_numpy(y.astype("int64")).to(device)
    return xt, yt


def make_torch_step(args, hvd, device, ddp=False):
    from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy
    from mihvd.optim import TFAdam

    model = MNISTConvNet(impl="torch", seed=42).to(device)
    lr = args.lr * hvd.size()
    if ddp:
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index] if device.type == "cuda" else None)
        opt = torch.optim.Adam(model.parameters(), lr=lr)
    else:
        net = model
        hvd.broadcast_parameters(model.state_dict(), 0)
        comp = hvd.Compression.bf16 if args.compression == "bf16" else hvd.Compression.none
        opt = hvd.DistributedOptimizer(TFAdam(model.parameters(), lr=lr), named_parameters=model.named_parameters(),
                                       compression=comp)
    X, Y = synthetic_pool(args.pool_batches, args.batch_size, device, seed=hvd.rank())
    state = {"i": 0}

    def step():
        i = state["i"] % args.pool_batches
        state["i"] += 1
        xb = X[i * args.batch_size:(i + 1) * args.batch_size]
        yb = Y[i * args.batch_size:(i + 1) * args.batch_size]
        opt.zero_grad(set_to_none=False) if not ddp else opt.zero_grad()
        loss = softmax_cross_entropy(net(xb), yb)
        loss.backward()
        opt.step()
        return loss

    return step, "fp32", lambda: None


def make_torch_graph_step(args, hvd, device):
    """Stock PyTorch-ROCm layers + mihvd DistributedOptimizer + FusedAdam (TF1 rule, device step
    count), the whole step (data gather, forward, backward, bucket allreduces, optimizer) captured
    in one HIP graph by mihvd.graphs.CapturedStep."""
    from mihvd.graphs import CapturedStep
    from mihvd.models.mnist import MNISTConvNet, softmax_cross_entropy
    from mihvd.optim import FusedAdam

    model = MNISTConvNet(impl="torch", seed=42).to(device)
    hvd.broadcast_parameters(model.state_dict(), 0)
    opt = hvd.DistributedOptimizer(FusedAdam(model.parameters(), lr=args.lr * hvd.size(), rule="tf"),
                                   named_parameters=model.named_parameters())
    X, Y = synthetic_pool(args.pool_batches, args.batch_size, device, seed=hvd.rank())
    B = args.batch_size
    X = X.view(args.pool_batches, B, 784)
    Y = Y.view(args.pool_batches, B)
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    xb = torch.empty(B, 784, device=device)
    yb = torch.empty(B, dtype=torch.int64, device=device)

    def step():
        i = ctr % args.pool_batches
        xb.copy_(X.index_select(0, i).squeeze(0))
        yb.copy_(Y.index_select(0, i).squeeze(0))
        opt.zero_grad(set_to_none=False)
        loss = softmax_cross_entropy(model(xb), yb)
        loss.backward()
        opt.step()
        ctr.add_(1)
        return loss

    graphed = CapturedStep(step, warmup=3)

    def run_step(n=None):
        graphed()

    return run_step, "fp32", None


def replay_schedule(n: int, k: int, lead: int) -> list:
    """Graph replays (steps each) for n steps: a lead graph of ``lead`` steps, whole k-step graphs,
    the remainder."""
    if n <= 0:
        return []
    if lead <= 0 or n <= lead:
        return [k] * (n // k) + ([n % k] if n % k else [])
    m = n - lead
    return [lead] + [k] * (m // k) + ([m % k] if m % k else [])


def make_fused_step(args, hvd, device):
    from mihvd.models.fused_mnist import FusedMNISTTrainer

    # the reference's learning-rate rule (tensorflow_mnist.py:123-130): x size for the average; x
    # local_size over NCCL (here RCCL) for Adasum, else x 1
    if args.use_adasum:
        lr_scaler = hvd.local_size() if hvd.nccl_built() else 1
    else:
        lr_scaler = hvd.size()
    tr = FusedMNISTTrainer(batch_size=args.batch_size, lr=args.lr * lr_scaler, seed=42, device=device,
                           compression=args.compression, precision=args.precision,
                           op=hvd.Adasum if args.use_adasum else None,
                           shard_optimizer=os.environ.get("MIHVD_SHARD_W3", "1") != "0")
    tr.broadcast(0)
    X, Y = synthetic_pool(args.pool_batches, args.batch_size, device, seed=hvd.rank())
    tr.set_device_dataset(X, Y)
    # N > 1: data plane of the factor gather (MIHVD_XGMI=auto: validate the direct xGMI collectives
    # against RCCL, time both planes, keep the faster; these steps are untimed and counted apart)
    tr.plane_report = tr.select_data_plane() if tr.collectives else {"plane": "none"}
    k = args.graph_steps or 20  # steps per HIP-graph replay (20: measured 66.6 vs 67.5 us at 10)
    tr.build_graph(steps_per_replay=k)
    # every run of n steps replays a short lead graph first, then whole k-step graphs, then the
    # remainder, so the timed region is exactly K steps: the host call that launches a 20-step graph
    # takes ~105 us (140 kernel nodes) before the GPU gets its first packet, so a 2-step lead graph
    # starts the GPU at once and the long graph is launched while the lead runs (measured for the
    # driver's 20 timed steps: 123.7 vs 126.1 us/step, scripts/launch_probe.py,
    # profiles/r04/launch_probe_r04u.txt)
    sizes = set(replay_schedule(args.steps, k, args.lead_steps)) | set(replay_schedule(args.warmup, k, args.lead_steps))
    for r in sorted(sizes - {k, 0}):
        tr.build_graph(steps_per_replay=r, warmup=0, primary=False)
    # setup, like the eager steps build_graph runs: untimed replays of every graph built, so the
    # first launch of a graph executable (one-time driver/queue setup, cold instruction caches) and
    # the device's ramp to its steady clock/memory state are not inside the short timed region. A
    # fresh process measured 125.8-127.6 us/step for the driver's 20 timed steps after one setup
    # replay of the main graph and 123.2-123.5 after ten (interleaved runs,
    # profiles/r04/setup_replays_r04aa.txt) -- the same as 400 timed steps (123.8-124.3): the first
    # milliseconds of GPU work in a process run slower, so the setup replays the main graph before the
    # --warmup steps: 100 times (2000 untimed training steps, ~0.25 s; round 5, three fresh processes
    # each: 119.5-121.8 us/step against 118.7-127.1 with 10 and 119.8-121.0 with 400,
    # profiles/r05/bench_setup_replays_r05aa.txt). MIHVD_BENCH_SETUP_REPLAYS sets the count.
    for _ in range(max(1, int(os.environ.get("MIHVD_BENCH_SETUP_REPLAYS", "100")))):
        tr.run_graph()
    for r in sorted(sizes - {k, 0}):
        tr.run_graph(r)
    torch.cuda.synchronize(device)

    def step(n=None):
        tr.run_graph(None if n == k else n)

    step.schedule = lambda n: replay_schedule(n, k, args.lead_steps)
    return step, args.precision, tr


def _launch_ranks(args) -> None:
    """``--gpus N`` without an outer launcher: start N ranks here, one child process per GPU, through
    the framework's own launcher (mihvd/runner/launch.py, the mpirun form of the reference's job,
    horovod/tensorflow-mnist.yaml:17-38), and exit with the job's code; rank 0's JSON line is the
    output. Runs before anything touches the GPU (the children own the devices; this process only
    waits). Under an outer launcher (torch.distributed.run / mihvdrun: WORLD_SIZE set) the world
    size must equal ``--gpus``: a mismatch exits non-zero instead of timing another GPU count."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    # a GPU job needs one device per rank (device_count() does not initialise the GPU on this image);
    # on a machine without GPUs the ranks run on the CPU over gloo (the tests' form)
    ndev = torch.cuda.device_count()
    if 0 < ndev < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) are visible")
    if args.gpus == 1:
        return
    from mihvd.runner.launch import LaunchSpec, launch

    spec = LaunchSpec(np=args.gpus, hosts=[("localhost", args.gpus)], master_addr="127.0.0.1",
                      command=[sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
    raise SystemExit(launch(spec))


def _host_wait_mode():
    """MIHVD_SYNC_WAIT=spin (default): the host waits for the GPU by spinning (hipDeviceScheduleSpin)
    instead of HIP's default scheduling, so the synchronize that closes the timed region returns as
    soon as the last kernel ends (driver form, fresh processes: 127.0 vs 128.8 µs/step median of 4,
    profiles/r04/sync_wait_r04w.txt). Set on this rank's device before torch creates its HIP
    context; MIHVD_SYNC_WAIT=auto keeps HIP's default."""
    mode = os.environ.get("MIHVD_SYNC_WAIT", "spin").strip().lower()
    if mode != "spin":
        return
    import ctypes

    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return
    count = ctypes.c_int(0)
    if hip.hipGetDeviceCount(ctypes.byref(count)) != 0 or count.value < 1:
        hip.hipGetLastError()
        return
    # the device mihvd.init() picks for this rank (local rank modulo the visible devices)
    dev = int(os.environ.get("LOCAL_RANK", "0")) % count.value
    if hip.hipSetDevice(ctypes.c_int(dev)) == 0:
        hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    hip.hipGetLastError()  # leave no sticky error for torch's launch checks


def _rccl_witness(tr, device) -> dict:
    """What RCCL itself reports (ncclCommCount / ncclCommUserRank) for the communicator the step's
    collectives ran on: the trainer's framework-owned NativeComm, or at one GPU without collectives a
    communicator created here, after the timed region, for the count alone. Every rank takes part (the
    creation is collective); rank 0's values are printed, and ``rccl_nranks_agree`` says whether every
    rank saw the same count."""
    if device.type != "cuda" or not dist.is_initialized() or dist.get_backend() != "nccl":
        return {"rccl_nranks": None}
    from mihvd.parallel.rccl import NativeComm

    comm = getattr(tr, "ncomm", None) if tr is not None else None
    if comm is None and tr is None:  # --impl torch / torch-graph: DistributedOptimizer's bucket plane
        from mihvd import basics

        plane = getattr(basics._ctx, "plane", None)
        comm = plane.comm if plane is not None else None
    own = comm is None
    try:
        if own:
            comm = NativeComm(device=device)
        n, r = comm.nranks(), comm.user_rank()
    except Exception as e:  # pragma: no cover - depends on the RCCL build
        return {"rccl_nranks": None, "rccl_error": repr(e)[:200]}
    finally:
        if own and comm is not None:
            comm.close()
    t = torch.tensor([n, -n], dtype=torch.int64, device=device)
    if dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"rccl_nranks": n, "rccl_user_rank": r, "rccl_nranks_agree": int(t[0]) == -int(t[1]) == n,
            "rccl_comm": ("trainer" if tr is not None else "bucket plane") if not own else "witness"}


def main():
    args = parse()
    _launch_ranks(args)  # before any GPU call
    _host_wait_mode()
    if args.impl == "fused":
        # the fused trainer issues its own collectives (in its HIP graph): no engine thread cycling
        # beside the timed steps
        os.environ.setdefault("MIHVD_ENGINE", "torch")
    import mihvd.torch as hvd

    hvd.init()
    device = hvd.device()
    n = hvd.size()
    if args.impl == "fused":
        step, dtype, tr = make_fused_step(args, hvd, device)
        per_call = tr.steps_per_replay
    elif args.impl == "torch-graph":
        step, dtype, _ = make_torch_graph_step(args, hvd, device)
        per_call = 1
    else:
        step, dtype, _ = make_torch_step(args, hvd, device, ddp=args.impl == "ddp")
        per_call = 1

    def run(n):
        """Exactly n steps: whole graphs of per_call steps, then one replay of the remainder (the
        fused trainer: its replay schedule, a short lead graph first)."""
        if hasattr(step, "schedule"):
            for s in step.schedule(n):
                step(s)
            return
        for _ in range(n // per_call):
            step()
        if n % per_call:
            step(n % per_call)

    if args.steps < 1:
        raise SystemExit("--steps must be >= 1")
    steps_timed = args.steps
    run(args.warmup)
    sync = (lambda: torch.cuda.synchronize()) if device.type == "cuda" else (lambda: None)
    # the barrier bracketing the timed region: at N > 1 on the fused trainer's framework-owned RCCL
    # communicator (one 4-byte allreduce on the current stream, then synchronize: ~10 us of RCCL
    # latency inside the timed region instead of the process group's barrier, which adds its own
    # stream hop and host wait), elsewhere hvd.barrier()
    forced = os.environ.get("MIHVD_FORCE_COLLECTIVES") == "1"  # (world 1 with collectives: the same path)
    comm = getattr(tr, "ncomm", None) if args.impl == "fused" and (n > 1 or forced) else None
    if comm is not None:
        token = torch.zeros(1, dtype=torch.float32, device=device)

        def barrier():
            comm.all_reduce_(token)
    else:
        barrier = hvd.barrier
    # no Python garbage collection inside the timed region (a collection pause on the host while the
    # lead graph runs could delay the long graph's launch past the lead's end). No gc.collect() in
    # front of it either: the GPU slows down while the host idles (a collection there measured
    # 118-129 us/step, profiles/r06/driver_form_gc_collect_r06ah.txt; scripts/idle_probe.py)
    gc.disable()
    sync()
    barrier()
    sync()
    # --device-span: events around the timed steps (their record calls add a few us of host time to
    # the bracket, so the headline runs without them)
    ev = ((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          if device.type == "cuda" and args.device_span else None)
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    run(steps_timed)
    if ev:
        ev[1].record()
    sync()
    barrier()
    sync()
    el = time.perf_counter() - t0
    gc.enable()
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    ms = el / steps_timed * 1000.0
    ips = steps_timed * args.batch_size * n / el
    loss_val = None
    if args.impl == "fused":
        loss_val = float(tr.last_loss())
    if args.impl != "fused":
        comm_desc = "RCCL allreduce of fp32 gradient buckets (DistributedOptimizer / DDP)"
    elif n == 1 and not tr.collectives:
        comm_desc = "none (1 GPU)"
    elif args.use_adasum:
        comm_desc = ("Adasum of the fp32 gradient buckets on the framework communicator: vector halving / distance "
                     "doubling over grouped ncclSend/ncclRecv, each level's dot products in one allreduce, HIP "
                     "combine kernels (mihvd/parallel/adasum.py adasum_vhdd_); every step, in the HIP graph")
    elif tr.f32 and tr.shard_w3 and tr.data_plane() == "xgmi":
        comm_desc = ("fp32 direct xGMI (hipIpc peer memory, device-side phase barriers, one stream): after the "
                     "gradient reduction one launch sums every rank's small gradients and this rank's 1/N of "
                     "dense/kernel's rows over the peers' regions in place (one-shot, all links) with both Adam "
                     "updates, a second gathers the peers' updated fp32 rows; every step, in the HIP graph")
    elif tr.f32 and tr.shard_w3 and getattr(tr, "f32_factor", False):
        comm_desc = ("fp32 factor gather over RCCL: all-gather of every rank's fp32 dz and all-to-all of the a2 "
                     "columns of each rank's dense/kernel rows (beside fc1_bwd's dgrad and the conv backward) -> "
                     "each rank's exact dW3 rows over all samples (one fp32 GEMM) and Adam on its 1/N of the rows "
                     "-> RCCL all-gather of the updated fp32 rows (overlapping the next step's convolutions); RCCL "
                     "allreduce of the other fp32 gradients; every step, in the HIP graph")
    elif tr.f32 and tr.data_plane() == "factor_rep":
        comm_desc = ("fp32 replicated factor gather over RCCL: all-gather of every rank's fp32 a2 (behind conv2_fwd) "
                     "and dz (behind the head) on a side stream beside fc1_fwd / head / fc1_bwd's dgrad -> every "
                     "rank forms all of dW3 over the N B samples with Adam on every row (no gradient reduce-scatter, "
                     "no row gather); RCCL allreduce of the other fp32 gradients; every step, in the HIP graph")
    elif tr.f32 and tr.shard_w3:
        comm_desc = ("RCCL reduce-scatter of dense/kernel's fp32 gradient by rows and each rank's Adam on its 1/N "
                     "of the rows on a side stream (overlapping the conv backward) -> RCCL all-gather of the "
                     "updated fp32 rows (overlapping the next step's convolutions); RCCL allreduce of the other "
                     "fp32 gradients + their Adam on the main stream over a second communicator; every step, in "
                     "the HIP graph")
    elif tr.f32:
        comm_desc = ("RCCL allreduce of the fp32 gradient fusion buffer every step: the fc bucket (98.4 % of the "
                     "bytes) on a side stream overlapping the conv backward, then the conv bucket; in the HIP graph")
    elif getattr(tr, "shard_w3", False) and tr.data_plane() == "xgmi":
        comm_desc = ("direct xGMI one-shot collectives (hipIpc peer memory, device-side phase barriers): each rank "
                     "reads the peers' bf16 fc1 factors (dz, and the a2 columns of its own dense/kernel rows), "
                     "computes the exact dW3 (all samples) for its 1/N of the rows and applies Adam to them, then "
                     "reads the peers' updated bf16 rows (overlapping the next step's convolutions); one-shot sum of "
                     "the other fp32 gradients; every step, in the HIP graph")
    elif getattr(tr, "shard_w3", False):
        comm_desc = ("RCCL all-gather of the bf16 fc1 factors (a2, dz) -> each rank computes the exact dW3 "
                     "(all samples) for its 1/N of dense/kernel's rows and applies Adam to them; RCCL all-gather "
                     "of the updated bf16 rows (overlapping the next step's convolutions); RCCL allreduce of the "
                     "other fp32 gradients; every step, in the HIP graph")
    elif getattr(tr, "gather", False):
        comm_desc = ("%s gather of the bf16 fc1 factors (a2, dz) -> exact dW3 over all samples; %s reduction of "
                     "the other fp32 gradients; every step, in the HIP graph"
                     % (("direct xGMI", "xGMI one-shot") if tr.data_plane() == "xgmi" else ("RCCL", "RCCL")))
    else:
        comm_desc = "RCCL allreduce of the fp32 gradient fusion buffer every step" + (
            " (bf16 wire)" if args.compression == "bf16" else "")
    rccl = _rccl_witness(tr if args.impl == "fused" else None, device)
    if hvd.rank() == 0:
        rec = {
            "metric": METRIC, "value": round(ips, 1), "unit": "images/sec", "n_gpus": n, "steps": steps_timed,
            "warmup": args.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": dtype, "data": "synthetic 28x28 uint8-derived images, device-resident; random-init weights",
            "config": {"model": "tensorflow_mnist 2-conv CNN (conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout0.5-fc10, 3,274,634 params)",
                       "global_batch": args.batch_size * n, "per_gpu_batch": args.batch_size, "seq_len": None,
                       "image_shape": [28, 28, 1], "parallelism": f"dp{n}", "impl": args.impl,
                       "optimizer": ("Adam (TF1 rule), lr=%g x %s, %s" % (
                           args.lr, "local_size" if args.use_adasum else "size",
                           "Adasum (vector halving / distance doubling)" if args.use_adasum else "average"))
                       if args.impl == "fused" else "Adam (TF1 rule), lr=%g x size" % args.lr,
                       "allreduce": comm_desc,
                       "steps_per_graph": per_call,
                       "replays_timed": (step.schedule(steps_timed) if hasattr(step, "schedule") else None),
                       "final_loss": loss_val,
                       # this rank's device time between events around the timed steps (the host
                       # bracket above adds the launch of the first replay and the final wait)
                       "device_ms_per_step": (round(ev[0].elapsed_time(ev[1]) / steps_timed, 5) if ev else None)},
        }
        rec["config"].update(rccl)
        if args.impl == "fused" and getattr(tr, "f32", False):
            k = tr.f32_products
            rec["config"]["fp32_products"] = (
                "fp32-input MFMA (v_mfma_f32_16x16x4_f32)" if k == 0 else
                f"fp32 operands split exactly into 3 bf16 parts, {k} part products on bf16 MFMA, fp32 accumulation "
                f"({'exact products' if k == 9 else 'dropped terms < 2^-24 relative'}) in conv2_fwd; fp32-input MFMA elsewhere")
        if args.impl == "fused" and tr.collectives:
            rec["config"]["data_plane"] = tr.plane_report
        print(json.dumps(rec), flush=True)
    if args.impl == "fused":
        tr.close()
    hvd.shutdown()


if __name__ == "__main__":
    main()
