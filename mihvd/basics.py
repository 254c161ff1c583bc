"""Process-world management: ``init / shutdown / rank / size / local_rank / local_size``.

Capability parity with the Horovod calls made by the reference:
``hvd.init()`` (horovod/tensorflow_mnist.py:90, tensorflow_mnist_gpu.py:93), ``hvd.rank()``
(:109,159), ``hvd.size()`` (:123,146), ``hvd.local_rank()`` (:155), ``hvd.local_size()`` and
``hvd.nccl_built()`` (:127).

MI355X design: one process per GPU. The data plane is ``torch.distributed`` with the ``nccl``
backend, which on ROCm *is* RCCL over xGMI; CPU-only runs (tests, BASELINE config 1) use
``gloo``. ``init()`` pins ``cuda:<local_rank>`` (the ``visible_device_list=str(local_rank)`` of
tensorflow_mnist.py:155), builds the local/cross sub-groups used by hierarchical reductions,
starts the native stall inspector and timeline, and registers ``shutdown`` at exit.
"""
from __future__ import annotations

import atexit
import datetime
import enum
import logging
import os
import threading

import torch
import torch.distributed as dist

from .config import Config
from .utils import env as _env

log = logging.getLogger("mihvd")


class ReduceOp(enum.IntEnum):
    Average = 0
    Sum = 1
    Adasum = 2
    Min = 3
    Max = 4
    Product = 5


Average = ReduceOp.Average
Sum = ReduceOp.Sum
Adasum = ReduceOp.Adasum
Min = ReduceOp.Min
Max = ReduceOp.Max
Product = ReduceOp.Product


class _Context:
    def __init__(self):
        self.initialized = False
        self.topology: _env.Topology | None = None
        self.config: Config | None = None
        self.backend: str | None = None
        self.device: torch.device = torch.device("cpu")
        self.world_group = None
        self.local_group = None
        self.cross_group = None
        self.owns_pg = False
        self.timeline = None
        self.stall = None
        self.health = None
        self.fault_plan = None
        self.store = None          # NativeStore (C++ TCP store) when launched by mihvdrun
        self.store_server = None   # StoreServer this process hosts (negotiation without mihvdrun)
        self.engine = None         # negotiated-collective Engine (MIHVD_NEGOTIATE=1)
        self.plane = None          # DistributedOptimizer's bucket data plane (collectives.BucketPlane)
        self.elastic_gen = None    # elastic: membership generation of the current world (kept across re-inits)
        self.lock = threading.RLock()


_ctx = _Context()


class NotInitializedError(RuntimeError):
    pass


def _require():
    if not _ctx.initialized:
        raise NotInitializedError("mihvd has not been initialized; call mihvd.init() first")
    return _ctx


def _choose_backend(cfg: Config) -> str:
    if cfg.backend in ("nccl", "rccl"):
        return "nccl"
    if cfg.backend == "gloo":
        return "gloo"
    return "nccl" if torch.cuda.is_available() else "gloo"


def init(comm=None, process_sets=None, config: Config | None = None):
    """Initialise the process world. Idempotent (repeated calls are no-ops)."""
    with _ctx.lock:
        if _ctx.initialized:
            return
        cfg = config or Config.from_env()
        elastic = os.environ.get("MIHVD_ELASTIC") == "1"
        # elastic workers take rank/size from the membership below, not from the launch env
        topo = _env.discover() if not elastic else _env.Topology(
            0, 1, 0, 1, 0, 1, os.environ.get("MASTER_ADDR", "127.0.0.1"),
            int(os.environ["MASTER_PORT"]) if os.environ.get("MASTER_PORT") else None, "elastic")
        native = None
        if elastic:
            # mihvd.elastic: rank/size come from the newest membership generation that includes
            # this worker (published by mihvdrun in its store), not from the launch environment
            from .elastic import wait_for_membership
            from .runner.store import NativeStore

            native = NativeStore.from_env(datetime.timedelta(seconds=cfg.timeout_s))
            if native is None:
                raise RuntimeError("MIHVD_ELASTIC=1 needs mihvdrun's store (MIHVD_STORE_ADDR)")
            wid = int(os.environ["MIHVD_WORKER_ID"])
            prev = -1 if _ctx.elastic_gen is None else _ctx.elastic_gen
            g, r, n, lr, ls = wait_for_membership(native, wid, prev, cfg.elastic_timeout_s)
            _ctx.elastic_gen = g
            topo = _env.Topology(r, n, lr, ls, 0, 1, topo.master_addr, topo.master_port, "elastic")
        backend = _choose_backend(cfg)
        # ProcessGroupNCCL's event cache hands a retired work's HIP event to the next collective;
        # when that collective is being captured into a HIP graph the watchdog may still query the
        # event through the old work and abort with hipErrorCapturedEvent. The fused trainer's
        # in-graph collectives run on its own communicator (MIHVD_COMM=native, the default) and
        # never reach the process group; this setting is for the paths that DO capture process-
        # group collectives: CapturedStep over DistributedOptimizer (mihvd/graphs.py, bench.py
        # --impl torch-graph) and MIHVD_COMM=torch. MIHVD_PG_CAPTURE=0 leaves torch's default.
        if os.environ.get("MIHVD_PG_CAPTURE", "1") == "1":
            os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        logging.basicConfig(level=getattr(logging, cfg.log_level, logging.INFO),
                            format="[%(asctime)s] [rank " + str(topo.rank) + "] %(message)s")
        if backend == "nccl":
            ndev = torch.cuda.device_count()
            if ndev == 0:
                raise RuntimeError("backend nccl (RCCL) requested but no GPU is visible")
            # an elastic worker keeps the GPU of its launch slot whatever its current rank
            dev_index = int(os.environ.get("MIHVD_DEVICE_INDEX", topo.local_rank)) if elastic else topo.local_rank
            device = torch.device("cuda", dev_index % ndev)
            torch.cuda.set_device(device)
        elif os.environ.get("MIHVD_GLOO_ON_GPU") == "1" and torch.cuda.device_count() > 0:
            # rehearsal mode: gloo collectives between ranks that share the GPU(s) of one box
            # (multi-rank code paths on a single-GPU machine; RCCL refuses two ranks per GPU)
            device = torch.device("cuda", topo.local_rank % torch.cuda.device_count())
            torch.cuda.set_device(device)
        else:
            device = torch.device("cpu")
        timeout = datetime.timedelta(seconds=cfg.timeout_s)
        if dist.is_initialized():
            _ctx.owns_pg = False
            if dist.get_world_size() != topo.size and topo.source != "single":
                raise RuntimeError("existing process group does not match the launcher environment")
            topo = _env.Topology(dist.get_rank(), dist.get_world_size(),
                                 topo.local_rank if topo.source != "single" else dist.get_rank(),
                                 topo.local_size if topo.source != "single" else dist.get_world_size(),
                                 topo.cross_rank, topo.cross_size, topo.master_addr, topo.master_port, "existing")
            backend = dist.get_backend()
        elif topo.size == 1 and topo.master_port is None and not elastic:
            # Single process without a launcher: an in-memory store, no sockets needed.
            dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1, timeout=timeout,
                                    **({"device_id": device} if backend == "nccl" else {}))
            _ctx.owns_pg = True
        elif elastic:
            kwargs = {"device_id": device} if backend == "nccl" else {}
            _ctx.store = native
            dist.init_process_group(backend, store=dist.PrefixStore(f"mihvd/pg/gen{_ctx.elastic_gen}", native),
                                    rank=topo.rank, world_size=topo.size, timeout=timeout, **kwargs)
            _ctx.owns_pg = True
        else:
            kwargs = {"device_id": device} if backend == "nccl" else {}
            native = None
            if cfg.store != "torch":
                from .runner.store import NativeStore

                native = NativeStore.from_env(timeout)
            if native is not None:
                # mihvdrun's rendezvous server (C++): RCCL's unique-id exchange runs over it
                _ctx.store = native
                dist.init_process_group(backend, store=dist.PrefixStore("mihvd/pg", native), rank=topo.rank,
                                        world_size=topo.size, timeout=timeout, **kwargs)
            else:
                port = topo.master_port or 29500
                url = f"tcp://{topo.master_addr}:{port}"
                dist.init_process_group(backend, init_method=url, rank=topo.rank, world_size=topo.size,
                                        timeout=timeout, **kwargs)
            _ctx.owns_pg = True
        _ctx.topology = topo
        _ctx.config = cfg
        _ctx.backend = backend
        _ctx.device = device
        _ctx.world_group = dist.group.WORLD
        _build_subgroups(topo)
        _start_observability(cfg, topo)
        _start_health(topo, backend)
        # Horovod's background engine, opt-in: MIHVD_ENGINE=native (the C++ engine thread over its
        # own RCCL communicator) or MIHVD_ENGINE=python / MIHVD_NEGOTIATE=1 (the store-negotiated
        # python executor). auto / torch: allreduces go straight to the process group, which
        # already orders them (every rank issues the DistributedOptimizer's buckets in the same
        # static order)
        if engine_wanted(cfg, topo.size, backend):
            _start_engine(cfg, topo, backend, device)
        _ctx.initialized = True
        atexit.register(shutdown)
        if process_sets:
            from .process_sets import add_process_set

            for ps in process_sets:
                add_process_set(ps)
        if topo.rank == 0:
            log.debug("mihvd initialised: %s backend=%s device=%s config=%s", topo, backend, device, cfg)


def engine_wanted(cfg: Config, world: int, backend: str) -> bool:
    """Whether ``init()`` starts a background engine (MIHVD_ENGINE / MIHVD_NEGOTIATE)."""
    if cfg.engine == "torch":
        return False
    if cfg.engine == "native":
        return True
    return world > 1 and (cfg.negotiate or cfg.engine == "python")


def _build_subgroups(topo: _env.Topology):
    """Local (same host) and cross (same local rank) groups for hierarchical reductions.

    ``new_group`` is collective over the world, so every rank creates every group in the same order.
    """
    if topo.size == 1:
        _ctx.local_group = dist.group.WORLD
        _ctx.cross_group = dist.group.WORLD
        return
    ls = topo.local_size
    if topo.size % ls != 0:
        _ctx.local_group = None
        _ctx.cross_group = None
        return
    nodes = topo.size // ls
    local_group = cross_group = None
    if nodes == 1:
        local_group = dist.group.WORLD
    else:
        for n in range(nodes):
            g = dist.new_group(list(range(n * ls, (n + 1) * ls)))
            if n == topo.rank // ls:
                local_group = g
    if ls == 1:
        cross_group = dist.group.WORLD
    else:
        for lr in range(ls):
            g = dist.new_group(list(range(lr, topo.size, ls)))
            if lr == topo.rank % ls:
                cross_group = g
    _ctx.local_group = local_group
    _ctx.cross_group = cross_group


def _start_observability(cfg: Config, topo: _env.Topology):
    from ._native import runtime

    rt = runtime()
    if cfg.timeline:
        path = cfg.timeline.replace("{rank}", str(topo.rank))
        if "{rank}" not in cfg.timeline and topo.size > 1:
            root, ext = os.path.splitext(path)
            path = f"{root}.rank{topo.rank}{ext or '.json'}"
        _ctx.timeline = rt.Timeline(path, topo.rank)
    if not cfg.stall_check_disable and cfg.stall_check_s > 0:
        _ctx.stall = rt.StallInspector(cfg.stall_check_s, cfg.stall_shutdown_s, min(1.0, cfg.stall_check_s / 4), topo.rank)
        _ctx.stall.start()
    if cfg.fault:
        _ctx.fault_plan = rt.FaultPlan(cfg.fault)


def _loaded_rccl_path() -> str | None:
    """Path of the librccl this process loaded (torch's bundled copy or /opt/rocm's)."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1]
                if "librccl" in os.path.basename(path) and os.path.isfile(path):
                    return path
    except OSError:  # pragma: no cover - non-Linux
        pass
    return None


def _start_health(topo: _env.Topology, backend: str):
    """Native communicator health monitor (csrc/runtime/health.cc): polls the RCCL communicator's
    async-error state and, on an error (or a ``collerr`` fault), aborts the communicator and exits
    with 134 so the launcher tears the job down — MPI's abort semantics, which the reference relies
    on (tensorflow-mnist.yaml:17-38). ``MIHVD_HEALTH=0`` disables it; ``MIHVD_HEALTH_POLL_S`` sets
    the poll interval (0.5 s)."""
    if os.environ.get("MIHVD_HEALTH", "1") == "0":
        return
    from ._native import runtime

    mon = runtime().HealthMonitor(topo.rank, float(os.environ.get("MIHVD_HEALTH_POLL_S", "0.5")), 134)
    # The monitor watches the communicators this framework owns (NativeComm and the native engine's
    # attach themselves, mihvd/parallel/rccl.py). The process group's communicator belongs to torch,
    # which can free it (destroy_process_group outside hvd.shutdown, or its watchdog's abort) while
    # the monitor thread still polls it; torch's own watchdog covers that communicator. Opt in with
    # MIHVD_HEALTH_PG=1 (then hvd.shutdown() must be the only teardown path).
    if backend == "nccl" and os.environ.get("MIHVD_HEALTH_PG", "0") == "1":
        try:
            comm = int(dist.group.WORLD._get_backend(torch.device("cuda"))._comm_ptr())
            lib = _loaded_rccl_path()
            if comm and lib and mon.attach_rccl(comm, lib):
                log.debug("health monitor attached to RCCL communicator %#x (%s)", comm, lib)
        except Exception as e:  # pragma: no cover - depends on the torch build
            log.debug("health monitor: no RCCL communicator to attach (%r)", e)
    mon.start()
    _ctx.health = mon


def _start_engine(cfg: Config, topo: _env.Topology, backend: str, device: torch.device):
    """Negotiated collectives. On the RCCL backend (``MIHVD_ENGINE`` auto/native): the native engine
    (``csrc/kernels/engine.cpp``, a C++ thread that owns an RCCL communicator and a high-priority
    stream, negotiates over the GPU and fuses into a persistent buffer). Otherwise
    (``MIHVD_ENGINE=python`` or gloo): ``mihvd/parallel/engine.py``, a native Negotiator per rank
    whose coordinator runs on rank 0, over mihvdrun's store or a store server rank 0 starts here."""
    import uuid

    if cfg.engine == "native" and backend != "nccl":
        raise RuntimeError("MIHVD_ENGINE=native needs the nccl (RCCL) backend")
    if backend == "nccl" and cfg.engine in ("auto", "native"):
        from .parallel.native_engine import NativeEngine

        _ctx.engine = NativeEngine(cfg, device)
        return

    from ._native import runtime
    from .parallel.engine import Engine
    from .runner.store import parse_addr, start_server

    if _ctx.store is not None:
        addr = f"{_ctx.store.host}:{_ctx.store.port}"
    elif topo.rank == 0:
        _ctx.store_server = start_server("0.0.0.0", 0)
        addr = f"{topo.master_addr}:{_ctx.store_server.port}"
    else:
        addr = None
    # rank 0 names the negotiation domain, so a re-init on the same store starts a fresh log
    obj = [(addr, f"mihvd/neg/{uuid.uuid4().hex[:12]}")] if topo.rank == 0 else [None]
    dist.broadcast_object_list(obj, src=0, device=device if backend == "nccl" else None)
    if _ctx.store is None:
        addr = obj[0][0]
    host, port = parse_addr(addr)
    warn = 0.0 if cfg.stall_check_disable else cfg.stall_check_s
    neg = runtime().Negotiator(host, port, topo.rank, topo.size, obj[0][1], cfg.cycle_time_ms / 1000.0, warn,
                               cfg.stall_shutdown_s)
    _ctx.engine = Engine(neg, cfg.fusion_threshold, topo.rank)


def suspend_engine(reason: str = "") -> bool:
    """Flush and stop the background engine, if one runs (a component that issues its own
    collectives, such as the fused trainer, calls this: an engine thread cycling RCCL calls on a
    second communicator beside them is the classic cross-communicator deadlock). Returns True if an
    engine was stopped. Collectives issued later go straight to the process group."""
    with _ctx.lock:
        eng = _ctx.engine
        if eng is None:
            return False
        eng.flush(timeout=30)
        eng.stop()
        _ctx.engine = None
    log.info("mihvd engine stopped%s", f": {reason}" if reason else "")
    return True


def engine_running() -> bool:
    return _ctx.engine is not None


def shutdown(abort: bool = False):
    """Tear down the world (``hvd.shutdown``). Safe to call more than once. ``abort``: after a
    failure (mihvd.elastic), the framework-owned communicators are aborted without draining the
    device first (a dead peer's collective would never complete)."""
    with _ctx.lock:
        if not _ctx.initialized:
            return
        try:
            from .parallel import collectives

            collectives._drain_all()
        except Exception:  # pragma: no cover
            pass
        if _ctx.engine is not None:
            _ctx.engine.flush(timeout=30)
            _ctx.engine.stop()
            _ctx.engine = None
        if _ctx.plane is not None:
            try:
                _ctx.plane.close(abort=abort)
            except Exception:  # pragma: no cover
                pass
            _ctx.plane = None
        if _ctx.stall is not None:
            _ctx.stall.stop()
            _ctx.stall = None
        if getattr(_ctx, "health", None) is not None:
            _ctx.health.stop()  # before the communicator is destroyed
            _ctx.health = None
        if _ctx.timeline is not None:
            _ctx.timeline.close()
            _ctx.timeline = None
        from .process_sets import _reset as _reset_process_sets

        _reset_process_sets()
        if _ctx.owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:  # pragma: no cover
                pass
        if _ctx.store_server is not None:
            _ctx.store_server.stop()
            _ctx.store_server = None
        _ctx.store = None
        _ctx.initialized = False
        _ctx.world_group = _ctx.local_group = _ctx.cross_group = None


def is_initialized() -> bool:
    return _ctx.initialized


def rank() -> int:
    return _require().topology.rank


def size() -> int:
    return _require().topology.size


def local_rank() -> int:
    return _require().topology.local_rank


def local_size() -> int:
    return _require().topology.local_size


def cross_rank() -> int:
    return _require().topology.cross_rank


def cross_size() -> int:
    return _require().topology.cross_size


def is_homogeneous() -> bool:
    t = _require().topology
    return t.size % t.local_size == 0


def device() -> torch.device:
    return _require().device


def backend() -> str:
    return _require().backend


def config() -> Config:
    return _require().config


def rccl_built() -> bool:
    """True when the collective data plane is RCCL (torch ``nccl`` backend on ROCm).

    Before ``init()`` this reports whether RCCL *can* be used on this machine.
    """
    if _ctx.initialized:
        return _ctx.backend == "nccl"
    return dist.is_nccl_available() and torch.cuda.is_available()


def nccl_built() -> bool:
    """Horovod-compatible alias of :func:`rccl_built` (used by the reference's Adasum LR rule,
    horovod/tensorflow_mnist.py:127)."""
    return rccl_built()


def gloo_built() -> bool:
    return dist.is_gloo_available()


def mpi_built() -> bool:
    return False


def ccl_built() -> bool:
    """Intel oneCCL: not part of this framework (Horovod API parity)."""
    return False


def ddl_built() -> bool:
    """IBM DDL: not part of this framework (Horovod API parity)."""
    return False


def mpi_enabled() -> bool:
    return False


def gloo_enabled() -> bool:
    return _ctx.initialized and _ctx.backend == "gloo"


def mpi_threads_supported() -> bool:
    return False


def rocm_built() -> bool:
    return torch.version.hip is not None


def cuda_built() -> bool:
    return False


def timeline():
    return _ctx.timeline


def start_timeline(path: str, mark_cycles: bool = False):
    from ._native import runtime

    c = _require()
    if c.timeline is not None:
        c.timeline.close()
    c.timeline = runtime().Timeline(path, c.topology.rank)


def stop_timeline():
    c = _require()
    if c.timeline is not None:
        c.timeline.close()
        c.timeline = None
