"""Direct xGMI collectives over hipIpc-shared device memory (SURVEY.md §2.3 N4 "optional xGMI
direct allreduce", §5.8).

RCCL's ring/tree collectives pay one link latency per hop; the messages of a B=100 MNIST step
(horovod/tensorflow_mnist.py:133 reduces 8 tensors every step, all but ``dense/kernel`` under
250 KB; the factor-gather plane moves sub-MB bf16 activations) are latency-bound, and on an MI355X
node every GPU has its own xGMI link to every other GPU. So the one-shot shape is shorter: every
rank reads all peers' copies over its own links at once (``csrc/kernels/xgmi.hip``). Each
collective is one launch with a device-side phase barrier (epochs on the device, so it replays
from a HIP graph).

Two objects:

* :class:`XGMIRegion` — a node-local communicator over one IPC-shared region per rank in which
  callers place named buffers (same offsets on every rank). Collectives read peers' buffers in
  place: ``gather_rows`` (every rank's row block of a ``[world*R][C]`` buffer into the local copy,
  optionally only a column range) and ``reduce`` (sum of a buffer over ranks into a local tensor).
  Phases: each call site uses its own phase id; see ``csrc/kernels/xgmi.hip`` for what entering a
  phase promises the peers.
* :class:`XGMIAllreduce` — allreduce of arbitrary fp32 tensors (staged into a double-buffered slot).

Both need every rank of the group on ONE node (IPC handles do not cross hosts): construction
checks that collectively (hostname + kernel boot id) and raises :class:`XGMIUnavailable`
everywhere otherwise, so callers fall back to RCCL consistently. At most 8 ranks.
"""
from __future__ import annotations

import os
import socket
import warnings

import torch
import torch.distributed as dist

from .. import ops as _ops

MAX_RANKS = 8
N_PHASES = 64


class XGMIUnavailable(RuntimeError):
    """The direct xGMI path cannot be used by this group (raised on every rank alike)."""


def _node_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:  # pragma: no cover - non-Linux
        boot = ""
    return f"{socket.gethostname()}/{boot}"


def check_single_node(group=None) -> bool:
    """Collective: True on every rank iff every rank of ``group`` runs on this node."""
    ids = [None] * dist.get_world_size(group)
    dist.all_gather_object(ids, _node_id(), group=group)
    return len(set(ids)) == 1


def _group_ok(ok: bool, group, device) -> bool:
    """Collective AND of a per-rank flag."""
    backend = dist.get_backend(group)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


class XGMIRegion:
    """Node-local peer-memory communicator. ``layout`` maps buffer names to ``(numel, dtype)``;
    ``extra_bytes`` reserves raw space (e.g. allreduce slots) at :attr:`extra_offset`.
    Collective: every rank of ``group`` constructs it with the same layout."""

    def __init__(self, layout: dict, group=None, device: torch.device | None = None, extra_bytes: int = 0):
        if not dist.is_initialized():
            raise XGMIUnavailable("the xGMI path needs an initialised process group")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > MAX_RANKS:
            raise XGMIUnavailable(f"the xGMI path supports at most {MAX_RANKS} ranks (one MI355X node)")
        device = torch.device(device) if device is not None else torch.device("cuda")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        if not check_single_node(group):
            raise XGMIUnavailable("ranks span several nodes: IPC handles do not cross hosts")
        self._o = _ops.load()
        self.offsets, off = {}, 0
        self.shapes = {}
        for name, (numel, dtype) in layout.items():
            self.offsets[name] = off
            self.shapes[name] = (int(numel), dtype)
            off += (int(numel) * torch.empty((), dtype=dtype).element_size() + 255) // 256 * 256
        self.extra_offset = off
        self.nbytes = off + (int(extra_bytes) + 255) // 256 * 256
        err = None
        self.ctx = None
        try:
            self.ctx = int(self._o.xgmi_create(self.device.index, max(self.nbytes, 256), self.rank, self.world))
            mine = bytes(self._o.xgmi_handle(self.ctx).numpy().tobytes())
        except Exception as e:  # pragma: no cover - depends on the driver
            err, mine = e, b""
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        if err is None and any(not h for h in handles):
            err = RuntimeError("a peer could not export its region")
        if err is None:
            try:
                table = torch.frombuffer(bytearray(b"".join(handles)), dtype=torch.uint8).view(self.world, -1).clone()
                self._o.xgmi_open(self.ctx, table)
            except Exception as e:  # pragma: no cover - depends on the driver / peer access
                err = e
        if not _group_ok(err is None, group, self.device):
            if self.ctx is not None:
                self._o.xgmi_destroy(self.ctx)
                self.ctx = None
            raise XGMIUnavailable(f"IPC setup failed on at least one rank ({err!r})")
        dist.barrier(group=group)  # every peer opened every region before the first signal
        # Ranks sharing one GPU (the one-GPU multi-rank tests): a collective whose blocks spin in the
        # phase barrier can then hold the CUs a peer's kernel needs to reach that barrier, so every
        # collective runs in the split form (one waiting block per rank, xgmi_role.h) instead of
        # co-launched or standalone with all its blocks waiting.
        props = torch.cuda.get_device_properties(self.device)
        keys = [None] * self.world
        dist.all_gather_object(keys, (props.pci_domain_id, props.pci_bus_id, props.pci_device_id), group=group)
        self.shared_device = len(set(keys)) < self.world
        # MIHVD_XGMI_COLAUNCH_SHARED=1 (tests): keep the co-launch form on a shared device at two
        # ranks -- the exact form every rank of a real node runs -- with the hosts' role blocks
        # bounded (MIHVD_XGMI_GATHER_NBLK, the bf16 plane's fixed nblk), so the two ranks' spinning
        # role blocks cannot hold every CU the other's launch needs to reach the phase
        self.colaunch_shared = (self.shared_device and self.world <= 2
                                and os.environ.get("MIHVD_XGMI_COLAUNCH_SHARED", "0") == "1")
        self.colaunched = 0  # collectives co-launched in a compute launch (not run split-form)
        self._views = {}
        self._closed = False

    # ------------------------------------------------------------------ buffers
    def view(self, name: str) -> torch.Tensor:
        """The 1-D tensor of buffer ``name`` in this rank's region (cached)."""
        v = self._views.get(name)
        if v is None:
            numel, dtype = self.shapes[name]
            v = self._views[name] = self._o.xgmi_view(self.ctx, self.offsets[name], numel, dtype)
        return v

    def raw_view(self, offset: int, numel: int, dtype=torch.float32) -> torch.Tensor:
        return self._o.xgmi_view(self.ctx, offset, numel, dtype)

    # ------------------------------------------------------------------ collectives
    def gather_rows(self, name: str, phase: int, row_bytes: int, rows_per_rank: int, total_rows: int | None = None,
                    col_lo: int = 0, col_hi: int | None = None):
        """Copy every peer's rows ``[p*R, (p+1)*R)`` (capped at ``total_rows``) of buffer ``name``
        (viewed as rows of ``row_bytes``), byte columns ``[col_lo, col_hi)``, into this rank's copy."""
        total = self.world * rows_per_rank if total_rows is None else int(total_rows)
        col_hi = row_bytes if col_hi is None else int(col_hi)
        self._o.xgmi_gather_(self.ctx, phase, self.offsets[name], row_bytes, rows_per_rank, total, col_lo,
                             col_hi - col_lo)

    def reduce(self, name: str, phase: int, out: torch.Tensor, scale: float = 1.0, offset_elems: int = 0):
        """``out = scale * sum over ranks`` of buffer ``name`` (fp32) starting at ``offset_elems``."""
        self._o.xgmi_reduce_(self.ctx, phase, self.offsets[name] + 4 * int(offset_elems), out, scale)

    # ------------------------------------------------------------------ prepared collectives
    # A prepared collective is a descriptor id (csrc/kernels/xgmi_role.h CollRole) that either runs
    # on its own (run) or is handed to a compute op's `coll` argument, whose launch then runs it on
    # its first nblk blocks (co-launch: no extra launch, no stream fork in the step's HIP graph).
    # Descriptors hold raw pointers: the tensors they name must outlive them.
    def prepare_gather(self, name: str, phase: int, row_bytes: int, rows_per_rank: int, total_rows: int | None = None,
                       col_lo: int = 0, col_hi: int | None = None, nblk: int = 0, offset_bytes: int = 0) -> int:
        total = self.world * rows_per_rank if total_rows is None else int(total_rows)
        col_hi = row_bytes if col_hi is None else int(col_hi)
        return int(self._o.xgmi_role_gather(self.ctx, phase, self.offsets[name] + int(offset_bytes), row_bytes,
                                            rows_per_rank, total, col_lo, col_hi - col_lo, nblk))

    def prepare_reduce(self, name: str, phase: int, out: torch.Tensor, scale: float = 1.0, adam: dict | None = None,
                       nblk: int = 0, offset_elems: int = 0) -> int:
        """``out = scale * sum over ranks`` of buffer ``name``; with ``adam`` (keys p, m, v, shadow,
        state, lr, b1, b2, eps, grad_scale, rule) also the Adam update of those parameters from the
        sum, in the same launch, advancing the forward step counter like ``adam_step(bump=1)``."""
        a = adam or {}
        return int(self._o.xgmi_role_reduce(self.ctx, phase, self.offsets[name] + 4 * int(offset_elems), out, scale,
                                            a.get("p"), a.get("m"), a.get("v"), a.get("shadow"), a.get("state"),
                                            a.get("lr", 0.0), a.get("b1", 0.0), a.get("b2", 0.0), a.get("eps", 0.0),
                                            a.get("grad_scale", 1.0), a.get("rule", 0), nblk))

    def prepare_reduce_f32(self, name: str, phase: int, n: int, adam: dict, out: torch.Tensor | None = None,
                           scale: float = 1.0, offset_elems: int = 0, bump: bool = False, nblk: int = 0) -> int:
        """The fp32 plane's reduction: the sum over ranks of ``n`` floats of buffer ``name`` from
        ``offset_elems`` (rank order, times ``scale``), the Adam update of the fp32 parameters
        ``adam["p"]`` (``m``, ``v``; no bf16 copy) from it, and with ``bump`` the forward step
        counter's advance; ``out`` (optional) also receives the sum."""
        a = adam
        return int(self._o.xgmi_role_reduce_f32(self.ctx, phase, self.offsets[name] + 4 * int(offset_elems), int(n),
                                                out, scale, a["p"], a["m"], a["v"], a["state"], a["lr"], a["b1"],
                                                a["b2"], a["eps"], a["grad_scale"], a["rule"], bool(bump), nblk))

    def run(self, role: int, in_step: bool = False):
        """Launch a prepared collective on its own (current stream). ``in_step``: a launch of the
        training step (keeps MIHVD_XGMI_DEBUG_STALE's injected stale reads). On a shared device:
        the split form."""
        if self.shared_device:
            self._o.xgmi_run_split(role, -1, bool(in_step), True)
        else:
            self._o.xgmi_run(role, bool(in_step))

    def colaunch(self, role: int, in_step: bool = True) -> int:
        """The id to hand a compute op for co-launching ``role``; on a shared device the role runs
        here, split form, before that op (same stream, so it still follows every earlier launch and
        precedes every later reader), and the op gets -1."""
        if role < 0:
            return role
        if not self.shared_device or self.colaunch_shared:
            self.colaunched += 1
            return role
        self._o.xgmi_run_split(role, -1, bool(in_step), True)
        return -1

    def run_split(self, role_a: int, role_b: int = -1, in_step: bool = False, enter: bool = True):
        """One or two prepared collectives (different phases) as a dedicated launch pair on the
        current stream: a one-block launch enters and leaves the phases (the only block that waits
        for the peers), then the data launch moves the bytes (csrc/kernels/xgmi_role.h, split
        form). ``in_step``: keep MIHVD_XGMI_DEBUG_STALE's injected stale reads. ``enter=False``: the
        data launch alone (a world of one: no peer to wait for)."""
        self._o.xgmi_run_split(role_a, role_b, bool(in_step), bool(enter))

    def check(self):
        """Wait for the current stream and raise if a device-side phase barrier timed out."""
        if self.ctx is None:
            return
        err = int(self._o.xgmi_error(self.ctx))
        if err:
            ranks = [r for r in range(MAX_RANKS) if err & (1 << r)]
            raise RuntimeError(f"xGMI collective timed out waiting for rank(s) {ranks} (error word {err:#x}); "
                               "the outputs of this and every later xGMI collective are NaN")

    def watch(self, on: bool = True) -> bool:
        """Hand the host-coherent mirror of the error word to the native health monitor
        (csrc/runtime/health.cc): a phase barrier that times out mid-replay then aborts the process
        within one poll interval (exit 134, so the launcher tears the job down) instead of surfacing
        at the next host sync. Arm it once the plane is chosen for training: during
        ``select_data_plane`` a timeout means "fall back to RCCL", not "abort". False when there
        is no monitor (``MIHVD_HEALTH=0``) or no mirror."""
        from .. import basics

        mon = getattr(basics._ctx, "health", None)
        addr = int(self._o.xgmi_error_word(self.ctx)) if self.ctx is not None else 0
        if mon is None or not addr:
            return False
        if on:
            mon.watch_word(addr, f"xGMI phase barrier (rank {self.rank} of {self.world})")
        else:
            mon.unwatch_word(addr)
        self._watched = bool(on)
        return True

    def close(self):
        if not self._closed and self.ctx is not None:
            if getattr(self, "_watched", False):
                self.watch(False)  # before the word is freed
            self._views.clear()
            self._o.xgmi_destroy(self.ctx)
            self._closed = True

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            if not getattr(self, "_closed", True) and torch.cuda.is_initialized():
                self.close()
        except Exception:
            pass


class XGMIAllreduce:
    """Allreduce of any contiguous fp32 tensor of at most ``capacity_numel`` elements over the
    direct xGMI path (stage into a double-buffered slot + one reduce launch)::

        ar = XGMIAllreduce(capacity_numel=1 << 20)   # collective: every rank of the group
        ar.allreduce_(t, average=True)               # in place, on the current stream
        ar.check()                                   # raises if a device-side barrier timed out
    """

    def __init__(self, capacity_numel: int, group=None, device: torch.device | None = None, phase: int = 0):
        self.capacity = int(capacity_numel)
        self._slot = (self.capacity * 4 + 255) // 256 * 256
        self.region = XGMIRegion({}, group=group, device=device, extra_bytes=2 * self._slot)
        self.world = self.region.world
        self.rank = self.region.rank
        self.device = self.region.device
        self.phase = int(phase)

    @property
    def ctx(self):
        return self.region.ctx

    def allreduce_(self, t: torch.Tensor, average: bool = False, scale: float = 1.0) -> torch.Tensor:
        s = scale / self.world if average else scale
        self.region._o.xgmi_allreduce_(self.region.ctx, self.phase, t, self.region.extra_offset, self._slot, s)
        return t

    def check(self):
        self.region.check()

    def close(self):
        self.region.close()


def env_mode() -> str:
    """``MIHVD_XGMI``: ``0``/``off`` (RCCL only), ``1``/``on`` (use it), ``auto`` (validate and time
    against RCCL during warm-up, keep the faster; the default for the fused trainer)."""
    v = os.environ.get("MIHVD_XGMI", os.environ.get("MIHVD_XGMI_ALLREDUCE", "auto")).strip().lower()
    if v in ("0", "off", "false", "no", "rccl"):
        return "off"
    if v in ("1", "on", "true", "yes", "force"):
        return "on"
    return "auto"


def warn_fallback(reason: str):
    warnings.warn(f"direct xGMI data plane unavailable, using RCCL: {reason}", RuntimeWarning, stacklevel=2)


__all__ = ["XGMIRegion", "XGMIAllreduce", "XGMIUnavailable", "check_single_node", "env_mode", "N_PHASES",
           "MAX_RANKS"]
