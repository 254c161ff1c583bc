"""Negotiated collective execution (Horovod's background loop: SURVEY.md §2.3 N1-N3, N8).

With ``MIHVD_NEGOTIATE=1`` (alias ``HOROVOD_NEGOTIATE``) every asynchronous collective
(``allreduce_async``, ``broadcast_async``, ``allgather_async``, the DistributedOptimizer's bucket
allreduces) is not launched by the calling thread. It is *submitted* to the native
:class:`Negotiator` (``csrc/runtime/negotiator.cc``) under its name, and a single executor thread
launches collectives in the order the coordinator (rank 0) publishes — the order in which names
became ready on **every** rank. Ranks may therefore enqueue tensors in different orders (different
autograd schedules, data-dependent control flow, several Python threads) without deadlocking or
mismatching RCCL/gloo calls, which is what Horovod's coordinator guarantees
(horovod/tensorflow_mnist.py:133 relies on it implicitly).

Consecutive ready allreduces with the same (dtype, device, op, process set, compression, scale
factors) are fused into one flat buffer up to the fusion threshold (``MIHVD_FUSION_THRESHOLD``,
64 MiB): one RCCL call per fused group (Horovod's MEMCPY_IN_FUSION_BUFFER / collective /
MEMCPY_OUT_FUSION_BUFFER). The fusion buffer is persistent — one per fuse key, allocated on first
use and only re-allocated to grow — so the negotiated path allocates nothing per step; the copy-out
is issued by the executor right behind the collective (stream-ordered on GPUs; gloo's CPU work is
waited for first), which is what makes the single buffer safe to refill for the next group. The coordinator also checks that all
ranks submitted the same signature (op, dtype, shape) for a name and reports tensors that some ranks
never submitted (the stall inspector, with the list of missing ranks).
"""
from __future__ import annotations

import collections
import logging
import threading

import torch
import torch.distributed as dist

log = logging.getLogger("mihvd.engine")


class _Entry:
    __slots__ = ("name", "kind", "launch", "fuse_key", "tensor", "nbytes", "work", "offset", "error", "launched",
                 "ready", "done")

    def __init__(self, name, kind, launch=None, fuse_key=None, tensor=None):
        self.name = name
        self.kind = kind
        self.launch = launch          # () -> work (unfused collectives)
        self.fuse_key = fuse_key      # fusable allreduce: (dtype, device, torch op, group id, ...)
        self.tensor = tensor          # fusable allreduce: the wire tensor, reduced in place
        self.nbytes = tensor.numel() * tensor.element_size() if tensor is not None else 0
        self.work = None
        self.offset = 0
        self.error = None
        self.launched = threading.Event()
        # device tensors: `ready` is recorded on the submitting thread's current stream (the
        # producer of the tensor), the executor's stream waits on it before reading; `done` is
        # recorded on the executor's stream behind a fused copy-out, and wait() orders the
        # caller's current stream after it
        self.ready = None
        self.done = None
        if tensor is not None and tensor.is_cuda:
            self.ready = torch.cuda.Event()
            self.ready.record(torch.cuda.current_stream(tensor.device))


class DeferredWork:
    """Work handle of a negotiated collective: waits for the executor to launch it, then for the
    collective, then copies a fused result back into the caller's tensor."""

    def __init__(self, entry: _Entry):
        self._e = entry
        self._copied = False

    def wait(self):
        e = self._e
        e.launched.wait()
        if e.error is not None:
            raise e.error
        if e.work is not None:
            e.work.wait()
        if e.done is not None:
            torch.cuda.current_stream(e.tensor.device).wait_event(e.done)
        return True

    def is_completed(self) -> bool:
        e = self._e
        if not e.launched.is_set():
            return False
        if e.work is not None and not e.work.is_completed():
            return False
        return e.done is None or e.done.query()


class Engine:
    def __init__(self, negotiator, fusion_threshold: int, rank: int):
        self.neg = negotiator
        self.threshold = int(fusion_threshold)
        self.rank = rank
        self._lock = threading.Lock()
        self._pending: dict[str, collections.deque] = collections.defaultdict(collections.deque)
        self._inflight = 0
        self._idle = threading.Condition(self._lock)
        self._stop = threading.Event()
        self.fused_launches = 0
        self.launches = 0
        self._fusion: dict = {}       # fuse key -> persistent flat buffer (grown, never per step)
        self.fusion_allocs = 0
        self._thread = threading.Thread(target=self._loop, name="mihvd-engine", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ submission (any thread)
    def _submit(self, entry: _Entry, signature: str) -> DeferredWork:
        with self._lock:
            self._pending[entry.name].append(entry)
            self._inflight += 1
        self.neg.submit(entry.name, signature)
        return DeferredWork(entry)

    def allreduce(self, name: str, wire: torch.Tensor, torch_op, group, fuse_extra=()) -> DeferredWork:
        """In-place allreduce of ``wire`` (contiguous). ``fuse_extra`` adds caller-side attributes
        that must match for two tensors to share a fusion buffer."""
        if not wire.is_contiguous():
            raise ValueError("negotiated allreduce needs a contiguous tensor")
        key = (wire.dtype, str(wire.device), register_op(torch_op, group), *fuse_extra)
        sig = f"allreduce|{wire.dtype}|{tuple(wire.shape)}|{torch_op}"
        return self._submit(_Entry(name, "allreduce", fuse_key=key, tensor=wire), sig)

    def collective(self, name: str, kind: str, signature: str, launch) -> DeferredWork:
        """Any other collective: ``launch()`` runs on the executor thread and returns a work object
        (or None when it completed synchronously)."""
        return self._submit(_Entry(name, kind, launch=launch), f"{kind}|{signature}")

    def flush(self, timeout: float | None = None):
        """Block until every submitted collective has been launched (barrier/join use this so a
        direct collective never interleaves with negotiated ones)."""
        with self._idle:
            self._idle.wait_for(lambda: self._inflight == 0, timeout=timeout)

    # ------------------------------------------------------------------ executor thread
    def _loop(self):
        while not self._stop.is_set():
            try:
                responses = self.neg.wait(0.05)
            except Exception as e:  # pragma: no cover
                log.error("negotiator failed: %s", e)
                return
            if not responses:
                continue
            # one coordinator record = one batch, identical on every rank: fusion never crosses it
            batches: list[list[_Entry]] = []
            last = None
            with self._lock:
                for r in responses:
                    q = self._pending.get(r.name)
                    if not q:
                        log.error("negotiation response for unknown collective %r", r.name)
                        continue
                    e = q.popleft()
                    if r.error:
                        e.error = RuntimeError(r.error)
                    if r.batch != last:
                        batches.append([])
                        last = r.batch
                    batches[-1].append(e)
            for b in batches:
                self._execute(b)

    def _done(self, entries):
        for e in entries:
            e.launched.set()
        with self._idle:
            self._inflight -= len(entries)
            self._idle.notify_all()

    def _execute(self, batch):
        i = 0
        while i < len(batch):
            e = batch[i]
            if e.error is not None:
                self._done([e])
                i += 1
                continue
            if e.kind != "allreduce":
                try:
                    e.work = e.launch()
                except Exception as exc:  # surfaced to the waiting thread
                    e.error = exc
                self.launches += 1
                self._done([e])
                i += 1
                continue
            # fuse the run of consecutive, compatible allreduces (order is identical on all ranks,
            # so every rank forms the same groups)
            group = [e]
            total = e.nbytes
            j = i + 1
            while (j < len(batch) and batch[j].kind == "allreduce" and batch[j].error is None
                   and batch[j].fuse_key == e.fuse_key and total + batch[j].nbytes <= self.threshold):
                group.append(batch[j])
                total += batch[j].nbytes
                j += 1
            self._launch_allreduce(group)
            i = j

    def _launch_allreduce(self, group):
        e0 = group[0]
        torch_op, process_group = _decode[e0.fuse_key[2]]
        try:
            cuda = e0.tensor.is_cuda
            if cuda:
                cur = torch.cuda.current_stream(e0.tensor.device)
                for g in group:  # the producers of every tensor of the group
                    if g.ready is not None:
                        cur.wait_event(g.ready)
            if len(group) == 1:
                e0.work = dist.all_reduce(e0.tensor, op=torch_op, group=process_group, async_op=True)
            else:
                n = sum(g.tensor.numel() for g in group)
                buf = self._fusion.get(e0.fuse_key)
                if buf is None or buf.numel() < n:
                    # geometric growth with a 64 K-element floor: readiness timing decides the groups,
                    # so a run of ever-larger ones costs O(log) allocations, not one per group
                    cap = max(n, 2 * (buf.numel() if buf is not None else 0), 1 << 16)
                    buf = torch.empty(cap, dtype=e0.tensor.dtype, device=e0.tensor.device)
                    self._fusion[e0.fuse_key] = buf
                    self.fusion_allocs += 1
                flat = buf[:n]
                off = 0
                for g in group:                                           # MEMCPY_IN_FUSION_BUFFER
                    k = g.tensor.numel()
                    flat[off:off + k].copy_(g.tensor.reshape(-1))
                    g.offset = off
                    off += k
                work = dist.all_reduce(flat, op=torch_op, group=process_group, async_op=True)
                # MEMCPY_OUT_FUSION_BUFFER right behind the collective: on GPUs the wait only orders
                # the current stream after it; gloo's CPU work completes here
                work.wait()
                done = None
                if cuda:
                    done = torch.cuda.Event()
                for g in group:
                    k = g.tensor.numel()
                    g.tensor.copy_(flat[g.offset:g.offset + k].view_as(g.tensor))
                    g.work = None
                if done is not None:
                    # the callers' streams wait for the copy-out, not just the collective
                    done.record(torch.cuda.current_stream(e0.tensor.device))
                    for g in group:
                        g.done = done
                self.fused_launches += 1
        except Exception as exc:
            for g in group:
                g.error = exc
        self.launches += 1
        self._done(group)

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=5)
        self.neg.stop()


# (op repr, group id) -> (torch op, group); filled by register_op so fuse keys stay hashable/cheap
_decode: dict = {}


def register_op(torch_op, group):
    key = (str(torch_op), id(group))
    _decode[key] = (torch_op, group)
    return key
