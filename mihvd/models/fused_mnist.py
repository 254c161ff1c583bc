"""Fused, graph-replayed data-parallel training step for the reference MNIST CNN on MI355X.

This is the flagship path (bench.py ``--impl fused``). The default precision is the reference's:
``precision="fp32"`` (horovod/tensorflow_mnist.py:118-121,130 train fp32 variables with fp32
placeholders and AdamOptimizer). Every operand stays fp32 and GEMM-shaped work runs on gfx950's
fp32-input matrix cores (``v_mfma_f32_16x16x4_f32``: exact products, fp32 accumulation;
csrc/kernels/f32_fwd.hip, f32_bwd.hip). At world size 1 a step is seven hand-written launches:

    f32_conv1_fwd   conv1 (K = 25 taps on MFMA), bias/ReLU/pool/argmax in registers
    f32_conv2_fwd   conv2 implicit GEMM (pool-window-major rows, W2 in registers), same epilogue
    f32_fc1_fwd     split-K GEMM over W3 -> fp32 partial slabs
    f32_head        slab sum + bias + ReLU + dropout(0.5) + fc2 + softmax-xent + fc2 backward -> dz
    f32_fc1_bwd     one block per 16 rows of W3: W3 is read once for the dgrad dz.W3^T (routed
                    through the pool argmax / ReLU mask -> dY2), dW3 of the same elements is formed in
                    registers and dense/kernel's Adam is applied from them (dW3 never goes through
                    HBM); db3, dW4, db4 into the flat gradient (= fusion) buffer
    f32_conv2_bwd   conv2 dgrad -> conv1 gradient on chip -> fused conv1 wgrad; conv2 wgrad slabs
    f32_conv_reduce slab/partial-row reduction + Adam of every parameter but dense/kernel + step bump

With collectives (size() > 1, or MIHVD_FORCE_COLLECTIVES=1 at size 1) the step's collectives run
on a framework-owned RCCL communicator (mihvd/parallel/rccl.py NativeComm, MIHVD_COMM=native, the
default; MIHVD_COMM=torch uses the process group's) on a side stream, inside the same HIP graph:
by default dense/kernel's gradient is reduce-scattered by rows while the conv backward runs, every
rank applies Adam to its 1/N of the rows, and the updated fp32 rows are all-gathered while the next
step's convolutions run (the sharded optimizer); the other gradients are allreduced.

``precision="bf16"`` is the MI355X analogue of the reference's ``mixed_float16`` GPU variant
(tensorflow_mnist_gpu.py:26-28): bf16 MFMA operands with fp32 accumulation, fp32 master weights,
gradients and Adam state (no loss scaling). Its multi-GPU data plane is the "factor gather": the
ranks all-gather the bf16 fc1 factors a2/dz so every rank forms the exact all-sample dW3 for the
rows whose optimizer it owns (over RCCL, or the direct hipIpc/xGMI plane of
mihvd/parallel/xgmi.py), then all-gather the updated bf16 rows.

Parameters, gradients and Adam slots live in flat fp32 buffers laid out in TF variable order
(horovod/tensorflow_mnist.py:49-70); every kernel writes its gradient straight into its slot of
the gradient buffer, which *is* the fusion buffer — there is no pack/unpack copy. The step counter
and dropout/data indices are device-resident, so ``build_graph(k)`` captures k whole steps
(including the RCCL calls) into one HIP graph that the host replays with a single launch.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import _native
from ..utils.tracing import trace_range
from .mnist import FC1_KS, TF_PARAM_ORDER, TF_PARAM_SHAPES, MNISTConvNet

ALIGN = 64  # elements (256 B)


# Flat-buffer order: TF variable order (horovod/tensorflow_mnist.py:49-70) except that dense/kernel
# (98 % of the bytes) is moved to the end, so bucket "fc" = {dense/bias, dense_1/*, dense/kernel} is
# one contiguous tail and "everything but dense/kernel" one contiguous head.
LAYOUT_ORDER = [n for n in TF_PARAM_ORDER if n != "dense/kernel"] + ["dense/kernel"]


def _layout():
    segs, off = {}, 0
    for name in LAYOUT_ORDER:
        n = math.prod(TF_PARAM_SHAPES[name])
        segs[name] = (off, n)
        off += (n + ALIGN - 1) // ALIGN * ALIGN
    return segs, off


SEGMENTS, FLAT_NUMEL = _layout()
FC_START = SEGMENTS["dense/bias"][0]    # bucket "fc" = [dense/bias .. dense/kernel]
W3_START = SEGMENTS["dense/kernel"][0]  # [0, W3_START) = every gradient except dense/kernel


def f32_plane_mode() -> str:
    """``MIHVD_F32_PLANE``: the fp32 data plane — ``auto`` (default: select_data_plane times the
    reduce-scatter, the sharded and the replicated factor-gather planes and keeps the fastest), ``rs``,
    ``factor`` (sharded) or ``factor_rep`` (replicated)."""
    v = os.environ.get("MIHVD_F32_PLANE", "auto").strip().lower()
    return v if v in ("rs", "factor", "factor_rep") else "auto"


def _check_tol() -> float:
    """``MIHVD_XGMI_CHECK_TOL``: relative distance allowed between a candidate plane's timed steps and
    the reference plane's from the same snapshot (select_data_plane)."""
    return float(os.environ.get("MIHVD_XGMI_CHECK_TOL", "1e-3"))


class _SyncOps:
    """torch.ops.mihvd with a synchronize + error check after every launch (MIHVD_DEBUG_SYNC)."""

    def __init__(self, ops):
        self._ops = ops

    def __getattr__(self, name):
        fn = getattr(self._ops, name)

        def call(*args, **kw):
            out = fn(*args, **kw)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:  # the asynchronous fault, attributed to its kernel
                raise RuntimeError(f"mihvd kernel {name} failed: {e}") from e
            return out

        return call


def _upload_graph(g, stream) -> bool:
    """hipGraphUpload the instantiated graph (kernel packets and arguments to the device) now, at
    build time, instead of inside its first replay; runs nothing. False if unavailable."""
    try:
        import ctypes

        exec_ptr = int(g.raw_cuda_graph_exec())
        path = "libamdhip64.so"
        with open("/proc/self/maps") as f:  # the HIP runtime torch already loaded
            for line in f:
                if "libamdhip64.so" in line and "/" in line:
                    path = line[line.index("/"):].strip()
                    break
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_NOLOAD | ctypes.RTLD_GLOBAL)
        rc = lib.hipGraphUpload(ctypes.c_void_p(exec_ptr), ctypes.c_void_p(stream.cuda_stream))
        return rc == 0
    except Exception:  # pragma: no cover - depends on the torch / HIP build
        return False


class FusedMNISTTrainer:
    def __init__(self, batch_size: int = 100, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 dropout: float = 0.5, seed: int = 0, device=None, compression: str = "none", op=None,
                 adam_rule: str = "tf", dropout_seed: int | None = None, world_size: int | None = None,
                 shard_optimizer: bool | None = None, precision: str | None = None,
                 f32_products: int | None = None):
        _native.require_kernels()
        from .. import basics

        # Operand precision of the hand-written step (MIHVD_PRECISION): "fp32" = exact fp32 operands
        # on the fp32-input MFMAs (the reference's launched config: fp32 placeholders and
        # AdamOptimizer, horovod/tensorflow_mnist.py:118-121,130; csrc/kernels/f32_*.hip), "bf16" =
        # bf16 MFMA operands with fp32 accumulation and fp32 master weights (the MI355X analogue of
        # the mixed_float16 variant, tensorflow_mnist_gpu.py:26-28).
        # "fp16" = the reference's mixed_float16 policy itself (tensorflow_mnist_gpu.py:26-28): fp16
        # MFMA operands (the fp16 build of the bf16 kernels) with in-graph dynamic loss scaling
        # (_launch_step_f16)
        precision = (precision or os.environ.get("MIHVD_PRECISION", "fp32")).lower()
        if precision not in ("fp32", "bf16", "fp16"):
            raise ValueError("precision must be 'fp32', 'bf16' or 'fp16'")
        self.precision = precision
        self.f32 = precision == "fp32"
        # How the fp32 step's GEMM-shaped kernels form their products (MIHVD_F32_PRODUCTS): 6 (default)
        # or 9 = fp32 operands split exactly into three bf16 parts, the 6 / 9 part products on the bf16
        # MFMAs with fp32 accumulation (csrc/kernels/f32_common.h: products exact (9) or within fp32's
        # rounding unit (6); measured closer to a float64 reference than the fp32-input MFMA path,
        # tests/test_f32_split_gpu.py); 0 = the fp32-input MFMAs (v_mfma_f32_16x16x4_f32).
        if f32_products is None:
            f32_products = int(os.environ.get("MIHVD_F32_PRODUCTS", "6"))
        if int(f32_products) not in (0, 6, 9):
            raise ValueError("f32_products must be 0 (fp32-input MFMA), 6 or 9 (split-bf16 part products)")
        self.f32_products = int(f32_products) if self.f32 else 0
        self.f16 = precision == "fp16"

        self.ops = torch.ops.mihvd
        # MIHVD_DEBUG_SYNC=1: serialized bisection mode (the HIP_LAUNCH_BLOCKING of this engine):
        # every kernel is followed by a device synchronize, a failure names the kernel, and steps
        # run eagerly (build_graph captures nothing).
        self.debug_sync = os.environ.get("MIHVD_DEBUG_SYNC", "0") == "1"
        if self.debug_sync:
            self.ops = _SyncOps(self.ops)
        self.device = torch.device(device) if device is not None else (basics.device() if basics.is_initialized()
                                                                       else torch.device("cuda"))
        if self.device.type != "cuda":
            raise RuntimeError("FusedMNISTTrainer runs on an MI355X (cuda/hip device)")
        if not 1 <= batch_size <= 128:
            raise ValueError("fused kernels support per-GPU batch sizes 1..128")
        self.B = batch_size
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.dropout = dropout
        self.rule = 0 if adam_rule == "tf" else 1
        self.seed = int(dropout_seed if dropout_seed is not None else (seed * 7919 + 17)) & 0x7FFFFFFF
        if world_size is None:
            world_size = basics.size() if basics.is_initialized() else 1
        self.world = int(world_size)
        # MIHVD_FORCE_COLLECTIVES=1 keeps the allreduce path even at size 1 (tests of the RCCL path)
        self.collectives = self.world > 1 or os.environ.get("MIHVD_FORCE_COLLECTIVES") == "1"
        # MIHVD_COMM=native (default): the step's collectives go through a framework-owned RCCL
        # communicator (mihvd/parallel/rccl.py) instead of the process group's; the process group
        # is the fallback (MIHVD_COMM=torch, or a communicator that cannot be created)
        self.ncomm = None
        # a second framework-owned communicator for the fp32 step's small-gradient allreduce, which
        # then runs on the main stream right behind the gradient reduction while the first carries
        # dense/kernel's row collectives on the side stream: every rank issues each communicator's
        # collectives in one program order on one stream, so the two never need a cross-stream
        # edge to order them (docs/ARCHITECTURE.md, "N > 1 fp32 step")
        self.ncomm_small = None
        if self.collectives:
            from ..parallel import rccl as _rccl

            # the trainer issues its own collectives inside its HIP graph: no engine thread may run
            # RCCL calls on another communicator beside them (unordered kernels of two communicators
            # across ranks can deadlock)
            basics.suspend_engine("the fused trainer owns the step's collectives")
            if _rccl.env_mode() == "native":
                import torch.distributed as dist

                if dist.is_initialized() and dist.get_backend() == "nccl":
                    try:
                        self.ncomm = _rccl.NativeComm(device=self.device)
                        if self.f32:
                            self.ncomm_small = _rccl.NativeComm(device=self.device)
                    except Exception as e:  # pragma: no cover - depends on the RCCL build
                        import warnings

                        warnings.warn(f"native RCCL communicator unavailable ({e!r}); using the process group's")
                    ok = self.ncomm is not None and (self.ncomm_small is not None or not self.f32)
                    # every rank must use the same communicators: any failure moves all to the fallback
                    flag = torch.tensor([0 if ok else 1], device=self.device)
                    dist.all_reduce(flag)
                    if int(flag.item()) != 0:
                        for c in (self.ncomm, self.ncomm_small):
                            if c is not None:
                                c.close()
                        self.ncomm = self.ncomm_small = None
        self.rank = basics.rank() if basics.is_initialized() else 0
        self.op = op
        self.compression = compression
        self.global_step = 0
        dev = self.device
        f32 = dict(device=dev, dtype=torch.float32)
        self.params = torch.zeros(FLAT_NUMEL, **f32)
        self.grads = torch.zeros(FLAT_NUMEL, **f32)
        self.m = torch.zeros(FLAT_NUMEL, **f32)
        self.v = torch.zeros(FLAT_NUMEL, **f32)
        # bf16 copy of the parameters that the bf16 kernels read (the fp32 kernels read params)
        self.op16 = torch.float16 if self.f16 else torch.bfloat16  # the 16-bit operand format
        self.shadow = None if self.f32 else torch.zeros(FLAT_NUMEL, device=dev, dtype=self.op16)
        if self.f16:
            from ..ops.functional import _Ops16

            self._o16 = _Ops16(fp16=True)
            # Keras LossScaleOptimizer's dynamic loss scale, on the device: [scale, found_nonfinite]
            # (start 2**15, halve on overflow and skip the step, double after 2000 clean steps)
            self.loss_scale = torch.tensor([2.0 ** 15, 0.0], device=dev, dtype=torch.float32)
            self._ls_tracker = torch.zeros(1, device=dev, dtype=torch.int32)
            self.ls_growth_interval = 2000
        self.state = torch.zeros(4, device=dev, dtype=torch.int64)  # [fwd step, opt step t, -, -]
        self.shard_w3 = False
        self.f32_factor = False
        ref = MNISTConvNet(impl="torch", seed=seed)
        self.load_model_weights(ref)
        B = self.B
        bf = dict(device=dev, dtype=self.op16)
        u8 = dict(device=dev, dtype=torch.uint8)
        self.a1 = torch.empty(B, 14, 14, 32, **bf)
        self.idx1 = torch.empty(B, 14, 14, 32, **u8)
        # Data-parallel "factor gather" (bf16 step, size > 1, op Average/Sum): dW3 = a2^T dz has rank
        # B, so instead of allreducing the 12.8 MB dW3 every rank all-gathers the bf16 factors a2 and dz
        # (832 KB per rank at B=100) and multiplies them over the batch of every rank — the exact sum
        # the allreduce would produce (fp32 accumulation over all samples), 4-16x fewer bytes. With
        # compression or Adasum the bf16 step reduces gradient buckets instead.
        from ..basics import ReduceOp

        avg_or_sum = op is None or ReduceOp(op) in (ReduceOp.Average, ReduceOp.Sum)
        self.gather = self.collectives and compression == "none" and not self.f32 and not self.f16 and avg_or_sum
        # Sharded dense/kernel optimizer (shard_optimizer=True or MIHVD_SHARD_W3=1). bf16 (factor-gather
        # plane): rank r owns W3 row tiles [r*T, (r+1)*T) of the 49 64-row tiles (T = ceil(49/size)); it
        # computes dW3 for those rows only (over every rank's samples, so the result is the exact
        # allreduced sum), applies Adam to them, and gathers the updated bf16 rows of the other ranks
        # into a padded shadow [size*T*64][1024] before the next fc1_fwd. fp32: dense/kernel's gradient
        # is reduce-scattered by rows (or formed from the exchanged factors, MIHVD_F32_PLANE), Adam
        # runs on this rank's 3136/size rows, and the updated fp32 rows are all-gathered while the
        # next step's convolutions run (at size 1 with MIHVD_FORCE_COLLECTIVES the same step runs with
        # R = 3136 rows: the exact multi-rank launch/collective sequence, capture-testable on one GPU).
        # fp32 master rows / Adam slots of other ranks' rows are not maintained here; call
        # gather_full_state() on every rank before variables()/to_model(). The flag can change between
        # steps (set_sharding, collective).
        if shard_optimizer is None:
            shard_optimizer = os.environ.get("MIHVD_SHARD_W3", "0") == "1"
        self._f32_can_shard = (self.f32 and self.collectives and 3136 % self.world == 0 and compression == "none"
                               and avg_or_sum)
        self.shard_w3 = bool(shard_optimizer) and (self._f32_can_shard if self.f32 else self.gather)
        self._shadow_ev = None
        self._small_ev = None
        self._full_state_valid = True
        self._T = -(-49 // self.world)
        lo, hi = self.rank * self._T, min((self.rank + 1) * self._T, 49)
        self._w3_mine = (lo, max(lo, hi))
        # Direct xGMI data plane for the factor gather (MIHVD_XGMI=auto|on|off, mihvd/parallel/xgmi.py):
        # a2, dz, the gradient buffer and the W3 row shadow live in one hipIpc-shared region per rank;
        # the plane's collectives read the peers' copies in place over xGMI (a2 only for the columns
        # this rank's W3 rows need) and run as the first blocks of compute launches of the step
        # (co-launch: no extra launch, no stream fork/join), instead of RCCL all-gathers/allreduce on
        # a side stream. "auto" validates it against RCCL and times both (select_data_plane); ranks
        # on several nodes or a failed IPC setup fall back to RCCL.
        self.xplane = None
        self.use_xgmi = False
        self._xgmi_mode = "off"
        self._roles = None
        self._f32_gather_pending = False  # fp32 xGMI plane: the last update's row gather not yet run
        if self.gather:
            from ..parallel import xgmi as _xg

            self._xgmi_mode = _xg.env_mode()
            if self._xgmi_mode != "off" and self.world <= _xg.MAX_RANKS:
                import torch.distributed as dist

                if dist.is_initialized():
                    layout = {"a2": (self.world * B * 3136, torch.bfloat16), "dz": (self.world * B * 1024, torch.bfloat16),
                              "grads": (FLAT_NUMEL, torch.float32),
                              "shadow3": (self.world * self._T * 64 * 1024, torch.bfloat16)}
                    try:
                        self.xplane = _xg.XGMIRegion(layout, device=dev)
                    except _xg.XGMIUnavailable as e:
                        _xg.warn_fallback(str(e))
            # "on": use it from the first step; "auto": RCCL until select_data_plane() validated it
            self.use_xgmi = self.xplane is not None and self._xgmi_mode == "on"
            if self.use_xgmi:
                self.xplane.watch(True)
        if self._f32_can_shard:
            # fp32 direct-xGMI plane (sharded dense/kernel optimizer; MIHVD_XGMI, picked by
            # select_data_plane under "auto"): the parameters and the gradient buffer live in the
            # hipIpc-shared region; after the gradient reduction one launch sums every rank's small
            # gradients and this rank's dense/kernel rows over the peers' regions in place (one-shot,
            # all 7 links at once) with both Adam updates, and a second gathers the peers' updated
            # rows: two launches on the one stream, no side stream, no RCCL ring
            from ..parallel import xgmi as _xg

            self._xgmi_mode = _xg.env_mode()
            if self._xgmi_mode != "off" and self.world <= _xg.MAX_RANKS:
                import torch.distributed as dist

                if dist.is_initialized():
                    try:
                        self.xplane = _xg.XGMIRegion({"params": (FLAT_NUMEL, torch.float32),
                                                      "grads": (FLAT_NUMEL, torch.float32)}, device=dev)
                    except _xg.XGMIUnavailable as e:
                        _xg.warn_fallback(str(e))
            if self.xplane is not None:
                pr = self.xplane.view("params")
                pr.copy_(self.params)
                self.params = pr
                self.grads = self.xplane.view("grads")
                self.grads.zero_()
            self.use_xgmi = self.xplane is not None and self._xgmi_mode == "on" and self.shard_w3
            if self.use_xgmi:
                self.xplane.watch(True)
        if self.gather:
            if self.xplane is not None:
                self.a2_all = self.xplane.view("a2").view(self.world * B, 3136)
                self.dz_all = self.xplane.view("dz").view(self.world * B, 1024)
                self.grads = self.xplane.view("grads")
                self.shadow3 = self.xplane.view("shadow3").view(self.world * self._T * 64, 1024)
                self.gred = torch.zeros(W3_START, **f32)  # xGMI sum of the small gradients
            else:
                self.a2_all = torch.empty(self.world * B, 3136, **bf)
                self.dz_all = torch.empty(self.world * B, 1024, **bf)
                self.shadow3 = torch.zeros(self.world * self._T * 64, 1024, **bf)
            self.a2 = self.a2_all[self.rank * B:(self.rank + 1) * B]   # conv2_fwd writes its rows in place
            self.dz = self.dz_all[self.rank * B:(self.rank + 1) * B]   # head writes its rows in place
            self._refresh_shadow()
        else:
            self.a2 = torch.empty(B, 3136, **bf)
            self.dz = torch.empty(B, 1024, **bf)
        self.idx2 = torch.empty(B, 3136, **u8)
        self.zpart = torch.empty(FC1_KS, B, 1024, **f32)  # fc1 split-K partial slabs
        self.h = torch.empty(B, 1024, **bf)
        self.dlog = torch.empty(B, 10, **f32)
        self.stats = torch.zeros(B, 2, **f32)
        self.g2 = torch.empty(B, 3136, **bf)        # pooled conv2 gradient, masked (fc1_dgrad output)
        self.slab = torch.empty(int(self.ops.conv2_wgrad_groups(B)), 51200, **f32)
        self.cpart = torch.empty(B, 896, **f32)     # per-image dW1 | db1 | db2 partial rows
        # fp32 step: the conv1 launch also writes two fragment copies of W2 (the register operands of
        # conv2_fwd and of the conv2_bwd dgrad blocks, in the order their waves load them: one
        # contiguous 1 KB per wave-load instead of scattered 64-byte row pieces), which both conv2
        # launches of the step then read (csrc/kernels/f32_fwd.hip, f32_w2_frag_block). Measured
        # (B = 100): conv2_fwd 21.2 -> 19.8 us, conv2_bwd 43.8 -> 40.5 us, whole step 124.7 -> 122.4 us
        # (profiles/r04/kbench_f32_r04m.txt); bitwise equal
        self.w2frag = torch.empty(2, 51200, device=dev, dtype=torch.float32) if self.f32 else None
        self.keep_w3_grad = False  # tests: also store dW3 into the gradient buffer when it is fused away
        self.f32_factor = False
        if self.f32:
            ops = self.ops
            self.a1 = torch.empty(B, 14, 14, 32, **f32)
            self.a2 = torch.empty(B, 3136, **f32)
            self.zpart = torch.empty(14, B, 1024, **f32)   # fc1 split-K slabs (14 x 224)
            self.h = torch.empty(B, 1024, **f32)
            self.dz = torch.empty(B, 1024, **f32)
            self.dY2 = torch.empty(B, 14, 14, 64, **f32)   # routed conv2 output gradient
            self.db2p = torch.empty(int(ops.f32_db2_rows(B)), 64, **f32)
            self.slab = torch.empty(int(ops.f32_wgrad_groups(B, self.f32_products)), 51200, **f32)
            self.cpart = torch.empty(int(ops.f32_dgrad_blocks(B, self.f32_products)), 832, **f32)
            self.g2 = None
            # sharded dense/kernel optimizer: this rank's rows of the reduced dW3
            self._f32_R = 3136 // self.world if self.world > 0 and 3136 % self.world == 0 else 0
            self.gshard = torch.empty(max(self._f32_R, 1), 1024, **f32) if self._f32_can_shard else None
            # fp32 factor-gather plane (sharded optimizer; MIHVD_F32_PLANE=factor, or timed by
            # select_data_plane under "auto"): dW3 = a2^T dz has rank B per rank, so instead of
            # reduce-scattering the 12.8 MB dW3 every rank all-gathers the fp32 dz of all ranks
            # ([N][B][1024]) and receives from each rank the a2 columns of its own R rows ([N][B][R],
            # all-to-all); its rows of dW3 are then the exact sum over all N B samples, formed by the
            # hand-written row kernel with Adam applied from the accumulators (csrc/kernels/
            # f32_factor.hip) on the side stream beside the conv backward, and fc1_bwd runs its dgrad
            # only. Per rank (N - 1) B (1024 + R) floats arrive instead of (N - 1) R 1024 (N = 8: 3.9
            # vs 11.2 MB).
            if self._f32_can_shard:
                N, R = self.world, self._f32_R
                self.dz_all32 = torch.empty(N, B, 1024, **f32)
                # (the head writes this rank's dz into self.dz, a buffer of its own: the all-gather
                # copies it into dz_all32 while fc1_bwd reads self.dz, so the two never alias)
                self.a2_send = torch.empty(N, B, R, **f32)
                self.a2_recv = torch.empty(N, B, R, **f32)
                self.f32_factor = self.shard_w3 and f32_plane_mode() == "factor"
            # replicated fp32 factor-gather plane (small N; MIHVD_F32_PLANE=factor_rep, or timed by
            # select_data_plane): every rank all-gathers every rank's fp32 a2 and dz ([N][B][3136],
            # [N][B][1024]: (N - 1) B 4160 floats arrive, 1.66 MB per peer at B = 100, on every link at
            # once) and forms ALL of dW3 over the N B samples with Adam on every row
            # (f32_factor_full): no reduce-scatter of the 12.8 MB gradient and no row gather, at
            # N B / B times fc1's wgrad MFMA work. N = 2 moves 1.66 MB per link per step instead of the
            # sharded planes' 12.85 MB.
            self._f32_can_factor = self.collectives and compression == "none" and avg_or_sum
            self.f32_factor_rep = False
            self._a2_own, self._dz_own = self.a2, self.dz
            if self._f32_can_factor:
                N = self.world
                self.a2_all32 = torch.empty(N, B, 3136, **f32)
                if getattr(self, "dz_all32", None) is None:
                    self.dz_all32 = torch.empty(N, B, 1024, **f32)
                self.f32_factor_rep = not self.shard_w3 and f32_plane_mode() == "factor_rep"
            self._bind_factor_views()
        # fp32 step on the resident set: the batch gathered one step ahead (xpre images, ypre labels)
        # by fc1_bwd's small-reduction blocks, so the next conv1 reads its images and the next head its
        # labels with one load instead of the dependent counter -> rows -> image / label chain;
        # _xpre_valid: they hold the batch of the device counter's step (anything else that moves the
        # counter, the epoch order or the set re-primes them: _prime_batch)
        self.xpre = torch.empty(B, 784, **f32) if self.f32 else None
        self.ypre = torch.empty(B, device=dev, dtype=torch.int32) if self.f32 else None
        self._xpre_valid = False
        self.gather_ahead = self.f32  # (tests: False gathers in conv1 / head as the host-fed step does)
        self.x_buf = torch.zeros(B, 784, **f32)
        self.y_buf = torch.zeros(B, device=dev, dtype=torch.int64)
        # Keras fit (mihvd/keras.py): every step adds its (sum of losses, correct count) on the device
        self.track_stats = False
        self._stat_acc = torch.zeros(B, 2, **f32)  # per-sample running (loss, correct) sums
        self._stat_steps = 0
        self.X = self.Y = self.rows = None
        self.graph = None
        self._graphs = {}
        self.steps_per_replay = 1
        # bf16 at world size 1: no separate optimizer launch. The dense/kernel update (98 % of the
        # optimizer's HBM traffic) streams in the tail of the conv2_bwd launch — tail-only blocks on
        # the CUs the conv roles leave idle, conv blocks joining as they finish — and
        # conv2_wgrad_reduce applies Adam to every other parameter as it produces the gradients.
        # Measured (B=100): 78.4 us/step vs 80.0 us with the flat adam_step launch.
        self.fused_opt = not self.collectives and not self.f32 and not self.f16
        self._side = torch.cuda.Stream(device=dev) if (self.collectives or self.f32) else None
        if compression == "bf16" and self.collectives:
            self.wire = torch.empty(FLAT_NUMEL, **bf)
        else:
            self.wire = None
        self._closed = False

    # ----------------------------------------------------------------------------- views
    def w3_shadow(self) -> torch.Tensor:
        """The bf16 dense/kernel the MFMA kernels read ([3136][1024], contiguous): on the
        factor-gather plane the first 3136 rows of the (row-gathered) shadow3 buffer."""
        if self.gather:
            return self.shadow3[:3136]
        return self.pview("dense/kernel", self.shadow)

    @property
    def _w3_tiles(self):
        """The dense/kernel 64-row tiles whose dW3 and Adam update this rank computes."""
        return self._w3_mine if self.shard_w3 else (0, 49)

    def pview(self, name, buf=None):
        off, n = SEGMENTS[name]
        return (self.params if buf is None else buf)[off:off + n].view(TF_PARAM_SHAPES[name])

    def gview(self, name):
        return self.pview(name, self.grads)

    def load_model_weights(self, model: MNISTConvNet):
        with torch.no_grad():
            for name, p in model.ordered_parameters():
                self.pview(name).copy_(p.detach().to(self.device, torch.float32))
        self._refresh_shadow()

    def _refresh_shadow(self):
        if self.shadow is None:  # fp32 step: the kernels read the fp32 parameters
            return
        if self.f16:
            self.ops.scale_cast_f16(self.params, self.shadow, 1.0)
        else:
            self.ops.scale_cast_bf16(self.params, self.shadow, 1.0)
        if getattr(self, "shadow3", None) is not None:
            self.shadow3[:3136].copy_(self.pview("dense/kernel", self.shadow))

    def _require_full_state(self):
        if not self._full_state_valid:
            raise RuntimeError("the dense/kernel optimizer is sharded across ranks: call gather_full_state() on "
                               "every rank first")

    def to_model(self, model: MNISTConvNet | None = None) -> MNISTConvNet:
        self._require_full_state()
        self._join()
        model = model or MNISTConvNet(impl="torch").to(self.device)
        with torch.no_grad():
            for name, p in model.ordered_parameters():
                p.copy_(self.pview(name))
        return model

    # ----------------------------------------------------------------------------- data
    def set_device_dataset(self, X: torch.Tensor, Y: torch.Tensor, shuffle: bool = True, seed: int = 0):
        """Keep a dataset resident on the device; batches are gathered by index inside conv1/head."""
        n = (X.shape[0] // self.B) * self.B
        if n < self.B:
            raise ValueError("dataset smaller than one batch")
        self.X = X[:n].to(self.device, torch.float32).contiguous()
        self.Y = Y[:n].to(self.device, torch.int64).contiguous()
        self._shuffle = shuffle
        self._rng = np.random.default_rng(seed + 1000 * self.rank)
        self._next_perm = None
        self.rows = torch.empty(n, device=self.device, dtype=torch.int32)
        self._xpre_valid = False
        self._reshuffle()
        self._epoch_steps = n // self.B
        self._prepare_next_perm()

    def _draw_perm(self):
        """The next epoch order from the set's RNG (``_rng_pre``: the RNG state before the draw)."""
        import copy

        n = self.X.shape[0]
        self._rng_pre = copy.deepcopy(self._rng.bit_generator.state)
        return self._rng.permutation(n) if self._shuffle else np.arange(n)

    def _prepare_next_perm(self):
        """Draw the next epoch's order now, on the host, while the GPU runs the steps just launched,
        and upload it to ``_rows_next`` on a copy stream: the epoch boundary itself then costs one
        device-to-device copy on the compute stream. Drawing and uploading at the boundary (a host
        permutation and a pinned host-to-device copy whose DMA the compute queue waited for) left
        the GPU idle for ~30 us in bench.py's 20-step timed region, where the boundary falls between
        the lead graph and the long graph (profiles/r06/driver_form_reshuffle_gap_r06z.txt). The
        same draws in the same order as drawing at the boundary."""
        if self.X is None or getattr(self, "_next_perm", None) is not None:
            return
        self._next_perm = self._draw_perm()
        if not self.rows.is_cuda:
            return
        n = self.rows.numel()
        if getattr(self, "_pin", None) is None or self._pin.numel() != n:
            self._pin = torch.empty(n, dtype=torch.int32).pin_memory()
            self._rows_next = torch.empty_like(self.rows)
            self._copy_stream = torch.cuda.Stream(device=self.device)
        if getattr(self, "_next_ev", None) is not None:
            self._next_ev.synchronize()  # the pinned buffer's last upload (done unless an order was dropped)
        self._pin.numpy()[:] = self._next_perm
        cs = self._copy_stream
        cs.wait_stream(torch.cuda.current_stream(self.device))  # the last boundary's read of _rows_next
        with torch.cuda.stream(cs):
            self._rows_next.copy_(self._pin, non_blocking=True)
            self._next_ev = torch.cuda.Event()
            self._next_ev.record(cs)

    def _reshuffle(self):
        """New epoch permutation of the resident dataset, copied into ``rows`` on the compute stream
        (stream order keeps it behind every step still reading the old order) from the order
        prepared and uploaded an epoch earlier (_prepare_next_perm)."""
        self._xpre_valid = False  # the batch gathered ahead came from the old order
        if getattr(self, "_next_perm", None) is None:
            self._prepare_next_perm()
        perm = self._next_perm
        self._next_perm = None
        if not self.rows.is_cuda:
            self.rows.copy_(torch.from_numpy(perm.astype(np.int32)))
            return
        self._next_ev.synchronize()  # the upload (issued an epoch ago) has long finished
        self.rows.copy_(self._rows_next)

    # ----------------------------------------------------------------------------- step
    def _launch_step(self, x, rows, labels):
        # track_stats (Keras fit): the head kernel adds each sample's (loss, correct) into _stat_acc
        # [B][2] as it writes them -- the epoch's running sums without an extra launch per step
        self._launch_step_core(x, rows, labels)

    def reset_stats(self):
        """Start a new accumulation of per-step (loss, accuracy) sums (``track_stats``)."""
        self._stat_acc.zero_()
        self._stat_steps = 0

    def epoch_stats(self):
        """Mean loss and accuracy over the steps since ``reset_stats`` (``track_stats``; reading
        synchronises)."""
        n = max(1, self._stat_steps) * self.B
        s = self._stat_acc.sum(0).tolist()
        return s[0] / n, s[1] / n

    def _launch_step_core(self, x, rows, labels):
        if self.f32:
            return self._launch_step_f32(x, rows, labels)
        if self.f16:
            return self._launch_step_f16(x, rows, labels)
        if self.gather:
            return self._launch_step_gather(x, rows, labels)
        o = self.ops
        st = self.state
        main = torch.cuda.current_stream(self.device)
        self._conv_forward(x, rows, st)
        o.fc1_fwd(self.a2, self.pview("dense/kernel", self.shadow), self.zpart)
        o.head_fwd_bwd(self.zpart, self.pview("dense/bias"), self.pview("dense_1/kernel"), self.pview("dense_1/bias"),
                       labels, rows, st, self.seed, self.dropout, self.h, self.dz, self.dlog, self.stats,
                       stats_acc=self._stat_acc if self.track_stats else None)
        b1, b2 = self.betas
        if self.fused_opt:
            # dgrad tiles and every wgrad role in one launch; dense/kernel's Adam streams in the tail
            # of conv2_bwd, every other parameter's in the gradient-reduction launch
            o.fc1_bwd(self.dz, self.a2, self.h, self.dlog, self.pview("dense/kernel", self.shadow),
                      self.gview("dense/kernel"), self.gview("dense/bias"), self.gview("dense_1/kernel"),
                      self.gview("dense_1/bias"), self.g2)
            t3 = slice(W3_START, FLAT_NUMEL)
            w2 = self.pview("conv_layer2/conv2d/kernel", self.shadow)
            o.conv2_bwd_adam(self.g2, self.idx2, self.a1, w2, x, rows, st, self.idx1, self.slab, self.cpart,
                             self.params[t3], self.grads[t3], self.m[t3], self.v[t3], self.shadow[t3], self.lr, b1,
                             b2, self.eps, 1.0, self.rule)
            o.conv2_wgrad_reduce_adam(self.slab, self.cpart, self.B, self.gview("conv_layer2/conv2d/kernel"),
                                      self.gview("conv_layer1/conv2d/kernel"), self.gview("conv_layer1/conv2d/bias"),
                                      self.gview("conv_layer2/conv2d/bias"), self.grads, self.params, self.m, self.v,
                                      self.shadow, st, FC_START, W3_START, self.lr, b1, b2, self.eps, 1.0, self.rule)
            return
        # bucket plane (bf16 step with compression or Adasum): bucket "fc" is complete after
        # fc1_wgrad and is reduced on the side stream while the conv backward runs
        o.fc1_wgrad(self.dz, self.a2, self.h, self.dlog, self.gview("dense/kernel"), self.gview("dense/bias"),
                    self.gview("dense_1/kernel"), self.gview("dense_1/bias"))
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side):
            self._allreduce(self.grads[FC_START:], FC_START, FLAT_NUMEL)
        o.fc1_dgrad(self.dz, self.pview("dense/kernel", self.shadow), self.a2, self.g2)
        self._conv_backward(x, rows, st)
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side):  # one communicator, one stream: the same order on every rank
            self._allreduce(self.grads[:FC_START], 0, FC_START)
        main.wait_stream(self._side)
        o.adam_step(self.params, self.grads, self.m, self.v, self.shadow, st, 0, self.lr, b1, b2, self.eps,
                    self._gscale(), self.rule, 1)

    def _launch_step_f16(self, x, rows, labels):
        """The Keras ``mixed_float16`` step (tensorflow_mnist_gpu.py:26-28,141-145): fp16 MFMA operands
        (the fp16 build of the bf16 kernel set), fp32 master weights, Adam state and gradients, and
        Keras LossScaleOptimizer's dynamic loss scaling entirely on the device, so the step replays
        from a HIP graph like the others:

            conv12 | fc1_fwd | head (dz and dlog times S = loss_scale[0]) | fc1_bwd | conv2_bwd |
            wgrad reduce | [allreduce of the S-scaled gradients] | non-finite check -> loss_scale[1] |
            Adam (skips itself on overflow, divides by S) | fp16 operand copy | scale update

        Every gradient carries S (the head scales dlog too), so one check and one unscale cover
        them all; a skipped update takes back the optimizer step the head advanced (update_scale_)."""
        o, o16 = self.ops, self._o16
        st = self.state
        P, G, S = self.pview, self.gview, self.shadow
        b1, b2 = self.betas
        o16.conv12_fwd(x, rows, st, P("conv_layer1/conv2d/kernel", S), P("conv_layer1/conv2d/bias"),
                       P("conv_layer2/conv2d/kernel", S), P("conv_layer2/conv2d/bias"), self.a1, self.idx1, self.a2,
                       self.idx2)
        o16.fc1_fwd(self.a2, P("dense/kernel", S), self.zpart)
        o16.head_fwd_bwd(self.zpart, P("dense/bias"), P("dense_1/kernel"), P("dense_1/bias"), labels, rows, st, self.seed,
                         self.dropout, self.h, self.dz, self.dlog, self.stats, -1, 1.0,
                         self._stat_acc if self.track_stats else None, self.loss_scale)
        o16.fc1_bwd(self.dz, self.a2, self.h, self.dlog, P("dense/kernel", S), G("dense/kernel"), G("dense/bias"),
                    G("dense_1/kernel"), G("dense_1/bias"), self.g2)
        o16.conv2_bwd(self.g2, self.idx2, self.a1, P("conv_layer2/conv2d/kernel", S), x, rows, st, self.idx1, self.slab,
                      self.cpart)
        o.conv2_wgrad_reduce(self.slab, self.cpart, self.B, G("conv_layer2/conv2d/kernel"),
                             G("conv_layer1/conv2d/kernel"), G("conv_layer1/conv2d/bias"), G("conv_layer2/conv2d/bias"))
        if self.collectives:
            # the S-scaled gradients: an overflow on any rank reaches every rank's sum, so every
            # rank skips the same steps
            self._allreduce(self.grads, 0, FLAT_NUMEL)
        o.grad_check_([self.grads], self.loss_scale, False)
        o.adam_step(self.params, self.grads, self.m, self.v, None, st, 0, self.lr, b1, b2, self.eps, self._gscale(),
                    self.rule, 1, loss_scale=self.loss_scale)
        o.scale_cast_f16(self.params, self.shadow, 1.0)
        o.update_scale_(self.loss_scale, self._ls_tracker, 2.0, 0.5, self.ls_growth_interval, 1.0, state=st)

    def _launch_step_f32(self, x, rows, labels):
        """Exact-fp32 step (csrc/kernels/f32_fwd.hip, f32_bwd.hip). At world size 1, seven launches on
        one stream:

            conv1 (+ W2 fragments) | conv2 | fc1_fwd | head | fc1_bwd (dgrad -> dY2; dW3 + W3 Adam in
            registers; db3, dW4, db4) | conv2_bwd (dgrad + fused conv1 wgrad, conv2 wgrad slabs) |
            conv_reduce (+ Adam of every other parameter, step bump)

        With collectives the step's second half moves to the side stream as soon as its inputs
        exist (_launch_step_f32_shard / _f32_collective_tail); the next step's conv1 joins it."""
        o = self.ops
        st = self.state
        P, G = self.pview, self.gview
        b1, b2 = self.betas
        w2 = P("conv_layer2/conv2d/kernel")
        w3 = P("dense/kernel")
        s3 = slice(W3_START, FLAT_NUMEL)
        main = torch.cuda.current_stream(self.device)
        if self._small_ev is not None:  # the previous step's small-parameter update (side stream)
            main.wait_event(self._small_ev)
            self._small_ev = None
        wf = self.w2frag
        pre = rows is not None and self.gather_ahead
        if pre:
            self._prime_batch()
        else:
            self._xpre_valid = False  # a host-fed step advances the counter
        # fp32 xGMI plane: the previous step's row gather (every peer's updated dense/kernel rows)
        # runs on the first blocks of this launch, beside conv1 (the next reader of W3 is fc1_fwd)
        coll = self._f32_gather_colaunch() if (self.collectives and self.shard_w3 and self.use_xgmi) else -1
        o.f32_conv1_fwd(x, rows, st, P("conv_layer1/conv2d/kernel"), P("conv_layer1/conv2d/bias"), self.a1,
                        self.idx1, w2, wf, coll=coll, xpre=self.xpre if pre else None)
        o.f32_conv2_fwd(self.a1, w2, P("conv_layer2/conv2d/bias"), self.a2, self.idx2, w2frag=wf[0],
                        products=self.f32_products)
        rep_factor = self.collectives and self.f32_factor_rep
        if self._shadow_ev is not None:  # the previous step's W3 row gather (side stream)
            main.wait_event(self._shadow_ev)
            self._shadow_ev = None
        o.f32_fc1_fwd(self.a2, w3, self.zpart, products=self.f32_products)
        o.f32_head_fwd_bwd(self.zpart, P("dense/bias"), P("dense_1/kernel"), P("dense_1/bias"), labels, rows, st,
                           self.seed, self.dropout, self.h, self.dz, self.dlog, self.stats,
                           stats_acc=self._stat_acc if self.track_stats else None, ypre=self.ypre if pre else None)
        # fc1_bwd's small-reduction blocks gather the next step's batch (every fp32 plane's fc1_bwd)
        self._pf = dict(px=x, plabels=labels, prows=rows, pstate=st, xpre=self.xpre, ypre=self.ypre) if pre else {}
        gconv = (G("conv_layer2/conv2d/kernel"), G("conv_layer1/conv2d/kernel"), G("conv_layer1/conv2d/bias"),
                 G("conv_layer2/conv2d/bias"))
        if not self.collectives:
            # dgrad, dW3 and dense/kernel's Adam from one read of W3 (dW3 stays in registers unless
            # keep_w3_grad); then the gradient reduction + Adam of every other parameter + the step
            # bump in one launch
            o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, w3, self.dY2, self.db2p, G("dense/kernel"),
                          G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), self.m[s3], self.v[s3], st, self.lr,
                          b1, b2, self.eps, 1.0, self.rule, self.keep_w3_grad, **self._pf)
            o.f32_conv2_bwd(self.dY2, w2, self.a1, self.idx1, x, rows, st, self.cpart, self.slab, w2frag=wf[1],
                            products=self.f32_products)
            o.f32_conv_reduce(self.slab, self.cpart, self.db2p, *gconv, self.params, self.grads, self.m, self.v, st,
                              SEGMENTS["conv_layer1/conv2d/kernel"][0], SEGMENTS["conv_layer1/conv2d/bias"][0],
                              SEGMENTS["conv_layer2/conv2d/kernel"][0], SEGMENTS["conv_layer2/conv2d/bias"][0],
                              FC_START, W3_START, self.lr, b1, b2, self.eps, 1.0, self.rule)
            return
        if rep_factor:
            return self._launch_step_f32_factor_rep(x, rows, st, w2, wf, gconv)
        if self.shard_w3 and self.use_xgmi:
            return self._launch_step_f32_xgmi(x, rows, st, w2, wf, gconv)
        if self.shard_w3:
            return self._launch_step_f32_shard(x, rows, st, w2, wf, gconv)
        # replicated optimizer (sizes that do not divide 3136, Adasum, MIHVD_SHARD_W3=0): the "fc"
        # bucket (98.4 % of the bytes) is complete after fc1_bwd; its allreduce and Adam run on the side
        # stream beside the conv backward, then the conv bucket's
        o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, w3, self.dY2, self.db2p, G("dense/kernel"),
                      G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), **self._pf)
        side = self._side
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._allreduce(self.grads[FC_START:], FC_START, FLAT_NUMEL)
            fc = slice(FC_START, FLAT_NUMEL)
            o.adam_step(self.params[fc], self.grads[fc], self.m[fc], self.v[fc], None, st, 0, self.lr, b1, b2, self.eps,
                        self._gscale(), self.rule, 0)
            self._shadow_ev = torch.cuda.Event()  # the next step's fc1_fwd (W3's first reader) joins it
            self._shadow_ev.record(side)
        o.f32_conv2_bwd(self.dY2, w2, self.a1, self.idx1, x, rows, st, self.cpart, self.slab, w2frag=wf[1],
                            products=self.f32_products)
        o.f32_conv_reduce(self.slab, self.cpart, self.db2p, *gconv)
        self._f32_small_tail(main, FC_START)

    def _bind_factor_views(self):
        """fp32: on the replicated factor plane conv2_fwd and the head write this rank's a2 and dz
        straight into its slices of the all-gather buffers (the gathers run in place); elsewhere
        into buffers of their own."""
        if not self.f32 or getattr(self, "_a2_own", None) is None:
            return
        if getattr(self, "f32_factor_rep", False):
            self.a2, self.dz = self.a2_all32[self.rank], self.dz_all32[self.rank]
        else:
            self.a2, self.dz = self._a2_own, self._dz_own

    def _gather_factors(self):
        """Every rank's a2 and dz into a2_all32 / dz_all32, in place (this rank's slices already hold
        its own): one RCCL group on the framework communicator (nothing to move at world 1), else
        the process group (mihvd/parallel/factor.py)."""
        from ..parallel.factor import factor_gather_all_

        factor_gather_all_(self.a2_all32, self.dz_all32, self.rank, self.world, self.ncomm)

    def _launch_step_f32_factor_rep(self, x, rows, st, w2, wf, gconv):
        """Rest of the fp32 step on the replicated factor-gather plane (after the head; conv2_fwd and
        the head wrote this rank's a2 and dz into its slices of a2_all32 / dz_all32), one stream:

            AG(a2, dz: one RCCL group, in place) | fc1_bwd (dgrad only) | dW3 of all N B samples +
            Adam, every row | conv2_bwd | conv_reduce | AR(small) + Adam

        dense/kernel's update is replicated, so nothing of it crosses the links after the step. The
        all-gathers stay on the compute stream: forked onto a side stream inside the HIP graph (a2
        beside fc1_fwd / head, dz beside fc1_bwd's dgrad) the step measured 149.9 us at forced world
        1, its three cross-queue edges ~10 us each (fc1_fwd started 11.8 us after conv2_fwd,
        fc1_bwd 11.0 us after the head, the join 9.5 us after fc1_bwd:
        profiles/r06/timeline_f32_factor_rep_forked_world1_r06y.txt) -- more than the 22-33 us of
        link time per step the fork could hide at N = 2. Serial with two copying all-gathers:
        122.8 us (profiles/r06/timeline_f32_factor_rep_world1_r06aa.txt)."""
        o, G = self.ops, self.gview
        main = torch.cuda.current_stream(self.device)
        b1, b2 = self.betas
        self._gather_factors()
        o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, self.pview("dense/kernel"), self.dY2, self.db2p,
                      G("dense/kernel"), G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), store_w3=False, **self._pf)
        s3 = slice(W3_START, FLAT_NUMEL)
        o.f32_factor_full(self.a2_all32.view(-1, 3136), self.dz_all32.view(-1, 1024), self.B,
                          G("dense/kernel") if self.keep_w3_grad else None, self.params[s3], self.m[s3], self.v[s3], st,
                          self.lr, b1, b2, self.eps, 1.0 / self.world, self.rule)
        o.f32_conv2_bwd(self.dY2, w2, self.a1, self.idx1, x, rows, st, self.cpart, self.slab, w2frag=wf[1],
                        products=self.f32_products)
        o.f32_conv_reduce(self.slab, self.cpart, self.db2p, *gconv)
        self._f32_small_tail(main, W3_START)

    def _prime_batch(self):
        """fp32, resident set: gather the batch of the device counter's step into xpre/ypre unless the
        previous step's head already did (stream-ordered, no host synchronisation)."""
        if self._xpre_valid or not self.gather_ahead:
            return
        self.ops.f32_prime_batch(self.X, self.Y, self.rows, self.state, self.xpre, self.ypre)
        self._xpre_valid = True

    def _f32_small_tail(self, main, hi):
        """After the gradient reduction: allreduce of gradients [0, hi), their Adam update and the
        step bump. With the second communicator (or host collectives, which run in host program
        order) on the main stream, right behind the reduction: no stream edge, and the next step's
        conv1 simply follows. On the process group's one RCCL communicator (MIHVD_COMM=torch) on the
        side stream instead, behind the row collectives (one communicator, one stream: every rank
        issues the step's collectives in one order); the next step's conv1 waits for its event."""
        b1, b2 = self.betas
        on_main = self.ncomm_small is not None or self._host_collectives()
        stream = main if on_main else self._side
        if not on_main:
            stream.wait_stream(main)
        elif self.ncomm_small is not None:
            # two RCCL communicators must not run collectives concurrently (kernels of two
            # communicators interleaved differently on different ranks can deadlock): the side
            # stream's row / bucket collectives on ncomm complete before ncomm_small's allreduce
            main.wait_stream(self._side)
        with torch.cuda.stream(stream):
            self._allreduce(self.grads[:hi], 0, hi, comm=self.ncomm_small)
            self.ops.adam_step(self.params[:hi], self.grads[:hi], self.m[:hi], self.v[:hi], None, self.state, 0, self.lr,
                               b1, b2, self.eps, self._gscale(), self.rule, 1)
            if not on_main:
                self._small_ev = torch.cuda.Event()
                self._small_ev.record(stream)

    def _launch_step_f32_shard(self, x, rows, st, w2, wf, gconv):
        """Rest of the fp32 step with dense/kernel's optimizer sharded by rows (after the head):

            main: fc1_bwd (dgrad, dW3) | conv2_bwd | conv_reduce |
            side:                      RS(dW3 rows) Adam(my rows) | AR(small) Adam(small) | AG(W3 rows)
                                                                  ^ next conv1 waits    ^ next fc1_fwd waits

        The reduce-scatter and this rank's row update overlap the conv backward; the small
        gradients' allreduce + update follow the reduction launch; the row all-gather of the updated
        fp32 W3 overlaps the next step's convolutions. On the factor plane fc1_bwd runs its dgrad only
        and the side stream exchanges the fc1 factors instead (_launch_step_f32_factor). Adam slots of
        other ranks' rows are not maintained (gather_full_state() collects them)."""
        o, G = self.ops, self.gview
        main, side = torch.cuda.current_stream(self.device), self._side
        b1, b2 = self.betas
        R, r = self._f32_R, self.rank
        gW3 = G("dense/kernel")
        mine = slice(W3_START + r * R * 1024, W3_START + (r + 1) * R * 1024)
        w3 = self.pview("dense/kernel")
        if self.f32_factor:
            side.wait_stream(main)  # the head wrote dz; conv2_fwd wrote a2
            with torch.cuda.stream(side):
                from ..parallel.factor import factor_exchange_

                factor_exchange_(self.a2, self.dz, self.dz_all32, self.a2_send, self.a2_recv, self.rank, self.world,
                                 self.ncomm)
            o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, w3, self.dY2, self.db2p, gW3,
                          G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), store_w3=False, **self._pf)
            side.wait_stream(main)  # fc1_bwd, the step's last reader of W3, is done
            with torch.cuda.stream(side):
                # this rank's dW3 rows over all N B samples, Adam from the accumulators
                o.f32_factor_rows(self.a2_recv, self.dz_all32, self.gshard if self.keep_w3_grad else None,
                                  self.params[mine], self.m[mine], self.v[mine], st, self.lr, b1, b2, self.eps,
                                  1.0 / self.world, self.rule)
        else:
            o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, w3, self.dY2, self.db2p, gW3,
                          G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), **self._pf)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                # in place: this rank's rows of the sum land in its own rows of dW3 (at world size 1
                # a no-op instead of a 12.8 MB copy)
                mine_g = gW3.view(3136, 1024)[r * R:(r + 1) * R]
                self._reduce_scatter_rows(gW3, mine_g, R)
                o.adam_step(self.params[mine], mine_g.reshape(-1), self.m[mine], self.v[mine], None, st, 0, self.lr,
                            b1, b2, self.eps, 1.0 / self.world, self.rule, 0)
        o.f32_conv2_bwd(self.dY2, w2, self.a1, self.idx1, x, rows, st, self.cpart, self.slab, w2frag=wf[1],
                            products=self.f32_products)
        o.f32_conv_reduce(self.slab, self.cpart, self.db2p, *gconv)
        self._f32_small_tail(main, W3_START)
        if self.ncomm_small is not None:
            side.wait_stream(main)  # the row all-gather (ncomm) after ncomm_small's allreduce
        with torch.cuda.stream(side):
            p3 = self.params[W3_START:].view(3136, 1024)
            self._all_gather_rows(p3, p3[r * R:(r + 1) * R])
            self._shadow_ev = torch.cuda.Event()
            self._shadow_ev.record(side)
        self._full_state_valid = False

    # phases of the fp32 xGMI plane (its own region), in step order
    PH32_SMALL, PH32_ROWS, PH32_GATHER = 0, 1, 2

    def _prepare_roles_f32(self):
        """The fp32 plane's prepared collectives (they hold the buffers' pointers and the optimizer
        hyper-parameters: a new learning rate, or keep_w3_grad, prepares them again)."""
        xp, W, R, r = self.xplane, self.world, self._f32_R, self.rank
        b1, b2 = self.betas
        hyper = dict(state=self.state, lr=self.lr, b1=b1, b2=b2, eps=self.eps, grad_scale=1.0 / W, rule=self.rule)
        h = slice(0, W3_START)
        mine = slice(W3_START + r * R * 1024, W3_START + (r + 1) * R * 1024)
        roles = {"lr": self.lr, "keep": self.keep_w3_grad}
        # the small gradients summed over every rank + their Adam + the forward step bump
        if self.keep_w3_grad and getattr(self, "gred32", None) is None:
            self.gred32 = torch.empty(W3_START, device=self.device, dtype=torch.float32)
        roles["small"] = xp.prepare_reduce_f32("grads", self.PH32_SMALL, W3_START,
                                               dict(p=self.params[h], m=self.m[h], v=self.v[h], **hyper),
                                               out=self.gred32 if self.keep_w3_grad else None, bump=True)
        # this rank's dense/kernel rows summed over every rank + their Adam
        roles["rows"] = xp.prepare_reduce_f32("grads", self.PH32_ROWS, R * 1024,
                                              dict(p=self.params[mine], m=self.m[mine], v=self.v[mine], **hyper),
                                              out=self.gshard if self.keep_w3_grad else None,
                                              offset_elems=W3_START + r * R * 1024)
        # every peer's updated rows into this rank's dense/kernel: as a split-form launch pair (the
        # flush before a state read, validation) and co-launched on the first blocks of the next
        # step's conv1 (one 256-thread block per CU beside conv1's small blocks; at world 1 a fence
        # of 8 blocks that enters and leaves the phase and moves nothing, so the forced step prices
        # the entry)
        roles["gather"] = xp.prepare_gather("params", self.PH32_GATHER, 4096, R, 3136, offset_bytes=W3_START * 4)
        roles["gather_co"] = xp.prepare_gather("params", self.PH32_GATHER, 4096, R, 3136, offset_bytes=W3_START * 4,
                                               nblk=self._gather_nblk())
        self._roles = roles

    def _gather_nblk(self) -> int:
        """Role blocks of the row gather co-launched in conv1: one 256-thread block per CU at N > 1
        (a multiple of 8 keeps conv1's XCD map), a fence of 8 blocks at world 1 (nothing to move).
        MIHVD_XGMI_GATHER_NBLK overrides (a multiple of 8; the shared-device co-launch test bounds
        it)."""
        env = os.environ.get("MIHVD_XGMI_GATHER_NBLK")
        if env:
            return max(8, int(env) // 8 * 8)
        if self.world == 1:
            return 8
        return max(8, min(256, torch.cuda.get_device_properties(self.device).multi_processor_count) // 8 * 8)

    def _f32_gather_colaunch(self) -> int:
        """The gather descriptor for this step's conv1 (on a shared GPU the gather runs split-form
        right here and conv1 gets -1; xgmi.py colaunch)."""
        R = self._roles
        if R is None or R.get("kind") == "bf16" or R["lr"] != self.lr or R["keep"] != self.keep_w3_grad:
            self._prepare_roles_f32()
            R = self._roles
        self._f32_gather_pending = False
        return self.xplane.colaunch(R["gather_co"])

    def flush_row_gather(self):
        """fp32 xGMI plane: run the row gather of the last update now, split form, instead of in the
        next step's conv1 launch (before the parameters are read as a whole, or the plane changes).
        Collective: every rank calls it at the same point (gather_full_state, _set_plane, close)."""
        if not getattr(self, "_f32_gather_pending", False) or self.xplane is None:
            self._f32_gather_pending = False
            return
        R = self._roles
        if R is None or R.get("kind") == "bf16":
            self._prepare_roles_f32()
            R = self._roles
        self.xplane.run_split(R["gather"], in_step=True)
        self._f32_gather_pending = False

    def _launch_step_f32_xgmi(self, x, rows, st, w2, wf, gconv):
        """Rest of the fp32 step on the direct xGMI plane (after the head), one stream:

            fc1_bwd (dgrad, dW3 -> region) | conv2_bwd | conv_reduce (small grads -> region) |
            xGMI: small sum + Adam + bump, my dense/kernel rows' sum + Adam |
            next step: conv1 [+ the row gather of every peer's updated rows, co-launched]

        The row gather overlaps the next step's conv1 (its blocks move the bytes on the CUs beside
        conv1's small blocks); fc1_fwd, W3's first reader, follows that launch. Buffer reuse follows
        the phase order (xgmi_role.h): a rank rewrites its gradients (next fc1_bwd / conv_reduce)
        only after the row gather's phase (in its next conv1), which every peer enters only after its
        reductions (the readers of those gradients) completed; it rewrites its rows (next
        reduction) only after every peer entered the next reduction phase, i.e. finished its conv1
        launch and with it this update's gather. A gather with nothing new to move (the first step,
        after a flush) copies rows equal to the local ones."""
        o, G = self.ops, self.gview
        R = self._roles
        if R is None or R.get("kind") == "bf16" or R["lr"] != self.lr or R["keep"] != self.keep_w3_grad:
            self._prepare_roles_f32()
            R = self._roles
        o.f32_fc1_bwd(self.dz, self.a2, self.idx2, self.h, self.dlog, self.pview("dense/kernel"), self.dY2, self.db2p,
                      G("dense/kernel"), G("dense/bias"), G("dense_1/kernel"), G("dense_1/bias"), **self._pf)
        o.f32_conv2_bwd(self.dY2, w2, self.a1, self.idx1, x, rows, st, self.cpart, self.slab, w2frag=wf[1],
                            products=self.f32_products)
        o.f32_conv_reduce(self.slab, self.cpart, self.db2p, *gconv)
        # (at world 1, forced collectives, the entry runs too: a self-peer phase, priced like N > 1)
        self.xplane.run_split(R["small"], R["rows"])
        # the row gather of this update runs in the next step's conv1 launch (or flush_row_gather)
        self._f32_gather_pending = True
        self._full_state_valid = False

    def _validate_xgmi_f32(self) -> bool:
        """Run the fp32 plane's collectives on random data (the reductions without their Adam
        update) and compare them with the same collectives over the process group: the sums to
        fp32 rounding, the row gather bitwise. Collective; the parameters and gradients are
        restored."""
        import torch.distributed as dist

        if self._roles is None or self._roles.get("kind") == "bf16" or self._roles["lr"] != self.lr:
            self._prepare_roles_f32()
        W, r, R = self.world, self.rank, self._f32_R
        g = torch.Generator(device="cpu").manual_seed(9173 + r)
        saved_p, saved_g = self.params.clone(), self.grads.clone()
        self.grads.copy_(torch.randn(FLAT_NUMEL, generator=g))
        p3 = self.params[W3_START:].view(3136, 1024)
        p3[r * R:(r + 1) * R].copy_(torch.randn(R, 1024, generator=g))
        ref_g = self.grads.clone()
        dist.all_reduce(ref_g)
        ref_p = p3.clone()
        self._all_gather_rows(ref_p, ref_p[r * R:(r + 1) * R])
        torch.cuda.synchronize(self.device)
        out_s = torch.empty(W3_START, device=self.device)
        out_r = torch.empty(R * 1024, device=self.device)
        if "v_small" not in self._roles:  # the reductions without their Adam update, into out_s / out_r
            self._val_out = (out_s, out_r)
            self._roles["v_small"] = self.xplane.prepare_reduce("grads", self.PH32_SMALL, out_s)
            self._roles["v_rows"] = self.xplane.prepare_reduce("grads", self.PH32_ROWS, out_r,
                                                               offset_elems=W3_START + r * R * 1024)
        out_s, out_r = self._val_out
        self.xplane.run_split(self._roles["v_small"], self._roles["v_rows"])
        self.xplane.run_split(self._roles["gather"])
        torch.cuda.synchronize(self.device)
        mine = slice(W3_START + r * R * 1024, W3_START + (r + 1) * R * 1024)
        ok = bool(torch.allclose(out_s, ref_g[:W3_START], rtol=1e-5, atol=1e-5))
        ok &= bool(torch.allclose(out_r, ref_g[mine], rtol=1e-5, atol=1e-5))
        ok &= bool(torch.equal(p3, ref_p))
        try:
            self.xplane.check()
        except RuntimeError:
            ok = False
        from ..parallel.xgmi import _group_ok

        ok = _group_ok(ok, None, self.device)
        dist.barrier()  # every peer finished reading this rank's buffers before they are restored
        self.params.copy_(saved_p)
        self.grads.copy_(saved_g)
        torch.cuda.synchronize(self.device)
        return ok

    def _reduce_scatter_rows(self, full, out, R):
        """out = this rank's R rows of the sum over ranks of ``full`` (rows x 1024)."""
        import torch.distributed as dist

        if self.ncomm is not None:
            self.ncomm.reduce_scatter(out, full.view(self.world * R, -1))
        elif dist.get_backend() == "nccl":
            dist.reduce_scatter_tensor(out, full.view(self.world * R, -1))
        else:  # gloo has no reduce-scatter: allreduce in place, keep this rank's rows
            dist.all_reduce(full)
            rows = full.view(self.world * R, -1)[self.rank * R:(self.rank + 1) * R]
            if out.data_ptr() != rows.data_ptr():
                out.copy_(rows)

    def _launch_step_gather(self, x, rows, labels):
        """Step with the factor-gather data plane over the process group (RCCL; see ``__init__``).
        Collectives run one at a time on the side stream, each overlapping compute on main
        (sharded optimizer shown):

            main: conv12 | fc1_fwd head | fc1_bwd (small grads + dgrad), conv2_bwd, dW2 | dW3 rows, Adam rows |
            side:        AG(a2)        AG(dz)                                          AR(other grads)    AG(W3 rows) ->
                                                                                                next step's fc1_fwd
        The xGMI plane runs the same collectives co-launched in one stream (_launch_step_xgmi).
        """
        if self.use_xgmi:
            return self._launch_step_xgmi(x, rows, labels)
        o = self.ops
        st = self.state
        main = torch.cuda.current_stream(self.device)
        side = self._side
        self._conv_forward(x, rows, st)
        # (whole a2 rows: an all-to-all of only the column slice each rank needs cannot be captured,
        # torch's RCCL process group watchdog queries the captured event and aborts)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._all_gather_rows(self.a2_all, self.a2)
        if self._shadow_ev is not None:
            # the previous step's W3 row gather (side stream) must land before the first reader
            main.wait_event(self._shadow_ev)
            self._shadow_ev = None
        o.fc1_fwd(self.a2, self.w3_shadow(), self.zpart)
        o.head_fwd_bwd(self.zpart, self.pview("dense/bias"), self.pview("dense_1/kernel"), self.pview("dense_1/bias"),
                       labels, rows, st, self.seed, self.dropout, self.h, self.dz, self.dlog, self.stats,
                       stats_acc=self._stat_acc if self.track_stats else None)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._all_gather_rows(self.dz_all, self.dz)
        gW3 = self.gview("dense/kernel")
        small = (self.dz, self.a2, self.h, self.dlog, gW3, self.gview("dense/bias"), self.gview("dense_1/kernel"),
                 self.gview("dense_1/bias"))
        # db3, dW4, db4 of the local batch + the dgrad tiles, one launch
        o.fc1_bwd(self.dz, self.a2, self.h, self.dlog, self.w3_shadow(), *small[4:], self.g2, 2)
        self._conv_backward(x, rows, st)
        main.wait_stream(side)   # both gathers done: the communicator is free
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._allreduce(self.grads[:W3_START], 0, W3_START)
        ar_done = torch.cuda.Event()
        ar_done.record(side)
        b1, b2 = self.betas
        lo, hi = self._w3_tiles
        if self.shard_w3 and hi > lo:
            # dW3 summed over every rank's samples, Adam applied to W3 in the same tiles
            self._fc1_wgrad_w3_adam(1, self.dz_all, self.a2_all, lo, hi)
        elif hi > lo:
            # dW3 rows of this rank's tiles over every rank's samples, then Adam on those rows
            o.fc1_wgrad(*small, 1, self.dz_all, self.a2_all, lo, hi)
            a, b = W3_START + lo * 64 * 1024, W3_START + hi * 64 * 1024
            o.adam_step(self.params[a:b], self.grads[a:b], self.m[a:b], self.v[a:b],
                        self.shadow3[lo * 64:hi * 64].view(-1), st, 0, self.lr, b1, b2, self.eps, 1.0 / self.world,
                        self.rule, 0)
        if self.shard_w3:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                T64 = self._T * 64
                self._all_gather_rows(self.shadow3, self.shadow3[self.rank * T64:(self.rank + 1) * T64])
                self._shadow_ev = torch.cuda.Event()
                self._shadow_ev.record(side)
            self._full_state_valid = False
        main.wait_event(ar_done)
        o.adam_step(self.params[:W3_START], self.grads[:W3_START], self.m[:W3_START], self.v[:W3_START],
                    self.shadow[:W3_START], st, 0, self.lr, b1, b2, self.eps, 1.0 / self.world, self.rule, 1)

    # xGMI phase ids of the factor-gather plane (csrc/kernels/xgmi_role.h), in step order
    PH_W3, PH_DZ, PH_A2, PH_SMALL = 3, 1, 0, 2

    def _prepare_roles(self):
        """Descriptors of the plane's xGMI collectives (built once; they hold the buffers' pointers
        and the optimizer hyper-parameters, so a new learning rate prepares them again)."""
        xp, W, B = self.xplane, self.world, self.B
        b1, b2 = self.betas
        lo, hi = self._w3_mine
        h = slice(0, W3_START)
        T64 = self._T * 64
        r = {"lr": self.lr, "kind": "bf16"}
        # dz rows, in fc1_bwd's launch (a multiple of 8 blocks: its dgrad tiles keep their XCD map)
        r["dz"] = xp.prepare_gather("dz", self.PH_DZ, 1024 * 2, B, nblk=64)
        # a2 columns of this rank's W3 row tiles (sharded) / whole rows (627 KB per peer), in the
        # launch with the longest window, conv2_bwd, on the CUs its 225 blocks leave idle (one
        # 512-thread block per CU: 144 KB of LDS)
        nb = max(2, 256 - (B + 5 * ((B + 3) // 4)) - 1)
        r["a2_shard"] = xp.prepare_gather("a2", self.PH_A2, 3136 * 2, B, col_lo=lo * 128, col_hi=hi * 128, nblk=nb)
        r["a2_full"] = xp.prepare_gather("a2", self.PH_A2, 3136 * 2, B, nblk=nb)
        # small gradients: one-shot sum + their Adam update (1/size of Average = the Adam gradient
        # scale) + the forward step bump, in fc1_wgrad's launch: 32 blocks of that launch's 512- or
        # 1024-thread blocks, so with the 8-rank slice's 224 32-feature tiles every block of the
        # launch is resident at once (one per CU)
        r["small"] = xp.prepare_reduce("grads", self.PH_SMALL, self.gred, 1.0, nblk=32, adam=dict(
            p=self.params[h], m=self.m[h], v=self.v[h], shadow=self.shadow[h], state=self.state, lr=self.lr, b1=b1,
            b2=b2, eps=self.eps, grad_scale=1.0 / W, rule=self.rule))
        # the other ranks' updated W3 rows (sharded), in the next step's conv12_fwd launch, on the
        # CUs its 2 x B image blocks leave idle
        r["w3"] = xp.prepare_gather("shadow3", self.PH_W3, 1024 * 2, T64, total_rows=min(W * T64, 3136),
                                    nblk=max(2, (256 - 2 * B) // 2 * 2))
        # replicated optimizer: the same phase moving no bytes (a fence): fc1_bwd rewrites the small
        # gradients the peers summed in the last step's phase PH_SMALL, so a phase must separate them
        r["fence"] = xp.prepare_gather("shadow3", self.PH_W3, 1024 * 2, T64, total_rows=0, col_lo=0, col_hi=0, nblk=2)
        self._roles = r

    def _launch_step_xgmi(self, x, rows, labels):
        """Factor-gather step on the direct xGMI plane: ONE stream, every collective co-launched
        with a compute kernel (csrc/kernels/xgmi_role.h), seven launches:

            conv12_fwd [+ W3 rows of the other ranks (sharded)] | fc1_fwd | head |
            fc1_bwd dgrad + db3/dW4/db4 [+ dz] | conv2_bwd [+ a2 columns] | conv2_wgrad_reduce |
            dW3 tiles of this rank with Adam in the epilogue [+ small-gradient sum + their Adam]

        Each bracketed collective reads what the peers produced in earlier launches; the phase
        order (W3 rows, dz, a2, small) gives every buffer rewrite a later phase that proves the
        peers finished reading it (docs/ARCHITECTURE.md, "xGMI plane")."""
        o = self.ops
        st = self.state
        if self._roles is None or self._roles["lr"] != self.lr:
            self._prepare_roles()
        R = self._roles
        co = self.xplane.colaunch  # the role id for the op, or run split-form first (shared GPU)
        b1, b2 = self.betas
        w2 = self.pview("conv_layer2/conv2d/kernel", self.shadow)
        o.conv12_fwd(x, rows, st, self.pview("conv_layer1/conv2d/kernel", self.shadow),
                     self.pview("conv_layer1/conv2d/bias"), w2, self.pview("conv_layer2/conv2d/bias"), self.a1, self.idx1,
                     self.a2, self.idx2, co(R["w3"] if self.shard_w3 else R["fence"]))
        o.fc1_fwd(self.a2, self.w3_shadow(), self.zpart)
        o.head_fwd_bwd(self.zpart, self.pview("dense/bias"), self.pview("dense_1/kernel"), self.pview("dense_1/bias"),
                       labels, rows, st, self.seed, self.dropout, self.h, self.dz, self.dlog, self.stats,
                       stats_acc=self._stat_acc if self.track_stats else None)
        gW3 = self.gview("dense/kernel")
        small = (self.dz, self.a2, self.h, self.dlog, gW3, self.gview("dense/bias"), self.gview("dense_1/kernel"),
                 self.gview("dense_1/bias"))
        o.fc1_bwd(self.dz, self.a2, self.h, self.dlog, self.w3_shadow(), *small[4:], self.g2, 2, co(R["dz"]))
        self._conv_backward(x, rows, st, co(R["a2_shard"] if self.shard_w3 else R["a2_full"]))
        lo, hi = self._w3_tiles
        w3 = slice(W3_START, FLAT_NUMEL)
        o.fc1_wgrad_adam(*small, 1, self.dz_all, self.a2_all, self.params[w3], self.m[w3], self.v[w3],
                         self.shadow3[:3136].view(-1), st, self.lr, b1, b2, self.eps, 1.0 / self.world, self.rule,
                         self.keep_w3_grad, lo, hi, co(R["small"]))
        if self.shard_w3:
            self._full_state_valid = False

    def _fc1_wgrad_w3_adam(self, roles, dz_all, a2_all, lo=0, hi=49):
        b1, b2 = self.betas
        w3 = slice(W3_START, FLAT_NUMEL)
        self.ops.fc1_wgrad_adam(self.dz, self.a2, self.h, self.dlog, self.gview("dense/kernel"), self.gview("dense/bias"),
                                self.gview("dense_1/kernel"), self.gview("dense_1/bias"), roles, dz_all, a2_all,
                                self.params[w3], self.m[w3], self.v[w3], self.w3_shadow().reshape(-1), self.state,
                                self.lr, b1, b2, self.eps, 1.0 / self.world, self.rule, self.keep_w3_grad, lo, hi)

    def _conv_forward(self, x, rows, st):
        # one launch: conv1 on MFMA into conv2's LDS input image (a1/idx1 still stored for the backward)
        self.ops.conv12_fwd(x, rows, st, self.pview("conv_layer1/conv2d/kernel", self.shadow),
                            self.pview("conv_layer1/conv2d/bias"), self.pview("conv_layer2/conv2d/kernel", self.shadow),
                            self.pview("conv_layer2/conv2d/bias"), self.a1, self.idx1, self.a2, self.idx2)

    def _conv_backward(self, x, rows, st, coll=-1):
        o = self.ops
        o.conv2_bwd(self.g2, self.idx2, self.a1, self.pview("conv_layer2/conv2d/kernel", self.shadow), x, rows, st,
                    self.idx1, self.slab, self.cpart, None, coll)
        o.conv2_wgrad_reduce(self.slab, self.cpart, self.B, self.gview("conv_layer2/conv2d/kernel"),
                             self.gview("conv_layer1/conv2d/kernel"), self.gview("conv_layer1/conv2d/bias"),
                             self.gview("conv_layer2/conv2d/bias"))

    def _all_gather_rows(self, full, mine):
        import torch.distributed as dist

        if self.ncomm is not None:
            self.ncomm.all_gather_into(full, mine)
        elif dist.get_backend() == "nccl":
            dist.all_gather_into_tensor(full, mine)  # in place: `mine` is this rank's slice of `full`
        else:
            dist.all_gather(list(full.chunk(self.world)), mine.clone())

    def _join(self):
        """Make the current stream wait for any side-stream work of the last step (the step's
        results are then complete)."""
        if self._small_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(self._small_ev)
            self._small_ev = None
        if self._shadow_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(self._shadow_ev)
            self._shadow_ev = None

    def gather_full_state(self):
        """Sharded optimizer: collect every rank's dense/kernel rows of the fp32 weights and Adam
        slots, so variables()/to_model() see the complete state. Collective: call on every rank."""
        if not self.shard_w3 or self._full_state_valid:
            return
        self._join()
        if self.f32:  # the fp32 rows are gathered every step (the last update's here); the Adam slots
            self.flush_row_gather()
            R = self._f32_R
            for buf in (self.m, self.v):
                w3 = buf[W3_START:].view(3136, 1024)
                self._all_gather_rows(w3, w3[self.rank * R:(self.rank + 1) * R])
            self._full_state_valid = True
            return
        T64 = self._T * 64
        lo, hi = self._w3_tiles
        for buf in (self.params, self.m, self.v):
            w3 = buf[W3_START:].view(3136, 1024)
            tmp = torch.zeros(self.world * T64, 1024, device=self.device, dtype=torch.float32)
            mine = tmp[self.rank * T64:(self.rank + 1) * T64]
            mine[:(hi - lo) * 64].copy_(w3[lo * 64:hi * 64])
            self._all_gather_rows(tmp, mine)
            w3.copy_(tmp[:3136])
        # the bf16 rows too (on the xGMI plane the other ranks' rows of the last update arrive
        # with the next step's conv12_fwd launch): the same rounding of the same fp32 values
        self._refresh_shadow()
        self._full_state_valid = True

    def _gscale(self) -> float:
        """Adam's gradient scale on the replicated paths: 1/N of the allreduced sum (the average), 1
        for Adasum, whose exchange already yields the combined gradient."""
        from ..basics import ReduceOp

        if self.op is not None and ReduceOp(self.op) == ReduceOp.Adasum:
            return 1.0
        return 1.0 / self.world

    def _allreduce(self, bucket, lo, hi, comm=None):
        import torch.distributed as dist

        from ..basics import ReduceOp

        if self.op is not None and ReduceOp(self.op) == ReduceOp.Adasum:
            from ..parallel.collectives import adasum_dispatch_

            segs = [(o - lo, o - lo + n) for o, n in SEGMENTS.values() if lo <= o < hi]
            adasum_dispatch_(bucket, segs, comm=comm if comm is not None else self.ncomm)
            return  # (the combined gradient: its Adam takes grad_scale 1, _gscale)
        comm = comm if comm is not None else self.ncomm
        reduce_ = comm.all_reduce_ if comm is not None else dist.all_reduce
        if self.wire is not None:
            w = self.wire[lo:hi]
            self.ops.scale_cast_bf16(bucket, w, 1.0)
            reduce_(w)
            self.ops.bf16_to_f32(w, bucket, 1.0)
        else:
            reduce_(bucket)

    def train_step(self, x: torch.Tensor, y: torch.Tensor):
        """One eager step on a host-fed batch (x: [B,784] in [0,1], y: [B] labels)."""
        self.x_buf.copy_(x.reshape(self.B, 784), non_blocking=True)
        self.y_buf.copy_(y.reshape(self.B), non_blocking=True)
        # Host-fed batches index rows 0..B-1 of x_buf (rows=None); the step counter still advances.
        with trace_range("mihvd.fused_step"):
            self._launch_step(self.x_buf, None, self.y_buf)
            self._join()
        self.global_step += 1
        self._stat_steps += 1
        return {"loss": self.stats[:, 0].mean(), "accuracy": self.stats[:, 1].mean()}

    def device_step(self):
        """One eager step on the resident dataset."""
        if self.X is None:
            raise RuntimeError("call set_device_dataset() first")
        self._maybe_reshuffle(1)
        with trace_range("mihvd.fused_step"):
            self._launch_step(self.X, self.rows, self.Y)
            self._join()
        self._prepare_next_perm()
        self.global_step += 1
        self._stat_steps += 1
        return {"loss": self.stats[:, 0].mean(), "accuracy": self.stats[:, 1].mean()}

    def _maybe_reshuffle(self, k):
        if self.X is None:
            return
        e0 = self.global_step // self._epoch_steps
        e1 = (self.global_step + k - 1) // self._epoch_steps
        if e1 != e0 or (self.global_step % self._epoch_steps == 0 and self.global_step > 0):
            self._reshuffle()  # stream-ordered: no host synchronisation

    def set_lr(self, lr: float):
        """A new learning rate for the following steps. The kernels take it as a launch argument,
        so the captured graphs (and the xGMI plane's prepared collectives) are rebuilt on their next
        use; the same value is a no-op."""
        lr = float(lr)
        if lr == self.lr:
            return
        self._join()
        self.lr = lr
        self._graphs = {}
        self.graph = None
        self._graph_tried = False

    # ----------------------------------------------------------------------------- graphs
    def build_graph(self, steps_per_replay: int = 10, warmup: int = 2, primary: bool = True):
        """Capture ``steps_per_replay`` whole training steps (resident data) into one HIP graph.

        Warm-up steps run eagerly first (they also initialise RCCL communicators). If capture is not
        possible (e.g. Adasum's data-dependent exchanges), training stays eager. ``primary=False``
        keeps an additional graph of that length (``run_graph(steps)``) next to the main one, e.g.
        for the remainder of a step count that is not a multiple of the main graph's length."""
        if self.X is None:
            raise RuntimeError("call set_device_dataset() before build_graph()")
        for _ in range(warmup):
            self.device_step()
        torch.cuda.synchronize(self.device)
        if primary:
            self.steps_per_replay = steps_per_replay
        if (self._adasum_host() or self.debug_sync or self._host_collectives()):
            # Adasum over the process group / serialized mode / gloo collectives (host-side, not
            # capturable): eager
            if primary:
                self.graph = None
            return False
        if self.f32:
            self._prime_batch()  # eagerly: the captured steps start from a gathered batch
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        try:
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for _ in range(steps_per_replay):
                        self._launch_step(self.X, self.rows, self.Y)
                    self._join()
        except Exception as e:  # pragma: no cover - depends on the RCCL build
            import warnings

            warnings.warn(f"HIP graph capture failed ({e!r}); falling back to eager steps")
            if primary:
                self.graph = None
            self._small_ev = self._shadow_ev = None
            torch.cuda.synchronize(self.device)
            return False
        torch.cuda.current_stream(self.device).wait_stream(s)
        # Capture does not execute: the device step counter is untouched, so replays continue
        # from the current global_step.
        _upload_graph(g, torch.cuda.current_stream(self.device))
        self._graphs[steps_per_replay] = g
        if primary:
            self.graph = g
        return True

    def _adasum_host(self) -> bool:
        """Adasum whose exchanges run over the process group (no framework communicator, or ranks
        on several nodes: the cross-node part): not capturable. On the framework-owned RCCL
        communicator of a one-node world every exchange is an RCCL call on the stream."""
        if self.op is None or int(self.op) != 2:
            return False
        from .. import basics

        one_node = not basics.is_initialized() or basics._ctx.topology.cross_size == 1
        return self.ncomm is None or not one_node

    def _host_collectives(self) -> bool:
        if not self.collectives:
            return False
        import torch.distributed as dist

        return dist.is_initialized() and dist.get_backend() != "nccl"

    def run_graph(self, steps: int | None = None):
        """Advance ``steps_per_replay`` steps (or ``steps``, for which a graph was built with
        ``primary=False``) by one graph replay, or eagerly if capture failed."""
        k = self.steps_per_replay if steps is None else int(steps)
        g = self.graph if steps is None else self._graphs.get(k)
        if g is None:
            for _ in range(k):
                self.device_step()
            return
        self._maybe_reshuffle(k)
        if self.f32:
            self._prime_batch()  # (a reshuffle or a host-side change broke the chain: re-gather)
        with trace_range(f"mihvd.graph_replay[{k} steps]"):
            g.replay()
        self._prepare_next_perm()  # (host work while the replay runs)
        if self.f32 and self.collectives and self.shard_w3 and self.use_xgmi:
            self._f32_gather_pending = True  # the replay's last update: gathered by the next conv1
        self.global_step += k
        self._stat_steps += k

    def run_steps(self, k: int, steps_per_replay: int = 10) -> int:
        """Advance exactly ``k`` steps on the resident dataset, graph-replayed: the first call
        captures a graph of ``steps_per_replay`` steps (after one eager warm-up step, which counts),
        whole replays follow, and a remainder replays a graph of that length (captured once).
        Falls back to eager steps where capture is impossible. Returns the steps advanced."""
        k = int(k)
        done = 0
        if k <= 0:
            return 0
        if self.graph is None and not getattr(self, "_graph_tried", False):
            self._graph_tried = True
            self.build_graph(steps_per_replay=steps_per_replay, warmup=1)  # the warm-up step counts
            done += 1
        spr = self.steps_per_replay
        while self.graph is not None and k - done >= spr:
            self.run_graph()
            done += spr
        r = k - done
        if r > 0:
            if self.graph is not None:
                if r not in self._graphs:
                    self.build_graph(steps_per_replay=r, warmup=0, primary=False)
                self.run_graph(r)
            else:
                for _ in range(r):
                    self.device_step()
            done += r
        return done

    def loss_tensor(self) -> torch.Tensor:
        """The last step's mean loss as a device scalar (reading it synchronises)."""
        return self.stats[:, 0].mean()

    def last_loss(self) -> float:
        self.check_xgmi()
        return float(self.stats[:, 0].mean())

    def last_accuracy(self) -> float:
        self.check_xgmi()
        return float(self.stats[:, 1].mean())

    # ----------------------------------------------------------------------------- xGMI plane
    def check_xgmi(self):
        """Raise if a direct-xGMI collective of this trainer timed out waiting for a peer (its
        outputs, and those of every later xGMI collective, are NaN). Waits for the current stream.
        A plane that select_data_plane() dropped after such a timeout is not checked again."""
        if not self.f32 and self.fused_opt and int(self.ops.conv_barrier_error(True)) != 0:
            raise RuntimeError("fused step: a conv2_bwd LDS barrier timed out (a broken wave count); the conv "
                               "gradients and optimizer state of that step are invalid")
        if self.xplane is not None and not getattr(self, "_xplane_failed", False):
            self.xplane.check()

    def _validate_xgmi(self, rounds: int = 2) -> bool:
        """Run the plane's prepared xGMI collectives (the descriptors the step co-launches, here
        launched on their own; the small-gradient sum without its Adam update) on random data and
        compare them with the same collectives over the process group: gathers bitwise, the sum to
        fp32 rounding. Collective. Clobbers a2 and dz (every step recomputes them); the gradients
        and the W3 row shadow are restored."""
        import torch.distributed as dist

        if self._roles is None or self._roles["lr"] != self.lr:
            self._prepare_roles()
        R = self._roles
        W, B, r = self.world, self.B, self.rank
        T64 = self._T * 64
        ok = True
        g = torch.Generator(device="cpu").manual_seed(9173 + r)
        saved_shadow3 = self.shadow3.clone()
        saved_grads = self.grads[:W3_START].clone()  # (the alignment gaps are never rewritten by a step)
        others = [q for q in range(W) if q != r]
        for it in range(rounds):
            shard = it % 2 == 0  # both a2 descriptors: this rank's columns, whole rows
            lo, hi = self._w3_mine if shard else (0, 49)
            cols = slice(lo * 64, hi * 64)
            self.a2.copy_(torch.randn(B, 3136, generator=g).to(torch.bfloat16))
            self.dz.copy_(torch.randn(B, 1024, generator=g).to(torch.bfloat16))
            self.grads[:W3_START].copy_(torch.randn(W3_START, generator=g))
            mine = self.shadow3[r * T64:(r + 1) * T64]
            mine.copy_(torch.randn(T64, 1024, generator=g).to(torch.bfloat16))
            ref_a2 = self.a2_all.clone()
            ref_dz = self.dz_all.clone()
            ref_s = self.shadow3.clone()
            self._all_gather_rows(ref_a2, ref_a2[r * B:(r + 1) * B])
            self._all_gather_rows(ref_dz, ref_dz[r * B:(r + 1) * B])
            self._all_gather_rows(ref_s, ref_s[r * T64:(r + 1) * T64])
            ref_g = self.grads[:W3_START].clone()
            dist.all_reduce(ref_g)
            torch.cuda.synchronize(self.device)
            self.xplane.run(R["w3"])
            self.xplane.run(R["a2_shard"] if shard else R["a2_full"])
            self.xplane.run(R["dz"])
            self.xplane.reduce("grads", self.PH_SMALL, self.gred)
            torch.cuda.synchronize(self.device)
            for q in others:
                rws = slice(q * B, (q + 1) * B)
                ok &= torch.equal(self.a2_all[rws, cols], ref_a2[rws, cols])
                ok &= torch.equal(self.dz_all[rws], ref_dz[rws])
                srows = slice(q * T64, min((q + 1) * T64, 3136))
                ok &= torch.equal(self.shadow3[srows], ref_s[srows])
            ok &= bool(torch.allclose(self.gred, ref_g, rtol=1e-5, atol=1e-5))
        try:
            self.xplane.check()
        except RuntimeError:
            ok = False
        from ..parallel.xgmi import _group_ok

        ok = _group_ok(ok, None, self.device)
        # every peer finished reading this rank's buffers before they are restored
        dist.barrier()
        self.shadow3.copy_(saved_shadow3)
        self.grads[:W3_START].copy_(saved_grads)
        return ok

    def _set_plane(self, xgmi: bool, shard: bool, factor: bool = False):
        """Switch data plane and sharding between steps (collective). Leaving the sharded xGMI
        plane, whose row gather of the last update would run in the next conv12_fwd launch,
        gathers the rows now. ``factor``: the fp32 factor-gather plane (sharded only)."""
        self._join()
        if self.use_xgmi and self.shard_w3 and self.f32:
            self.flush_row_gather()  # (collective: every rank switches planes together)
        if self.use_xgmi and self.shard_w3 and not self.f32 and not (xgmi and shard):
            torch.cuda.synchronize(self.device)
            T64 = self._T * 64
            self._all_gather_rows(self.shadow3, self.shadow3[self.rank * T64:(self.rank + 1) * T64])
            torch.cuda.synchronize(self.device)
        self.use_xgmi = bool(xgmi) and self.xplane is not None and not getattr(self, "_xplane_failed", False)
        self.set_sharding(shard)
        self.f32_factor = bool(factor) and self.f32 and self.shard_w3
        self.f32_factor_rep = bool(factor) and self.f32 and not self.shard_w3 and getattr(self, "_f32_can_factor", False)
        self._bind_factor_views()
        self._graphs = {}
        self.graph = None

    def set_sharding(self, shard: bool):
        """Switch the dense/kernel optimizer between sharded and replicated (factor-gather plane;
        collective). Sharded -> replicated first collects every rank's fp32 rows and Adam slots."""
        if self.f32:
            shard = bool(shard) and self._f32_can_shard
        else:
            shard = bool(shard) and self.gather
        if shard == self.shard_w3:
            return
        self._join()
        if not shard:
            self.gather_full_state()
            self._refresh_shadow()
        self.shard_w3 = shard
        self.f32_factor = self.f32_factor and shard
        self.f32_factor_rep = getattr(self, "f32_factor_rep", False) and not shard
        self._bind_factor_views()
        self._graphs = {}
        self.graph = None

    def select_data_plane(self, steps: int = 40, steps_per_replay: int = 20, shard_options=None) -> dict:
        """Pick the data plane of the factor gather (MIHVD_XGMI=auto) and whether the dense/kernel
        optimizer is sharded: validate the direct xGMI collectives against the process group's,
        then time ``steps`` training steps of each candidate (graph-replayed when capturable) and
        keep the fastest. Collective; the decision is the same on every rank (max time over
        ranks). Runs real training steps. ``shard_options``: the sharding settings to try (default:
        MIHVD_SHARD_W3 if set, else both). Returns a report."""
        import time

        import torch.distributed as dist

        rep = {"mode": self._xgmi_mode, "available": self.xplane is not None}
        if self.f32 and self._f32_can_shard and shard_options is None:
            # fp32 over RCCL: dW3 bucket allreduce + every rank's full Adam, or reduce-scatter +
            # sharded Adam + row all-gather; timed like the factor-gather planes below
            env = os.environ.get("MIHVD_SHARD_W3")
            shard_options = [env != "0"] if env is not None else [True, False]
        elif not self.gather:
            rep["plane"] = "rccl" if self.collectives else "none"
            return rep
        if shard_options is None:
            env = os.environ.get("MIHVD_SHARD_W3")
            # (one rank owns every tile either way: replicated, which has no row gather)
            shard_options = [env != "0"] if env is not None else ([True, False] if self.world > 1 else [False])
        shard_options = [bool(x) for x in shard_options]
        planes = ["rccl"]
        if self.xplane is not None and self._xgmi_mode != "off":
            self.xplane.watch(False)  # a timeout while the plane is on trial means "use RCCL"
            valid = self._validate_xgmi_f32() if self.f32 else self._validate_xgmi()
            rep["valid"] = valid
            if valid:
                planes = ["xgmi"] if self._xgmi_mode == "on" else ["xgmi", "rccl"]
            else:
                from ..parallel.xgmi import warn_fallback

                warn_fallback("validation against the process group's collectives failed")
        cands = [(p, sh) for p in planes for sh in dict.fromkeys(shard_options)]
        if self.f32:  # the fp32 xGMI plane exists in the sharded form only
            cands = [c for c in cands if not (c[0] == "xgmi" and not c[1])]
        if self.f32 and self._f32_can_shard and True in shard_options:
            # the fp32 factor-gather plane (sharded): MIHVD_F32_PLANE=auto (default) times it beside
            # the reduce-scatter plane, "factor" uses it alone, "rs" leaves it out
            fmode = f32_plane_mode()
            if fmode == "factor":
                cands = [("factor", True)]
            elif fmode != "rs" and fmode != "factor_rep":
                cands.append(("factor", True))
        if self.f32 and getattr(self, "_f32_can_factor", False) and False in shard_options:
            # the replicated fp32 factor-gather plane (every row's dW3 from the gathered factors)
            fmode = f32_plane_mode()
            if fmode == "factor_rep":
                cands = [("factor", False)]
            elif fmode == "auto":
                cands.append(("factor", False))
        host = self._host_collectives()
        # host (gloo) collectives cannot be captured or timed meaningfully: the candidates still run
        # (eagerly) for the consistency check below, and the first consistent candidate is kept
        if len(cands) == 1:
            self._set_plane(cands[0][0] == "xgmi", cands[0][1], cands[0][0] == "factor")
            rep["plane"], rep["shard"] = cands[0]
            self._watch_plane()
            return rep
        times = {}
        finals = {}
        k = max(1, min(steps_per_replay, steps))
        # the timed candidates run real training steps: the model, optimizer, step state and data
        # order are restored before each candidate and afterwards, so every candidate trains the
        # same steps on the same batches and selection leaves no trace (nor NaN from a poisoned
        # collective)
        snap = self._snapshot()
        for plane, sh in cands:
            self._set_plane(plane == "xgmi", sh, plane == "factor")
            self._restore(snap)
            captured = self.build_graph(steps_per_replay=k, warmup=1)
            torch.cuda.synchronize(self.device)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(max(1, steps // k)):
                self.run_graph()
            torch.cuda.synchronize(self.device)
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=self.device)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            times[(plane, sh)] = float(el.item()) / (max(1, steps // k) * k) * 1e6
            rep["captured"] = captured
            self.gather_full_state()
            finals[(plane, sh)] = self.params.clone()
        # End-to-end check of the xGMI plane's cross-GPU visibility (xgmi_role.h): the graph-replayed
        # steps of every xGMI candidate must land where RCCL's steps with the same sharding landed,
        # from the same snapshot on the same batches — to fp32 summation-order differences (the
        # one-shot sum adds ranks in rank order, RCCL's ring in ring order). A stale peer read
        # (a gather that saw the previous step's rows) moves the result by the size of a whole
        # gradient term; on any mismatch, on any rank, every rank drops the plane.
        cons = {}
        fcons = None
        for (plane, sh), fin in finals.items():
            ref = finals.get(("rccl", sh))
            if plane == "rccl" or ref is None:
                continue
            upd = (ref - snap["params"]).norm().item()
            d = (fin - ref).norm().item() / max(upd, 1e-30)
            d = d if math.isfinite(d) else float("inf")
            if plane == "factor":
                fcons = max(d, fcons or 0.0)  # the fp32 factor planes: same exact sums in another order
            else:
                cons[f"xgmi-{'shard' if sh else 'replicated'}"] = d
        if fcons is not None:
            from ..parallel.xgmi import _group_ok

            ok = _group_ok(fcons <= _check_tol(), None, self.device)
            rep["factor_consistency"] = round(fcons, 9)
            if not ok:
                import warnings

                warnings.warn("fp32 factor-gather steps disagree with the reduce-scatter plane's; not used")
                times = {key: t for key, t in times.items() if key[0] != "factor"}
        if cons:
            from ..parallel.xgmi import _group_ok, warn_fallback

            tol = _check_tol()
            ok = _group_ok(all(v <= tol for v in cons.values()), None, self.device)
            rep["consistency"] = {key: round(v, 9) for key, v in cons.items()}
            rep["consistent"] = ok
            if not ok:
                times = {key: t for key, t in times.items() if key[0] != "xgmi"}
                self._xplane_failed = True
                warn_fallback("graph-replayed steps on the xGMI plane disagree with RCCL's from the same snapshot")
        if any(p == "xgmi" for p, _ in cands):
            # a device-side phase barrier that timed out (a peer that never arrived) poisoned its
            # outputs: every rank then drops the plane for good and keeps RCCL
            from ..parallel.xgmi import _group_ok, warn_fallback
            err = int(self.ops.xgmi_error(self.xplane.ctx)) if self.xplane is not None else 1
            if not _group_ok(err == 0, None, self.device):
                times = {key: t for key, t in times.items() if key[0] != "xgmi"}
                self._xplane_failed = True
                rep["timing_error"] = True
                warn_fallback("a collective timed out while the plane was timed")
                if not times:  # pragma: no cover - 'on' mode: nothing else was timed
                    times = {("rccl", cands[0][1]): float("nan")}
        if host:
            plane, sh = next(c for c in cands if c in times)
        else:
            plane, sh = min(times, key=lambda key: (times[key] != times[key], times[key]))
        self._set_plane(plane == "xgmi", sh, plane == "factor")
        self._restore(snap)
        rep["us_per_step"] = {f"{p}{'-shard' if s else '-replicated'}": round(t, 2) for (p, s), t in times.items()}
        rep["plane"], rep["shard"] = plane, sh
        self._watch_plane()
        return rep

    def _watch_plane(self):
        """Arm (or disarm) the health monitor's watch of the xGMI timeout word for the chosen plane."""
        if self.xplane is not None:
            self.xplane.watch(self.use_xgmi)

    def _snapshot(self) -> dict:
        """Device copies of everything a training step changes (weights, Adam slots, step state)."""
        import copy

        self._join()
        self.gather_full_state()
        snap = {"params": self.params.clone(), "m": self.m.clone(), "v": self.v.clone(), "state": self.state.clone(),
                "global_step": self.global_step}
        if self.rows is not None:  # the resident dataset's current epoch order and its RNG
            torch.cuda.synchronize(self.device)
            snap["rows"] = self.rows.clone()
            # (the state before a prepared next order was drawn: the restored run draws it again)
            pre = self._rng_pre if getattr(self, "_next_perm", None) is not None else self._rng.bit_generator.state
            snap["rng"] = copy.deepcopy(pre)
        return snap

    def _restore(self, snap: dict):
        """Back to a _snapshot() (collective when the dense/kernel optimizer is sharded)."""
        self._join()
        torch.cuda.synchronize(self.device)
        for name in ("params", "m", "v", "state"):
            getattr(self, name).copy_(snap[name])
        if "rows" in snap and self.rows is not None:
            self.rows.copy_(snap["rows"])
            self._rng.bit_generator.state = snap["rng"]
            self._next_perm = None
        self.global_step = snap["global_step"]
        self._xpre_valid = False
        self._full_state_valid = True
        self._f32_gather_pending = False  # every rank's rows are the snapshot's
        self._refresh_shadow()  # (and the full W3 row shadow of the factor-gather plane)
        torch.cuda.synchronize(self.device)

    def reduced_grads(self) -> torch.Tensor:
        """The flat gradient buffer after the step's reduction (sums over ranks; the xGMI plane
        reduces the small gradients into a separate buffer instead of in place). On the
        factor-gather plane (both the xGMI and the RCCL form compute dW3 + Adam in one tile
        epilogue) the dense/kernel segment is written only with
        keep_w3_grad=True, and then only for the rows whose optimizer this rank owns; otherwise it
        holds stale values."""
        if self.use_xgmi and self.gather:
            return torch.cat([self.gred, self.grads[W3_START:]])
        if self.f32 and self.shard_w3:
            # the reduce-scatter plane leaves this rank's reduced dense/kernel rows in place in the
            # gradient buffer, the factor and xGMI planes in gshard (keep_w3_grad); the xGMI plane's
            # small-gradient sums are in gred32 (keep_w3_grad)
            g = self.grads.clone()
            if self.use_xgmi and getattr(self, "gred32", None) is not None:
                g[:W3_START] = self.gred32
            if self.f32_factor or self.use_xgmi:
                R = self._f32_R
                g[W3_START + self.rank * R * 1024:W3_START + (self.rank + 1) * R * 1024] = self.gshard.view(-1)
            return g
        return self.grads

    def data_plane(self) -> str:
        if not self.collectives:
            return "none"
        if self.gather:
            return "xgmi" if self.use_xgmi else "rccl"
        if self.f32 and self.f32_factor:
            return "factor"
        if self.f32 and getattr(self, "f32_factor_rep", False):
            return "factor_rep"
        if self.f32 and self.use_xgmi and self.shard_w3:
            return "xgmi"
        return "rccl"

    def close(self):
        """Release the direct-xGMI regions (collective when they exist: peers may still read this
        rank's region, so every rank synchronises and meets at a barrier first). The trainer is
        unusable afterwards."""
        if self._closed:
            return
        self._closed = True
        for c in (self.ncomm, self.ncomm_small):
            if c is not None:
                c.close()
        self.ncomm = self.ncomm_small = None
        if self.xplane is None:
            return
        import torch.distributed as dist

        if self.f32 and self.use_xgmi and self.shard_w3 and not getattr(self, "_xplane_failed", False):
            self.flush_row_gather()  # every rank's rows complete before the region goes away
        torch.cuda.synchronize(self.device)
        self.graph = None
        self._graphs = {}
        if dist.is_initialized():
            dist.barrier()
        if self.xplane is not None:
            if self.f32:  # the parameters and gradients lived in the region: keep readable copies
                self.params = self.params.clone()
                self.grads = self.grads.clone()
            else:
                for name in ("a2_all", "dz_all", "a2", "dz", "grads", "shadow3"):
                    if hasattr(self, name):
                        setattr(self, name, None)
            self.xplane.close()
            self.xplane = None
            self.use_xgmi = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ----------------------------------------------------------------------------- state
    def sync(self):
        self._join()
        torch.cuda.synchronize(self.device)
        self.check_xgmi()

    def variables(self) -> dict[str, torch.Tensor]:
        """TF1 global variables (names of tensorflow_mnist.py's graph) for the checkpoint layout."""
        self._require_full_state()
        self.sync()
        out = {}
        for name in TF_PARAM_ORDER:
            out[name] = self.pview(name).detach().clone()
            out[name + "/Adam"] = self.pview(name, self.m).detach().clone()
            out[name + "/Adam_1"] = self.pview(name, self.v).detach().clone()
        t = int(self.state[1].item())
        b1, b2 = self.betas
        out["beta1_power"] = torch.tensor(b1 ** (t + 1), dtype=torch.float32)
        out["beta2_power"] = torch.tensor(b2 ** (t + 1), dtype=torch.float32)
        out["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return out

    def load_variables(self, variables: dict[str, torch.Tensor]):
        with torch.no_grad():
            for name in TF_PARAM_ORDER:
                self.pview(name).copy_(variables[name].to(self.device))
                if name + "/Adam" in variables:
                    self.pview(name, self.m).copy_(variables[name + "/Adam"].to(self.device))
                    self.pview(name, self.v).copy_(variables[name + "/Adam_1"].to(self.device))
        self.global_step = int(variables.get("global_step", torch.tensor(0)))
        t = self.global_step
        if "beta1_power" in variables:
            bp = float(variables["beta1_power"])
            if 0 < bp < 1:
                t = round(math.log(bp) / math.log(self.betas[0])) - 1
        self.state.copy_(torch.tensor([self.global_step, t, 0, 0], dtype=torch.int64))
        self._xpre_valid = False
        self._refresh_shadow()
        self._full_state_valid = True

    def broadcast(self, root_rank: int = 0):
        """Broadcast weights, Adam slots and counters from ``root_rank`` (BroadcastGlobalVariablesHook)."""
        from .. import basics

        if not basics.is_initialized() or basics.size() == 1:
            return
        import torch.distributed as dist

        self._join()
        self.gather_full_state()  # collective; no-op unless the dense/kernel optimizer is sharded
        for buf in (self.params, self.m, self.v, self.state):  # (~39 MB: weights + Adam slots + counters)
            if self.ncomm is not None:  # the framework-owned communicator, on the current stream
                self.ncomm.broadcast_(buf, root_rank)
            else:
                dist.broadcast(buf, src=root_rank)
        from ..parallel.collectives import broadcast_object

        self.global_step = int(broadcast_object(self.global_step, root_rank))
        self._xpre_valid = False
        self._refresh_shadow()
