#!/usr/bin/env python3
"""Per-kernel microbenchmark of the fused MNIST step (no profiler): each op is replayed N times
back to back inside a HIP graph and timed with events, so launch overhead is excluded and the
number is the kernel's own duration. Usage: python scripts/kbench.py [--iters 200] [--batch 100]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--json", default="")
    ap.add_argument("--roles", action="store_true", help="also time each block role of multi-role launches")
    ap.add_argument("--phases", action="store_true", help="time conv2_bwd's dgrad role cut after each phase")
    ap.add_argument("--only", default="", help="';'-separated job names (e.g. 'conv2_bwd[role0]'); skips the step")
    args = ap.parse_args()
    from mihvd.models.fused_mnist import FC_START as FC, W3_START as W3, FusedMNISTTrainer

    B = args.batch
    tr = FusedMNISTTrainer(batch_size=B, seed=0, device="cuda", precision="bf16")
    x = torch.rand(B, 784, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    tr.train_step(x, y)
    torch.cuda.synchronize()
    o = tr.ops
    st = tr.state
    sh = tr.shadow
    TS = tr.tail_split  # dense/kernel rows below it: updated in the reduce launch
    dz8 = tr.dz.repeat(8, 1).contiguous()
    a2T = torch.zeros(3136, 128, device="cuda", dtype=torch.bfloat16)
    dzT = torch.zeros(1024, 128, device="cuda", dtype=torch.bfloat16)
    a2T[:, :B].copy_(tr.a2.t())
    dzT[:, :B].copy_(tr.dz.t())
    a28 = tr.a2.repeat(8, 1).contiguous()
    ops = {
        "conv1_fwd": lambda: o.conv1_fwd(tr.x_buf, None, st, tr.pview("conv_layer1/conv2d/kernel"),
                                         tr.pview("conv_layer1/conv2d/bias"), tr.a1, tr.idx1),
        "conv2_fwd": lambda: o.conv2_fwd(tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh),
                                         tr.pview("conv_layer2/conv2d/bias"), tr.a2, tr.idx2),
        "conv12_fwd": lambda: o.conv12_fwd(tr.x_buf, None, st, tr.pview("conv_layer1/conv2d/kernel", sh),
                                           tr.pview("conv_layer1/conv2d/bias"),
                                           tr.pview("conv_layer2/conv2d/kernel", sh),
                                           tr.pview("conv_layer2/conv2d/bias"), tr.a1, tr.idx1, tr.a2, tr.idx2),
        "fc1_fwd": lambda: o.fc1_fwd(tr.a2, tr.pview("dense/kernel", sh), tr.zpart),
        "head": lambda: o.head_fwd_bwd(tr.zpart, tr.pview("dense/bias"), tr.pview("dense_1/kernel"),
                                       tr.pview("dense_1/bias"), tr.y_buf, None, st, tr.seed, 0.5, tr.h, tr.dz, tr.dlog,
                                       tr.stats),
        "fc1_wgrad": lambda: o.fc1_wgrad(tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"),
                                         tr.gview("dense_1/kernel"), tr.gview("dense_1/bias")),
        "fc1_dgrad": lambda: o.fc1_dgrad(tr.dz, tr.pview("dense/kernel", sh), tr.a2, tr.g2),
        "fc1_bwd": lambda: o.fc1_bwd(tr.dz, tr.a2, tr.h, tr.dlog, tr.pview("dense/kernel", sh), tr.gview("dense/kernel"),
                                     tr.gview("dense/bias"), tr.gview("dense_1/kernel"), tr.gview("dense_1/bias"), tr.g2),
        "conv2_bwd": lambda: o.conv2_bwd(tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh), tr.x_buf,
                                         None, st, tr.idx1, tr.slab, tr.cpart),
        "conv2_wgrad_reduce": lambda: o.conv2_wgrad_reduce(tr.slab, tr.cpart, B, tr.gview("conv_layer2/conv2d/kernel"),
                                                           tr.gview("conv_layer1/conv2d/kernel"),
                                                           tr.gview("conv_layer1/conv2d/bias"),
                                                           tr.gview("conv_layer2/conv2d/bias")),
        "fc1_wgrad_adam": lambda: o.fc1_wgrad_adam(
            tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
            tr.gview("dense_1/bias"), 3, None, None, tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], st, 0.0, 0.9,
            0.999, 1e-8, 1.0, 0, False),
        # dW3 over the all-gathered factors of 8 ranks (the N=8 factor-gather data plane, Kw = 800)
        "fc1_wgrad_k8x": lambda: o.fc1_wgrad(tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"),
                                             tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
                                             tr.gview("dense_1/bias"), 1, dz8, a28),
        # the fused optimizer pair (the reduce re-arms the tail counter, so it is timed as a pair)
        # the trainer's split of dense/kernel between the reduce launch and conv2_bwd's streamers
        "conv2_bwd_adam+reduce_adam": lambda: (o.conv2_bwd_adam(
            tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh), tr.x_buf, None, st, tr.idx1, tr.slab,
            tr.cpart, tr.params[TS:], tr.grads[TS:], tr.m[TS:], tr.v[TS:], sh[TS:], 0.0, 0.9, 0.999, 1e-8, 1.0, 0),
            o.conv2_wgrad_reduce_adam(
            tr.slab, tr.cpart, B, tr.gview("conv_layer2/conv2d/kernel"), tr.gview("conv_layer1/conv2d/kernel"),
            tr.gview("conv_layer1/conv2d/bias"), tr.gview("conv_layer2/conv2d/bias"), tr.grads, tr.params, tr.m, tr.v,
            sh, st, FC, TS, 0.0, 0.9, 0.999, 1e-8, 1.0, 0)),
        "conv2_bwd_adam_fold": lambda: o.conv2_bwd_adam_fold(
            tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh), tr.x_buf, None, st, tr.idx1, tr.slab,
            tr.cpart, tr.gview("conv_layer2/conv2d/kernel"), tr.gview("conv_layer1/conv2d/kernel"),
            tr.gview("conv_layer1/conv2d/bias"), tr.gview("conv_layer2/conv2d/bias"), tr.grads, tr.params, tr.m, tr.v,
            sh, tr.fold_sync, FC, W3, 0.0, 0.9, 0.999, 1e-8, 1.0, 0),
        "conv2_bwd_adam": lambda: o.conv2_bwd_adam(
            tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh), tr.x_buf, None, st, tr.idx1, tr.slab,
            tr.cpart, tr.params[TS:], tr.grads[TS:], tr.m[TS:], tr.v[TS:], sh[TS:], 0.0, 0.9, 0.999, 1e-8, 1.0, 0),
        "reduce_adam": lambda: o.conv2_wgrad_reduce_adam(
            tr.slab, tr.cpart, B, tr.gview("conv_layer2/conv2d/kernel"), tr.gview("conv_layer1/conv2d/kernel"),
            tr.gview("conv_layer1/conv2d/bias"), tr.gview("conv_layer2/conv2d/bias"), tr.grads, tr.params, tr.m, tr.v,
            sh, st, FC, TS, 0.0, 0.9, 0.999, 1e-8, 1.0, 0),
        "fc1_bwd[roles=2]": lambda: o.fc1_bwd(tr.dz, tr.a2, tr.h, tr.dlog, tr.pview("dense/kernel", sh),
                                              tr.gview("dense/kernel"), tr.gview("dense/bias"),
                                              tr.gview("dense_1/kernel"), tr.gview("dense_1/bias"), tr.g2, 2, -1,
                                              a2T, dzT),
        "conv2_bwd_w3adam+reduce_adam": lambda: (o.conv2_bwd_w3adam(
            tr.g2, tr.idx2, tr.a1, tr.pview("conv_layer2/conv2d/kernel", sh), tr.x_buf, None, st, tr.idx1, tr.slab,
            tr.cpart, dzT, a2T, tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], None, 0.0, 0.9, 0.999, 1e-8, 1.0,
            0), o.conv2_wgrad_reduce_adam(
            tr.slab, tr.cpart, B, tr.gview("conv_layer2/conv2d/kernel"), tr.gview("conv_layer1/conv2d/kernel"),
            tr.gview("conv_layer1/conv2d/bias"), tr.gview("conv_layer2/conv2d/bias"), tr.grads, tr.params, tr.m, tr.v,
            sh, st, FC, W3, 0.0, 0.9, 0.999, 1e-8, 1.0, 0)),
        "fc1_wgrad_adam_k8x": lambda: o.fc1_wgrad_adam(
            tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
            tr.gview("dense_1/bias"), 1, dz8, a28, tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], st, 0.0, 0.9,
            0.999, 1e-8, 1.0, 0, False),
        # the sharded optimizer at N=8: this rank's 7 of 49 row tiles of dW3 (K = 800), Adam on them
        "fc1_wgrad_k8x_slice": lambda: o.fc1_wgrad(tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"),
                                                   tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
                                                   tr.gview("dense_1/bias"), 1, dz8, a28, 0, 7),
        # the sharded xGMI plane's last launch at N=8: dW3 of this rank's 7 row tiles over all ranks'
        # samples (K = 800) with Adam fused into the tiles
        "fc1_wgrad_adam_k8x_slice": lambda: o.fc1_wgrad_adam(
            tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
            tr.gview("dense_1/bias"), 1, dz8, a28, tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], st, 0.0, 0.9,
            0.999, 1e-8, 1.0, 0, False, 0, 7),
        # the sharded xGMI plane's last launch at N=2 / N=4 (K = 200 / 400; 25 / 13 row tiles)
        "fc1_wgrad_adam_k2x_slice": lambda: o.fc1_wgrad_adam(
            tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
            tr.gview("dense_1/bias"), 1, dz8[:2 * B], a28[:2 * B], tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:],
            st, 0.0, 0.9, 0.999, 1e-8, 1.0, 0, False, 0, 25),
        "fc1_wgrad_adam_k4x_slice": lambda: o.fc1_wgrad_adam(
            tr.dz, tr.a2, tr.h, tr.dlog, tr.gview("dense/kernel"), tr.gview("dense/bias"), tr.gview("dense_1/kernel"),
            tr.gview("dense_1/bias"), 1, dz8[:4 * B], a28[:4 * B], tr.params[W3:], tr.m[W3:], tr.v[W3:], sh[W3:],
            st, 0.0, 0.9, 0.999, 1e-8, 1.0, 0, False, 0, 13),
        "adam_w3_slice8": lambda: o.adam_step(tr.params[W3:W3 + 7 * 65536], tr.grads[W3:W3 + 7 * 65536],
                                              tr.m[W3:W3 + 7 * 65536], tr.v[W3:W3 + 7 * 65536],
                                              sh[W3:W3 + 7 * 65536], st, 0, 0.0, 0.9, 0.999, 1e-8, 1.0, 0, 0),
        "adam_w3": lambda: o.adam_step(tr.params[W3:], tr.grads[W3:], tr.m[W3:], tr.v[W3:], sh[W3:], st, 0, 0.0,
                                       0.9, 0.999, 1e-8, 1.0, 0, 0),
        "adam": lambda: o.adam_step(tr.params, tr.grads, tr.m, tr.v, sh, st, 0, 0.0, 0.9, 0.999, 1e-8, 1.0, 0),
        # the same update on a capped grid (grid-stride loop): how the streaming rate depends on the
        # number of resident waves (the optimizer tail of conv2_bwd has one block per CU)
        **{f"adam_w3[blocks={nb}]": (lambda nb=nb: o.adam_step(tr.params[W3:], tr.grads[W3:], tr.m[W3:], tr.v[W3:],
                                                               sh[W3:], st, 0, 0.0, 0.9, 0.999, 1e-8, 1.0, 0, 0,
                                                               None, nb)) for nb in (256, 512, 1024)},
        "adam_small": lambda: o.adam_step(tr.params[:W3], tr.grads[:W3], tr.m[:W3], tr.v[:W3], sh[:W3], st, 0, 0.0,
                                          0.9, 0.999, 1e-8, 1.0, 0),
    }
    jobs = [(name, fn, None) for name, fn in ops.items()]
    if args.roles:  # MIHVD_ROLE_ONLY is read by the host wrappers at launch (i.e. capture) time
        for name, n_roles in (("fc1_wgrad", 2), ("conv2_bwd", 2), ("conv2_bwd_adam+reduce_adam", 3), ("conv2_bwd_adam", 3),
                              ("conv2_bwd_w3adam+reduce_adam", 3)):
            jobs += [(f"{name}[role{r}]", ops[name], r) for r in range(n_roles)]
    if args.phases:  # MIHVD_DEBUG_EXIT: conv2_bwd dgrad role cut after phase p (1 staging, 2 GEMM, 3 epilogue,
        # then conv1's weight gradient: 7 first barrier, 8 dY1 scatter stores, 4 + bias folds and barrier,
        # 5 bias sums + shifted images, 6 GEMM)
        jobs += [(f"conv2_bwd[role0,exit{p}]", ops["conv2_bwd"], (0, p)) for p in (1, 2, 3, 7, 8, 4, 5, 6)]
    if args.only:
        keep = set(args.only.split(";"))
        jobs = [j for j in jobs if j[0] in keep]
    res = {}
    s = torch.cuda.Stream()
    for name, fn, role in jobs:
        os.environ.pop("MIHVD_DEBUG_EXIT", None)
        if role is None:
            os.environ.pop("MIHVD_ROLE_ONLY", None)
        elif isinstance(role, tuple):
            os.environ["MIHVD_ROLE_ONLY"] = str(role[0])
            os.environ["MIHVD_DEBUG_EXIT"] = str(role[1])
        else:
            os.environ["MIHVD_ROLE_ONLY"] = str(role)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(args.iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1000.0 / args.iters
        print(f"{name:24s} {res[name]:8.2f} us", flush=True)
    os.environ.pop("MIHVD_ROLE_ONLY", None)
    os.environ.pop("MIHVD_DEBUG_EXIT", None)
    if args.only:
        if args.json:
            with open(args.json, "w") as f:
                json.dump(res, f, indent=1)
        return
    # whole step, graph-replayed
    from mihvd.utils.data import synthetic_mnist

    (xs, ys), _ = synthetic_mnist(n_train=6000, n_test=10)
    tr.set_device_dataset(torch.from_numpy(xs.reshape(-1, 784)).float().cuda() / 255,
                          torch.from_numpy(ys.astype("int64")).cuda())
    tr.build_graph(steps_per_replay=20)
    for _ in range(3):
        tr.run_graph()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        tr.run_graph()
    e1.record()
    torch.cuda.synchronize()
    res["step"] = e0.elapsed_time(e1) * 1000.0 / 200
    step_ops = (["conv12_fwd"] if tr.conv12 else ["conv1_fwd", "conv2_fwd"]) + ["fc1_fwd", "head", "fc1_dgrad"]
    if tr.fused_opt and getattr(tr, "w3_tail", False):
        step_ops = [k for k in step_ops if not (tr.fc1_merged and k == "fc1_dgrad")]
        step_ops += ["fc1_bwd[roles=2]", "conv2_bwd_w3adam+reduce_adam"]
    elif tr.fused_opt:
        step_ops = [k for k in step_ops if not (tr.fc1_merged and k == "fc1_dgrad")]
        step_ops += ["fc1_bwd" if tr.fc1_merged else "fc1_wgrad",
                     "conv2_bwd_adam_fold" if tr.fold_reduce else "conv2_bwd_adam+reduce_adam"]
    elif tr.fuse_w3:
        step_ops += ["fc1_wgrad_adam", "conv2_bwd", "conv2_wgrad_reduce", "adam_small"]
    else:
        step_ops += ["fc1_wgrad", "conv2_bwd", "conv2_wgrad_reduce", "adam"]
    res["sum_kernels"] = sum(res[k] for k in step_ops if k in res)
    print(f"{'step':12s} {res['step']:8.2f} us   (sum of kernels {res['sum_kernels']:.2f} us)", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
