#!/usr/bin/env python3
"""Fixed cost of a short timed region (the driver's ``bench.py --steps 20 --warmup 5``): the same 20
fp32 steps replayed as one 20-step HIP graph or as several shorter graphs (a short first graph
starts the GPU sooner; the rest are enqueued while it runs), each bracketed like bench.py
(synchronize, timer, replays, synchronize). Also splits one 20-step replay into host launch time
and device time (events around it).

    python scripts/launch_probe.py [--reps 15]
"""
import argparse
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    B = 100
    (x, y), _ = synthetic_mnist(n_train=B * 40, n_test=10, seed=1)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=B, lr=1e-3, seed=0, device="cuda", precision="fp32")
    tr.set_device_dataset(X, Y)
    tr.build_graph(steps_per_replay=20)
    sizes = sorted({1, 2, 4, 5, 10, 15, 16, 18, 19})
    for k in sizes:
        tr.build_graph(steps_per_replay=k, warmup=0, primary=False)
    for k in [None] + sizes:
        tr.run_graph(k)
    torch.cuda.synchronize()
    schedules = {"20": [None], "1+19": [1, 19], "2+18": [2, 18], "4+16": [4, 16], "5+15": [5, 15],
                 "1+4+15": [1, 4, 15], "5x4": [4] * 5, "10+10": [10, 10]}
    res = {}
    for name, sched in schedules.items():
        ts = []
        for _ in range(a.reps):
            tr.run_graph(5 if 5 in sizes else None)  # the warm-up replay before the timed region
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in sched:
                tr.run_graph(k)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 20 * 1e6)
        res[name] = statistics.median(ts)
        print(f"{name:8s} {res[name]:8.2f} us/step (median of {a.reps}; min {min(ts):.2f})", flush=True)
    # one 20-step replay: host launch call, device time between events, and the whole bracket
    hl, dev, tot = [], [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.reps):
        tr.run_graph(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        t1 = time.perf_counter()
        tr.run_graph()
        t2 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        hl.append((t2 - t1) * 1e6)
        dev.append(e0.elapsed_time(e1) * 1e3)
        tot.append((t3 - t0) * 1e6)
    print(f"20-step replay: host launch call {statistics.median(hl):.1f} us, device (events) "
          f"{statistics.median(dev):.1f} us = {statistics.median(dev) / 20:.2f} us/step, bracket "
          f"{statistics.median(tot):.1f} us", flush=True)


if __name__ == "__main__":
    main()
