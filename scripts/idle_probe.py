#!/usr/bin/env python3
"""Where the driver form's fixed cost goes: bench.py's 20 timed steps (a 2-step lead graph + an
18-step graph, bracketed by synchronize + timer) with the host idling 0 / 0.1 / 1 / 10 ms after the
synchronize before the timer starts, split into the host bracket and the device span between events
recorded around the replays (host - device = launch-to-first-dispatch + last-kernel-to-host latency).

    python scripts/idle_probe.py [--reps 15]
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
    import bench

    bench._host_wait_mode()  # hipDeviceScheduleSpin, as bench.py
    from mihvd.models.fused_mnist import FusedMNISTTrainer
    from mihvd.utils.data import synthetic_mnist

    B = 100
    (x, y), _ = synthetic_mnist(n_train=B * 600, n_test=10, seed=1)
    X = torch.from_numpy(x.reshape(-1, 784)).float().cuda() / 255.0
    Y = torch.from_numpy(y.astype("int64")).cuda()
    tr = FusedMNISTTrainer(batch_size=B, lr=1e-3, seed=0, device="cuda", precision="fp32")
    tr.set_device_dataset(X, Y)
    tr.build_graph(steps_per_replay=20)
    for k in (2, 18):
        tr.build_graph(steps_per_replay=k, warmup=0, primary=False)
    for _ in range(100):
        tr.run_graph()
    tr.run_graph(2)
    tr.run_graph(18)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for idle_ms in (0.0, 0.1, 1.0, 10.0):
        host, dev = [], []
        for _ in range(a.reps):
            tr.run_graph(2)  # a warm-up replay before the bracket (bench.py: --warmup)
            torch.cuda.synchronize()
            t = time.perf_counter()
            while time.perf_counter() - t < idle_ms * 1e-3:
                pass
            t0 = time.perf_counter()
            e0.record()
            tr.run_graph(2)
            tr.run_graph(18)
            e1.record()
            torch.cuda.synchronize()
            host.append((time.perf_counter() - t0) * 1e6)
            dev.append(e0.elapsed_time(e1) * 1e3)
        h, d = statistics.median(host), statistics.median(dev)
        print(f"idle {idle_ms:5.1f} ms: bracket {h:8.1f} us ({h / 20:6.2f} us/step), device span {d:8.1f} us "
              f"({d / 20:6.2f} us/step), bracket - span {h - d:6.1f} us (median of {a.reps})", flush=True)


if __name__ == "__main__":
    main()
