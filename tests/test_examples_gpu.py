"""The reference entrypoint on one MI355X: the fused HIP step through the example's hooks,
checkpointing and restore (launcher -np 1, RCCL backend)."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(tmp_path, *args, script="tensorflow_mnist.py", impl=("--impl", "fused"), timeout=110):
    env = dict(os.environ, PYTHONPATH=ROOT, HOME=str(tmp_path), MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "mihvd.runner", "-np", "1", sys.executable,
           os.path.join(ROOT, "examples", script), *impl, *args]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    return out


def test_fused_example_trains_checkpoints_restores(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = _launch(tmp_path, "--num-steps", "60")
    losses = [float(v) for v in re.findall(r"\[rank 0/1\] step=\d+ loss=([0-9.e+-]+)", out)]
    assert len(losses) >= 5 and losses[-1] < losses[0], out[-2000:]
    assert (tmp_path / "checkpoints" / "model.ckpt-60.pt").is_file()
    out2 = _launch(tmp_path, "--num-steps", "80")
    assert "restored ./checkpoints/model.ckpt-60 (global_step=60)" in out2, out2[-2000:]
    assert (tmp_path / "checkpoints" / "model.ckpt-80.pt").is_file()


def test_fused_example_throughput_matches_bench(tmp_path):
    """The reference entrypoint runs the benched path: device-resident data and 10-step graph
    replays between hook invocations. Its logged img/s is within 1.5x of bench.py's (same fp32
    step, same batch) although the hooks read the loss every 10 steps."""
    import json

    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = _launch(tmp_path, "--num-steps", "4000", "--log-step-count-steps", "1000", timeout=150)
    rates = [float(v) for v in re.findall(r"img_per_sec=([0-9.]+)", out)]
    assert len(rates) >= 3, out[-2000:]
    example = max(rates[1:])  # the first interval includes the graph capture
    env = dict(os.environ, PYTHONPATH=ROOT)
    b = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1000", "--warmup", "20"], env=env,
                       capture_output=True, text=True, timeout=150, cwd=ROOT)
    assert b.returncode == 0, b.stderr[-2000:]
    bench = json.loads([line for line in b.stdout.splitlines() if line.startswith("{")][-1])
    assert bench["dtype"] == "fp32"
    assert example * 1.5 >= bench["value"], (example, bench["value"])


@pytest.mark.parametrize("policy", ["mixed_bfloat16", "float32", "mixed_float16"])
def test_keras_example_trains_on_hip_kernels(tmp_path, policy):
    """tensorflow_mnist_gpu.py's Model.fit through MNISTConvNet(impl="hip"): one epoch on the HIP
    kernels -- the fused graph-replayed trainer under every policy (fp32 / bf16 / fp16 operands; the
    mixed_float16 step keeps its dynamic loss scale on the device; it prints its images/sec) -- then
    evaluation, best checkpoint and the final save."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    out = _launch(tmp_path, "--num-steps", "20", "--policy", policy, script="tensorflow_mnist_gpu.py",
                  impl=("--impl", "hip"), timeout=150)
    acc = [float(v) for v in re.findall(r"Test accuracy: ([0-9.]+)", out)]
    assert acc and acc[-1] > 0.8, out[-2000:]
    # every policy: fit drives the fused, graph-replayed step
    ips = [float(v) for v in re.findall(r"fit throughput: ([0-9.]+) images/sec", out)]
    assert len(ips) == 1 and ips[0] > 1e5, out[-2000:]
    assert (tmp_path / "checkpoints" / "mnist-1.h5").is_file()
    assert (tmp_path / "final_model" / "model.pt").is_file()
