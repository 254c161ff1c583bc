"""The reference entrypoint on one MI355X: the fused HIP step through the example's hooks,
checkpointing and restore (launcher -np 1, RCCL backend)."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(tmp_path, *args):
    env = dict(os.environ, PYTHONPATH=ROOT, HOME=str(tmp_path), MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "mihvd.runner", "-np", "1", sys.executable,
           os.path.join(ROOT, "examples", "tensorflow_mnist.py"), "--impl", "fused", *args]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
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
