"""End-to-end runs of the example entrypoints under the launcher (CPU, gloo, two ranks).

These are the reference's own validation mechanisms (loss logging, held-out
evaluation, rank-0 checkpoints restored and broadcast on restart), exercised on the reference's
launch line (horovod/tensorflow-mnist.yaml:19-38) instead of being eyeballed on a cluster.
"""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN_FLAGS = ("--allow-run-as-root -bind-to none -map-by slot -x LD_LIBRARY_PATH -x PATH "
                "-mca pml ob1 -mca btl ^openib").split()


def _launch(tmp_path, script, *args, np_=2, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, HOME=str(tmp_path), MIHVD_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "mihvd.runner", "-np", str(np_), *MPIRUN_FLAGS, sys.executable,
           os.path.join(ROOT, "examples", script), *args]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    return out


def _small_dataset(home, ranks=2, n_train=4000, n_test=500):
    """Per-rank dataset files where the reference keeps them (~/.keras/datasets/MNIST-data-<rank>,
    tensorflow_mnist.py:108-109), small enough for a unit test."""
    from mihvd.utils.data import synthetic_mnist

    (xtr, ytr), (xte, yte) = synthetic_mnist(n_train=n_train, n_test=n_test, seed=3)
    d = home / ".keras" / "datasets"
    d.mkdir(parents=True, exist_ok=True)
    for r in range(ranks):
        np.savez(d / f"MNIST-data-{r}.npz", x_train=xtr, y_train=ytr, x_test=xte, y_test=yte)


def test_tf1_example_logs_checkpoints_and_restores(tmp_path):
    out = _launch(tmp_path, "tensorflow_mnist.py", "--num-steps", "40")
    # LoggingTensorHook({'step','loss'}, every_n_iter=10) on every rank (tensorflow_mnist.py:148-149)
    for r in (0, 1):
        assert re.search(rf"\[rank {r}/2\] step=1 loss=", out), out[-2000:]
        assert re.search(rf"\[rank {r}/2\] step=11 loss=", out), out[-2000:]
    ck = tmp_path / "checkpoints"
    # StopAtStepHook(last_step=num_steps // size()) -> 20 steps; rank 0 alone writes ./checkpoints
    assert (ck / "checkpoint").read_text().startswith('model_checkpoint_path: "model.ckpt-20"')
    assert (ck / "model.ckpt-20.pt").is_file()
    out2 = _launch(tmp_path, "tensorflow_mnist.py", "--num-steps", "60")
    assert "restored ./checkpoints/model.ckpt-20 (global_step=20)" in out2, out2[-2000:]
    assert re.search(r"\[rank 1/2\] step=21 loss=", out2)  # rank 1 continues from the broadcast step
    assert not re.search(r"step=1 loss=", out2)
    assert 'model_checkpoint_path: "model.ckpt-30"' in (ck / "checkpoint").read_text()


def test_tf1_example_adasum(tmp_path):
    out = _launch(tmp_path, "tensorflow_mnist.py", "--num-steps", "20", "--use-adasum")
    assert re.search(r"\[rank 0/2\] step=1 loss=", out)
    assert (tmp_path / "checkpoints" / "model.ckpt-10.pt").is_file()


def test_keras_example_fit_evaluate_save(tmp_path):
    _small_dataset(tmp_path)
    out = _launch(tmp_path, "tensorflow_mnist_gpu.py", "--num-steps", "40")
    # steps_per_epoch = 4000 // (100 * 2) = 20, epochs = 40 // 20 = 2 (tensorflow_mnist_gpu.py:166-170);
    # verbose on rank 0 only, evaluation and final save on rank 0
    assert "Epoch 2/2" in out and "Epoch 3/" not in out, out[-2000:]
    assert out.count("Test accuracy:") == 1
    acc = float(re.search(r"Test accuracy: ([0-9.]+)", out).group(1))
    assert acc > 0.9, out[-2000:]
    assert list((tmp_path / "checkpoints").glob("mnist-*.h5"))
    assert (tmp_path / "final_model").is_dir() and any((tmp_path / "final_model").iterdir())
    assert (tmp_path / "logs").is_dir()


@pytest.mark.parametrize("ranks", [1])
def test_tf1_example_single_rank_minimum_slice(tmp_path, ranks):
    """SURVEY.md §7.3's minimum slice at -np 1: train, checkpoint on rank 0, restore on rerun."""
    _launch(tmp_path, "tensorflow_mnist.py", "--num-steps", "15", np_=ranks)
    out = _launch(tmp_path, "tensorflow_mnist.py", "--num-steps", "25", np_=ranks)
    assert "restored ./checkpoints/model.ckpt-15 (global_step=15)" in out
    assert (tmp_path / "checkpoints" / "model.ckpt-25.pt").is_file()
