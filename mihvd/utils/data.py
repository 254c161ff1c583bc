"""MNIST data: local files when present, otherwise synthetic (there is no network on the GPU box).

* ``load_mnist(path)`` mirrors ``keras.datasets.mnist.load_data('MNIST-data-%d' % rank)``
  (horovod/tensorflow_mnist.py:108-109): it looks for ``~/.keras/datasets/<path>`` as a Keras
  ``.npz`` (read with ``allow_pickle=False``) or for raw IDX files under ``$MIHVD_MNIST_DIR``.
  Without either it returns a deterministic, *learnable* synthetic set of the same shapes
  (60 000 / 10 000 images of 28×28 uint8, 10 classes): each class is a fixed random stroke pattern
  plus per-image jitter and noise, so convergence tests are meaningful.
* ``ensure_cache_dir()`` is the reference's EEXIST-tolerant mkdir race guard (:92-105).
* ``train_input_generator`` reproduces the reference generator (:76-85): a fresh permutation each
  pass over the data, contiguous batches, tail dropped, no per-rank sharding.
"""
from __future__ import annotations

import errno
import gzip
import os
import struct

import numpy as np


def ensure_cache_dir() -> str:
    cache_dir = os.path.join(os.path.expanduser("~"), ".keras", "datasets")
    if not os.path.exists(cache_dir):
        try:
            os.makedirs(cache_dir)
        except OSError as e:
            if not (e.errno == errno.EEXIST and os.path.isdir(cache_dir)):
                raise
    return cache_dir


def _read_idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    zero, dtype_code, ndim = struct.unpack(">HBB", data[:4])
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(dirname, stem):
    for suffix in ("", ".gz"):
        for name in (stem, stem.replace("-idx", ".idx")):
            p = os.path.join(dirname, name + suffix)
            if os.path.exists(p):
                return p
    return None


def load_idx_dir(dirname: str):
    names = ["train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"]
    paths = [_find(dirname, n) for n in names]
    if any(p is None for p in paths):
        return None
    xtr, ytr, xte, yte = (_read_idx(p) for p in paths)
    return (xtr, ytr), (xte, yte)


def synthetic_mnist(n_train: int = 60000, n_test: int = 10000, seed: int = 1234, sample_seed: int | None = None):
    """MNIST-shaped synthetic data: 10 class templates (random strokes, drawn from ``seed``), samples
    = a template shifted by up to 2 px, scaled and noised. ``sample_seed`` draws the samples from a
    separate generator with the SAME templates: data-parallel ranks must share the class templates
    and differ only in their samples (per-rank templates would give each rank its own labelling of
    the classes, and the averaged gradient of N conflicting labellings trains towards chance)."""
    rng = np.random.default_rng(seed)
    templates = np.zeros((10, 28, 28), dtype=np.float32)
    for c in range(10):
        # a few random strokes per class
        for _ in range(4):
            y0, x0 = rng.integers(4, 24, size=2)
            dy, dx = rng.integers(-3, 4, size=2)
            for t in range(8):
                y = int(np.clip(y0 + dy * t / 2, 0, 27))
                x = int(np.clip(x0 + dx * t / 2, 0, 27))
                templates[c, max(0, y - 1):y + 2, max(0, x - 1):x + 2] = 1.0

    def make(n, rs):
        labels = rs.integers(0, 10, size=n).astype(np.uint8)
        imgs = templates[labels]
        shifts = rs.integers(-2, 3, size=(n, 2))
        out = np.empty((n, 28, 28), dtype=np.float32)
        for s0 in range(-2, 3):
            for s1 in range(-2, 3):
                m = (shifts[:, 0] == s0) & (shifts[:, 1] == s1)
                if m.any():
                    out[m] = np.roll(imgs[m], (s0, s1), axis=(1, 2))
        out = out * rs.uniform(0.6, 1.0, size=(n, 1, 1)).astype(np.float32)
        out += rs.normal(0, 0.15, size=out.shape).astype(np.float32)
        return (np.clip(out, 0, 1) * 255).astype(np.uint8), labels

    s0 = seed if sample_seed is None else 7919 * sample_seed + 104729
    xtr, ytr = make(n_train, np.random.default_rng(s0 + 1))
    xte, yte = make(n_test, np.random.default_rng(s0 + 2))
    return (xtr, ytr), (xte, yte)


def load_mnist(path: str = "mnist.npz", allow_synthetic: bool = True):
    """Returns ``((x_train, y_train), (x_test, y_test))`` as uint8 arrays like Keras, plus the source."""
    cache = ensure_cache_dir()
    cand = [path if os.path.isabs(path) else os.path.join(cache, path)]
    cand += [c + ".npz" for c in cand if not c.endswith(".npz")]
    for c in cand:
        if os.path.isfile(c):
            with np.load(c, allow_pickle=False) as f:
                return ((f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])), "npz:" + c
    d = os.environ.get("MIHVD_MNIST_DIR")
    if d:
        r = load_idx_dir(d)
        if r is not None:
            return r, "idx:" + d
    if not allow_synthetic:
        raise FileNotFoundError(f"MNIST not found at {cand} or $MIHVD_MNIST_DIR")
    return synthetic_mnist(), "synthetic"


def train_input_generator(x_train, y_train, batch_size: int = 64, rng: np.random.Generator | None = None):
    assert len(x_train) == len(y_train)
    rng = rng or np.random.default_rng()
    while True:
        p = rng.permutation(len(x_train))
        x_train, y_train = x_train[p], y_train[p]
        index = 0
        while index <= len(x_train) - batch_size:
            yield x_train[index:index + batch_size], y_train[index:index + batch_size]
            index += batch_size
