"""MNIST loaders — no network.

``load_data()`` mirrors ``tf.keras.datasets.mnist.load_data()``
(mnist_keras_distributed.py:207-208): returns ``(x_train, y_train), (x_test,
y_test)`` as uint8 arrays of shape (60000, 28, 28)/(10000, 28, 28) and labels
(60000,)/(10000,).  If a real ``mnist.npz`` is present (``path`` argument,
``$TDE_MNIST_PATH`` or ``~/.keras/datasets/mnist.npz``) it is read with
``numpy.load(allow_pickle=False)``; otherwise a deterministic synthetic
MNIST-shaped set is generated: each class has a fixed random stroke template,
samples are shifted/noised copies, so models can actually learn it.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np

N_TRAIN, N_TEST = 60000, 10000


def _templates(rng):
    t = np.zeros((10, 28, 28), dtype=np.float32)
    for c in range(10):
        for _ in range(6):  # random strokes
            y0, x0 = rng.integers(4, 24, size=2)
            dy, dx = rng.integers(-3, 4, size=2)
            for s in range(8):
                y, x = y0 + dy * s // 2, x0 + dx * s // 2
                if 1 <= y < 27 and 1 <= x < 27:
                    t[c, y - 1:y + 2, x - 1:x + 2] += 1.0
    return np.clip(t, 0, 1.5) / 1.5


def synthetic(n, seed=0, num_classes=10):
    rng = np.random.default_rng(seed)
    templ = _templates(np.random.default_rng(1234))
    labels = rng.integers(0, num_classes, size=n).astype(np.uint8)
    imgs = templ[labels % 10]
    shifts = rng.integers(-2, 3, size=(n, 2))
    out = np.empty((n, 28, 28), dtype=np.float32)
    for sy in range(-2, 3):
        for sx in range(-2, 3):
            m = (shifts[:, 0] == sy) & (shifts[:, 1] == sx)
            if m.any():
                out[m] = np.roll(imgs[m], (sy, sx), axis=(1, 2))
    out += rng.normal(0.0, 0.15, size=out.shape).astype(np.float32)
    return (np.clip(out, 0, 1) * 255).astype(np.uint8), labels


def _find(path):
    cands = [path, os.environ.get("TDE_MNIST_PATH"), str(Path.home() / ".keras" / "datasets" / "mnist.npz")]
    for c in cands:
        if c and Path(c).is_file():
            return c
    return None


def load_data(path=None, synthetic_data=None, seed=0):
    if synthetic_data is None:
        synthetic_data = os.environ.get("TDE_SYNTHETIC_MNIST", "0") not in ("", "0")   # --synthetic
    f = None if synthetic_data else _find(path)
    if f is not None:
        with np.load(f, allow_pickle=False) as d:
            return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
    xtr, ytr = synthetic(N_TRAIN, seed)
    xte, yte = synthetic(N_TEST, seed + 1)
    return (xtr, ytr), (xte, yte)


def is_synthetic(path=None):
    return _find(path) is None
