"""tensorflow_datasets-style loader (distributed_with_keras.py:25-28):
``load(name='mnist', data_dir='/tmp/data', with_info=True, as_supervised=True)``.

No network: MNIST comes from data.mnist (a local mnist.npz if present, else the
deterministic synthetic set).  Images are uint8 (28, 28, 1), labels int64 —
the same element spec as TFDS, so the reference's ``scale`` map works unchanged.
"""
from __future__ import annotations

import numpy as np

from . import mnist
from .dataset import Dataset


class DatasetInfo:
    def __init__(self, name, splits, features):
        self.name = name
        self.splits = splits
        self.features = features

    def __repr__(self):
        return f"DatasetInfo(name={self.name!r}, splits={self.splits})"


class _SplitInfo:
    def __init__(self, n):
        self.num_examples = n


def disable_progress_bar():
    pass


def load(name="mnist", split=None, data_dir=None, with_info=False, as_supervised=False, shuffle_files=False,
         download=False, **kw):
    if name != "mnist":
        raise ValueError(f"dataset {name!r} is not available offline (only 'mnist')")
    (xtr, ytr), (xte, yte) = mnist.load_data()
    parts = {"train": (xtr[..., None], ytr.astype(np.int64)), "test": (xte[..., None], yte.astype(np.int64))}

    def make(x, y):
        if as_supervised:
            return Dataset.from_tensor_slices((x, y))
        return Dataset.from_tensor_slices({"image": x, "label": y})

    if split is not None:
        out = make(*parts[split])
    else:
        out = {k: make(*v) for k, v in parts.items()}
    if with_info:
        info = DatasetInfo("mnist", {k: _SplitInfo(len(v[1])) for k, v in parts.items()},
                           {"image": ((28, 28, 1), "uint8"), "label": ((), "int64")})
        return out, info
    return out
