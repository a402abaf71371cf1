"""Model weight files.

Formats (chosen by extension / ``save_format``):
  * TensorBundle (``tf``; default for a bare prefix): ``<prefix>.index`` +
    ``<prefix>.data-00000-of-00001`` + ``checkpoint`` state file, written by the
    native C++ writer (csrc/io/tensor_bundle.cpp) with TF1 variable names.
  * ``.safetensors`` and ``.npz`` interchange formats.
Writes are atomic (temp file + rename) so a crash never corrupts the latest file.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np


def _fmt(path, save_format):
    if save_format:
        return {"tf": "tf", "h5": "h5", "safetensors": "safetensors", "npz": "npz"}[save_format]
    p = str(path)
    if p.endswith(".safetensors"):
        return "safetensors"
    if p.endswith(".npz"):
        return "npz"
    if p.endswith(".h5") or p.endswith(".keras"):
        return "h5"
    return "tf"


def _atomic_write_bytes(path, data: bytes):
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def save_model_weights(model, filepath, save_format=None):
    fmt = _fmt(filepath, save_format)
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    Path(filepath).parent.mkdir(parents=True, exist_ok=True) if Path(filepath).parent != Path("") else None
    if fmt == "npz":
        tmp = f"{filepath}.tmp{os.getpid()}.npz"
        np.savez(tmp, **{k.replace("/", "__"): v for k, v in sd.items()})
        os.replace(tmp, filepath)
    elif fmt == "safetensors":
        from safetensors.numpy import save
        _atomic_write_bytes(filepath, save({k: np.ascontiguousarray(v) for k, v in sd.items()}))
    elif fmt == "tf":
        from . import tensor_bundle as TB
        TB.write_bundle(str(filepath), sd)
    else:
        raise ValueError("HDF5 (.h5) weights need h5py, which is not available; use a TensorBundle prefix, "
                         ".safetensors or .npz")


def load_model_weights(model, filepath):
    p = str(filepath)
    if p.endswith(".npz"):
        with np.load(p, allow_pickle=False) as d:
            sd = {k.replace("__", "/"): d[k] for k in d.files}
    elif p.endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(p)
    else:
        from . import tensor_bundle as TB
        sd = TB.read_bundle(p)
    names = set(model.variable_names())
    model.load_state_dict({k: v for k, v in sd.items() if k in names}, strict=False)
