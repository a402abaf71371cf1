"""Model weight files.

Formats (chosen by extension / ``save_format``):
  * TensorBundle (``tf``; default for a bare prefix): ``<prefix>.index`` +
    ``<prefix>.data-00000-of-00001``, written by the native C++ writer
    (csrc/io/tensor_bundle.cpp) in the TF2 object-based layout of Keras ``save_weights``
    (io/object_graph.py: ``layer_with_weights-i/...`` keys, optimizer slots and step, the
    serialized object graph); ``tf1`` writes the TF1 variable names an Estimator uses.
    Loading accepts both.
  * ``.safetensors`` and ``.npz`` interchange formats.
Writes are atomic (temp file + rename) so a crash never corrupts the latest file.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np


def _fmt(path, save_format):
    if save_format:
        return {"tf": "tf", "tf1": "tf1", "h5": "h5", "safetensors": "safetensors", "npz": "npz"}[save_format]
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
        # TF2 Keras save_weights: the object-based layout (io/object_graph.py) with the optimizer state
        from . import object_graph as OG
        from . import tensor_bundle as TB
        slots, it = _optimizer_state(model)
        TB.write_bundle(str(filepath), OG.build(model, sd, slots, it))
    elif fmt == "tf1":
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
        from . import object_graph as OG
        from . import tensor_bundle as TB
        sd = TB.read_bundle(p)
        if OG.GRAPH_KEY in sd:
            # object-based (TF2 save_weights) checkpoint: matched by the model's object-graph position
            # (layer_with_weights-i / attribute), as TF does, not by (session-unique) variable names
            keys = OG.variable_keys(model)
            _restore_optimizer_state(model, sd, keys)
            sd = {n: sd[k] for n, k in keys.items() if k in sd}
    names = set(model.variable_names())
    model.load_state_dict({k: v for k, v in sd.items() if k in names}, strict=False)


def _optimizer_state(model):
    """({slot: {variable: array}}, iterations) of a compiled model, or (None, None)."""
    opt = getattr(model, "optimizer", None)
    if opt is None or not getattr(model, "built", False):
        return None, None
    st = model._store
    slots = {}
    for sname in opt.slot_names():
        if sname not in st.slots:
            continue
        flat = st.slots[sname].detach().cpu()
        slots[sname] = {n: flat[st.segments[n].offset: st.segments[n].offset + st.segments[n].numel]
                        .view(st.segments[n].shape).numpy().copy() for n in st.names(trainable=True)}
    return slots, int(opt.iterations)


def _restore_optimizer_state(model, bundle, keys):
    """Step counter and slots of an object-based checkpoint (``keys``: {variable: checkpoint key})."""
    import torch

    from . import object_graph as OG
    opt = getattr(model, "optimizer", None)
    if opt is None:
        return
    st = model._store
    it = bundle.get(f"optimizer/iter{OG.VAR}")
    if it is not None:
        model._set_iterations(int(np.asarray(it)))
    for sname in opt.slot_names():
        slot = st.slot(sname)
        for n in st.names(trainable=True):
            k = keys.get(n)
            sk = None if k is None else f"{k[:-len(OG.VAR)]}/.OPTIMIZER_SLOT/optimizer/{sname}{OG.VAR}"
            if sk in bundle:
                seg = st.segments[n]
                slot[seg.offset: seg.offset + seg.numel].copy_(
                    torch.as_tensor(np.asarray(bundle[sk]).reshape(-1), dtype=slot.dtype))
