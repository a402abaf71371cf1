"""Model export for serving (FinalExporter at mnist_keras_distributed.py:264,
serving_input_fn at :151-162 — a float32 ``[None, 784]`` placeholder).

Layout written under ``<export_dir_base>/<unix_timestamp>/``:
    saved_model.pb                   TF1 SavedModel protobuf: the serving graph in TensorFlow's standard ops,
                                     the save/restore subgraph + SaverDef, SignatureDef ``serving_default``
                                     (io/saved_model_pb.py; loading by TF itself is parity-unpinned)
    saved_model.json                 architecture (Sequential config), dtype policy,
                                     signature ``serving_default``: inputs/outputs specs
    variables/variables.index        TensorBundle (native writer), TF1 variable names
    variables/variables.data-00000-of-00001
``load(path)`` rebuilds the model from the JSON spec and serves through the HIP kernels on GPU (torch
reference ops on CPU).
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

import numpy as np


class TensorSpec:
    def __init__(self, shape, dtype="float32", name=None):
        self.shape = [None if d is None else int(d) for d in shape]
        self.dtype = str(dtype).replace("torch.", "").replace("tf.", "")
        self.name = name

    def to_json(self):
        return {"shape": self.shape, "dtype": self.dtype, "name": self.name}


def placeholder(dtype, shape=None, name=None):
    """tf.compat.v1.placeholder equivalent: a serving input signature spec."""
    return TensorSpec(shape if shape is not None else [None], dtype, name)


class ServingInputReceiver:
    def __init__(self, features, receiver_tensors, receiver_tensors_alternatives=None):
        self.features = features
        self.receiver_tensors = receiver_tensors


class TensorServingInputReceiver(ServingInputReceiver):
    pass


def export_saved_model(model, export_dir_base, serving_input_receiver_fn):
    from . import tensor_bundle as TB
    recv = serving_input_receiver_fn() if serving_input_receiver_fn is not None else None
    feats = recv.features if recv is not None else TensorSpec([None] + list(model.input_shape[1:]))
    if isinstance(feats, dict):
        feats = next(iter(feats.values()))
    base = Path(export_dir_base)
    ts = int(time.time())
    out = base / str(ts)
    while out.exists():
        ts += 1
        out = base / str(ts)
    tmp = base / f".tmp-{ts}-{os.getpid()}"
    (tmp / "variables").mkdir(parents=True, exist_ok=True)
    TB.write_bundle(str(tmp / "variables" / "variables"), {k: v.numpy() for k, v in model.state_dict().items()})
    last = model.layers[-1]
    out_name = "probabilities" if getattr(last, "activation", None) == "softmax" else "logits"
    spec = {
        "format": "tensorflow_distributed_example_amd.saved_model",
        "version": 1,
        "model": {"class_name": type(model).__name__, "config": model.get_config()},
        "signatures": {"serving_default": {
            "inputs": {"input": feats.to_json()},
            "outputs": {out_name: {"shape": [None] + list(model.output_shape[1:]), "dtype": "float32"}},
        }},
        "variables": "variables/variables",
    }
    (tmp / "saved_model.json").write_text(json.dumps(spec, indent=1, default=str))
    from .saved_model_pb import saved_model_bytes
    (tmp / "saved_model.pb").write_bytes(saved_model_bytes(model, input_shape=feats.shape, output_key=out_name))
    os.replace(tmp, out)
    return str(out).encode()


class Loaded:
    def __init__(self, path, model, spec):
        self.path = path
        self.model = model
        self.spec = spec
        sig = spec["signatures"]["serving_default"]
        self.input_spec = sig["inputs"]["input"]
        self.output_name = next(iter(sig["outputs"]))
        self.signatures = {"serving_default": self.serve}

    def serve(self, x, batch_size=256):
        x = np.asarray(x, dtype=np.float32)
        shape = self.input_spec["shape"]
        if len(shape) == x.ndim and any(d is not None and d != s for d, s in zip(shape[1:], x.shape[1:])):
            raise ValueError(f"input shape {x.shape} does not match signature {shape}")
        return {self.output_name: self.model.predict(x, batch_size=batch_size)}

    __call__ = serve


def load(path):
    from ..models.model import Functional, Sequential
    from . import tensor_bundle as TB
    p = Path(path.decode() if isinstance(path, bytes) else path)
    spec = json.loads((p / "saved_model.json").read_text())
    cls = Functional if spec["model"]["class_name"] == "Functional" else Sequential
    m = cls.from_config(spec["model"]["config"])
    m.build()
    vals = TB.read_bundle(str(p / spec["variables"]))
    m._store.load_dict({k: v for k, v in vals.items() if k in m._store.segments})
    from ..losses import SparseCategoricalCrossentropy
    m.loss = SparseCategoricalCrossentropy(from_logits=getattr(m.layers[-1], "activation", None) != "softmax")
    return Loaded(str(p), m, spec)
