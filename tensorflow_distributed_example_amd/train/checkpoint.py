"""Estimator-style checkpoint management.

``CheckpointManager(model_dir, max_to_keep=5)`` writes ``model.ckpt-<step>``
TensorBundles (native writer) with TF1 variable names plus ``global_step``,
maintains the ``checkpoint`` state file, deletes checkpoints beyond
``max_to_keep``, and restores the latest one on (re)start (implicit resume,
mnist_keras_distributed.py:245).  Optimizer slots are saved under
``<var>/.OPTIMIZER_SLOT/<slot>`` and the data-iterator position/RNG seed under
``tde/...`` keys so a resumed run continues deterministically.
Only the chief writes; every task may read.
"""
from __future__ import annotations

import os
import time
from pathlib import Path

import numpy as np

from ..io import tensor_bundle as TB


class CheckpointManager:
    def __init__(self, model_dir, max_to_keep=5, prefix="model.ckpt", write_meta=False):
        self.dir = Path(model_dir)
        self.max_to_keep = max_to_keep
        self.prefix = prefix
        # Estimator checkpoints (write_meta): model.ckpt-N.meta (MetaGraphDef + SaverDef over the bundle) beside
        # every bundle and graph.pbtxt once in model_dir, as a TF1 Saver / Estimator lays out model_dir
        self.write_meta = write_meta

    def _paths(self):
        st = TB.read_checkpoint_state(self.dir)
        return list(st["all_model_checkpoint_paths"]) if st else []

    @property
    def latest(self):
        return TB.latest_checkpoint(self.dir)

    def save(self, model, global_step: int, extra: dict | None = None, state: dict | None = None) -> str:
        """``state``: a ``model.state_dict()`` taken on EVERY worker (its SyncOnRead reduction is a
        collective) when only the chief writes."""
        self.dir.mkdir(parents=True, exist_ok=True)
        tensors = {k: v.numpy() for k, v in (state if state is not None else model.state_dict()).items()}
        tensors["global_step"] = np.array(int(global_step), dtype=np.int64)
        opt = model.optimizer
        if opt is not None and model._store is not None:
            for slot, buf in model._store.slots.items():
                for name in model._store.names(trainable=True):
                    seg = model._store.segments[name]
                    tensors[f"{name}/.OPTIMIZER_SLOT/{slot}"] = \
                        buf[seg.offset: seg.offset + seg.numel].view(seg.shape).detach().cpu().numpy()
        for k, v in (extra or {}).items():
            tensors[f"tde/{k}"] = np.asarray(v)
        name = f"{self.prefix}-{int(global_step)}"
        TB.write_bundle(str(self.dir / name), tensors)
        if self.write_meta:
            self._write_meta(model, name, tensors)
        paths = [p for p in self._paths() if p != name] + [name]
        while len(paths) > self.max_to_keep:
            old = paths.pop(0)
            for suffix in (".index", ".data-00000-of-00001", ".meta"):
                try:
                    os.remove(self.dir / (old + suffix))
                except FileNotFoundError:
                    pass
        TB.write_checkpoint_state(self.dir, name, paths)
        return str(self.dir / name)

    def _write_meta(self, model, name, tensors):
        from ..io import saved_model_pb as SM
        try:
            meta = SM.checkpoint_meta_graph_bytes(model, tensors)
            pbtxt = None if (self.dir / "graph.pbtxt").exists() else SM.graph_pbtxt(model)
        except NotImplementedError:   # a layer with no TensorFlow op mapping: the bundle alone is the checkpoint
            return
        _atomic_write(self.dir / (name + ".meta"), meta)
        if pbtxt is not None:
            _atomic_write(self.dir / "graph.pbtxt", pbtxt.encode())

    def restore(self, model, path=None):
        """Load the latest (or given) checkpoint into ``model``; returns (global_step, extras) or None."""
        path = path or self.latest
        if path is None:
            return None
        vals = TB.read_bundle(path)
        names = set(model.variable_names())
        model.load_state_dict({k: v for k, v in vals.items() if k in names}, strict=False)
        if model._store is not None:
            for k, v in vals.items():
                if "/.OPTIMIZER_SLOT/" in k:
                    var, slot = k.split("/.OPTIMIZER_SLOT/")
                    if var in model._store.segments:
                        seg = model._store.segments[var]
                        import torch
                        model._store.slot(slot)[seg.offset: seg.offset + seg.numel].copy_(
                            torch.from_numpy(np.ascontiguousarray(v).reshape(-1)))
            model._weights_changed()
        step = int(vals.get("global_step", np.array(0)))
        extras = {k[4:]: v for k, v in vals.items() if k.startswith("tde/")}
        return step, extras


def _atomic_write(path: Path, data: bytes):
    tmp = path.with_name(path.name + ".tmp")
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def wait_for_new_checkpoint(model_dir, last=None, timeout=None, poll=0.5):
    """Block until a checkpoint different from ``last`` appears (evaluator polling, C8)."""
    t0 = time.time()
    while True:
        p = TB.latest_checkpoint(model_dir)
        if p is not None and p != last:
            return p
        if timeout is not None and time.time() - t0 > timeout:
            return None
        time.sleep(poll)
