"""Flat, HBM-resident variable storage for one replica.

All trainable variables of a model live in ONE contiguous fp32 buffer (``w``)
with a matching gradient buffer (``g``) and optimizer slot buffers; the
non-trainable state (BN moving statistics — SyncOnRead/MEAN variables, SURVEY
§2.6 C4) lives in ``state``.  Consequences of this layout on MI355X:

  * the gradient all-reduce is ONE RCCL call over ``g`` (a single flat bucket;
    1.0-1.4 MB for the MNIST models — latency bound, so one call is optimal),
  * the optimizer is ONE multi-tensor kernel over ``w/g/m/v``,
  * the initial-variable broadcast (C1) is ONE call over ``w`` and ``state``.

Segment offsets are aligned to 64 elements (256 B) so every variable starts on
its own cache-line group.  Variable names are the TF1/Keras ones
(``conv2d/kernel``, ``batch_normalization/moving_mean``...) used as checkpoint keys.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

ALIGN = 64


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


@dataclass
class Segment:
    name: str
    shape: tuple
    offset: int
    numel: int
    trainable: bool
    aggregation: str = "none"


class ParamStore:
    def __init__(self, specs, device, init=True, generator=None):
        self.device = torch.device(device)
        self.segments: dict[str, Segment] = {}
        self.order: list[str] = []
        off_t = 0
        off_s = 0
        for s in specs:
            n = int(np.prod(s.shape)) if len(s.shape) else 1
            if s.trainable:
                seg = Segment(s.full_name, s.shape, off_t, n, True, s.aggregation)
                off_t += _round(n)
            else:
                seg = Segment(s.full_name, s.shape, off_s, n, False, s.aggregation)
                off_s += _round(n)
            if seg.name in self.segments:
                raise ValueError(f"duplicate variable name {seg.name}")
            self.segments[seg.name] = seg
            self.order.append(seg.name)
        self.n_trainable = max(off_t, ALIGN)
        self.n_state = max(off_s, ALIGN)
        self.w = torch.zeros(self.n_trainable, dtype=torch.float32, device=self.device)
        self.g = torch.zeros(self.n_trainable, dtype=torch.float32, device=self.device)
        self.state = torch.zeros(self.n_state, dtype=torch.float32, device=self.device)
        self.slots: dict[str, torch.Tensor] = {}
        self._views = {}
        self._gviews = {}
        for name in self.order:
            seg = self.segments[name]
            buf = self.w if seg.trainable else self.state
            self._views[name] = buf[seg.offset: seg.offset + seg.numel].view(seg.shape)
            if seg.trainable:
                self._gviews[name] = self.g[seg.offset: seg.offset + seg.numel].view(seg.shape)
        if init:
            gen = generator
            host = {}
            for s in specs:
                host[s.full_name] = s.initializer(s.shape, gen)
            self.load_dict(host)

    # ------------------------------------------------------------------ access
    def view(self, name) -> torch.Tensor:
        return self._views[name]

    def grad(self, name) -> torch.Tensor:
        return self._gviews[name]

    def names(self, trainable=None):
        return [n for n in self.order if trainable is None or self.segments[n].trainable == trainable]

    def slot(self, name: str) -> torch.Tensor:
        if name not in self.slots:
            self.slots[name] = torch.zeros_like(self.w)
        return self.slots[name]

    def load_dict(self, values: dict, strict=False):
        for name, v in values.items():
            if name not in self._views:
                if strict:
                    raise KeyError(name)
                continue
            t = torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v)
            dst = self._views[name]
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(dst.shape)}")
            dst.copy_(t.to(dtype=torch.float32))

    def to_dict(self) -> dict:
        return {n: self._views[n].detach().cpu().clone() for n in self.order}

    def copy_from(self, other: "ParamStore"):
        self.w.copy_(other.w, non_blocking=True)
        self.state.copy_(other.state, non_blocking=True)
        for k, v in other.slots.items():
            self.slot(k).copy_(v, non_blocking=True)

    def clone_to(self, device) -> "ParamStore":
        st = ParamStore.__new__(ParamStore)
        st.device = torch.device(device)
        st.segments = dict(self.segments)
        st.order = list(self.order)
        st.n_trainable, st.n_state = self.n_trainable, self.n_state
        st.w = self.w.to(st.device, copy=True)
        st.g = torch.zeros_like(st.w)
        st.state = self.state.to(st.device, copy=True)
        st.slots = {k: v.to(st.device, copy=True) for k, v in self.slots.items()}
        st._views, st._gviews = {}, {}
        for name in st.order:
            seg = st.segments[name]
            buf = st.w if seg.trainable else st.state
            st._views[name] = buf[seg.offset: seg.offset + seg.numel].view(seg.shape)
            if seg.trainable:
                st._gviews[name] = st.g[seg.offset: seg.offset + seg.numel].view(seg.shape)
        return st

    def num_trainable_elements(self):
        return sum(s.numel for s in self.segments.values() if s.trainable)
