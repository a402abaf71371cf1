"""Fused per-image plan for small classifiers: LeNet-5, dense MLPs, conv/pool/dense chains.

Model families: BASELINE.json config 2 (MNIST LeNet-5, ``zoo.lenet5``) and config 1's dense MLP
(``tf2_mnist_distributed.py``'s plumbing model, ``zoo.mnist_mlp``); any Sequential chain of
``Conv2D(stride 1, same/valid, relu|linear) [MaxPooling2D(2)]`` stages, ``Flatten``/``Reshape``,
``Dense(relu|linear)`` layers and a ``Dense`` head (logits, or softmax fed to the probability form of
``SparseCategoricalCrossentropy``) whose per-image activations fit in one workgroup's LDS.

A training step is two HIP launches (``csrc/kernels/smallnet.hip``): one workgroup per image runs the
forward, the loss and the whole input-gradient chain out of LDS and leaves per-image conv weight
gradients and the dense layers' inputs / pre-activation gradients in HBM; the second launch reduces
them over the batch and either stores the gradients in the flat bucket (step mode "plain": the
Program's all-reduce and multi-tensor optimizer follow) or applies the optimizer element-wise where
each gradient is finished (step mode "local", one replica).  Compute is fp32 throughout (the weights'
own precision), so there is no bf16 weight shadow to refresh.

Replaces the layer-wise plan's ~20 launches per LeNet-5 step (``train/layerwise.py``); selected by
``program.make_plan`` ahead of it (``TDE_SMALLNET=0`` keeps the layer-wise plan).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import _native as N
from ..losses import SparseCategoricalCrossentropy
from ..models import layers as L
from .program import OptimizerKernel, ReplicaPlan

CONV, POOL, DENSE = 0, 1, 2
_FIELDS = ("kind", "relu", "mask_in", "need_gin", "H", "W", "C", "Ho", "Wo", "Co", "kh", "kw", "pt", "pl",
           "w_off", "b_off", "in", "out", "wl", "part", "xo", "go")


def _limits():
    out = (np.zeros(4, dtype=np.int32))
    N.hip().tde_smallnet_limits(out.ctypes.data)
    return dict(max_layers=int(out[0]), lds=int(out[1]), scratch=int(out[2]), ints=int(out[3]))


def _a4(n):
    return (n + 3) & ~3


def _chain(model):
    nodes = model._nodes()
    prev = 0
    out = []
    for layer, ins, o in nodes:
        if len(ins) != 1 or ins[0] != prev:
            return None
        prev = o
        out.append(layer)
    return out


def match_smallnet(model, loss):
    """Per-layer description of a supported model, or None."""
    if not isinstance(loss, SparseCategoricalCrossentropy):
        return None
    chain = _chain(model)
    if not chain:
        return None
    ls = [l for l in chain if not isinstance(l, L.InputLayer)]
    shape = tuple(model.input_shape[1:])
    if len(shape) == 1:
        shape = (1, 1, shape[0])
    elif len(shape) != 3:
        return None
    spec = []     # dicts: kind, layer, in_shape, out_shape, relu, pads
    for layer in ls:
        if isinstance(layer, (L.Reshape, L.Flatten)):
            n = int(np.prod(shape))
            tgt = tuple(layer.compute_output_shape(shape if len(shape) == 3 else shape))
            if isinstance(layer, L.Flatten) or len(tgt) == 1:
                shape = (1, 1, n)
            elif len(tgt) == 3:
                shape = tgt
            else:
                return None
            continue
        if isinstance(layer, L.Activation):
            if layer.activation != "relu" or not spec or spec[-1]["kind"] == POOL or spec[-1]["relu"]:
                return None
            spec[-1]["relu"] = 1
            continue
        if isinstance(layer, L.Conv2D):
            if layer.strides != (1, 1) or layer.activation not in (None, "linear", "relu"):
                return None
            H, W, C = shape
            (pt, pb), (pl, pr) = layer.pads((H, W, C))
            Ho, Wo, Co = layer.compute_output_shape((H, W, C))
            if Ho < 1 or Wo < 1:
                return None
            spec.append(dict(kind=CONV, layer=layer, inp=(H, W, C), outp=(Ho, Wo, Co),
                             relu=int(layer.activation == "relu"), pt=pt, pl=pl, pb=pb, pr=pr))
            shape = (Ho, Wo, Co)
            continue
        if isinstance(layer, L.MaxPooling2D):
            if layer.pool_size != (2, 2) or layer.strides != (2, 2) or layer.padding != "valid":
                return None
            H, W, C = shape
            if H < 2 or W < 2 or not spec or spec[-1]["kind"] != CONV:
                return None
            spec.append(dict(kind=POOL, layer=layer, inp=shape, outp=(H // 2, W // 2, C), relu=0))
            shape = (H // 2, W // 2, C)
            continue
        if isinstance(layer, L.Dense):
            if shape[0] != 1 or shape[1] != 1 or layer.activation not in (None, "linear", "relu", "softmax"):
                return None
            spec.append(dict(kind=DENSE, layer=layer, inp=shape, outp=(1, 1, layer.units),
                             relu=int(layer.activation == "relu")))
            shape = (1, 1, layer.units)
            continue
        return None       # Dropout, BatchNormalization, strided conv, ...: other plans
    if not spec or spec[-1]["kind"] != DENSE:
        return None
    head = spec[-1]["layer"]
    if head.activation == "relu" or spec[-1]["relu"]:
        return None
    if (head.activation == "softmax") == bool(loss.from_logits):
        return None
    for i, s in enumerate(spec[:-1]):
        if s["kind"] == DENSE and s["layer"].activation == "softmax":
            return None
    if any(s["kind"] == DENSE and s["outp"][2] > 256 for s in spec):
        return None
    return spec


class SmallNetPlan(ReplicaPlan):
    kind = "fused_smallnet"
    input_dtype = torch.float32

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss, spec):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        self.loss = loss
        lim = _limits()
        if len(spec) > lim["max_layers"]:
            raise ValueError("too many layers for the fused small-net plan")
        self.lib = N.hip()
        seg = store.segments
        H0, W0, C0 = spec[0]["inp"]
        self.x_stride = H0 * W0 * C0
        # a same-padded first conv reads the image from a zero-padded LDS copy (then it is a valid conv)
        pad = spec[0]["kind"] == CONV and any(spec[0][k] for k in ("pt", "pb", "pl", "pr"))
        if pad:
            s0 = spec[0]
            Hp, Wp = H0 + s0["pt"] + s0["pb"], W0 + s0["pl"] + s0["pr"]
            self.img = np.array([H0, W0, C0, s0["pt"], s0["pl"], Hp, Wp], dtype=np.int32)
            spec = [dict(spec[0], inp=(Hp, Wp, C0), pt=0, pl=0, pb=0, pr=0)] + list(spec[1:])
        else:
            self.img = np.array([H0, W0, C0, 0, 0, H0, W0], dtype=np.int32)
        off = lim["scratch"]                      # [0, scratch): dense slice partials
        self.in0, self.n_in0 = off, int(self.img[5] * self.img[6] * C0)
        off = _a4(off + self.n_in0)
        rows = []
        part = 0
        rec = 0
        ranges = []
        dense = []
        prev_out, prev_kind, prev_relu = self.in0, None, 0
        for i, s in enumerate(spec):
            lay = s["layer"]
            H, W, C = s["inp"]
            Ho, Wo, Co = s["outp"]
            r = dict.fromkeys(_FIELDS, 0)
            r.update(kind=s["kind"], relu=s["relu"], H=H, W=W, C=C, Ho=Ho, Wo=Wo, Co=Co, b_off=-1,
                     **{"in": prev_out})
            r["need_gin"] = int(i > 0)
            r["mask_in"] = int(prev_kind in (CONV, DENSE) and prev_relu == 1)
            if s["kind"] == POOL:
                r["mask_in"] = int(prev_relu == 1)    # routes to the conv output's maxima, ReLU mask there
            if s["kind"] in (CONV, DENSE):
                r["w_off"] = seg[f"{lay.name}/kernel"].offset
                if lay.use_bias:
                    r["b_off"] = seg[f"{lay.name}/bias"].offset
            if s["kind"] == CONV:
                kh, kw = lay.kernel_size
                r.update(kh=kh, kw=kw, pt=s["pt"], pl=s["pl"], wl=off, part=part)
                nw = kh * kw * C * Co
                off = _a4(off + nw + Co)
                ranges.append((part, nw, r["w_off"]))
                part += nw
                if r["b_off"] >= 0:
                    ranges.append((part, Co, r["b_off"]))
                    part += Co
            if s["kind"] == DENSE:
                In = C
                r.update(C=In, xo=rec, go=rec + In)
                # wgrad workgroups: 16-row strips x groups of 4 16-column tiles (smallnet_wgrad_kernel)
                dense.append([In, Co, rec, rec + In, r["w_off"], r["b_off"], 0, -(-In // 16) * -(-(-(-Co // 16)) // 4)])
                rec += In + Co
            r["out"] = off
            off = _a4(off + Ho * Wo * Co)
            rows.append([r[f] for f in _FIELDS])
            prev_out, prev_kind, prev_relu = r["out"], s["kind"], s["relu"]
        if off > lim["lds"]:
            raise ValueError(f"per-image activations need {off} floats of LDS (> {lim['lds']})")
        self.lds = off
        self.layers = np.ascontiguousarray(np.array(rows, dtype=np.int32))
        assert self.layers.shape[1] == lim["ints"]
        self.npart = max(part, 1)
        self.nrec = rec + 2                       # + per-image loss, correct
        self.conv_nblk = -(-part // 32) if part else 0
        blk = 1 + self.conv_nblk
        for d in dense:
            d[6] = blk
            blk += d[7]
        self.ranges = np.ascontiguousarray(np.array(ranges if ranges else [(0, 0, 0)], dtype=np.int32))
        self.nranges = len(ranges)
        self.dense = np.ascontiguousarray(np.array(dense, dtype=np.int32))
        self.ncls = spec[-1]["outp"][2]
        self.probs_softmax = int(spec[-1]["layer"].activation == "softmax")
        dev = self.device
        B = self.B
        self.part = torch.zeros(B, self.npart, dtype=torch.float32, device=dev)
        self.rec = torch.zeros(B, self.nrec, dtype=torch.float32, device=dev)
        self.probs = torch.zeros(B, self.ncls, dtype=torch.float32, device=dev)
        self.opt = OptimizerKernel(store, optimizer, {}, self.iterations) if optimizer is not None else None
        self.stamps = None       # int64[64] to record workgroup 0's phase clock (bench/smallnet_phases.py)

    # ------------------------------------------------------------------ step modes
    def supports_step_mode(self, mode):
        # "xgmi": data parallel, the xGMI all-reduce applies the update to the f32 weights
        return mode == "plain" or (mode in ("local", "xgmi") and self.optimizer is not None and
                                   self.device.type == "cuda")

    def xg_apply_spec(self):
        from .program import f32_xg_apply_spec
        return f32_xg_apply_spec(self)

    def _step(self, mode, x, y, B, probs=None):
        if B > self.B:
            raise ValueError(f"batch {B} > plan batch {self.B}")
        if tuple(x.shape[1:]) and int(np.prod(x.shape[1:])) != self.x_stride:
            raise ValueError(f"input rows of {int(np.prod(x.shape[1:]))} values, plan expects {self.x_stride}")
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError("the small-net plan reads a contiguous float32 input ring")
        if y is not None and y.dtype != torch.int32:
            raise ValueError("labels must be int32")
        train = mode == 0
        rc = self.lib.tde_smallnet_step(
            self.layers.ctypes.data, len(self.layers), mode, B, self.store.w.data_ptr(), x.data_ptr(),
            self.x_stride, self.in0, self.n_in0, self.img.ctypes.data, N.ptr(y),
            self.part.data_ptr() if train else None, self.npart,
            self.rec.data_ptr() if train else None, self.nrec, self.metrics.data_ptr(),
            self.iterations.data_ptr(), float(self.scale), N.ptr(probs), self.probs_softmax, N.ptr(self.stamps),
            N.stream_ptr())
        N.check(rc, "tde_smallnet_step")

    def train_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._step(0, x, y, B)
        local = self.step_mode == "local"
        st, opt = self.store, self.optimizer
        m = v = None
        kind, lr, hp = 0, 0.0, dict(mom=0.0, b1=0.0, b2=0.0, eps=0.0)
        if local:
            sl = opt.slot_names()
            m = st.slot(sl[0]) if sl else None
            v = st.slot(sl[1]) if len(sl) > 1 else None
            kind, lr, hp = opt.kind_id, float(opt.learning_rate), opt.hparams()
        rc = self.lib.tde_smallnet_wgrad(
            self.ranges.ctypes.data, self.nranges, self.dense.ctypes.data, len(self.dense), self.conv_nblk, B,
            self.part.data_ptr(), self.npart, self.rec.data_ptr(), self.nrec, st.w.data_ptr(), st.g.data_ptr(),
            N.ptr(m), N.ptr(v), self.iterations.data_ptr(), self.metrics.data_ptr(), int(local), kind, lr,
            hp["mom"], hp["b1"], hp["b2"], hp["eps"], N.stream_ptr())
        N.check(rc, "tde_smallnet_wgrad")

    def apply(self):
        self.opt.apply()

    def eval_step(self, x, y, B=None):
        self._step(1, x, y, self.B if B is None else B)

    def predict(self, x, B=None):
        B = self.B if B is None else B
        self._step(2, x, None, B, probs=self.probs)
        return self.probs[:B]


def try_make(model, store, device, batch, global_batch, optimizer, loss):
    if os.environ.get("TDE_SMALLNET", "1") == "0":
        return None
    spec = match_smallnet(model, loss)
    if spec is None:
        return None
    try:
        return SmallNetPlan(model, store, device, batch, global_batch, optimizer, loss, spec)
    except ValueError:
        return None
