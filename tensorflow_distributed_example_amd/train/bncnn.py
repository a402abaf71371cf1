"""Fused float32 plan of the BN-CNN family: Model B of mnist_keras_distributed.py:79-109
(== tf2_mnist_distributed.py:105-135) and its relatives.

Matches ``[Reshape] · (Conv2D(no bias, linear) · BatchNormalization · ReLU) x L · Flatten ·
Dense(no bias, linear) · BatchNormalization · ReLU · [Dropout] · Dense(+bias)[softmax]`` trained with
SparseCategoricalCrossentropy under the float32 policy (the reference's precision).  A training step
is 4 + L + 3 HIP launches of csrc/kernels/bncnn.hip — one statistics exchange per BatchNormalization
each way, every GEMM on the exact-f32 MFMA — instead of the ~25 launches of the layer-wise plan;
gradients land in the flat bucket (one all-reduce under data parallelism) and the multi-tensor
optimizer applies them.

Keras semantics kept: BN normalises with the batch mean / biased variance in training and the moving
statistics in inference; moving_variance is updated with the Bessel-corrected variance for 4-D inputs
(TF's fused batch norm) and the biased one for the 2-D Dense BN; epsilon / momentum from the layer;
Dropout is inverted (x / keep) with a counter-based Philox mask per step; the softmax head with the
probability-form loss is computed from the logits (Q5); ``set_learning_phase(1)`` (Q4) keeps batch
statistics and dropout in evaluation and prediction.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from .. import _native as N
from .. import backend as Kb
from ..losses import SparseCategoricalCrossentropy
from ..models import layers as L
from .program import OptimizerKernel, ReplicaPlan

BN_NONE, BN_TRAIN, BN_MOVING, BN_BATCH, BN_SAVED = 0, 1, 2, 3, 4

N.register_hip({
    "tde_bncnn_conv_fwd_lds": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "tde_bncnn_conv_fwd": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_longlong, C.c_void_p]),
    "tde_bncnn_dense_fwd": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p]),
    "tde_bncnn_head": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
                                 C.c_ulonglong, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_float, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p]),
    "tde_bncnn_dense_bwd": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "tde_bncnn_conv_bwd_plan": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "tde_bncnn_conv_bwd": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_int, C.c_void_p]),
    "tde_bncnn_reduce": (C.c_int, [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
})


class Geo(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("H", "W", "C", "Ho", "Wo", "Co", "kh", "kw", "sh", "sw", "pt", "pl")]


class Bn(C.Structure):
    _fields_ = [("mode", C.c_int), ("C", C.c_int), ("pmean", C.c_void_p), ("pm2", C.c_void_p), ("pn", C.c_void_p),
                ("npart", C.c_int), ("gamma", C.c_void_p), ("beta", C.c_void_p), ("eps", C.c_float),
                ("momentum", C.c_float), ("bessel", C.c_float), ("mmean", C.c_void_p), ("mvar", C.c_void_p),
                ("saved", C.c_void_p)]


class BnBwd(C.Structure):
    _fields_ = [("psg", C.c_void_p), ("psgx", C.c_void_p), ("npart", C.c_int), ("dbeta", C.c_void_p),
                ("dgamma", C.c_void_p)]


_P = N.ptr


def _chain(model):
    nodes = model._nodes()
    prev, out = 0, []
    for layer, ins, o in nodes:
        if len(ins) != 1 or ins[0] != prev:
            return None
        prev = o
        out.append(layer)
    return out


def match_bncnn(model, loss):
    """dict(convs=[(conv, bn)], dense=(dense, bn, dropout|None), head=dense) or None."""
    if not isinstance(loss, SparseCategoricalCrossentropy):
        return None
    chain = _chain(model)
    if not chain:
        return None
    ls = [l for l in chain if not isinstance(l, L.InputLayer)]
    if ls and isinstance(ls[0], L.Reshape):
        if len(ls[0].target_shape) != 3:
            return None
        ls = ls[1:]
    convs, i = [], 0

    def bn_relu(j):
        return (j + 1 < len(ls) and isinstance(ls[j], L.BatchNormalization) and isinstance(ls[j + 1], L.Activation)
                and ls[j + 1].activation == "relu")

    while i < len(ls) and isinstance(ls[i], L.Conv2D):
        c = ls[i]
        if c.use_bias or c.activation not in (None, "linear") or not bn_relu(i + 1):
            return None
        if c.input_shape is None or len(c.input_shape) != 3 or c.input_shape[-1] > 32 or c.filters > 32:
            return None
        convs.append((c, ls[i + 1]))
        i += 3
    if not convs or i >= len(ls) or not isinstance(ls[i], L.Flatten):
        return None
    i += 1
    if i >= len(ls) or not isinstance(ls[i], L.Dense):
        return None
    d = ls[i]
    if d.use_bias or d.activation not in (None, "linear") or not bn_relu(i + 1) or d.units > 240:
        return None
    bn_d = ls[i + 1]
    i += 3
    drop = None
    if i < len(ls) and isinstance(ls[i], L.Dropout):
        drop = ls[i]
        i += 1
    if i != len(ls) - 1 or not isinstance(ls[i], L.Dense):
        return None
    head = ls[i]
    if not head.use_bias or head.units > 16 or head.activation not in (None, "linear", "softmax"):
        return None
    if (head.activation == "softmax") == bool(loss.from_logits):
        return None
    return dict(convs=convs, dense=(d, bn_d, drop), head=head)


def _fwd_cfg(Co, K):
    """(tiles per wave, N tiles, K split) of a forward conv: ~50 f32 MFMAs per wave, >= 4 waves per tile row."""
    nt = 1 if Co <= 16 else 2
    steps = (K + 3) // 4
    if steps <= 8:
        return (4, 1, 1) if nt == 1 else (2, 2, 1)
    if nt == 2:
        return (1, 2, 4) if steps >= 64 else (1, 2, 1)
    return (1, 1, 4) if steps >= 96 else (1, 1, 1)


class BnCnnPlan(ReplicaPlan):
    kind = "fused_bncnn"
    compute_dtype = "fp32"
    input_dtype = torch.float32

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss, spec):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        self.lib = N.hip()
        self.loss = loss
        st = store
        dev = self.device
        B = self.B
        f32 = dict(dtype=torch.float32, device=dev)
        self.blocks = []
        for conv, bn in spec["convs"]:
            H, W_, Cin = conv.input_shape
            Ho, Wo, Co = conv.output_shape
            (pt, _), (pl, _) = conv.pads(conv.input_shape)
            kh, kw = conv.kernel_size
            g = Geo(H, W_, Cin, Ho, Wo, Co, kh, kw, conv.strides[0], conv.strides[1], pt, pl)
            K = kh * kw * Cin
            cfg = _fwd_cfg(Co, K)
            M = Ho * Wo
            mtw = (4 // cfg[2]) * cfg[0]
            nchunk = -(-(-(-M // 16)) // mtw)
            lds = self.lib.tde_bncnn_conv_fwd_lds(C.byref(g), *cfg)
            if lds < 0 or lds > 160 * 1024:
                raise ValueError(f"{conv.name}: forward tile does not fit in LDS ({lds} B)")
            blk = dict(conv=conv, bn=bn, geo=g, K=K, cfg=cfg, nchunk=nchunk,
                       w=st.view(f"{conv.name}/kernel"), gw=st.grad(f"{conv.name}/kernel"),
                       z=torch.zeros(B * M * Co, **f32), g=torch.zeros(B * M * Co, **f32),
                       pmean=torch.zeros(B * nchunk * Co, **f32), pm2=torch.zeros(B * nchunk * Co, **f32),
                       pn=torch.zeros(B * nchunk, **f32), saved=torch.zeros(2 * Co, **f32),
                       dwpart=torch.zeros(B * K * Co, **f32))
            blk.update(self._bn_vars(bn))
            blk["bessel_R"] = M   # rows per image of this BN (Bessel factor uses B * M)
            self.blocks.append(blk)
        # backward grids (input-gradient roles of layer l produce layer l-1's BN partial sums)
        for li, blk in enumerate(self.blocks):
            out = (C.c_int * 12)()
            if self.lib.tde_bncnn_conv_bwd_plan(C.byref(blk["geo"]), int(li > 0), out) != 0:
                raise ValueError(f"{blk['conv'].name}: backward tiles do not fit")
            blk["bwd"] = list(out)
        for li, blk in enumerate(self.blocks[:-1]):
            n_dg = self.blocks[li + 1]["bwd"][0]
            Co = blk["geo"].Co
            blk["psg"] = torch.zeros(B * n_dg * Co, **f32)
            blk["psgx"] = torch.zeros(B * n_dg * Co, **f32)
            blk["npart_bwd"] = n_dg   # per image
        dense, bn_d, drop = spec["dense"]
        last = self.blocks[-1]
        self.K = last["geo"].Ho * last["geo"].Wo * last["geo"].Co
        self.D = dense.units
        self.Dp = -(-self.D // 16) * 16
        self.kc = -(-(-(-self.K // 8)) // 4) * 4
        nkt = -(-self.K // 16)
        last["psg"] = torch.zeros(nkt * last["geo"].Co, **f32)
        last["psgx"] = torch.zeros(nkt * last["geo"].Co, **f32)
        last["npart_bwd"] = None   # fixed: one per dense k-tile
        self.nkt = nkt
        self.dense = dense
        self.wd, self.gwd = st.view(f"{dense.name}/kernel"), st.grad(f"{dense.name}/kernel")
        self.bnd = dict(layer=bn_d, saved=torch.zeros(2 * self.D, **f32), **self._bn_vars(bn_d))
        self.drop = drop
        self.drop_seed = 0
        if drop is not None:
            gen = Kb.make_generator(7919 + 97)
            self.drop_seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen).item()) if drop.seed is None \
                else int(drop.seed)
        head = spec["head"]
        self.head = head
        self.NC = head.units
        self.softmax = head.activation == "softmax"
        self.wh, self.bh = st.view(f"{head.name}/kernel"), st.view(f"{head.name}/bias")
        self.gwh, self.gbh = st.grad(f"{head.name}/kernel"), st.grad(f"{head.name}/bias")
        self.h = torch.zeros(B * self.Dp, **f32)
        self.dh = torch.zeros(B * self.Dp, **f32)
        self.probs = torch.zeros(B, self.NC, **f32)
        H0, W0, C0 = self.blocks[0]["geo"].H, self.blocks[0]["geo"].W, self.blocks[0]["geo"].C
        self.x_stride = H0 * W0 * C0
        self.opt = OptimizerKernel(store, optimizer, {}, self.iterations) if optimizer is not None else None

    def _bn_vars(self, bn):
        st, n = self.store, bn.name
        seg = st.segments
        v = dict(gamma=st.view(f"{n}/gamma") if bn.scale else None, beta=st.view(f"{n}/beta") if bn.center else None,
                 mmean=st.view(f"{n}/moving_mean"), mvar=st.view(f"{n}/moving_variance"),
                 dgamma=st.grad(f"{n}/gamma") if bn.scale and seg[f"{n}/gamma"].trainable else None,
                 dbeta=st.grad(f"{n}/beta") if bn.center and seg[f"{n}/beta"].trainable else None,
                 eps=bn.epsilon, momentum=bn.momentum)
        return v

    # ------------------------------------------------------------------ descriptors
    def _bn(self, blk, mode, B, C_=None, npart=None, pm=None, bessel=1.0):
        Cc = C_ if C_ is not None else blk["geo"].Co
        src = pm if pm is not None else blk
        return Bn(mode, Cc, _P(src.get("pmean")), _P(src.get("pm2")), _P(src.get("pn")), int(npart or 0),
                  _P(blk["gamma"]), _P(blk["beta"]), float(blk["eps"]), float(blk["momentum"]), float(bessel),
                  _P(blk["mmean"]), _P(blk["mvar"]), _P(blk["saved"]))

    def _fwd_mode(self, training):
        if training == "train":
            return BN_TRAIN
        return BN_BATCH if training else BN_MOVING

    # ------------------------------------------------------------------ forward
    def _forward(self, x, B, phase):
        """phase: "train" | True (batch statistics, no update: learning phase 1) | False (moving statistics)."""
        lib, s = self.lib, N.stream_ptr()
        mode = self._fwd_mode(phase)
        batch_stats = mode in (BN_TRAIN, BN_BATCH)
        inp = x
        bn_in = Bn(BN_NONE, self.blocks[0]["geo"].C)
        for li, blk in enumerate(self.blocks):
            tpw, nt, ks = blk["cfg"]
            zero, nzero = (self.h, B * self.Dp) if li == 0 else (None, 0)
            rc = lib.tde_bncnn_conv_fwd(C.byref(blk["geo"]), B, _P(inp), C.byref(bn_in), _P(blk["w"]), _P(blk["z"]),
                                        _P(blk["pmean"]) if batch_stats else None,
                                        _P(blk["pm2"]) if batch_stats else None,
                                        _P(blk["pn"]) if batch_stats else None, tpw, nt, ks, _P(zero), nzero, s)
            if rc < 0:
                raise RuntimeError(f"tde_bncnn_conv_fwd({blk['conv'].name}) failed with {rc}")
            R = B * blk["geo"].Ho * blk["geo"].Wo
            bn_in = self._bn(blk, mode, B, npart=B * blk["nchunk"], bessel=R / max(R - 1, 1))
            inp = blk["z"]
        rc = lib.tde_bncnn_dense_fwd(B, self.K, self.D, self.Dp, self.kc, _P(inp), C.byref(bn_in), _P(self.wd),
                                     _P(self.h), s)
        N.check(rc, "tde_bncnn_dense_fwd")
        return bn_in

    def _head(self, B, hmode, phase, labels, scale, probs=None):
        mode = self._fwd_mode(phase)
        bnd = self.bnd
        bn = Bn(mode, self.D, None, None, None, 0, _P(bnd["gamma"]), _P(bnd["beta"]), float(bnd["eps"]),
                float(bnd["momentum"]), 1.0, _P(bnd["mmean"]), _P(bnd["mvar"]), _P(bnd["saved"]))
        drop_on = int(self.drop is not None and self.drop.rate > 0 and phase is not False)
        train = hmode == 0
        rc = self.lib.tde_bncnn_head(
            B, self.D, self.Dp, self.NC, hmode, _P(self.h), C.byref(bn), float(self.drop.rate if self.drop else 0.0),
            self.drop_seed, _P(self.iterations), 0, drop_on, _P(self.wh), _P(self.bh), _P(labels), float(scale),
            _P(self.metrics), _P(probs), int(self.softmax), _P(self.gwh) if train else None,
            _P(self.gbh) if train else None, _P(bnd["dbeta"]) if train else None,
            _P(bnd["dgamma"]) if train else None, _P(self.dh) if train else None, N.stream_ptr())
        N.check(rc, "tde_bncnn_head")

    # ------------------------------------------------------------------ plan interface
    def _check_input(self, x, B):
        if B > self.B:
            raise ValueError(f"batch {B} > plan batch {self.B}")
        if x.dtype != torch.float32 or not x.is_contiguous() or x[:B].numel() != B * self.x_stride:
            raise ValueError("the BN-CNN plan reads a contiguous float32 input ring of the model's input shape")

    def train_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._check_input(x, B)
        lib, s = self.lib, N.stream_ptr()
        self._forward(x, B, "train")
        self._head(B, 0, "train", y, self.scale)
        last = self.blocks[-1]
        bn_last = self._bn(last, BN_SAVED, B)
        rc = lib.tde_bncnn_dense_bwd(B, self.K, self.D, self.Dp, _P(last["z"]), C.byref(bn_last), _P(self.wd),
                                     _P(self.dh), _P(self.gwd), _P(last["g"]), _P(last["psg"]), _P(last["psgx"]), s)
        if rc < 0:
            raise RuntimeError(f"tde_bncnn_dense_bwd failed with {rc}")
        npart = rc
        for li in range(len(self.blocks) - 1, -1, -1):
            blk = self.blocks[li]
            bb = BnBwd(_P(blk["psg"]), _P(blk["psgx"]), int(npart), _P(blk["dbeta"]), _P(blk["dgamma"]))
            if li > 0:
                prev = self.blocks[li - 1]
                inp, bn_in = prev["z"], self._bn(prev, BN_SAVED, B)
                gin, psg_in, psgx_in = prev["g"], prev["psg"], prev["psgx"]
            else:
                inp, bn_in = x, Bn(BN_NONE, blk["geo"].C)
                gin = psg_in = psgx_in = None
            rc = lib.tde_bncnn_conv_bwd(C.byref(blk["geo"]), B, _P(blk["z"]), C.byref(self._bn(blk, BN_SAVED, B)),
                                        C.byref(bb), _P(blk["g"]), _P(blk["w"]), _P(inp), C.byref(bn_in), _P(gin),
                                        _P(psg_in), _P(psgx_in), _P(blk["dwpart"]), int(li > 0), s)
            if rc < 0:
                raise RuntimeError(f"tde_bncnn_conv_bwd({blk['conv'].name}) failed with {rc}")
            npart = B * rc
        n = len(self.blocks)
        parts = (C.c_void_p * n)(*[b["dwpart"].data_ptr() for b in self.blocks])
        outs = (C.c_void_p * n)(*[b["gw"].data_ptr() for b in self.blocks])
        lens = (C.c_longlong * n)(*[b["K"] * b["geo"].Co for b in self.blocks])
        N.check(lib.tde_bncnn_reduce(n, B, parts, outs, lens, s), "tde_bncnn_reduce")

    def apply(self):
        self.opt.apply()

    def eval_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._check_input(x, B)
        phase = bool(Kb.resolve_training(False))
        self._forward(x, B, phase)
        self._head(B, 1, phase, y, self.scale)

    def predict(self, x, B=None):
        B = self.B if B is None else B
        self._check_input(x, B)
        phase = bool(Kb.resolve_training(False))
        self._forward(x, B, phase)
        self._head(B, 2, phase, None, 1.0, probs=self.probs)
        return self.probs[:B]


def try_make(model, store, device, batch, global_batch, optimizer, loss):
    if os.environ.get("TDE_BNCNN", "1") == "0" or Kb.global_policy().compute_dtype != torch.float32:
        return None
    spec = match_bncnn(model, loss)
    if spec is None:
        return None
    try:
        return BnCnnPlan(model, store, device, batch, global_batch, optimizer, loss, spec)
    except ValueError:
        return None
