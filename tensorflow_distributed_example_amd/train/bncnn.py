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

_vp, _i = C.c_void_p, C.c_int
N.register_hip({
    "tde_bncnn_conv_fwd_cfg": (_i, [_vp, _vp]),
    # geo, B, in, bn_in, w, z, acc, inc_iter, stream
    "tde_bncnn_conv_fwd": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    # B, K, D, Dp, in, bn, w, h, hstat, keep, rate, seed, iter, layer_id, stream
    "tde_bncnn_dense_fwd": (_i, [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, C.c_float, C.c_ulonglong, _vp, _i, _vp]),
    # B, D, Dp, NC, mode, h, hstat, bn, rate, seed, iter, layer_id, drop_on, wh, bh, labels, scale, metrics, out,
    # out_softmax, dwh_part, dbh_part, g, gstat, stream
    "tde_bncnn_head": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, C.c_float, C.c_ulonglong, _vp, _i, _i, _vp, _vp, _vp,
                            C.c_float, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    # B, K, D, Dp, in, bn, w, gh, h, gstat, nrt, bnd, dbeta_d, dgamma_d, dwpart, g, acc, stream
    "tde_bncnn_dense_bwd": (_i, [_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                                 _vp]),
    # B, K, D, Dp, NC, in, bn, w, h, hstat, bnd, keep, rate, wh, bh, labels, scale, metrics, dwh_part, dbh_part,
    # dbeta_d, dgamma_d, dwpart, g, acc, stream
    "tde_bncnn_dense_bwd_head": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_float, _vp, _vp, _vp,
                                      C.c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "tde_bncnn_conv_bwd_plan": (_i, [_vp, _i, _vp]),
    # geo, B, z, bn, bb, gout, w, in, bn_in, gin, acc_in, dwpart, dgrad, wstack, stream
    "tde_bncnn_conv_bwd": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    # n, cnt, part, out, len, opt, push_seg, push, stream
    "tde_bncnn_reduce": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    # B, D, rate, seed, iter, layer_id, out, stream
    "tde_bncnn_dropout_mask": (_i, [_i, _i, C.c_float, C.c_ulonglong, _vp, _i, _vp, _vp]),
})


class BnOpt(C.Structure):
    """Fused optimizer of the reduce launch (step mode "local")."""
    _fields_ = [("kind", C.c_int), ("lr", C.c_float), ("mom", C.c_float), ("b1", C.c_float), ("b2", C.c_float),
                ("eps", C.c_float), ("g", C.c_void_p), ("w", C.c_void_p), ("m", C.c_void_p), ("v", C.c_void_p),
                ("iterations", C.c_void_p)]


class Geo(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("H", "W", "C", "Ho", "Wo", "Co", "kh", "kw", "sh", "sw", "pt", "pl")]


class Bn(C.Structure):
    """acc: f64 [npart][2][C] per-workgroup partial batch sums (sum, sum of squares) over `count` values."""
    _fields_ = [("mode", C.c_int), ("C", C.c_int), ("acc", C.c_void_p), ("npart", C.c_int), ("count", C.c_double),
                ("gamma", C.c_void_p), ("beta", C.c_void_p), ("eps", C.c_float), ("momentum", C.c_float),
                ("bessel", C.c_float), ("mmean", C.c_void_p), ("mvar", C.c_void_p), ("saved", C.c_void_p)]


class BnBwd(C.Structure):
    """acc: f64 [npart][2][C] per-workgroup partial backward sums (sum g, sum g*xhat)."""
    _fields_ = [("acc", C.c_void_p), ("npart", C.c_int), ("dbeta", C.c_void_p), ("dgamma", C.c_void_p)]


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
    too_wide = []   # the family's structure with widths past the fused kernels' limits: said, not silent

    def bn_relu(j):
        return (j + 1 < len(ls) and isinstance(ls[j], L.BatchNormalization) and isinstance(ls[j + 1], L.Activation)
                and ls[j + 1].activation == "relu")

    while i < len(ls) and isinstance(ls[i], L.Conv2D):
        c = ls[i]
        if c.use_bias or c.activation not in (None, "linear") or not bn_relu(i + 1):
            return None
        if c.input_shape is None or len(c.input_shape) != 3:
            return None
        if c.input_shape[-1] > 32 or c.filters > 32:
            too_wide.append(f"{c.name}: {c.input_shape[-1]} -> {c.filters} channels (<= 32)")
        convs.append((c, ls[i + 1]))
        i += 3
    if not convs or i >= len(ls) or not isinstance(ls[i], L.Flatten):
        return None
    if len(convs) > 3:
        too_wide.append(f"{len(convs)} conv blocks (<= 3)")
    i += 1
    if i >= len(ls) or not isinstance(ls[i], L.Dense):
        return None
    d = ls[i]
    if d.use_bias or d.activation not in (None, "linear") or not bn_relu(i + 1):
        return None
    if d.units > 256:
        too_wide.append(f"{d.name}: {d.units} units (<= 256)")
    bn_d = ls[i + 1]
    i += 3
    drop = None
    if i < len(ls) and isinstance(ls[i], L.Dropout):
        drop = ls[i]
        i += 1
    if i != len(ls) - 1 or not isinstance(ls[i], L.Dense):
        return None
    head = ls[i]
    if not head.use_bias or head.activation not in (None, "linear", "softmax"):
        return None
    if (head.activation == "softmax") == bool(loss.from_logits):
        return None
    if head.units > 16:
        too_wide.append(f"{head.name}: {head.units} classes (<= 16)")
    if too_wide:
        import warnings
        warnings.warn(f"model {model.name!r}: no fused BN-CNN step ({'; '.join(too_wide)}); running the per-layer "
                      "kernel plan")
        return None
    return dict(convs=convs, dense=(d, bn_d, drop), head=head)


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
        f64 = dict(dtype=torch.float64, device=dev)
        self.blocks = []
        for conv, bn in spec["convs"]:
            H, W_, Cin = conv.input_shape
            Ho, Wo, Co = conv.output_shape
            (pt, _), (pl, _) = conv.pads(conv.input_shape)
            kh, kw = conv.kernel_size
            g = Geo(H, W_, Cin, Ho, Wo, Co, kh, kw, conv.strides[0], conv.strides[1], pt, pl)
            K = kh * kw * Cin
            M = Ho * Wo
            cfg = (C.c_int * 4)()
            rc = self.lib.tde_bncnn_conv_fwd_cfg(C.byref(g), cfg)
            if rc != 0:
                raise ValueError(f"{conv.name}: no forward tile configuration fits ({rc})")
            msplit = cfg[2]   # forward workgroups per image = BN statistics partials per image
            blk = dict(conv=conv, bn=bn, geo=g, K=K, cfg=list(cfg), msplit=msplit,
                       w=st.view(f"{conv.name}/kernel"), gw=st.grad(f"{conv.name}/kernel"),
                       z=torch.zeros(B * M * Co, **f32), g=torch.zeros(B * M * Co, **f32),
                       acc=torch.zeros(msplit * B * 2 * Co, **f64), accb=torch.zeros(B * 2 * Co, **f64),
                       saved=torch.zeros(2 * Co, **f32), dwpart=torch.zeros(B * K * Co, **f32))
            blk.update(self._bn_vars(bn))
            self.blocks.append(blk)
        # backward grids (the input-gradient roles of layer l accumulate layer l-1's BN backward sums)
        for li, blk in enumerate(self.blocks):
            out = (C.c_int * 12)()
            if self.lib.tde_bncnn_conv_bwd_plan(C.byref(blk["geo"]), int(li > 0), out) != 0:
                raise ValueError(f"{blk['conv'].name}: backward tiles do not fit")
            blk["bwd"] = list(out)
            # the input-gradient role's class-stacked weights, staged by the training forward of the layer
            blk["wstack"] = torch.zeros(out[5], **f32) if li > 0 and out[5] > 0 else None
        dense, bn_d, drop = spec["dense"]
        last = self.blocks[-1]
        self.K = last["geo"].Ho * last["geo"].Wo * last["geo"].Co
        self.D = dense.units
        self.Dp = -(-self.D // 16) * 16
        self.dense = dense
        self.wd, self.gwd = st.view(f"{dense.name}/kernel"), st.grad(f"{dense.name}/kernel")
        self.nrb = -(-B // 64)   # dense dW partials: one per 64-row block
        self.dwd_part = torch.zeros(self.nrb * self.K * self.D, **f32)
        # the dense backward (grid K/32 x row blocks) produces the last conv BN's backward partials
        last["accb"] = torch.zeros(-(-self.K // 32) * self.nrb * 2 * last["geo"].Co, **f64)
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
        nrt = -(-B // 16)   # 16-row tiles of the dense / head launches
        self.hstat = torch.zeros(nrt * 2 * self.Dp, **f64)     # dense BN statistics partials per row tile
        self.gstat = torch.zeros(nrt * 2 * self.Dp, **f64)     # its backward partials
        self.gh = torch.zeros(B * self.Dp, **f32)              # dL/d(dense BN output) through the masks
        self.dwh_part = torch.zeros(nrt * self.D * self.NC, **f32)
        self.dbh_part = torch.zeros(nrt * self.NC, **f32)
        self.probs = torch.zeros(B, self.NC, **f32)
        # the training head folded into the dense backward (csrc/kernels/bncnn.hip dense_bwd_kernel<true>):
        # dense_fwd stores the dropout keep flags in MFMA tile layout for it
        self.keep = torch.zeros(nrt * (self.Dp // 16) * 64, dtype=torch.int32, device=self.device)
        H0, W0, C0 = self.blocks[0]["geo"].H, self.blocks[0]["geo"].W, self.blocks[0]["geo"].C
        self.x_stride = H0 * W0 * C0
        self.opt = OptimizerKernel(store, optimizer, {}, self.iterations) if optimizer is not None else None
        self._bn_segs = self._bn_gradient_segments()
        self._opt_key_set = None
        self._push = None     # fused DP exchange (step mode "xgmi", set_push)
        self._pushed = False

    def head_fold_ok(self, B):
        """TDE_BNCNN_HEAD_FOLD=1: the training head runs inside the dense backward launch (one launch fewer per
        step) when its state fits one workgroup: B <= 128, Dp <= 224, NC <= 16 and the head's LDS (activations +
        Wh + dl + sums) <= 160 KiB.  Off by default: correct, but every dense-backward workgroup recomputes the head
        of all 128 rows (the dense BN's backward sums need every row's g), 18.5 us against the head launch's 7.7 us
        plus one boundary — Model B 1.019 M -> 0.920 M img/s (profiles/r6_head_fold/)."""
        if os.environ.get("TDE_BNCNN_HEAD_FOLD", "0") != "1" or self.device.type != "cuda":
            return False
        nrt, Dp = -(-B // 16), self.Dp
        lds = (nrt * 16 * (Dp + 4) + Dp * 17 + nrt * 16 * 17) * 4 + max(nrt * 2 * Dp * 8, 16 * 256 * 4)
        return B <= 128 and Dp <= 224 and self.D <= 256 and self.NC <= 16 and lds <= 160 * 1024

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
    def _bn(self, blk, mode, B):
        """Descriptor of a conv block's BN; its forward partials come from the block's conv workgroups."""
        g = blk["geo"]
        R = B * g.Ho * g.Wo
        return Bn(mode, g.Co, _P(blk["acc"]), int(B * blk["msplit"]), float(R), _P(blk["gamma"]), _P(blk["beta"]),
                  float(blk["eps"]), float(blk["momentum"]), float(R / max(R - 1, 1)), _P(blk["mmean"]),
                  _P(blk["mvar"]), _P(blk["saved"]))

    def _fwd_mode(self, training):
        if training == "train":
            return BN_TRAIN
        return BN_BATCH if training else BN_MOVING

    # ------------------------------------------------------------------ forward
    def _forward(self, x, B, phase, keep=False):
        """phase: "train" | True (batch statistics, no update: learning phase 1) | False (moving statistics)."""
        lib, s = self.lib, N.stream_ptr()
        mode = self._fwd_mode(phase)
        batch_stats = mode in (BN_TRAIN, BN_BATCH)
        inp = x
        bn_in = Bn(BN_NONE, self.blocks[0]["geo"].C)
        for li, blk in enumerate(self.blocks):
            # a training step's first launch advances the step counter (dropout seed, Adam's t)
            inc = _P(self.iterations) if (phase == "train" and li == 0) else None
            ws = _P(blk["wstack"]) if phase == "train" else None
            rc = lib.tde_bncnn_conv_fwd(C.byref(blk["geo"]), B, _P(inp), C.byref(bn_in), _P(blk["w"]), _P(blk["z"]),
                                        _P(blk["acc"]) if batch_stats else None, inc, ws, s)
            if rc != 0:
                raise RuntimeError(f"tde_bncnn_conv_fwd({blk['conv'].name}) failed with {rc}")
            bn_in = self._bn(blk, mode, B)
            inp = blk["z"]
        drop = keep and self.drop is not None and self.drop.rate > 0
        rc = lib.tde_bncnn_dense_fwd(B, self.K, self.D, self.Dp, _P(inp), C.byref(bn_in), _P(self.wd), _P(self.h),
                                     _P(self.hstat), _P(self.keep) if drop else None,
                                     float(self.drop.rate) if drop else 0.0, self.drop_seed if drop else 0,
                                     _P(self.iterations) if drop else None, 0, s)
        N.check(rc, "tde_bncnn_dense_fwd")
        return bn_in

    def _head(self, B, hmode, phase, labels, scale, probs=None):
        mode = self._fwd_mode(phase)
        bnd = self.bnd
        bn = Bn(mode, self.D, None, 0, float(B), _P(bnd["gamma"]), _P(bnd["beta"]), float(bnd["eps"]),
                float(bnd["momentum"]), 1.0, _P(bnd["mmean"]), _P(bnd["mvar"]), _P(bnd["saved"]))
        drop_on = int(self.drop is not None and self.drop.rate > 0 and phase is not False)
        train = hmode == 0
        rc = self.lib.tde_bncnn_head(
            B, self.D, self.Dp, self.NC, hmode, _P(self.h), _P(self.hstat), C.byref(bn),
            float(self.drop.rate if self.drop else 0.0), self.drop_seed, _P(self.iterations), 0, drop_on,
            _P(self.wh), _P(self.bh), _P(labels), float(scale), _P(self.metrics) if hmode != 2 else None, _P(probs),
            int(self.softmax), _P(self.dwh_part) if train else None, _P(self.dbh_part) if train else None,
            _P(self.gh) if train else None, _P(self.gstat) if train else None, N.stream_ptr())
        N.check(rc, "tde_bncnn_head")

    def dropout_mask(self, B=None):
        """Debug export: the [B, D] keep scales (1/(1-rate) kept, 0 dropped) the head applies at the
        current step counter (read on the device, so call it after the step's forward advanced it)."""
        B = self.B if B is None else B
        if self.drop is None or not self.drop.rate > 0:
            return torch.ones(B, self.D, dtype=torch.float32, device=self.device)
        out = torch.empty(B, self.D, dtype=torch.float32, device=self.device)
        rc = self.lib.tde_bncnn_dropout_mask(B, self.D, float(self.drop.rate), self.drop_seed, _P(self.iterations), 0,
                                             _P(out), N.stream_ptr())
        N.check(rc, "tde_bncnn_dropout_mask")
        return out

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
        fold = self.head_fold_ok(B)
        self._forward(x, B, "train", keep=fold)
        last = self.blocks[-1]
        bn_last = self._bn(last, BN_SAVED, B)
        bnd = self.bnd
        if fold:
            # the head inside the dense backward: the dense BN in training mode (its statistics, saved / moving
            # update), the dropout flags dense_fwd stored
            bn_t = Bn(BN_TRAIN, self.D, None, 0, float(B), _P(bnd["gamma"]), _P(bnd["beta"]), float(bnd["eps"]),
                      float(bnd["momentum"]), 1.0, _P(bnd["mmean"]), _P(bnd["mvar"]), _P(bnd["saved"]))
            drop = self.drop is not None and self.drop.rate > 0
            rc = lib.tde_bncnn_dense_bwd_head(
                B, self.K, self.D, self.Dp, self.NC, _P(last["z"]), C.byref(bn_last), _P(self.wd), _P(self.h),
                _P(self.hstat), C.byref(bn_t), _P(self.keep) if drop else None,
                float(self.drop.rate) if drop else 0.0, _P(self.wh), _P(self.bh), _P(y), float(self.scale),
                _P(self.metrics), _P(self.dwh_part), _P(self.dbh_part), _P(bnd["dbeta"]), _P(bnd["dgamma"]),
                _P(self.dwd_part), _P(last["g"]), _P(last["accb"]), s)
            N.check(rc, "tde_bncnn_dense_bwd_head")
        else:
            self._head(B, 0, "train", y, self.scale)
            bn_d = Bn(BN_SAVED, self.D, None, 0, float(B), _P(bnd["gamma"]), _P(bnd["beta"]), float(bnd["eps"]),
                      float(bnd["momentum"]), 1.0, _P(bnd["mmean"]), _P(bnd["mvar"]), _P(bnd["saved"]))
            rc = lib.tde_bncnn_dense_bwd(B, self.K, self.D, self.Dp, _P(last["z"]), C.byref(bn_last), _P(self.wd),
                                         _P(self.gh), _P(self.h), _P(self.gstat), -(-B // 16), C.byref(bn_d),
                                         _P(bnd["dbeta"]), _P(bnd["dgamma"]), _P(self.dwd_part), _P(last["g"]),
                                         _P(last["accb"]), s)
            N.check(rc, "tde_bncnn_dense_bwd")
        # backward partials of block li's BN: from the dense backward (last block) or from the input-gradient
        # role of block li + 1's conv backward (one per image)
        nkt_nrb = -(-self.K // 32) * -(-B // 64)
        for li in range(len(self.blocks) - 1, -1, -1):
            blk = self.blocks[li]
            npart = nkt_nrb if li == len(self.blocks) - 1 else B
            bb = BnBwd(_P(blk["accb"]), int(npart), _P(blk["dbeta"]), _P(blk["dgamma"]))
            if li > 0:
                prev = self.blocks[li - 1]
                inp, bn_in, gin, acc_in = prev["z"], self._bn(prev, BN_SAVED, B), prev["g"], prev["accb"]
            else:
                inp, bn_in, gin, acc_in = x, Bn(BN_NONE, blk["geo"].C), None, None
            rc = lib.tde_bncnn_conv_bwd(C.byref(blk["geo"]), B, _P(blk["z"]), C.byref(self._bn(blk, BN_SAVED, B)),
                                        C.byref(bb), _P(blk["g"]), _P(blk["w"]), _P(inp), C.byref(bn_in), _P(gin),
                                        _P(acc_in), _P(blk["dwpart"]), int(li > 0),
                                        _P(blk["wstack"]) if li > 0 else None, s)
            if rc != 0:
                raise RuntimeError(f"tde_bncnn_conv_bwd({blk['conv'].name}) failed with {rc}")
        # weight-gradient partials -> the bucket: per image for the convs, per 64-row block for the dense
        # (fused step: the optimizer applied in the same launch, BN gradients included)
        segs = [(b["dwpart"], b["gw"], b["K"] * b["geo"].Co, B) for b in self.blocks]
        segs.append((self.dwd_part, self.gwd, self.K * self.D, -(-B // 64)))
        segs.append((self.dwh_part, self.gwh, self.D * self.NC, -(-B // 16)))
        segs.append((self.dbh_part, self.gbh, self.NC, -(-B // 16)))
        opt = None
        if self.step_mode == "local":
            segs += self._bn_segs
            opt = C.byref(self._bnopt)
        # fused DP exchange: the Dense kernel's summed gradient (segment len(blocks)) goes to the xGMI owners
        push = self._push if self.step_mode == "xgmi" else None
        self._pushed = push is not None
        n = len(segs)
        cnt = (C.c_int * n)(*[sg[3] for sg in segs])
        parts = (C.c_void_p * n)(*[sg[0].data_ptr() for sg in segs])
        outs = (C.c_void_p * n)(*[sg[1].data_ptr() for sg in segs])
        lens = (C.c_longlong * n)(*[sg[2] for sg in segs])
        N.check(lib.tde_bncnn_reduce(n, cnt, parts, outs, lens, opt, len(self.blocks),
                                     C.byref(push) if push is not None else None, s), "tde_bncnn_reduce")

    # ------------------------------------------------------------------ fused optimizer ("local")
    def supports_step_mode(self, mode):
        if mode == "plain":
            return True
        if mode == "xgmi":   # data parallel: the xGMI all-reduce applies the update to the f32 weights
            return self.optimizer is not None and self.device.type == "cuda"
        return mode == "local" and self.optimizer is not None and self.device.type == "cuda" and \
            self._bn_segs is not None

    def xg_apply_spec(self):
        from .program import f32_xg_apply_spec
        return f32_xg_apply_spec(self)

    def push_range(self):
        """Bucket range the reduce launch can push into the xGMI owners itself: the Dense(200) kernel's
        gradient (94 % of Model B's gradient bytes)."""
        seg = self.store.segments[f"{self.dense.name}/kernel"]
        return seg.offset, seg.offset + seg.numel

    def set_push(self, spec):
        if spec is not None and self.step_mode != "xgmi":
            raise ValueError("the fused exchange needs step mode 'xgmi'")
        self._push = spec

    def set_step_mode(self, mode):
        super().set_step_mode(mode)
        if mode != "xgmi":
            self._push = None
        self._opt_key_set = self._opt_key()
        if mode == "local":
            o, st = self.optimizer, self.store
            sl = o.slot_names()
            m = st.slot(sl[0]) if sl else None
            v = st.slot(sl[1]) if len(sl) > 1 else None
            hp = o.hparams()
            self._bnopt = BnOpt(o.kind_id, float(o.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"],
                                _P(st.g), _P(st.w), _P(m), _P(v), _P(self.iterations))

    def _opt_key(self):
        o = self.optimizer
        return (o.kind_id, float(o.learning_rate), tuple(sorted(o.hparams().items()))) if o is not None else None

    def refresh(self):
        # the launch descriptor carries lr / hyper-parameters by value
        if self.step_mode == "local" and self._opt_key_set != self._opt_key():
            self.set_step_mode("local")

    def _bn_gradient_segments(self):
        """(part, out, len, 1) of every BN gamma / beta gradient (the backward writes them into the bucket),
        or None when the fused reduce would not cover every trainable variable."""
        segs, names = [], set()
        for blk in self.blocks + [self.bnd]:
            for key, var in (("dbeta", "beta"), ("dgamma", "gamma")):
                if blk.get(key) is not None:
                    g = blk[key]
                    segs.append((g, g, g.numel(), 1))
        covered = {g.data_ptr() for g, *_ in segs}
        for b in self.blocks:
            covered.add(b["gw"].data_ptr())
        covered |= {self.gwd.data_ptr(), self.gwh.data_ptr(), self.gbh.data_ptr()}
        for name in self.store.names(trainable=True):
            if self.store.grad(name).data_ptr() not in covered:
                return None
        return segs

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
