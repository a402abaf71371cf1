"""Host wrappers for the float32 layer-wise kernel library (csrc/kernels/layers_f32.hip).

The float32 twin of ``layer_ops``: activations, activation gradients and logits are f32, the GEMMs read
the f32 master kernels in their Keras layouts (HWIO conv kernels, [in, out] dense kernels) on the
exact-f32 MFMA, BN statistics / backward sums are f64.  Every wrapper validates operand sizes on the host
against the geometry it hands the kernel, so a kernel never indexes outside its buffers.
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native as N
from .layer_ops import (A_COLM, A_CONV, A_DGRAD, A_ROWK, A_WGRAD, B_DGRADW, B_KN, B_NK, STAT_SLOTS, ConvGeom, DropSpec,
                        dgrad_phases)

_P = N.ptr
_vp, _i, _i64, _f, _u64 = C.c_void_p, C.c_int, C.c_longlong, C.c_float, C.c_ulonglong
N.register_hip({
    # a, lda, akind, b, ldb, bkind, M, N, K, geo, c, ldc, accum, bias, relu, colstats, splits, part, phase, stream
    "tde_igemm32": (_i, [_vp, _i64, _i, _vp, _i64, _i, _i, _i, _i, _vp, _vp, _i64, _i, _vp, _i, _vp, _i, _vp, _vp,
                         _vp]),
    "tde_colstats32": (_i, [_vp, _i64, _i, _vp, _vp]),
    "tde_bn_fwd32": (_i, [_vp, _vp, _vp, _i64, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _f, _f, _vp, _i, _f, _u64,
                          _vp, _i, _i, _vp]),
    "tde_bn_bwd32": (_i, [_vp, _vp, _vp, _i64, _i, _i, _vp, _vp, _vp, _i, _f, _u64, _vp, _i, _i, _vp, _vp, _i, _vp,
                          _i, _vp, _vp, _vp, _vp]),
    "tde_act_bwd32": (_i, [_vp, _vp, _i64, _i, _i, _vp, _vp, _vp]),
    "tde_maxpool32": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _vp]),
    "tde_maxpool32_bwd_relu": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "tde_gap32": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "tde_pad32": (_i, [_vp, _vp, _vp, _i, _i, _vp]),
    "tde_xent32": (_i, [_vp, _vp, _i, _i, _f, _vp, _vp, _vp, _i, _vp, _vp]),
})

_NODROP = DropSpec()


def _s():
    return N.stream_ptr()


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def _f32(t, n, what):
    _req(t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= n,
         f"{what}: f32 [{n}] expected")


def _f64(t, n, what):
    _req(t is not None and t.dtype == torch.float64 and t.is_contiguous() and t.numel() >= n,
         f"{what}: f64 [{n}] expected")


def tiles(M, N_):
    """Output tiles of an igemm32 launch (64 x 64 by default: layers_f32.hip tile_n)."""
    return -(-M // 64) * -(-N_ // 64)


def wgrad_splits(M, N_, K, target=256):
    """Split-K factor of a weight-gradient GEMM: its output tiles alone rarely fill the 256 CUs while its
    K (= pixels x batch) is long; the partials are summed in split order (deterministic)."""
    tiles_ = tiles(M, N_)
    chunks = -(-K // 16)
    if tiles_ >= target or chunks < 16:
        return 1
    return max(1, min(-(-target // tiles_), chunks // 8))


def wgrad_part_elems(M, N_, K):
    s = wgrad_splits(M, N_, K)
    return s * M * N_ if s > 1 else 0


def fd_splits(M, N_, K, target=256):
    """Split-K factor of a forward / input-gradient GEMM whose output tiles are too few to fill the chip
    while K is long (a Dense layer on a wide flattened input: M = batch, K = 10,816); the partials are
    summed in split order by the reduce launch, which then applies bias / ReLU / BN statistics."""
    tiles_ = tiles(M, N_)
    chunks = -(-K // 16)
    if tiles_ >= 128 or chunks < 32:
        return 1
    return max(1, min(-(-target // tiles_), chunks // 8))


def fd_part_elems(M, N_, K):
    s = fd_splits(M, N_, K)
    return s * M * N_ if s > 1 else 0


def _fd(M, N_, K, part):
    s = fd_splits(M, N_, K) if part is not None else 1
    return (s, part) if s > 1 and part.numel() >= s * M * N_ else (1, None)


def igemm32(a, lda, ak, b, ldb, bk, M, N_, K, c, ldc, *, geo=None, accum=False, bias=None, relu=False,
            colstats=None, splits=1, part=None, phase=None):
    if splits > 1:
        _f32(part, splits * M * N_, "igemm32 split-K partials")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * N_, "igemm32 colstats")
    ph = (C.c_int * len(phase))(*phase) if phase is not None else None
    rc = N.hip().tde_igemm32(_P(a), int(lda), ak, _P(b), int(ldb), bk, int(M), int(N_), int(K),
                             geo.carray() if geo is not None else None, _P(c), int(ldc), int(accum), _P(bias),
                             int(relu), _P(colstats), int(splits), _P(part), ph, _s())
    N.check(rc, "tde_igemm32")


# ---------------------------------------------------------------- Conv2D / Dense
def conv_fwd(x, W, y, g: ConvGeom, bias=None, relu=False, colstats=None, part=None):
    """y[B*Ho*Wo, Co] = conv(x, W) (+bias, ReLU, BN statistics); W the HWIO f32 master kernel."""
    _f32(x, g.B * g.H * g.W * g.C, "conv_fwd x")
    _f32(W, g.K * g.Co, "conv_fwd W")
    _f32(y, g.B * g.Ho * g.Wo * g.Co, "conv_fwd y")
    M = g.B * g.Ho * g.Wo
    s, pt = _fd(M, g.Co, g.K, part)
    igemm32(x, 0, A_CONV, W, g.Co, B_KN, M, g.Co, g.K, y, g.Co, geo=g, bias=bias, relu=relu,
            colstats=colstats, splits=s, part=pt)


def conv_dgrad(dy, W, dx, g: ConvGeom, accum=False, part=None):
    """dx = conv input gradient.  Strided convs run every stride phase in ONE launch, each phase over only
    the taps that reach its pixels (the other (s^2-1)/s^2 of the implicit-GEMM K would multiply zeros)."""
    _f32(dy, g.B * g.Ho * g.Wo * g.Co, "conv_dgrad dy")
    _f32(W, g.K * g.Co, "conv_dgrad W")
    _f32(dx, g.B * g.H * g.W * g.C, "conv_dgrad dx")
    if g.sh > 1 or g.sw > 1:
        phases = dgrad_phases(g)
        if 1 <= len(phases) <= 4 and len(phases) == g.sh * g.sw:
            table = [len(phases)] + [v for ph in phases for v in ph]
            Mx = max(g.B * ph[2] * ph[3] for ph in phases)
            Kx = max(ph[6] * ph[7] * g.Co for ph in phases)
            igemm32(dy, 0, A_DGRAD, W, 0, B_DGRADW, Mx, g.C, Kx, dx, g.C, geo=g, accum=accum, phase=table)
            return
    M, K = g.B * g.H * g.W, g.KH * g.KW * g.Co
    s, pt = _fd(M, g.C, K, part)
    igemm32(dy, 0, A_DGRAD, W, 0, B_DGRADW, M, g.C, K, dx, g.C, geo=g, accum=accum, splits=s, part=pt)


def conv_wgrad(x, dy, dW, g: ConvGeom, part=None):
    """dW[KH*KW*C, Co] = sum over pixels x (patch) . dy (stored)."""
    _f32(x, g.B * g.H * g.W * g.C, "conv_wgrad x")
    _f32(dy, g.B * g.Ho * g.Wo * g.Co, "conv_wgrad dy")
    _f32(dW, g.K * g.Co, "conv_wgrad dW")
    K = g.B * g.Ho * g.Wo
    s = wgrad_splits(g.K, g.Co, K) if part is not None else 1
    igemm32(x, 0, A_WGRAD, dy, g.Co, B_KN, g.K, g.Co, K, dW, g.Co, geo=g, splits=s, part=part)


def dense_fwd(x, W, rows, y, bias=None, relu=False, colstats=None, part=None):
    fin, fout = W.shape
    _f32(x, rows * fin, "dense_fwd x")
    _f32(y, rows * fout, "dense_fwd y")
    s, pt = _fd(rows, fout, fin, part)
    igemm32(x, fin, A_ROWK, W, fout, B_KN, rows, fout, fin, y, fout, bias=bias, relu=relu, colstats=colstats,
            splits=s, part=pt)


def dense_dgrad(dy, W, dx, rows, accum=False, part=None):
    fin, fout = W.shape
    _f32(dy, rows * fout, "dense_dgrad dy")
    _f32(dx, rows * fin, "dense_dgrad dx")
    s, pt = _fd(rows, fin, fout, part)
    igemm32(dy, fout, A_ROWK, W, fout, B_NK, rows, fin, fout, dx, fin, accum=accum, splits=s, part=pt)


def dense_wgrad(x, dy, dW, rows, part=None):
    fin, fout = dW.shape
    _f32(x, rows * fin, "dense_wgrad x")
    _f32(dy, rows * fout, "dense_wgrad dy")
    s = wgrad_splits(fin, fout, rows) if part is not None else 1
    igemm32(x, fin, A_COLM, dy, fout, B_KN, fin, fout, rows, dW, fout, splits=s, part=part)


# ---------------------------------------------------------------- BatchNormalization / activations
def colstats(x, R, Cc, stats):
    _f32(x, R * Cc, "colstats32 x")
    _f64(stats, 2 * STAT_SLOTS * Cc, "colstats32 stats")
    N.check(N.hip().tde_colstats32(_P(x), int(R), int(Cc), _P(stats), _s()), "tde_colstats32")


def bn_fwd(y, out, R, Cc, *, mode, stats=None, saved=None, gamma=None, beta=None, eps=1e-3, mmean=None, mvar=None,
           momentum=0.99, bessel=1.0, zero_buf=None, res=None, relu=False, drop: DropSpec = _NODROP, iter_offset=0):
    """out = dropout(relu(bn(y) + res)); mode 0 identity, 1 batch stats (from ``stats``), 2 moving stats."""
    n = R * Cc
    _f32(y, n, "bn_fwd32 y")
    _f32(out, n, "bn_fwd32 out")
    _req(Cc <= 2048, "bn_fwd32: at most 2048 channels")
    if res is not None:
        _f32(res, n, "bn_fwd32 res")
    if mode == 1:
        _f64(stats, 2 * STAT_SLOTS * Cc, "bn_fwd32 stats")
        _f32(saved, 2 * Cc, "bn_fwd32 saved")
    if mode == 2:
        _f32(mmean, Cc, "bn_fwd32 moving_mean")
        _f32(mvar, Cc, "bn_fwd32 moving_variance")
    if zero_buf is not None:
        _f64(zero_buf, 2 * STAT_SLOTS * Cc, "bn_fwd32 zero_buf")
    rc = N.hip().tde_bn_fwd32(_P(y), _P(out), _P(res), int(R), int(Cc), int(mode), _P(stats), _P(saved), _P(gamma),
                              _P(beta), float(eps), _P(mmean), _P(mvar), float(momentum), float(bessel), _P(zero_buf),
                              int(relu), float(drop.rate), int(drop.seed) & (2 ** 64 - 1), _P(drop.iterations),
                              int(iter_offset), int(drop.layer_id), _s())
    N.check(rc, "tde_bn_fwd32")


def bn_bwd(dout, y, R, Cc, *, mode, saved=None, gamma=None, beta=None, res=None, relu=False,
           drop: DropSpec = _NODROP, iter_offset=-1, dstats=None, dx=None, dx_accum=False, dres=None,
           dres_accum=False, dgamma=None, dbeta=None, zero_fwd=None):
    n = R * Cc
    _f32(dout, n, "bn_bwd32 dout")
    _f32(y, n, "bn_bwd32 y")
    _req(Cc <= 2048, "bn_bwd32: at most 2048 channels")
    if mode == 1:
        _f32(saved, 2 * Cc, "bn_bwd32 saved")
        _f64(dstats, 2 * STAT_SLOTS * Cc, "bn_bwd32 dstats")
    if zero_fwd is not None:
        _f64(zero_fwd, 2 * STAT_SLOTS * Cc, "bn_bwd32 zero_fwd")
    for t, what in ((dx, "dx"), (dres, "dres"), (res, "res")):
        if t is not None:
            _f32(t, n, f"bn_bwd32 {what}")
    rc = N.hip().tde_bn_bwd32(_P(dout), _P(y), _P(res), int(R), int(Cc), int(mode), _P(saved), _P(gamma), _P(beta),
                              int(relu), float(drop.rate), int(drop.seed) & (2 ** 64 - 1), _P(drop.iterations),
                              int(iter_offset), int(drop.layer_id), _P(dstats), _P(dx), int(dx_accum), _P(dres),
                              int(dres_accum), _P(dgamma), _P(dbeta), _P(zero_fwd), _s())
    N.check(rc, "tde_bn_bwd32")


def act_bwd(dout, out, R, Cc, *, relu, dz=None, dbias=None):
    n = R * Cc
    _f32(dout, n, "act_bwd32 dout")
    if relu:
        _f32(out, n, "act_bwd32 out")
    if dz is not None:
        _f32(dz, n, "act_bwd32 dz")
    if dbias is not None:
        _f32(dbias, Cc, "act_bwd32 dbias")
    rc = N.hip().tde_act_bwd32(_P(dout), _P(out), int(R), int(Cc), int(relu), _P(dz), _P(dbias), _s())
    N.check(rc, "tde_act_bwd32")


# ---------------------------------------------------------------- pooling / padding / head
def maxpool_fwd(x, y, idx, g: ConvGeom):
    _f32(x, g.B * g.H * g.W * g.C, "maxpool32 x")
    _f32(y, g.B * g.Ho * g.Wo * g.C, "maxpool32 y")
    _req(idx is None or (idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * g.C), "maxpool32 idx")
    N.check(N.hip().tde_maxpool32(_P(x), _P(y), _P(idx), None, None, 0, g.carray(), 0, _s()), "tde_maxpool32")


def maxpool_bwd(dy, idx, dx, g: ConvGeom, accum=False):
    _f32(dy, g.B * g.Ho * g.Wo * g.C, "maxpool32 dy")
    _f32(dx, g.B * g.H * g.W * g.C, "maxpool32 dx")
    _req(idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * g.C, "maxpool32 idx")
    N.check(N.hip().tde_maxpool32(None, None, _P(idx), _P(dy), _P(dx), int(accum), g.carray(), 1, _s()),
            "tde_maxpool32")


def maxpool_bwd_relu(dy, y, idx, dx, g: ConvGeom, dbias=None, accum=False):
    """Max-pool backward fused with the producer's ReLU (+ bias) backward: dx = dy * (y > 0) at each window's
    winner, 0 elsewhere; dbias += the column sums of that over the pooled cells.  Non-overlapping windows."""
    _f32(dy, g.B * g.Ho * g.Wo * g.C, "maxpool_bwd_relu dy")
    _f32(y, g.B * g.Ho * g.Wo * g.C, "maxpool_bwd_relu y")
    _f32(dx, g.B * g.H * g.W * g.C, "maxpool_bwd_relu dx")
    _req(idx.numel() >= g.B * g.Ho * g.Wo * g.C and (dbias is None or dbias.numel() == g.C), "maxpool_bwd_relu")
    N.check(N.hip().tde_maxpool32_bwd_relu(_P(dy), _P(y), _P(idx), _P(dx), _P(dbias), int(accum), g.carray(), _s()),
            "tde_maxpool32_bwd_relu")


def pool_relu_fusable(g: ConvGeom):
    return g.C % 4 == 0 and g.sh >= g.KH and g.sw >= g.KW and g.KH * g.KW <= 255


def gap_fwd(x, y, B, HW, Cc):
    _f32(x, B * HW * Cc, "gap32 x")
    _f32(y, B * Cc, "gap32 y")
    N.check(N.hip().tde_gap32(_P(x), _P(y), int(B), int(HW), int(Cc), 0, 0, _s()), "tde_gap32")


def gap_bwd(dy, dx, B, HW, Cc, accum=False):
    _f32(dy, B * Cc, "gap32 dy")
    _f32(dx, B * HW * Cc, "gap32 dx")
    N.check(N.hip().tde_gap32(_P(dy), _P(dx), int(B), int(HW), int(Cc), 1, int(accum), _s()), "tde_gap32")


def pad_fwd(x, y, g: ConvGeom):
    _f32(x, g.B * g.H * g.W * g.C, "pad32 x")
    _f32(y, g.B * g.Ho * g.Wo * g.C, "pad32 y")
    N.check(N.hip().tde_pad32(_P(x), _P(y), g.carray(), 0, 0, _s()), "tde_pad32")


def pad_bwd(dy, dx, g: ConvGeom, accum=False):
    _f32(dy, g.B * g.Ho * g.Wo * g.C, "pad32 dy")
    _f32(dx, g.B * g.H * g.W * g.C, "pad32 dx")
    N.check(N.hip().tde_pad32(_P(dy), _P(dx), g.carray(), 1, int(accum), _s()), "tde_pad32")


def xent(logits, labels, B, Cc, *, scale=1.0, dlogits=None, metrics=None, probs=None, probs_are_logits=False,
         iterations=None):
    _f32(logits, B * Cc, "xent32 logits")
    _req(labels.dtype == torch.int32 and labels.numel() >= B, "xent32 labels")
    if dlogits is not None:
        _f32(dlogits, B * Cc, "xent32 dlogits")
    if probs is not None:
        _f32(probs, B * Cc, "xent32 probs")
    rc = N.hip().tde_xent32(_P(logits), _P(labels), int(B), int(Cc), float(scale), _P(dlogits), _P(metrics),
                            _P(probs), int(probs_are_logits), _P(iterations), _s())
    N.check(rc, "tde_xent32")
