"""Thin, allocation-free Python entry points to the gfx950 HIP kernels.

Every function takes pre-allocated device tensors, enqueues on the current HIP
stream (so it is hipGraph-capturable), and raises if the native call reports an
error.  Shapes are validated on the host before launch: a kernel never sees an
operand shape it does not support (a faulting kernel can reset the node).
"""
from __future__ import annotations

import ctypes as _ct

import torch

from .. import _native as N

_P = N.ptr

_FLAT_RANGES = 4


class OptHyper(_ct.Structure):
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float)]


class StepOpt(_ct.Structure):
    """``TdeStepOpt`` (csrc/kernels/convnet.hip): the optimizer of a fused training step."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float), ("w", _ct.c_void_p), ("g", _ct.c_void_p), ("m", _ct.c_void_p), ("v", _ct.c_void_p),
                ("iterations", _ct.c_void_p), ("pend", _ct.c_void_p), ("grep", _ct.c_int),
                ("grep_stride", _ct.c_longlong), ("fly_count", _ct.c_void_p), ("hsrc_w2", _ct.c_void_p),
                ("hsrc_b2", _ct.c_void_p), ("hsrc_b1", _ct.c_void_p), ("hsnap", _ct.c_void_p), ("hC", _ct.c_int)]


class FlatApply(_ct.Structure):
    """``FlatApply`` (csrc/include/tde_optim.h): an update of element ranges of the flat buffers."""
    _fields_ = [("w", _ct.c_void_p), ("g", _ct.c_void_p), ("m", _ct.c_void_p), ("v", _ct.c_void_p),
                ("iterations", _ct.c_void_p), ("pend", _ct.c_void_p), ("h", OptHyper), ("nr", _ct.c_int),
                ("lo", _ct.c_int * _FLAT_RANGES), ("n", _ct.c_int * _FLAT_RANGES), ("grep", _ct.c_int),
                ("grep_stride", _ct.c_longlong), ("count", _ct.c_void_p)]


class XgApply(_ct.Structure):
    """``TdeXgApply`` (csrc/comm/xgmi_allreduce.hip): the optimizer fused into the all-reduce."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float), ("w", _ct.c_void_p), ("m", _ct.c_void_p), ("v", _ct.c_void_p),
                ("iterations", _ct.c_void_p), ("sh", _ct.c_void_p), ("sh_lo", _ct.c_longlong), ("sh_hi", _ct.c_longlong),
                ("sht", _ct.c_void_p), ("sh_cols", _ct.c_int), ("sht_ld", _ct.c_longlong),
                ("push_lo", _ct.c_longlong), ("push_hi", _ct.c_longlong), ("rep", _ct.c_void_p), ("nrep", _ct.c_int),
                ("rep_lo", _ct.c_longlong), ("rep_hi", _ct.c_longlong), ("rep_stride", _ct.c_longlong)]


class XgPush(_ct.Structure):
    """``TdeXgPush`` / ``XgPush`` (csrc/include/tde_xgmi.h): a producer kernel stores its gradient range
    straight into the owners' contribution areas of the next xGMI all-reduce call."""
    _fields_ = [("peer", _ct.c_void_p * 8), ("epoch", _ct.c_void_p), ("L", _ct.c_longlong), ("cap", _ct.c_longlong),
                ("off", _ct.c_longlong), ("rank", _ct.c_int), ("nranks", _ct.c_int)]


class BwdOpt(_ct.Structure):
    """``TdeBwdOpt`` (csrc/kernels/convnet.hip): the fused-step part of the trunk backward."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float),
                ("b2", _ct.c_float), ("eps", _ct.c_float), ("w", _ct.c_void_p), ("m", _ct.c_void_p),
                ("v", _ct.c_void_p), ("off_w1", _ct.c_longlong), ("off_w2", _ct.c_longlong),
                ("off_b2", _ct.c_longlong), ("off_b1", _ct.c_longlong), ("W1c", _ct.c_void_p),
                ("ldw1c", _ct.c_int), ("iterations", _ct.c_void_p), ("iter_prev", _ct.c_void_p),
                ("commit", FlatApply), ("pend_set", _ct.c_void_p), ("crep", _ct.c_int),
                ("crep_stride", _ct.c_longlong)]


def step_opt(optimizer, w, g, m, v, iterations, pend):
    hp = optimizer.hparams()
    return StepOpt(optimizer.kind_id, float(optimizer.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"],
                   _P(w), _P(g), _P(m), _P(v), _P(iterations), _P(pend))


def flat_apply_spec(optimizer, w, g, m, v, iterations, pend, ranges):
    """ranges: [(lo, n), ...] element ranges of the flat buffers (<= 4)."""
    _req(len(ranges) <= _FLAT_RANGES, "flat_apply: at most 4 ranges")
    hp = optimizer.hparams()
    f = FlatApply()
    f.w, f.g, f.m, f.v = _P(w), _P(g), _P(m), _P(v)
    f.iterations, f.pend = _P(iterations), _P(pend)
    f.h = OptHyper(optimizer.kind_id, float(optimizer.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"])
    f.nr = len(ranges)
    for i, (lo, n) in enumerate(ranges):
        f.lo[i], f.n[i] = int(lo), int(n)
    return f


def flat_apply(spec: FlatApply):
    """One-workgroup update of ``spec``'s ranges (skipped while ``*pend == 0``; clears ``*pend``)."""
    rng = (_ct.c_int * (2 * _FLAT_RANGES))()
    for i in range(spec.nr):
        rng[2 * i], rng[2 * i + 1] = spec.lo[i], spec.n[i]
    h = spec.h
    rc = N.hip().tde_flat_apply(spec.w, spec.g, spec.m, spec.v, spec.iterations, spec.pend, h.kind, h.lr, h.mom,
                                h.b1, h.b2, h.eps, rng, spec.nr, int(spec.grep), int(spec.grep_stride), spec.count,
                                _s())
    N.check(rc, "tde_flat_apply")


def _s():
    return N.stream_ptr()


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def gemm_pick_splits(M, N_, K):
    return N.hip().tde_gemm_pick_splits(M, N_, K)


def gemm_nt(A, Bt, C, *, M=None, N_=None, K=None, alpha=1.0, mode="store", splits=0,
            bias=None, relu=False, Cbf=None):
    """C[M,N] (=, +=, atomic+=) alpha * A[M,K] @ Bt[N,K]^T with bf16 operands (MFMA)."""
    _req(A.dtype == torch.bfloat16 and Bt.dtype == torch.bfloat16, "gemm_nt: bf16 operands")
    _req(A.stride(-1) == 1 and Bt.stride(-1) == 1, "gemm_nt: K-contiguous operands")
    M = A.shape[0] if M is None else M
    K = A.shape[1] if K is None else K
    N_ = Bt.shape[0] if N_ is None else N_
    lda, ldb = A.stride(0), Bt.stride(0)
    _req(lda % 8 == 0 and ldb % 8 == 0, "gemm_nt: leading dims must be multiples of 8")
    _req(A.shape[0] >= M and Bt.shape[0] >= N_ and A.shape[1] >= K and Bt.shape[1] >= K, "gemm_nt: shape")
    m = {"store": 0, "accum": 1, "atomic": 2}[mode]
    ldc = C.stride(0) if C is not None else N_
    if C is not None:
        _req(C.dtype == torch.float32 and C.shape[0] >= M and C.shape[1] >= N_, "gemm_nt: C shape")
    ldcb = Cbf.stride(0) if Cbf is not None else 0
    rc = N.hip().tde_gemm_nt_bf16(_P(A), lda, _P(Bt), ldb, _P(C), ldc, M, N_, K, float(alpha), m,
                                  int(splits), _P(bias), int(relu), _P(Cbf), ldcb, _s())
    N.check(rc, "tde_gemm_nt_bf16")


def conv3x3c1_relu_pool_fwd(x, w, b, P, Pt, amax, zbuf=None):
    """x[B,H,W,1] f32 -> P[B,Hp*Wp*C] bf16, Pt[Hp*Wp*C, ldPt] bf16, amax u8."""
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    C = w.shape[-1]
    _req(w.numel() == 9 * C and C % 16 == 0 and W % 2 == 0, "conv3x3c1: unsupported shape")
    Hp, Wp = (H - 2) // 2, (W - 2) // 2
    K = Hp * Wp * C
    _req(P.shape[0] >= B and P.shape[1] == K and amax.shape == P.shape, "conv3x3c1: output shape")
    ldPt = 0
    if Pt is not None:
        ldPt = Pt.stride(0)
        _req(Pt.shape[0] == K and ldPt >= B and ldPt % 8 == 0, "conv3x3c1: Pt shape")
    zn = 0 if zbuf is None else zbuf.numel()
    rc = N.hip().tde_conv3x3c1_relu_pool_fwd(_P(x), _P(w), _P(b), _P(P), _P(Pt), ldPt, _P(amax), B, H, W,
                                             C, _P(zbuf), zn, _s())
    N.check(rc, "tde_conv3x3c1_relu_pool_fwd")


def conv3x3c1_relu_pool_bwd(x, amax, G, W1, dw, db):
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    C = dw.shape[-1]
    Hd = G.shape[1]
    _req(W1.shape[1] == Hd and G.stride(0) % 8 == 0 and W1.stride(0) % 8 == 0, "conv bwd: shapes")
    _req(C % 16 == 0 and C <= 256, "conv bwd: C")
    rc = N.hip().tde_conv3x3c1_relu_pool_bwd(_P(x), _P(amax), _P(G), G.stride(0), _P(W1), W1.stride(0), Hd,
                                             _P(dw), _P(db), B, H, W, C, _s())
    N.check(rc, "tde_conv3x3c1_relu_pool_bwd")


def head_xent(hin, W2, b2, labels, *, B, scale, pre_bias=None, pre_relu=False, compute_grad=True,
              dW2=None, db2=None, dpre_bias=None, G=None, Gt=None, Gf=None, metrics=None,
              probs=None, probs_are_logits=False, row_loss=None, zero_hin=False, iterations=None, stamps=None):
    H, C = W2.shape
    hb = hin.dtype == torch.bfloat16
    _req((hin.dtype == torch.float32 or hb and not zero_hin) and hin.dim() == 2 and hin.shape[1] >= H
         and hin.stride(1) == 1, "head: f32 or bf16 [B, H] input")
    _req(C <= 64 and H * C <= 16384, "head: too large for the fused head")
    _req(labels.dtype == torch.int32, "head: int32 labels")
    ldg = G.stride(0) if G is not None else 0
    ldgt = Gt.stride(0) if Gt is not None else 0
    ldgf = Gf.stride(0) if Gf is not None else 0
    rc = N.hip().tde_head_xent(_P(hin), hin.stride(0), _P(pre_bias), int(pre_relu), _P(W2), _P(b2), _P(labels),
                               B, H, C, float(scale), int(compute_grad), _P(dW2), _P(db2), _P(dpre_bias),
                               _P(G), ldg, _P(Gt), ldgt, _P(Gf), ldgf, _P(metrics), _P(probs),
                               int(probs_are_logits), _P(row_loss), int(zero_hin), _P(iterations), _P(stamps),
                               int(hb), _s())
    N.check(rc, "tde_head_xent")


def convnet_fwd(x, wc, bc, W1, hpre, Pt=None, amax=None, stamps=None, *, opt: StepOpt | None = None,
                off_wc=0, off_bc=0, inc_iter=None, hrep=1):
    """Fused Conv2D(32,3x3,relu)+MaxPool(2)+Dense(64) matmul forward; hpre += (atomic).

    Precision follows W1: a bf16 Dense(64) kernel shadow, row-major [K, 64] or transposed [64, K],
    runs the bf16 MFMA form (csrc/kernels/convnet.hip); the f32 master kernel [K, 64] runs the
    float32 form (csrc/kernels/convnet_f32.hip, exact-f32 MFMA), whose Pt must then be f32 too.
    amax: uint8 view of a [P, 4, lda] uint64 buffer (lane-contiguous pool argmax).
    opt (fused step): while ``*opt.pend`` the conv weights used are the optimizer step of
    (w, g) at offsets off_wc / off_bc of the flat buffers (the deferred update).
    inc_iter (training): the int64 step counter, advanced by one.
    hrep: hpre is [hrep, >=B, 64] replicas (workgroup i adds into replica i % hrep) or [>=B, 64]."""
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    Kf = ((H - 2) // 2) * ((W - 2) // 2) * 32
    _req(wc.shape == (3, 3, 1, 32) and bc is not None and bc.numel() == 32, "convnet_fwd: conv must be 3x3x1x32")
    f32 = W1.dtype == torch.float32
    _req((f32 or W1.dtype == torch.bfloat16) and W1.stride(-1) == 1, "convnet_fwd: W1 bf16 or f32")
    rows = tuple(W1.shape) == (Kf, 64)
    if f32:
        _req(rows and W1.stride(0) == 64, "convnet_fwd: f32 W1 must be the [K,64] master kernel")
    else:
        _req(rows and W1.stride(0) == 64 or tuple(W1.shape) == (64, Kf) and W1.stride(0) % 8 == 0,
             "convnet_fwd: W1 must be [K,64] or [64,K]")
    _req(W % 2 == 0 and x.shape[3] == 1 and x.is_contiguous() and x.dtype == torch.float32, "convnet_fwd: input")
    hp = hpre if hrep == 1 and hpre.dim() == 2 else hpre.reshape(-1, *hpre.shape[-2:])
    _req(hp.shape[0] == hrep and hpre.is_contiguous() if hp.dim() == 3 else hrep == 1, "convnet_fwd: hpre replicas")
    _req(hp.shape[-2] >= B and hp.shape[-1] == 64 and hpre.is_contiguous(), "convnet_fwd: hpre")
    _req(inc_iter is None or inc_iter.dtype == torch.int64, "convnet_fwd: int64 step counter")
    ldPt = 0
    if Pt is not None:
        ldPt = Pt.stride(0)
        _req(Pt.shape[0] == Kf and ldPt >= B and ldPt % 8 == 0 and Pt.dtype == W1.dtype, "convnet_fwd: Pt")
    lda = 0
    if amax is not None:
        lda = amax.shape[-1]
        _req(amax.dtype == torch.int64 and amax.shape[:2] == (Kf // 32, 4) and lda >= B, "convnet_fwd: amax")
    optp = _ct.byref(opt) if opt is not None else None
    hstride = hp.stride(0) if hp.dim() == 3 else 0
    if f32:
        rc = N.hip().tde_convnet_fwd_f32(_P(x), _P(wc), _P(bc), _P(W1), W1.stride(0), _P(hpre), _P(Pt), ldPt,
                                         _P(amax), lda, B, H, W, _P(stamps), optp, int(off_wc), int(off_bc),
                                         _P(inc_iter), int(hrep), hstride, _s())
        N.check(rc, "tde_convnet_fwd_f32")
        return
    rc = N.hip().tde_convnet_fwd(_P(x), _P(wc), _P(bc), _P(W1), W1.stride(0), _P(hpre), _P(Pt), ldPt,
                                 _P(amax), lda, B, H, W, _P(stamps), int(rows), optp, int(off_wc), int(off_bc),
                                 _P(inc_iter), int(hrep), hstride, _s())
    N.check(rc, "tde_convnet_fwd")


def convnet_bwd(x, amax, hpre, hzero, b1, W2, b2, labels, *, scale, pre_relu, metrics, W1row, Pt, dW1, dwc, dbc,
                dW2=None, db2=None, db1=None, B=None, stamps=None, opt: BwdOpt | None = None, cpart=None,
                push: XgPush | None = None, crep=1, crep_stride=0):
    """Trunk backward with the classifier head fused in: from this step's Dense(64) pre-activation
    ``hpre`` [B, 64] (f32) every workgroup recomputes the head (loss, dlogits, Dense(64) input gradient)
    and runs the trunk backward; ``hzero`` (the other parity buffer) is zeroed for the next forward.
    ``hpre`` / ``hzero`` may be [R, B, 64] replica stacks (summed on load; all zeroed).
    Precision follows ``W1row``: the bf16 row-major shadow (bf16 form) or the f32 master kernel
    (float32 form; ``Pt`` f32, and in the fused step ``W1row`` is the memory ``opt`` updates).
    Plain (``opt`` None): dW1 stored, conv grads atomically added, dW2 / db2 / db1 added, metrics
    accumulated.  ``opt`` (fused step): the updates are applied instead (see ``BwdOpt``).
    ``cpart`` (deterministic mode): the conv gradients are stored per workgroup there instead of added
    atomically; ``convnet_cgrad_reduce`` sums them in order.  ``push`` (float32 form, plain step): dW1 is
    stored into the xGMI owners' contribution areas of the next all-reduce call instead of into ``dW1``
    (the fused data-parallel exchange).  ``crep`` > 1 (float32 form, plain step): workgroup x adds its conv
    gradients into replica x % crep of dwc / dbc (stride ``crep_stride`` elements), summed by the all-reduce."""
    B = x.shape[0] if B is None else B
    H, W = x.shape[1], x.shape[2]
    Kf = ((H - 2) // 2) * ((W - 2) // 2) * 32
    Hd, C = W2.shape
    f32 = W1row.dtype == torch.float32
    _req(dwc.shape == (3, 3, 1, 32) and Hd == 64 and C <= 16, "convnet_bwd: specialised for Conv2D(32) + Dense(64)")
    _req(W1row.shape == (Kf, 64) and W1row.stride(0) == 64 and dW1.shape == (Kf, 64) and Pt.shape[0] == Kf,
         "convnet_bwd: shapes")
    _req(Pt.dtype == W1row.dtype and (f32 or W1row.dtype == torch.bfloat16), "convnet_bwd: W1 / Pt dtypes")
    _req(Pt.stride(0) >= B and Pt.stride(0) % 8 == 0, "convnet_bwd: Pt ld")
    _req(amax.dtype == torch.int64 and amax.shape[:2] == (Kf // 32, 4) and amax.shape[-1] >= B, "convnet_bwd: amax")
    hp = hpre if hpre.dim() == 3 else hpre.unsqueeze(0)
    _req(hp.shape[0] <= 1024 and hp.shape[1] >= B and hp.shape[2] == 64 and hpre.is_contiguous()
         and hzero.shape == hpre.shape and hzero.is_contiguous(), "convnet_bwd: hpre / hzero")
    _req(labels.dtype == torch.int32 and labels.numel() >= B, "convnet_bwd: int32 labels")
    _req(W2.is_contiguous() and b2.numel() == C and (b1 is None or b1.numel() == 64), "convnet_bwd: head variables")
    _req(push is None or f32, "convnet_bwd: the fused exchange is implemented for the float32 form")
    fn = N.hip().tde_convnet_bwd_f32 if f32 else N.hip().tde_convnet_bwd
    rc = fn(_P(x), _P(amax), amax.shape[-1], _P(hpre), _P(hzero), hp.shape[0], hp.stride(0),
            _P(b1), _P(W2), _P(b2), C,
            int(pre_relu), _P(labels), float(scale), _P(metrics), _P(W1row), W1row.stride(0),
            _P(Pt), Pt.stride(0), _P(dW1), _P(dwc), _P(dbc), _P(dW2), _P(db2), _P(db1), B, H,
            W, _P(stamps), _ct.byref(opt) if opt is not None else None, _P(cpart),
            *((_ct.byref(push) if push is not None else None, int(crep), int(crep_stride)) if f32 else ()), _s())
    N.check(rc, "tde_convnet_bwd_f32" if f32 else "tde_convnet_bwd")


class CgenOpt(_ct.Structure):
    """``TdeCgenOpt`` (csrc/kernels/convnet_gen.hip): the optimizer the generic fused backward applies to the
    Dense kernel rows in place (w / m / v at the Dense kernel's elements of the flat buffers)."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float), ("w", _ct.c_void_p), ("m", _ct.c_void_p), ("v", _ct.c_void_p),
                ("iterations", _ct.c_void_p)]


class CgenFly(_ct.Structure):
    """``TdeCgenFly`` (csrc/kernels/convnet_gen.hip): the generic fused step's forward side — the previous
    step's conv update applied on the fly while ``*pend``, and the head snapshot."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float), ("pend", _ct.c_void_p), ("gwc", _ct.c_void_p), ("gbc", _ct.c_void_p),
                ("grep", _ct.c_int), ("grep_stride", _ct.c_longlong), ("mwc", _ct.c_void_p), ("mbc", _ct.c_void_p),
                ("vwc", _ct.c_void_p), ("vbc", _ct.c_void_p), ("iter_prev", _ct.c_void_p), ("sb1", _ct.c_void_p),
                ("sw2", _ct.c_void_p), ("sb2", _ct.c_void_p), ("hsnap", _ct.c_void_p), ("hC", _ct.c_int)]


class CgenHead(_ct.Structure):
    """``TdeCgenHead`` (csrc/kernels/convnet_gen.hip): the generic fused step's head update in the backward's
    head workgroup (flat buffers + the head's element offsets)."""
    _fields_ = [("kind", _ct.c_int), ("lr", _ct.c_float), ("mom", _ct.c_float), ("b1", _ct.c_float), ("b2", _ct.c_float),
                ("eps", _ct.c_float), ("w", _ct.c_void_p), ("m", _ct.c_void_p), ("v", _ct.c_void_p),
                ("off_w2", _ct.c_longlong), ("off_b2", _ct.c_longlong), ("off_b1", _ct.c_longlong),
                ("iterations", _ct.c_void_p), ("pend_set", _ct.c_void_p), ("iter_prev", _ct.c_void_p)]


def cgen_supported(filters, units):
    return bool(N.hip().tde_cgen_supported(int(filters), int(units)))


def cgen_fwd(x, wc, bc, W1, hpre, Pt, amax, *, B, inc_iter=None, fly: CgenFly | None = None, stamps=None):
    """Generic-width fused small-CNN forward, float32 (csrc/kernels/convnet_gen.hip): Conv2D(CC, 3x3) + ReLU +
    MaxPool(2) + the Dense(HD) matmul, hpre [R, >=B, HD] += (workgroup i adds into replica i % R).
    W1 the f32 master kernel [P*CC, HD]; Pt [P*CC, ldPt] f32; amax int64 [P, CC/8, lda]; inc_iter (int64 step
    counter, nullable) advanced by one; ``fly`` (fused step): the deferred conv update applied on the fly and the
    head snapshot."""
    H, W = x.shape[1], x.shape[2]
    CC = wc.shape[-1]
    Pn = ((H - 2) // 2) * ((W - 2) // 2)
    HD = W1.shape[1]
    _req(x.dtype == torch.float32 and x.is_contiguous() and x.shape[3] == 1 and x.shape[0] >= B, "cgen_fwd: input")
    _req(wc.numel() == 9 * CC and bc.numel() == CC and W1.dtype == torch.float32 and W1.is_contiguous()
         and tuple(W1.shape) == (Pn * CC, HD), "cgen_fwd: weights")
    hp = hpre if hpre.dim() == 3 else hpre.unsqueeze(0)
    _req(hpre.is_contiguous() and hp.shape[1] >= B and hp.shape[2] == HD, "cgen_fwd: hpre")
    _req(Pt.dtype == torch.float32 and Pt.shape[0] == Pn * CC and Pt.stride(0) >= B and Pt.stride(1) == 1,
         "cgen_fwd: Pt")
    _req(amax.dtype == torch.int64 and amax.shape[:2] == (Pn, CC // 8) and amax.shape[-1] >= B, "cgen_fwd: amax")
    rc = N.hip().tde_cgen_fwd(CC, HD, _P(x), _P(wc), _P(bc), _P(W1), _P(hpre), hp.shape[0], hp.stride(0), _P(Pt),
                              Pt.stride(0), _P(amax), amax.shape[-1], _P(inc_iter),
                              _ct.byref(fly) if fly is not None else None, _P(stamps), B, H, W, _s())
    N.check(rc, "tde_cgen_fwd")


def cgen_bwd(x, amax, hpre, hzero, b1, W2, b2, labels, *, scale, pre_relu, metrics, W1, Pt, dW1, dwc, dbc,
             dW2=None, db2=None, db1=None, B, iterations=None, opt: CgenOpt | None = None, stamps=None, crep=1,
             crep_stride=0, hopt: CgenHead | None = None, fcommit: FlatApply | None = None,
             push: XgPush | None = None):
    """Generic-width fused small-CNN backward, float32 (plain step): from hpre [R, >=B, HD] every workgroup
    recomputes the head, then the Dense(HD) weight / input gradients and the conv gradients; hzero (the
    other parity) is zeroed.  dW1 stored, dwc / dbc atomically added, dW2 / db2 / db1 added, metrics added,
    ``iterations`` (int64 step counter) advanced.  ``opt`` (fused step): dW1 is applied to W1 in place by the
    optimizer instead of stored (``dW1`` may be None).  ``stamps`` (diagnostics): int64 [P + 1, 8] phase
    clocks per workgroup.  ``crep`` > 1: workgroup x adds its conv gradients into replica x % crep of dwc / dbc
    (``crep_stride`` elements apart), summed by the consumer.  ``hopt`` + ``fcommit`` (fused step, with ``opt``):
    the head workgroup updates the head in place (``b1`` / ``W2`` / ``b2`` are then the forward's snapshot) and
    commits the previous step's deferred conv update.  ``push``
    (plain step under the xGMI communicator): dW1 into the owners' windows of the next all-reduce call."""
    H, W = x.shape[1], x.shape[2]
    CC = dwc.shape[-1]
    Pn = ((H - 2) // 2) * ((W - 2) // 2)
    HD, C = W2.shape
    hp = hpre if hpre.dim() == 3 else hpre.unsqueeze(0)
    _req(hpre.is_contiguous() and hzero.shape == hpre.shape and hzero.is_contiguous() and hp.shape[2] == HD
         and hp.shape[1] >= B, "cgen_bwd: hpre / hzero")
    _req(tuple(W1.shape) == (Pn * CC, HD) and W1.is_contiguous() and (dW1 is None and opt is not None or
                                                                        dW1.shape == W1.shape) and dbc.numel() == CC,
         "cgen_bwd: shapes")
    _req(Pt.shape[0] == Pn * CC and Pt.dtype == torch.float32 and Pt.stride(0) >= B, "cgen_bwd: Pt")
    _req(amax.dtype == torch.int64 and amax.shape[:2] == (Pn, CC // 8) and amax.shape[-1] >= B, "cgen_bwd: amax")
    _req(labels.dtype == torch.int32 and labels.numel() >= B and C <= 16, "cgen_bwd: labels / classes")
    _req(hopt is None or (opt is not None and fcommit is not None and fcommit.pend), "cgen_bwd: fused head update")
    _req(W2.is_contiguous() and b2.numel() == C and (b1 is None or b1.numel() == HD), "cgen_bwd: head variables")
    rc = N.hip().tde_cgen_bwd(CC, HD, _P(x), _P(amax), amax.shape[-1], _P(hpre), _P(hzero), hp.shape[0],
                              hp.stride(0), _P(b1), _P(W2), _P(b2), C, int(pre_relu), _P(labels), float(scale),
                              _P(metrics), _P(W1), _P(Pt), Pt.stride(0), _P(dW1), _P(dwc), _P(dbc), _P(dW2),
                              _P(db2), _P(db1), _P(iterations), _ct.byref(opt) if opt is not None else None,
                              _P(stamps), int(crep), int(crep_stride),
                              _ct.byref(hopt) if hopt is not None else None,
                              _ct.byref(fcommit) if fcommit is not None else None,
                              _ct.byref(push) if push is not None else None, B, H, W, _s())
    N.check(rc, "tde_cgen_bwd")


def convnet_cgrad_reduce(cpart, nwg, dwc, dbc):
    """Deterministic mode: dwc / dbc += the backward's per-workgroup conv-gradient partials, in order."""
    _req(cpart.dtype == torch.float32 and cpart.numel() >= nwg * 320, "convnet_cgrad_reduce: cpart")
    N.check(N.hip().tde_convnet_cgrad_reduce(_P(cpart), int(nwg), _P(dwc), _P(dbc), _s()), "tde_convnet_cgrad_reduce")


def noop(blocks=1, threads=64):
    N.check(N.hip().tde_noop(blocks, threads, _s()), "tde_noop")
