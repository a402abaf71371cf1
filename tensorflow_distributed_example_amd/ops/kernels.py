"""Thin, allocation-free Python entry points to the gfx950 HIP kernels.

Every function takes pre-allocated device tensors, enqueues on the current HIP
stream (so it is hipGraph-capturable), and raises if the native call reports an
error.  Shapes are validated on the host before launch: a kernel never sees an
operand shape it does not support (a faulting kernel can reset the node).
"""
from __future__ import annotations

import torch

from .. import _native as N

_P = N.ptr


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
    _req(hin.dtype == torch.float32 and hin.shape[1] >= H, "head: input")
    _req(C <= 64 and H * C <= 16384, "head: too large for the fused head")
    _req(labels.dtype == torch.int32, "head: int32 labels")
    ldg = G.stride(0) if G is not None else 0
    ldgt = Gt.stride(0) if Gt is not None else 0
    ldgf = Gf.stride(0) if Gf is not None else 0
    rc = N.hip().tde_head_xent(_P(hin), hin.stride(0), _P(pre_bias), int(pre_relu), _P(W2), _P(b2), _P(labels),
                               B, H, C, float(scale), int(compute_grad), _P(dW2), _P(db2), _P(dpre_bias),
                               _P(G), ldg, _P(Gt), ldgt, _P(Gf), ldgf, _P(metrics), _P(probs),
                               int(probs_are_logits), _P(row_loss), int(zero_hin), _P(iterations), _P(stamps), _s())
    N.check(rc, "tde_head_xent")


def convnet_fwd(x, wc, bc, W1col, hpre, Pt=None, amax=None, stamps=None):
    """Fused Conv2D(32,3x3,relu)+MaxPool(2)+Dense(64) matmul forward; hpre += (atomic).

    amax: uint8 view of a [P, 4, lda] uint64 buffer (lane-contiguous pool argmax)."""
    B, H, W = x.shape[0], x.shape[1], x.shape[2]
    Kf = ((H - 2) // 2) * ((W - 2) // 2) * 32
    _req(wc.shape == (3, 3, 1, 32) and bc is not None and bc.numel() == 32, "convnet_fwd: conv must be 3x3x1x32")
    _req(W1col.shape == (64, Kf) and W1col.stride(0) % 8 == 0 and W1col.dtype == torch.bfloat16, "convnet_fwd: W1col")
    _req(W % 2 == 0 and x.shape[3] == 1 and x.is_contiguous(), "convnet_fwd: input")
    _req(hpre.shape[0] >= B and hpre.shape[1] == 64 and hpre.is_contiguous(), "convnet_fwd: hpre")
    ldPt = 0
    if Pt is not None:
        ldPt = Pt.stride(0)
        _req(Pt.shape[0] == Kf and ldPt >= B and ldPt % 8 == 0, "convnet_fwd: Pt")
    lda = 0
    if amax is not None:
        lda = amax.shape[-1]
        _req(amax.dtype == torch.int64 and amax.shape[:2] == (Kf // 32, 4) and lda >= B, "convnet_fwd: amax")
    rc = N.hip().tde_convnet_fwd(_P(x), _P(wc), _P(bc), _P(W1col), W1col.stride(0), _P(hpre), _P(Pt), ldPt,
                                 _P(amax), lda, B, H, W, _P(stamps), _s())
    N.check(rc, "tde_convnet_fwd")


def convnet_bwd(x, amax, G, Gt, W1row, Pt, dW1, dwc, dbc, B=None, stamps=None):
    B = x.shape[0] if B is None else B
    H, W = x.shape[1], x.shape[2]
    Kf = ((H - 2) // 2) * ((W - 2) // 2) * 32
    _req(dwc.shape == (3, 3, 1, 32) and G.shape[1] == 64, "convnet_bwd: specialised for Conv2D(32) + Dense(64)")
    _req(W1row.shape == (Kf, 64) and dW1.shape == (Kf, 64) and Pt.shape[0] == Kf, "convnet_bwd: shapes")
    _req(Gt.shape[0] == 64 and Gt.stride(0) >= B and Pt.stride(0) >= B, "convnet_bwd: ld")
    _req(amax.dtype == torch.int64 and amax.shape[:2] == (Kf // 32, 4) and amax.shape[-1] >= B, "convnet_bwd: amax")
    rc = N.hip().tde_convnet_bwd(_P(x), _P(amax), amax.shape[-1], _P(G), G.stride(0), _P(Gt), Gt.stride(0),
                                 _P(W1row), W1row.stride(0), _P(Pt), Pt.stride(0), _P(dW1), _P(dwc), _P(dbc), B, H,
                                 W, _P(stamps), _s())
    N.check(rc, "tde_convnet_bwd")


def noop(blocks=1, threads=64):
    N.check(N.hip().tde_noop(blocks, threads, _s()), "tde_noop")
