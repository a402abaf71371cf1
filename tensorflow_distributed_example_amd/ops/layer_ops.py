"""Host wrappers for the layer-wise kernel library (csrc/kernels/layers.hip).

All activations are NHWC bf16 (Keras ``mixed_bfloat16``: bf16 compute/activations,
fp32 variables, fp32 BN statistics), weight grads accumulate in the fp32 flat
gradient bucket.  Every wrapper validates operand sizes on the host against the
geometry it hands the kernel, so a kernel never indexes outside its buffers.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import torch

from .. import _native as N

_P = N.ptr
A_ROWK, A_CONV, A_DGRAD, A_COLM, A_WGRAD = range(5)
STAT_SLOTS = 8   # BN statistics buffers are [STAT_SLOTS][2][C] f64 (layers.hip kStatSlots)
B_NK, B_DGRADW, B_KN = range(3)
bf16 = torch.bfloat16


def _s():
    return N.stream_ptr()


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def _bf(t, n, what):
    _req(t is not None and t.dtype == bf16 and t.is_contiguous() and t.numel() >= n, f"{what}: bf16 [{n}] expected")


def _f64(t, n, what):
    _req(t is not None and t.dtype == torch.float64 and t.is_contiguous() and t.numel() >= n,
         f"{what}: f64 [{n}] expected")


def _f32(t, n, what):
    _req(t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= n,
         f"{what}: f32 [{n}] expected")


@dataclass(frozen=True)
class ConvGeom:
    B: int
    H: int
    W: int
    C: int
    Ho: int
    Wo: int
    Co: int
    KH: int
    KW: int
    sh: int
    sw: int
    pt: int
    pl: int

    def carray(self):
        return (C.c_int * 13)(self.B, self.H, self.W, self.C, self.Ho, self.Wo, self.Co, self.KH, self.KW,
                              self.sh, self.sw, self.pt, self.pl)

    @property
    def K(self):
        return self.KH * self.KW * self.C

    def with_batch(self, B):
        return ConvGeom(B, *[getattr(self, f) for f in ("H", "W", "C", "Ho", "Wo", "Co", "KH", "KW", "sh", "sw",
                                                        "pt", "pl")])


def pick_splits(M, N_, K, target=512):
    """0 = let the kernel pick (weight-grad GEMMs size their split-K from the tile they run)."""
    return 0


def fwd_splits(M, N_, K):
    """Split-K factor for an activation-producing GEMM (fwd / dgrad): only when the output tiles
    alone cannot fill the 256 CUs and the K loop is long (latency-bound); the partial sums go
    through the f32 scratch + finalize pass."""
    target = _FWD_SPLIT_TARGET
    tiles = -(-M // 64) * -(-N_ // 64)
    ktiles = -(-K // 32)
    if target <= 0 or tiles >= 256 or ktiles < 8:
        return 1
    return max(1, min(-(-target // tiles), ktiles // 4))


# workgroups a split-K fwd/dgrad GEMM aims for (TDE_FWD_SPLIT_TARGET; 0 = never split, the default since the
# LDS-DMA k loop: the split's extra finalize launch costs more than the parallelism it buys —
# scripts/split_sweep.sh, profiles/r2_split_sweep.txt: Model B 489k -> 512k, LeNet-5 676k -> 697k,
# MLP 3.17M -> 3.53M img/s, ResNet-18 neutral)
_FWD_SPLIT_TARGET = int(os.environ.get("TDE_FWD_SPLIT_TARGET", "0"))


def scratch_elems(M, N_, K):
    return M * N_ if fwd_splits(M, N_, K) > 1 else 0


def _igemm(a, lda, ak, b, ldb, bk, M, N_, K, geo=None, splits=1, cf=None, ldc=0, cf_mode=0, alpha=1.0,
           cb=None, ldcb=0, cb_accum=False, bias=None, relu=False, colstats=None, scratch=None, phase=None):
    g = geo.carray() if geo is not None else None
    if splits > 1 and scratch is not None:
        _f32(scratch, M * N_, "igemm split-K scratch")
    ph = (C.c_int * len(phase))(*phase) if phase is not None else None
    rc = N.hip().tde_igemm(_P(a), int(lda), ak, _P(b), int(ldb), bk, int(M), int(N_), int(K), g, int(splits),
                           _P(cf), int(ldc), int(cf_mode), float(alpha), _P(cb), int(ldcb), int(cb_accum), _P(bias),
                           int(relu), _P(colstats), _P(scratch), ph, _s())
    N.check(rc, "tde_igemm")


def dgrad_phases(g: ConvGeom):
    """Stride phases of a strided conv's input gradient: (ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp) per phase —
    the phase's pixel grid and the only taps that reach it (the other (s^2-1)/s^2 of the implicit-GEMM K
    would multiply zeros)."""
    out = []
    for ph in range(g.sh):
        Hp = -(-(g.H - ph) // g.sh) if g.H > ph else 0
        kh0 = (ph + g.pt) % g.sh
        KHp = -(-(g.KH - kh0) // g.sh) if g.KH > kh0 else 0
        for pw in range(g.sw):
            Wp = -(-(g.W - pw) // g.sw) if g.W > pw else 0
            kw0 = (pw + g.pl) % g.sw
            KWp = -(-(g.KW - kw0) // g.sw) if g.KW > kw0 else 0
            if Hp and Wp:
                out.append((ph, pw, Hp, Wp, kh0, kw0, KHp, KWp))
    return out


def _fs(M, N_, K, scratch):
    if scratch is None:
        return 1
    s = fwd_splits(M, N_, K)
    return s if s > 1 and scratch.numel() >= M * N_ else 1


# ---------------------------------------------------------------- Conv2D
def conv_fwd(x, Wt, y, g: ConvGeom, bias=None, relu=False, colstats=None, scratch=None):
    """y[B,Ho,Wo,Co] = conv(x[B,H,W,C], W) (+bias, ReLU); Wt = [Co, KH*KW*C] bf16 (transposed shadow)."""
    _bf(x, g.B * g.H * g.W * g.C, "conv_fwd x")
    _req(Wt.dtype == bf16 and tuple(Wt.shape) == (g.Co, g.K) and Wt.is_contiguous(), "conv_fwd Wt")
    _bf(y, g.B * g.Ho * g.Wo * g.Co, "conv_fwd y")
    if bias is not None:
        _f32(bias, g.Co, "conv_fwd bias")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * g.Co, "conv_fwd colstats")
    M = g.B * g.Ho * g.Wo
    _igemm(x, 0, A_CONV, Wt, g.K, B_NK, M, g.Co, g.K, g, splits=_fs(M, g.Co, g.K, scratch), cb=y, ldcb=g.Co,
           bias=bias, relu=relu, colstats=colstats, scratch=scratch)


def halo_ok(g: ConvGeom, dgrad=False):
    """The persistent halo-tile kernel (csrc/kernels/haloconv.hip) covers 3x3 / stride-1 / SAME convs with 64
    input and output channels (ResNet-18 stage 1), forward and input gradient.  TDE_HALO=0 disables it."""
    if os.environ.get("TDE_HALO", "1") == "0":
        return False
    if (g.KH, g.KW, g.sh, g.sw, g.pt, g.pl) != (3, 3, 1, 1, 1, 1) or (g.Ho, g.Wo) != (g.H, g.W):
        return False
    return bool(N.hip().tde_halo_conv_ok(g.C, g.Co, g.H, g.W, g.B))


def halo_conv(x, w, y, g: ConvGeom, *, dgrad=False, accum=False, colstats=None, grid=0):
    """Forward: y = conv3x3(x, W) with ``w`` = Wt [Co, 9*C] (the transposed shadow; element (tap, co, ci) at
    co*9C + tap*C + ci).  Input gradient (``dgrad``): y (=|+=) conv3x3(dY, W') with ``w`` = the HWIO shadow
    [3,3,C,Co] read with flipped taps (element (tap, ci, co) at (8-tap)*C*Co + ci*Co + co)."""
    n = g.B * g.H * g.W * 64
    _bf(x, n, "halo_conv x")
    _bf(y, n, "halo_conv y")
    _bf(w, 9 * 64 * 64, "halo_conv w")
    _req(halo_ok(g, dgrad), "halo_conv: geometry not covered")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * 64, "halo_conv colstats")
    wst, wsn = (64 * 64, 64) if dgrad else (64, 9 * 64)
    N.check(N.hip().tde_halo_conv3x3(_P(x), _P(w), wst, wsn, int(dgrad), _P(y), int(accum), _P(colstats), g.B, g.H,
                                     g.W, int(grid), _s()), "tde_halo_conv3x3")


def halo_wgrad_ok(g: ConvGeom):
    """The halo-tile weight gradient (csrc/kernels/haloconv.hip wgrad3x3_kernel): the same 3x3 / stride-1 / SAME
    64 -> 64 channel convs.  TDE_HALO_WGRAD=0 (or TDE_HALO=0) disables it."""
    if os.environ.get("TDE_HALO", "1") == "0" or os.environ.get("TDE_HALO_WGRAD", "1") == "0":
        return False
    if (g.KH, g.KW, g.sh, g.sw, g.pt, g.pl) != (3, 3, 1, 1, 1, 1) or (g.Ho, g.Wo) != (g.H, g.W):
        return False
    return bool(N.hip().tde_halo_wgrad_ok(g.C, g.Co, g.H, g.W, g.B))


def halo_wgrad_scratch_elems(g: ConvGeom):
    """f32 per-workgroup partials one halo weight-gradient launch stores (reduced into dW in workgroup order)."""
    return int(N.hip().tde_halo_wgrad_scratch_elems(g.B, g.H, g.W))


def halo_wgrad(x, dy, dW, g: ConvGeom, scratch):
    """dW[3,3,64,64] (f32, HWIO) += sum over pixels of x (x) dy: one pass over x and dy for all 9 taps (per-workgroup
    partials in ``scratch``, then the ordered reduction into dW)."""
    n = g.B * g.H * g.W * 64
    _bf(x, n, "halo_wgrad x")
    _bf(dy, n, "halo_wgrad dy")
    _f32(dW, 9 * 64 * 64, "halo_wgrad dW")
    _req(halo_wgrad_ok(g), "halo_wgrad: geometry not covered")
    need = halo_wgrad_scratch_elems(g)
    _f32(scratch, need, "halo_wgrad scratch")
    N.check(N.hip().tde_halo_wgrad3x3(_P(x), _P(dy), _P(dW), _P(scratch), int(scratch.numel()), g.B, g.H, g.W, _s()),
            "tde_halo_wgrad3x3")


class BnSum(C.Structure):
    """csrc/kernels/layers.hip BnSum: the backward sums of the BatchNormalization that consumes an input gradient."""
    _fields_ = [("y", C.c_void_p), ("res", C.c_void_p), ("saved", C.c_void_p), ("gamma", C.c_void_p),
                ("beta", C.c_void_p), ("relu", C.c_int), ("dstats", C.c_void_p)]


def dgrad_bnsum_ok(g: ConvGeom):
    """Input gradients whose epilogue can take the consumer BN's backward sums (tde_igemm_dgrad_bnsum): stride 1,
    the LDS-DMA implicit GEMM (C % 8 == 0, Co a multiple of the K step), unsplit; never in deterministic mode."""
    if N.hip().tde_layers_is_deterministic():
        return False
    kb = 64 if g.Co % 64 == 0 else 32
    M, K = g.B * g.H * g.W, g.KH * g.KW * g.Co
    return (g.sh == 1 and g.sw == 1 and g.C % 8 == 0 and g.Co % 8 == 0 and g.Co % kb == 0
            and fwd_splits(M, g.C, K) == 1 and N.hip().tde_bnsum_bytes() == C.sizeof(BnSum))


def conv_dgrad(dy, Wrow, dx, g: ConvGeom, accum=False, scratch=None, bnsum=None):
    """dx[B,H,W,C] (=|+=) conv_transpose(dy[B,Ho,Wo,Co], W); Wrow = HWIO bf16.  bnsum (dict y, res, saved, gamma,
    beta, relu, dstats): the BN consuming dx's tensor takes its backward sums in this launch's epilogue."""
    _bf(dy, g.B * g.Ho * g.Wo * g.Co, "conv_dgrad dy")
    _bf(Wrow, g.K * g.Co, "conv_dgrad W")
    _bf(dx, g.B * g.H * g.W * g.C, "conv_dgrad dx")
    if bnsum is not None:
        n = g.B * g.H * g.W * g.C
        _bf(bnsum["y"], n, "conv_dgrad bnsum y")
        if bnsum.get("res") is not None:
            _bf(bnsum["res"], n, "conv_dgrad bnsum res")
        _f32(bnsum["saved"], 2 * g.C, "conv_dgrad bnsum saved")
        _f32(bnsum["dstats"], 2 * STAT_SLOTS * g.C, "conv_dgrad bnsum dstats")
        _req(dgrad_bnsum_ok(g), "conv_dgrad: bnsum on a shape without the fused epilogue")
        s = BnSum(_P(bnsum["y"]), _P(bnsum.get("res")), _P(bnsum["saved"]), _P(bnsum.get("gamma")),
                  _P(bnsum.get("beta")), int(bool(bnsum.get("relu"))), _P(bnsum["dstats"]))
        M, K = g.B * g.H * g.W, g.KH * g.KW * g.Co
        N.check(N.hip().tde_igemm_dgrad_bnsum(_P(dy), _P(Wrow), M, g.C, K, g.carray(), _P(dx), g.C, int(accum),
                                              C.byref(s), _s()), "tde_igemm_dgrad_bnsum")
        return
    if g.sh > 1 or g.sw > 1:
        phases = dgrad_phases(g)
        untapped = [ph for ph in phases if ph[6] * ph[7] == 0]
        skip_untapped = bool(untapped) and (accum or g.C % 8 == 0)
        if untapped and not accum:
            # phases no tap reaches (3 of the 4 of a 1x1 stride-2 projection) are zero: one HIP pass zeroes
            # exactly their pixels and the tapped phases store theirs, instead of K = 0 GEMM launches
            if g.C % 8 == 0:
                mask = sum(1 << (ph[0] * g.sw + ph[1]) for ph in untapped)
                N.check(N.hip().tde_dgrad_phase_zero(_P(dx), g.carray(), mask, _s()), "tde_dgrad_phase_zero")
        run = [ph for ph in phases if not (ph[6] * ph[7] == 0 and skip_untapped)]
        if 1 < len(run) <= 4 and os.environ.get("TDE_DGRAD_MULTIPHASE", "1") != "0":
            # every stride phase in one launch (grid z = phase): M / K of the largest phase size the grid
            table = [-1, len(run)] + [v for ph in run for v in ph]
            Mx = max(g.B * ph[2] * ph[3] for ph in run)
            Kx = max(ph[6] * ph[7] * g.Co for ph in run)
            _igemm(dy, 0, A_DGRAD, Wrow, 0, B_DGRADW, Mx, g.C, Kx, g, cb=dx, ldcb=g.C, cb_accum=accum,
                   phase=table)
            return
        for ph in run:
            _igemm(dy, 0, A_DGRAD, Wrow, 0, B_DGRADW, g.B * ph[2] * ph[3], g.C, ph[6] * ph[7] * g.Co, g,
                   cb=dx, ldcb=g.C, cb_accum=accum, phase=ph)
        return
    M, K = g.B * g.H * g.W, g.KH * g.KW * g.Co
    _igemm(dy, 0, A_DGRAD, Wrow, 0, B_DGRADW, M, g.C, K, g, splits=_fs(M, g.C, K, scratch), cb=dx, ldcb=g.C,
           cb_accum=accum, scratch=scratch)


# ---------------------------------------------------------------- explicit im2col (C % 8 != 0, e.g. the RGB stem)
def im2col(x, g: ConvGeom, xcol, Wt=None, Wt_pad=None):
    """xcol[B*Ho*Wo, Kp] = patches of x (Kp = K rounded up to 8, zero tail); optionally Wt [Co, K] ->
    Wt_pad [Co, Kp].  Lets the conv GEMMs run the 16-byte vector path."""
    Kp = -(-g.K // 8) * 8
    _bf(x, g.B * g.H * g.W * g.C, "im2col x")
    _bf(xcol, g.B * g.Ho * g.Wo * Kp, "im2col out")
    if Wt is not None:
        _req(tuple(Wt.shape) == (g.Co, g.K) and Wt.dtype == bf16 and Wt.is_contiguous(), "im2col Wt")
        _bf(Wt_pad, g.Co * Kp, "im2col Wt_pad")
    N.check(N.hip().tde_im2col(_P(x), g.carray(), Kp, _P(xcol), _P(Wt), _P(Wt_pad), _s()), "tde_im2col")
    return Kp


# ---------------------------------------------------------------- packed stem (C <= 4, stride 2 along W)
def stem_geometry(g: ConvGeom):
    """The packed stem's virtual conv (csrc/kernels/layers.hip tde_stem_pack): input [B, Hp, Wv, 8] (two
    real pixels x 4 channels per virtual pixel), KW' = ceil(KW/2) taps, stride (sh, 1), valid."""
    kwv = -(-g.KW // 2)
    hp, wv = (g.Ho - 1) * g.sh + g.KH, g.Wo + kwv - 1
    return ConvGeom(g.B, hp, wv, 8, g.Ho, g.Wo, g.Co, g.KH, kwv, g.sh, 1, 0, 0)


def stem_pack_ok(g: ConvGeom):
    """Eligible: C <= 4, stride 2 along W, and the virtual conv's kernel row is one 32-wide k-tile (KW in
    7..8) or the 16-byte vector path (any KW)."""
    return g.C <= 4 and g.sw == 2 and g.KW >= 2


def stem_pack(x, g: ConvGeom, xp, Wt=None, Wv=None):
    gv = stem_geometry(g)
    _bf(x, g.B * g.H * g.W * g.C, "stem_pack x")
    _bf(xp, gv.B * gv.H * gv.W * 8, "stem_pack xp")
    if Wt is not None:
        _req(tuple(Wt.shape) == (g.Co, g.K) and Wt.dtype == bf16 and Wt.is_contiguous(), "stem_pack Wt")
        _bf(Wv, g.Co * gv.K, "stem_pack Wv")
    N.check(N.hip().tde_stem_pack(_P(x), g.carray(), _P(xp), _P(Wt), _P(Wv), _s()), "tde_stem_pack")


def stem_wgrad_ok(gv: ConvGeom):
    """The packed stem's weight gradient on the tile kernel (csrc/kernels/haloconv.hip stem_wgrad_kernel): the virtual
    geometry of ``stem_geometry`` with 4 taps along W, 8 channels, 64 filters.  TDE_STEM_WGRAD=0 disables it."""
    if os.environ.get("TDE_STEM_WGRAD", "1") == "0":
        return False
    return bool(N.hip().tde_stem_wgrad_ok(gv.B, gv.H, gv.W, gv.Ho, gv.Wo, gv.KH, gv.KW, gv.sh, gv.C, gv.Co))


def stem_wgrad_scratch_elems(gv: ConvGeom):
    return int(N.hip().tde_stem_wgrad_scratch_elems(gv.B, gv.Ho, gv.KH))


def stem_wgrad(xp, dy, gWv, gv: ConvGeom, scratch):
    """gWv[KH][4][8][64] (f32) += the packed stem's weight gradient (xp: the packed input, dy: the stem output's
    gradient); per-workgroup partials in ``scratch`` reduced in a fixed order."""
    _bf(xp, gv.B * gv.H * gv.W * 8, "stem_wgrad xp")
    _bf(dy, gv.B * gv.Ho * gv.Wo * gv.Co, "stem_wgrad dy")
    _f32(gWv, gv.K * gv.Co, "stem_wgrad gWv")
    _req(stem_wgrad_ok(gv), "stem_wgrad: geometry not covered")
    _f32(scratch, stem_wgrad_scratch_elems(gv), "stem_wgrad scratch")
    N.check(N.hip().tde_stem_wgrad(_P(xp), _P(dy), _P(gWv), _P(scratch), int(scratch.numel()), gv.B, gv.H, gv.W,
                                   gv.Ho, gv.Wo, gv.KH, gv.sh, _s()), "tde_stem_wgrad")


def stem_fwd_ok(gv: ConvGeom):
    """The packed stem's forward on the tile kernel (csrc/kernels/haloconv.hip stem_fwd_kernel; no bias / ReLU: the
    BN follows).  TDE_STEM_FWD=0 disables it."""
    if os.environ.get("TDE_STEM_FWD", "1") == "0":
        return False
    return bool(N.hip().tde_stem_fwd_ok(gv.B, gv.H, gv.W, gv.Ho, gv.Wo, gv.KH, gv.KW, gv.sh, gv.C, gv.Co))


def stem_fwd(xp, Wv, y, gv: ConvGeom, colstats=None):
    """y [B, Ho, Wo, 64] (bf16) = the packed stem conv of xp with Wv [64, KH*32]; colstats (f64 [8][2][64], nullable)
    += the BN sums of the stored y (as conv_fwd's epilogue)."""
    _bf(xp, gv.B * gv.H * gv.W * 8, "stem_fwd xp")
    _req(Wv.dtype == bf16 and Wv.numel() == gv.Co * gv.K and Wv.is_contiguous(), "stem_fwd Wv")
    _bf(y, gv.B * gv.Ho * gv.Wo * gv.Co, "stem_fwd y")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * gv.Co, "stem_fwd colstats")
    _req(stem_fwd_ok(gv), "stem_fwd: geometry not covered")
    N.check(N.hip().tde_stem_fwd(_P(xp), _P(Wv), _P(y), _P(colstats), gv.B, gv.H, gv.W, gv.Ho, gv.Wo, gv.KH, gv.sh,
                                 _s()), "tde_stem_fwd")


def stem_unpack_wgrad(gWv, g: ConvGeom, gW):
    gv = stem_geometry(g)
    _f32(gWv, gv.K * g.Co, "stem_unpack gWv")
    _f32(gW, g.K * g.Co, "stem_unpack gW")
    N.check(N.hip().tde_stem_unpack_wgrad(_P(gWv), g.carray(), _P(gW), _s()), "tde_stem_unpack_wgrad")


def conv_fwd_im2col(xcol, Wt_pad, y, g: ConvGeom, Kp, bias=None, relu=False, colstats=None, scratch=None):
    M = g.B * g.Ho * g.Wo
    _bf(y, M * g.Co, "conv_fwd_im2col y")
    _igemm(xcol, Kp, A_ROWK, Wt_pad, Kp, B_NK, M, g.Co, Kp, splits=_fs(M, g.Co, Kp, scratch), cb=y, ldcb=g.Co,
           bias=bias, relu=relu, colstats=colstats, scratch=scratch)


def conv_wgrad_im2col(xcol, dy, dW, g: ConvGeom, Kp):
    """dW[K, Co] += xcol[:, :K]^T @ dy (the padded columns are read, never written)."""
    M = g.B * g.Ho * g.Wo
    _bf(dy, M * g.Co, "conv_wgrad_im2col dy")
    _f32(dW, g.K * g.Co, "conv_wgrad_im2col dW")
    _igemm(xcol, Kp, A_COLM, dy, g.Co, B_KN, g.K, g.Co, M, splits=0, cf=dW, ldc=g.Co, cf_mode=2)


# ---------------------------------------------------------------- narrow convolutions (direct, VALU)
def smallconv_ok(g: ConvGeom, dgrad=False):
    return bool(N.hip().tde_smallconv_ok(g.C, g.Co, g.KH, g.KW, int(dgrad)))


def smallconv_fwd(x, Wrow, y, g: ConvGeom, bias=None, relu=False, colstats=None):
    """Direct convolution for C_out <= 32: one thread per output pixel, all channels in registers."""
    _bf(x, g.B * g.H * g.W * g.C, "smallconv_fwd x")
    _bf(Wrow, g.K * g.Co, "smallconv_fwd W")
    _bf(y, g.B * g.Ho * g.Wo * g.Co, "smallconv_fwd y")
    if bias is not None:
        _f32(bias, g.Co, "smallconv_fwd bias")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * g.Co, "smallconv_fwd colstats")
    _req(smallconv_ok(g), "smallconv_fwd: layer too wide for the direct kernel")
    N.check(N.hip().tde_smallconv_fwd(_P(x), _P(Wrow), _P(bias), int(relu), _P(y), _P(colstats), g.carray(), _s()),
            "tde_smallconv_fwd")


def smallconv_dgrad(dy, Wrow, dx, g: ConvGeom, accum=False):
    """Direct input-gradient for C_in <= 32 (only the taps of each pixel's stride phase)."""
    _bf(dy, g.B * g.Ho * g.Wo * g.Co, "smallconv_dgrad dy")
    _bf(Wrow, g.K * g.Co, "smallconv_dgrad W")
    _bf(dx, g.B * g.H * g.W * g.C, "smallconv_dgrad dx")
    _req(smallconv_ok(g, True), "smallconv_dgrad: layer too wide for the direct kernel")
    N.check(N.hip().tde_smallconv_dgrad(_P(dy), _P(Wrow), _P(dx), int(accum), g.carray(), _s()), "tde_smallconv_dgrad")


def smallconv_wgrad_ok(g: ConvGeom):
    return bool(N.hip().tde_smallconv_wgrad_ok(g.C, g.Co, g.KH, g.KW))


def smallconv_wgrad(x, dy, dW, g: ConvGeom):
    """dW[KH,KW,C,Co] (f32) += sum_pixels x (x) dy for filters whose K*Co partial sums fit in registers."""
    _bf(x, g.B * g.H * g.W * g.C, "smallconv_wgrad x")
    _bf(dy, g.B * g.Ho * g.Wo * g.Co, "smallconv_wgrad dy")
    _f32(dW, g.K * g.Co, "smallconv_wgrad dW")
    _req(smallconv_wgrad_ok(g), "smallconv_wgrad: filter too large for the register kernel")
    N.check(N.hip().tde_smallconv_wgrad(_P(x), _P(dy), _P(dW), g.carray(), _s()), "tde_smallconv_wgrad")


def wgrad_scratch_elems(M, N_, K):
    """f32 scratch the split-K weight gradient of an [M, N] x K GEMM stores its partials in (0: no split)."""
    return int(N.hip().tde_igemm_wgrad_scratch_elems(int(M), int(N_), int(K)))


def _wscratch(M, N_, K, scratch):
    if scratch is None:
        return None
    need = wgrad_scratch_elems(M, N_, K)
    return scratch if need and scratch.numel() >= need else None


def conv_wgrad(x, dy, dW, g: ConvGeom, splits=None, scratch=None):
    """dW[KH,KW,C,Co] (f32) += sum_pixels x (x) dy  (split-K partials through ``scratch`` when given)."""
    _bf(x, g.B * g.H * g.W * g.C, "conv_wgrad x")
    _bf(dy, g.B * g.Ho * g.Wo * g.Co, "conv_wgrad dy")
    _f32(dW, g.K * g.Co, "conv_wgrad dW")
    M, N_, K = g.K, g.Co, g.B * g.Ho * g.Wo
    s = pick_splits(M, N_, K) if splits is None else splits
    _igemm(x, 0, A_WGRAD, dy, g.Co, B_KN, M, N_, K, g, splits=s, cf=dW, ldc=g.Co, cf_mode=2,
           scratch=_wscratch(M, N_, K, scratch) if s == 0 else None)


# ---------------------------------------------------------------- Dense
def dense_fwd(x, Wt, B, *, y=None, logits=None, bias=None, relu=False, colstats=None, scratch=None):
    """[B,out] = x[B,in] @ W (+bias, ReLU) -> bf16 ``y`` and/or f32 ``logits``; Wt = [out, in] bf16."""
    out, fin = Wt.shape
    _bf(x, B * fin, "dense_fwd x")
    _req(Wt.dtype == bf16 and Wt.is_contiguous(), "dense_fwd Wt")
    if y is not None:
        _bf(y, B * out, "dense_fwd y")
    if logits is not None:
        _f32(logits, B * out, "dense_fwd logits")
    if bias is not None:
        _f32(bias, out, "dense_fwd bias")
    if colstats is not None:
        _f64(colstats, 2 * STAT_SLOTS * out, "dense_fwd colstats")
    _igemm(x, fin, A_ROWK, Wt, fin, B_NK, B, out, fin, splits=_fs(B, out, fin, scratch), cf=logits, ldc=out,
           cf_mode=1 if logits is not None else 0, cb=y, ldcb=out, bias=bias, relu=relu, colstats=colstats,
           scratch=scratch)


def dense_dgrad(dy, Wrow, dx, B, accum=False, scratch=None):
    """dx[B,in] (=|+=) dy[B,out] @ W^T; Wrow = [in, out] bf16."""
    fin, out = Wrow.shape
    _bf(dy, B * out, "dense_dgrad dy")
    _req(Wrow.dtype == bf16 and Wrow.is_contiguous(), "dense_dgrad W")
    _bf(dx, B * fin, "dense_dgrad dx")
    _igemm(dy, out, A_ROWK, Wrow, out, B_NK, B, fin, out, splits=_fs(B, fin, out, scratch), cb=dx, ldcb=fin,
           cb_accum=accum, scratch=scratch)


def dense_wgrad(x, dy, dW, B, splits=None, scratch=None):
    """dW[in,out] (f32) += x[B,in]^T @ dy[B,out]."""
    fin, out = dW.shape
    _bf(x, B * fin, "dense_wgrad x")
    _bf(dy, B * out, "dense_wgrad dy")
    _f32(dW, fin * out, "dense_wgrad dW")
    s = pick_splits(fin, out, B) if splits is None else splits
    _igemm(x, fin, A_COLM, dy, out, B_KN, fin, out, B, splits=s, cf=dW, ldc=out, cf_mode=2,
           scratch=_wscratch(fin, out, B, scratch) if s == 0 else None)


# ---------------------------------------------------------------- BN / activation / dropout
@dataclass
class DropSpec:
    rate: float = 0.0
    seed: int = 0
    iterations: torch.Tensor = None
    layer_id: int = 0


_NODROP = DropSpec()


def bn_fwd(y, out, R, Cc, *, mode, stats=None, saved=None, gamma=None, beta=None, eps=1e-3, mmean=None, mvar=None,
           momentum=0.99, bessel=1.0, zero_buf=None, res=None, relu=False, drop: DropSpec = _NODROP, iter_offset=0):
    """out = dropout(relu(bn(y) + res)); mode 0 identity, 1 batch stats (from ``stats``), 2 moving stats."""
    n = R * Cc
    _bf(y, n, "bn_fwd y")
    _bf(out, n, "bn_fwd out")
    _req(Cc <= 2048, "bn_fwd: at most 2048 channels")
    if res is not None:
        _bf(res, n, "bn_fwd res")
    if mode == 1:
        _f64(stats, 2 * STAT_SLOTS * Cc, "bn_fwd stats")
        _f32(saved, 2 * Cc, "bn_fwd saved")
    if mode == 2:
        _f32(mmean, Cc, "bn_fwd moving_mean")
        _f32(mvar, Cc, "bn_fwd moving_variance")
    if zero_buf is not None:
        _f32(zero_buf, 2 * STAT_SLOTS * Cc, "bn_fwd zero_buf")
    rc = N.hip().tde_bn_fwd(_P(y), _P(out), _P(res), int(R), int(Cc), int(mode), _P(stats), _P(saved), _P(gamma),
                            _P(beta), float(eps), _P(mmean), _P(mvar), float(momentum), float(bessel), _P(zero_buf),
                            int(relu), float(drop.rate), int(drop.seed) & (2 ** 64 - 1), _P(drop.iterations),
                            int(iter_offset), int(drop.layer_id), _s())
    N.check(rc, "tde_bn_fwd")


def bn_bwd(dout, y, R, Cc, *, mode, saved=None, gamma=None, beta=None, res=None, relu=False,
           drop: DropSpec = _NODROP, iter_offset=-1, dstats=None, dx=None, dx_accum=False, dres=None,
           dres_accum=False, dgamma=None, dbeta=None, zero_fwd=None, sums_ready=False):
    """sums_ready: ``dstats`` already holds the backward sums (taken by ``conv_dgrad(..., bnsum=)``): apply pass only."""
    n = R * Cc
    _bf(dout, n, "bn_bwd dout")
    _bf(y, n, "bn_bwd y")
    _req(Cc <= 1024, "bn_bwd: at most 1024 channels")
    if mode == 1:
        _f32(saved, 2 * Cc, "bn_bwd saved")
        _f32(dstats, 2 * STAT_SLOTS * Cc, "bn_bwd dstats")
    if zero_fwd is not None:
        _f64(zero_fwd, 2 * STAT_SLOTS * Cc, "bn_bwd zero_fwd")
    if dx is not None:
        _bf(dx, n, "bn_bwd dx")
    if dres is not None:
        _bf(dres, n, "bn_bwd dres")
    if res is not None:
        _bf(res, n, "bn_bwd res")
    rc = N.hip().tde_bn_bwd(_P(dout), _P(y), _P(res), int(R), int(Cc), int(mode), _P(saved), _P(gamma), _P(beta),
                            int(relu), float(drop.rate), int(drop.seed) & (2 ** 64 - 1), _P(drop.iterations),
                            int(iter_offset), int(drop.layer_id), _P(dstats), _P(dx), int(dx_accum), _P(dres),
                            int(dres_accum), _P(dgamma), _P(dbeta), _P(zero_fwd), int(bool(sums_ready)), _s())
    N.check(rc, "tde_bn_bwd")


def act_bwd(dout, out, R, Cc, *, relu, dz=None, dbias=None):
    n = R * Cc
    _bf(dout, n, "act_bwd dout")
    if relu:
        _bf(out, n, "act_bwd out")
    if dz is not None:
        _bf(dz, n, "act_bwd dz")
    if dbias is not None:
        _f32(dbias, Cc, "act_bwd dbias")
    _req(Cc <= 1024, "act_bwd: at most 1024 channels")
    rc = N.hip().tde_act_bwd(_P(dout), _P(out), int(R), int(Cc), int(relu), _P(dz), _P(dbias), _s())
    N.check(rc, "tde_act_bwd")


def colstats(x, R, Cc, stats):
    _bf(x, R * Cc, "colstats x")
    _f64(stats, 2 * STAT_SLOTS * Cc, "colstats stats")
    N.check(N.hip().tde_colstats(_P(x), int(R), int(Cc), _P(stats), _s()), "tde_colstats")


# ---------------------------------------------------------------- pooling / padding / casts
def maxpool_fwd(x, y, idx, g: ConvGeom):
    _bf(x, g.B * g.H * g.W * g.C, "maxpool x")
    _bf(y, g.B * g.Ho * g.Wo * g.C, "maxpool y")
    if idx is not None:
        _req(idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * g.C, "maxpool idx")
    N.check(N.hip().tde_maxpool(_P(x), _P(y), _P(idx), None, None, 0, g.carray(), 0, _s()), "tde_maxpool")


def bn_relu_maxpool_fwd(y, R, Cc, pooled, idx, g: ConvGeom, *, mode, stats=None, saved=None, gamma=None, beta=None,
                        eps=1e-3, mmean=None, mvar=None, momentum=0.99, bessel=1.0, zero_buf=None):
    """pooled, idx = maxpool(relu(bn(y))) without storing the BN output (the ResNet stem; see
    csrc/kernels/layers.hip bn_relu_maxpool_fwd_kernel).  mode 1 batch statistics from ``stats`` (+ saved
    mean/rstd, moving averages, zeroed backward accumulators as bn_fwd), 2 moving statistics."""
    _bf(y, R * Cc, "bn_pool y")
    _req(g.C == Cc and g.B * g.H * g.W == R, "bn_pool geometry")
    _bf(pooled, g.B * g.Ho * g.Wo * Cc, "bn_pool pooled")
    _req(idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * Cc, "bn_pool idx")
    if mode == 1:
        _f64(stats, 2 * STAT_SLOTS * Cc, "bn_pool stats")
        _f32(saved, 2 * Cc, "bn_pool saved")
    else:
        _f32(mmean, Cc, "bn_pool mmean")
        _f32(mvar, Cc, "bn_pool mvar")
    if zero_buf is not None:
        _f32(zero_buf, 2 * STAT_SLOTS * Cc, "bn_pool zero_buf")
    rc = N.hip().tde_bn_relu_maxpool_fwd(_P(y), int(R), int(Cc), int(mode), _P(stats), _P(saved), _P(gamma),
                                         _P(beta), float(eps), _P(mmean), _P(mvar), float(momentum), float(bessel),
                                         _P(zero_buf), _P(pooled), _P(idx), g.carray(), _s())
    N.check(rc, "tde_bn_relu_maxpool_fwd")


def bn_pool_ok(g: ConvGeom):
    """Geometries the fused BN + ReLU + MaxPool pair runs (tde_bn_pool_bwd's host checks): 8-channel vectors with
    256 % (C / 8) == 0, C <= 512, windows covering each pixel at most 2 x 2 times, one pooled row <= 4096
    elements in LDS."""
    C8 = g.C // 8
    return (g.C % 8 == 0 and g.C <= 512 and 256 % C8 == 0 and -(-g.KH // g.sh) <= 2 and (g.KW + g.sw) // g.sw <= 2
            and g.KH * g.KW < 255 and g.Wo * g.C <= 4096 and (g.Wo * g.C) % 16 == 0)


def bn_pool_bwd(dpool, idx, y, R, Cc, g: ConvGeom, *, saved, dstats, dx, gamma=None, beta=None, relu=True,
                dx_accum=False, dgamma=None, dbeta=None, zero_fwd=None):
    """Backward of bn_relu_maxpool_fwd: the BN input gradient ``dx`` from the POOLED gradient + argmax bytes (the
    pool's input gradient is gathered per element, never stored); two passes (sums, apply) as bn_bwd."""
    _bf(dpool, g.B * g.Ho * g.Wo * Cc, "bn_pool_bwd dpool")
    _req(idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * Cc, "bn_pool_bwd idx")
    _bf(y, R * Cc, "bn_pool_bwd y")
    _bf(dx, R * Cc, "bn_pool_bwd dx")
    _f32(saved, 2 * Cc, "bn_pool_bwd saved")
    _f32(dstats, 2 * STAT_SLOTS * Cc, "bn_pool_bwd dstats")
    if zero_fwd is not None:
        _f64(zero_fwd, 2 * STAT_SLOTS * Cc, "bn_pool_bwd zero_fwd")
    rc = N.hip().tde_bn_pool_bwd(_P(dpool), _P(idx), _P(y), int(R), int(Cc), _P(saved), _P(gamma), _P(beta), int(relu),
                                 _P(dstats), _P(dx), int(dx_accum), _P(dgamma), _P(dbeta), _P(zero_fwd), g.carray(),
                                 _s())
    N.check(rc, "tde_bn_pool_bwd")


def maxpool_bwd(dy, idx, dx, g: ConvGeom, accum=False):
    _bf(dy, g.B * g.Ho * g.Wo * g.C, "maxpool dy")
    _req(idx.dtype == torch.uint8 and idx.numel() >= g.B * g.Ho * g.Wo * g.C, "maxpool idx")
    _bf(dx, g.B * g.H * g.W * g.C, "maxpool dx")
    N.check(N.hip().tde_maxpool(None, None, _P(idx), _P(dy), _P(dx), int(accum), g.carray(), 1, _s()),
            "tde_maxpool")


def gap_fwd(x, y, B, HW, Cc):
    _bf(x, B * HW * Cc, "gap x")
    _bf(y, B * Cc, "gap y")
    N.check(N.hip().tde_gap(_P(x), _P(y), B, HW, Cc, 0, 0, _s()), "tde_gap")


def gap_bwd(dy, dx, B, HW, Cc, accum=False):
    _bf(dy, B * Cc, "gap dy")
    _bf(dx, B * HW * Cc, "gap dx")
    N.check(N.hip().tde_gap(_P(dy), _P(dx), B, HW, Cc, 1, int(accum), _s()), "tde_gap")


def pad_fwd(x, y, g: ConvGeom):
    _bf(x, g.B * g.H * g.W * g.C, "pad x")
    _bf(y, g.B * g.Ho * g.Wo * g.C, "pad y")
    N.check(N.hip().tde_pad(_P(x), _P(y), g.carray(), 0, 0, _s()), "tde_pad")


def pad_bwd(dy, dx, g: ConvGeom, accum=False):
    _bf(dy, g.B * g.Ho * g.Wo * g.C, "pad dy")
    _bf(dx, g.B * g.H * g.W * g.C, "pad dx")
    N.check(N.hip().tde_pad(_P(dy), _P(dx), g.carray(), 1, int(accum), _s()), "tde_pad")


def cast_bf16(x, y):
    _req(x.dtype == torch.float32 and x.is_contiguous(), "cast x")
    _bf(y, x.numel(), "cast y")
    N.check(N.hip().tde_cast_f32_bf16(_P(x), _P(y), x.numel(), _s()), "tde_cast_f32_bf16")


def xent(logits, labels, B, Cc, *, scale=1.0, dlogits=None, metrics=None, probs=None, probs_are_logits=False,
         iterations=None):
    _f32(logits, B * Cc, "xent logits")
    _req(labels.dtype == torch.int32 and labels.numel() >= B, "xent labels")
    if dlogits is not None:
        _bf(dlogits, B * Cc, "xent dlogits")
    if probs is not None:
        _f32(probs, B * Cc, "xent probs")
    rc = N.hip().tde_xent(_P(logits), Cc, _P(labels), int(B), int(Cc), float(scale), _P(dlogits), Cc, _P(metrics),
                          _P(probs), int(probs_are_logits), _P(iterations), _s())
    N.check(rc, "tde_xent")
