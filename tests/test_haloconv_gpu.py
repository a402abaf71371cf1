"""The persistent halo-tile 3x3 conv (csrc/kernels/haloconv.hip) vs a float64 host oracle of the same op on the
same bf16 operands: forward (+ BN statistics of the stored bf16 outputs), input gradient (flipped taps of the
HWIO shadow), accumulated input gradient, and grids that split an image's tiles over several workgroups or
give one workgroup tiles of two images (the ring's non-contiguous refill)."""
import pytest
import torch
import torch.nn.functional as F

from tensorflow_distributed_example_amd import _native as N
from tensorflow_distributed_example_amd.ops import layer_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
bf = torch.bfloat16


def _r(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(bf)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _geo(B, H, W):
    return O.ConvGeom(B, H, W, 64, H, W, 64, 3, 3, 1, 1, 1, 1)


CASES = [(2, 56, 56, 0), (3, 56, 56, 5), (2, 56, 56, 37), (4, 28, 32, 0), (2, 8, 64, 3), (2, 16, 32, 3), (3, 24, 24, 2)]


@pytest.mark.parametrize("B,H,W,grid", CASES)
def test_halo_forward_and_stats(B, H, W, grid):
    g = _geo(B, H, W)
    assert O.halo_ok(g)
    x = _r(B, H, W, 64, seed=1)
    w = _r(3, 3, 64, 64, seed=2) * 0.05           # HWIO
    wt = w.permute(3, 0, 1, 2).reshape(64, 576).contiguous()   # [Co, kh, kw, ci]
    y = torch.zeros(B * H * W * 64, dtype=bf, device=DEV)
    st = torch.zeros(2 * O.STAT_SLOTS * 64, dtype=torch.float64, device=DEV)
    O.halo_conv(x.to(DEV).reshape(-1), wt.to(DEV), y, g, colstats=st, grid=grid)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(3, 2, 0, 1), padding=1).permute(0, 2, 3, 1)
    out = y.view(B, H, W, 64).cpu()
    assert _rel(out, ref) < 4e-3
    q = out.double().reshape(-1, 64)
    s = st.view(O.STAT_SLOTS, 2, 64).sum(0).cpu()
    assert torch.allclose(s[0], q.sum(0), rtol=2e-5, atol=1e-3)   # f32 per-lane partials, f64 atomics
    assert torch.allclose(s[1], (q * q).sum(0), rtol=2e-5, atol=1e-3)


@pytest.mark.parametrize("B,H,W,grid", CASES[:3])
@pytest.mark.parametrize("accum", [False, True])
def test_halo_input_gradient(B, H, W, grid, accum):
    g = _geo(B, H, W)
    dy = _r(B, H, W, 64, seed=3)
    w = _r(3, 3, 64, 64, seed=4) * 0.05           # HWIO: the row shadow
    base = _r(B, H, W, 64, seed=5)
    dx = (base.clone() if accum else torch.zeros_like(base)).to(DEV).reshape(-1)
    O.halo_conv(dy.to(DEV).reshape(-1), w.contiguous().to(DEV), dx, g, dgrad=True, accum=accum, grid=grid)
    torch.cuda.synchronize()
    xd = torch.zeros(B, 64, H, W, dtype=torch.float64, requires_grad=True)
    yd = F.conv2d(xd, w.double().permute(3, 2, 0, 1), padding=1)
    yd.backward(dy.double().permute(0, 3, 1, 2))
    ref = xd.grad.permute(0, 2, 3, 1)
    if accum:
        ref = ref + base.double()
    assert _rel(dx.view(B, H, W, 64).cpu(), ref) < 4e-3


def test_halo_rejects_other_geometries():
    assert not O.halo_ok(O.ConvGeom(2, 28, 28, 128, 28, 28, 128, 3, 3, 1, 1, 1, 1))
    assert not O.halo_ok(O.ConvGeom(2, 56, 56, 64, 28, 28, 64, 3, 3, 2, 2, 0, 0))
    assert N.hip().tde_halo_conv_ok(64, 64, 56, 60, 2) == 0   # W % 8


WG_CASES = [(2, 56, 56), (3, 8, 64), (1, 16, 32), (4, 28, 32), (2, 6, 16), (5, 12, 8)]


@pytest.mark.parametrize("mf", [32, 16])
@pytest.mark.parametrize("B,H,W", WG_CASES)
def test_halo_weight_gradient(B, H, W, mf):
    """The halo-tile weight gradient (every input and dY byte loaded once for all 9 taps, per-workgroup partials
    reduced in order) vs float64 autograd of the same bf16 operands, accumulated onto an existing f32 gradient,
    bitwise reproducible run to run."""
    g = _geo(B, H, W)
    assert O.halo_wgrad_ok(g)
    x = _r(B, H, W, 64, seed=6)
    dy = _r(B, H, W, 64, seed=7)
    base = torch.randn(3, 3, 64, 64, generator=torch.Generator().manual_seed(8))
    need = O.halo_wgrad_scratch_elems(g)
    outs = []
    N.hip().tde_halo_wgrad_mfma(mf)   # v_mfma_f32_32x32x16_bf16 or the 16x16x32 form (default)
    for _ in range(2):
        dW = base.clone().to(DEV)
        scr = torch.full((need,), float("nan"), device=DEV)
        O.halo_wgrad(x.to(DEV).reshape(-1), dy.to(DEV).reshape(-1), dW, g, scr)
        torch.cuda.synchronize()
        outs.append(dW.cpu())
    wd = torch.zeros(64, 64, 3, 3, dtype=torch.float64, requires_grad=True)
    yd = F.conv2d(x.double().permute(0, 3, 1, 2), wd, padding=1)
    yd.backward(dy.double().permute(0, 3, 1, 2))
    ref = wd.grad.permute(2, 3, 1, 0) + base.double()      # HWIO
    N.hip().tde_halo_wgrad_mfma(16)
    assert _rel(outs[0] - base, ref - base.double()) < 1e-5
    assert torch.equal(outs[0], outs[1])


def test_halo_wgrad_rejects_other_geometries():
    assert not O.halo_wgrad_ok(O.ConvGeom(2, 28, 28, 128, 28, 28, 128, 3, 3, 1, 1, 1, 1))
    assert not O.halo_wgrad_ok(O.ConvGeom(2, 56, 56, 64, 28, 28, 64, 3, 3, 2, 2, 0, 0))
    assert N.hip().tde_halo_wgrad_ok(64, 64, 56, 60, 2) == 0   # W % 8
    assert N.hip().tde_halo_wgrad_ok(64, 64, 7, 8, 2) == 0     # H has no 2- or 4-row tiling


@pytest.mark.parametrize("B,H", [(2, 224), (3, 32), (1, 64)])
def test_stem_weight_gradient(B, H):
    """The packed RGB stem's weight gradient on the tile kernel (haloconv.hip stem_wgrad_kernel) — the 7x7 stride-2
    SAME conv on 3 channels as layers.hip's virtual conv over 8-channel pixel pairs — unpacked into the real HWIO
    gradient, vs float64 autograd of the real conv, accumulated onto an existing gradient."""
    Ho = H // 2
    pt = ((Ho - 1) * 2 + 7 - H) // 2            # TF SAME: (2, 3) at 224 / 64 / 32
    g = O.ConvGeom(B, H, H, 3, Ho, Ho, 64, 7, 7, 2, 2, pt, pt)
    gv = O.stem_geometry(g)
    assert O.stem_pack_ok(g) and O.stem_wgrad_ok(gv)
    x = _r(B, H, H, 3, seed=31)
    dy = _r(B, g.Ho, g.Wo, 64, seed=32)
    xp = torch.zeros(gv.B * gv.H * gv.W * 8, dtype=bf, device=DEV)
    O.stem_pack(x.to(DEV).reshape(-1), g, xp)
    gWv = torch.zeros(gv.K * 64, device=DEV)
    scr = torch.full((O.stem_wgrad_scratch_elems(gv),), float("nan"), device=DEV)
    O.stem_wgrad(xp, dy.to(DEV).reshape(-1), gWv, gv, scr)
    base = torch.randn(7, 7, 3, 64, generator=torch.Generator().manual_seed(33))
    gW = base.clone().to(DEV).reshape(-1)
    O.stem_unpack_wgrad(gWv, g, gW)
    torch.cuda.synchronize()
    pb = (g.Ho - 1) * 2 + 7 - H - pt
    wd = torch.zeros(64, 3, 7, 7, dtype=torch.float64, requires_grad=True)
    yd = F.conv2d(F.pad(x.double().permute(0, 3, 1, 2), (pt, pb, pt, pb)), wd, stride=2)
    yd.backward(dy.double().permute(0, 3, 1, 2))
    ref = wd.grad.permute(2, 3, 1, 0)
    assert _rel(gW.cpu().view(7, 7, 3, 64) - base, ref) < 1e-5
    assert float(gWv.abs().max()) == 0.0   # the unpack pass consumed (zeroed) the virtual gradient


@pytest.mark.parametrize("B,H", [(2, 224), (3, 32), (1, 64)])
def test_stem_forward_tile_kernel(B, H):
    """The packed stem's forward on the tile kernel (haloconv.hip stem_fwd_kernel) vs the implicit GEMM on the same
    packed operands: the stored bf16 output within one bf16 rounding and the BN statistics slots (sums of the stored
    values) to f32 accumulation noise; and vs float64 conv of the real 7x7 stride-2 SAME conv."""
    Ho = H // 2
    pt = ((Ho - 1) * 2 + 7 - H) // 2
    g = O.ConvGeom(B, H, H, 3, Ho, Ho, 64, 7, 7, 2, 2, pt, pt)
    gv = O.stem_geometry(g)
    assert O.stem_pack_ok(g) and O.stem_fwd_ok(gv)
    x = _r(B, H, H, 3, seed=41)
    w = torch.randn(7, 7, 3, 64, generator=torch.Generator().manual_seed(42)) * 0.1
    Wt = w.permute(3, 0, 1, 2).reshape(64, -1).to(bf).contiguous().to(DEV)
    xp = torch.zeros(gv.B * gv.H * gv.W * 8, dtype=bf, device=DEV)
    Wv = torch.zeros(gv.Co * gv.K, dtype=bf, device=DEV)
    O.stem_pack(x.to(DEV).reshape(-1), g, xp, Wt, Wv)
    n = B * Ho * Ho * 64
    y1 = torch.full((n,), float("nan"), dtype=bf, device=DEV)
    y0 = torch.zeros(n, dtype=bf, device=DEV)
    cs1 = torch.zeros(2 * O.STAT_SLOTS * 64, dtype=torch.float64, device=DEV)
    cs0 = torch.zeros_like(cs1)
    O.stem_fwd(xp, Wv, y1, gv, colstats=cs1)
    O.conv_fwd(xp, Wv.view(64, -1), y0, gv, colstats=cs0)
    torch.cuda.synchronize()
    assert torch.isfinite(y1.float()).all()
    d = (y1.float() - y0.float()).abs()
    assert float((d / (y0.float().abs() + 1e-3)).max()) < 1e-2
    s1 = cs1.view(O.STAT_SLOTS, 2, 64).sum(0)
    s0 = cs0.view(O.STAT_SLOTS, 2, 64).sum(0)
    assert _rel(s1.cpu(), s0.cpu()) < 1e-5
    assert float(s1[0].sum().cpu()) == pytest.approx(float(y1.double().sum().cpu()), rel=1e-5)
    pb = (Ho - 1) * 2 + 7 - H - pt
    xd = x.to(bf).double().permute(0, 3, 1, 2)
    wd = w.to(bf).double().permute(3, 2, 0, 1)
    yd = F.conv2d(F.pad(xd, (pt, pb, pt, pb)), wd, stride=2).permute(0, 2, 3, 1).reshape(-1)
    assert _rel(y1.double().cpu(), yd) < 5e-3
