"""T0/T1 for the layer-wise kernel library (csrc/kernels/layers.hip): every kernel vs a
plain PyTorch fp32 reference of the same op on bf16-rounded operands, then whole-model
gradients of the layer-wise plan (Model B, a small ResNet) vs the torch autograd plan."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("bf16_policy")]   # the layer-wise kernel library: bf16
DEV = "cuda"
bf = torch.bfloat16


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(bf).to(DEV)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


from tensorflow_distributed_example_amd.ops.layer_ops import STAT_SLOTS as SLOTS  # noqa: E402


def _stats_buf(C):
    return torch.zeros(2 * SLOTS * C, dtype=torch.float64, device=DEV)


def _sum_slots(st, C):
    """[slots][2][C] -> [2*C] (sum, sum of squares)."""
    return st.view(SLOTS, 2, C).sum(0).reshape(-1)


def _cpu64(t):
    """float64 CPU copy: the torch oracles run on the host, so no vendor GPU kernel is part of a check."""
    return t.detach().double().cpu()


def _dev(t):
    return t.to(DEV)


def _tf_same(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


CONV_CASES = [
    # B, H, W, C, Co, k, s, padding
    (4, 28, 28, 1, 6, 3, 1, "same"),     # Model B conv1
    (4, 28, 28, 6, 12, 6, 2, "same"),    # Model B conv2
    (4, 14, 14, 12, 24, 6, 2, "same"),   # Model B conv3
    (2, 16, 16, 16, 64, 3, 1, "same"),   # vector paths
    (2, 17, 15, 8, 24, 3, 2, "same"),    # odd sizes, stride 2, asymmetric pads
    (2, 15, 15, 3, 64, 7, 2, "same"),    # ResNet stem shape family
    (2, 8, 8, 64, 128, 1, 2, "valid"),   # projection shortcut
    (3, 10, 9, 32, 40, 3, 1, "valid"),   # N tail
]


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(B, H, W, C, Co, k, s, pad):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    x = _r(B, H, W, C, seed=1)
    w = _r(k, k, C, Co, seed=2, scale=0.2)
    bias = torch.randn(Co, generator=torch.Generator().manual_seed(4)).to(DEV)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    # forward (+bias, ReLU, column statistics)
    y = torch.zeros(B, Ho, Wo, Co, dtype=bf, device=DEV)
    stats_raw = _stats_buf(Co)
    Wt = w.reshape(-1, Co).t().contiguous()
    O.conv_fwd(x, Wt, y, g, bias=bias, relu=False, colstats=stats_raw)
    stats = _sum_slots(stats_raw, Co)
    xr = _cpu64(x).permute(0, 3, 1, 2).requires_grad_(True)
    wr = _cpu64(w).permute(3, 2, 0, 1).requires_grad_(True)
    ref = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wr, _cpu64(bias), stride=s).permute(0, 2, 3, 1)
    dy = _r(B, Ho, Wo, Co, seed=3)
    ref.backward(_cpu64(dy))
    ref, xr_grad, wr_grad = _dev(ref.detach()), _dev(xr.grad), _dev(wr.grad)
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2
    # the statistics are of the STORED bf16 activation: exact up to the f32 per-tile / f64 cross-tile summation (a
    # bf16 rounding of the f64 reference may land one ulp away on a few elements, which is not an error of the sums)
    ys = y.double()
    assert (stats[:Co] - ys.sum((0, 1, 2))).abs().max().item() <= 1e-6 * ys.abs().sum((0, 1, 2)).max().item() + 1e-6
    assert _rel(stats[Co:], (ys ** 2).sum((0, 1, 2))) < 1e-6
    rs = ref.to(bf).double()
    assert _rel(stats[Co:], (rs ** 2).sum((0, 1, 2))) < 1e-3
    dx = torch.zeros(B, H, W, C, dtype=bf, device=DEV)
    O.conv_dgrad(dy, w.contiguous(), dx, g)
    dW = torch.zeros(k, k, C, Co, device=DEV)
    O.conv_wgrad(x, dy, dW, g)
    torch.cuda.synchronize()
    assert _rel(dx.float(), xr_grad.permute(0, 2, 3, 1)) < 1e-2
    assert _rel(dW, wr_grad.permute(2, 3, 1, 0)) < 1e-3
    # split-K partials through a scratch + reduction pass (added onto an existing gradient)
    need = O.wgrad_scratch_elems(g.K, Co, B * Ho * Wo)
    if need:
        dW0 = torch.randn(k, k, C, Co, device=DEV)
        dW2 = dW0.clone()
        O.conv_wgrad(x, dy, dW2, g, scratch=torch.full((need,), float("nan"), device=DEV))
        torch.cuda.synchronize()
        assert _rel(dW2 - dW0, wr_grad.permute(2, 3, 1, 0)) < 1e-3
    # accumulate mode
    dx2 = dx.clone()
    O.conv_dgrad(dy, w.contiguous(), dx2, g, accum=True)
    torch.cuda.synchronize()
    assert _rel(dx2.float(), 2 * dx.float()) < 1e-2


@pytest.mark.parametrize("B,fin,out,relu", [(128, 1176, 200, False), (37, 64, 10, True), (256, 512, 1000, False),
                                             (5, 13, 7, True)])
def test_dense_fwd_dgrad_wgrad(B, fin, out, relu):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    x = _r(B, fin, seed=4)
    w = _r(fin, out, seed=5, scale=0.1)
    bias = torch.randn(out, device=DEV)
    y = torch.zeros(B, out, dtype=bf, device=DEV)
    logits = torch.zeros(B, out, device=DEV)
    O.dense_fwd(x, w.t().contiguous(), B, y=y, logits=logits, bias=bias, relu=relu)
    ref = x.float() @ w.float() + bias
    if relu:
        ref = F.relu(ref)
    dy = _r(B, out, seed=6)
    dx = torch.zeros(B, fin, dtype=bf, device=DEV)
    O.dense_dgrad(dy, w.contiguous(), dx, B)
    dW = torch.zeros(fin, out, device=DEV)
    O.dense_wgrad(x, dy, dW, B)
    torch.cuda.synchronize()
    assert _rel(logits, ref) < 1e-4
    assert _rel(y.float(), ref) < 1e-2
    assert _rel(dx.float(), dy.float() @ w.float().t()) < 1e-2
    assert _rel(dW, x.float().t() @ dy.float()) < 1e-4
    need = O.wgrad_scratch_elems(fin, out, B)
    if need:
        dW2 = torch.zeros(fin, out, device=DEV)
        O.dense_wgrad(x, dy, dW2, B, scratch=torch.full((need,), float("nan"), device=DEV))
        torch.cuda.synchronize()
        assert _rel(dW2, x.float().t() @ dy.float()) < 1e-4


@pytest.mark.parametrize("R,C,relu,res,fused", [(4 * 784, 6, True, False, True), (128, 200, True, False, False),
                                                (2 * 64, 64, True, True, True), (50, 24, False, False, True),
                                                (3136, 512, True, True, True), (1000, 128, False, True, False),
                                                (300, 8, True, False, True)])
def test_batchnorm_fwd_bwd(R, C, relu, res, fused):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    y = _r(R, C, seed=7, scale=2.0) + 0.5
    r = _r(R, C, seed=8) if res else None
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    stats = _stats_buf(C)
    O.colstats(y, R, C, stats)
    saved = torch.zeros(2 * C, device=DEV)
    mm, mv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    out = torch.zeros(R, C, dtype=bf, device=DEV)
    dstats = torch.full((2 * SLOTS * C,), 7.0, device=DEV)
    bessel = R / (R - 1) if fused else 1.0
    O.bn_fwd(y, out, R, C, mode=1, stats=stats, saved=saved, gamma=gamma, beta=beta, eps=1e-3, mmean=mm, mvar=mv,
             momentum=0.99, bessel=bessel, zero_buf=dstats, res=r, relu=relu)
    yr = y.float().requires_grad_(True)
    mean, var = yr.mean(0), yr.var(0, unbiased=False)
    z = (yr - mean) * torch.rsqrt(var + 1e-3) * gamma + beta
    if res:
        z = z + r.float()
    if relu:
        z = F.relu(z)
    torch.cuda.synchronize()
    assert _rel(out.float(), z) < 1e-2
    assert torch.allclose(mm, 0.01 * mean.detach(), atol=1e-5, rtol=1e-3)
    assert torch.allclose(mv, 0.99 + 0.01 * var.detach() * bessel, atol=1e-5, rtol=1e-3)
    assert dstats.abs().max().item() == 0.0   # zeroed for the backward
    dout = _r(R, C, seed=9)
    z.backward(dout.float())
    dx = torch.zeros(R, C, dtype=bf, device=DEV)
    dres = torch.zeros(R, C, dtype=bf, device=DEV) if res else None
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    O.bn_bwd(dout, y, R, C, mode=1, saved=saved, gamma=gamma, beta=beta, res=r, relu=relu, dstats=dstats, dx=dx,
             dres=dres, dgamma=dg, dbeta=db, zero_fwd=stats)
    torch.cuda.synchronize()
    zz = (yr.detach() - mean.detach()) * torch.rsqrt(var.detach() + 1e-3) * gamma + beta + (r.float() if res else 0)
    dz = dout.float() * (zz > 0) if relu else dout.float()
    assert _rel(dx.float(), yr.grad) < 2e-2
    assert _rel(db, dz.sum(0)) < 1e-3
    xhat = (yr.detach() - mean.detach()) * torch.rsqrt(var.detach() + 1e-3)
    assert _rel(dg, (dz * xhat).sum(0)) < 1e-2
    if res:
        assert _rel(dres.float(), dz) < 1e-2
    assert stats.abs().max().item() == 0.0


@pytest.mark.parametrize("C", [200, 64])   # flat and channel-tiled kernels
def test_dropout_mask_regenerated_in_backward(C):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    R = 512
    y = _r(R, C, seed=10).abs() + 0.1
    it = torch.tensor([5], dtype=torch.int64, device=DEV)
    d = O.DropSpec(0.5, 1234, it, 3)
    out = torch.zeros(R, C, dtype=bf, device=DEV)
    O.bn_fwd(y, out, R, C, mode=0, relu=True, drop=d, iter_offset=0)
    it += 1  # the loss kernel advances the step counter between forward and backward
    dout = torch.ones(R, C, dtype=bf, device=DEV)
    dx = torch.zeros(R, C, dtype=bf, device=DEV)
    O.bn_bwd(dout, y, R, C, mode=0, relu=True, drop=d, iter_offset=-1, dx=dx)
    torch.cuda.synchronize()
    kept = out.float() != 0
    frac = kept.float().mean().item()
    assert 0.45 < frac < 0.55
    assert torch.equal(kept, dx.float() != 0)
    assert torch.allclose(dx.float()[kept], torch.full_like(dx.float()[kept], 2.0))
    assert torch.allclose(out.float()[kept], 2 * y.float()[kept], rtol=1e-2)
    # a different step gives a different mask
    out2 = torch.zeros_like(out)
    O.bn_fwd(y, out2, R, C, mode=0, relu=True, drop=d, iter_offset=0)
    torch.cuda.synchronize()
    assert not torch.equal(out2 != 0, kept)


@pytest.mark.parametrize("C", [200, 64, 256])   # flat and channel-tiled kernels
def test_bn_bwd_accumulates(C):
    """dx_accum / dres_accum add into the existing gradient buffers (multi-consumer tensors)."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    R = 384
    y, r, dout = _r(R, C, seed=20) + 0.3, _r(R, C, seed=21), _r(R, C, seed=22)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    stats = _stats_buf(C)
    O.colstats(y, R, C, stats)
    saved = torch.zeros(2 * C, device=DEV)
    dstats = torch.zeros(2 * SLOTS * C, device=DEV)
    out = torch.zeros(R, C, dtype=bf, device=DEV)
    O.bn_fwd(y, out, R, C, mode=1, stats=stats, saved=saved, gamma=gamma, beta=beta, eps=1e-3, zero_buf=dstats,
             res=r, relu=True)
    fresh = [torch.zeros(R, C, dtype=bf, device=DEV) for _ in range(2)]
    base = [_r(R, C, seed=23), _r(R, C, seed=24)]
    acc = [b.clone() for b in base]
    for (dx, dres, accum) in ((fresh[0], fresh[1], False), (acc[0], acc[1], True)):
        dstats.zero_()
        O.bn_bwd(dout, y, R, C, mode=1, saved=saved, gamma=gamma, beta=beta, res=r, relu=True, dstats=dstats,
                 dx=dx, dx_accum=accum, dres=dres, dres_accum=accum)
    torch.cuda.synchronize()
    for f, b, a in zip(fresh, base, acc):
        assert _rel(a.float(), f.float() + b.float()) < 1e-2


@pytest.mark.parametrize("H,W,k,s,pad,C", [(112, 112, 3, 2, "same", 16), (112, 112, 3, 2, "same", 64),
                                           (26, 26, 2, 2, "valid", 32), (11, 11, 3, 1, "same", 8),
                                           (9, 7, 3, 2, "same", 16), (9, 7, 3, 2, "same", 6)])
def test_maxpool(H, W, k, s, pad, C):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    B = 2
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    x = _r(B, H, W, C, seed=11)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, C, k, k, s, s, pt, pl)
    y = torch.zeros(B, Ho, Wo, C, dtype=bf, device=DEV)
    idx = torch.zeros(B * Ho * Wo * C, dtype=torch.uint8, device=DEV)
    O.maxpool_fwd(x, y, idx, g)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(F.pad(xr, (pl, pr, pt, pb), value=float("-inf")), k, s).permute(0, 2, 3, 1)
    dy = _r(B, Ho, Wo, C, seed=12)
    ref.backward(dy.float())
    dx = torch.zeros(B, H, W, C, dtype=bf, device=DEV)
    O.maxpool_bwd(dy, idx, dx, g)
    torch.cuda.synchronize()
    assert torch.equal(y.float(), ref.detach())
    assert _rel(dx.float(), xr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_gap_pad_xent():
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    B, H, W, C = 3, 7, 7, 512
    x = _r(B, H, W, C, seed=13)
    y = torch.zeros(B, C, dtype=bf, device=DEV)
    O.gap_fwd(x, y, B, H * W, C)
    dy = _r(B, C, seed=14)
    dx = torch.zeros(B, H, W, C, dtype=bf, device=DEV)
    O.gap_bwd(dy, dx, B, H * W, C)
    g = O.ConvGeom(B, H, W, C, H + 3, W + 1, C, 1, 1, 1, 1, 1, 0)
    yp = torch.zeros(B, H + 3, W + 1, C, dtype=bf, device=DEV)
    O.pad_fwd(x, yp, g)
    dxp = torch.zeros(B, H, W, C, dtype=bf, device=DEV)
    O.pad_bwd(yp, dxp, g)
    Bx, Cx = 37, 1000
    logits = torch.randn(Bx, Cx, device=DEV) * 3
    labels = torch.randint(0, Cx, (Bx,), device=DEV, dtype=torch.int32)
    labels[:5] = logits[:5].argmax(1).int()
    dl = torch.zeros(Bx, Cx, dtype=bf, device=DEV)
    met = torch.zeros(4, device=DEV)
    it = torch.zeros(1, dtype=torch.int64, device=DEV)
    O.xent(logits, labels, Bx, Cx, scale=0.5, dlogits=dl, metrics=met, iterations=it)
    probs = torch.zeros(Bx, Cx, device=DEV)
    O.xent(logits, labels, Bx, Cx, probs=probs)
    torch.cuda.synchronize()
    assert _rel(y.float(), x.float().mean((1, 2))) < 1e-2
    assert _rel(dx.float(), dy.float()[:, None, None, :].expand(B, H, W, C) / (H * W)) < 1e-2
    assert torch.equal(yp[:, 1:1 + H, :W].float(), x.float()) and yp[:, 0].abs().sum() == 0
    assert torch.equal(dxp, x)
    lr = logits.requires_grad_(True)
    loss = F.cross_entropy(lr, labels.long(), reduction="sum")
    (loss * 0.5).backward()
    assert abs(met[0].item() - loss.item()) < 1e-3 * loss.item()
    assert met[1].item() == (logits.argmax(1) == labels).sum().item() and met[2].item() == Bx
    assert _rel(dl.float(), lr.grad) < 1e-2
    assert _rel(probs, torch.softmax(logits.detach(), 1)) < 1e-5
    assert it.item() == 1
    # the per-pass (C > 1024) xent form and the per-element GAP form (C % 64 != 0)
    lg2 = torch.randn(5, 1500, device=DEV)
    pr2 = torch.zeros(5, 1500, device=DEV)
    O.xent(lg2, labels[:5] % 1500, 5, 1500, probs=pr2)
    x3 = _r(2, 5, 5, 40, seed=15)
    y3 = torch.zeros(2, 40, dtype=bf, device=DEV)
    O.gap_fwd(x3, y3, 2, 25, 40)
    torch.cuda.synchronize()
    assert _rel(pr2, torch.softmax(lg2, 1)) < 1e-5
    assert _rel(y3.float(), x3.float().mean((1, 2))) < 1e-2


def _emulated_compare(model, x, y, B, tol):
    """Layer-wise HIP plan vs the float64 oracle that rounds to bf16 where the plan stores bf16."""
    from tensorflow_distributed_example_amd.train import program as PG
    from tensorflow_distributed_example_amd.train.layerwise import LayerwisePlan, emulate_step
    st = model._store
    plan = PG.make_plan(model, st, "cuda", B, B, model.optimizer, model.loss)
    assert isinstance(plan, LayerwisePlan)
    xt = torch.from_numpy(x).cuda()
    yt = torch.from_numpy(y).int().cuda()
    want, _ = emulate_step(plan, xt, yt)
    plan.train_step(xt, yt)
    torch.cuda.synchronize()
    errs = {n: _rel(st.grad(n) if st.segments[n].trainable else st.view(n), w) for n, w in want.items()}
    print("layerwise vs bf16-emulating oracle rel err", errs)
    bad = {n: e for n, e in errs.items() if e > tol}
    assert not bad, bad
    return plan


def test_model_b_layerwise_matches_bf16_oracle():
    import tensorflow_distributed_example_amd as tde
    m = tde.zoo.mnist_bn_cnn()
    for l in m.layers:
        if isinstance(l, tde.keras.layers.Dropout):
            l.rate = 0.0
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
    m.build()
    rng = np.random.default_rng(0)
    _emulated_compare(m, rng.random((64, 784), dtype=np.float32), rng.integers(0, 10, 64), 64, 1e-2)


@pytest.mark.parametrize("name", ["lenet5", "mnist_mlp"])
def test_baseline_config_models_layerwise_match_bf16_oracle(name, monkeypatch):
    """LeNet-5 (5x5 narrow convs, two pools, three Dense) and the dense MLP on the layer-wise plan (the
    default plan for them is the fused small-net plan: tests/test_smallnet_gpu.py)."""
    import tensorflow_distributed_example_amd as tde
    monkeypatch.setenv("TDE_SMALLNET", "0")
    tde.backend.set_random_seed(0)
    m = getattr(tde.zoo, name)()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(2)
    _emulated_compare(m, rng.random((128, 28, 28, 1), dtype=np.float32), rng.integers(0, 10, 128), 128, 1e-2)


def _mini_resnet(tde):
    # stem + identity block + projection block: every ResNet stage kind, shallow enough that
    # 1-ulp bf16 rounding flips (fp32 vs fp64 accumulation order) do not compound
    return tde.zoo.resnet((1, 1), (16, 32), input_shape=(32, 32, 3), classes=10, name="mini_resnet")


def test_small_resnet_layerwise_matches_bf16_oracle():
    import tensorflow_distributed_example_amd as tde
    m = _mini_resnet(tde)
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(1)
    # BN backward at small spatial sizes amplifies 1-ulp bf16 rounding flips (fp32 vs fp64 accumulation
    # order) by ~3x per block going backwards (head 5e-4 -> stem 3e-2); a wiring error (lost shortcut
    # gradient, wrong accumulate flag, wrong residual) is O(1)
    _emulated_compare(m, rng.standard_normal((16, 32, 32, 3), dtype=np.float32), rng.integers(0, 10, 16), 16, 6e-2)


def test_small_resnet_halo_stage_matches_bf16_oracle():
    """A 64-filter first stage at 16x16 runs its 3x3 convs (forward and input gradient, accumulated into the
    shortcut's gradient) through the persistent halo-tile kernel (csrc/kernels/haloconv.hip)."""
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import layerwise as LW
    m = tde.zoo.resnet((1, 1), (64, 32), input_shape=(64, 64, 3), classes=10, name="halo_resnet")
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(3)
    plan = _emulated_compare(m, rng.standard_normal((8, 64, 64, 3), dtype=np.float32), rng.integers(0, 10, 8), 8,
                             6e-2)
    halo = [st for st in plan.stages if isinstance(st, LW._Gemm) and st.halo]
    assert len(halo) == 2, [st.layer.name for st in halo]


def _grad_compare(model, x, y, B, thresholds, default=0.05):
    from tensorflow_distributed_example_amd.train import program as PG
    from tensorflow_distributed_example_amd.train.layerwise import LayerwisePlan
    st = model._store
    st_ref = st.clone_to("cuda")
    plan = PG.make_plan(model, st, "cuda", B, B, model.optimizer, model.loss)
    assert isinstance(plan, LayerwisePlan)
    ref = PG.ReferencePlan(model, st_ref, "cuda", B, B, model.optimizer, model.loss)
    xt = torch.from_numpy(x).cuda()
    yt = torch.from_numpy(y).int().cuda()
    plan.train_step(xt, yt)
    ref.train_step(xt, yt.long())
    torch.cuda.synchronize()
    errs = {}
    for name in st.names(trainable=True):
        errs[name] = _rel(st.grad(name), st_ref.grad(name))
    for name in st.names(trainable=False):   # BN moving statistics after one update
        errs[name] = _rel(st.view(name), st_ref.view(name))
    print("layerwise vs reference rel err", errs)
    for name, e in errs.items():
        lim = next((v for k, v in thresholds.items() if k in name), default)
        assert e < lim, (name, e)
    return plan, ref


def test_model_b_layerwise_gradients_near_fp32_reference():
    """Against fp32 autograd: bf16 mixed precision is as far off as torch autocast-bf16 is
    (scripts/diag/bf16_grad_noise.py: 0.08-0.28 on the BN-CNN's early layers), so this is a
    coarse wiring check; the tight check is the bf16-emulating oracle above."""
    import tensorflow_distributed_example_amd as tde
    m = tde.zoo.mnist_bn_cnn()
    for l in m.layers:
        if isinstance(l, tde.keras.layers.Dropout):
            l.rate = 0.0      # the reference plan draws its mask from torch's RNG
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
    m.build()
    rng = np.random.default_rng(0)
    x = rng.random((64, 784), dtype=np.float32)
    y = rng.integers(0, 10, 64)
    plan, ref = _grad_compare(m, x, y, 64, {"moving": 1e-2, "dense_1": 0.05}, default=0.4)
    lf = tde.metrics.logs_from(plan.metrics, ["accuracy"])
    lr = tde.metrics.logs_from(ref.metrics, ["accuracy"])
    assert abs(lf["loss"] - lr["loss"]) < 1e-2 * lr["loss"]


def test_small_resnet_layerwise_gradients_near_fp32_reference():
    import tensorflow_distributed_example_amd as tde
    m = _mini_resnet(tde)
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01),
              metrics=["accuracy"])
    m.build()
    rng = np.random.default_rng(1)
    x = rng.standard_normal((16, 32, 32, 3), dtype=np.float32)
    y = rng.integers(0, 10, 16)
    _grad_compare(m, x, y, 16, {"moving": 2e-2, "fc": 0.05}, default=0.5)


def test_model_b_trains_with_dropout_and_graph():
    import tensorflow_distributed_example_amd as tde
    (xt, yt), _ = tde.data.mnist.load_data()
    xt = (xt[:4096] / 255.0).astype(np.float32).reshape(-1, 784)
    yt = yt[:4096]
    m = tde.zoo.mnist_bn_cnn()
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.05), metrics=["accuracy"],
              steps_per_execution=8)
    h = m.fit(xt, yt, batch_size=128, epochs=3, shuffle=False, verbose=0)
    prog = m._program("train", 128)
    assert prog.plan_kind == "layerwise" and prog.use_graph
    assert h.history["loss"][-1] < h.history["loss"][0]
    ev = m.evaluate(xt[:1024], yt[:1024], batch_size=128, verbose=0, return_dict=True)
    assert ev["accuracy"] > 0.5
    p = m.predict(xt[:200], batch_size=128)
    assert p.shape == (200, 10) and np.allclose(p.sum(1), 1.0, atol=1e-3)


@pytest.mark.parametrize("relu,accum", [(False, False), (True, True)])
def test_split_k_epilogue_matches_single_pass(monkeypatch, relu, accum):
    """Split-K into the f32 scratch + finalize pass == the fused single-pass epilogue."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    B, H, W, C, Co, k = 4, 14, 14, 16, 48, 3
    g = O.ConvGeom(B, H, W, C, H, W, Co, k, k, 1, 1, 1, 1)
    x = _r(B, H, W, C, seed=21)
    w = _r(k, k, C, Co, seed=22, scale=0.2)
    Wt = w.reshape(-1, Co).t().contiguous()
    bias = torch.randn(Co, device=DEV)
    y1 = _r(B, H, W, Co, seed=23)
    y2 = y1.clone()
    s1 = _stats_buf(Co)
    s2 = torch.zeros_like(s1)
    O.conv_fwd(x, Wt, y1, g, bias=bias, relu=relu, colstats=s1)
    scratch = torch.zeros(B * H * W * Co, device=DEV)
    monkeypatch.setattr(O, "fwd_splits", lambda M, N_, K: 4)
    if accum:   # exercise the += path through conv_dgrad's accumulate flag instead
        dx1 = _r(B, H, W, C, seed=24)
        dx2 = dx1.clone()
        monkeypatch.setattr(O, "fwd_splits", lambda M, N_, K: 1)
        O.conv_dgrad(y1, w.contiguous(), dx1, g, accum=True)
        monkeypatch.setattr(O, "fwd_splits", lambda M, N_, K: 4)
        O.conv_dgrad(y1, w.contiguous(), dx2, g, accum=True, scratch=scratch)
        torch.cuda.synchronize()
        assert _rel(dx2.float(), dx1.float()) < 1e-2
    O.conv_fwd(x, Wt, y2, g, bias=bias, relu=relu, colstats=s2, scratch=scratch)
    torch.cuda.synchronize()
    assert _rel(y2.float(), y1.float()) < 1e-2
    assert _rel(_sum_slots(s2, Co), _sum_slots(s1, Co)) < 1e-4
    assert scratch.abs().max().item() == 0.0      # finalize re-zeroed it


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", [c for c in CONV_CASES if c[4] <= 32])
def test_smallconv_direct_kernels(B, H, W, C, Co, k, s, pad):
    """Direct VALU conv (narrow layers) vs the torch fp32 reference: forward (+bias, ReLU, BN stats) and dgrad."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    if not O.smallconv_ok(g):
        pytest.skip("too wide for the direct kernel")
    x = _r(B, H, W, C, seed=31)
    w = _r(k, k, C, Co, seed=32, scale=0.2)
    bias = torch.randn(Co, generator=torch.Generator().manual_seed(34)).to(DEV)
    y = torch.zeros(B, Ho, Wo, Co, dtype=bf, device=DEV)
    st_raw = _stats_buf(Co)
    O.smallconv_fwd(x, w.contiguous(), y, g, bias=bias, relu=False, colstats=st_raw)
    st = _sum_slots(st_raw, Co)
    xr = _cpu64(x).permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), _cpu64(w).permute(3, 2, 0, 1), _cpu64(bias), stride=s)
    ref = ref.permute(0, 2, 3, 1)
    dy = _r(B, Ho, Wo, Co, seed=33)
    ref.backward(_cpu64(dy))
    ref, xgrad = _dev(ref.detach()), _dev(xr.grad)
    dx = torch.zeros(B, H, W, C, dtype=bf, device=DEV)
    O.smallconv_dgrad(dy, w.contiguous(), dx, g)
    torch.cuda.synchronize()
    rs = ref.detach().to(bf).double()
    assert _rel(y.float(), ref) < 1e-2
    assert (st[:Co] - rs.sum((0, 1, 2))).abs().max().item() <= 1e-4 * rs.abs().sum((0, 1, 2)).max().item() + 1e-3
    assert _rel(st[Co:], (rs ** 2).sum((0, 1, 2))) < 1e-3
    assert _rel(dx.float(), xgrad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("B,H,W,C,Co,k,s", [(3, 224, 224, 3, 64, 7, 2), (2, 15, 17, 3, 8, 7, 2), (2, 28, 28, 6, 12, 6, 2),
                                            (1, 9, 9, 5, 4, 3, 1)])
def test_im2col_exact(B, H, W, C, Co, k, s):
    """im2col is a pure copy: bitwise equal to a torch-built patch matrix (row-staged LDS kernel for
    the ResNet stem, zero columns up to Kp) and the zero-padded weight copy."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
    Ho, Wo = -(-H // s), -(-W // s)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    x = _r(B, H, W, C, seed=44)
    w = _r(k, k, C, Co, seed=45)
    Kp = -(-g.K // 8) * 8
    xcol = torch.full((B * Ho * Wo * Kp,), 7.0, dtype=bf, device=DEV)
    Wt_pad = torch.full((Co * Kp,), 7.0, dtype=bf, device=DEV)
    wt = w.reshape(-1, Co).t().contiguous()
    O.im2col(x, g, xcol, wt, Wt_pad)
    xp = F.pad(x, (0, 0, pl, pr + s, pt, pb + s))
    taps = [xp[:, i:i + s * (Ho - 1) + 1:s, j:j + s * (Wo - 1) + 1:s, :] for i in range(k) for j in range(k)]
    ref = torch.stack(taps, 3).reshape(B * Ho * Wo, g.K)
    ref = F.pad(ref, (0, Kp - g.K)).reshape(-1)
    torch.cuda.synchronize()
    assert torch.equal(xcol, ref)
    assert torch.equal(Wt_pad, F.pad(wt, (0, Kp - g.K)).reshape(-1))


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", [(2, 15, 15, 3, 64, 7, 2, "same"), (4, 28, 28, 6, 12, 6, 2, "same"),
                                                (2, 14, 14, 12, 24, 6, 2, "same")])
def test_im2col_conv_path(B, H, W, C, Co, k, s, pad):
    """Explicit im2col (C % 8 != 0) + vector GEMMs: forward with BN statistics and weight gradient."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
    Ho, Wo = -(-H // s), -(-W // s)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    x = _r(B, H, W, C, seed=41)
    w = _r(k, k, C, Co, seed=42, scale=0.2)
    Kp = -(-g.K // 8) * 8
    xcol = torch.zeros(B * Ho * Wo * Kp, dtype=bf, device=DEV)
    Wt_pad = torch.zeros(Co * Kp, dtype=bf, device=DEV)
    O.im2col(x, g, xcol, w.reshape(-1, Co).t().contiguous(), Wt_pad)
    y = torch.zeros(B, Ho, Wo, Co, dtype=bf, device=DEV)
    st_raw = _stats_buf(Co)
    O.conv_fwd_im2col(xcol, Wt_pad, y, g, Kp, colstats=st_raw)
    st = _sum_slots(st_raw, Co)
    dy = _r(B, Ho, Wo, Co, seed=43)
    dW = torch.zeros(k, k, C, Co, device=DEV)
    O.conv_wgrad_im2col(xcol, dy, dW, g, Kp)
    xr = _cpu64(x).permute(0, 3, 1, 2)
    wr = _cpu64(w).permute(3, 2, 0, 1).requires_grad_(True)
    ref = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wr, stride=s).permute(0, 2, 3, 1)
    ref.backward(_cpu64(dy))
    ref, wgrad = _dev(ref.detach()), _dev(wr.grad)
    torch.cuda.synchronize()
    assert _rel(y.float(), ref) < 1e-2
    assert _rel(st[Co:], (ref.detach().to(bf).double() ** 2).sum((0, 1, 2))) < 1e-3
    assert _rel(dW, wgrad.permute(2, 3, 1, 0)) < 1e-3


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", [(128, 28, 28, 1, 6, 3, 1, "same"), (7, 13, 11, 1, 16, 2, 2, "same"),
                                                (3, 9, 9, 2, 5, 2, 1, "valid"), (5, 12, 12, 1, 32, 2, 1, "same"),
                                                # tap-chunked (K*round8(Co) > 128): LeNet-5 conv1, Co=24 and 32
                                                (128, 28, 28, 1, 6, 5, 1, "same"), (4, 10, 10, 2, 20, 3, 1, "same"),
                                                (3, 11, 11, 3, 32, 3, 2, "valid")])
def test_smallconv_wgrad(B, H, W, C, Co, k, s, pad):
    """Register-resident weight gradient (Model B conv1: 3x3x1 -> 6 over B*784 pixels) vs the fp64 oracle."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    assert O.smallconv_wgrad_ok(g)
    x = _r(B, H, W, C, seed=41)
    dy = _r(B, Ho, Wo, Co, seed=42)
    dW0 = torch.randn(k, k, C, Co, device=DEV)
    dW = dW0.clone()
    O.smallconv_wgrad(x, dy, dW, g)
    wr = torch.zeros(Co, C, k, k, dtype=torch.float64, requires_grad=True)
    out = F.conv2d(F.pad(_cpu64(x).permute(0, 3, 1, 2), (pl, pr, pt, pb)), wr, stride=s)
    out.backward(_cpu64(dy).permute(0, 3, 1, 2))
    ref = _dev(wr.grad.permute(2, 3, 1, 0)) + dW0.double()
    torch.cuda.synchronize()
    assert _rel(dW.double(), ref) < 1e-5


def test_conv_and_dense_with_largest_tiles():
    """TDE_IGEMM_TILE_MIN=1 makes every fwd/dgrad/dense GEMM take the largest tile (128x128 / 128x64)
    that the 2048-workgroup default now rarely picks; same fp32 references, in a child process (the
    library reads the knob once)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import test_layers_gpu as t\n"
            "for c in t.CONV_CASES: t.test_conv_fwd_dgrad_wgrad(*c)\n"
            "t.test_dense_fwd_dgrad_wgrad(256, 512, 1000, False)\nprint('ok')\n" % here)
    env = dict(os.environ, TDE_IGEMM_TILE_MIN="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=os.path.dirname(here), capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_conv_big_tiles_forced():
    """The 256-row "big" implicit-GEMM tiles forced on every eligible conv case (big_min = 1) against the
    same fp32 references: fwd through g_big (KB = 64 forced so the K < 256 layers qualify too), dgrad
    through the dgrad toggle (which moves dgrad to KB = 64).  The launch counter proves the big kernels
    ran for both; defaults restored after."""
    from tensorflow_distributed_example_amd import _native as N
    lib = N.hip()
    cases = list(CONV_CASES) + [(4, 20, 20, 64, 128, 3, 1, "same"), (2, 14, 14, 128, 64, 3, 2, "same"),
                                (2, 16, 16, 64, 64, 3, 1, "same")]
    try:
        for kb in (0, 64):
            lib.tde_igemm_tune(512, 16, kb, 1, 1, 1)
            lib.tde_igemm_big_dgrad(1)
            n0 = lib.tde_igemm_big_launches()
            for c in cases:
                test_conv_fwd_dgrad_wgrad(*c)
            assert lib.tde_igemm_big_launches() > n0
        # dgrad alone (fwd big tiles off): the 64-channel stride-1 and stride-2 (phase) cases must go big
        lib.tde_igemm_tune(512, 16, 0, 1, 0, 1)
        lib.tde_igemm_big_dgrad(1)
        for c in [(2, 16, 16, 64, 64, 3, 1, "same"), (2, 14, 14, 128, 64, 3, 2, "same")]:
            n0 = lib.tde_igemm_big_launches()
            test_conv_fwd_dgrad_wgrad(*c)
            assert lib.tde_igemm_big_launches() > n0, c
    finally:
        lib.tde_igemm_tune(512, 16, 0, 1, 0, 192)
        lib.tde_igemm_big_dgrad(0)


# shapes that reach the LDS-DMA weight gradient (row-padded, batch-inner pixel order): Co > 64, C and Co
# multiples of 8, Wo <= 64 and B a multiple of the output rows per k-tile (64 / pow2(Wo))
WGRAD_DMA_CASES = [
    (8, 14, 14, 64, 128, 3, 1, "same"),    # stride 1 -> 128x128 tiles at 2 stages (Wo 14 -> 16-wide rows)
    (8, 15, 15, 64, 128, 3, 2, "same"),    # stride 2 -> 128x64 at 3 stages, asymmetric TF pads
    (8, 16, 16, 64, 128, 1, 2, "valid"),   # 1x1 stride-2 projection
    (8, 7, 7, 128, 96, 3, 1, "same"),      # Wo 7 (8-wide rows, 8 batch rows per k-tile), N tail of 96
    (4, 28, 28, 24, 96, 3, 1, "same"),     # M = 216: partial M tile, C = 24 (three 8-channel chunks per tap)
]


@pytest.mark.parametrize("mode", [3, 1, 2])
def test_conv_wgrad_lds_dma_paths(mode):
    """Every conv case above through the LDS-DMA weight gradient (auto per-shape choice, forced 3 stages,
    forced 2 stages) against the float64 references of test_conv_fwd_dgrad_wgrad; the launch counter
    proves the path ran; the default (3 = per shape) is restored after."""
    from tensorflow_distributed_example_amd import _native as N
    lib = N.hip()
    try:
        lib.tde_igemm_wgrad_dma(mode)
        for c in WGRAD_DMA_CASES:
            n0 = lib.tde_igemm_wgrad_dma_launches()
            test_conv_fwd_dgrad_wgrad(*c)
            assert lib.tde_igemm_wgrad_dma_launches() > n0, c
    finally:
        lib.tde_igemm_wgrad_dma(3)


def _hyp():
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    return HealthCheck, given, settings, st


_HC, _given, _settings, _st = _hyp()


@_settings(max_examples=30, deadline=None, suppress_health_check=[_HC.too_slow], derandomize=True)
@_given(B=_st.integers(1, 4), H=_st.integers(3, 20), W=_st.integers(3, 20), C=_st.sampled_from([1, 3, 8, 16, 24, 64]),
        Co=_st.sampled_from([6, 8, 16, 40, 64, 96, 128]), k=_st.integers(1, 5), s=_st.integers(1, 3),
        pad=_st.sampled_from(["same", "valid"]))
def test_conv_kernels_random_geometries(B, H, W, C, Co, k, s, pad):
    """Property test: random (B, H, W, C, Co, k, s, padding) — TF-SAME asymmetric pads,
    strides 1-3, channel counts on and off the 16-byte vector paths — through the HIP implicit-GEMM fwd /
    dgrad (stride-phase) / wgrad against the float64 references of test_conv_fwd_dgrad_wgrad.  Derandomized
    so a GPU run is reproducible."""
    if pad == "valid" and (k > H or k > W):
        return
    test_conv_fwd_dgrad_wgrad(B, H, W, C, Co, k, s, pad)


@pytest.mark.parametrize("B,H,W,C,Co,k,s", [(2, 32, 32, 3, 64, 7, 2), (3, 29, 23, 3, 16, 7, 2), (2, 20, 20, 1, 8, 3, 2),
                                            (2, 17, 18, 4, 64, 5, 2)])
def test_stem_pack_conv_fwd_wgrad(B, H, W, C, Co, k, s):
    """The packed stem (tde_stem_pack: two pixels x 4 channels per virtual pixel, a valid stride-(s, 1) conv
    with ceil(k/2) taps, row-tile LDS-DMA when that row is one 32-wide k-tile) against the float64 conv of
    the real layer with TF-SAME pads; its weight gradient unpacked into the real [k, k, C, Co] layout."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
    Ho, Wo = -(-H // s), -(-W // s)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    gv = O.stem_geometry(g)
    x = _r(B, H, W, C, seed=11)
    w = _r(k, k, C, Co, seed=12, scale=0.2)
    bias = torch.randn(Co, device=DEV)
    xp = torch.full((gv.B * gv.H * gv.W * 8,), float("nan"), device=DEV).to(bf)
    Wv = torch.full((Co * gv.K,), float("nan"), device=DEV).to(bf)
    O.stem_pack(x, g, xp, w.reshape(-1, Co).t().contiguous(), Wv)
    y = torch.zeros(B, Ho, Wo, Co, dtype=bf, device=DEV)
    O.conv_fwd(xp, Wv.view(Co, -1), y, gv, bias=bias)
    xr = _cpu64(x).permute(0, 3, 1, 2).requires_grad_(True)
    wr = _cpu64(w).permute(3, 2, 0, 1).requires_grad_(True)
    ref = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wr, _cpu64(bias), stride=s).permute(0, 2, 3, 1)
    dy = _r(B, Ho, Wo, Co, seed=13)
    ref.backward(_cpu64(dy))
    torch.cuda.synchronize()
    assert _rel(y.float(), _dev(ref.detach())) < 1e-2
    gWv = torch.zeros(gv.K * Co, device=DEV)
    gW = torch.randn(k, k, C, Co, device=DEV)
    gW0 = gW.clone()
    O.conv_wgrad(xp, dy, gWv, gv)
    O.stem_unpack_wgrad(gWv, g, gW)
    torch.cuda.synchronize()
    assert _rel(gW - gW0, _dev(wr.grad.permute(2, 3, 1, 0))) < 1e-3
    assert float(gWv.abs().max()) == 0.0   # re-armed for the next step's accumulation


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", [(4, 14, 14, 16, 24, 6, 2, "same"), (2, 17, 15, 8, 24, 3, 2, "same"),
                                                (2, 15, 15, 64, 128, 3, 2, "same")])
def test_strided_dgrad_single_launch_matches_per_phase(B, H, W, C, Co, k, s, pad, monkeypatch):
    """All stride phases of a strided conv's input gradient in ONE launch (grid z = phase, per-phase M / K
    from the kernel's phase table) equals the per-phase launches bit for bit, store and accumulate modes."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    (pt, _), (pl, _) = _tf_same(H, k, s), _tf_same(W, k, s)
    Ho, Wo = -(-H // s), -(-W // s)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    w = _r(k, k, C, Co, seed=21, scale=0.2)
    dy = _r(B, Ho, Wo, Co, seed=22)
    outs = []
    for multi in ("1", "0"):
        monkeypatch.setenv("TDE_DGRAD_MULTIPHASE", multi)
        dx = torch.full((B, H, W, C), float("nan"), device=DEV).to(bf)
        O.conv_dgrad(dy, w.contiguous(), dx, g)
        dx2 = _r(B, H, W, C, seed=23)
        O.conv_dgrad(dy, w.contiguous(), dx2, g, accum=True)
        outs.append((dx, dx2))
    torch.cuda.synchronize()
    assert not torch.isnan(outs[0][0].float()).any()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("B,H,W,C,mode", [(2, 112, 112, 64, 1), (3, 15, 13, 16, 1), (2, 16, 16, 64, 2)])
def test_bn_relu_maxpool_fused_matches_two_passes(B, H, W, C, mode):
    """The stem's BN + ReLU + MaxPool(3, 2, same) in one pass (tde_bn_relu_maxpool_fwd) gives the pooled
    output, argmax bytes, saved statistics, moving averages and zeroed accumulators of bn_fwd + maxpool_fwd
    bit for bit (the BN output is never stored)."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    R = B * H * W
    Ho, Wo = -(-H // 2), -(-W // 2)
    (pt, _), (pl, _) = _tf_same(H, 3, 2), _tf_same(W, 3, 2)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, C, 3, 3, 2, 2, pt, pl)
    y = _r(R, C, seed=41, scale=2.0) + 0.2
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.3
    stats = _stats_buf(C)
    O.colstats(y, R, C, stats)
    outs = []
    for fused in (False, True):
        saved = torch.zeros(2 * C, device=DEV)
        mm, mv = torch.full((C,), 0.1, device=DEV), torch.full((C,), 0.9, device=DEV)
        zb = torch.full((2 * SLOTS * C,), 3.0, device=DEV)
        pooled = torch.full((B * Ho * Wo * C,), float("nan"), device=DEV).to(bf)
        idx = torch.full((B * Ho * Wo * C,), 77, dtype=torch.uint8, device=DEV)
        kw = dict(mode=mode, stats=stats if mode == 1 else None, saved=saved if mode == 1 else None, gamma=gamma,
                  beta=beta, eps=1e-5, mmean=mm, mvar=mv, momentum=0.9, bessel=R / (R - 1),
                  zero_buf=zb if mode == 1 else None)
        if fused:
            O.bn_relu_maxpool_fwd(y, R, C, pooled, idx, g, **kw)
        else:
            out = torch.zeros(R, C, dtype=bf, device=DEV)
            O.bn_fwd(y, out, R, C, relu=True, **kw)
            O.maxpool_fwd(out, pooled, idx, g)
        outs.append((pooled, idx, saved, mm, mv, zb))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert not torch.isnan(outs[1][0].float()).any()
    # and against fp64 torch: relu(bn(y)) then max_pool2d with TF-SAME padding (-inf pads)
    mean, var = _cpu64(y).mean(0), _cpu64(y).var(0, unbiased=False)
    if mode == 2:
        mean, var = torch.full((C,), 0.1, dtype=torch.float64), torch.full((C,), 0.9, dtype=torch.float64)
    z = torch.relu((_cpu64(y) - mean) / torch.sqrt(var + 1e-5) * _cpu64(gamma) + _cpu64(beta))
    z = z.view(B, H, W, C).permute(0, 3, 1, 2)
    (_, pb), (_, pr) = _tf_same(H, 3, 2), _tf_same(W, 3, 2)
    ref = F.max_pool2d(F.pad(z, (pl, pr, pt, pb), value=float("-inf")), 3, 2).permute(0, 2, 3, 1).reshape(-1)
    assert _rel(outs[1][0].float().cpu(), ref) < 1e-2
    if mode != 1:
        return
    # backward: pool backward + two-pass BN backward vs the fused gather (the pool's input gradient never stored)
    idx, saved = outs[1][1], outs[1][2]
    dpool = _r(B * Ho * Wo * C, seed=42)
    grads = []
    for fused in (False, True):
        dst = torch.zeros(2 * SLOTS * C, device=DEV)
        dx = torch.full((R, C), float("nan"), device=DEV).to(bf)
        dg, db = torch.ones(C, device=DEV), torch.ones(C, device=DEV)
        zf = _stats_buf(C).fill_(1.0)
        if fused:
            O.bn_pool_bwd(dpool, idx, y, R, C, g, saved=saved, dstats=dst, dx=dx, gamma=gamma, beta=beta, relu=True,
                          dgamma=dg, dbeta=db, zero_fwd=zf)
        else:
            dout = torch.full((R, C), float("nan"), device=DEV).to(bf)
            O.maxpool_bwd(dpool, idx, dout, g)
            O.bn_bwd(dout, y, R, C, mode=1, saved=saved, gamma=gamma, beta=beta, relu=True, dstats=dst, dx=dx,
                     dgamma=dg, dbeta=db, zero_fwd=zf)
        grads.append((dx, dg, db, zf))
    torch.cuda.synchronize()
    (dx0, dg0, db0, zf0), (dx1, dg1, db1, zf1) = grads
    assert not torch.isnan(dx1.float()).any()
    assert _rel(dx1.float(), dx0.float()) < 2e-3
    assert _rel(dg1, dg0) < 1e-4 and _rel(db1, db0) < 1e-4
    assert zf1.abs().max().item() == 0.0 and zf0.abs().max().item() == 0.0


def test_resnet18_plan_fuses_stem_bn_pool():
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import layerwise as LW
    m = tde.zoo.resnet18()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1))
    plan = m._program("train", 8).plans[0]
    fused = [st for st in plan.stages if isinstance(st, LW._Elementwise) and st.pool is not None]
    assert [st.layer.name for st in fused] == ["conv1_bn"]
    assert fused[0].pool.fused


def test_fused_stem_fit_evaluate_predict_match_unfused(monkeypatch):
    """A mini ResNet trained, evaluated and used for prediction with the fused stem (BN + ReLU + MaxPool,
    TDE_BN_POOL=1) and without it: same losses, metrics, moving statistics and predictions (the forward is
    bit-identical; the backward differs only in the BN sums' summation order)."""
    import tensorflow_distributed_example_amd as tde
    rng = np.random.default_rng(5)
    x = rng.standard_normal((32, 32, 32, 3), dtype=np.float32)
    y = rng.integers(0, 10, 32)
    runs = []
    init = None
    for fused in ("0", "1"):
        monkeypatch.setenv("TDE_BN_POOL", fused)
        tde.backend.set_random_seed(3)
        m = _mini_resnet(tde)
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01),
                  metrics=["accuracy"])
        m.build()
        if init is None:
            init = m.get_weights()
        else:
            m.set_weights(init)
        h = m.fit(x, y, batch_size=16, epochs=1, verbose=0, shuffle=False)
        ev = m.evaluate(x, y, batch_size=16, verbose=0, return_dict=True)
        pr = m.predict(x, batch_size=16)
        runs.append((h.history["loss"][0], ev, np.asarray(pr), m.get_weights()))
    (l0, e0, p0, w0), (l1, e1, p1, w1) = runs
    assert abs(l0 - l1) <= 1e-3 * abs(l0)
    assert abs(e0["loss"] - e1["loss"]) <= 1e-2 * abs(e0["loss"])
    assert np.abs(p0 - p1).max() <= 1e-2 * (np.abs(p0).max() + 1e-6)
    for a, b in zip(w0, w1):
        assert np.abs(a - b).max() <= 1e-2 * (np.abs(a).max() + 1e-3)


@pytest.mark.parametrize("R,C,drop", [(128, 200, 0.5), (128, 200, 0.0), (1000, 72, 0.3)])
def test_bn_bwd_few_rows_with_dropout(R, C, drop):
    """BN + ReLU + dropout backward over few rows (a Dense layer's BN; bn_bwd_reduce_cols_kernel): the
    regenerated per-element dropout masks match the forward's, and dgamma / dbeta / dx match torch."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    y = _r(R, C, seed=51, scale=1.5) + 0.2
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    stats = _stats_buf(C)
    O.colstats(y, R, C, stats)
    saved = torch.zeros(2 * C, device=DEV)
    dstats = torch.zeros(2 * SLOTS * C, device=DEV)
    out = torch.zeros(R, C, dtype=bf, device=DEV)
    it = torch.zeros(1, dtype=torch.int64, device=DEV)
    d = O.DropSpec(drop, 1234, it, 3) if drop else O.DropSpec()
    O.bn_fwd(y, out, R, C, mode=1, stats=stats, saved=saved, gamma=gamma, beta=beta, eps=1e-3, zero_buf=dstats,
             relu=True, drop=d, iter_offset=0)
    dout = _r(R, C, seed=52)
    dx = torch.zeros(R, C, dtype=bf, device=DEV)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    O.bn_bwd(dout, y, R, C, mode=1, saved=saved, gamma=gamma, beta=beta, relu=True, drop=d, iter_offset=0,
             dstats=dstats, dx=dx, dgamma=dg, dbeta=db)
    torch.cuda.synchronize()
    yd = _cpu64(y)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    xhat = (yd - mean) / torch.sqrt(var + 1e-3)
    zr = torch.relu(xhat * _cpu64(gamma) + _cpu64(beta))
    o = _cpu64(out)
    if drop:
        # the mask the kernels draw for this (seed, step, layer): the same dropout over an all-ones input
        # normalised by moving statistics (0, 1) reads it out exactly
        ones = torch.ones(R, C, dtype=bf, device=DEV)
        out2 = torch.zeros(R, C, dtype=bf, device=DEV)
        O.bn_fwd(ones, out2, R, C, mode=2, eps=0.0, mmean=torch.zeros(C, device=DEV), mvar=torch.ones(C, device=DEV),
                 relu=True, drop=d, iter_offset=0)
        torch.cuda.synchronize()
        inv = torch.tensor(1.0 / (1 - drop)).to(torch.bfloat16).item()
        ks = _cpu64(out2)
        assert set(torch.unique(ks).tolist()) <= {0.0, inv}
        ks = (ks > 0).double() / (1 - drop)
        assert 0.3 < (ks > 0).double().mean().item() < 0.9
        assert torch.allclose(o, (zr * ks).to(torch.bfloat16).double(), rtol=2e-2, atol=2e-2)   # the forward's mask
    else:
        ks = torch.ones_like(zr)
    dz = _cpu64(dout) * ks * (zr > 0)
    assert _rel(db.cpu(), dz.sum(0)) < 1e-2
    assert _rel(dg.cpu(), (dz * xhat).sum(0)) < 1e-2
    dxr = _cpu64(gamma) / torch.sqrt(var + 1e-3) * (dz - dz.mean(0) - xhat * (dz * xhat).mean(0))
    assert _rel(dx.float().cpu(), dxr) < 3e-2


def test_igemm_mfma32_paths():
    """Every LDS-DMA implicit-GEMM path on v_mfma_f32_32x32x16_bf16 (TDE_MFMA32 mask 7: fwd / dense, dgrad,
    weight gradients) against the float64 references of the conv / dense tests, at the default tile choice and
    with the largest tiles forced (128x128 / 128x64: 2x2 / 2x1 fragments of 32x32 per wave); the launch counter
    proves the 32x32 kernels ran; the defaults are restored after."""
    from tensorflow_distributed_example_amd import _native as N
    lib = N.hip()
    cases = (list(CONV_CASES) + list(WGRAD_DMA_CASES)
             + [(4, 20, 20, 64, 128, 3, 1, "same"), (2, 14, 14, 128, 64, 3, 2, "same"), (2, 16, 16, 64, 64, 3, 1, "same"),
                (2, 12, 12, 256, 256, 3, 1, "same")])
    try:
        lib.tde_igemm_mfma32(7)
        for tmin in (2048, 1):
            lib.tde_igemm_tile_min(tmin)
            n0 = lib.tde_igemm_mfma32_launches()
            for c in cases:
                test_conv_fwd_dgrad_wgrad(*c)
            for d in [(128, 1176, 200, False), (256, 512, 1000, False), (37, 64, 10, True)]:
                test_dense_fwd_dgrad_wgrad(*d)
            assert lib.tde_igemm_mfma32_launches() > n0, tmin
    finally:
        lib.tde_igemm_mfma32(-1)
        lib.tde_igemm_tile_min(2048)


def test_wgrad_many_split_scratch_reduction():
    """Weight gradients split 8+ ways through the partial scratch (TDE_WG_SCRATCH_MAX=64) reduce with the grouped
    fixed-order kernel (16 split groups per 64 elements): same float64 references, in a child process (the library
    reads the knob once)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import test_layers_gpu as t\n"
            "t.test_conv_fwd_dgrad_wgrad(16, 28, 28, 128, 128, 3, 1, 'same')\n"
            "t.test_conv_fwd_dgrad_wgrad(8, 16, 16, 64, 128, 3, 1, 'same')\nprint('ok')\n" % here)
    env = dict(os.environ, TDE_WG_SCRATCH_MAX="64")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=os.path.dirname(here), capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("B,H,W,C,Co,res,accum", [(4, 12, 12, 128, 128, True, False), (2, 9, 11, 64, 256, False, True),
                                                     (3, 14, 14, 256, 64, True, True)])
def test_conv_dgrad_bn_sums_match_the_reduction_pass(B, H, W, C, Co, res, accum):
    """tde_igemm_dgrad_bnsum: the consumer BN's backward sums (sum g, sum g * xhat; g masked by the BN's ReLU over
    y + residual) taken in the input-gradient epilogue equal those of the separate reduction pass over the stored
    gradient, and the apply pass that reads them gives the same BN input gradient; the GEMM output itself is
    unchanged (bitwise), also when it accumulates into an existing gradient."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    g = O.ConvGeom(B, H, W, C, H, W, Co, 3, 3, 1, 1, 1, 1)
    assert O.dgrad_bnsum_ok(g)
    n = B * H * W * C
    dy = _r(B, H, W, Co, seed=21)
    w = _r(3, 3, C, Co, seed=22, scale=0.05).contiguous()
    y = _r(B, H, W, C, seed=23)
    rs_ = _r(B, H, W, C, seed=24) if res else None
    gen = torch.Generator(device="cpu").manual_seed(25)
    saved = torch.cat([torch.randn(C, generator=gen) * 0.1, torch.rand(C, generator=gen) + 0.5]).to(DEV)
    gamma = (torch.rand(C, generator=gen) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=gen) * 0.1).to(DEV)
    base = _r(B, H, W, C, seed=26).reshape(-1)
    outs = []
    for fused in (False, True):
        dx = base.clone() if accum else torch.zeros(n, dtype=bf, device=DEV)
        ds = torch.zeros(2 * O.STAT_SLOTS * C, device=DEV)
        bn = dict(y=y.reshape(-1), res=rs_.reshape(-1) if res else None, saved=saved, gamma=gamma, beta=beta,
                  relu=True, dstats=ds)
        O.conv_dgrad(dy.reshape(-1), w, dx, g, accum=accum, bnsum=bn if fused else None)
        dxb = torch.zeros(n, dtype=bf, device=DEV)
        O.bn_bwd(dx, y.reshape(-1), B * H * W, C, mode=1, saved=saved, gamma=gamma, beta=beta,
                 res=rs_.reshape(-1) if res else None, relu=True, dstats=ds, dx=dxb, sums_ready=fused)
        torch.cuda.synchronize()
        outs.append((dx.clone(), ds.view(O.STAT_SLOTS, 2, C).sum(0).double(), dxb.clone()))
    (dxa, sa, ba), (dxf, sf, bf_) = outs
    assert torch.equal(dxa, dxf)
    for q in range(2):
        assert (sa[q] - sf[q]).abs().max().item() <= 1e-4 * sa[q].abs().max().item() + 1e-4, q
    assert _rel(bf_.float(), ba.float()) < 1e-2


def test_resnet_bn_sums_in_dgrad_epilogue_match_bf16_oracle(monkeypatch):
    """BatchNormalization backward sums taken by the epilogue of the stride-1 input-gradient GEMM that writes the
    BN output's gradient last (csrc/kernels/layers.hip BnSum; those BNs run their apply pass only): a ResNet whose
    stages (96 / 128 filters) take the LDS-DMA input gradient — the float64 bf16-emulating oracle, and the same
    step with the separate reduction pass (TDE_BN_SUM_FUSE=0, the default)."""
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import layerwise as LW

    def build():
        tde.backend.set_random_seed(4)
        m = tde.zoo.resnet((1, 1), (96, 128), input_shape=(32, 32, 3), classes=10, name="bnsum_resnet")
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
        m.build()
        return m

    monkeypatch.setenv("TDE_BN_SUM_FUSE", "1")
    rng = np.random.default_rng(5)
    x, y = rng.standard_normal((16, 32, 32, 3), dtype=np.float32), rng.integers(0, 10, 16)
    # (BN backward at 8x8 / 4x4 spatial sizes amplifies 1-ulp bf16 rounding flips ~3x per block going backwards,
    # as in the mini-ResNet test; a wiring error is O(1)): both plans within 0.12 of the oracle, and the fused
    # plan no further from it than the separate-pass plan plus that noise
    m = build()
    plan = _emulated_compare(m, x, y, 16, 0.12)
    fused = [st.layer.name for st in plan.stages if isinstance(st, LW._Elementwise) and st.sums_fused]
    assert len(fused) >= 2, fused
    monkeypatch.setenv("TDE_BN_SUM_FUSE", "0")
    m2 = build()
    plan2 = _emulated_compare(m2, x, y, 16, 0.12)
    assert not any(getattr(st, "sums_fused", False) for st in plan2.stages)
