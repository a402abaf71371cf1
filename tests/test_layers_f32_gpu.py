"""The float32 layer-wise kernel library (csrc/kernels/layers_f32.hip): every kernel vs a float64 torch
reference of the same op on the host, then whole models on the float32 LayerwisePlan vs the float64
oracle (train/layerwise.emulate_step, no rounding anywhere): the float32 policy — the reference's
precision (distributed_with_keras.py:21) — never computes in bf16 for models outside the fused plans."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("fp32_policy")]
DEV = "cuda"
from tensorflow_distributed_example_amd.ops.layer_ops import STAT_SLOTS as SLOTS  # noqa: E402


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _c64(t):
    return t.detach().double().cpu()


def _tf_same(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


CONV_CASES = [
    # B, H, W, C, Co, k, s, padding
    (4, 28, 28, 1, 6, 3, 1, "same"),     # Model B conv1 (C = 1: scalar gathers)
    (4, 28, 28, 6, 12, 6, 2, "same"),    # Model B conv2 (C % 4 != 0)
    (2, 16, 16, 16, 64, 3, 1, "same"),   # vector paths
    (2, 17, 15, 8, 24, 3, 2, "same"),    # odd sizes, stride 2, asymmetric pads
    (2, 15, 15, 3, 64, 7, 2, "same"),    # ResNet stem shape family
    (2, 8, 8, 64, 128, 1, 2, "valid"),   # projection shortcut
    (3, 10, 9, 32, 40, 3, 1, "valid"),   # N tail
    (2, 14, 14, 24, 48, 6, 2, "same"),   # Model B x2 conv3 (phased stride-2 input gradient, C % 4 == 0)
    (2, 9, 9, 16, 32, 1, 2, "same"),     # 1x1 stride 2 "same": three of the four phases untapped (zeros)
]


@pytest.mark.parametrize("B,H,W,C,Co,k,s,pad", CONV_CASES)
def test_conv32_fwd_dgrad_wgrad(B, H, W, C, Co, k, s, pad):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    x = _r(B, H, W, C, seed=1)
    w = _r(k, k, C, Co, seed=2, scale=0.2)
    bias = _r(Co, seed=3)
    g = O.ConvGeom(B, H, W, C, Ho, Wo, Co, k, k, s, s, pt, pl)
    xc = F.pad(_c64(x).permute(0, 3, 1, 2), (pl, pr, pt, pb))
    ref = F.conv2d(xc, _c64(w).permute(3, 2, 0, 1), stride=s).permute(0, 2, 3, 1) + _c64(bias)
    ref = F.relu(ref)
    y = torch.zeros(B, Ho, Wo, Co, device=DEV)
    stats = torch.zeros(2 * SLOTS * Co, dtype=torch.float64, device=DEV)
    O32.conv_fwd(x, w, y, g, bias=bias, relu=True, colstats=stats)
    torch.cuda.synchronize()
    assert _rel(y, ref) < 1e-6
    st = _c64(stats).view(SLOTS, 2, Co).sum(0)
    yr = _c64(y).reshape(-1, Co)
    assert _rel(st[0], yr.sum(0)) < 1e-9 and _rel(st[1], (yr * yr).sum(0)) < 1e-9
    # input / weight gradients of the linear conv
    dy = _r(B, Ho, Wo, Co, seed=4)
    xr = _c64(x).requires_grad_(True)
    wr = _c64(w).requires_grad_(True)
    o = F.conv2d(F.pad(xr.permute(0, 3, 1, 2), (pl, pr, pt, pb)), wr.permute(3, 2, 0, 1), stride=s)
    o.permute(0, 2, 3, 1).backward(_c64(dy))
    dx = torch.full((B, H, W, C), 0.5, device=DEV)
    O32.conv_dgrad(dy, w, dx, g, accum=True)   # += onto 0.5
    dW = torch.zeros_like(w)
    part = torch.empty(O32.wgrad_part_elems(g.K, Co, B * Ho * Wo) + 1, device=DEV)
    O32.conv_wgrad(x, dy, dW, g, part=part)
    torch.cuda.synchronize()
    assert _rel(dx, xr.grad + 0.5) < 1e-6
    assert _rel(dW, wr.grad) < 1e-6


def test_split_k_forward_and_input_gradient_match_float64():
    """Few output tiles, long K (a Dense(128) on Conv2D(64)'s 10,816 pooled features; a 7x7x256 conv at batch
    2): the forward / input-gradient GEMMs split K over the grid and the ordered reduce launch applies bias,
    ReLU and the BN column statistics — vs float64, and the split is really taken."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    B, fin, out = 64, 10816, 128
    assert O32.fd_splits(B, out, fin) > 1
    x, w, b = _r(B, fin, seed=11), _r(fin, out, seed=12, scale=0.02), _r(out, seed=13)
    part = torch.empty(max(O32.fd_part_elems(B, out, fin), O32.fd_part_elems(B, fin, out)) + 1, device=DEV)
    y = torch.zeros(B, out, device=DEV)
    stats = torch.zeros(2 * SLOTS * out, dtype=torch.float64, device=DEV)
    O32.dense_fwd(x, w, B, y, bias=b, relu=True, colstats=stats, part=part)
    dy = _r(B, out, seed=14)
    dx = torch.full((B, fin), 0.25, device=DEV)
    O32.dense_dgrad(dy, w, dx, B, accum=True, part=part)
    torch.cuda.synchronize()
    X, Wt = _c64(x), _c64(w)
    ref = F.relu(X @ Wt + _c64(b))
    assert _rel(y, ref) < 1e-6
    st = _c64(stats).view(SLOTS, 2, out).sum(0)
    yr = _c64(y)
    assert _rel(st[0], yr.sum(0)) < 1e-9 and _rel(st[1], (yr * yr).sum(0)) < 1e-9
    assert _rel(dx, _c64(dy) @ Wt.t() + 0.25) < 1e-6
    # conv forward / input gradient (stride 1) at few tiles
    g = O.ConvGeom(2, 7, 7, 256, 7, 7, 64, 3, 3, 1, 1, 1, 1)
    assert O32.fd_splits(g.B * g.Ho * g.Wo, g.Co, g.K) > 1 and O32.fd_splits(g.B * g.H * g.W, g.C, 9 * g.Co) > 1
    xc, wc = _r(2, 7, 7, 256, seed=15), _r(3, 3, 256, 64, seed=16, scale=0.05)
    part = torch.empty(max(O32.fd_part_elems(98, 64, g.K), O32.fd_part_elems(98, 256, 9 * 64)) + 1, device=DEV)
    yc = torch.zeros(2, 7, 7, 64, device=DEV)
    O32.conv_fwd(xc, wc, yc, g, part=part)
    dyc = _r(2, 7, 7, 64, seed=17)
    dxc = torch.zeros(2, 7, 7, 256, device=DEV)
    O32.conv_dgrad(dyc, wc, dxc, g, part=part)
    torch.cuda.synchronize()
    xr = _c64(xc).requires_grad_(True)
    o = F.conv2d(xr.permute(0, 3, 1, 2), _c64(wc).permute(3, 2, 0, 1), padding=1)
    assert _rel(yc, o.permute(0, 2, 3, 1)) < 1e-6
    o.permute(0, 2, 3, 1).backward(_c64(dyc))
    assert _rel(dxc, xr.grad) < 1e-6


@pytest.mark.parametrize("B,fin,out", [(128, 1176, 200), (37, 64, 10), (256, 512, 1000), (5, 3, 7)])
def test_dense32_fwd_dgrad_wgrad(B, fin, out):
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    x, w, b = _r(B, fin, seed=5), _r(fin, out, seed=6, scale=0.1), _r(out, seed=7)
    y = torch.zeros(B, out, device=DEV)
    O32.dense_fwd(x, w, B, y, bias=b)
    dy = _r(B, out, seed=8)
    dx = torch.zeros(B, fin, device=DEV)
    O32.dense_dgrad(dy, w, dx, B)
    dW = torch.zeros(fin, out, device=DEV)
    part = torch.empty(O32.wgrad_part_elems(fin, out, B) + 1, device=DEV)
    O32.dense_wgrad(x, dy, dW, B, part=part)
    torch.cuda.synchronize()
    X, Wt, D = _c64(x), _c64(w), _c64(dy)
    assert _rel(y, X @ Wt + _c64(b)) < 1e-6
    assert _rel(dx, D @ Wt.t()) < 1e-6
    assert _rel(dW, X.t() @ D) < 1e-6


@pytest.mark.parametrize("R,C,relu,res,rate", [(4 * 784, 6, True, False, 0.0), (128, 200, True, False, 0.5),
                                               (2 * 64, 64, True, True, 0.0), (3 * 49, 24, False, True, 0.3)])
def test_bn32_fwd_bwd(R, C, relu, res, rate):
    """Batch-statistics BN + residual + ReLU + Philox dropout forward / backward vs float64 autograd (the
    dropout mask is the host Philox4x32-10 mask at the step counter), moving statistics, accumulators."""
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    from tensorflow_distributed_example_amd.ops.philox import keep_scales
    y = _r(R, C, seed=9, scale=2.0) + 0.3
    rr = _r(R, C, seed=10) if res else None
    gamma, beta = _r(C, seed=11) * 0.2 + 1.0, _r(C, seed=12) * 0.1
    mm, mv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    stats = torch.zeros(2 * SLOTS * C, dtype=torch.float64, device=DEV)
    O32.colstats(y, R, C, stats)
    saved = torch.zeros(2 * C, device=DEV)
    dstats = torch.full((2 * SLOTS * C,), 7.0, dtype=torch.float64, device=DEV)   # zeroed by the forward
    it = torch.full((1,), 5, dtype=torch.int64, device=DEV)
    drop = O.DropSpec(rate, 1234567, it, 3) if rate > 0 else O.DropSpec()
    out = torch.zeros(R, C, device=DEV)
    O32.bn_fwd(y, out, R, C, mode=1, stats=stats, saved=saved, gamma=gamma, beta=beta, eps=1e-3, mmean=mm, mvar=mv,
               momentum=0.9, bessel=R / (R - 1), zero_buf=dstats, res=rr, relu=relu, drop=drop, iter_offset=0)
    mask = torch.ones(R, C, dtype=torch.float64)
    if rate > 0:
        mask = torch.from_numpy(keep_scales(rate, 1234567, 5, 3, R * C).reshape(R, C)).double()
    Y = _c64(y).requires_grad_(True)
    G, Bt = _c64(gamma).requires_grad_(True), _c64(beta).requires_grad_(True)
    RR = _c64(rr).requires_grad_(True) if res else None
    mean, var = Y.mean(0), Y.var(0, unbiased=False)
    z = (Y - mean) / torch.sqrt(var + 1e-3) * G + Bt
    if res:
        z = z + RR
    o = F.relu(z) if relu else z
    o = o * mask
    torch.cuda.synchronize()
    assert _rel(out, o) < 1e-6
    assert _rel(mm, 0.1 * mean.detach()) < 1e-6 and _rel(mv, 0.9 + 0.1 * var.detach() * R / (R - 1)) < 1e-6
    dout = _r(R, C, seed=13)
    o.backward(_c64(dout))
    dx = torch.zeros(R, C, device=DEV)
    dres = torch.full((R, C), 1.0, device=DEV) if res else None
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    zf = torch.full((2 * SLOTS * C,), 3.0, dtype=torch.float64, device=DEV)
    O32.bn_bwd(dout, y, R, C, mode=1, saved=saved, gamma=gamma, beta=beta, res=rr, relu=relu, drop=drop,
               iter_offset=0, dstats=torch.zeros(2 * SLOTS * C, dtype=torch.float64, device=DEV), dx=dx,
               dres=dres, dres_accum=True, dgamma=dg, dbeta=db, zero_fwd=zf)
    torch.cuda.synchronize()
    assert _rel(dx, Y.grad) < 1e-5
    assert _rel(dg, G.grad) < 1e-5 and _rel(db, Bt.grad) < 1e-5
    if res:
        assert _rel(dres, RR.grad + 1.0) < 1e-6
    assert float(_c64(dstats).abs().max()) == 0.0 and float(_c64(zf).abs().max()) == 0.0


@pytest.mark.parametrize("H,W,k,s,pad,C", [(26, 26, 2, 2, "valid", 32), (112, 112, 3, 2, "same", 16),
                                           (9, 7, 3, 2, "same", 5)])
def test_maxpool32(H, W, k, s, pad, C):
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    B = 2
    if pad == "same":
        (pt, pb), (pl, pr) = _tf_same(H, k, s), _tf_same(W, k, s)
        Ho, Wo = -(-H // s), -(-W // s)
    else:
        pt = pb = pl = pr = 0
        Ho, Wo = (H - k) // s + 1, (W - k) // s + 1
    g = O.ConvGeom(B, H, W, C, Ho, Wo, C, k, k, s, s, pt, pl)
    x = _r(B, H, W, C, seed=14)
    y = torch.zeros(B, Ho, Wo, C, device=DEV)
    idx = torch.zeros(B * Ho * Wo * C, dtype=torch.uint8, device=DEV)
    O32.maxpool_fwd(x, y, idx, g)
    X = _c64(x).requires_grad_(True)
    xp = F.pad(X.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=float("-inf"))
    ref = F.max_pool2d(xp, k, s).permute(0, 2, 3, 1)
    dy = _r(B, Ho, Wo, C, seed=15)
    ref.backward(_c64(dy))
    dx = torch.zeros(B, H, W, C, device=DEV)
    O32.maxpool_bwd(dy, idx, dx, g)
    torch.cuda.synchronize()
    assert torch.equal(_c64(y), ref.detach())
    assert _rel(dx, X.grad) < 1e-7


def test_gap_pad_xent32():
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.ops import layer_ops32 as O32
    B, HW, C = 3, 49, 40
    x = _r(B, HW, C, seed=16)
    y = torch.zeros(B, C, device=DEV)
    O32.gap_fwd(x, y, B, HW, C)
    dy = _r(B, C, seed=17)
    dx = torch.ones(B, HW, C, device=DEV)
    O32.gap_bwd(dy, dx, B, HW, C, accum=True)
    torch.cuda.synchronize()
    assert _rel(y, _c64(x).mean(1)) < 1e-6
    # f32: 1/HW, the product and the +1 residual each round once (≈ 3 half-ulps of a value near 1)
    assert _rel(dx, _c64(dy)[:, None, :] / HW + 1.0) < 4e-7
    g = O.ConvGeom(2, 5, 6, 3, 8, 9, 3, 1, 1, 1, 1, 1, 2)
    xp = _r(2, 5, 6, 3, seed=18)
    yp = torch.zeros(2, 8, 9, 3, device=DEV)
    O32.pad_fwd(xp, yp, g)
    ref = F.pad(_c64(xp), (0, 0, 2, 1, 1, 2))
    dyp = _r(2, 8, 9, 3, seed=19)
    dxp = torch.zeros(2, 5, 6, 3, device=DEV)
    O32.pad_bwd(dyp, dxp, g)
    torch.cuda.synchronize()
    assert torch.equal(_c64(yp), ref) and torch.equal(_c64(dxp), _c64(dyp)[:, 1:6, 2:8, :])
    Bx, Cx = 70, 1000
    logits = _r(Bx, Cx, seed=20, scale=3.0)
    labels = torch.randint(0, Cx, (Bx,), generator=torch.Generator().manual_seed(0)).int().to(DEV)
    dl = torch.zeros(Bx, Cx, device=DEV)
    met = torch.zeros(4, device=DEV)
    it = torch.zeros(1, dtype=torch.int64, device=DEV)
    O32.xent(logits, labels, Bx, Cx, scale=0.5, dlogits=dl, metrics=met, iterations=it)
    L = _c64(logits).requires_grad_(True)
    loss = F.cross_entropy(L, _c64(labels).long(), reduction="sum")
    (loss * 0.5).backward()
    torch.cuda.synchronize()
    assert abs(met[0].item() - loss.item()) < 1e-5 * loss.item() and met[2].item() == Bx
    assert met[1].item() == (L.argmax(1) == _c64(labels).long()).sum().item()
    assert _rel(dl, L.grad) < 1e-6 and it.item() == 1


def _f32_oracle_compare(model, x, y, B, tol):
    """The float32 layer-wise plan vs the float64 oracle (no rounding): every gradient and moving
    statistic."""
    from tensorflow_distributed_example_amd.train import program as PG
    from tensorflow_distributed_example_amd.train.layerwise import LayerwisePlan, emulate_step
    st = model._store
    plan = PG.make_plan(model, st, "cuda", B, B, model.optimizer, model.loss, prefer="layerwise")
    assert isinstance(plan, LayerwisePlan) and plan.compute_dtype == "fp32" and plan.f32
    assert all(t.buf is None or t.buf.dtype == torch.float32 for t in plan.T.values())
    xt = torch.from_numpy(x).cuda()
    yt = torch.from_numpy(y).int().cuda()
    want, _ = emulate_step(plan, xt, yt)
    plan.train_step(xt, yt)
    torch.cuda.synchronize()
    errs = {n: _rel(st.grad(n) if st.segments[n].trainable else st.view(n), w) for n, w in want.items()}
    print("f32 layerwise vs float64 oracle rel err", errs)
    bad = {n: e for n, e in errs.items() if e > tol}
    assert not bad, bad
    return plan


def test_model_a_wide_f32_layerwise_matches_float64():
    """Model A (distributed_with_keras.py:33-39) at Conv2D(64) / Dense(128) on the float32 layer-wise plan
    (chosen explicitly: by default this width runs the generic fused plan, tests/test_convnet_gen_gpu.py)."""
    import tensorflow_distributed_example_amd as tde
    L = tde.keras.layers
    tde.backend.set_random_seed(0)
    m = tde.Sequential([L.Conv2D(64, 3, activation="relu", input_shape=(28, 28, 1)), L.MaxPooling2D(),
                        L.Flatten(), L.Dense(128, activation="relu"), L.Dense(10)])
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.001))
    m.build()
    rng = np.random.default_rng(0)
    plan = _f32_oracle_compare(m, rng.random((64, 28, 28, 1), dtype=np.float32), rng.integers(0, 10, 64), 64, 1e-5)
    # the conv's ReLU / bias backward runs inside the pool's backward; the Dense(128) forward splits K
    from tensorflow_distributed_example_amd.train import layerwise as LW
    pools = [st for st in plan.stages if isinstance(st, LW._MaxPool)]
    assert pools and pools[0].relu_from is not None and pools[0].relu_from.dz is None
    assert plan.wpart is not None


def test_model_b_doubled_f32_layerwise_matches_float64():
    """Model B (mnist_keras_distributed.py:79-109) at doubled widths (12/24/48 filters, Dense(400)), dropout
    off: past the fused BN-CNN plan's limits, so it runs on the float32 layer-wise plan."""
    import tensorflow_distributed_example_amd as tde
    L = tde.keras.layers
    tde.backend.set_random_seed(1)
    m = tde.Sequential([
        L.Reshape(input_shape=(784,), target_shape=(28, 28, 1)),
        L.Conv2D(12, 3, padding="same", use_bias=False), L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(24, 6, padding="same", use_bias=False, strides=2), L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(48, 6, padding="same", use_bias=False, strides=2), L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Flatten(), L.Dense(400, use_bias=False), L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"), L.Dropout(0.0), L.Dense(10, activation="softmax")])
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(1)
    _f32_oracle_compare(m, rng.random((128, 784), dtype=np.float32), rng.integers(0, 10, 128), 128, 1e-5)


def test_small_resnet_f32_layerwise_matches_float64():
    """Stem (padding, 7x7/2 conv, BN, ReLU, 3x3/2 max pool) + identity and projection blocks (Add) + GAP +
    Dense on the float32 layer-wise plan."""
    import tensorflow_distributed_example_amd as tde
    tde.backend.set_random_seed(2)
    m = tde.zoo.resnet((1, 1), (16, 32), input_shape=(32, 32, 3), classes=10, name="mini_resnet")
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(3)
    _f32_oracle_compare(m, rng.standard_normal((16, 32, 32, 3), dtype=np.float32), rng.integers(0, 10, 16), 16, 1e-5)


def test_f32_layerwise_fit_trains_in_graph(monkeypatch):
    """fit() on the float32 layer-wise plan (hipGraph executions): the loss falls and the plan computes
    in fp32 (no bf16 shadow exists)."""
    import tensorflow_distributed_example_amd as tde
    monkeypatch.setenv("TDE_SMALLNET", "0")
    monkeypatch.setenv("TDE_EXECUTOR", "layerwise")   # this width's default is the generic fused plan
    L = tde.keras.layers
    tde.backend.set_random_seed(4)
    m = tde.Sequential([L.Conv2D(64, 3, activation="relu", input_shape=(28, 28, 1)), L.MaxPooling2D(),
                        L.Flatten(), L.Dense(128, activation="relu"), L.Dense(10)])
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.05),
              metrics=["accuracy"], steps_per_execution=4)
    rng = np.random.default_rng(5)
    x = rng.random((64 * 8, 28, 28, 1), dtype=np.float32)
    y = (x.reshape(len(x), -1)[:, :10].argmax(1)).astype(np.int64)   # learnable labels
    h = m.fit(x, y, batch_size=64, epochs=3, verbose=0)
    prog = m._program("train", 64)
    assert prog.plan_kind == "layerwise" and prog.plans[0].compute_dtype == "fp32" and prog.use_graph
    assert not prog.plans[0].shadows
    assert h.history["loss"][-1] < h.history["loss"][0]
