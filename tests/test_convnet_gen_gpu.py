"""The generic-width fused small-CNN step (csrc/kernels/convnet_gen.hip, ``ConvNetGenPlan``) vs float64.

distributed_with_keras.py:33-43 / tf2_mnist_distributed.py:66-72 with the user's own Conv2D filters and
Dense units: the kernels must match float64 autograd at fp32 accuracy (<= 1e-5 norm-wise relative) for
every instantiated family member tested here, and a fit() of such a model must follow the float64 SGD
trajectory.  Inputs and conv weights are quantized so the conv pre-activations are exact in f32 (the pool
argmax / ReLU decisions are then the same in both precisions; see test_fp32_gpu.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("fp32_policy")]

DEV = "cuda"
TOL = 1e-5


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _qdata(B, seed, H=28, W=28, ncls=10):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randint(0, 17, (B, H, W, 1), generator=g).float() / 16.0
    y = torch.randint(0, ncls, (B,), generator=g).int()
    return x.to(DEV), y.to(DEV)


def _ref_convpool(x, w, b):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b)
    return F.max_pool2d(F.relu(y), 2).permute(0, 2, 3, 1)


CASES = [  # (filters, units, batch, Dense ReLU, H, W, classes)
    (16, 32, 64, True, 28, 28, 10),
    (64, 128, 130, True, 28, 28, 10),
    (48, 96, 37, False, 28, 28, 10),
    (32, 128, 64, True, 28, 28, 10),
    (64, 32, 100, True, 20, 24, 16),
    (16, 64, 200, True, 28, 28, 3),
    (32, 256, 64, True, 28, 28, 10),
    (48, 192, 70, True, 28, 28, 10),
    (64, 160, 64, False, 28, 28, 10),
    (16, 224, 96, True, 24, 20, 12),
]


@pytest.mark.parametrize("CC,HD,B,relu,H,W,NC", CASES)
def test_cgen_step_kernels_match_float64(CC, HD, B, relu, H, W, NC):
    """Forward (pooled tile, argmax, Dense pre-activation into 4 split-K replicas) and backward (every
    gradient, metrics, the other parity zeroed, the step counter advanced) vs float64 torch."""
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(100 + CC + HD)
    Pn = ((H - 2) // 2) * ((W - 2) // 2)
    Kf = Pn * CC
    Bp = (B + 7) // 8 * 8
    x, lab = _qdata(B, 5 + CC, H, W, NC)
    w = (torch.randint(-32, 33, (3, 3, 1, CC), generator=g).float() / 64).to(DEV)
    b = (torch.randint(-8, 9, (CC,), generator=g).float() / 64).to(DEV)
    W1 = (torch.randn(Kf, HD, generator=g) * 0.03).to(DEV)
    b1 = (torch.randn(HD, generator=g) * 0.1).to(DEV)
    W2 = (torch.randn(HD, NC, generator=g) * 0.3).to(DEV)
    b2 = (torch.randn(NC, generator=g) * 0.1).to(DEV)
    hpre = torch.zeros(4, B, HD, device=DEV)
    hzero = torch.full((4, B, HD), 7.0, device=DEV)
    Pt = torch.zeros(Kf, Bp, device=DEV)
    amax = torch.zeros(Pn, CC // 8, Bp, dtype=torch.int64, device=DEV)
    Kk.cgen_fwd(x, w, b, W1, hpre, Pt, amax, B=B)
    d = torch.float64
    wr, br = w.double().clone().requires_grad_(), b.double().clone().requires_grad_()
    pooled = _ref_convpool(x.double(), wr, br).reshape(B, Kf)
    pre = pooled.detach() @ W1.double()
    torch.cuda.synchronize()
    assert torch.equal(Pt[:, :B].double().T, pooled.detach())
    assert _rel(hpre.sum(0), pre) < TOL, _rel(hpre.sum(0), pre)
    amax_b = amax.view(torch.uint8).view(Pn, CC // 8, Bp, 8).permute(2, 0, 1, 3).reshape(Bp, Kf)[:B]
    assert torch.equal(amax_b != 255, pooled.detach() > 0)

    scale = 1.0 / 256
    dW1 = torch.full((Kf, HD), 9.0, device=DEV)
    dw, db = torch.zeros(3, 3, 1, CC, device=DEV), torch.zeros(CC, device=DEV)
    dW2, db2, db1 = torch.zeros(HD, NC, device=DEV), torch.zeros(NC, device=DEV), torch.zeros(HD, device=DEV)
    met = torch.zeros(4, device=DEV)
    it = torch.zeros(1, dtype=torch.int64, device=DEV)
    hkeep = hpre.clone()
    Kk.cgen_bwd(x, amax, hpre, hzero, b1, W2, b2, lab, scale=scale, pre_relu=relu, metrics=met, W1=W1, Pt=Pt,
                dW1=dW1, dwc=dw, dbc=db, dW2=dW2, db2=db2, db1=db1, B=B, iterations=it)
    h = hkeep.sum(0).to(d) + b1.to(d)
    if relu:
        h = h.clamp_min(0)
    logits = h @ W2.to(d) + b2.to(d)
    pr = torch.softmax(logits, 1)
    onehot = F.one_hot(lab.long(), NC).to(d)
    dl = (pr - onehot) * scale
    dH = dl @ W2.to(d).T
    if relu:
        dH = dH * (h > 0)
    (pooled * (dH @ W1.double().T)).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(hpre, hkeep) and torch.all(hzero == 0) and int(it) == 1
    for name, got, ref in [("dW1", dW1, pooled.detach().T @ dH), ("dconv_w", dw, wr.grad), ("dconv_b", db, br.grad),
                           ("dW2", dW2, h.T @ dl), ("db2", db2, dl.sum(0)), ("db1", db1, dH.sum(0))]:
        assert _rel(got, ref) < TOL, (name, _rel(got, ref))
    loss = -(torch.log(pr) * onehot).sum()
    assert abs(met[0].item() - loss.item()) < 1e-5 * abs(loss.item())
    assert met[1].item() == (logits.argmax(1) == lab.long()).sum().item() and met[2].item() == B
    # conv gradients into 5 replicas (workgroup x -> replica x % 5): the replicas sum to the same gradient
    gc = torch.zeros(5, 10 * CC + 4, device=DEV)
    Kk.cgen_bwd(x, amax, hpre, hzero, b1, W2, b2, lab, scale=scale, pre_relu=relu, metrics=None, W1=W1, Pt=Pt,
                dW1=dW1, dwc=gc[0, :9 * CC].view(3, 3, 1, CC), dbc=gc[0, 9 * CC:10 * CC], B=B, crep=5,
                crep_stride=10 * CC + 4)
    torch.cuda.synchronize()
    tot = gc.sum(0)
    assert torch.all(gc[:, 10 * CC:] == 0) and int((gc.abs().sum(1) > 0).sum()) == 5
    assert _rel(tot[:9 * CC], dw.reshape(-1)) < 1e-6 and _rel(tot[9 * CC:10 * CC], db) < 1e-6


def test_cgen_family_matches_the_python_rule():
    """The kernels' instantiation rule (the backward's LDS at 8 waves) agrees with train/program.gen_fits."""
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    from tensorflow_distributed_example_amd.train import program as PG
    for f in (8, 16, 24, 32, 48, 64, 96):
        for u in range(16, 320, 16):
            assert Kk.cgen_supported(f, u) == PG.gen_fits(f, u), (f, u)


def _model(tde, filters, units, opt, spe):
    m = tde.zoo.mnist_cnn(filters=filters, units=units)
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=opt,
              metrics=["accuracy"], steps_per_execution=spe)
    m.build()
    st = m._store
    for n in (f"{m.layers[0].name}/kernel", f"{m.layers[0].name}/bias"):
        st.view(n).copy_(torch.round(st.view(n) * 64) / 64)
    return m


def _grads64(m, W, x, y, B):
    W = {n: w.detach().clone().requires_grad_(True) for n, w in W.items()}
    c, d1, d2 = m.layers[0].name, m.layers[3].name, m.layers[4].name
    P = _ref_convpool(x.double(), W[f"{c}/kernel"], W[f"{c}/bias"]).reshape(B, -1)
    h = F.relu(P @ W[f"{d1}/kernel"] + W[f"{d1}/bias"])
    logits = h @ W[f"{d2}/kernel"] + W[f"{d2}/bias"]
    (F.cross_entropy(logits, y.long(), reduction="sum") / B).backward()
    return {n: w.grad for n, w in W.items()}


@pytest.mark.parametrize("filters,units,mode,kind", [(64, 128, "local", "sgd"), (16, 32, "local", "sgd"),
                                                     (64, 128, "plain", "sgd"), (32, 96, "local", "momentum"),
                                                     (48, 64, "local", "adam"), (16, 128, "plain", "adam"),
                                                     (32, 256, "local", "sgd"), (48, 192, "local", "momentum")])
def test_generic_plan_graph_trajectory_matches_float64(filters, units, mode, kind, monkeypatch):
    """A Conv2D(filters)/Dense(units) model runs the generic fused plan in hipGraph executions of 4 steps —
    step mode "local" (the default with one replica: the Dense rows updated by the backward workgroups that own
    them, the head by the head workgroup, the conv update deferred into the next forward / backward and flushed
    at the end of each execution) or "plain" (TDE_FUSED_STEP=0: gradients, then the multi-tensor optimizer);
    after each execution the weights match the float64 trajectory of the same optimizer (Keras forms) at fp32
    accuracy, the step counter advanced once per step and nothing is left pending."""
    import tensorflow_distributed_example_amd as tde
    if mode == "plain":
        monkeypatch.setenv("TDE_FUSED_STEP", "0")
    O = tde.optimizers
    lr = {"sgd": 0.05, "momentum": 0.02, "adam": 2e-3}[kind]
    opt = {"sgd": lambda: O.SGD(lr), "momentum": lambda: O.SGD(lr, momentum=0.9), "adam": lambda: O.Adam(lr)}[kind]()
    m = _model(tde, filters, units, opt, 4)
    st = m._store
    names = st.names(trainable=True)
    w64 = {n: st.view(n).detach().double().clone() for n in names}
    slots = {n: [torch.zeros_like(w64[n]), torch.zeros_like(w64[n])] for n in names}
    prog = m._program("train", 64)
    plan = prog.plans[0]
    assert prog.use_graph and plan.kind == "fused_convnet_generic" and plan.step_mode == mode
    t = 0
    for e in range(3):
        data = [_qdata(64, 300 + 4 * e + s) for s in range(4)]
        prog.stage([(torch.stack([d[0] for d in data]), torch.stack([d[1] for d in data]))])
        prog.run()
        prog.sync()
        for x, y in data:
            g = _grads64(m, w64, x, y, 64)
            t += 1
            for n in names:
                if kind == "sgd":
                    w64[n] = w64[n] - lr * g[n]
                elif kind == "momentum":
                    slots[n][0] = 0.9 * slots[n][0] - lr * g[n]
                    w64[n] = w64[n] + slots[n][0]
                else:
                    b1, b2, eps = 0.9, 0.999, 1e-7
                    slots[n][0] = b1 * slots[n][0] + (1 - b1) * g[n]
                    slots[n][1] = b2 * slots[n][1] + (1 - b2) * g[n] ** 2
                    lr_t = lr * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)
                    w64[n] = w64[n] - lr_t * slots[n][0] / (slots[n][1].sqrt() + eps)
        for n in names:
            # after the first update the conv weights are no longer quantized: the f32 conv sums differ from
            # float64 in the last bit, and a pool-argmax near-tie decided the other way moves one image's
            # pooled gradient (the kernel tests pin each step at 1e-5 with exact conv sums).  The zero-
            # initialised biases ARE their accumulated update, so one such decision shows ~1e-4 there
            # (Adam's normalised steps make every bias entry a full-size step: 1e-3).
            # The conv kernel collects every image's pooled gradients: such decisions show there as a few 1e-5
            # (a deferred or lost update would be ~1e-3).
            bias, conv = n.endswith("/bias"), n == f"{m.layers[0].name}/kernel"
            tol = (1e-3 if kind == "adam" else 5e-4) if bias else (5e-5 if conv or kind == "adam" else 1e-5)
            assert _rel(st.view(n), w64[n]) < tol, (e, n, _rel(st.view(n), w64[n]))
        assert int(plan.iterations) == 4 * (e + 1)
        if mode == "local":   # after each execution: nothing pending, nothing left in the bucket or the replicas
            iv = plan.step_invariants()
            assert plan.crep > 1 and iv["pending"] == [0, 0] and iv["gconv_abs_max"] == 0.0, iv
            assert float(st.g.abs().max()) == 0.0


def test_generic_plan_fit_evaluate_predict():
    """Keras surface on the generic plan: fit() learns a separable synthetic task, evaluate() and predict()
    agree with the torch reference executor at the same weights."""
    import tensorflow_distributed_example_amd as tde
    rng = np.random.default_rng(4)
    y = rng.integers(0, 10, 64 * 16)
    x = rng.random((64 * 16, 28, 28, 1), dtype=np.float32) * 0.2
    for i, c in enumerate(y):   # class c lights up row band c
        x[i, 2 + 2 * c: 4 + 2 * c, :, 0] += 0.8
    tde.backend.set_random_seed(11)
    m = tde.zoo.mnist_cnn_wide()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1),
              metrics=["accuracy"], steps_per_execution=4)
    h = m.fit(x, y, batch_size=64, epochs=3, shuffle=False, verbose=0)
    assert m._program("train", 64).plan_kind == "fused_convnet_generic"
    assert h.history["accuracy"][-1] > 0.9, h.history
    loss, acc = m.evaluate(x, y, batch_size=64, verbose=0)
    probs = m.predict(x[:128], batch_size=64, verbose=0)
    w = m.get_weights()
    tde.backend.clear_session()
    import os
    os.environ["TDE_EXECUTOR"] = "reference"
    try:
        r = tde.zoo.mnist_cnn_wide()
        r.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1),
                  metrics=["accuracy"])
        r.set_weights(w)
        rl, ra = r.evaluate(x, y, batch_size=64, verbose=0)
        rp = r.predict(x[:128], batch_size=64, verbose=0)
    finally:
        del os.environ["TDE_EXECUTOR"]
    assert abs(loss - rl) < 1e-5 * max(1.0, abs(rl)) and acc == ra
    np.testing.assert_allclose(probs, rp, rtol=1e-4, atol=1e-6)
