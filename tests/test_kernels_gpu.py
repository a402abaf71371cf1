"""T0: every HIP kernel vs a plain PyTorch fp32 reference of the same op, at the
reference's shapes plus odd shapes for the tail paths."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,mode,splits", [
    (64, 64, 5408, "atomic", 0),      # Dense(64) forward, split-K
    (5408, 64, 64, "store", 1),       # dW of Dense(64)
    (70, 50, 200, "store", 1),        # tails in M, N, K
    (128, 200, 1176, "atomic", 4),    # Model B Dense(200)
    (33, 10, 64, "accum", 1),
])
def test_gemm_nt(M, N, K, mode, splits):
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(0)
    A = _bf(torch.randn(M, K, generator=g)).to(DEV)
    Bt = _bf(torch.randn(N, K, generator=g)).to(DEV)
    C0 = torch.randn(M, N, generator=g).to(DEV) if mode == "accum" else torch.zeros(M, N, device=DEV)
    C = C0.clone()
    Kk.gemm_nt(A, Bt, C, alpha=0.5, mode=mode, splits=splits)
    ref = 0.5 * (A.double() @ Bt.double().T) + (C0.double() if mode == "accum" else 0)
    torch.cuda.synchronize()
    err = (C.double() - ref).abs().max().item()
    assert err <= 1e-3 * (K ** 0.5) + 1e-4, err


def test_gemm_epilogue_bias_relu_bf16out():
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(1)
    M, N, K = 96, 80, 160
    A = _bf(torch.randn(M, K, generator=g)).to(DEV)
    Bt = _bf(torch.randn(N, K, generator=g)).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    C = torch.zeros(M, N, device=DEV)
    Cb = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    Kk.gemm_nt(A, Bt, C, mode="store", bias=bias, relu=True, Cbf=Cb)
    ref = F.relu(A.float() @ Bt.float().T + bias)
    torch.cuda.synchronize()
    assert torch.allclose(C, ref, atol=2e-3, rtol=1e-3)
    assert torch.allclose(Cb.float(), ref, atol=5e-2, rtol=1e-2)


def _ref_convpool(x, w, b):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b)
    y = F.max_pool2d(F.relu(y), 2)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B", [64, 37, 130])
def test_conv3x3c1_relu_pool_fwd(B):
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.rand(B, 28, 28, 1, generator=g).to(DEV)
    w = (torch.randn(3, 3, 1, 32, generator=g) * 0.4).to(DEV)
    b = (torch.randn(32, generator=g) * 0.1).to(DEV)
    K = 13 * 13 * 32
    Bp = (B + 7) // 8 * 8
    P = torch.zeros(B, K, dtype=torch.bfloat16, device=DEV)
    Pt = torch.full((K, Bp), 7.0, dtype=torch.bfloat16, device=DEV)
    amax = torch.zeros(B, K, dtype=torch.uint8, device=DEV)
    z = torch.ones(100, device=DEV)
    Kk.conv3x3c1_relu_pool_fwd(x, w, b, P, Pt, amax, zbuf=z)
    ref = _ref_convpool(x, w, b).reshape(B, K)
    torch.cuda.synchronize()
    assert torch.allclose(P.float(), ref, atol=1e-2, rtol=8e-3)
    assert torch.equal(Pt[:, :B], P.T)
    assert torch.all(Pt[:, B:] == 0)
    assert torch.all(z == 0)
    active = amax != 255
    assert torch.equal(active, ref > 0)


@pytest.mark.parametrize("B", [64, 50])
def test_conv3x3c1_relu_pool_bwd(B):
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(3)
    Hd, C = 64, 32
    K = 13 * 13 * C
    x = torch.rand(B, 28, 28, 1, generator=g).to(DEV)
    w = (torch.randn(3, 3, 1, C, generator=g) * 0.4).to(DEV)
    b = (torch.randn(C, generator=g) * 0.1).to(DEV)
    G = _bf(torch.randn(B, Hd, generator=g) * 0.1).to(DEV)
    W1 = _bf(torch.randn(K, Hd, generator=g) * 0.05).to(DEV)
    P = torch.zeros(B, K, dtype=torch.bfloat16, device=DEV)
    amax = torch.zeros(B, K, dtype=torch.uint8, device=DEV)
    Kk.conv3x3c1_relu_pool_fwd(x, w, b, P, None, amax)
    dw = torch.zeros(3, 3, 1, C, device=DEV)
    db = torch.zeros(C, device=DEV)
    Kk.conv3x3c1_relu_pool_bwd(x, amax, G, W1, dw, db)
    # reference via autograd
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    out = _ref_convpool(x, wr, br).reshape(B, K)
    dP = G.float() @ W1.float().T
    (out * dP).sum().backward()
    torch.cuda.synchronize()
    assert torch.allclose(dw, wr.grad, atol=2e-3, rtol=2e-3), (dw - wr.grad).abs().max()
    assert torch.allclose(db, br.grad, atol=2e-3, rtol=2e-3), (db - br.grad).abs().max()


@pytest.mark.parametrize("B", [64, 37, 130])
def test_convnet_fwd_fused(B):
    """conv+pool+Dense-matmul fused forward vs torch fp32 (conv -> relu -> pool -> flatten -> bf16 @ W1)."""
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(12)
    C, Hd = 32, 64
    Kf = 13 * 13 * C
    x = torch.rand(B, 28, 28, 1, generator=g).to(DEV)
    w = (torch.randn(3, 3, 1, C, generator=g) * 0.4).to(DEV)
    b = (torch.randn(C, generator=g) * 0.1).to(DEV)
    W1 = (torch.randn(Kf, Hd, generator=g) * 0.02).to(DEV)
    W1c = W1.T.contiguous().to(torch.bfloat16)
    Bp = (B + 7) // 8 * 8
    hpre = torch.zeros(B, Hd, device=DEV)
    Pt = torch.full((Kf, Bp), 5.0, dtype=torch.bfloat16, device=DEV)
    amax = torch.zeros(Kf // 32, 4, Bp, dtype=torch.int64, device=DEV)
    Kk.convnet_fwd(x, w, b, W1c, hpre, Pt, amax)
    amax_b = amax.view(torch.uint8).view(Kf // 32, 4, Bp, 8).permute(2, 0, 1, 3).reshape(Bp, Kf)[:B]
    pooled = _ref_convpool(x, w, b).reshape(B, Kf)
    ref = pooled.to(torch.bfloat16).float() @ W1c.float().T
    torch.cuda.synchronize()
    assert torch.allclose(hpre, ref, atol=2e-2, rtol=2e-2), (hpre - ref).abs().max()
    assert torch.allclose(Pt[:, :B].float().T, pooled, atol=1e-2, rtol=8e-3)
    assert torch.all(Pt[:, B:] == 0)
    assert torch.equal(amax_b != 255, pooled > 0)
    # the same forward reading the row-major [K, 64] shadow (the training default)
    hpre2 = torch.zeros(B, Hd, device=DEV)
    Kk.convnet_fwd(x, w, b, W1c.T.contiguous(), hpre2, Pt, amax)
    torch.cuda.synchronize()
    assert torch.allclose(hpre2, ref, atol=2e-2, rtol=2e-2), (hpre2 - ref).abs().max()


@pytest.mark.parametrize("B,relu", [(64, True), (50, True), (128, False)])
def test_convnet_bwd_fused(B, relu):
    """Trunk backward with the head fused in (csrc/kernels/convnet.hip) vs float64 torch: the head's
    dlogits / Dense(64) input gradient G (rounded to bf16 where the kernel rounds it), dW1 = P^T G,
    conv weight / bias gradients through the pool argmax and ReLU, the head gradients dW2 / db2 / db1,
    the loss / accuracy metrics, and the other parity buffer zeroed."""
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(13)
    C, Hd, NC = 32, 64, 10
    Kf = 13 * 13 * C
    Bp = (B + 7) // 8 * 8
    x = torch.rand(B, 28, 28, 1, generator=g).to(DEV)
    w = (torch.randn(3, 3, 1, C, generator=g) * 0.4).to(DEV)
    b = (torch.randn(C, generator=g) * 0.1).to(DEV)
    W1 = (torch.randn(Kf, Hd, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    hpre = (torch.randn(B, Hd, generator=g) * 0.5).to(DEV)
    hzero = torch.full((B, Hd), 7.0, device=DEV)
    b1 = (torch.randn(Hd, generator=g) * 0.1).to(DEV)
    W2 = (torch.randn(Hd, NC, generator=g) * 0.3).to(DEV)
    b2 = (torch.randn(NC, generator=g) * 0.1).to(DEV)
    lab = torch.randint(0, NC, (B,), generator=g).to(DEV).int()
    scale = 1.0 / 256
    Pt = torch.zeros(Kf, Bp, dtype=torch.bfloat16, device=DEV)
    amax = torch.zeros(Kf // 32, 4, Bp, dtype=torch.int64, device=DEV)
    Kk.convnet_fwd(x, w, b, W1, torch.zeros(B, Hd, device=DEV), Pt, amax)
    dW1 = torch.full((Kf, Hd), 9.0, device=DEV)
    dw = torch.zeros(3, 3, 1, C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dW2, db2, db1 = torch.ones(Hd, NC, device=DEV), torch.ones(NC, device=DEV), torch.ones(Hd, device=DEV)
    met = torch.zeros(4, device=DEV)
    hkeep = hpre.clone()
    Kk.convnet_bwd(x, amax, hpre, hzero, b1, W2, b2, lab, scale=scale, pre_relu=relu, metrics=met, W1row=W1, Pt=Pt,
                   dW1=dW1, dwc=dw, dbc=db, dW2=dW2, db2=db2, db1=db1)
    d = torch.float64
    h = hpre.to(d) + b1.to(d)
    if relu:
        h = h.clamp_min(0)
    logits = h @ W2.to(d) + b2.to(d)
    pr = torch.softmax(logits, 1)
    onehot = torch.nn.functional.one_hot(lab.long(), NC).to(d)
    dl = (pr - onehot) * scale
    dH = dl @ W2.to(d).T
    if relu:
        dH = dH * (h > 0)
    G = dH.to(torch.bfloat16)
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    out = _ref_convpool(x, wr, br).reshape(B, Kf)
    (out * (G.float() @ W1.float().T)).sum().backward()
    dW1_ref = Pt[:, :B].double() @ G.double()
    torch.cuda.synchronize()
    assert torch.equal(hpre, hkeep) and torch.all(hzero == 0)
    assert torch.allclose(dW1.double(), dW1_ref, atol=1e-4, rtol=1e-2), (dW1.double() - dW1_ref).abs().max()
    tol = 1e-2 * wr.grad.abs().max().item() + 1e-5
    assert (dw - wr.grad).abs().max().item() < tol, (dw - wr.grad).abs().max()
    assert (db - br.grad).abs().max().item() < 1e-2 * br.grad.abs().max().item() + 1e-5
    assert torch.allclose(dW2.double() - 1, h.T @ dl, atol=1e-6, rtol=1e-4)
    assert torch.allclose(db2.double() - 1, dl.sum(0), atol=1e-6, rtol=1e-4)
    assert torch.allclose(db1.double() - 1, dH.sum(0), atol=1e-6, rtol=1e-4)
    loss = -(torch.log(pr) * onehot).sum()
    correct = (logits.argmax(1) == lab.long()).sum()
    assert abs(met[0].item() - loss.item()) < 1e-3 * abs(loss.item()) and met[1].item() == correct.item()
    assert met[2].item() == B


@pytest.mark.parametrize("B,H,C,relu,softmax_probs", [(64, 64, 10, True, False), (45, 200, 10, False, True)])
def test_head_xent(B, H, C, relu, softmax_probs):
    from tensorflow_distributed_example_amd.ops import kernels as Kk
    g = torch.Generator(device="cpu").manual_seed(4)
    hpre = torch.randn(B, H, generator=g).to(DEV)
    b1 = (torch.randn(H, generator=g) * 0.1).to(DEV)
    W2 = (torch.randn(H, C, generator=g) * 0.2).to(DEV)
    b2 = (torch.randn(C, generator=g) * 0.1).to(DEV)
    lab = torch.randint(0, C, (B,), generator=g).to(DEV)
    scale = 1.0 / 128
    Bp = (B + 7) // 8 * 8
    dW2 = torch.zeros(H, C, device=DEV)
    db2 = torch.zeros(C, device=DEV)
    db1 = torch.zeros(H, device=DEV)
    G = torch.zeros(B, H, dtype=torch.bfloat16, device=DEV)
    Gt = torch.full((H, Bp), 3.0, dtype=torch.bfloat16, device=DEV)
    met = torch.zeros(4, device=DEV)
    probs = torch.zeros(B, C, device=DEV)
    Kk.head_xent(hpre, W2, b2, lab.int(), B=B, scale=scale, pre_bias=b1, pre_relu=relu, dW2=dW2, db2=db2,
                 dpre_bias=db1, G=G, Gt=Gt, metrics=met, probs=probs, probs_are_logits=False)
    hp = hpre.clone().requires_grad_()
    b1r, W2r, b2r = b1.clone().requires_grad_(), W2.clone().requires_grad_(), b2.clone().requires_grad_()
    h = hp + b1r
    if relu:
        h = F.relu(h)
    logits = h @ W2r + b2r
    ls = F.cross_entropy(logits, lab, reduction="none")
    (ls.sum() * scale).backward()
    torch.cuda.synchronize()
    assert torch.allclose(dW2, W2r.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(db2, b2r.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(db1, b1r.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(G.float(), hp.grad, atol=1e-4, rtol=1e-2)
    assert torch.equal(Gt[:, :B], G.T) and torch.all(Gt[:, B:] == 0)
    assert abs(met[0].item() - ls.sum().item()) < 1e-3 * B
    assert met[1].item() == (logits.argmax(1) == lab).sum().item()
    assert met[2].item() == B
    assert torch.allclose(probs, torch.softmax(logits, 1), atol=1e-5)


@pytest.mark.parametrize("kind", ["sgd", "momentum", "nesterov", "adam"])
def test_optimizer_kernel_matches_reference(kind):
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train.program import OptimizerKernel
    m = tde.zoo.mnist_cnn()
    m.build()
    st = m._store
    st2 = st.clone_to(DEV)
    st_ref = st.clone_to(DEV)
    opt = {"sgd": tde.optimizers.SGD(0.1), "momentum": tde.optimizers.SGD(0.1, momentum=0.9),
           "nesterov": tde.optimizers.SGD(0.1, momentum=0.9, nesterov=True), "adam": tde.optimizers.Adam(0.01)}[kind]
    for s in opt.slot_names():
        st2.slot(s)
        st_ref.slot(s)
    it = torch.zeros(1, dtype=torch.int64, device=DEV)
    ok = OptimizerKernel(st2, opt, {"dense/kernel": ("row", "col")}, it)
    g = torch.Generator(device="cpu").manual_seed(5)
    for step in range(3):
        grad = torch.randn(st2.g.shape, generator=g).to(DEV)
        st2.g.copy_(grad)
        it += 1  # the step's loss kernel advances the counter before the optimizer runs
        ok.apply()
        opt.apply_reference(st_ref.w, grad, {s: st_ref.slot(s) for s in opt.slot_names()}, step)
    torch.cuda.synchronize()
    assert it.item() == 3
    for name in st2.names(trainable=True):
        assert torch.all(st2.grad(name) == 0), name
        assert torch.allclose(st2.view(name), st_ref.view(name), atol=1e-5, rtol=1e-5), name
    W = st2.view("dense/kernel")
    assert torch.equal(ok.shadow_views[("dense/kernel", "row")], W.to(torch.bfloat16))
    assert torch.equal(ok.shadow_views[("dense/kernel", "col")], W.T.to(torch.bfloat16))


@pytest.mark.parametrize("fpw", [1, 4])
def test_convnet_fwd_geometries(fpw):
    """The non-default forward geometries (TDE_CONVNET_FPW = 1 / 4 pooled positions per workgroup; the
    library reads the knob once per process) against the same fp32 reference, in a child process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import test_kernels_gpu as t\n"
            "for B in (64, 37, 130): t.test_convnet_fwd_fused(B)\n"
            "t.test_convnet_bwd_fused(64, True)\nprint('ok')\n" % here)
    env = dict(os.environ, TDE_CONVNET_FPW=str(fpw))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=os.path.dirname(here), capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("sizes", [[64 * 784 * 20, 64 * 20], [3, 17, 0, 4096], [1]])
def test_copy_pairs_stages_every_pair(sizes):
    """tde_copy_pairs (the per-execution input staging, csrc/kernels/gather.hip): up to 4 (src, dst) pairs in
    one launch, 16-byte vectors where sizes and pointers allow, 4-byte words for the rest (odd element counts,
    an empty pair, a misaligned destination offset); bytes past each pair untouched."""
    import ctypes as C
    from tensorflow_distributed_example_amd import _native as N
    g = torch.Generator(device="cpu").manual_seed(1)
    srcs = [torch.randn(n, generator=g).to(DEV) for n in sizes]
    # destinations: one element of offset for odd-numbered pairs (4-byte, not 16-byte, aligned), a guard tail
    bufs = [torch.full((n + 8,), -7.0, device=DEV) for n in sizes]
    dsts = [b[(i % 2): (i % 2) + n] for i, (b, n) in enumerate(zip(bufs, sizes))]
    k = len(sizes)
    rc = N.hip().tde_copy_pairs(k, (C.c_void_p * k)(*[s.data_ptr() for s in srcs]),
                                (C.c_void_p * k)(*[d.data_ptr() for d in dsts]),
                                (C.c_longlong * k)(*[4 * n for n in sizes]), N.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    for i, (s, d, b, n) in enumerate(zip(srcs, dsts, bufs, sizes)):
        assert torch.equal(s, d), i
        off = i % 2
        assert bool((b[:off] == -7.0).all()) and bool((b[off + n:] == -7.0).all()), i
