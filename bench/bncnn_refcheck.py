#!/usr/bin/env python
"""Diagnostic: fused BN-CNN plan vs the torch ReferencePlan, driven step by step on the GPU with the
same data and the same initial weights; prints per-step, per-variable gradient differences."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402

steps = int(os.environ.get("STEPS", "3"))
if os.environ.get("EXACT"):
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True


def model():
    m = tde.zoo.mnist_bn_cnn()
    for lyr in m.layers:
        if isinstance(lyr, tde.keras.layers.Dropout):
            lyr.rate = 0.0
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
    m.build()
    g = torch.Generator(device="cpu").manual_seed(3)
    for n in m._store.names():
        if n.endswith("/beta"):
            v = m._store.view(n)
            v.copy_((torch.rand(v.shape, generator=g) - 0.5).to(v.device) * 0.2)
    return m


mf = model()
mr = model()
mr.set_weights(mf.get_weights())
pf = PG.make_plan(mf, mf._store, "cuda", 128, 128, mf.optimizer, mf.loss)
pr = PG.ReferencePlan(mr, mr._store, "cuda", 128, 128, mr.optimizer, mr.loss)
print(json.dumps({"fused": pf.kind, "ref": pr.kind}))
rng = np.random.default_rng(int(os.environ.get("SEED", "0")))
for step in range(steps):
    x = torch.as_tensor(rng.random((128, 784), dtype=np.float32), device="cuda")
    y = torch.as_tensor(rng.integers(0, 10, 128), device="cuda").int()
    wdiff = {n: float((mf._store.view(n) - mr._store.view(m)).abs().max())
             for n, m in zip(mf._store.order, mr._store.order)}
    pf.train_step(x, y)
    pr.train_step(x, y)
    torch.cuda.synchronize()
    g_first = mr._store.g.clone()
    mr._store.g.zero_()
    mv = {n: mr._store.view(n).clone() for n in mr._store.order if "moving" in n}
    pr.train_step(x, y)   # the reference again on the same step: its own run-to-run spread
    torch.cuda.synchronize()
    for n, v in mv.items():
        mr._store.view(n).copy_(v)
    ref_rr = float((mr._store.g - g_first).norm() / g_first.norm())
    out = {"step": step, "max_w_diff": max(wdiff.values()), "ref_self_diff": ref_rr}
    for n, m in zip(mf._store.names(trainable=True), mr._store.names(trainable=True)):
        a, b = mf._store.grad(n).double(), mr._store.grad(m).double()
        out[n] = round(float((a - b).norm() / (b.norm() + 1e-30)), 9)
    # float64 truth on the CPU (pure autograd, its own ReLU decisions) for the first conv's gradient
    import torch.nn.functional as F
    st0 = mf._store
    W64 = {n: st0.view(n).detach().double().cpu().clone().requires_grad_(st0.segments[n].trainable) for n in st0.order}
    h = x.double().cpu().view(128, 28, 28, 1)
    for blk in pf.blocks:
        conv, bn = blk["conv"], blk["bn"]
        (pt, pb), (pl, pr_) = conv.pads(conv.input_shape)
        z = F.conv2d(F.pad(h.permute(0, 3, 1, 2), (pl, pr_, pt, pb)), W64[f"{conv.name}/kernel"].permute(3, 2, 0, 1),
                     stride=conv.strides).permute(0, 2, 3, 1)
        h = torch.relu((z - z.mean((0, 1, 2))) / torch.sqrt(z.var((0, 1, 2), unbiased=False) + bn.epsilon)
                       + W64[f"{bn.name}/beta"])
    hd = h.reshape(128, -1) @ W64[f"{pf.dense.name}/kernel"]
    bnl = pf.bnd["layer"]
    hd = torch.relu((hd - hd.mean(0)) / torch.sqrt(hd.var(0, unbiased=False) + bnl.epsilon) + W64[f"{bnl.name}/beta"])
    logits = hd @ W64[f"{pf.head.name}/kernel"] + W64[f"{pf.head.name}/bias"]
    (F.cross_entropy(logits, y.long().cpu(), reduction="sum") / 128).backward()
    g64 = W64["conv2d/kernel"].grad
    gf = mf._store.grad("conv2d/kernel").double().cpu()
    gr = g_first[mr._store.segments[mr._store.order[0]].offset:][: g64.numel()].double().cpu().view(g64.shape)
    out["fused_vs_f64"] = round(float((gf - g64).norm() / g64.norm()), 9)
    out["ref_vs_f64"] = round(float((gr - g64).norm() / g64.norm()), 9)
    # ReLU decisions of the fused plan vs float64 truth (per conv BN)
    import torch.nn.functional as F
    st = mf._store
    a = x.double().view(128, 28, 28, 1)
    for li, blk in enumerate(pf.blocks):
        conv, bn = blk["conv"], blk["bn"]
        (pt, pb), (pl, pr_) = conv.pads(conv.input_shape)
        z = F.conv2d(F.pad(a.permute(0, 3, 1, 2), (pl, pr_, pt, pb)),
                     st.view(f"{conv.name}/kernel").double().permute(3, 2, 0, 1), stride=conv.strides).permute(0, 2, 3, 1)
        mean, var = z.mean((0, 1, 2)), z.var((0, 1, 2), unbiased=False)
        pre = (z - mean) / torch.sqrt(var + bn.epsilon) + st.view(f"{bn.name}/beta").double()
        g = blk["geo"]
        z32 = blk["z"][: 128 * g.Ho * g.Wo * g.Co].view(128, g.Ho, g.Wo, g.Co)
        sv = blk["saved"]
        pre32 = (z32 - sv[: g.Co]) * sv[g.Co:] + st.view(f"{bn.name}/beta")
        mis = (pre > 0) != (pre32 > 0)
        out[f"flips{li}"] = int(mis.sum())
        out[f"zdiff{li}"] = float((z32.double() - z).abs().max())
        out[f"meandiff{li}"] = float((sv[: g.Co].double() - mean).abs().max())
        out[f"rsdiff{li}"] = float(((sv[g.Co:].double() - 1 / torch.sqrt(var + bn.epsilon)) / (1 / torch.sqrt(var + bn.epsilon))).abs().max())
        out[f"minpre{li}"] = float(pre.abs().min())
        a = pre.clamp_min(0)
    print(json.dumps(out))
    pf.apply()
    pr.apply()
    pf.iterations += 0   # ReferencePlan.apply advances its own counter; the fused plan's optimizer does
    torch.cuda.synchronize()
