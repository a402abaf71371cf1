#!/usr/bin/env python
"""Diagnostic: the FIRST fused BN-CNN training step of a fresh process vs a float64 CPU autograd of the
same step; prints the relative error of every intermediate the plan keeps (raw conv outputs z, the
dense pre-activation h, the BN-output gradients g, dL/dh) and of the gradients, in chain order."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402

m = tde.zoo.mnist_bn_cnn()
for lyr in m.layers:
    if isinstance(lyr, tde.keras.layers.Dropout):
        lyr.rate = 0.0
m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
m.build()
gen = torch.Generator(device="cpu").manual_seed(int(os.environ.get("SEED", "3")))
st = m._store
for n in st.names():
    if n.endswith("/beta"):
        v = st.view(n)
        v.copy_((torch.rand(v.shape, generator=gen) - 0.5).to(v.device) * 0.2)
if os.environ.get("MIMIC"):
    # the refcheck sequence: a second model with the same weights and a torch ReferencePlan
    m2 = tde.zoo.mnist_bn_cnn()
    m2.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01))
    m2.build()
    m2.set_weights(m.get_weights())
    pr = PG.ReferencePlan(m2, m2._store, "cuda", 128, 128, m2.optimizer, m2.loss)
plan = PG.make_plan(m, st, "cuda", 128, 128, m.optimizer, m.loss)
x = torch.rand(128, 784, generator=gen).cuda()
y = torch.randint(0, 10, (128,), generator=gen).int().cuda()
plan.train_step(x, y)
torch.cuda.synchronize()

W = {n: st.view(n).detach().double().cpu().clone().requires_grad_(st.segments[n].trainable) for n in st.order}
a = x.double().cpu().view(128, 28, 28, 1)
zs, pres = [], []
for blk in plan.blocks:
    conv, bn = blk["conv"], blk["bn"]
    (pt, pb), (pl, pr) = conv.pads(conv.input_shape)
    z = F.conv2d(F.pad(a.permute(0, 3, 1, 2), (pl, pr, pt, pb)), W[f"{conv.name}/kernel"].permute(3, 2, 0, 1),
                 stride=conv.strides).permute(0, 2, 3, 1)
    z.retain_grad()
    pre = (z - z.mean((0, 1, 2))) / torch.sqrt(z.var((0, 1, 2), unbiased=False) + bn.epsilon) + W[f"{bn.name}/beta"]
    pre.retain_grad()
    zs.append(z)
    pres.append(pre)
    a = torch.relu(pre)
h = a.reshape(128, -1) @ W[f"{plan.dense.name}/kernel"]
h.retain_grad()
bnl = plan.bnd["layer"]
hpre = (h - h.mean(0)) / torch.sqrt(h.var(0, unbiased=False) + bnl.epsilon) + W[f"{bnl.name}/beta"]
hpre.retain_grad()
hp = torch.relu(hpre)
logits = hp @ W[f"{plan.head.name}/kernel"] + W[f"{plan.head.name}/bias"]
(F.cross_entropy(logits, y.long().cpu(), reduction="sum") * plan.scale).backward()


def rel(t32, t64):
    t32 = t32.detach().double().cpu().reshape(t64.shape)
    return round(float((t32 - t64).norm() / (t64.norm() + 1e-30)), 9)


out = {}
for i, blk in enumerate(plan.blocks):
    gz = blk["geo"]
    n = 128 * gz.Ho * gz.Wo * gz.Co
    out[f"z{i}"] = rel(blk["z"][:n], zs[i].detach())
D, Dp = plan.D, plan.Dp
out["h"] = rel(plan.h[: 128 * Dp].view(128, Dp)[:, :D], h.detach())
out["gh"] = rel(plan.gh[: 128 * Dp].view(128, Dp)[:, :D], hpre.grad)
for i in reversed(range(len(plan.blocks))):
    gz = plan.blocks[i]["geo"]
    n = 128 * gz.Ho * gz.Wo * gz.Co
    out[f"g{i}"] = rel(plan.blocks[i]["g"][:n], pres[i].grad)
for n in st.names(trainable=True):
    out["grad:" + n] = rel(st.grad(n), W[n].grad)
for i, blk in enumerate(plan.blocks):
    Co = blk["geo"].Co
    gsum = pres[i].grad.sum((0, 1, 2))
    z = zs[i].detach()
    xh = (z - z.mean((0, 1, 2))) / torch.sqrt(z.var((0, 1, 2), unbiased=False) + blk["bn"].epsilon)
    gx = (pres[i].grad * xh).sum((0, 1, 2))
    acc = blk["accb"].view(64, 2, Co).sum(0).cpu()
    out[f"accb{i}"] = max(rel(acc[0], gsum), rel(acc[1], gx))
for i in reversed(range(len(plan.blocks))):
    if out[f"g{i}"] < 1e-4:
        continue
    gz = plan.blocks[i]["geo"]
    n = 128 * gz.Ho * gz.Wo * gz.Co
    e = (plan.blocks[i]["g"][:n].double().cpu().view(pres[i].grad.shape) - pres[i].grad).abs()
    ref = pres[i].grad.abs().max().item()
    per_img = e.amax((1, 2, 3))
    bad_imgs = (per_img > 1e-4 * ref).nonzero().flatten().tolist()
    info = {"block": i, "bad_images": bad_imgs[:20], "n_bad_images": len(bad_imgs)}
    if bad_imgs:
        b0 = bad_imgs[0]
        eb = e[b0]
        badpix = (eb.amax(-1) > 1e-4 * ref).nonzero().tolist()
        info["bad_pixels_img0"] = badpix[:40]
        info["n_bad_pixels_img0"] = len(badpix)
        info["bad_channels_img0"] = (eb.amax((0, 1)) > 1e-4 * ref).nonzero().flatten().tolist()
    out[f"diag{i}"] = info
print(json.dumps(out))
