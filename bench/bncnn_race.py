#!/usr/bin/env python
"""Diagnostic: repeat the same fused BN-CNN training step (same weights, inputs, zeroed statistics) many
times in one process and report the first intermediate buffer whose contents differ between
repetitions beyond floating-point reordering noise (race hunting)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402

reps = int(os.environ.get("REPS", "40"))
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
st = m._store
plan = PG.make_plan(m, st, "cuda", 128, 128, m.optimizer, m.loss)
x = torch.rand(128, 784, generator=g).cuda()
y = torch.randint(0, 10, (128,), generator=g).int().cuda()
w0 = st.w.clone()
moving = {n: st.view(n).clone() for n in st.order if "moving" in n}


def bufs():
    out = {}
    for i, b in enumerate(plan.blocks):
        for k in ("z", "g", "saved", "dwpart"):
            out[f"b{i}.{k}"] = b[k]
        out[f"b{i}.acc"] = b["acc"].view(-1, b["acc"].numel() // 64 if b["acc"].numel() % 64 == 0 else 1).sum(0)
        out[f"b{i}.accb"] = b["accb"].view(64, -1).sum(0)
    for k in ("h", "hpart", "logits", "dh", "dwd_part"):
        out[k] = getattr(plan, k)
    out["grad"] = st.g
    return {k: v.detach().double().clone() for k, v in out.items()}


def one():
    st.w.copy_(w0)
    st.g.zero_()
    for n, v in moving.items():
        st.view(n).copy_(v)
    for b in plan.blocks:
        b["acc"].zero_()
        b["accb"].zero_()
    plan.train_step(x, y)
    torch.cuda.synchronize()
    return bufs()


ref = one()
order = list(ref.keys())
bad = {}
for r in range(reps):
    cur = one()
    for k in order:
        a, b = cur[k], ref[k]
        d = float((a - b).abs().max() / (b.abs().max() + 1e-30))
        if d > 1e-6:
            bad.setdefault(k, []).append((r, d))
print(json.dumps({"reps": reps, "differing": {k: v[:5] for k, v in bad.items()},
                  "n_bad_reps": len({r for v in bad.values() for r, _ in v})}))
