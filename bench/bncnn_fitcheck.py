#!/usr/bin/env python
"""Diagnostic: Model B after N fit() steps on the fused BN-CNN plan vs the torch reference executor,
and vs the same plan driven step by step without hipGraphs.  Prints per-variable relative
differences (normalised by the update size) as JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402

steps = int(os.environ.get("STEPS", "4"))
rng = np.random.default_rng(0)
x = rng.random((128 * steps, 784), dtype=np.float32)
y = rng.integers(0, 10, 128 * steps)


def model():
    m = tde.zoo.mnist_bn_cnn()
    for lyr in m.layers:
        if isinstance(lyr, tde.keras.layers.Dropout):
            lyr.rate = 0.0
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
    m.build()
    if os.environ.get("BETA"):
        import torch
        g = torch.Generator(device="cpu").manual_seed(3)
        for n in m._store.names():
            if n.endswith("/beta"):
                v = m._store.view(n)
                v.copy_((torch.rand(v.shape, generator=g) - 0.5).to(v.device) * 0.2)
    return m


def run(executor, w0, graph=True):
    tde.backend.clear_session()
    if executor:
        os.environ["TDE_EXECUTOR"] = executor
    else:
        os.environ.pop("TDE_EXECUTOR", None)
    if not graph:
        os.environ["TDE_GRAPH"] = "0"
    else:
        os.environ.pop("TDE_GRAPH", None)
    m = model()
    if w0 is not None:
        m.set_weights(w0)
    h = m.fit(x, y, batch_size=128, epochs=1, shuffle=False, verbose=0)
    return m, h.history["loss"][0]


m0 = model()
w0 = m0.get_weights()
mf, lf = run(None, w0)
kind = mf._program("train", 128).plan_kind
mr, lr = run("reference", w0)
mn, ln = run(None, w0, graph=False)
print(json.dumps({"plan": kind, "loss_fused": lf, "loss_ref": lr, "loss_nograph": ln}))
for name, a, b, c, w in zip(mf.variable_names(), mf.get_weights(), mr.get_weights(), mn.get_weights(), w0):
    den = np.linalg.norm(b - w) + np.linalg.norm(b) * 1e-6 + 1e-12
    print(json.dumps({"var": name, "fused_vs_ref": float(np.linalg.norm(a - b) / den),
                      "nograph_vs_ref": float(np.linalg.norm(c - b) / den),
                      "upd": float(np.linalg.norm(b - w)), "w": float(np.linalg.norm(w))}))
