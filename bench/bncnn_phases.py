#!/usr/bin/env python
"""Per-launch phase timeline of the fused BN-CNN step (csrc/kernels/bncnn.hip): every workgroup of one
training step records its wall clock (100 MHz) at the kernel's phase points; prints, per launch, the
dispatch spread (first .. last workgroup start), the median / max duration of each phase, and the
launch's span.  Prints one JSON line per launch."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd import _native as N  # noqa: E402
from tensorflow_distributed_example_amd.train import bncnn as BC  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402

B = int(os.environ.get("B", "128"))
m = tde.zoo.mnist_bn_cnn() if hasattr(tde, "zoo") and hasattr(tde.zoo, "mnist_bn_cnn") else None
if m is None:
    raise SystemExit("tde.zoo.mnist_bn_cnn missing")
m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
m.build()
plan = PG.make_plan(m, m._store, "cuda", B, B, m.optimizer, m.loss)
assert plan.kind == "fused_bncnn", plan.kind
x = torch.rand(B, 784, device="cuda")
y = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
for _ in range(20):
    plan.train_step(x, y)
torch.cuda.synchronize()
n_launch = 32
stride = 8192 * 8
buf = torch.zeros(n_launch * stride, dtype=torch.int64, device="cuda")
lib = N.hip()
lib.tde_bncnn_stamps.restype = None
lib.tde_bncnn_stamps.argtypes = [C.c_void_p, C.c_int]
lib.tde_bncnn_stamps(buf.data_ptr(), n_launch)
plan.train_step(x, y)
lib.tde_bncnn_stamps(None, 0)
torch.cuda.synchronize()
st = buf.view(n_launch, 8192, 8).cpu().numpy()
def summary(s, t0):
    out = {"first_start_us": round((s[:, 0].min() - t0) / 100.0, 2),
           "last_start_us": round((s[:, 0].max() - t0) / 100.0, 2)}
    last = s[:, 0].copy()
    ends = s[:, 0].copy()
    for k in range(1, 8):
        col = s[:, k]
        ok = col > 0
        if not ok.any():
            continue
        d = (col[ok] - last[ok]) / 100.0
        out[f"ph{k}_med_us"] = round(float(np.median(d)), 2)
        out[f"ph{k}_max_us"] = round(float(d.max()), 2)
        last = np.where(ok, col, last)
        ends = np.maximum(ends, np.where(ok, col, 0))
    out["last_end_us"] = round((ends.max() - t0) / 100.0, 2)
    out["wg_med_us"] = round(float(np.median(ends - s[:, 0])) / 100.0, 2)
    return out


fold = plan.head_fold_ok(B)
names = [f"conv_fwd{i}" for i in range(len(plan.blocks))] + ["dense_fwd"] + ([] if fold else ["head"]) + [
    "dense_bwd_head" if fold else "dense_bwd"]
names += [f"conv_bwd{i}" for i in reversed(range(len(plan.blocks)))] + ["reduce"]
t0 = None
for li, name in enumerate(names):
    s = st[li]
    used = s[:, 0] > 0
    if not used.any():
        print(json.dumps({"launch": name, "stamped": False}))
        continue
    s = s[used]
    if t0 is None:
        t0 = s[:, 0].min()
    out = {"launch": name, "wgs": int(used.sum())}
    out.update(summary(s, t0))
    if name.startswith("conv_bwd") and len(s) == 2 * B:
        # rows [0, B): the weight-gradient role (blockIdx.y = 0), [B, 2B): the input-gradient role
        out["wgrad"] = summary(s[:B], t0)
        out["dgrad"] = summary(s[B:], t0)
    print(json.dumps(out))
