#!/usr/bin/env python
"""Phase timeline of the fused small-net step (workgroup 0's wall clock after every layer):
where the per-image kernel spends its time.  Prints one JSON line per model."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402

for name in sys.argv[1:] or ["lenet5", "mnist_mlp"]:
    m = getattr(tde.zoo, name)()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    plan = PG.make_plan(m, m._store, "cuda", 128, 128, m.optimizer, m.loss)
    x = torch.rand((128,) + tuple(m.input_shape[1:]), device="cuda")
    y = torch.randint(0, 10, (128,), dtype=torch.int32, device="cuda")
    plan.stamps = torch.zeros(64, dtype=torch.int64, device="cuda")
    for _ in range(20):
        plan.train_step(x, y)
    torch.cuda.synchronize()
    st = plan.stamps.cpu().numpy()
    labels = ["start"] + [f"fwd{i}:{'CPD'[k]}" for i, k in enumerate(plan.layers[:, 0])] + ["loss"]
    for i, k in reversed(list(enumerate(plan.layers[:, 0]))):
        labels += [f"bwd{i}:wgrad", f"bwd{i}:dgrad"] if k == 0 else [f"bwd{i}:{'CPD'[k]}"]
    n = len(labels)
    us = (st[:n] - st[0]) / 100.0     # 100 MHz wall clock -> us
    print(json.dumps({"model": name, "phase_end_us": {l: round(float(u), 2) for l, u in zip(labels, us)}}))
