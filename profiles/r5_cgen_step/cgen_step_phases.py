#!/usr/bin/env python
"""The generic fused CNN step as one launch (cgen_step_kernel: forward, grid barrier, backward) vs two launches:
graph-timed per-step time of the plan's own local step, and the single launch's per-workgroup phase clocks
(100 MHz): forward start / staged / conv+pool / Dense slice + hpre atomics, barrier passed (= backward start),
then the backward's phases (bench/cgen_micro.py --phases numbering).

    python bench/cgen_step_phases.py [--width 32x64] [--steps 200]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("TDE_CONVNET_GENERIC", "1")
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd.models import layers as L  # noqa: E402
from tensorflow_distributed_example_amd.ops import kernels as K  # noqa: E402
from tensorflow_distributed_example_amd.train import program as PG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", default="32x64")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    CC, HD = (int(v) for v in a.width.split("x"))
    tde.backend.set_global_policy("float32")
    m = tde.models.Sequential([L.Conv2D(CC, 3, activation="relu", input_shape=(28, 28, 1)), L.MaxPooling2D(),
                               L.Flatten(), L.Dense(HD, activation="relu"), L.Dense(10)])
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    plan = PG.make_plan(m, m._store, "cuda", 64, 64, m.optimizer, m.loss)
    assert plan.kind == "fused_convnet_generic", plan.kind
    plan.set_step_mode("local")
    x = torch.rand(64, 28, 28, 1, device="cuda")
    y = torch.randint(0, 10, (64,), dtype=torch.int32, device="cuda")
    can = plan.single
    res = {"width": a.width, "single_fits": can}
    for single in ([False, True] if can else [False]):
        plan.single = single
        for _ in range(4):
            plan.train_step(x, y)
        plan.finish()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            plan.train_step(x, y)
            plan.train_step(x, y)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            for _ in range(a.steps):
                plan.train_step(x, y)
        g.replay()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / a.steps)
        plan.finish()
        res["us_per_step_single" if single else "us_per_step_two"] = round(best, 2)
    print(json.dumps(res), flush=True)
    if not can:
        return
    # phase clocks of one single-launch step
    plan.single = True
    P = plan.P
    sf = torch.zeros(P + 1, 8, dtype=torch.int64, device="cuda")
    sb = torch.zeros(P + 1, 8, dtype=torch.int64, device="cuda")
    of, ob = K.cgen_fwd, K.cgen_bwd
    K.cgen_fwd = lambda *p, **k: of(*p, stamps=sf, **k)
    K.cgen_bwd = lambda *p, **k: ob(*p, stamps=sb, **k)
    try:
        plan.train_step(x, y)
    finally:
        K.cgen_fwd, K.cgen_bwd = of, ob
    plan.finish()
    torch.cuda.synchronize()
    f = sf.double() * 0.01
    b = sb.double() * 0.01
    t0 = float(f[:, 0].min())
    trunk = slice(0, P)

    def ph(t, i, j, rows=trunk):
        d = t[rows, j] - t[rows, i] if not isinstance(i, torch.Tensor) else t[rows, j] - i[rows]
        return [round(float(d.median()), 2), round(float(d.max()), 2)]
    out = {"launch": "cgen_step_phases", "last_start_us": round(float(f[:, 0].max()) - t0, 2),
           "fwd_staged": ph(f, 0, 1), "fwd_conv": ph(f, 1, 2), "fwd_dense": ph(f, 2, 3),
           "last_arrival_us": round(float(f[trunk, 3].max()) - t0, 2),
           "barrier_exit_us": [round(float(b[:, 0].min()) - t0, 2), round(float(b[:, 0].max()) - t0, 2)],
           "bwd_head": ph(b, 0, 2), "bwd_dH": ph(b, 2, 3), "bwd_tiles": ph(b, 3, 4), "bwd_routing": ph(b, 4, 5),
           "bwd_out": ph(b, 5, 7), "last_end_us": round(float(b[trunk, 7].max()) - t0, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
