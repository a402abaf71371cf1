#!/usr/bin/env python
"""Kernel microbenchmarks for the fused MNIST-CNN plan on one MI355X.

* launch floor: empty-kernel cost, eager and inside a hipGraph;
* per-kernel standalone time: each kernel of the step replayed 200x in a graph;
* phase stamps: s_memrealtime stamps at phase boundaries of each workgroup
  (diagnostic only) -> where inside each kernel the time goes.
Prints one JSON object; used to build profiles/*.md.
"""
from __future__ import annotations

import json
import sys

import os
sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys as _sys
_sys.path.insert(0, sys_path_root)
import numpy as np
import torch


def graph_time(fn, reps=200, inner=1):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def eager_time(fn, reps=500):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def stamps_summary(st, nslots):
    st = st.cpu().numpy().astype(np.float64)
    used = st[:, :nslots]
    used = used[(used > 0).all(axis=1)]
    if len(used) == 0:
        return {}
    t0 = used[:, 0].min()
    rel = (used - t0) * 0.01  # 100 MHz ticks -> us
    return {f"slot{i}": {"min": round(float(rel[:, i].min()), 2), "med": round(float(np.median(rel[:, i])), 2),
                         "max": round(float(rel[:, i].max()), 2)} for i in range(nslots)}


def main():
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.ops import kernels as K
    torch.cuda.set_device(0)
    out = {}
    out["noop_eager_us"] = eager_time(lambda: K.noop(1, 64))
    out["noop_graph_us"] = graph_time(lambda: K.noop(1, 64))
    out["noop_graph_256wg_us"] = graph_time(lambda: K.noop(256, 256))
    out["noop_graph_1024thr_43wg_us"] = graph_time(lambda: K.noop(43, 1024))

    tde.backend.set_random_seed(0)
    m = tde.zoo.mnist_cnn()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.001),
              metrics=["accuracy"])
    prog = m._program("train", 64)
    plan = prog.plans[0]
    x = torch.rand(64, 28, 28, 1, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda", dtype=torch.int32)

    def k_fwd(stamps=None):
        q = plan.parity
        local = plan.step_mode == "local"
        K.convnet_fwd(x, plan._v("wc"), plan._v("bc"), plan.W1fwd, plan.hpre2[q], plan.Pt, plan.amax, stamps=stamps,
                      opt=plan._fopt[q] if local else None,
                      off_wc=plan.store.segments[plan.names["wc"]].offset,
                      off_bc=plan.store.segments[plan.names["bc"]].offset, inc_iter=plan.iterations,
                      hrep=plan.hrep)

    def k_bwd(stamps=None):
        q = plan.parity
        local = plan.step_mode == "local"
        dwc, dbc = plan._gconv_views(q) if local else (plan._g("wc"), plan._g("bc"))
        K.convnet_bwd(x, plan.amax, plan.hpre2[q], plan.hpre2[1 - q], plan._v("b1"), plan._v("w2"), plan._v("b2"), y,
                      scale=plan.scale, pre_relu=True, metrics=plan.metrics, W1row=plan.W1row, Pt=plan.Pt,
                      dW1=plan._g("w1"), dwc=dwc, dbc=dbc, dW2=plan._g("w2"), db2=plan._g("b2"), db1=plan._g("b1"),
                      B=64, stamps=stamps, opt=plan._bopt[q] if local else None)

    def k_opt():
        plan.opt.apply()

    def step():
        plan.train_step(x, y)
        plan.apply()

    def step_local():
        plan.train_step(x, y)

    plan.set_step_mode("plain")
    out["w1_source"] = "rows" if plan.w1_rows else "col"
    out["kernel_graph_us"] = {n: graph_time(f) for n, f in
                              [("convnet_fwd", k_fwd), ("convnet_bwd_head", k_bwd), ("optim", k_opt)]}
    out["step_graph_us"] = graph_time(step, reps=100)
    out["step_eager_us"] = eager_time(step, reps=200)
    # fused single-replica step: the optimizer inside the two launches, one flush per execution
    plan.set_step_mode("local")
    out["local_kernel_graph_us"] = {n: graph_time(f) for n, f in
                                    [("convnet_fwd", k_fwd), ("convnet_bwd_head", k_bwd), ("flush", plan.finish)]}
    out["local_step_graph_us"] = graph_time(step_local, reps=100)
    plan.finish()
    plan.set_step_mode("plain")
    st = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    for name, f, ns in [("convnet_fwd", k_fwd, 5), ("convnet_bwd_head", k_bwd, 6)]:
        st.zero_()
        f()
        torch.cuda.synchronize()
        st.zero_()
        f(stamps=st)
        torch.cuda.synchronize()
        out[f"stamps_{name}"] = stamps_summary(st.view(-1, 8), ns)
        rows = st.view(-1, 8).cpu().numpy().astype(np.float64)
        head = rows[rows[:, 7] > 0]
        if len(head):   # the backward's head workgroup: start and end, on the trunk's clock
            t0 = rows[rows[:, 0] > 0, 0].min()
            out[f"stamps_{name}_head_wg"] = {"start": round((head[0, 0] - t0) * 0.01, 2),
                                            "end": round((head[0, 7] - t0) * 0.01, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
