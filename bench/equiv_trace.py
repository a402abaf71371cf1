#!/usr/bin/env python
"""Repeatability of the fused single-replica training step, step by step (diagnostics).

Trains ``--trials`` fresh copies of a zoo model in ONE process, each on the same seeded init and the
same synthetic batches (``bench/dp_equiv.py``'s stream: 3 executions x 4 steps, lr 0.05), with
``Program.enable_trace`` recording the weights and the plan's cross-step state after every step inside
the captured hipGraph.  Every trial is compared, step by step, with the torch float32 reference plan run
on the CPU (same stream), and the ConvNet plan's deferred-update invariants (commit counter, pending
flags, gradient replicas) are read after each execution.

    python bench/equiv_trace.py --trials 20 --out gpurun_out/equiv_trace.npz

Prints one line per trial: the first step whose weights are > --tol away from the reference, the
per-variable differences there, and the invariants.  Diverging trials' traces go to ``--out``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def train(device, model_name, execs, spe, lr, trace=True):
    import numpy as np
    import torch

    import tensorflow_distributed_example_amd as tde
    tde.backend.clear_session()
    tde.backend.set_random_seed(77)
    tde.backend.set_global_policy("float32")
    strategy = tde.distribute.OneDeviceStrategy(device)
    with strategy.scope():
        model = getattr(tde.zoo, model_name)()
        model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tde.optimizers.SGD(learning_rate=lr), metrics=["accuracy"], steps_per_execution=spe)
    prog = model._program("train", 128)
    plan = prog.plans[0]
    if trace:
        prog.enable_trace()
    gen = torch.Generator().manual_seed(4242)
    shape = tuple(prog.x_shape)
    steps, inv = [], []
    for e in range(execs):
        x = torch.rand((spe, 128) + shape, generator=gen)
        y = torch.randint(0, 10, (spe, 128), generator=gen).to(torch.int32)
        prog.stage([(x.to(device), y.to(device))])
        prog.run()
        prog.sync()
        if trace:
            steps.append(prog.trace[0].detach().cpu().numpy().copy())
        if hasattr(plan, "step_invariants") and plan.step_mode == "local":
            inv.append(plan.step_invariants())
    st = plan.store
    names = st.names(trainable=True)
    segs = [(n, st.segments[n].offset, st.segments[n].numel) for n in names]
    m = prog.local_metrics()
    loss = float(m[0] / m[2])
    tr = np.concatenate(steps, 0) if steps else st.w.detach().cpu().numpy()[None].copy()   # untraced: final weights
    if steps and plan.kind == "fused_convnet" and plan.step_mode == "local":
        # the stored conv weights lag by the pending (deferred) update: the weights the next forward uses
        # are w - lr * sum(replicas of the pending parity) (SGD)
        nw_, ng = int(st.w.numel()), int(plan.gconv.numel())
        g = tr[:, nw_: nw_ + ng].reshape(len(tr), 2, plan.crep, plan._conv_span).sum(axis=2)
        pend = tr[:, nw_ + ng: nw_ + ng + 2]
        lo, span = plan._conv_lo, plan._conv_span
        tr = tr.copy()
        for q in (0, 1):
            tr[:, lo: lo + span] -= lr * g[:, q] * (pend[:, q:q + 1] != 0)
    return dict(trace=tr, segs=segs, inv=inv, loss=loss, kind=plan.kind, mode=plan.step_mode,
                nw=int(st.w.numel()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--model", default="mnist_cnn")
    ap.add_argument("--execs", type=int, default=3)
    ap.add_argument("--spe", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--tol", type=float, default=1e-5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-trace", action="store_true", help="no per-step copies in the graph: final weights only")
    a = ap.parse_args()
    import numpy as np

    ref = train("cpu", a.model, a.execs, a.spe, a.lr)
    nw = ref["nw"]
    print(f"[equiv_trace] reference cpu plan={ref['kind']} loss={ref['loss']:.6f}", flush=True)
    bad = {}
    for t in range(a.trials):
        r = train("cuda:0", a.model, a.execs, a.spe, a.lr, trace=not a.no_trace)
        w = r["trace"][:, :nw]
        d = np.abs(w - (ref["trace"][-1:, :nw] if a.no_trace else ref["trace"][:, :nw]))
        per_step = d.max(axis=1)
        first = int(np.argmax(per_step > a.tol)) if (per_step > a.tol).any() else -1
        inv = r["inv"]
        total = a.execs * a.spe
        ok_inv = all(iv["commits"] == (e + 1) * a.spe and iv["applied_on_the_fly"] == (e + 1) * (a.spe - 1)
                     and iv["pending"] == [0, 0] and iv["gconv_abs_max"] == 0.0 for e, iv in enumerate(inv))
        line = dict(trial=t, plan=r["kind"], mode=r["mode"], loss=round(r["loss"], 6),
                    max_diff=float(per_step.max()), first_step_over_tol=first, invariants_ok=ok_inv,
                    commits=inv[-1]["commits"] if inv else None, steps=total)
        if first >= 0:
            s = first
            line["at_first"] = {n: float(d[s, o: o + k].max()) for n, o, k in r["segs"]}
            line["per_step_max"] = [float(v) for v in per_step]
            bad[f"trial{t}"] = r["trace"]
        if not ok_inv:
            line["invariants"] = inv
        print("[equiv_trace] " + json.dumps(line), flush=True)
    if a.out and bad:
        np.savez(a.out, reference=ref["trace"], **bad)
    print(f"[equiv_trace] trials={a.trials} diverged={len(bad)}", flush=True)


if __name__ == "__main__":
    main()
