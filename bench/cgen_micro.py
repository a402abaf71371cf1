#!/usr/bin/env python
"""Per-launch device time of the generic fused small-CNN kernels (csrc/kernels/convnet_gen.hip) across the
instantiated widths, beside the hand-tuned Conv2D(32)/Dense(64) kernels (convnet_f32.hip) at B=64.

    python bench/cgen_micro.py [--iters 200] [--widths 32x64,64x128]

Each launch kind is replayed ``iters`` times inside one HIP graph (as the training Program runs it) and timed
with events; prints one JSON line per (width, launch)."""
from __future__ import annotations

import argparse
import json

import torch


def _time_graph(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--widths", default="16x32,32x64,32x128,64x64,64x128")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hrep", type=int, default=4, help="pre-activation split-K replicas")
    ap.add_argument("--crep", type=int, default=8, help="conv-gradient replicas")
    ap.add_argument("--phases", action="store_true",
                    help="also print the backward's per-workgroup phase clocks (median / max over the trunk)")
    a = ap.parse_args()
    from tensorflow_distributed_example_amd.ops import kernels as K
    dev = "cuda"
    B, H, W, NC = a.batch, 28, 28, 10
    Pn = 13 * 13
    Bp = (B + 7) // 8 * 8
    torch.manual_seed(0)
    x = torch.rand(B, H, W, 1, device=dev)
    y = torch.randint(0, NC, (B,), device=dev, dtype=torch.int32)
    for spec in a.widths.split(","):
        CC, HD = (int(v) for v in spec.split("x"))
        Kf = Pn * CC
        wc = torch.randn(3, 3, 1, CC, device=dev) * 0.1
        bc = torch.zeros(CC, device=dev)
        W1 = torch.randn(Kf, HD, device=dev) * 0.01
        b1 = torch.zeros(HD, device=dev)
        W2 = torch.randn(HD, NC, device=dev) * 0.1
        b2 = torch.zeros(NC, device=dev)
        hp = torch.zeros(2, a.hrep, B, HD, device=dev)
        Pt = torch.zeros(Kf, Bp, device=dev)
        amax = torch.zeros(Pn, CC // 8, Bp, dtype=torch.int64, device=dev)
        gc = torch.zeros(a.crep, 10 * CC, device=dev)
        g = dict(dW1=torch.zeros(Kf, HD, device=dev), dwc=gc[0, :9 * CC].view(3, 3, 1, CC), dbc=gc[0, 9 * CC:],
                 dW2=torch.zeros(HD, NC, device=dev), db2=torch.zeros(NC, device=dev), db1=torch.zeros(HD, device=dev),
                 crep=a.crep, crep_stride=10 * CC)
        met = torch.zeros(4, device=dev)
        fwd = lambda: K.cgen_fwd(x, wc, bc, W1, hp[0], Pt, amax, B=B)  # noqa: E731
        bwd = lambda: K.cgen_bwd(x, amax, hp[0], hp[1], b1, W2, b2, y, scale=1.0 / B, pre_relu=True,  # noqa: E731
                                 metrics=met, W1=W1, Pt=Pt, B=B, **g)
        fwd()
        for name, fn in (("cgen_fwd", fwd), ("cgen_bwd", bwd)):
            print(json.dumps({"width": spec, "launch": name, "hrep": a.hrep, "crep": a.crep,
                              "us": round(_time_graph(fn, a.iters), 2)}), flush=True)
        if a.phases:
            # phase clocks (100 MHz): 0 start, 1 staged, 2 softmax, 3 dH, 4 GEMM tiles, 5 routing, 6 dW1 out,
            # 7 conv-gradient atomics issued
            st = torch.zeros(Pn + 1, 8, dtype=torch.int64, device=dev)
            for _ in range(3):
                bwd()
            torch.cuda.synchronize()
            K.cgen_bwd(x, amax, hp[0], hp[1], b1, W2, b2, y, scale=1.0 / B, pre_relu=True, metrics=met, W1=W1, Pt=Pt,
                       B=B, stamps=st, **g)
            torch.cuda.synchronize()
            sf = torch.zeros(Pn * ((B + 63) // 64), 8, dtype=torch.int64, device=dev)
            K.cgen_fwd(x, wc, bc, W1, hp[0], Pt, amax, B=B, stamps=sf)
            torch.cuda.synchronize()
            tf = sf.double() * 0.01
            f0 = float(tf[:, 0].min())
            print(json.dumps({"width": spec, "launch": "cgen_fwd_phases", "last_start_us": round(float(tf[:, 0].max()) - f0, 2),
                              "last_end_us": round(float(tf[:, 3].max()) - f0, 2),
                              **{f"ph{i}": (round(float((tf[:, i] - tf[:, i - 1]).median()), 2),
                                            round(float((tf[:, i] - tf[:, i - 1]).max()), 2)) for i in (1, 2, 3)}}),
                  flush=True)
            t = st[:Pn].double() * 0.01   # us
            t0 = float(t[:, 0].min())
            ph = {f"ph{i}": (round(float((t[:, i] - t[:, i - 1]).median()), 2),
                             round(float((t[:, i] - t[:, i - 1]).max()), 2)) for i in range(1, 8)}
            print(json.dumps({"width": spec, "launch": "cgen_bwd_phases", "last_start_us": round(float(t[:, 0].max()) - t0, 2),
                              "last_end_us": round(float(t[:, 7].max()) - t0, 2), **ph}), flush=True)
        if (CC, HD) == (32, 64):   # the hand-tuned kernels at the reference width, plain step
            amax32 = torch.zeros(Kf // 32, 4, Bp, dtype=torch.int64, device=dev)
            h1 = torch.zeros(4, B, HD, device=dev)
            h2 = torch.zeros(4, B, HD, device=dev)
            f32 = lambda: K.convnet_fwd(x, wc, bc, W1, h1, Pt, amax32, hrep=4)  # noqa: E731
            b32 = lambda: K.convnet_bwd(x, amax32, h1, h2, b1, W2, b2, y, scale=1.0 / B, pre_relu=True,  # noqa: E731
                                        metrics=met, W1row=W1, Pt=Pt, dW1=g["dW1"], dwc=g["dwc"], dbc=g["dbc"],
                                        dW2=g["dW2"], db2=g["db2"], db1=g["db1"], crep=a.crep, crep_stride=10 * CC)
            f32()
            for name, fn in (("convnet32_fwd", f32), ("convnet32_bwd", b32)):
                print(json.dumps({"width": spec, "launch": name, "us": round(_time_graph(fn, a.iters), 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
