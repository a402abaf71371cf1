#!/usr/bin/env python
"""Per-layer GEMM timings of the ResNet-18 layer-wise plan on one MI355X (B = 64, bf16).

For every Conv2D stage of the compiled plan: forward (implicit GEMM + BN-statistics epilogue),
input gradient and weight gradient, each replayed in a hipGraph; prints µs and TFLOP/s per op and
the totals.  ``--sweep`` re-times the weight gradients under the split-K / K-step knobs of
``tde_igemm_tune`` (csrc/kernels/layers.hip) to pick the defaults.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))
import torch  # noqa: E402

from micro import graph_time  # noqa: E402


def _convs(plan, LW):
    # the stem (im2col or packed-stem path) has its own kernels: timed by the model bench, not here
    return [st for st in plan.stages if isinstance(st, LW._Gemm) and st.conv and not st.use_im2col
            and not st.use_stem_pack]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sweep-tile", action="store_true", help="sweep the fwd/dgrad tile-size threshold only")
    ap.add_argument("--sweep-big-dgrad", action="store_true", help="A/B the dgrad big tiles only")
    ap.add_argument("--sweep-fd", action="store_true", help="fwd / dgrad per layer over tile threshold x K step")
    ap.add_argument("--sweep-wgrad", action="store_true", help="weight-gradient path x stages x tile cap x split target")
    ap.add_argument("--ab-mfma32", action="store_true",
                    help="per layer: fwd / dgrad / wgrad on the 16x16x32 vs 32x32x16 MFMA kernels (A/B/A/B)")
    a = ap.parse_args()
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd import _native as N
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    from tensorflow_distributed_example_amd.train import layerwise as LW
    torch.cuda.set_device(0)
    tde.backend.set_global_policy("mixed_bfloat16")   # ResNet-18's BASELINE config (the bf16 kernel forms)
    tde.backend.set_random_seed(0)
    m = tde.zoo.resnet18()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1))
    B = a.batch
    prog = m._program("train", B)
    plan = prog.plans[0]
    x = torch.rand((1, B, 224, 224, 3)).cuda()
    y = torch.randint(0, 1000, (1, B)).to(torch.int32).cuda()
    prog.stage([(x, y)])
    prog.run()
    torch.cuda.synchronize()
    rows = []
    for st in _convs(plan, LW):
        g = st.geo.with_batch(B)
        dout = st.out.root().grad
        flop = 2.0 * g.B * g.Ho * g.Wo * g.Co * g.K
        t_f = graph_time(lambda: st.fwd(plan, B, True), a.reps)
        t_w = graph_time(lambda: O.conv_wgrad(st.inp.buf, dout, st.gW, g, scratch=plan.wscratch), a.reps)
        t_d = graph_time(lambda: O.conv_dgrad(dout, st.Wrow, st.inp.root().grad, g, scratch=plan.scratch),
                         a.reps) if st.need_dgrad else 0.0
        rows.append(dict(layer=st.layer.name, shape=f"{g.H}x{g.W}x{g.C}->{g.Ho}x{g.Wo}x{g.Co} k{g.KH}s{g.sh}",
                         fwd_us=t_f, dgrad_us=t_d, wgrad_us=t_w, gflop=flop / 1e9))
    tot = {k: round(sum(r[k] for r in rows), 1) for k in ("fwd_us", "dgrad_us", "wgrad_us")}
    for r in rows:
        def tf(us):
            return r["gflop"] / us * 1e3 if us else 0.0
        print(f"{r['layer']:<14} {r['shape']:<28} fwd {r['fwd_us']:7.1f} us {tf(r['fwd_us']):5.0f} TF | dgrad "
              f"{r['dgrad_us']:7.1f} us {tf(r['dgrad_us']):5.0f} TF | wgrad {r['wgrad_us']:7.1f} us "
              f"{tf(r['wgrad_us']):5.0f} TF", flush=True)
    print("TOTAL", json.dumps(tot), flush=True)
    if a.ab_mfma32:
        lib = N.hip()
        tot = {}
        for rnd, mask in enumerate((0, 7, 0, 7)):
            lib.tde_igemm_mfma32(mask)
            for st in _convs(plan, LW):
                g = st.geo.with_batch(B)
                dout = st.out.root().grad
                # igemm forward even where the plan runs the halo kernel (stage 1)
                t_f = graph_time(lambda: O.conv_fwd(st.inp.buf, st.Wt, st.out.root().buf, g, colstats=st.colstats,
                                                    scratch=plan.scratch), a.reps)
                t_d = graph_time(lambda: O.conv_dgrad(dout, st.Wrow, st.inp.root().grad, g, scratch=plan.scratch),
                                 a.reps) if st.need_dgrad else 0.0
                t_w = graph_time(lambda: O.conv_wgrad(st.inp.buf, dout, st.gW, g, scratch=plan.wscratch), a.reps)
                if rnd >= 2:
                    print(f"AB32 mask={mask} {st.layer.name:<20} fwd {t_f:6.1f} dgrad {t_d:6.1f} wgrad {t_w:6.1f}",
                          flush=True)
                k = tot.setdefault(mask, [0.0, 0.0, 0.0])
                k[0] += t_f / 2
                k[1] += t_d / 2
                k[2] += t_w / 2
        for mask, (f, d, w) in tot.items():
            print(f"AB32 TOTAL mask={mask}: fwd {f:.1f} dgrad {d:.1f} wgrad {w:.1f} us (mean of 2 rounds)", flush=True)
        lib.tde_igemm_mfma32(-1)
    if a.sweep_tile:
        lib = N.hip()
        for tmin in (512, 1024, 1536, 2048, 3072, 4096, 100000):
            lib.tde_igemm_tile_min(tmin)
            tf_ = sum(graph_time(lambda: st.fwd(plan, B, True), a.reps) for st in _convs(plan, LW))
            td_ = sum(graph_time(lambda: O.conv_dgrad(st.out.root().grad, st.Wrow, st.inp.root().grad,
                                                      st.geo.with_batch(B), scratch=plan.scratch), a.reps)
                      for st in _convs(plan, LW) if st.need_dgrad)
            print(f"SWEEP tile_min={tmin}: fwd {tf_:.1f} us dgrad {td_:.1f} us", flush=True)
        lib.tde_igemm_tile_min(2048)
    if a.sweep_fd:
        # fwd / dgrad per layer under (tile_min, K step): picks the per-shape defaults
        lib = N.hip()
        cfgs = [(tm, kb, 0) for kb in (32, 64) for tm in (64, 160, 256, 1024, 2048, 4096)] + [(2048, 64, 1)]
        for st in _convs(plan, LW):
            g = st.geo.with_batch(B)
            res = []
            for tm, kb, big in cfgs:
                lib.tde_igemm_tile_min(tm)
                lib.tde_igemm_tune(512, 16, kb, -1, big, 64)
                lib.tde_igemm_big_dgrad(big)
                tf_ = graph_time(lambda: st.fwd(plan, B, True), a.reps)
                td_ = graph_time(lambda: O.conv_dgrad(st.out.root().grad, st.Wrow, st.inp.root().grad, g,
                                                      scratch=plan.scratch), a.reps) if st.need_dgrad else 0.0
                res.append(f"t{tm}/k{kb}{'/big' if big else ''}: {tf_:.1f}/{td_:.1f}")
            print(f"SWEEPFD {st.layer.name} {g.H}x{g.W}x{g.C}->{g.Co} s{g.sh} | " + " | ".join(res), flush=True)
        lib.tde_igemm_tile_min(2048)
        lib.tde_igemm_tune(512, 16, 0, -1, 0, 192)
        lib.tde_igemm_big_dgrad(0)
    if a.sweep_wgrad:
        lib = N.hip()
        for mode, cap, target in [(0, 0, 512), (3, 0, 512), (1, 0, 512), (2, 0, 512), (1, 1, 512), (2, 1, 512),
                                  (3, 0, 256), (3, 0, 1024), (0, 0, 512), (3, 0, 512)]:
            lib.tde_igemm_wgrad_dma(mode)
            lib.tde_igemm_wgrad_tile_cap(cap)
            lib.tde_igemm_tune(target, 16, 0, -1, -1, 0)
            per = []
            for st in _convs(plan, LW):
                g = st.geo.with_batch(B)
                per.append(graph_time(lambda: O.conv_wgrad(st.inp.buf, st.out.root().grad, st.gW, g,
                                                           scratch=plan.wscratch), a.reps))
            print(f"SWEEPWG dma={mode} cap={cap} target={target}: {sum(per):.1f} us | "
                  + " ".join(f"{t:.1f}" for t in per), flush=True)
        lib.tde_igemm_wgrad_dma(3)
        lib.tde_igemm_wgrad_tile_cap(0)
        lib.tde_igemm_tune(512, 16, 0, -1, -1, 0)
    if a.sweep_big_dgrad:
        lib = N.hip()
        for bd in (0, 1, 0, 1):
            lib.tde_igemm_big_dgrad(bd)
            td_ = sum(graph_time(lambda: O.conv_dgrad(st.out.root().grad, st.Wrow, st.inp.root().grad,
                                                      st.geo.with_batch(B), scratch=plan.scratch), a.reps)
                      for st in _convs(plan, LW) if st.need_dgrad)
            print(f"SWEEP big_dgrad={bd}: dgrad {td_:.1f} us", flush=True)
        lib.tde_igemm_big_dgrad(0)
    if a.sweep:
        lib = N.hip()
        for target, mkt, kb in [(1024, 8, 0), (512, 8, 0), (256, 8, 0), (512, 16, 0), (256, 16, 0), (2048, 4, 0),
                                (1024, 8, 32), (512, 8, 32), (2048, 4, 32)]:
            lib.tde_igemm_tune(target, mkt, kb, -1, -1, 0)
            tw = 0.0
            for st in _convs(plan, LW):
                g = st.geo.with_batch(B)
                tw += graph_time(lambda: O.conv_wgrad(st.inp.buf, st.out.root().grad, st.gW, g, scratch=plan.wscratch), a.reps)
            print(f"SWEEP wgrad target={target} min_kt={mkt} kb={kb}: {tw:.1f} us", flush=True)
        for glds, kb, big, bmin in ((1, 0, 0, 0), (1, 0, 1, 64), (1, 0, 1, 128), (1, 0, 1, 192), (1, 0, 1, 256),
                                    (0, 0, 0, 0)):
            lib.tde_igemm_tune(512, 16, kb, glds, big, bmin)
            tf_ = sum(graph_time(lambda: st.fwd(plan, B, True), a.reps) for st in _convs(plan, LW))
            td_ = sum(graph_time(lambda: O.conv_dgrad(st.out.root().grad, st.Wrow, st.inp.root().grad,
                                                      st.geo.with_batch(B), scratch=plan.scratch), a.reps)
                      for st in _convs(plan, LW) if st.need_dgrad)
            print(f"SWEEP glds={glds} kb={kb} big={big} min={bmin}: fwd {tf_:.1f} us dgrad {td_:.1f} us", flush=True)
        lib.tde_igemm_tune(512, 16, 0, 1, 0, 192)
        # dgrad on the 256-row big tiles (KB = 64) vs the default KB = 32 tiles, A/B/A/B
        for bd in (0, 1, 0, 1):
            lib.tde_igemm_big_dgrad(bd)
            td_ = sum(graph_time(lambda: O.conv_dgrad(st.out.root().grad, st.Wrow, st.inp.root().grad,
                                                      st.geo.with_batch(B), scratch=plan.scratch), a.reps)
                      for st in _convs(plan, LW) if st.need_dgrad)
            print(f"SWEEP big_dgrad={bd}: dgrad {td_:.1f} us", flush=True)
        lib.tde_igemm_big_dgrad(0)


if __name__ == "__main__":
    main()
