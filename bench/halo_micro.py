#!/usr/bin/env python
"""Stage-1 ResNet-18 conv (B=64, 56x56x64 -> 56x56x64, 3x3 s1 SAME, bf16): the persistent halo-tile kernel
(csrc/kernels/haloconv.hip) against the implicit GEMM (csrc/kernels/layers.hip), forward (+BN statistics)
and input gradient, each timed inside a hipGraph (bench/micro.py graph_time).  Prints one JSON line."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--grids", default="0")
    a = ap.parse_args()
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    torch.cuda.set_device(0)
    B, H = a.batch, a.hw
    g = O.ConvGeom(B, H, H, 64, H, H, 64, 3, 3, 1, 1, 1, 1)
    x = torch.randn(B * H * H * 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(3, 3, 64, 64, device="cuda") * 0.05).to(torch.bfloat16)
    wt = w.permute(3, 0, 1, 2).reshape(64, 576).contiguous()
    y = torch.empty_like(x)
    y2 = torch.empty_like(x)
    st = torch.zeros(2 * O.STAT_SLOTS * 64, dtype=torch.float64, device="cuda")
    scratch = torch.zeros(max(O.scratch_elems(B * H * H, 64, 576), 1), dtype=torch.float32, device="cuda")
    flop = 2.0 * B * H * H * 64 * 576
    res = {}
    res["igemm_fwd_us"] = graph_time(lambda: O.conv_fwd(x, wt, y, g, colstats=st, scratch=scratch), reps=a.reps)
    res["igemm_dgrad_us"] = graph_time(lambda: O.conv_dgrad(x, w, y, g, scratch=scratch), reps=a.reps)
    for gr in [int(v) for v in a.grids.split(",")]:
        res[f"halo_fwd_us_grid{gr}"] = graph_time(lambda: O.halo_conv(x, wt, y2, g, colstats=st, grid=gr),
                                                  reps=a.reps)
        res[f"halo_dgrad_us_grid{gr}"] = graph_time(lambda: O.halo_conv(x, w, y2, g, dgrad=True, grid=gr),
                                                    reps=a.reps)
    # phase clocks of one forward launch (s_memrealtime, 100 MHz): per-workgroup means relative to the
    # earliest workgroup start
    from tensorflow_distributed_example_amd import _native as N
    stamps = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    for name, fn in (("fwd", lambda: O.halo_conv(x, wt, y2, g, colstats=st)),
                     ("dgrad", lambda: O.halo_conv(x, w, y2, g, dgrad=True))):
        fn()
        torch.cuda.synchronize()
        N.hip().tde_halo_stamps(stamps.data_ptr())
        fn()
        torch.cuda.synchronize()
        N.hip().tde_halo_stamps(None)
        sv = stamps.view(-1, 8)[:256].double()
        t0 = sv[:, 0].min()
        rel = (sv[:, :8] - t0) * 0.01   # us
        res[f"{name}_phase_us"] = {"start": round(rel[:, 0].mean().item(), 2),
                                   "first_rows_ready": round(rel[:, 1].mean().item(), 2),
                                   "tile0_mfma_done": round(rel[:, 2].mean().item(), 2),
                                   "tile0_loop_clock_ghz": round(((sv[:, 7] - sv[:, 6]) / ((sv[:, 2] - sv[:, 1]) * 10.0)).mean().item(), 3),
                                   "tile1_mfma_done": round(rel[:, 3].mean().item(), 2),
                                   "loop_done": round(rel[:, 4].mean().item(), 2),
                                   "end_mean": round(rel[:, 5].mean().item(), 2),
                                   "end_max": round(rel[:, 5].max().item(), 2)}
    # agreement of the two forward paths on the same operands
    O.conv_fwd(x, wt, y, g, scratch=scratch)
    O.halo_conv(x, wt, y2, g)
    torch.cuda.synchronize()
    res["fwd_rel_diff"] = ((y.float() - y2.float()).norm() / y.float().norm()).item()
    res["tflops"] = {k: round(flop / v * 1e-6, 1) for k, v in res.items() if isinstance(v, float) and (k.endswith("us") or "_us_" in k)}
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
