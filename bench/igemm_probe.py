#!/usr/bin/env python
"""Where does an implicit-GEMM conv spend its time?  Times one ResNet-18 stage-1 conv
(64x56x56x64 -> 64, 3x3) under epilogue / operand variants (hipGraph replays, µs)."""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))
import torch  # noqa: E402

from micro import graph_time  # noqa: E402


def main():
    from tensorflow_distributed_example_amd.ops import layer_ops as O
    torch.cuda.set_device(0)
    bf = torch.bfloat16
    cfgs = [(64, 56, 64, 64), (64, 28, 128, 128), (64, 7, 512, 512)]
    if len(sys.argv) > 1:
        cfgs = [cfgs[int(sys.argv[1])]]
    for (B, H, C, Co) in cfgs:
        g = O.ConvGeom(B, H, H, C, H, H, Co, 3, 3, 1, 1, 1, 1)
        M, K = B * H * H, 9 * C
        x = torch.randn(B * H * H * C, device="cuda").to(bf)
        Wt = torch.randn(Co, K, device="cuda").to(bf)
        y = torch.zeros(M * Co, device="cuda", dtype=bf)
        yf = torch.zeros(M * Co, device="cuda")
        st = torch.zeros(2 * 8 * Co, device="cuda", dtype=torch.float64)
        xcol = torch.randn(M * K, device="cuda").to(bf)
        fl = 2.0 * M * Co * K
        res = {}
        res["conv bf16+stats"] = graph_time(lambda: O.conv_fwd(x, Wt, y, g, colstats=st), 20)
        res["conv bf16"] = graph_time(lambda: O.conv_fwd(x, Wt, y, g), 20)
        res["conv f32 out"] = graph_time(lambda: O._igemm(x, 0, O.A_CONV, Wt, K, O.B_NK, M, Co, K, g, cf=yf, ldc=Co,
                                                         cf_mode=1), 20)
        res["dense(im2col) bf16"] = graph_time(lambda: O._igemm(xcol, K, O.A_ROWK, Wt, K, O.B_NK, M, Co, K, cb=y,
                                                               ldcb=Co), 20)
        res["conv K/9 bf16"] = graph_time(lambda: O._igemm(x, 0, O.A_CONV, Wt, K, O.B_NK, M, Co, C, g, cb=y,
                                                          ldcb=Co), 20)
        if os.environ.get("PROBE_TORCH", "1") == "1":   # library reference point (hipBLASLt), same GEMM
            xm, wm = xcol.view(M, K), Wt.t()
            res["torch.mm(im2col) bf16"] = graph_time(lambda: torch.mm(xm, wm, out=y.view(M, Co)), 20)
        dW = torch.zeros(K * Co, device="cuda")
        dy = torch.randn(M * Co, device="cuda").to(bf)
        res["wgrad atomics"] = graph_time(lambda: O.conv_wgrad(x, dy, dW, g), 20)
        print(f"B{B} {H}x{H}x{C}->{Co}: " + " | ".join(f"{k} {v:.1f}us ({fl / v * 1e-6 if 'K/9' not in k else fl / 9 / v * 1e-6:.0f}TF)"
                                                      for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
