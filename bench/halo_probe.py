#!/usr/bin/env python
"""Counter-pass probe: 20 launches of ONE halo-tile conv (csrc/kernels/haloconv.hip) on the ResNet-18 stage-1
geometry (B=64, 56x56x64), forward by default, ``dgrad`` for the input gradient.  scripts/pmc_halo.sh runs it
under rocprofv3 --pmc."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tensorflow_distributed_example_amd.ops import layer_ops as O  # noqa: E402

torch.cuda.set_device(0)
mode = sys.argv[1] if len(sys.argv) > 1 else "fwd"
B, H = 64, 56
g = O.ConvGeom(B, H, H, 64, H, H, 64, 3, 3, 1, 1, 1, 1)
x = torch.randn(B * H * H * 64, device="cuda").to(torch.bfloat16)
w = (torch.randn(3, 3, 64, 64, device="cuda") * 0.05).to(torch.bfloat16)
wt = w.permute(3, 0, 1, 2).reshape(64, 576).contiguous()
y = torch.empty_like(x)
st = torch.zeros(2 * O.STAT_SLOTS * 64, dtype=torch.float64, device="cuda")
for _ in range(20):
    if mode == "dgrad":
        O.halo_conv(x, w, y, g, dgrad=True)
    else:
        O.halo_conv(x, wt, y, g, colstats=st)
torch.cuda.synchronize()
print("ok")
