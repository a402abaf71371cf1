"""Diagnostic: reveal the operand mapping of the weight-grad (transposed-LDS) GEMM path."""
import torch

from tensorflow_distributed_example_amd.ops import layer_ops as O

bf = torch.bfloat16
B, fin, out = 32, 128, 128
x = torch.zeros(B, fin, dtype=bf, device="cuda")
for b in range(B):
    x[b, b] = 1.0                       # dW[i, n] = dy[i, n] for i < 32
dy = (torch.arange(B, device="cuda")[:, None] * 1000 + torch.arange(out, device="cuda")[None, :]).to(torch.float32)
dyb = dy.to(bf)
dW = torch.zeros(fin, out, device="cuda")
O.dense_wgrad(x, dyb, dW, B, splits=1)
torch.cuda.synchronize()
ref = x.float().t() @ dyb.float()
print("max err", (dW - ref).abs().max().item())
bad = (dW - ref).abs() > 1e-3 * ref.abs().clamp(min=1)
idx = bad.nonzero()[:12].tolist()
for i, n in idx:
    print("dW[%d,%d] = %g  want %g" % (i, n, dW[i, n].item(), ref[i, n].item()))
for C in (1, 8, 16):
    g = O.ConvGeom(2, 6, 6, C, 6, 6, 8, 3, 3, 1, 1, 1, 1)
    xx = torch.randn(2, 6, 6, C, device="cuda").to(bf)
    d = torch.randn(2, 6, 6, 8, device="cuda").to(bf)
    dw = torch.zeros(3, 3, C, 8, device="cuda")
    O.conv_wgrad(xx, d, dw, g, splits=1)
    xr = xx.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros(8, C, 3, 3, device="cuda", requires_grad=True)
    torch.nn.functional.conv2d(xr, wr, padding=1).backward(d.float().permute(0, 3, 1, 2))
    torch.cuda.synchronize()
    print("conv C=%d rel" % C, ((dw - wr.grad.permute(2, 3, 1, 0)).norm() / wr.grad.norm()).item())
