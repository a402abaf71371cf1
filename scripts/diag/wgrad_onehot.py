"""Diagnostic: separate the A- and B-operand mappings of the weight-grad GEMM with one-hot inputs."""
import torch

from tensorflow_distributed_example_amd.ops import layer_ops as O

bf = torch.bfloat16
B, fin, out = 32, 128, 128
eye = torch.zeros(B, 128, device="cuda")
eye[torch.arange(B), torch.arange(B)] = 1
# test 1: A(m,k) = delta(m,k), B(k,n) = delta(n,0)  ->  dW[m,0] = 1 for m < 32
x = eye.to(bf)
dy = torch.zeros(B, out, device="cuda")
dy[:, 0] = 1
dW = torch.zeros(fin, out, device="cuda")
O.dense_wgrad(x, dy.to(bf), dW, B, splits=1)
torch.cuda.synchronize()
print("test1 col0 (want 1 for m<32):", dW[:40, 0].tolist())
print("test1 nonzero other cols:", (dW[:, 1:] != 0).sum().item())
# test 2: A(m,k) = delta(m,0), B(k,n) = delta(k,n)  ->  dW[0,n] = 1 for n < 32
x = torch.zeros(B, fin, device="cuda")
x[:, 0] = 1
dW.zero_()
O.dense_wgrad(x.to(bf), eye.to(bf), dW, B, splits=1)
torch.cuda.synchronize()
print("test2 row0 (want 1 for n<32):", dW[0, :40].tolist())
print("test2 nonzero other rows:", (dW[1:] != 0).sum().item())
# test 3: A(m,k) = delta(m,k) (k<32), B(k,n) = k+1  ->  dW[m,n] = m+1
dW.zero_()
dy = (torch.arange(B, device="cuda")[:, None] + 1).float().expand(B, out).contiguous()
O.dense_wgrad(eye.to(bf), dy.to(bf), dW, B, splits=1)
torch.cuda.synchronize()
print("test3 dW[:40,0] (want m+1):", dW[:40, 0].tolist())
