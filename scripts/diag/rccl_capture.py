"""GPU check of the RCCL communicator inside hipGraph capture on one device: a 1-rank clique built
through the multi-process init path (ncclCommInitRank + unique id), all-reduce captured with a
kernel, replayed, and the MWMS training program with that communicator captured end to end."""
import torch

import tensorflow_distributed_example_amd as tde
from tensorflow_distributed_example_amd.parallel import comm as CM

dev = torch.device("cuda", 0)
uid = CM.RcclCommunicator.unique_id()
c = CM.RcclCommunicator([dev], rank0=0, nranks=1, unique_id=uid)
x = torch.ones(1 << 20, device=dev)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    c.all_reduce_([x])
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    x.mul_(2.0)
    c.all_reduce_([x])
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("rccl capture ok", x[0].item(), "expect", 2.0 ** 3, "nccl version", c.lib.tde_nccl_version())
c.check_health()
