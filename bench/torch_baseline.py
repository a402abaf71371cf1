#!/usr/bin/env python
"""Stock PyTorch-ROCm baseline for the BASELINE.md comparison (the reference publishes no numbers):
the same models, batch sizes, optimizer and synthetic data as bench.py, written the way a PyTorch
user would — torch.nn modules (MIOpen convolutions, hipBLASLt GEMMs), bf16 autocast, SGD, and
DistributedDataParallel over RCCL for N>1.  ``--graph`` additionally captures the whole training
step in a CUDA(HIP) graph, the strongest stock-PyTorch configuration without a compiler.

    python bench/torch_baseline.py --model mnist_cnn --steps 400 --warmup 64 [--graph]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench/torch_baseline.py --gpus N ...

Prints one JSON line in bench.py's format (metric/config identical, "impl": "torch-baseline").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

MODELS = {  # per-GPU batch, lr, image shape (NHWC), classes
    "mnist_cnn": (64, 0.001, (28, 28, 1), 10),
    "mnist_bn_cnn": (128, 0.01, (28, 28, 1), 10),
    "mnist_cnn_wide": (64, 0.001, (28, 28, 1), 10),
    "mnist_bn_cnn_x2": (128, 0.01, (28, 28, 1), 10),
    "resnet18": (64, 0.1, (224, 224, 3), 1000),
    "lenet5": (128, 0.01, (28, 28, 1), 10),
    "mnist_mlp": (128, 0.01, (28, 28, 1), 10),
}


class LeNet5(nn.Module):  # models/zoo.py lenet5
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(1, 6, 5, padding=2)
        self.c2 = nn.Conv2d(6, 16, 5)
        self.f1 = nn.Linear(400, 120)
        self.f2 = nn.Linear(120, 84)
        self.f3 = nn.Linear(84, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.c1(x)), 2)
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        return self.f3(F.relu(self.f2(F.relu(self.f1(x.flatten(1))))))


class MLP(nn.Module):  # models/zoo.py mnist_mlp
    def __init__(self):
        super().__init__()
        self.f1 = nn.Linear(784, 128)
        self.f2 = nn.Linear(128, 10)

    def forward(self, x):
        return self.f2(F.relu(self.f1(x.flatten(1))))


class MnistCNN(nn.Module):  # distributed_with_keras.py:33-39
    def __init__(self, filters=32, units=64):
        super().__init__()
        self.conv = nn.Conv2d(1, filters, 3)
        self.fc1 = nn.Linear(13 * 13 * filters, units)
        self.fc2 = nn.Linear(units, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv(x)), 2)
        return self.fc2(F.relu(self.fc1(x.flatten(1))))


class MnistBNCNN(nn.Module):  # mnist_keras_distributed.py:79-109 (TF-SAME pads are symmetric here)
    def __init__(self, m=1):
        super().__init__()
        self.c1 = nn.Conv2d(1, 6 * m, 3, padding=1, bias=False)
        self.b1 = nn.BatchNorm2d(6 * m, eps=1e-3, momentum=0.01, affine=True)
        self.c2 = nn.Conv2d(6 * m, 12 * m, 6, stride=2, padding=2, bias=False)
        self.b2 = nn.BatchNorm2d(12 * m, eps=1e-3, momentum=0.01)
        self.c3 = nn.Conv2d(12 * m, 24 * m, 6, stride=2, padding=2, bias=False)
        self.b3 = nn.BatchNorm2d(24 * m, eps=1e-3, momentum=0.01)
        self.fc1 = nn.Linear(7 * 7 * 24 * m, 200 * m, bias=False)
        self.b4 = nn.BatchNorm1d(200 * m, eps=1e-3, momentum=0.01)
        self.fc2 = nn.Linear(200 * m, 10)

    def forward(self, x):
        x = F.relu(self.b1(self.c1(x)))
        x = F.relu(self.b2(self.c2(x)))
        x = F.relu(self.b3(self.c3(x)))
        x = F.dropout(F.relu(self.b4(self.fc1(x.flatten(1)))), 0.5, self.training)
        return self.fc2(x)


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = self.b2(self.c2(F.relu(self.b1(self.c1(x)))))
        return F.relu(y + (self.proj(x) if self.proj is not None else x))


class ResNet18(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for i, c in enumerate([64, 128, 256, 512]):
            layers += [Block(cin, c, 1 if i == 0 else 2), Block(c, c, 1)]
            cin = c
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, classes)

    def forward(self, x):
        return self.fc(self.layers(self.stem(x)).mean((2, 3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--model", default="mnist_cnn", choices=sorted(MODELS))
    ap.add_argument("--batch-per-gpu", type=int, default=None)
    ap.add_argument("--graph", action="store_true", help="capture the whole step in a HIP graph")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="bf16",
                    help="bf16: torch.autocast bf16; fp32: plain float32 (the reference's precision, TF32 off)")
    a = ap.parse_args()
    if a.dtype == "fp32":   # like-for-like with our float32 kernels: no reduced-precision math anywhere
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
    B0, lr, img, ncls = MODELS[a.model]
    B = a.batch_per_gpu or B0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
    torch.manual_seed(1234)
    model = {"mnist_cnn": MnistCNN, "mnist_bn_cnn": MnistBNCNN, "resnet18": lambda: ResNet18(ncls),
             "lenet5": LeNet5, "mnist_mlp": MLP, "mnist_cnn_wide": lambda: MnistCNN(64, 128),
             "mnist_bn_cnn_x2": lambda: MnistBNCNN(2)}[a.model]()
    model = model.to(dev)
    mf = torch.channels_last if a.channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[local], gradient_as_bucket_view=True)
    opt = torch.optim.SGD(model.parameters(), lr=lr, foreach=True)
    H, W, C = img
    pool = 4
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    xs = torch.rand((pool, B, C, H, W), generator=g).to(dev)
    ys = torch.randint(0, ncls, (pool, B), generator=g).to(dev)
    sx, sy = xs[0].clone().contiguous(memory_format=mf), ys[0].clone()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
            loss = F.cross_entropy(model(sx), sy)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        return loss

    graph = None
    if a.graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()

    def run(i):
        sx.copy_(xs[i % pool], non_blocking=True)
        sy.copy_(ys[i % pool], non_blocking=True)
        if graph is not None:
            graph.replay()
        else:
            step()

    for i in range(a.warmup):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        run(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        print(json.dumps({"metric": "images/sec (whole node) torch baseline", "impl": "torch-baseline",
                          "value": round(B * world * a.steps / el, 1), "unit": "images/sec", "n_gpus": world,
                          "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 5),
                          "dtype": "bf16-autocast" if a.dtype == "bf16" else "fp32", "config": {"model": a.model, "global_batch": B * world,
                                                               "per_gpu_batch": B, "hipgraph": a.graph,
                                                               "channels_last": a.channels_last}}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
