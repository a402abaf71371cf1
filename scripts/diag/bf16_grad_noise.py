"""Diagnostic: how far do bf16 mixed-precision gradients of Model B sit from fp32 ones?
Compares (a) the layer-wise HIP plan and (b) torch autocast-bf16 autograd against the fp32
torch reference, for one training step on the same weights/batch."""
import numpy as np
import torch

import tensorflow_distributed_example_amd as tde
from tensorflow_distributed_example_amd.train import program as PG


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    m = tde.zoo.mnist_bn_cnn()
    for l in m.layers:
        if isinstance(l, tde.keras.layers.Dropout):
            l.rate = 0.0
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01))
    m.build()
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.random((64, 784), dtype=np.float32)).cuda()
    y = torch.from_numpy(rng.integers(0, 10, 64)).int().cuda()
    st = m._store
    st_ref, st_amp = st.clone_to("cuda"), st.clone_to("cuda")
    plan = PG.make_plan(m, st, "cuda", 64, 64, m.optimizer, m.loss)
    ref = PG.ReferencePlan(m, st_ref, "cuda", 64, 64, m.optimizer, m.loss)
    amp = PG.ReferencePlan(m, st_amp, "cuda", 64, 64, m.optimizer, m.loss)
    plan.train_step(x, y)
    ref.train_step(x, y.long())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        amp.train_step(x, y.long())
    torch.cuda.synchronize()
    print(f"{'variable':40s} {'hip_vs_fp32':>12s} {'amp_vs_fp32':>12s} {'hip_vs_amp':>12s}")
    for n in st.names(trainable=True):
        print(f"{n:40s} {rel(st.grad(n), st_ref.grad(n)):12.4f} {rel(st_amp.grad(n), st_ref.grad(n)):12.4f} "
              f"{rel(st.grad(n), st_amp.grad(n)):12.4f}")


if __name__ == "__main__":
    main()
