"""Optimizers: Keras SGD (v2: distributed_with_keras.py:42,
tf2_mnist_distributed.py:137), TF1 GradientDescentOptimizer
(mnist_keras_distributed.py:111) and Adam (BASELINE north star).

On the GPU the update runs as ONE multi-tensor HIP kernel over the flat
parameter buffer (csrc/kernels/optim.hip) that also zeroes gradients, refreshes
bf16 weight shadows and advances the device-resident ``iterations`` counter.
``apply_reference`` is the torch implementation of the same math (CPU backend
and numerics oracle).
"""
from __future__ import annotations

import math

import torch

KIND = {"sgd": 0, "momentum": 1, "nesterov": 2, "adam": 3}


class Optimizer:
    kind = "sgd"

    def __init__(self, learning_rate=0.01, name=None):
        self.learning_rate = float(learning_rate)
        self.name = name or type(self).__name__
        self.iterations = 0  # host mirror; device counter lives in the program

    @property
    def lr(self):
        return self.learning_rate

    @property
    def kind_id(self):
        return KIND[self.kind]

    def slot_names(self):
        return []

    def hparams(self):
        return dict(mom=0.0, b1=0.9, b2=0.999, eps=1e-7)

    def apply_reference(self, w, g, slots, step):
        raise NotImplementedError

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate}


class SGD(Optimizer):
    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, name="SGD", **kw):
        lr = kw.pop("lr", learning_rate)
        super().__init__(lr, name)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        if self.momentum < 0:
            raise ValueError("momentum must be >= 0")

    @property
    def kind(self):
        if self.momentum == 0.0:
            return "sgd"
        return "nesterov" if self.nesterov else "momentum"

    def slot_names(self):
        return ["momentum"] if self.momentum else []

    def hparams(self):
        return dict(mom=self.momentum, b1=0.9, b2=0.999, eps=1e-7)

    @torch.no_grad()
    def apply_reference(self, w, g, slots, step):
        lr = self.learning_rate
        if self.momentum == 0.0:
            w.sub_(lr * g)
            return
        v = slots["momentum"]
        v.mul_(self.momentum).sub_(lr * g)
        if self.nesterov:
            w.add_(self.momentum * v - lr * g)
        else:
            w.add_(v)

    def get_config(self):
        return {**super().get_config(), "momentum": self.momentum, "nesterov": self.nesterov}


class GradientDescentOptimizer(SGD):
    """TF1 ``tf.train.GradientDescentOptimizer(learning_rate)`` (mnist_keras_distributed.py:111)."""

    def __init__(self, learning_rate, use_locking=False, name="GradientDescent"):
        super().__init__(learning_rate, 0.0, False, name)


class Adam(Optimizer):
    kind = "adam"

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, name="Adam", **kw):
        super().__init__(kw.pop("lr", learning_rate), name)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)

    def slot_names(self):
        return ["m", "v"]

    def hparams(self):
        return dict(mom=0.0, b1=self.beta_1, b2=self.beta_2, eps=self.epsilon)

    @torch.no_grad()
    def apply_reference(self, w, g, slots, step):
        t = step + 1
        m, v = slots["m"], slots["v"]
        m.mul_(self.beta_1).add_((1 - self.beta_1) * g)
        v.mul_(self.beta_2).add_((1 - self.beta_2) * g * g)
        lr_t = self.learning_rate * math.sqrt(1 - self.beta_2 ** t) / (1 - self.beta_1 ** t)
        w.sub_(lr_t * m / (v.sqrt() + self.epsilon))

    def get_config(self):
        return {**super().get_config(), "beta_1": self.beta_1, "beta_2": self.beta_2, "epsilon": self.epsilon}


def get(identifier):
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, str):
        k = identifier.lower()
        if k == "sgd":
            return SGD()
        if k == "adam":
            return Adam()
    raise ValueError(f"unsupported optimizer {identifier!r}")
