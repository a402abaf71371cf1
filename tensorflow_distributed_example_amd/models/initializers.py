"""Keras default initializers: glorot_uniform for kernels,
zeros for biases/beta/moving_mean, ones for gamma/moving_variance.

fan_in/fan_out follow Keras `_compute_fans`: for a conv kernel (kh, kw, cin, cout)
receptive = kh*kw, fan_in = receptive*cin, fan_out = receptive*cout.
Initial values are drawn on the host from a seeded generator so every replica /
worker can reproduce them (the chief broadcast makes them identical anyway).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _fans(shape):
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = int(np.prod(shape[:-2]))
    return shape[-2] * receptive, shape[-1] * receptive


def glorot_uniform(shape, gen):
    fi, fo = _fans(shape)
    limit = math.sqrt(6.0 / (fi + fo))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(limit).float()


def glorot_normal(shape, gen):
    fi, fo = _fans(shape)
    std = math.sqrt(2.0 / (fi + fo))
    return _truncated_normal(shape, gen, std)


def he_normal(shape, gen):
    fi, _ = _fans(shape)
    return _truncated_normal(shape, gen, math.sqrt(2.0 / fi))


def he_uniform(shape, gen):
    fi, _ = _fans(shape)
    limit = math.sqrt(6.0 / fi)
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(limit).float()


def _truncated_normal(shape, gen, std):
    # Keras truncated normal: resample beyond 2 std; scale by 1/0.8796 like VarianceScaling.
    std = std / 0.87962566103423978
    x = torch.randn(shape, generator=gen, dtype=torch.float64)
    bad = x.abs() > 2
    while bad.any():
        x[bad] = torch.randn(int(bad.sum()), generator=gen, dtype=torch.float64)
        bad = x.abs() > 2
    return (x * std).float()


def zeros(shape, gen=None):
    return torch.zeros(shape)


def ones(shape, gen=None):
    return torch.ones(shape)


_REG = {
    "glorot_uniform": glorot_uniform, "glorot_normal": glorot_normal, "he_normal": he_normal,
    "he_uniform": he_uniform, "zeros": zeros, "ones": ones,
}


def get(name):
    if callable(name):
        return name
    try:
        return _REG[name]
    except KeyError:
        raise ValueError(f"unknown initializer {name!r}") from None
