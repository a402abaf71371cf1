"""Keras-compatible layers (channels_last / NHWC activations, HWIO conv kernels,
[in, out] dense kernels — byte-compatible with Keras/TF checkpoints).

Layers used by the reference models:
  * Model A (distributed_with_keras.py:33-39, tf2_mnist_distributed.py:66-72):
    Conv2D(32,3,relu) · MaxPooling2D · Flatten · Dense(64,relu) · Dense(10)
  * Model B (mnist_keras_distributed.py:79-109, tf2_mnist_distributed.py:105-135):
    Reshape · Conv2D(same, no bias) · BatchNormalization(scale=False) ·
    Activation('relu') · ... · Dropout(0.5) · Dense(10, softmax)
plus ResNet building blocks (ZeroPadding2D, GlobalAveragePooling2D, Add) for the
ResNet-18 stress config.

Each layer declares its weights (``WeightSpec``) and a reference forward made of
plain torch ops (``ref_call``) — the CPU backend's kernel library and the
numerics oracle for the HIP kernels.  On the GPU the training program replaces
layer chains by fused HIP stages (train/program.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .. import backend as K
from . import initializers


@dataclass
class WeightSpec:
    name: str            # short name: "kernel", "bias", "beta", "moving_mean", ...
    shape: tuple
    initializer: Callable
    trainable: bool = True
    aggregation: str = "none"   # SyncOnRead aggregation for non-trainables ("mean")
    layer: "Layer" = field(default=None, repr=False)

    @property
    def full_name(self):
        return f"{self.layer.name}/{self.name}"


def _tuple2(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def get_activation(a):
    if a is None or a == "linear":
        return None
    if callable(a):
        return a
    if a not in ("relu", "softmax", "sigmoid", "tanh"):
        raise ValueError(f"unsupported activation {a!r}")
    return a


def apply_activation(x, act):
    if act is None:
        return x
    if act == "relu":
        return F.relu(x)
    if act == "softmax":
        return torch.softmax(x, dim=-1)
    if act == "sigmoid":
        return torch.sigmoid(x)
    if act == "tanh":
        return torch.tanh(x)
    return act(x)


def tf_same_pads(n, k, s):
    """TF 'SAME' padding: pad_total = max((ceil(n/s)-1)*s + k - n, 0); before = total//2."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


class KerasTensor:
    """Symbolic tensor of the functional API: a shape plus the layer call that produces it."""

    def __init__(self, shape, producer=None, inputs=(), name=None):
        self.shape = (None,) + tuple(int(d) for d in shape)
        self.producer = producer
        self.inputs = list(inputs)
        self.name = name

    def __repr__(self):
        who = self.producer.name if self.producer is not None else self.name
        return f"<KerasTensor shape={self.shape} from {who}>"


def Input(shape=None, batch_size=None, name=None, dtype=None, batch_shape=None):
    """``keras.Input``: the symbolic model input (channels_last image or feature vector)."""
    if shape is None and batch_shape is not None:
        shape = tuple(batch_shape[1:])
    return KerasTensor(tuple(shape), name=name or K.unique_name("input"))


class Layer:
    _prefix = "layer"
    multi_input = False

    def __init__(self, name: Optional[str] = None, input_shape=None, trainable=True, **kwargs):
        for k in kwargs:
            if k not in ("dtype", "batch_input_shape", "input_dim"):
                raise TypeError(f"{type(self).__name__}: unexpected argument {k!r}")
        if "input_dim" in kwargs and input_shape is None:
            input_shape = (kwargs["input_dim"],)
        self.name = name or K.unique_name(self._prefix)
        self.input_shape_arg = tuple(input_shape) if input_shape is not None else None
        self.trainable = trainable
        self.built = False
        self.weight_specs: list[WeightSpec] = []
        self.input_shape = None
        self.output_shape = None
        self._model = None  # owning model (weights live in its ParamStore)

    # ---- building
    def add_weight(self, name, shape, initializer="zeros", trainable=True, aggregation="none"):
        spec = WeightSpec(name, tuple(int(s) for s in shape), initializers.get(initializer),
                          trainable and self.trainable, aggregation, self)
        self.weight_specs.append(spec)
        return spec

    def build(self, input_shape):
        self.built = True

    def compute_output_shape(self, input_shape):
        return input_shape

    def _build_shapes(self, input_shape):
        if self.multi_input:
            self.input_shape = [tuple(x) for x in input_shape]
            self.built = True
            self.output_shape = tuple(self.compute_output_shape(self.input_shape))
            return self.output_shape
        self.input_shape = tuple(input_shape)
        if not self.built:
            self.build(self.input_shape)
            self.built = True
        self.output_shape = tuple(self.compute_output_shape(self.input_shape))
        return self.output_shape

    # ---- functional API: calling a layer on symbolic tensors records a graph node
    def __call__(self, inputs, **kw):
        multi = isinstance(inputs, (list, tuple))
        ins = list(inputs) if multi else [inputs]
        if not all(isinstance(t, KerasTensor) for t in ins):
            raise TypeError(f"{self.name}: layers are called on symbolic tensors from Input(); "
                            "use model.predict()/model(x) for eager execution")
        shapes = [t.shape[1:] for t in ins]
        out = self._build_shapes(shapes if multi else shapes[0])
        return KerasTensor(out, producer=self, inputs=ins)

    # ---- weights (views into the owning model's ParamStore)
    def w(self, name):
        return self._model._store.view(f"{self.name}/{name}")

    @property
    def weights(self):
        return [self.w(s.name) for s in self.weight_specs]

    @property
    def trainable_weights(self):
        return [self.w(s.name) for s in self.weight_specs if s.trainable]

    def count_params(self):
        return int(sum(np.prod(s.shape) for s in self.weight_specs))

    # ---- reference forward (torch ops)
    def ref_call(self, x, W: dict, training: bool, rng=None, state_updates=None):
        raise NotImplementedError

    def get_config(self):
        return {"name": self.name}

    def __repr__(self):
        return f"<{type(self).__name__} {self.name}>"


class InputLayer(Layer):
    _prefix = "input"

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        return x


class Conv2D(Layer):
    _prefix = "conv2d"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 data_format=None, dilation_rate=(1, 1), **kw):
        super().__init__(**kw)
        if data_format not in (None, "channels_last"):
            raise ValueError("only channels_last is supported (Keras default)")
        if _tuple2(dilation_rate) != (1, 1):
            raise ValueError("dilation is not supported")
        self.filters = int(filters)
        self.kernel_size = _tuple2(kernel_size)
        self.strides = _tuple2(strides)
        self.padding = padding.lower()
        if self.padding not in ("valid", "same"):
            raise ValueError(padding)
        self.activation = get_activation(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def build(self, input_shape):
        cin = input_shape[-1]
        kh, kw = self.kernel_size
        self.add_weight("kernel", (kh, kw, cin, self.filters), self.kernel_initializer)
        if self.use_bias:
            self.add_weight("bias", (self.filters,), self.bias_initializer)
        self.built = True

    def pads(self, input_shape):
        H, W = input_shape[0], input_shape[1]
        if self.padding == "valid":
            return (0, 0), (0, 0)
        return tf_same_pads(H, self.kernel_size[0], self.strides[0]), tf_same_pads(W, self.kernel_size[1], self.strides[1])

    def compute_output_shape(self, s):
        H, W = s[0], s[1]
        kh, kw = self.kernel_size
        sh, sw = self.strides
        if self.padding == "valid":
            Ho, Wo = (H - kh) // sh + 1, (W - kw) // sw + 1
        else:
            Ho, Wo = -(-H // sh), -(-W // sw)
        return (Ho, Wo, self.filters)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        (pt, pb), (pl, pr) = self.pads(x.shape[1:])
        xc = x.permute(0, 3, 1, 2)
        if pt or pb or pl or pr:
            xc = F.pad(xc, (pl, pr, pt, pb))
        k = W["kernel"].permute(3, 2, 0, 1)
        y = F.conv2d(xc, k, W.get("bias"), stride=self.strides)
        return apply_activation(y.permute(0, 2, 3, 1), self.activation)

    def get_config(self):
        return dict(name=self.name, filters=self.filters, kernel_size=self.kernel_size, strides=self.strides,
                    padding=self.padding, activation=self.activation, use_bias=self.use_bias)


class Dense(Layer):
    _prefix = "dense"

    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = get_activation(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def build(self, input_shape):
        self.add_weight("kernel", (input_shape[-1], self.units), self.kernel_initializer)
        if self.use_bias:
            self.add_weight("bias", (self.units,), self.bias_initializer)
        self.built = True

    def compute_output_shape(self, s):
        return tuple(s[:-1]) + (self.units,)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        y = x @ W["kernel"]
        if self.use_bias:
            y = y + W["bias"]
        return apply_activation(y, self.activation)

    def get_config(self):
        return dict(name=self.name, units=self.units, activation=self.activation, use_bias=self.use_bias)


class MaxPooling2D(Layer):
    _prefix = "max_pooling2d"

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", **kw):
        super().__init__(**kw)
        self.pool_size = _tuple2(pool_size)
        self.strides = _tuple2(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()

    def compute_output_shape(self, s):
        H, W, C = s
        ph, pw = self.pool_size
        sh, sw = self.strides
        if self.padding == "valid":
            return ((H - ph) // sh + 1, (W - pw) // sw + 1, C)
        return (-(-H // sh), -(-W // sw), C)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        xc = x.permute(0, 3, 1, 2)
        if self.padding == "same":
            (pt, pb) = tf_same_pads(x.shape[1], self.pool_size[0], self.strides[0])
            (pl, pr) = tf_same_pads(x.shape[2], self.pool_size[1], self.strides[1])
            xc = F.pad(xc, (pl, pr, pt, pb), value=float("-inf"))
        y = F.max_pool2d(xc, self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1)

    def get_config(self):
        return dict(name=self.name, pool_size=self.pool_size, strides=self.strides, padding=self.padding)


class GlobalAveragePooling2D(Layer):
    _prefix = "global_average_pooling2d"

    def compute_output_shape(self, s):
        return (s[-1],)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        return x.mean(dim=(1, 2))


class ZeroPadding2D(Layer):
    _prefix = "zero_padding2d"

    def __init__(self, padding=(1, 1), **kw):
        super().__init__(**kw)
        if isinstance(padding, int):
            padding = ((padding, padding), (padding, padding))
        elif isinstance(padding[0], int):
            padding = ((padding[0], padding[0]), (padding[1], padding[1]))
        self.padding = padding

    def compute_output_shape(self, s):
        (t, b), (l, r) = self.padding
        return (s[0] + t + b, s[1] + l + r, s[2])

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        (t, b), (l, r) = self.padding
        return F.pad(x, (0, 0, l, r, t, b))

    def get_config(self):
        return dict(name=self.name, padding=self.padding)


class Flatten(Layer):
    _prefix = "flatten"

    def compute_output_shape(self, s):
        return (int(np.prod(s)),)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        return x.reshape(x.shape[0], -1)  # row-major over (H, W, C): Keras order


class Reshape(Layer):
    _prefix = "reshape"

    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def compute_output_shape(self, s):
        if int(np.prod(s)) != int(np.prod(self.target_shape)):
            raise ValueError(f"cannot reshape {s} to {self.target_shape}")
        return self.target_shape

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        return x.reshape((x.shape[0],) + self.target_shape)

    def get_config(self):
        return dict(name=self.name, target_shape=self.target_shape)


class Activation(Layer):
    _prefix = "activation"

    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = get_activation(activation)

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        return apply_activation(x, self.activation)

    def get_config(self):
        return dict(name=self.name, activation=self.activation)


class ReLU(Activation):
    _prefix = "re_lu"

    def __init__(self, **kw):
        super().__init__("relu", **kw)

    def get_config(self):
        return dict(name=self.name)


class Dropout(Layer):
    _prefix = "dropout"

    def __init__(self, rate, noise_shape=None, seed=None, **kw):
        super().__init__(**kw)
        self.rate = float(rate)
        self.seed = seed

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        if not K.resolve_training(training) or self.rate == 0.0:
            return x
        keep = 1.0 - self.rate
        mask = torch.rand(x.shape, generator=rng, device="cpu" if rng is not None else x.device)
        mask = (mask.to(x.device) < keep).to(x.dtype)
        return x * mask / keep

    def get_config(self):
        return dict(name=self.name, rate=self.rate)


class BatchNormalization(Layer):
    _prefix = "batch_normalization"

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True,
                 beta_initializer="zeros", gamma_initializer="ones",
                 moving_mean_initializer="zeros", moving_variance_initializer="ones", **kw):
        super().__init__(**kw)
        if axis not in (-1,):
            raise ValueError("BatchNormalization: only axis=-1 (channels_last) is supported")
        self.momentum = float(momentum)
        self.epsilon = float(epsilon)
        self.center = center
        self.scale = scale
        self.inits = (beta_initializer, gamma_initializer, moving_mean_initializer, moving_variance_initializer)

    def build(self, input_shape):
        c = input_shape[-1]
        if self.scale:
            self.add_weight("gamma", (c,), self.inits[1])
        if self.center:
            self.add_weight("beta", (c,), self.inits[0])
        self.add_weight("moving_mean", (c,), self.inits[2], trainable=False, aggregation="mean")
        self.add_weight("moving_variance", (c,), self.inits[3], trainable=False, aggregation="mean")
        self.built = True

    @property
    def fused(self):
        # TF/Keras uses the fused kernel (Bessel-corrected moving variance) for 4-D input.
        return self.input_shape is not None and len(self.input_shape) == 3

    def ref_call(self, x, W, training, rng=None, state_updates=None):
        axes = tuple(range(x.dim() - 1))
        gamma = W.get("gamma")
        beta = W.get("beta")
        if K.resolve_training(training):
            mean = x.mean(dim=axes)
            var = x.var(dim=axes, unbiased=False)
            if state_updates is not None:
                n = x.numel() // x.shape[-1]
                var_upd = var * (n / max(n - 1, 1)) if self.fused else var
                m = self.momentum
                state_updates.append((f"{self.name}/moving_mean", W["moving_mean"] * m + mean.detach() * (1 - m)))
                state_updates.append((f"{self.name}/moving_variance",
                                      W["moving_variance"] * m + var_upd.detach() * (1 - m)))
        else:
            mean, var = W["moving_mean"], W["moving_variance"]
        y = (x - mean) * torch.rsqrt(var + self.epsilon)
        if gamma is not None:
            y = y * gamma
        if beta is not None:
            y = y + beta
        return y

    def get_config(self):
        return dict(name=self.name, momentum=self.momentum, epsilon=self.epsilon, center=self.center,
                    scale=self.scale)


class Add(Layer):
    """Element-wise sum of same-shaped inputs (ResNet shortcut join)."""
    _prefix = "add"
    multi_input = True

    def compute_output_shape(self, shapes):
        for s_ in shapes[1:]:
            if tuple(s_) != tuple(shapes[0]):
                raise ValueError(f"{self.name}: shape mismatch {shapes}")
        return tuple(shapes[0])

    def ref_call(self, xs, W, training, rng=None, state_updates=None):
        out = xs[0]
        for x in xs[1:]:
            out = out + x
        return out


LAYER_CLASSES = {c.__name__: c for c in [InputLayer, Conv2D, Dense, MaxPooling2D, GlobalAveragePooling2D,
                                         ZeroPadding2D, Flatten, Reshape, Activation, ReLU, Dropout,
                                         BatchNormalization, Add]}


def from_config(cls_name, cfg):
    cfg = dict(cfg)
    cls = LAYER_CLASSES[cls_name]
    return cls(**cfg)
