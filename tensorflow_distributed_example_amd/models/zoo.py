"""The reference's model architectures (random-init, Keras-default initializers).

* ``mnist_cnn()``    — Model A, distributed_with_keras.py:33-39 (== tf2_mnist_distributed.py:66-72):
  347,146 trainable params.
* ``mnist_bn_cnn()`` — Model B, mnist_keras_distributed.py:79-109 (== tf2_mnist_distributed.py:105-135):
  250,466 trainable + 484 non-trainable params.
"""
from __future__ import annotations

from . import layers as L
from .model import Sequential


def mnist_cnn(name=None):
    return Sequential([
        L.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        L.MaxPooling2D(),
        L.Flatten(),
        L.Dense(64, activation="relu"),
        L.Dense(10),
    ], name=name)


def mnist_bn_cnn(name=None):
    return Sequential([
        L.Reshape(input_shape=(28 * 28,), target_shape=(28, 28, 1)),
        L.Conv2D(filters=6, kernel_size=3, padding="same", use_bias=False),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(filters=12, kernel_size=6, padding="same", use_bias=False, strides=2),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(filters=24, kernel_size=6, padding="same", use_bias=False, strides=2),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Flatten(),
        L.Dense(200, use_bias=False),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Dropout(0.5),
        L.Dense(10, activation="softmax"),
    ], name=name)
