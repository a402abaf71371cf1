"""The reference's model architectures (random-init, Keras-default initializers).

* ``mnist_cnn()``    — Model A, distributed_with_keras.py:33-39 (== tf2_mnist_distributed.py:66-72):
  347,146 trainable params.
* ``mnist_bn_cnn()`` — Model B, mnist_keras_distributed.py:79-109 (== tf2_mnist_distributed.py:105-135):
  250,466 trainable + 484 non-trainable params.

Models for the remaining BASELINE.json configs (not in the reference):

* ``lenet5()``    — "MNIST LeNet-5 CNN bf16, MirroredStrategy on 1 MI355X": LeNet-5 with ReLU and max
  pooling, 61,706 trainable params.
* ``mnist_mlp()`` — "tf2_mnist_distributed.py dense MLP on CPU, MirroredStrategy devices=1":
  Flatten · Dense(128, relu) · Dense(10), 101,770 trainable params.
* ``resnet18()``  — "Synthetic 224x224x3 ResNet-18 bf16 on 8xMI355X".
"""
from __future__ import annotations

from . import layers as L
from .model import Sequential


def mnist_cnn(name=None, filters=32, units=64):
    return Sequential([
        L.Conv2D(filters, 3, activation="relu", input_shape=(28, 28, 1)),
        L.MaxPooling2D(),
        L.Flatten(),
        L.Dense(units, activation="relu"),
        L.Dense(10),
    ], name=name)


def mnist_cnn_wide(name=None):
    """Model A with every width doubled: Conv2D(64) / Dense(128) (a user edit of distributed_with_keras.py
    :33-39 that the fused small-CNN step was not specialised for)."""
    return mnist_cnn(name, filters=64, units=128)


def mnist_bn_cnn(name=None, mult=1):
    return Sequential([
        L.Reshape(input_shape=(28 * 28,), target_shape=(28, 28, 1)),
        L.Conv2D(filters=6 * mult, kernel_size=3, padding="same", use_bias=False),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(filters=12 * mult, kernel_size=6, padding="same", use_bias=False, strides=2),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Conv2D(filters=24 * mult, kernel_size=6, padding="same", use_bias=False, strides=2),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Flatten(),
        L.Dense(200 * mult, use_bias=False),
        L.BatchNormalization(scale=False, center=True),
        L.Activation("relu"),
        L.Dropout(0.5),
        L.Dense(10, activation="softmax"),
    ], name=name)


def mnist_bn_cnn_x2(name=None):
    """Model B with every width doubled (12/24/48 filters, Dense(400)): runs on the layer-wise plan."""
    return mnist_bn_cnn(name, mult=2)


def lenet5(name=None):
    return Sequential([
        L.Conv2D(6, 5, padding="same", activation="relu", input_shape=(28, 28, 1)),
        L.MaxPooling2D(),
        L.Conv2D(16, 5, activation="relu"),
        L.MaxPooling2D(),
        L.Flatten(),
        L.Dense(120, activation="relu"),
        L.Dense(84, activation="relu"),
        L.Dense(10),
    ], name=name)


def mnist_mlp(name=None):
    return Sequential([
        L.Flatten(input_shape=(28, 28, 1)),
        L.Dense(128, activation="relu"),
        L.Dense(10),
    ], name=name)


def _basic_block(x, filters, stride, name):
    """ResNet v1 BasicBlock: 3x3(s) - BN - ReLU - 3x3 - BN, + (projection) shortcut, ReLU."""
    y = L.Conv2D(filters, 3, strides=stride, padding="same", use_bias=False, kernel_initializer="he_normal",
                 name=f"{name}_conv1")(x)
    y = L.BatchNormalization(epsilon=1e-5, momentum=0.9, name=f"{name}_bn1")(y)
    y = L.Activation("relu", name=f"{name}_relu1")(y)
    y = L.Conv2D(filters, 3, padding="same", use_bias=False, kernel_initializer="he_normal", name=f"{name}_conv2")(y)
    y = L.BatchNormalization(epsilon=1e-5, momentum=0.9, name=f"{name}_bn2")(y)
    if stride != 1 or x.shape[-1] != filters:
        s = L.Conv2D(filters, 1, strides=stride, use_bias=False, kernel_initializer="he_normal",
                     name=f"{name}_proj")(x)
        s = L.BatchNormalization(epsilon=1e-5, momentum=0.9, name=f"{name}_proj_bn")(s)
    else:
        s = x
    y = L.Add(name=f"{name}_add")([y, s])
    return L.Activation("relu", name=f"{name}_out")(y)


def resnet(stage_blocks=(2, 2, 2, 2), filters=(64, 128, 256, 512), input_shape=(224, 224, 3), classes=1000,
           stem_filters=None, name="resnet"):
    """BasicBlock ResNet v1 (functional API, TF-'SAME' padding: asymmetric (2,3) for the 7x7/2 stem at
    224): 7x7/2 conv-BN-ReLU stem, 3x3/2 max-pool, stages of BasicBlocks (first block of stages 2+
    strides 2 with a 1x1 projection shortcut), global average pool, Dense logits."""
    from .model import Model
    inp = L.Input(input_shape)
    x = L.Conv2D(stem_filters or filters[0], 7, strides=2, padding="same", use_bias=False,
                 kernel_initializer="he_normal", name="conv1")(inp)
    x = L.BatchNormalization(epsilon=1e-5, momentum=0.9, name="conv1_bn")(x)
    x = L.Activation("relu", name="conv1_relu")(x)
    x = L.MaxPooling2D(3, strides=2, padding="same", name="pool1")(x)
    for i, (nb, f) in enumerate(zip(stage_blocks, filters)):
        for j in range(nb):
            x = _basic_block(x, f, 2 if (i > 0 and j == 0) else 1, f"stage{i + 1}_block{j + 1}")
    x = L.GlobalAveragePooling2D(name="avg_pool")(x)
    out = L.Dense(classes, name="fc")(x)
    return Model(inputs=inp, outputs=out, name=name)


def resnet18(input_shape=(224, 224, 3), classes=1000, name="resnet18"):
    """ResNet-18 (BASELINE.json stress config; not in the reference): 11.69M parameters at 224/1000."""
    return resnet((2, 2, 2, 2), (64, 128, 256, 512), input_shape, classes, name=name)


def mini_resnet(input_shape=(32, 32, 3), classes=10, name="mini_resnet"):
    """A two-stage BasicBlock ResNet (16 / 32 filters) on 32x32x3: ResNet-18's layer kinds (stem conv, BN,
    max-pool, projection shortcut, residual add, GAP, Dense) at test size."""
    return resnet((1, 1), (16, 32), input_shape, classes, name=name)

