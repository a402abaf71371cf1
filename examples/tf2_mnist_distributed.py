#!/usr/bin/env python
"""In-spirit port of tf2_mnist_distributed.py (reference: TF 1.15-style Estimator
under tf.distribute.experimental.ParameterServerStrategy(), constants instead of
flags, model_dir hard-coded to '/tmp/mode').

Same constants (TF2M:26-35), Model B (TF2M:105-135) with the v2 SGD optimizer
(TF2M:137) — using the learning_rate ARGUMENT (the reference ignored it, Q6) —
input_fn / serving_input_fn, RunConfig(train_distribute=strategy) and
train_and_evaluate.  The reference's unused custom ``model_fn`` (TF2M:65-91) is
kept, fixed (Q9), as an example of a custom Estimator model_fn.
TF_CONFIG must be set externally for distributed runs (no CLUSTER_SPEC translation).
"""
import argparse
import logging
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402

BATCH_SIZE = 128
BUFFER_SIZE = 10000
LEARNING_RATE = 1e-4
MODEL_DIR = os.environ.get("TDE_MODEL_DIR", "/tmp/mode")
MAX_STEPS = int(os.environ["TDE_MAX_STEPS"]) if os.environ.get("TDE_MAX_STEPS") else None


def input_fn(features, labels, batch_size, mode):
    inputs = features if labels is None else (features, labels)
    dataset = tde.data.Dataset.from_tensor_slices(inputs)
    if mode == tde.estimator.ModeKeys.TRAIN:
        dataset = dataset.shuffle(1000).repeat().batch(batch_size)
        dataset = dataset.prefetch(100)
    if mode in (tde.estimator.ModeKeys.EVAL, tde.estimator.ModeKeys.PREDICT):
        dataset = dataset.batch(batch_size)
    return dataset


def model_fn(features, labels, mode):
    """Custom model_fn of the reference (dead code there): Model A + SCCE(from_logits) + SGD."""
    model = tde.keras.Sequential([
        tde.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        tde.keras.layers.MaxPooling2D(),
        tde.keras.layers.Flatten(),
        tde.keras.layers.Dense(64, activation="relu"),
        tde.keras.layers.Dense(10),
    ])
    logits = model(features, training=False)
    if mode == tde.estimator.ModeKeys.PREDICT:
        return tde.estimator.EstimatorSpec(mode=mode, predictions={"logits": logits})   # Q9: no labels=
    loss_object = tde.keras.losses.SparseCategoricalCrossentropy(from_logits=True, reduction="none")
    loss = loss_object(labels, logits).sum() * (1.0 / BATCH_SIZE)
    return tde.estimator.EstimatorSpec(mode=mode, loss=loss, train_op=None if mode == "eval" else "minimize")


def create_model(model_dir, config, learning_rate):
    l = tde.keras.layers
    model = tde.keras.Sequential([
        l.Reshape(input_shape=(28 * 28,), target_shape=(28, 28, 1)),
        l.Conv2D(filters=6, kernel_size=3, padding="same", use_bias=False),
        l.BatchNormalization(scale=False, center=True),
        l.Activation("relu"),
        l.Conv2D(filters=12, kernel_size=6, padding="same", use_bias=False, strides=2),
        l.BatchNormalization(scale=False, center=True),
        l.Activation("relu"),
        l.Conv2D(filters=24, kernel_size=6, padding="same", use_bias=False, strides=2),
        l.BatchNormalization(scale=False, center=True),
        l.Activation("relu"),
        l.Flatten(),
        l.Dense(200, use_bias=False),
        l.BatchNormalization(scale=False, center=True),
        l.Activation("relu"),
        l.Dropout(0.5),
        l.Dense(10, activation="softmax"),
    ])
    optimizer = tde.compat.v2.optimizers.SGD(learning_rate)   # Q6: honour the argument
    model.compile(optimizer=optimizer, loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    tde.keras.backend.set_learning_phase(True)
    model.summary()
    return tde.keras.estimator.model_to_estimator(keras_model=model, model_dir=model_dir, config=config)


def serving_input_fn():
    feature_placeholder = tde.compat.v1.placeholder(tde.float32, [None, 28 * 28])
    return tde.estimator.export.TensorServingInputReceiver(feature_placeholder, feature_placeholder)


def main(argv=None):
    # the reference has no CLI (its parser is commented out, TF2M:28-31): only the framework flags
    ap = tde.utils.flags.add_framework_flags(argparse.ArgumentParser())
    args, _ = ap.parse_known_args(argv)
    tde.utils.flags.apply_framework_flags(args)
    logging.getLogger().setLevel(logging.INFO)
    tde.get_logger().setLevel(logging.INFO)
    strategy = tde.distribute.experimental.ParameterServerStrategy()
    (train_images, train_labels), (test_images, test_labels) = tde.keras.datasets.mnist.load_data()
    train_images = (train_images / 255.0).astype(np.float32).reshape(-1, 784)
    test_images = (test_images / 255.0).astype(np.float32).reshape(-1, 784)
    train_labels = np.asarray(train_labels).astype("int").reshape((-1, 1))
    test_labels = np.asarray(test_labels).astype("int").reshape((-1, 1))
    train_steps = MAX_STEPS or math.ceil(len(train_images) / BATCH_SIZE)   # Q3: 468.75 -> 469

    config = tde.estimator.RunConfig(train_distribute=strategy)
    classifier = create_model(model_dir=MODEL_DIR, config=config, learning_rate=LEARNING_RATE)
    train_spec = tde.estimator.TrainSpec(
        input_fn=lambda: input_fn(train_images, train_labels, BATCH_SIZE, mode=tde.estimator.ModeKeys.TRAIN),
        max_steps=train_steps, hooks=tde.utils.flags.profiler_hooks(args, MODEL_DIR))
    exporter = tde.estimator.FinalExporter("exporter", serving_input_fn)
    eval_spec = tde.estimator.EvalSpec(
        input_fn=lambda: input_fn(test_images, test_labels, BATCH_SIZE, mode=tde.estimator.ModeKeys.EVAL),
        steps=None, name="mnist-eval", exporters=[exporter], start_delay_secs=10, throttle_secs=10)
    return tde.estimator.train_and_evaluate(classifier, train_spec, eval_spec)


if __name__ == "__main__":
    out = main()
    if out and out[0]:
        print("eval:", out[0], "exports:", out[1])
