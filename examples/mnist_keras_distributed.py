#!/usr/bin/env python
"""In-spirit port of mnist_keras_distributed.py (reference: TF1 Estimator via
model_to_estimator; ParameterServerStrategy for training, MirroredStrategy for
evaluation; CLUSTER_SPEC/TASK_INDEX/JOB_NAME -> TF_CONFIG; TensorBoard on TB_PORT).

Same flags (MKD:33-65, parse_known_args), model (MKD:79-109: Model B, BN-CNN),
optimizer (GradientDescentOptimizer), set_learning_phase(True) + summary
(MKD:116-117), input_fn / serving_input_fn (MKD:123-162), RunConfig (MKD:240-248),
Train/EvalSpec + FinalExporter (MKD:255-275) and train_and_evaluate (MKD:283).
Quirks: --num-epochs is honoured (Q2: max_steps = ceil(epochs * N / batch)) unless
--max-steps is given; local mode is a well-defined chief (Q1); floats are ceil'ed (Q3).

Local run:        python examples/mnist_keras_distributed.py --working-dir /tmp/mkd
Cluster (1 ps + master + worker on this host):
    python -m tensorflow_distributed_example_amd.launch --ps 1 --master 1 --workers 1 \
        examples/mnist_keras_distributed.py --working-dir /tmp/mkd
"""
import argparse
import json
import logging
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402


def get_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--working-dir", type=str, required=True,
                        help="directory for checkpoints, summaries and exports")
    parser.add_argument("--num-epochs", type=float, default=5, help="number of times to go through the data")
    parser.add_argument("--batch-size", default=128, type=int, help="number of records to read during each step")
    parser.add_argument("--learning-rate", default=0.01, type=float, help="learning rate for gradient descent")
    parser.add_argument("--verbosity", choices=["DEBUG", "ERROR", "FATAL", "INFO", "WARN"], default="INFO")
    # framework additions
    parser.add_argument("--max-steps", type=int, default=None, help="override the epoch-derived step count")
    parser.add_argument("--eval-steps", type=int, default=None)
    parser.add_argument("--reference-steps", action="store_true",
                        help="reproduce the reference's one-epoch max_steps = len(train)/batch_size (Q2)")
    parser.add_argument("--no-tensorboard", action="store_true")
    tde.utils.flags.add_framework_flags(parser)
    args, _ = parser.parse_known_args(argv)
    return args


def create_model(model_dir, config, learning_rate):
    l = tde.keras.layers
    model = tde.keras.Sequential([
        l.Reshape(input_shape=(28 * 28,), target_shape=(28, 28, 1)),
        l.Conv2D(filters=6, kernel_size=3, padding="same", use_bias=False),
        l.BatchNormalization(scale=False, center=True),   # no bias necessary before batch norm
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
        l.Dropout(0.5),                                    # Dropout on dense layer only
        l.Dense(10, activation="softmax"),
    ])
    optimizer = tde.train.GradientDescentOptimizer(learning_rate=learning_rate)
    model.compile(optimizer=optimizer, loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    tde.keras.backend.set_learning_phase(True)            # Q4: reproduced faithfully
    model.summary()
    return tde.keras.estimator.model_to_estimator(keras_model=model, model_dir=model_dir, config=config)


def input_fn(features, labels, batch_size, mode):
    inputs = features if labels is None else (features, labels)
    dataset = tde.data.Dataset.from_tensor_slices(inputs)
    if mode == tde.estimator.ModeKeys.TRAIN:
        dataset = dataset.shuffle(1000).repeat().batch(batch_size)
        dataset = dataset.prefetch(100)
    if mode in (tde.estimator.ModeKeys.EVAL, tde.estimator.ModeKeys.PREDICT):
        dataset = dataset.batch(batch_size)
    return dataset


def serving_input_fn():
    """The serving signature: a raw float32 [None, 784] image vector."""
    feature_placeholder = tde.compat.v1.placeholder(tde.float32, [None, 28 * 28])
    features = feature_placeholder
    return tde.estimator.export.TensorServingInputReceiver(features, feature_placeholder)


def _get_session_config_from_env_var():
    """Session device filters from TF_CONFIG (MKD:165-189)."""
    tf_config = json.loads(os.environ.get("TF_CONFIG", "{}"))
    if tf_config and "task" in tf_config and "type" in tf_config["task"] and "index" in tf_config["task"]:
        if tf_config["task"]["type"] == "master":
            return tde.ConfigProto(device_filters=["/job:ps", "/job:master"])
        elif tf_config["task"]["type"] == "worker":
            return tde.ConfigProto(device_filters=["/job:ps", "/job:worker/task:%d" % tf_config["task"]["index"]])
    return None


def train_and_evaluate(args):
    (train_images, train_labels), (test_images, test_labels) = tde.keras.datasets.mnist.load_data()
    train_images = (train_images / 255.0).astype(np.float32).reshape(-1, 784)
    test_images = (test_images / 255.0).astype(np.float32).reshape(-1, 784)
    train_labels = np.asarray(train_labels).astype("int").reshape((-1, 1))
    test_labels = np.asarray(test_labels).astype("int").reshape((-1, 1))

    if args.max_steps:
        train_steps = args.max_steps
    elif args.reference_steps:
        train_steps = math.ceil(len(train_images) / args.batch_size)
    else:
        train_steps = math.ceil(args.num_epochs * len(train_images) / args.batch_size)

    job_type, job_index = "chief", 0
    if tde.distribute.cluster.translate_launcher_env():
        job_index = int(os.environ["TASK_INDEX"])
        job_type = os.environ["JOB_NAME"]

    # hook = tde.estimator.ProfilerHook(save_steps=100, output_dir=args.working_dir, show_memory=True)
    run_config = tde.estimator.RunConfig(
        experimental_distribute=tde.contrib.distribute.DistributeConfig(
            train_distribute=tde.contrib.distribute.ParameterServerStrategy(),
            eval_distribute=tde.contrib.distribute.MirroredStrategy()),
        session_config=_get_session_config_from_env_var(),
        model_dir=args.working_dir,
        save_summary_steps=100,
        log_step_count_steps=100,
        save_checkpoints_steps=500)
    estimator = create_model(model_dir=args.working_dir, config=run_config, learning_rate=args.learning_rate)
    train_spec = tde.estimator.TrainSpec(
        input_fn=lambda: input_fn(train_images, train_labels, args.batch_size, mode=tde.estimator.ModeKeys.TRAIN),
        max_steps=train_steps, hooks=tde.utils.flags.profiler_hooks(args, args.working_dir))
    exporter = tde.estimator.FinalExporter("exporter", serving_input_fn)
    eval_spec = tde.estimator.EvalSpec(
        input_fn=lambda: input_fn(test_images, test_labels, args.batch_size, mode=tde.estimator.ModeKeys.EVAL),
        steps=args.eval_steps, name="mnist-eval", exporters=[exporter], start_delay_secs=10, throttle_secs=10)

    # TensorBoard on the chief / first worker (the reference's `is 0` check crashed in local mode, Q1)
    tb = None
    if not args.no_tensorboard and ((job_type == "worker" and job_index == 0) or job_type in ("chief", "master")):
        os.makedirs(args.working_dir, exist_ok=True)
        tb = tde.start_tensorboard(args.working_dir)
    result = tde.estimator.train_and_evaluate(estimator, train_spec, eval_spec)
    if hasattr(tb, "shutdown"):
        tb.shutdown()
    return result


if __name__ == "__main__":
    args = tde.utils.flags.apply_framework_flags(get_args())
    logger = tde.get_logger()
    logger.setLevel(args.verbosity)
    out = train_and_evaluate(args)
    if out and out[0]:
        print("eval:", out[0], "exports:", out[1])
