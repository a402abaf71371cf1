#!/usr/bin/env python
"""In-spirit port of distributed_with_keras.py (reference: Keras fit under
MultiWorkerMirroredStrategy), running on the MI355X-native framework.

Same constants and flow as the reference (DWK:12-16, 18-44, 47-63):
BUFFER_SIZE=10000, BATCH_SIZE=64 per worker, NUM_WORKERS=2, GLOBAL_BATCH_SIZE=128,
the strategy is created first (it reads TF_CONFIG), datasets and the model are
built inside strategy.scope(), AutoShardPolicy.OFF, fit(epochs=3, steps_per_epoch=5).

Run one process per worker, e.g. two workers on this host:
    python -m tensorflow_distributed_example_amd.launch --workers 2 examples/distributed_with_keras.py
or as a single local worker (TF_CONFIG unset): python examples/distributed_with_keras.py
Data: MNIST via tde.tfds (local mnist.npz if present, else synthetic MNIST-shaped data).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import tensorflow_distributed_example_amd as tde  # noqa: E402

from tensorflow_distributed_example_amd.utils import flags as fw  # noqa: E402

# framework flags (--devices/--dtype/--synthetic/--profile-steps) take effect before the
# strategy below is built, as the reference builds it at import time (DWK:16)
FW_ARGS = fw.apply_framework_flags(fw.add_framework_flags(argparse.ArgumentParser(add_help=False))
                                   .parse_known_args()[0])

tfds = tde.tfds
tfds.disable_progress_bar()

BUFFER_SIZE = 10000
BATCH_SIZE = 64
NUM_WORKERS = 2                     # reference hard-codes this (Q7) ...
strategy = tde.distribute.experimental.MultiWorkerMirroredStrategy()
if strategy.num_workers > 1:        # ... we derive it from the cluster when one is configured
    NUM_WORKERS = strategy.num_workers
GLOBAL_BATCH_SIZE = BATCH_SIZE * NUM_WORKERS


def make_datasets_unbatched():
    # Scaling MNIST data from (0, 255] to (0., 1.]
    def scale(image, label):
        image = image.astype("float32")
        image /= 255
        return image, label

    datasets, info = tfds.load(name="mnist", data_dir="/tmp/data", with_info=True, as_supervised=True)
    return datasets["train"].map(scale).cache().shuffle(BUFFER_SIZE)


def build_and_compile_cnn_model():
    model = tde.keras.Sequential([
        tde.keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        tde.keras.layers.MaxPooling2D(),
        tde.keras.layers.Flatten(),
        tde.keras.layers.Dense(64, activation="relu"),
        tde.keras.layers.Dense(10),
    ])
    model.compile(
        loss=tde.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
        optimizer=tde.keras.optimizers.SGD(learning_rate=0.001),
        metrics=["accuracy"])
    return model


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--steps-per-epoch", type=int, default=5)
    ap.add_argument("--verbose", type=int, default=1)
    ap.add_argument("--profile-dir", default="/tmp/dwk_profile", help="where --profile-steps timelines go")
    fw.add_framework_flags(ap)
    args, _ = ap.parse_known_args(argv)
    with strategy.scope():
        # Creation of dataset, and model building/compiling need to be within `strategy.scope()`.
        train_datasets = make_datasets_unbatched().batch(GLOBAL_BATCH_SIZE)
        options = tde.data.Options()
        options.experimental_distribute.auto_shard_policy = tde.data.experimental.AutoShardPolicy.OFF
        train_datasets_no_auto_shard = train_datasets.with_options(options)
        multi_worker_model = build_and_compile_cnn_model()
    # Keras' `model.fit()` trains the model with specified number of epochs and number of steps per epoch.
    history = multi_worker_model.fit(x=train_datasets_no_auto_shard, epochs=args.epochs,
                                     steps_per_epoch=args.steps_per_epoch,
                                     verbose=args.verbose if strategy.is_chief else 0,
                                     callbacks=fw.profiler_callbacks(args, args.profile_dir))
    return history


if __name__ == "__main__":
    h = main()
    if strategy.is_chief:
        print("history:", {k: [round(v, 4) for v in vs] for k, vs in h.history.items()})
    print(f"worker {strategy.worker_index}/{strategy.num_workers} done: {strategy.num_replicas_in_sync} replicas "
          f"in sync, {len(h.history.get('loss', []))} epochs", flush=True)
