#!/usr/bin/env python
"""End-to-end ``Model.fit`` throughput with the host input pipeline in the loop (1 MI355X).

``bench.py`` feeds device-resident synthetic batches (the driver's metric); this measures what a
user of ``distributed_with_keras.py`` sees: ``from_tensor_slices -> map(scale) -> cache ->
shuffle(10000) -> batch(128)`` (DWK:18-30,54) on a 60000-image synthetic MNIST, the native
shuffle/gather engine (csrc/data/pipeline.cpp), S-step staging into pinned buffers and the
captured training step.  Prints one JSON line per configuration.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1200)
    ap.add_argument("--spe", type=int, default=16, help="steps_per_execution")
    ap.add_argument("--prefetch", type=int, default=4)
    a = ap.parse_args()
    import tensorflow_distributed_example_amd as tde
    D = tde.data.Dataset
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (60000, 28, 28, 1), dtype=np.uint8)
    y = rng.integers(0, 10, 60000).astype(np.int64)

    def scale(img, lab):
        return img.astype(np.float32) / 255.0, lab

    for native, device in (("1", "1"), ("1", "0"), ("0", "0")):
        os.environ["TDE_NATIVE_DATA"] = native
        os.environ["TDE_DEVICE_DATA"] = device
        from tensorflow_distributed_example_amd.data import dataset as DS
        DS._HOST.clear()
        tde.backend.set_random_seed(0)
        m = tde.zoo.mnist_cnn()
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tde.optimizers.SGD(0.001), metrics=["accuracy"], steps_per_execution=a.spe)
        ds = D.from_tensor_slices((x, y)).map(scale).cache().shuffle(10000).repeat().batch(128)
        if a.prefetch:
            ds = ds.prefetch(a.prefetch)
        m.fit(ds, epochs=1, steps_per_epoch=4 * a.spe, verbose=0)      # warm-up: capture + cache fill
        t = time.perf_counter()
        m.fit(ds, epochs=1, steps_per_epoch=a.steps, verbose=0)
        dt = time.perf_counter() - t
        print(json.dumps({"what": "fit() img/s, DWK pipeline", "native_pipeline": native == "1",
                          "device_feed": bool(m._device_feed),
                          "img_per_s": round(128 * a.steps / dt), "ms_per_step": round(dt / a.steps * 1e3, 4),
                          "steps_per_execution": a.spe, "prefetch": a.prefetch}), flush=True)


if __name__ == "__main__":
    main()
