"""Run-to-run spread of fit() weights: device feed vs host staging (diagnostic for tests/test_plan_gpu.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorflow_distributed_example_amd as tde  # noqa: E402

rng = np.random.default_rng(4)
x = rng.random((64 * 7 + 23, 28, 28, 1), dtype=np.float32)
y = rng.integers(0, 10, size=len(x))


def run(zoo, dev, w0=None, shuffle=True):
    os.environ["TDE_DEVICE_DATA"] = dev
    tde.backend.clear_session()
    tde.backend.set_random_seed(9)
    m = getattr(tde.zoo, zoo)()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tde.optimizers.SGD(float(os.environ.get("LR", "0.05")), momentum=float(os.environ.get("MOM", "0.9"))), metrics=["accuracy"], steps_per_execution=3)
    if w0 is not None:
        m.set_weights(w0)
    w = m.get_weights()
    ds = tde.data.Dataset.from_tensor_slices((x, y)).cache()
    if shuffle:
        ds = ds.shuffle(100, seed=11)
    ds = ds.repeat(2).batch(64)
    m.fit(ds, epochs=2, verbose=0)
    return m.get_weights(), w


for zoo in ("mnist_cnn", "lenet5"):
    a, w0 = run(zoo, "0")
    for tag, dev in (("host-host", "0"), ("dev-host", "1"), ("dev-host", "1")):
        b, _ = run(zoo, dev, w0)
        rels = [float(np.linalg.norm((p - w) - (q - w)) / (np.linalg.norm(q - w) + 1e-12)) for p, q, w in zip(b, a, w0)]
        print(zoo, tag, ["%.2e" % r for r in rels], flush=True)
