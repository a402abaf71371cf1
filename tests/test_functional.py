"""T1 for the functional API (keras.Input / Model(inputs, outputs) / Add) and the ResNet family, plus
the reference script's CLI defaults (mnist_keras_distributed.py:33-65)."""
import importlib.util
import sys
from pathlib import Path

import numpy as np
import pytest

import tensorflow_distributed_example_amd as tde

REPO = Path(__file__).resolve().parents[1]


def test_resnet18_params_and_graph():
    m = tde.zoo.resnet18()
    m.build()
    assert m.count_params() == 11_699_112
    assert m.output_shape == (None, 1000)
    assert isinstance(m, tde.keras.Model)
    adds = [l for l in m.layers if isinstance(l, tde.keras.layers.Add)]
    assert len(adds) == 8
    lines = []
    m.summary(print_fn=lines.append)
    text = "\n".join(lines)
    assert "Connected to" in text and "Total params: 11,699,112" in text
    # TF-'SAME' stem padding at 224/k7/s2 is asymmetric (2, 3)
    stem = m.layers[0]
    assert stem.pads((224, 224, 3)) == ((2, 3), (2, 3))


def test_functional_config_roundtrip_and_forward():
    inp = tde.keras.Input((8, 8, 3))
    x = tde.keras.layers.Conv2D(4, 3, padding="same", use_bias=False)(inp)
    y = tde.keras.layers.BatchNormalization()(x)
    s = tde.keras.layers.Conv2D(4, 1)(inp)
    z = tde.keras.layers.Add()([y, s])
    z = tde.keras.layers.Activation("relu")(z)
    z = tde.keras.layers.GlobalAveragePooling2D()(z)
    out = tde.keras.layers.Dense(3)(z)
    m = tde.keras.Model(inputs=inp, outputs=out)
    m.build()
    x_in = np.random.default_rng(0).random((5, 8, 8, 3), dtype=np.float32)
    ref = np.asarray(m(x_in))
    cfg = m.get_config()
    m2 = type(m).from_config(cfg, keep_names=False)
    m2.build()
    m2.set_weights(m.get_weights())
    np.testing.assert_allclose(np.asarray(m2(x_in)), ref, rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        tde.keras.layers.Add()([tde.keras.Input((2,)), tde.keras.Input((3,))])


def test_functional_resnet_trains_on_cpu():
    tde.backend.set_random_seed(3)
    m = tde.zoo.resnet((1, 1), (8, 16), input_shape=(16, 16, 3), classes=4)
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.05),
              metrics=["accuracy"])
    rng = np.random.default_rng(1)
    x = rng.standard_normal((64, 16, 16, 3)).astype(np.float32)
    y = (x[:, :, :, 0].mean((1, 2)) > 0).astype(np.int64) + 2 * (x[:, :, :, 1].mean((1, 2)) > 0)
    h = m.fit(x, y, batch_size=16, epochs=6, verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]


def test_functional_export_and_load(tmp_path):
    m = tde.zoo.resnet((1,), (8,), input_shape=(12, 12, 3), classes=5)
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.01))
    m.build()
    from tensorflow_distributed_example_amd.io import export as EX
    path = EX.export_saved_model(m, str(tmp_path / "exp"), lambda: EX.TensorServingInputReceiver(
        tde.compat.v1.placeholder(tde.float32, [None, 12, 12, 3]), None))
    loaded = tde.saved_model.load(path)
    x = np.random.default_rng(2).random((3, 12, 12, 3), dtype=np.float32)
    out = next(iter(loaded(x).values()))
    np.testing.assert_allclose(out, m.predict(x), rtol=1e-5, atol=1e-6)


def test_mnist_keras_distributed_cli_defaults(monkeypatch):
    spec = importlib.util.spec_from_file_location("mkd", REPO / "examples" / "mnist_keras_distributed.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.setattr(sys, "argv", ["mkd", "--working-dir", "/tmp/x", "--unknown-launcher-flag", "1"])
    args = mod.get_args()
    assert args.working_dir == "/tmp/x" and args.num_epochs == 5 and args.batch_size == 128
    assert args.learning_rate == 0.01 and args.verbosity == "INFO"
