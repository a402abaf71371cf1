"""T6 end-to-end: the three in-spirit reference scripts (examples/) on synthetic MNIST, on CPU
(the same scripts run on the MI355X in tests/test_examples_gpu.py).

* distributed_with_keras.py   — MultiWorkerMirroredStrategy + compile/fit (1 and 2 workers)
* mnist_keras_distributed.py  — Estimator train_and_evaluate, local mode and a localhost
                                ps/master/worker cluster driven by CLUSTER_SPEC/TASK_INDEX/JOB_NAME
* tf2_mnist_distributed.py    — Estimator under ParameterServerStrategy (local mode)
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _env(**extra):
    env = dict(os.environ, PYTHONPATH=str(REPO), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="2", **extra)
    for k in ("TF_CONFIG", "CLUSTER_SPEC", "TASK_INDEX", "JOB_NAME", "TDE_FAULT"):
        if k not in extra:
            env.pop(k, None)
    return env


def _run(args, env, timeout=300, cwd=None):
    p = subprocess.run([sys.executable, *args], env=env, capture_output=True, text=True, timeout=timeout,
                       cwd=cwd or str(REPO))
    return p.returncode, p.stdout + p.stderr


def test_distributed_with_keras_single_worker():
    rc, out = _run(["examples/distributed_with_keras.py", "--epochs", "2", "--steps-per-epoch", "3", "--verbose", "0"],
                   _env())
    assert rc == 0, out
    assert "loss" in out


def test_distributed_with_keras_two_workers(tmp_path):
    rc, out = _run(["-m", "tensorflow_distributed_example_amd.launch", "--workers", "2", "--timeout", "240",
                    "examples/distributed_with_keras.py", "--epochs", "2", "--steps-per-epoch", "3", "--verbose", "0"],
                   _env(TDE_HEARTBEAT_TIMEOUT="20"))
    assert rc == 0, out
    assert "[worker:0]" in out and "[worker:1]" in out


def test_mnist_keras_distributed_local(tmp_path):
    wd = tmp_path / "wd"
    rc, out = _run(["examples/mnist_keras_distributed.py", "--working-dir", str(wd), "--max-steps", "30",
                    "--eval-steps", "4", "--no-tensorboard", "--verbosity", "WARN"], _env())
    assert rc == 0, out
    # checkpoints with TF1 names, exported serving model, events
    assert (wd / "checkpoint").exists()
    assert list(wd.glob("model.ckpt-30.index"))
    exports = list((wd / "export" / "exporter").glob("*/saved_model.json"))
    assert exports, out
    spec = json.loads(exports[0].read_text())
    assert spec["signatures"]["serving_default"]["inputs"]["input"]["shape"] == [None, 784]
    assert list(wd.glob("events.out.tfevents.*"))
    # auto-resume: a second run with a larger max_steps continues from step 30
    rc, out = _run(["examples/mnist_keras_distributed.py", "--working-dir", str(wd), "--max-steps", "40",
                    "--eval-steps", "2", "--no-tensorboard", "--verbosity", "WARN"], _env())
    assert rc == 0, out
    assert list(wd.glob("model.ckpt-40.index"))


def test_mnist_keras_distributed_ps_cluster(tmp_path):
    """ps + master + worker on localhost from CLUSTER_SPEC/TASK_INDEX/JOB_NAME (mnist_keras_distributed.py:221-233):
    async PS training stops at exactly max_steps global updates."""
    wd = tmp_path / "wd"
    rc, out = _run(["-m", "tensorflow_distributed_example_amd.launch", "--ps", "1", "--master", "1", "--workers", "1",
                    "--launcher-env", "--timeout", "280", "examples/mnist_keras_distributed.py", "--working-dir",
                    str(wd), "--max-steps", "40", "--eval-steps", "2", "--no-tensorboard"], _env(), timeout=300)
    assert rc == 0, out
    assert "global_step = 40" in out, out
    assert "global_step = 41" not in out
    assert list(wd.glob("model.ckpt-40.index"))


def test_tf2_mnist_distributed_local(tmp_path):
    rc, out = _run(["examples/tf2_mnist_distributed.py"],
                   _env(TDE_MODEL_DIR=str(tmp_path / "mode"), TDE_MAX_STEPS="20"))
    assert rc == 0, out
    assert list((tmp_path / "mode").glob("model.ckpt-20.index")), out


def test_framework_flags_devices_dtype_synthetic_profile(tmp_path, monkeypatch):
    """SURVEY.md §5.6 framework flags: --devices / --dtype / --synthetic set the global state strategies and
    loaders read; --profile-steps yields a ProfilerCallback (Keras) that writes Chrome-trace timelines."""
    import argparse

    import numpy as np

    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd import backend as Kb
    from tensorflow_distributed_example_amd.utils import flags as fw
    monkeypatch.delenv("TDE_SYNTHETIC_MNIST", raising=False)
    ap = fw.add_framework_flags(argparse.ArgumentParser())
    args = ap.parse_args(["--devices", "cpu,cpu", "--dtype", "fp32", "--synthetic", "--profile-steps", "2"])
    try:
        fw.apply_framework_flags(args)
        assert Kb.global_policy().name == "float32"
        assert tde.keras.datasets.mnist.load_data()[0][0].shape == (60000, 28, 28)
        strategy = tde.distribute.MirroredStrategy()
        assert strategy.num_replicas_in_sync == 2 and all(d.type == "cpu" for d in strategy.local_devices)
        cbs = fw.profiler_callbacks(args, str(tmp_path))
        with strategy.scope():
            m = tde.zoo.mnist_cnn()
            m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
        x = np.random.default_rng(0).random((8 * 16, 28, 28, 1), dtype=np.float32)
        y = np.random.default_rng(1).integers(0, 10, 8 * 16)
        m.fit(x, y, batch_size=16, epochs=1, verbose=0, callbacks=cbs)
        assert cbs[0].written and all((tmp_path / p.split("/")[-1]).exists() for p in cbs[0].written)
        assert len(fw.profiler_hooks(args, str(tmp_path))) == 1
    finally:
        Kb.set_default_devices(None)
        Kb.set_global_policy(None)
        monkeypatch.delenv("TDE_SYNTHETIC_MNIST", raising=False)
        monkeypatch.delenv("TDE_EXECUTOR", raising=False)
