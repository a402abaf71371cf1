"""T6 on the MI355X: the three in-spirit reference scripts end to end on the GPU (HIP plans, hipGraph
steps, bf16), synthetic MNIST.  One GPU: multi-worker RCCL cliques need one GPU per rank, so the
2-worker MWMS run stays in the CPU suite (tests/test_examples.py)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _env(**extra):
    env = dict(os.environ, PYTHONPATH=str(REPO), **extra)
    for k in ("TF_CONFIG", "CLUSTER_SPEC", "TASK_INDEX", "JOB_NAME", "TDE_FAULT"):
        if k not in extra:
            env.pop(k, None)
    return env


def _run(args, env, timeout=300):
    p = subprocess.run([sys.executable, *args], env=env, capture_output=True, text=True, timeout=timeout,
                       cwd=str(REPO))
    return p.returncode, p.stdout + p.stderr


def test_distributed_with_keras_gpu():
    rc, out = _run(["examples/distributed_with_keras.py", "--epochs", "3", "--steps-per-epoch", "5", "--verbose", "0"],
                   _env())
    assert rc == 0, out


def test_mnist_keras_distributed_gpu(tmp_path):
    wd = tmp_path / "wd"
    rc, out = _run(["examples/mnist_keras_distributed.py", "--working-dir", str(wd), "--max-steps", "60",
                    "--eval-steps", "4", "--no-tensorboard", "--verbosity", "WARN"], _env())
    assert rc == 0, out
    assert list(wd.glob("model.ckpt-60.index"))
    spec = json.loads(next((wd / "export" / "exporter").glob("*/saved_model.json")).read_text())
    assert spec["signatures"]["serving_default"]["inputs"]["input"]["shape"] == [None, 784]


def test_mnist_keras_distributed_ps_cluster_gpu(tmp_path):
    wd = tmp_path / "wd"
    rc, out = _run(["-m", "tensorflow_distributed_example_amd.launch", "--ps", "1", "--master", "1", "--workers", "1",
                    "--launcher-env", "--timeout", "280", "examples/mnist_keras_distributed.py", "--working-dir",
                    str(wd), "--max-steps", "40", "--eval-steps", "2", "--no-tensorboard"], _env(), timeout=300)
    assert rc == 0, out
    assert "global_step = 40" in out, out


def test_tf2_mnist_distributed_gpu(tmp_path):
    rc, out = _run(["examples/tf2_mnist_distributed.py"], _env(TDE_MODEL_DIR=str(tmp_path / "mode"), TDE_MAX_STEPS="30"))
    assert rc == 0, out
    assert list((tmp_path / "mode").glob("model.ckpt-30.index")), out
