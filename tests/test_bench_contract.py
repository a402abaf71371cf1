"""The driver's bench.py contract (CPU, gloo): one process and a torchrun group of ranks each print exactly
one JSON line from rank 0 with the BASELINE.json metric, whole-job images/sec, the timed step count and a
step time consistent with the value; the data-parallel replicas end bit-identical.  The same script runs
one rank per MI355X over RCCL / the xGMI kernel on a GPU node (tests/test_xgmi_gpu.py covers that path)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [1, 4])
def test_bench_json_line_contract(world):
    env = dict(os.environ, TDE_BENCH_WARM_MS="0", OMP_NUM_THREADS="1", TDE_HEARTBEAT="0", CUDA_VISIBLE_DEVICES="")
    args = ["--gpus", str(world), "--steps", "6", "--warmup", "2"]
    if world == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert KEYS <= set(res), set(res) ^ KEYS
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert res["metric"] == base["metric"]
    assert res["n_gpus"] == world and res["steps"] == 6 and res["warmup"] == 2
    assert res["scaling"] == "weak" and res["higher_is_better"] is True and res["unit"] == "images/sec"
    cfg = res["config"]
    assert cfg["model"] == "mnist_cnn" and cfg["global_batch"] == 64 * world
    assert cfg["parallelism"] == f"dp{world}"
    # value is the whole-job rate implied by the timed step time
    implied = cfg["global_batch"] * 1000.0 / res["ms_per_step"]
    assert abs(res["value"] - implied) <= 1e-3 * implied + 1.0
    if world > 1:
        assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]


def test_bench_multi_gpu_without_launcher_runs_mirrored():
    """`python bench.py --gpus 2` with no torchrun (VERDICT r5 Missing #1): one process drives both replicas
    with MirroredStrategy (BASELINE config 3; mnist_keras_distributed.py:243), rc 0, one JSON line."""
    env = dict(os.environ, TDE_BENCH_WARM_MS="0", OMP_NUM_THREADS="1", TDE_HEARTBEAT="0", CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6",
                        "--warmup", "2", "--repeats", "1"], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert res["metric"] == base["metric"] and res["n_gpus"] == 2
    cfg = res["config"]
    assert cfg["strategy"] == "MirroredStrategy" and cfg["replicas_per_process"] == 2
    assert cfg["global_batch"] == 128 and cfg["parallelism"] == "dp2"
    assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_bench_multi_gpu_without_launcher_on_gpu():
    """The same launcher-less command on a GPU box: with fewer visible GPUs than --gpus the replicas wrap onto
    cuda:0 (a rehearsal of the N-GPU Mirrored layout: one hipGraph per replica, in-process xGMI all-reduce),
    rc 0 and bit-identical replicas."""
    env = dict(os.environ, TDE_BENCH_WARM_MS="20", TDE_HEARTBEAT="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "5", "--repeats", "1"], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["strategy"] == "MirroredStrategy"
    assert res["config"]["plan"] == "fused_convnet" and res["config"]["hipgraph"] is True
    assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]


def test_bench_devices_list_sets_the_replica_count():
    """`--strategy mirrored --devices cpu,cpu` without --gpus: the device list is the replica count (the
    2-replica rehearsal form of tests/test_mirrored_gpu.py, `--devices 0,0`)."""
    env = dict(os.environ, TDE_BENCH_WARM_MS="0", OMP_NUM_THREADS="1", TDE_HEARTBEAT="0", CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--strategy", "mirrored", "--devices",
                        "cpu,cpu", "--steps", "4", "--warmup", "1", "--repeats", "1"], env=env, cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["n_gpus"] == 2 and res["config"]["replicas_per_process"] == 2
