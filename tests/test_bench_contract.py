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
