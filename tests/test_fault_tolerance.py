"""T5: failure detection, fault injection and checkpoint-based recovery for multi-worker training
 on localhost CPU workers (gloo control/data plane; the RCCL abort path
is the same watchdog with ``comm.abort()``)."""
import os
import subprocess
import sys
import textwrap
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]

WORKER = textwrap.dedent("""
    import sys
    import numpy as np
    import tensorflow_distributed_example_amd as tde
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        m = tde.zoo.mnist_cnn()
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"])
    rng = np.random.default_rng(0)
    x = rng.random((64 * 20, 28, 28, 1), dtype=np.float32)
    y = rng.integers(0, 10, 64 * 20)
    ds = tde.data.Dataset.from_tensor_slices((x, y)).batch(64)
    h = m.fit(ds, epochs=4, steps_per_epoch=5, verbose=0,
              callbacks=[tde.keras.callbacks.BackupAndRestore(sys.argv[1])])
    print("RESULT epochs=%d iterations=%d" % (len(h.history["loss"]), m.optimizer.iterations), flush=True)
""")


def _launch(tmp_path, env_extra, timeout=180):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ, PYTHONPATH=str(REPO), TDE_HEARTBEAT_TIMEOUT="3", **env_extra)
    env.pop("TDE_FAULT", None) if "TDE_FAULT" not in env_extra else None
    t0 = time.time()
    p = subprocess.run([sys.executable, "-m", "tensorflow_distributed_example_amd.launch", "--workers", "2",
                        str(script), str(tmp_path / "backup")], env=env, capture_output=True, text=True,
                       timeout=timeout, cwd=str(tmp_path))
    return p.returncode, p.stdout + p.stderr, time.time() - t0


def test_fault_parse_and_match(monkeypatch):
    from tensorflow_distributed_example_amd.utils import fault
    cfg = fault.parse("task=worker:1, step=7 ,kind=hang")
    assert cfg == {"task": "worker:1", "step": "7", "kind": "hang"}
    monkeypatch.setenv("TF_CONFIG", '{"cluster": {"worker": ["a:1", "b:2"]}, "task": {"type": "worker", "index": 1}}')
    assert fault.matches(cfg)
    assert not fault.matches({"task": "worker:0"})
    monkeypatch.setenv("TDE_FAULT", "task=worker:1,step=3,kind=raise")
    fault.maybe_inject(2)
    with pytest.raises(fault.InjectedFault):
        fault.maybe_inject(3)
    fault._fired = False


def test_worker_crash_then_resume_from_backup(tmp_path):
    rc, out, _ = _launch(tmp_path, {"TDE_FAULT": "task=worker:1,step=12,kind=exit"})
    assert rc == 13, out
    assert "injecting 'exit' at step 12" in out
    backups = list((tmp_path / "backup").glob("backup-*.index"))
    assert [b.name for b in backups] == ["backup-10.index"], out       # 2 finished epochs of 5 steps
    rc, out, _ = _launch(tmp_path, {})
    assert rc == 0, out
    # the relaunch resumes at epoch 3: two more epochs, 20 optimizer steps in total
    assert out.count("RESULT epochs=2 iterations=20") == 2, out
    assert not (tmp_path / "backup").exists()                          # deleted after success


def test_hung_peer_detected_by_heartbeat_watchdog(tmp_path):
    rc, out, dt = _launch(tmp_path, {"TDE_FAULT": "task=worker:1,step=7,kind=hang"})
    assert rc == 75, out
    assert "rank1 stopped heartbeating" in out, out
    assert dt < 120


def test_health_monitor_store_protocol():
    """Heartbeats + dead-member query + done markers on the native TCP store."""
    from tensorflow_distributed_example_amd.parallel.store import TCPStore, TCPStoreServer
    srv = TCPStoreServer("127.0.0.1", 0)
    try:
        a, b = TCPStore("127.0.0.1", srv.port), TCPStore("127.0.0.1", srv.port)
        a.heartbeat("rank0")
        b.heartbeat("rank1")
        assert a.dead_members(5.0) == []
        time.sleep(0.6)
        a.heartbeat("rank0")
        assert a.dead_members(0.3) == ["rank1"]
        b.set("done/rank1", b"1")
        assert a.check("done/rank1")
    finally:
        srv.stop()
