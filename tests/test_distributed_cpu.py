"""T3/T4 on CPU: MirroredStrategy (in-process replicas) and
MultiWorkerMirroredStrategy (2 processes over the native control plane: the chief's C++ TCP store,
torch.distributed never initialised) — the DP invariants: replicas stay identical, and R replicas at
global batch G match 1 replica at G."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import tensorflow_distributed_example_amd as tde

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=256, seed=0):
    rng = np.random.default_rng(seed)
    return rng.random((n, 28, 28, 1), dtype=np.float32), rng.integers(0, 10, size=n)


def _train(strategy, x, y, w0, gb=64, epochs=1):
    with strategy.scope():
        m = tde.zoo.mnist_cnn()
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.1),
                  metrics=["accuracy"])
    m.set_weights(w0)
    ds = tde.data.Dataset.from_tensor_slices((x, y)).batch(gb)
    h = m.fit(ds, epochs=epochs, verbose=0)
    return m, h


def test_mirrored_two_cpu_replicas_match_single():
    x, y = _data()
    w0 = tde.zoo.mnist_cnn().get_weights()
    tde.backend.clear_session()
    m1, h1 = _train(tde.distribute.OneDeviceStrategy("cpu"), x, y, w0)
    tde.backend.clear_session()
    st = tde.distribute.MirroredStrategy(devices=["/cpu:0", "/cpu:0"])
    assert st.num_replicas_in_sync == 2
    m2, h2 = _train(st, x, y, w0)
    stores = m2._replica_stores(st)
    assert len(stores) == 2
    assert np.array_equal(stores[0].w.numpy(), stores[1].w.numpy())   # replicas identical
    for a, b in zip(m1.get_weights(), m2.get_weights()):
        assert np.allclose(a, b, atol=2e-5, rtol=1e-4)
    assert abs(h1.history["loss"][0] - h2.history["loss"][0]) < 1e-4


WORKER = textwrap.dedent("""
    import json, os, sys, numpy as np
    sys.path.insert(0, {root!r})
    import tensorflow_distributed_example_amd as tde
    tde.backend.set_random_seed(0)
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    rng = np.random.default_rng(0)
    x = rng.random((256, 28, 28, 1), dtype=np.float32); y = rng.integers(0, 10, size=256)
    with strategy.scope():
        m = tde.zoo.mnist_cnn()
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tde.optimizers.SGD(0.1), metrics=['accuracy'])
    w0 = np.load({w0!r}, allow_pickle=False)
    m.set_weights([w0['arr_%d' % i] for i in range(6)])
    opts = tde.data.Options(); opts.experimental_distribute.auto_shard_policy = tde.data.AutoShardPolicy.OFF
    ds = tde.data.Dataset.from_tensor_slices((x, y)).batch(64).with_options(opts)
    h = m.fit(ds, epochs=1, verbose=0)
    out = {{"rank": strategy.worker_index, "replicas": strategy.num_replicas_in_sync,
           "loss": h.history["loss"][0], "w": [float(np.abs(a).sum()) for a in m.get_weights()]}}
    np.savez({outp!r} + str(strategy.worker_index) + ".npz", *m.get_weights())
    import torch.distributed as dist
    out["torch_dist"] = dist.is_initialized()
    out["comm"] = type(strategy.comm).__name__
    print("RESULT" + json.dumps(out), flush=True)
""")


def test_multi_worker_mirrored_native_control_plane_two_processes(tmp_path):
    x, y = _data()
    w0 = tde.zoo.mnist_cnn().get_weights()
    np.savez(tmp_path / "w0.npz", *w0)
    port = _free_port()
    cluster = {"worker": [f"127.0.0.1:{port}", f"127.0.0.1:{_free_port()}"]}
    script = WORKER.format(root=ROOT, w0=str(tmp_path / "w0.npz"), outp=str(tmp_path / "out"))
    procs = []
    for i in range(2):
        env = dict(os.environ, TF_CONFIG=json.dumps({"cluster": cluster, "task": {"type": "worker", "index": i}}),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o
        outs.append(json.loads(o.split("RESULT")[1].strip()))
    assert outs[0]["replicas"] == 2
    assert not any(o["torch_dist"] for o in outs) and all(o["comm"] == "StoreCommunicator" for o in outs)
    wa = np.load(tmp_path / "out0.npz")
    wb = np.load(tmp_path / "out1.npz")
    for k in wa.files:
        assert np.array_equal(wa[k], wb[k])      # workers hold identical variables
    # 2 workers x per-replica 32 at global 64, AutoShard OFF == 1 replica at global 64
    tde.backend.clear_session()
    m1, h1 = _train(tde.distribute.OneDeviceStrategy("cpu"), x, y, w0)
    for k, a in zip(wa.files, m1.get_weights()):
        assert np.allclose(wa[k], a, atol=2e-5, rtol=1e-4)
    assert abs(outs[0]["loss"] - h1.history["loss"][0]) < 1e-4


def test_replica_consistency_checker_detects_divergence():
    """all replicas bit-identical after training; a perturbed replica is reported."""
    from tensorflow_distributed_example_amd.utils import debug
    x, y = _data(128)
    w0 = tde.zoo.mnist_cnn().get_weights()
    tde.backend.clear_session()
    st = tde.distribute.MirroredStrategy(["cpu", "cpu"])
    with st.scope():
        m = tde.zoo.mnist_cnn()
        m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tde.optimizers.SGD(0.1), metrics=["accuracy"])
    m.set_weights(w0)
    ds = tde.data.Dataset.from_tensor_slices((x, y)).batch(64)
    m.fit(ds, epochs=2, verbose=0, callbacks=[tde.keras.callbacks.ReplicaConsistencyCheck(1)])
    fps = debug.check_replicas(m)
    assert len(fps) == 2 and fps[0][2] == fps[1][2]
    stores = m._stores[id(st)]
    stores[1].w.view(-1)[123] += 1e-6          # one flipped low bit is enough
    with pytest.raises(debug.ReplicaDivergence, match="replica 1"):
        debug.check_replicas(m)


def test_reverse_order_gradient_buckets_cover_bucket_exactly():
    """plan_grad_buckets: buckets tile [0, total) from the end, each is emitted only after every
    variable inside it has had its backward stage, and they respect the size target."""
    from tensorflow_distributed_example_amd.train.layerwise import plan_grad_buckets
    m = tde.zoo.resnet18()
    m.build()
    st = m._store
    names = st.names(trainable=True)
    segs = [(n, st.segments[n].offset) for n in names]
    # stages in reverse layer order, one per layer (what the layer-wise plan's backward visits)
    by_layer = {}
    for n in names:
        by_layer.setdefault(n.rsplit("/", 1)[0], []).append(n)
    stage_params = list(reversed(list(by_layer.values())))
    total = st.g.numel()
    target = 2 * 2 ** 20
    bk = plan_grad_buckets(stage_params, segs, total, target)
    assert len(bk) >= 4
    assert bk[0][2] == total and bk[-1][1] == 0
    assert all(a[1] == b[2] for a, b in zip(bk, bk[1:]))            # contiguous, descending
    assert [b[0] for b in bk] == sorted(b[0] for b in bk)             # in backward order
    done_at = {n: i for i, lst in enumerate(stage_params) for n in lst}
    for i, lo, hi in bk:
        inside = [n for n, off in segs if lo <= off < hi]
        assert inside and all(done_at[n] <= i for n in inside)
        assert hi - lo >= target or lo == 0 or any(done_at[n] == i and st.segments[n].numel >= target
                                                   for n in inside)
    # one bucket when the target exceeds the model
    assert plan_grad_buckets(stage_params, segs, total, total + 1) == [(len(stage_params) - 1, 0, total)]


AGREE = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, {root!r})
    from tensorflow_distributed_example_amd.parallel import cluster as CL, control as CP
    cp = CP.ControlPlane.for_topology(CL.worker_topology(), timeout=60)
    fail = os.environ.get("FAIL_RANK") == str(cp.rank)
    errs = cp.agree("rank %d: injected setup failure" % cp.rank if fail else None)
    uid = cp.broadcast_bytes(b"\\x01uid-bytes" if cp.rank == 0 else None)
    got = cp.all_gather_bytes(bytes([cp.rank]) * 3)
    s = cp.all_reduce_array(__import__("numpy").full(5, cp.rank + 1.0))
    cp.barrier()
    import torch.distributed as dist
    print("RESULT" + json.dumps({{"errs": errs, "uid": uid.hex(), "got": [g.hex() for g in got],
                                  "sum": s.tolist(), "keys": cp.store.num_keys(), "dist": dist.is_initialized()}}),
          flush=True)
    cp.shutdown()
""")


def test_native_control_plane_agreement_two_processes():
    """The MWMS control plane (parallel/control.py) over the chief's native store: a failure injected on ONE
    rank is seen by every rank (the rank-agreed fallback), the chief's broadcast (the ncclUniqueId path),
    all-gather and rank-ordered host reductions, and no torch.distributed group anywhere."""
    port = _free_port()
    cluster = {"worker": [f"127.0.0.1:{port}", f"127.0.0.1:{_free_port()}"]}
    script = AGREE.format(root=ROOT)
    procs = []
    for i in range(2):
        env = dict(os.environ, TF_CONFIG=json.dumps({"cluster": cluster, "task": {"type": "worker", "index": i}}),
                   FAIL_RANK="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=120)
        assert p.returncode == 0, o
        outs.append(json.loads(o.split("RESULT")[1].strip()))
    for o in outs:
        assert o["errs"] == ["rank 1: injected setup failure"], o
        assert bytes.fromhex(o["uid"]) == b"\x01uid-bytes" and o["got"] == ["000000", "010101"], o
        assert o["sum"] == [3.0] * 5 and not o["dist"], o
