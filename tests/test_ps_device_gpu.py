"""Same-node GPU data plane of ParameterServerStrategy (parallel/ps_device.py, csrc/kernels/ps_device.hip;
reference mnist_keras_distributed.py:242): the exchange kernel against exact host arithmetic, and the
Estimator's async PS training on a localhost cluster (ps + master + worker) with exact max_steps accounting."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PS_SERVER = r"""
import os, sys, threading
sys.path.insert(0, {root!r})
from tensorflow_distributed_example_amd.parallel.ps import run_ps_server
ev = threading.Event()
threading.Thread(target=lambda: (sys.stdin.read(), ev.set()), daemon=True).start()
run_ps_server("127.0.0.1:{port}", stop_event=ev, index={index})
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("nps,kind", [(1, 0), (2, 1), (2, 2)])
def test_device_plane_exchange_is_exact(nps, kind):
    """Trainer against the ps tasks' windows (variables round-robin over ``nps`` tasks, each window sized
    for its shard on request): the SGD / momentum / Nesterov update (f32 atomics, slot compare-and-swap),
    the BN moving average applied to the PS value from the recovered batch statistic, the pull and the
    counters — checked against host arithmetic over 3 steps; then the pipelined loop's ticket guard (a push
    computed under a ticket past max_steps is dropped, a live one applied)."""
    import torch

    from tensorflow_distributed_example_amd.parallel import ps as PS
    from tensorflow_distributed_example_amd.parallel import ps_device as PD
    from tensorflow_distributed_example_amd.train.params import ParamStore

    class _Spec:
        def __init__(self, name, shape, trainable):
            self.full_name, self.shape, self.trainable, self.aggregation = name, shape, trainable, "none"
            self.initializer = lambda shape, gen: np.zeros(shape, np.float32)

    ports = [_free_port() for _ in range(nps)]
    env = dict(os.environ, TDE_PS_DEVICE="1")
    srvs = [subprocess.Popen([sys.executable, "-c", PS_SERVER.format(root=ROOT, port=p, index=i)], env=env,
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            for i, p in enumerate(ports)]
    lr, mm = 0.5, 0.9
    try:
        os.environ["TDE_PS_DEVICE"] = "1"
        specs = [_Spec("d/kernel", (300, 7), True), _Spec("bn/moving_mean", (5,), False), _Spec("d/bias", (7,), True),
                 _Spec("e/kernel", (7, 3), True)]
        store = ParamStore(specs, "cuda:0")
        shapes = {n: tuple(store.segments[n].shape) for n in store.order}
        t0 = time.time()
        while True:
            try:
                client = PS.PSClient([f"127.0.0.1:{p}" for p in ports], shapes)
                break
            except ConnectionError:
                assert time.time() - t0 < 60 and all(s.poll() is None for s in srvs)
                time.sleep(0.2)
        assert len(set(client.placement.values())) == nps
        g = torch.Generator().manual_seed(0)
        w0 = torch.randn(store.w.numel(), generator=g)
        s0 = torch.rand(store.state.numel(), generator=g)
        store.w.copy_(w0.cuda())
        store.state.copy_(s0.cuda())
        session = PD.new_session()
        _, sizes = PD.layout(store, client.placement, nps, slots=kind != 0)
        PD.request_windows(client, sizes, session)
        plane = PD.DevicePlane(client, store, {"bn/moving_mean": 0.9}, lr=lr, kind=kind, momentum=mm,
                               session=session, timeout=60)
        assert len(plane.wins) == nps and not plane.initialized()
        plane.initialize(7, 7)
        assert plane.global_step() == 7 and plane.initialized()
        plane.pull()
        W, S = w0.double().clone(), s0.double().clone()
        M = torch.zeros_like(W)
        live = torch.zeros(store.w.numel())
        for n in ("d/kernel", "d/bias", "e/kernel"):
            live[store.segments[n].offset: store.segments[n].offset + store.segments[n].numel] = 1.0
        for step in range(3):
            gr = torch.randn(store.w.numel(), generator=g) * live   # the flat buffer's alignment gaps stay 0
            batch_stat = torch.rand(store.state.numel(), generator=g)
            store.g.copy_(gr.cuda())
            # what the local forward does to the moving statistic: m*pulled + (1-m)*batch
            store.state.copy_((0.9 * S + 0.1 * batch_stat.double()).float().cuda())
            gs, t = plane.step(dstep=1, dticket=2)
            gd = gr.double()
            if kind == 0:
                W = W - lr * gd
            else:
                M = mm * M - lr * gd
                W = W + (mm * M - lr * gd if kind == 2 else M)
            S = 0.9 * S + 0.1 * batch_stat.double()
            assert (gs, t) == (8 + step, 9 + 2 * step)
            # trainable elements only (the flat buffer also has alignment padding)
            for n in ("d/kernel", "d/bias", "e/kernel"):
                seg = store.segments[n]
                sl = slice(seg.offset, seg.offset + seg.numel)
                assert torch.allclose(store.w[sl].double().cpu(), W[sl], rtol=0, atol=2e-5), (step, n)
            assert torch.allclose(store.state.double().cpu(), S, rtol=0, atol=1e-6), step
            assert float(store.g.abs().max()) == 0.0
        assert plane.counter_add(1, 1) == 14 and plane.global_step() == 10
        # the pipelined loop's guard (step_async, max_steps 14): a push computed under a ticket past max_steps is
        # dropped — weights, slots and counters untouched, the gradient discarded ...
        w_before = store.w.clone()
        plane.set_claim(15)
        store.g.copy_((torch.randn(store.w.numel(), generator=g) * live).cuda())
        plane.step_async(14)
        torch.cuda.synchronize()
        assert plane.observed() == (10, 15) and plane.global_step() == 10 and plane.tickets() == 14
        assert torch.equal(store.w, w_before) and float(store.g.abs().max()) == 0.0
        # ... and one computed under a live ticket is applied and claims the next ticket
        plane.set_claim(14)
        gr = torch.randn(store.w.numel(), generator=g) * live
        store.g.copy_(gr.cuda())
        store.state.copy_(S.float().cuda())
        plane.step_async(14)
        torch.cuda.synchronize()
        gd = gr.double()
        if kind == 0:
            W = W - lr * gd
        else:
            M = mm * M - lr * gd
            W = W + (mm * M - lr * gd if kind == 2 else M)
        assert plane.observed() == (11, 15) and plane.global_step() == 11
        for n in ("d/kernel", "d/bias", "e/kernel"):
            seg = store.segments[n]
            sl = slice(seg.offset, seg.offset + seg.numel)
            assert torch.allclose(store.w[sl].double().cpu(), W[sl], rtol=0, atol=2e-5), ("live guard", n)
        plane.close()
        client.close()
    finally:
        os.environ.pop("TDE_PS_DEVICE", None)
        for srv in srvs:
            try:
                srv.stdin.close()
            except OSError:
                pass
            try:
                srv.wait(20)
            except subprocess.TimeoutExpired:
                srv.kill()
                srv.wait()


@pytest.mark.parametrize("plane,nps,momentum", [("device", 1, 0.0), ("tcp", 1, 0.0), ("device", 2, 0.9),
                                                 ("tcp", 2, 0.9)])
def test_ps_estimator_two_trainers_exact_max_steps(plane, nps, momentum):
    """ps x nps + master + worker on localhost (all on cuda:0): async Estimator training of Model B stops at
    EXACTLY max_steps global updates (step tickets), on the device data plane (every ps task serving its
    shard's window, momentum slots in the windows) and on the TCP plane."""
    env = dict(os.environ, OMP_NUM_THREADS="2", TDE_HEARTBEAT="0")
    if plane == "device":
        env["TDE_PS_DEVICE"] = "1"
    cmd = [sys.executable, "-m", "tensorflow_distributed_example_amd.launch", "--ps", str(nps), "--master", "1",
           "--workers", "1", "--timeout", "150", os.path.join(ROOT, "bench", "ps_throughput.py"), "--max-steps", "800",
           "--warm", "100", "--momentum", str(momentum)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-4000:]
    # the launcher prefixes each task's lines with "[task:index] "
    lines = [l[l.index("{"):] for l in r.stdout.splitlines() if '{"metric"' in l]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    print(res)
    assert res["data_plane"] == plane and res["trainers"] == 2 and res["ps_tasks"] == nps, res
    assert res["momentum"] == momentum, res
    assert res["final_global_step"] == 800, res
    assert res["value"] > 0


def test_ps_estimator_second_session_follows_its_own_chief():
    """Two consecutive train() sessions against the same ps tasks on the device plane: the chief
    clears its plane record and the windows' initialised counter at session end, so the worker of session 2
    waits for session 2's chief instead of claiming session 1's tickets; both sessions end at exactly their
    max_steps."""
    env = dict(os.environ, OMP_NUM_THREADS="2", TDE_HEARTBEAT="0", TDE_PS_DEVICE="1")
    cmd = [sys.executable, "-m", "tensorflow_distributed_example_amd.launch", "--ps", "1", "--master", "1",
           "--workers", "1", "--timeout", "150", os.path.join(ROOT, "bench", "ps_throughput.py"), "--max-steps", "600",
           "--warm", "50", "--sessions", "2"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l[l.index("{"):] for l in r.stdout.splitlines() if '{"metric"' in l]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    print(res)
    assert res["session_planes"] == ["device", "device"], res
    assert res["session_end_steps"] == [300, 600], res
