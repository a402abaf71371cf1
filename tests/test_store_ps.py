"""T3: native TCP store (rendezvous/barrier/heartbeat) and parameter server, multi-process on 127.0.0.1."""
import multiprocessing as mp
import threading
import time

import numpy as np
import pytest

from tensorflow_distributed_example_amd.parallel import ps as PS
from tensorflow_distributed_example_amd.parallel.store import Heartbeat, StoreTimeout, TCPStore, TCPStoreServer


def test_store_set_get_add_wait():
    srv = TCPStoreServer("127.0.0.1", 0)
    try:
        a = TCPStore("127.0.0.1", srv.port)
        b = TCPStore("127.0.0.1", srv.port)
        a.set("k", b"v1")
        assert b.get("k") == b"v1"
        assert b.check("k") and not b.check("nope")
        assert a.add("ctr", 5) == 5 and b.add("ctr", -2) == 3
        with pytest.raises(StoreTimeout):
            a.get("missing", timeout=0.2)
        t = threading.Timer(0.2, lambda: b.set("late", b"x" * 100000))
        t.start()
        assert a.get("late", timeout=5) == b"x" * 100000   # blocking get + large value
        assert a.delete("k") and not a.check("k")
        a.close()
        b.close()
    finally:
        srv.stop()


def _barrier_member(port, i, q):
    st = TCPStore("127.0.0.1", port)
    time.sleep(0.05 * i)
    st.barrier("b0", 3, timeout=10)
    q.put((i, time.time()))


def test_store_barrier_three_processes():
    srv = TCPStoreServer("127.0.0.1", 0)
    try:
        q = mp.get_context("spawn").Queue()
        ps = [mp.get_context("spawn").Process(target=_barrier_member, args=(srv.port, i, q)) for i in range(3)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(30)
            assert p.exitcode == 0
        times = sorted(q.get()[1] for _ in range(3))
        assert times[-1] - times[0] < 0.5
    finally:
        srv.stop()


def test_heartbeat_failure_detection():
    srv = TCPStoreServer("127.0.0.1", 0)
    try:
        h1 = Heartbeat("127.0.0.1", srv.port, "worker:0", interval=0.05).start()
        h2 = Heartbeat("127.0.0.1", srv.port, "worker:1", interval=0.05).start()
        st = TCPStore("127.0.0.1", srv.port)
        time.sleep(0.3)
        assert st.dead_members(timeout=0.5) == []
        h2.stop()  # worker 1 "dies"
        time.sleep(0.8)
        assert st.dead_members(timeout=0.5) == ["worker:1"]
        h1.stop()
    finally:
        srv.stop()


def _ps_worker(addrs, wid, steps, q):
    shapes = {"w": (4,), "b": (2,)}
    c = PS.PSClient(addrs, shapes)
    c.initialize(None, is_chief=False)
    for _ in range(steps):
        c.pull()
        c.push({"w": np.ones(4, np.float32), "b": np.ones(2, np.float32)}, lr=0.01)
        c.step_add(1)
    q.put(wid)
    c.close()


def test_parameter_server_async_push_pull_two_ps_two_workers():
    s1, s2 = PS.PSServer("127.0.0.1", 0), PS.PSServer("127.0.0.1", 0)
    addrs = [f"127.0.0.1:{s1.port}", f"127.0.0.1:{s2.port}"]
    try:
        chief = PS.PSClient(addrs, {"w": (4,), "b": (2,)})
        assert chief.placement == {"w": 0, "b": 1}   # round-robin placement
        chief.initialize({"w": np.zeros(4), "b": np.full(2, 5.0)}, is_chief=True)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_ps_worker, args=(addrs, i, 25, q)) for i in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        v = chief.pull()
        assert np.allclose(v["w"], -0.01 * 50)          # 2 workers x 25 async SGD updates
        assert np.allclose(v["b"], 5.0 - 0.01 * 50)
        assert chief.global_step() == 50
        chief.moving_avg({"b": np.zeros(2, np.float32)}, momentum=0.9)
        assert np.allclose(chief.pull(["b"])["b"], 0.9 * (5.0 - 0.5))
        pushes, pulls = chief.stats()[0]
        assert pushes == 50 and pulls >= 50
        chief.close()
    finally:
        s1.stop()
        s2.stop()


def test_ps_device_filters_restrict_connections():
    s1 = PS.PSServer("127.0.0.1", 0)
    try:
        addrs = [f"127.0.0.1:{s1.port}", "127.0.0.1:1"]  # second ps unreachable but filtered out
        c = PS.PSClient(addrs, {"w": (2,)}, filters=["/job:ps/task:0", "/job:worker/task:0"])
        assert c.ps == [addrs[0]]
        c.close()
    finally:
        s1.stop()


def test_parameter_server_one_round_trip_step_over_flat_mirrors():
    """PSClient.step (the Estimator's PS loop): gradients from the flat pinned mirror, BN moving averages,
    global-step and ticket counters and the fresh values of every variable in ONE round trip per ps task;
    pulled values land at their ParamStore segment offsets."""
    from tensorflow_distributed_example_amd.train.params import ParamStore

    class _Spec:
        def __init__(self, name, shape, trainable):
            self.full_name, self.shape, self.trainable, self.aggregation = name, shape, trainable, "none"
            self.initializer = lambda shape, gen: np.zeros(shape, np.float32)

    specs = [_Spec("d/kernel", (3, 2), True), _Spec("bn/moving_mean", (2,), False), _Spec("d/bias", (2,), True)]
    store = ParamStore(specs, "cpu")
    s1, s2 = PS.PSServer("127.0.0.1", 0), PS.PSServer("127.0.0.1", 0)
    addrs = [f"127.0.0.1:{s1.port}", f"127.0.0.1:{s2.port}"]
    try:
        shapes = {n: tuple(store.segments[n].shape) for n in store.order}
        c = PS.PSClient(addrs, shapes)
        c.initialize({"d/kernel": np.ones((3, 2)), "bn/moving_mean": np.full(2, 4.0), "d/bias": np.zeros(2)},
                     is_chief=True)
        c.bind_store(store)
        c.pull()
        assert np.allclose(c.hw.numpy()[store.segments["d/kernel"].offset:][:6], 1.0)
        c.hg.numpy()[:] = 0.0
        seg_k, seg_b = store.segments["d/kernel"], store.segments["d/bias"]
        c.hg.numpy()[seg_k.offset: seg_k.offset + 6] = 2.0
        c.hg.numpy()[seg_b.offset: seg_b.offset + 2] = -1.0
        gs, t = c.step(0.5, {"bn/moving_mean": (0.9, np.zeros(2, np.float32))}, dstep=1, dticket=3)
        assert (gs, t) == (1, 3)
        assert np.allclose(c.host["d/kernel"], 1.0 - 0.5 * 2.0)     # pulled AFTER this step's push
        assert np.allclose(c.host["d/bias"], 0.5)
        assert np.allclose(c.host["bn/moving_mean"], 0.9 * 4.0)
        assert np.allclose(c.hs.numpy()[store.segments["bn/moving_mean"].offset:][:2], 3.6)
        gs, t = c.step(0.0, dstep=2, dticket=0)
        assert (gs, t) == (3, 3) and c.global_step() == 3
        assert c.stats()[0][0] == 2
        c.close()
    finally:
        s1.stop()
        s2.stop()


def test_ps_step_advances_global_step_only_after_every_shard_applied():
    """ps 0 owns the global step, so it is exchanged with LAST.  Whenever an observer reads
    global step g, the shard on ps 1 already holds >= g updates (a chief that saves the final checkpoint
    at g == max_steps sees every update).  Two trainers step concurrently; the observer checks the
    invariant on every poll and at the end."""
    import threading

    from tensorflow_distributed_example_amd.train.params import ParamStore

    class _Spec:
        def __init__(self, name, shape):
            self.full_name, self.shape, self.trainable, self.aggregation = name, shape, True, "none"
            self.initializer = lambda shape, gen: np.zeros(shape, np.float32)

    s1, s2 = PS.PSServer("127.0.0.1", 0), PS.PSServer("127.0.0.1", 0)
    addrs = [f"127.0.0.1:{s1.port}", f"127.0.0.1:{s2.port}"]
    shapes = {"a/kernel": (64,), "b/kernel": (64,)}   # round-robin: a on ps 0, b on ps 1
    max_steps = 400
    try:
        chief = PS.PSClient(addrs, shapes)
        chief.initialize({n: np.zeros(s) for n, s in shapes.items()}, is_chief=True)
        errors = []

        def trainer():
            try:
                store = ParamStore([_Spec(n, s) for n, s in shapes.items()], "cpu")
                c = PS.PSClient(addrs, shapes)
                c.bind_store(store)
                c.hg.numpy()[:] = -1.0          # lr 1: every applied update adds exactly 1.0
                while True:
                    gs, _ = c.step(1.0, dstep=1)
                    if gs >= max_steps:
                        break
                c.close()
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ts = [threading.Thread(target=trainer) for _ in range(2)]
        for t in ts:
            t.start()
        polls = 0
        while any(t.is_alive() for t in ts):
            g = chief.global_step()
            b = float(chief.pull(["b/kernel"])["b/kernel"][0])
            assert b >= g, f"global step {g} visible before ps 1 applied it (b={b})"
            polls += 1
        for t in ts:
            t.join()
        assert not errors, errors
        g = chief.global_step()
        v = chief.pull()
        assert g >= max_steps and polls > 0
        assert float(v["a/kernel"][0]) == g and float(v["b/kernel"][0]) == g
        chief.close()
    finally:
        s1.stop()
        s2.stop()


def test_ps_device_plane_shard_layout():
    """The device data plane's shard layout (parallel/ps_device.layout): round-robin variables, each shard
    [trainable | momentum slots | BN statistics], segment offsets into the local flat buffers."""
    import numpy as np

    from tensorflow_distributed_example_amd.parallel import ps_device as PD
    from tensorflow_distributed_example_amd.train.params import ParamStore

    class _Spec:
        def __init__(self, name, shape, trainable):
            self.full_name, self.shape, self.trainable, self.aggregation = name, shape, trainable, "none"
            self.initializer = lambda shape, gen: np.zeros(shape, np.float32)

    specs = [_Spec("a/kernel", (10, 3), True), _Spec("a/bias", (3,), True), _Spec("bn/moving_mean", (4,), False),
             _Spec("b/kernel", (3, 2), True), _Spec("bn/moving_variance", (4,), False)]
    st = ParamStore(specs, "cpu")
    placement = {n: i % 2 for i, n in enumerate(st.order)}
    segs, sizes = PD.layout(st, placement, 2, slots=True)
    by = {(int(s["win"]), int(s["state"]), int(s["loff"])): s for s in segs}
    assert len(segs) == 5
    # shard 0: a/kernel (30), bn/moving_mean (4), bn/moving_variance (4): trainable 30, slots 30, stats 8
    assert sizes[0] == 30 + 30 + 8 and sizes[1] == (3 + 6) * 2
    k = by[(0, 0, st.segments["a/kernel"].offset)]
    assert (k["woff"], k["n"], k["moff"], k["state"]) == (0, 30, 30, 0)
    mm = by[(0, 1, st.segments["bn/moving_mean"].offset)]
    assert (mm["woff"], mm["moff"], mm["state"]) == (60, -1, 1)
    b = by[(1, 0, st.segments["b/kernel"].offset)]
    assert (b["woff"], b["moff"]) == (3, 9 + 3)
    segs0, sizes0 = PD.layout(st, placement, 2, slots=False)
    assert sizes0 == [38, 9] and (segs0["moff"][segs0["state"] == 0] == -1).all()
