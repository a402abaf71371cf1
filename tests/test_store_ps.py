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
