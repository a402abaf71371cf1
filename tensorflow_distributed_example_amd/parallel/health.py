"""Peer failure detection for synchronous multi-worker training.

The chief hosts the native TCP store (csrc/comm/tcp_store.cpp); every worker process runs a
heartbeat thread against it and a watchdog that polls ``dead_members(timeout)``.  When a peer
stops heartbeating (crash, kill, wedged process) or the chief's store becomes unreachable,
the watchdog logs which task died, aborts the RCCL communicator (so no rank stays blocked in a
collective — ncclCommAbort) and terminates the process with ``EXIT_PEER_FAILURE``; a relaunch
resumes from the latest checkpoint (Estimator auto-restore / ``BackupAndRestore``).

Clean shutdown marks ``done/<rank>`` first, so finishing at different times is not a failure.
Knobs: ``TDE_HEARTBEAT=0`` disables it, ``TDE_HEARTBEAT_TIMEOUT`` (s, default 60),
``TDE_HEARTBEAT_INTERVAL`` (s, default 0.5).
"""
from __future__ import annotations

import atexit
import os
import sys
import threading
import time

EXIT_PEER_FAILURE = 75


class HealthMonitor:
    def __init__(self, rank, world, comm=None, timeout=None, interval=None, on_failure=None, control=None):
        self.rank, self.world, self.comm = rank, world, comm
        self.control = control
        self.timeout = float(timeout if timeout is not None else os.environ.get("TDE_HEARTBEAT_TIMEOUT", 60))
        self.interval = float(interval if interval is not None else os.environ.get("TDE_HEARTBEAT_INTERVAL", 0.5))
        self.on_failure = on_failure or self._default_failure
        self._stop = threading.Event()
        self.server = None
        self.store = None
        self.failed = None
        self._threads = []

    # ------------------------------------------------------------------ bootstrap
    def start(self):
        from .store import TCPStore, TCPStoreServer
        if self.control is not None:
            # the job's control-plane store (hosted by the chief) also keeps the heartbeats
            host, port = self.control.host, self.control.port
        else:
            self.server = TCPStoreServer("0.0.0.0", 0)
            host, port = "127.0.0.1", self.server.port
        self.store = TCPStore(host, port, timeout=max(self.timeout, 10.0))
        self._beat_store = TCPStore(host, port, timeout=max(self.timeout, 10.0))
        self._beat()
        if self.control is not None:
            self.control.barrier("health")
        for fn in (self._heartbeat_loop, self._watch_loop):
            t = threading.Thread(target=fn, daemon=True, name=f"tde-health-{fn.__name__}")
            t.start()
            self._threads.append(t)
        atexit.register(self.stop)
        from ..utils import fault
        fault.on_hang(self._stop.set)   # an injected hang also silences the heartbeat
        return self

    def _beat(self):
        self._beat_store.heartbeat(f"rank{self.rank}")

    # ------------------------------------------------------------------ threads
    def _heartbeat_loop(self):
        while not self._stop.wait(self.interval):
            try:
                self._beat()
            except Exception as e:  # chief (store host) gone
                if not self._stop.is_set():
                    self._fail(f"lost the chief's store ({e})")
                return

    def _watch_loop(self):
        while not self._stop.wait(self.interval):
            try:
                dead = self.store.dead_members(self.timeout)
                dead = [d for d in dead if d != f"rank{self.rank}" and not self.store.check(f"done/{d}")]
            except Exception as e:
                if not self._stop.is_set():
                    self._fail(f"lost the chief's store ({e})")
                return
            if dead and not self._stop.is_set():
                self._fail(f"peer(s) {', '.join(sorted(dead))} stopped heartbeating for > {self.timeout:.1f}s")
                return

    def _fail(self, why):
        if self.failed is not None:
            return
        self.failed = why
        self.on_failure(why)

    def _default_failure(self, why):
        print(f"[tde.health] rank {self.rank}/{self.world}: {why}; aborting collectives and exiting "
              f"(code {EXIT_PEER_FAILURE}). Relaunch to resume from the latest checkpoint.", file=sys.stderr,
              flush=True)
        try:
            if self.comm is not None and hasattr(self.comm, "abort"):
                self.comm.abort()
        finally:
            os._exit(EXIT_PEER_FAILURE)

    def stop(self):
        if self._stop.is_set():
            return
        try:
            self.store.set(f"done/rank{self.rank}", b"1")
        except Exception:
            pass
        self._stop.set()


def maybe_start(rank, world, comm, control=None):
    if world <= 1 or os.environ.get("TDE_HEARTBEAT", "1") == "0":
        return None
    return HealthMonitor(rank, world, comm, control=control).start()
