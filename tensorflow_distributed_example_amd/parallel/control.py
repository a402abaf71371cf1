"""Native control plane of a multi-worker job (reference: the gRPC server
and CollectiveAllReduce bootstrap that ``MultiWorkerMirroredStrategy()`` starts at
distributed_with_keras.py:16).

The chief (rank 0) hosts the C++ TCP key-value store (csrc/comm/tcp_store.cpp) at the chief's
``TF_CONFIG`` cluster address — the address TF's gRPC server would bind — or, under a torchrun-style
environment whose ``MASTER_PORT`` the launcher's own rendezvous store already holds, at
``MASTER_PORT + 1`` (``TDE_STORE_PORT`` overrides either).  Every worker connects to it (retrying
until ``timeout``), and everything the strategy needs before and beside the RCCL data plane goes
through it:

* the RCCL ``ncclUniqueId`` (published by the chief, fetched by everyone),
* the xGMI IPC window handles and the rank-agreed setup decisions (``all_gather_bytes`` /
  ``agree``: a failure on any rank makes every rank take the same fallback),
* barriers, and small host reductions (bench timings),
* ``StoreCommunicator``: the CPU collectives of the CPU plumbing config (rank-ordered reduction, so
  every worker computes bit-identical sums),
* the heartbeat / dead-member detection of ``parallel/health.py``.

``torch.distributed`` is never initialised on this path.  Every call is collective (SPMD order):
keys carry a per-process call sequence number, and the last reader of a round deletes its keys.
"""
from __future__ import annotations

import json
import os

import numpy as np

from .store import StoreTimeout, TCPStore, TCPStoreServer


class ControlPlane:
    def __init__(self, rank, world, host, port, timeout=300.0):
        self.rank, self.world = int(rank), int(world)
        self.host = "127.0.0.1" if host in ("localhost", "") else host
        self.timeout = float(timeout)
        self.server = None
        if self.rank == 0:
            try:
                self.server = TCPStoreServer("0.0.0.0", int(port))
            except OSError as e:
                raise OSError(f"chief cannot host the control-plane store on port {port}: {e} "
                              "(set TDE_STORE_PORT to a free port)") from e
        self.port = self.server.port if self.server is not None else int(port)
        self.store = TCPStore(self.host, self.port, timeout=self.timeout)
        self._seq = 0
        self._closed = False
        import atexit
        atexit.register(self.shutdown)

    @classmethod
    def for_topology(cls, topo, timeout=None):
        """The control plane of ``parallel.cluster.worker_topology()``."""
        port = os.environ.get("TDE_STORE_PORT")
        if port is None:
            # TF_CONFIG: the chief's own cluster port; torchrun: the launcher's store holds MASTER_PORT
            port = topo.master_port if topo.source == "tf_config" else topo.master_port + 1
        t = float(timeout if timeout is not None else os.environ.get("TDE_STORE_TIMEOUT", 300))
        return cls(topo.rank, topo.world, topo.master_addr, int(port), timeout=t)

    # ------------------------------------------------------------------ primitives
    def _round(self, tag):
        self._seq += 1
        return f"cp/{self._seq}/{tag}"

    def _done(self, k, keys):
        """Last reader of round ``k`` removes its keys (the store stays small over a long job)."""
        if self.store.add(f"{k}/read", 1) == self.world:
            for key in keys:
                self.store.delete(key)
            self.store.delete(f"{k}/read")

    def barrier(self, tag="barrier"):
        k = self._round(tag)
        self.store.barrier(k, self.world, timeout=self.timeout)
        self._done(k, [f"{k}/count", f"{k}/done"])

    def all_gather_bytes(self, data: bytes, tag="ag") -> list:
        k = self._round(tag)
        self.store.set(f"{k}/{self.rank}", bytes(data))
        out = [self.store.get(f"{k}/{r}", timeout=self.timeout) for r in range(self.world)]
        self._done(k, [f"{k}/{r}" for r in range(self.world)])
        return out

    def broadcast_bytes(self, data: bytes | None, src=0, tag="bc") -> bytes:
        k = self._round(tag)
        if self.rank == src:
            self.store.set(f"{k}/v", bytes(data))
        out = self.store.get(f"{k}/v", timeout=self.timeout)
        self._done(k, [f"{k}/v"])
        return out

    # JSON-able values (control messages: hosts, decisions, error strings)
    def all_gather_json(self, obj, tag="agj") -> list:
        return [json.loads(b.decode()) for b in self.all_gather_bytes(json.dumps(obj).encode(), tag)]

    def broadcast_json(self, obj, src=0, tag="bcj"):
        return json.loads(self.broadcast_bytes(json.dumps(obj).encode() if self.rank == src else None, src,
                                               tag).decode())

    def agree(self, err: str | None, tag="agree") -> list:
        """Every rank's error (None = ok); all ranks get the same list and can take the same branch."""
        return [e for e in self.all_gather_json(err, tag) if e]

    def all_reduce_max(self, value: float) -> float:
        return max(self.all_gather_json(float(value), "max"))

    def all_reduce_array(self, arr: np.ndarray, op="sum") -> np.ndarray:
        """Rank-ordered reduction of a host array (identical result bits on every rank)."""
        a = np.ascontiguousarray(arr)
        parts = self.all_gather_bytes(a.tobytes(), "ar")
        vals = [np.frombuffer(p, dtype=a.dtype).reshape(a.shape) for p in parts]
        acc = vals[0].copy()
        for v in vals[1:]:
            if op in ("sum", "mean"):
                acc += v
            elif op == "max":
                np.maximum(acc, v, out=acc)
            elif op == "min":
                np.minimum(acc, v, out=acc)
            elif op == "prod":
                acc *= v
            else:
                raise ValueError(op)
        if op == "mean":
            acc = acc / self.world
        return acc

    def shutdown(self, timeout=10.0):
        """Leave the job: every rank signs off; the chief keeps hosting the store until all have (bounded
        by ``timeout``), so no rank loses the store in the middle of its last control-plane call."""
        if self._closed:
            return
        import time
        try:
            n = self.store.add("cp/bye", 1)
            if self.rank == 0:
                t_end = time.monotonic() + timeout
                while n < self.world and time.monotonic() < t_end:
                    time.sleep(0.01)
                    n = self.store.add("cp/bye", 0)
        except Exception:  # noqa: BLE001 - the chief is gone already: nothing left to wait for
            pass
        self.close()

    def close(self):
        self._closed = True
        try:
            self.store.close()
        finally:
            if self.server is not None:
                self.server.stop()
                self.server = None


_current = None


def current():
    """The process's control plane (set by MultiWorkerMirroredStrategy), or None."""
    return _current


def set_current(cp):
    global _current
    _current = cp


__all__ = ["ControlPlane", "StoreTimeout", "current", "set_current"]
