"""ParameterServerStrategy — asynchronous between-graph data parallelism
(reference: mnist_keras_distributed.py:242,
tf2_mnist_distributed.py:189).

* ``ps`` tasks run the native parameter server (csrc/ps/param_server.cpp):
  ``run_ps_server(address)`` blocks forever like TF's ``server.join()``.
* Variables are placed round-robin over the ps tasks in creation order (TF's
  replica_device_setter default).
* Workers / the chief (``master``/``chief``) pull all variables, run the
  forward/backward on their local GPU through the HIP plan, push gradients
  (the PS applies ``w -= lr*g`` on receipt, no barrier) and BN moving-statistic
  updates, and increment the global step; training stops when the global step
  reaches ``max_steps`` (counted over ALL workers, like the Estimator).
* Session device filters (mnist_keras_distributed.py:176-189) restrict which
  tasks a process connects to: a worker never talks to other workers.
* With no cluster (TF_CONFIG unset) the strategy degrades to local training
  (TF1 "local mode").
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import torch

from .. import _native as N
from .. import backend as Kb
from . import cluster as CL
from . import comm as CM
from .strategy import Strategy

N.register_host({
    "tde_ps_server_start": (C.c_void_p, [C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
    "tde_ps_server_stop": (None, [C.c_void_p]),
    "tde_ps_server_step": (C.c_longlong, [C.c_void_p]),
    "tde_ps_connect": (C.c_void_p, [C.c_char_p, C.c_int, C.c_int]),
    "tde_ps_close": (None, [C.c_void_p]),
    "tde_ps_init": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_longlong]),
    "tde_ps_pull": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p),
                              C.POINTER(C.c_longlong)]),
    "tde_ps_push": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p),
                              C.POINTER(C.c_longlong), C.c_float]),
    "tde_ps_moving_avg": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_longlong), C.c_float]),
    "tde_ps_assign": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_longlong]),
    "tde_ps_step_add": (C.c_longlong, [C.c_void_p, C.c_longlong]),
    "tde_ps_step_get": (C.c_longlong, [C.c_void_p]),
    "tde_ps_counter_add": (C.c_longlong, [C.c_void_p, C.c_int, C.c_longlong]),
    "tde_ps_set_optimizer": (C.c_int, [C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float]),
    "tde_ps_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "tde_ps_step": (C.c_int, [C.c_void_p, C.c_float,
                              C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), C.POINTER(C.c_longlong),
                              C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_void_p),
                              C.POINTER(C.c_longlong), C.c_longlong, C.c_longlong,
                              C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p), C.POINTER(C.c_longlong),
                              C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
})

INIT_FLAG = "__tde_initialized__"


class PSServer:
    def __init__(self, host="0.0.0.0", port=0):
        p = C.c_int()
        self._h = N.host().tde_ps_server_start(host.encode(), int(port), C.byref(p))
        if not self._h:
            raise OSError(f"parameter server cannot listen on {host}:{port}")
        self.port = p.value

    @property
    def global_step(self):
        return N.host().tde_ps_server_step(self._h)

    def stop(self):
        if self._h:
            N.host().tde_ps_server_stop(self._h)
            self._h = None


def run_ps_server(address: str, stop_event=None, index: int = 0):
    """Serve variables forever (TF ``server.join()``), or until ``stop_event`` is set.  With
    ``TDE_PS_DEVICE=1`` every ps task also serves its shard's window of the same-node GPU data plane
    (parallel/ps_device.py), allocated on the chief's request per training session (``TDE_PS_GPU``: the
    GPU, default 0)."""
    host, port = address.rsplit(":", 1)
    srv = PSServer("0.0.0.0", int(port))
    print(f"[ps] serving on {address}", flush=True)
    win = None
    from . import ps_device as PD
    if PD.enabled():
        win = PD.WindowServer(srv.port, int(os.environ.get("TDE_PS_GPU", "0")), index)
    try:
        while stop_event is None or not stop_event.is_set():
            if win is not None:
                win.poll()
            time.sleep(0.05 if win is not None else 0.2)
    finally:
        if win is not None:
            win.close()
        srv.stop()


class _Conn:
    def __init__(self, address, timeout=60.0):
        host, port = address.rsplit(":", 1)
        self.lib = N.host()
        self.h = self.lib.tde_ps_connect(host.encode(), int(port), int(timeout * 1000))
        if not self.h:
            raise ConnectionError(f"cannot reach parameter server {address}")
        self.address = address

    def close(self):
        if self.h:
            self.lib.tde_ps_close(self.h)
            self.h = None


def _arr(names):
    return (C.c_char_p * len(names))(*[n.encode() for n in names])


class PSClient:
    """Client side of the PS: placement, batched pull/push per ps task."""

    def __init__(self, ps_addresses, var_shapes: dict, filters=None):
        self.ps = [a for i, a in enumerate(ps_addresses) if CL.filter_allows(filters, "ps", i)]
        if not self.ps:
            raise ValueError("no reachable ps task (check TF_CONFIG / device filters)")
        self.conns = [_Conn(a) for a in self.ps]
        self.names = list(var_shapes)
        self.shapes = dict(var_shapes)
        self.placement = {n: i % len(self.conns) for i, n in enumerate(self.names)}
        self.by_ps = [[n for n in self.names if self.placement[n] == k] for k in range(len(self.conns))]
        self.host = {n: np.zeros(int(np.prod(s)) if s else 1, dtype=np.float32) for n, s in var_shapes.items()}

    def close(self):
        for c in self.conns:
            c.close()

    # ------------------------------------------------------------------ flat fast path
    def bind_store(self, store):
        """Lay the client's host copies out like ``store``'s flat buffers: ``hw`` (trainable), ``hs``
        (non-trainable state) and ``hg`` (gradients) are ONE pinned host tensor each, every variable a
        view at its segment offset.  Pulls land straight in them, so loading the pulled values is ONE
        async H2D copy per buffer and reading the gradients ONE D2H copy (instead of a copy per
        variable), and each training step is ONE round trip per ps task (``step``)."""
        pin = store.device.type == "cuda"
        self.hw = torch.zeros(store.n_trainable, dtype=torch.float32, pin_memory=pin)
        self.hs = torch.zeros(store.n_state, dtype=torch.float32, pin_memory=pin)
        self.hg = torch.zeros(store.n_trainable, dtype=torch.float32, pin_memory=pin)
        self.hs_new = torch.zeros(store.n_state, dtype=torch.float32, pin_memory=pin)
        w, st, g = self.hw.numpy(), self.hs.numpy(), self.hg.numpy()
        self.gview = {}
        for n in self.names:
            seg = store.segments[n]
            buf = w if seg.trainable else st
            self.host[n] = buf[seg.offset: seg.offset + seg.numel]
            if seg.trainable:
                self.gview[n] = g[seg.offset: seg.offset + seg.numel]
        self.trainable = [n for n in self.names if store.segments[n].trainable]
        self._step_args = []
        for k, c in enumerate(self.conns):
            push = [n for n in self.by_ps[k] if n in self.gview]
            pull = list(self.by_ps[k])
            self._step_args.append((
                push, _arr(push), (C.c_void_p * len(push))(*[self.gview[n].ctypes.data for n in push]),
                (C.c_longlong * len(push))(*[self.gview[n].size for n in push]),
                pull, _arr(pull), (C.c_void_p * len(pull))(*[self.host[n].ctypes.data for n in pull]),
                (C.c_longlong * len(pull))(*[self.host[n].size for n in pull])))

    def step(self, lr, averages=None, dstep=1, dticket=0):
        """One async training step's exchange with every ps task: push the gradients held in ``hg``,
        the BN moving-average values ``averages`` ({name: (momentum, values)}), advance the global step
        by ``dstep`` and the ticket counter by ``dticket`` (both on ps 0), and pull fresh values of every
        variable into ``hw`` / ``hs``.  Returns (global step, ticket counter).

        ps 0 (which owns the counters) is exchanged with LAST: every ``tde_ps_step`` returns only after
        that ps task applied the push, so when the global step advances every shard already holds
        this step's update.  A chief that sees ``global_step == max_steps`` and saves the final
        checkpoint therefore never misses the last updates of the shards on ps 1..N-1."""
        averages = averages or {}
        gstep = ticket = None
        for k in list(range(1, len(self.conns))) + [0]:
            c = self.conns[k]
            push, pn, pp, ps_, pull, ln, lp, ls = self._step_args[k]
            av = [n for n in self.by_ps[k] if n in averages]
            vals = [np.ascontiguousarray(averages[n][1], dtype=np.float32).reshape(-1) for n in av]
            so, to = C.c_longlong(), C.c_longlong()
            rc = c.lib.tde_ps_step(
                c.h, float(lr), len(push), pn, pp, ps_,
                len(av), _arr(av), (C.c_float * len(av))(*[float(averages[n][0]) for n in av]),
                (C.c_void_p * len(av))(*[v.ctypes.data for v in vals]), (C.c_longlong * len(av))(*[v.size for v in vals]),
                int(dstep) if k == 0 else 0, int(dticket) if k == 0 else 0,
                len(pull), ln, lp, ls, C.byref(so), C.byref(to))
            if rc != 0:
                raise ConnectionError(f"step exchange with {c.address} failed ({rc})")
            if k == 0:
                gstep, ticket = so.value, to.value
        return gstep, ticket

    def set_optimizer(self, kind, momentum=0.0, beta1=0.9, beta2=0.999, epsilon=1e-7):
        """The update every ps task applies on a push: 0 SGD, 1 momentum, 2 Nesterov, 3 Adam (Keras forms)."""
        for c in self.conns:
            c.lib.tde_ps_set_optimizer(c.h, int(kind), float(momentum), float(beta1), float(beta2), float(epsilon))

    def initialize(self, values: dict, is_chief: bool, timeout=120.0):
        """Chief creates every variable; others wait until the chief's init flag exists."""
        if is_chief:
            for n in self.names:
                v = np.ascontiguousarray(np.asarray(values[n], dtype=np.float32).reshape(-1))
                c = self.conns[self.placement[n]]
                c.lib.tde_ps_init(c.h, n.encode(), v.ctypes.data, v.size)
            flag = np.ones(1, np.float32)
            c0 = self.conns[0]
            c0.lib.tde_ps_init(c0.h, INIT_FLAG.encode(), flag.ctypes.data, 1)
            return True
        deadline = time.time() + timeout
        c0 = self.conns[0]
        buf = np.zeros(1, np.float32)
        names = _arr([INIT_FLAG])
        ptrs = (C.c_void_p * 1)(buf.ctypes.data)
        sizes = (C.c_longlong * 1)(1)
        while time.time() < deadline:
            if c0.lib.tde_ps_pull(c0.h, 1, names, ptrs, sizes) == 0:
                return False
            time.sleep(0.05)
        raise TimeoutError("parameter servers were not initialized by the chief")

    def pull(self, names=None) -> dict:
        names = self.names if names is None else names
        for k, c in enumerate(self.conns):
            mine = [n for n in self.by_ps[k] if n in names]
            if not mine:
                continue
            ptrs = (C.c_void_p * len(mine))(*[self.host[n].ctypes.data for n in mine])
            sizes = (C.c_longlong * len(mine))(*[self.host[n].size for n in mine])
            rc = c.lib.tde_ps_pull(c.h, len(mine), _arr(mine), ptrs, sizes)
            if rc != 0:
                raise ConnectionError(f"pull from {c.address} failed ({rc})")
        return {n: self.host[n].reshape(self.shapes[n]) for n in names}

    def push(self, grads: dict, lr: float):
        for k, c in enumerate(self.conns):
            mine = [n for n in self.by_ps[k] if n in grads]
            if not mine:
                continue
            arrs = [np.ascontiguousarray(grads[n], dtype=np.float32).reshape(-1) for n in mine]
            ptrs = (C.c_void_p * len(mine))(*[a.ctypes.data for a in arrs])
            sizes = (C.c_longlong * len(mine))(*[a.size for a in arrs])
            rc = c.lib.tde_ps_push(c.h, len(mine), _arr(mine), ptrs, sizes, float(lr))
            if rc != 0:
                raise ConnectionError(f"push to {c.address} failed ({rc})")

    def moving_avg(self, values: dict, momentum: float):
        for k, c in enumerate(self.conns):
            mine = [n for n in self.by_ps[k] if n in values]
            if not mine:
                continue
            arrs = [np.ascontiguousarray(values[n], dtype=np.float32).reshape(-1) for n in mine]
            ptrs = (C.c_void_p * len(mine))(*[a.ctypes.data for a in arrs])
            sizes = (C.c_longlong * len(mine))(*[a.size for a in arrs])
            c.lib.tde_ps_moving_avg(c.h, len(mine), _arr(mine), ptrs, sizes, float(momentum))

    def step_add(self, d=1) -> int:
        c = self.conns[0]
        return int(c.lib.tde_ps_step_add(c.h, int(d)))

    def counter_add(self, idx, d=1) -> int:
        """Atomic add on PS counter ``idx`` (0 = global_step, 1 = step tickets); returns the new value."""
        c = self.conns[0]
        return int(c.lib.tde_ps_counter_add(c.h, int(idx), int(d)))

    def global_step(self) -> int:
        c = self.conns[0]
        return int(c.lib.tde_ps_step_get(c.h))

    def stats(self):
        out = []
        for c in self.conns:
            a, b = C.c_longlong(), C.c_longlong()
            c.lib.tde_ps_stats(c.h, C.byref(a), C.byref(b))
            out.append((a.value, b.value))
        return out


class ParameterServerStrategy(Strategy):
    """Async PS data parallelism; local single-device training when no cluster is configured."""

    def __init__(self, cluster_resolver=None, variable_partitioner=None):
        self.cluster_resolver = cluster_resolver or CL.TFConfigClusterResolver()
        spec = self.cluster_resolver.cluster_spec()
        self.task_type = self.cluster_resolver.task_type
        self.task_id = self.cluster_resolver.task_id
        self.ps_addresses = spec.job_tasks("ps")
        self.is_distributed = bool(spec) and bool(self.ps_addresses)
        self.device_filters = CL.device_filters()
        dev = Kb.default_device()
        n_workers = spec.num_tasks("worker") + spec.num_tasks("chief") + spec.num_tasks("master")
        super().__init__([dev], CM.NullCommunicator(), num_workers=1, worker_index=0,
                         name="ParameterServerStrategy")
        self.num_ps = len(self.ps_addresses)
        self.num_training_tasks = max(n_workers, 1)

    @property
    def is_chief(self):
        if not self.is_distributed:
            return True
        return self.task_type in ("chief", "master") or (
            self.task_type == "worker" and self.task_id == 0 and
            not (self.cluster_resolver.cluster_spec().num_tasks("chief") or
                 self.cluster_resolver.cluster_spec().num_tasks("master")))

    def client(self, var_shapes: dict) -> PSClient:
        return PSClient(self.ps_addresses, var_shapes, self.device_filters)
