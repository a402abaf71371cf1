"""Distribution strategies.

* ``MirroredStrategy(devices)``  — synchronous DP over the GPUs of ONE process
  (mnist_keras_distributed.py:243 uses it as the eval strategy; BASELINE trains
  with it).  In-process RCCL clique (ncclCommInitAll) over xGMI.
* ``MultiWorkerMirroredStrategy()`` — synchronous DP over worker processes
  (distributed_with_keras.py:16).  Reads TF_CONFIG (or torchrun env) at
  construction, starts the native control plane (the chief hosts the C++ TCP store
  at its cluster address: parallel/control.py), distributes the RCCL unique id from
  the chief through it and builds one clique over ALL replicas of ALL workers
  (``TDE_GPUS_PER_WORKER`` GPUs per process; default 1 = one process per GPU, the
  MI355X-preferred layout).  Initial variables are broadcast from replica 0 (C1).
  torch.distributed is not used.
* the default strategy — one replica on the default device.

Replicated variables (MirroredVariable) are realised as one flat ParamStore per
replica; they stay identical because every replica applies the same all-reduced
gradient (SUM of per-replica losses pre-scaled by 1/global_batch).
"""
from __future__ import annotations

import contextlib
import enum
import os
import threading

import torch

from .. import backend as Kb
from . import cluster as CL
from . import comm as CM

_tls = threading.local()


def _stack():
    if not hasattr(_tls, "stack"):
        _tls.stack = []
    return _tls.stack


def get_strategy():
    st = _stack()
    return st[-1] if st else _default()


def has_strategy():
    return bool(_stack())


_default_strategy = None


def _default():
    global _default_strategy
    if _default_strategy is None:
        _default_strategy = Strategy([Kb.default_device()], CM.NullCommunicator(), name="default")
    return _default_strategy


class ReduceOp(enum.Enum):
    SUM = "sum"
    MEAN = "mean"


class CommunicationImplementation(enum.Enum):
    AUTO = "AUTO"
    RING = "RING"     # torch.distributed (gloo) ring — the CPU path
    NCCL = "NCCL"     # RCCL over xGMI


class CommunicationOptions:
    def __init__(self, bytes_per_pack=0, timeout_seconds=None, implementation=CommunicationImplementation.AUTO):
        self.bytes_per_pack = bytes_per_pack
        self.timeout_seconds = timeout_seconds
        self.implementation = implementation


class PerReplica:
    def __init__(self, values):
        self.values = tuple(values)

    def __repr__(self):
        return f"PerReplica({list(self.values)})"


class _Extended:
    def __init__(self, strategy):
        self._s = strategy

    @property
    def worker_devices(self):
        return tuple(str(d) for d in self._s.local_devices)

    @property
    def parameter_devices(self):
        return self.worker_devices


class Strategy:
    control = None   # the native control plane of a multi-worker strategy (parallel/control.py)

    def __init__(self, local_devices, communicator, num_workers=1, worker_index=0, name=None):
        self.local_devices = [torch.device(d) for d in local_devices]
        self.comm = communicator
        self.num_workers = num_workers
        self.worker_index = worker_index
        self.name = name or type(self).__name__
        self.extended = _Extended(self)

    # ------------------------------------------------------------------ topology
    @property
    def num_local_replicas(self):
        return len(self.local_devices)

    @property
    def num_replicas_in_sync(self):
        return self.num_local_replicas * self.num_workers

    def global_replica_id(self, local_index):
        return self.worker_index * self.num_local_replicas + local_index

    @property
    def is_chief(self):
        return self.worker_index == 0

    def barrier(self):
        """All workers of the strategy (a no-op for one process)."""

    # ------------------------------------------------------------------ scope
    @contextlib.contextmanager
    def scope(self):
        _stack().append(self)
        try:
            yield self
        finally:
            _stack().pop()

    # ------------------------------------------------------------------ variables
    def replicate_store(self, store):
        """Per-local-replica ParamStores; variables broadcast from replica 0 (C1)."""
        stores = [store if store.device == self.local_devices[0] else store.clone_to(self.local_devices[0])]
        for d in self.local_devices[1:]:
            stores.append(store.clone_to(d))
        self.broadcast_stores(stores)
        return stores

    def broadcast_stores(self, stores):
        if self.num_replicas_in_sync > 1:
            self.comm.broadcast_([s.w for s in stores], root=0)
            self.comm.broadcast_([s.state for s in stores], root=0)
            for k in stores[0].slots:
                self.comm.broadcast_([s.slot(k) for s in stores], root=0)
            self._sync_all(stores)

    def _sync_all(self, stores):
        for s in stores:
            if s.device.type == "cuda":
                torch.cuda.synchronize(s.device)

    # ------------------------------------------------------------------ data
    def experimental_distribute_dataset(self, dataset, options=None):
        from ..data.distributed import DistributedDataset
        return DistributedDataset(dataset, self)

    distribute_datasets_from_function = None

    # ------------------------------------------------------------------ generic run/reduce
    def run(self, fn, args=(), kwargs=None):
        kwargs = kwargs or {}
        outs = []
        for i, dev in enumerate(self.local_devices):
            a = tuple(x.values[i] if isinstance(x, PerReplica) else x for x in args)
            ctx = torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()
            with ctx:
                outs.append(fn(*a, **kwargs))
        return outs[0] if len(outs) == 1 else PerReplica(outs)

    def reduce(self, reduce_op, value, axis=None):
        vals = list(value.values) if isinstance(value, PerReplica) else [value]
        vals = [torch.as_tensor(v, dtype=torch.float32) for v in vals]
        if axis is not None:
            vals = [v.sum(dim=axis) if reduce_op in (ReduceOp.SUM, "sum") else v.mean(dim=axis) for v in vals]
        tens = [v.to(self.local_devices[i % len(self.local_devices)]).clone() for i, v in enumerate(vals)]
        while len(tens) < self.num_local_replicas:
            tens.append(torch.zeros_like(tens[0]).to(self.local_devices[len(tens)]))
        op = "mean" if reduce_op in (ReduceOp.MEAN, "mean") else "sum"
        if self.num_replicas_in_sync > 1:
            self.comm.all_reduce_(tens, op=op)
            self._sync_all_dev()
            return tens[0].cpu()
        return tens[0].cpu()

    def _sync_all_dev(self):
        for d in self.local_devices:
            if d.type == "cuda":
                torch.cuda.synchronize(d)

    def __repr__(self):
        return f"<{self.name} replicas={self.num_replicas_in_sync} devices={[str(d) for d in self.local_devices]}>"


def _parse_devices(devices):
    if devices is None and Kb.default_devices():
        devices = Kb.default_devices()
    if devices is None:
        if torch.cuda.is_available():
            return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
        return [torch.device("cpu")]
    out = []
    for d in devices:
        if isinstance(d, torch.device):
            out.append(d)
            continue
        out.append(Kb.parse_device(d))
    return out


class MirroredStrategy(Strategy):
    """Single-process synchronous data parallelism over local devices."""

    def __init__(self, devices=None, cross_device_ops=None):
        devs = _parse_devices(devices)
        n = len(devs)
        if n == 1:
            comm = CM.NullCommunicator()
        elif all(d.type == "cuda" for d in devs):
            comm = _local_gpu_comm(devs)
        else:
            comm = CM.LocalCommunicator(n)
        super().__init__(devs, comm, name="MirroredStrategy")


def _local_gpu_comm(devs):
    """Communicator of several GPU replicas in ONE process: the in-process xGMI peer all-reduce for the
    gradient bucket (graph-captured per replica, optimizer fused), RCCL (ncclCommInitAll) for the rest.
    Replicas sharing a device (a 1-GPU rehearsal of the N-GPU layout) cannot form an RCCL clique: their
    non-gradient collectives use torch copies."""
    distinct = len({d.index for d in devs}) == len(devs)
    base = CM.RcclCommunicator(devs) if distinct else CM.LocalCommunicator(len(devs))
    if os.environ.get("TDE_MIRRORED_XGMI", "1") == "0":
        return base
    return CM.peer_xgmi(devs, base)


class OneDeviceStrategy(Strategy):
    def __init__(self, device):
        super().__init__(_parse_devices([device]), CM.NullCommunicator(), name="OneDeviceStrategy")


class MultiWorkerMirroredStrategy(Strategy):
    """Synchronous DP across worker processes; must be created first (DWK:16)."""

    def __init__(self, communication=CommunicationImplementation.AUTO, cluster_resolver=None,
                 communication_options=None, gpus_per_worker=None):
        if communication_options is not None:
            communication = communication_options.implementation
        topo = CL.worker_topology()
        self.topology = topo
        gpw = gpus_per_worker or int(os.environ.get("TDE_GPUS_PER_WORKER", "1"))
        use_gpu = torch.cuda.is_available()
        if Kb.default_devices() and gpus_per_worker is None and "TDE_GPUS_PER_WORKER" not in os.environ:
            devs = _parse_devices(None)   # --devices: this worker's local replicas
        elif use_gpu:
            ndev = torch.cuda.device_count()
            if topo.world == 1 and topo.source == "local" and gpus_per_worker is None and \
                    "TDE_GPUS_PER_WORKER" not in os.environ:
                devs = [torch.device("cuda", i) for i in range(ndev)]  # TF: single worker uses all local GPUs
            else:
                base = (topo.local_rank * gpw) % max(ndev, 1)
                devs = [torch.device("cuda", (base + i) % ndev) for i in range(gpw)]
        else:
            devs = [torch.device("cpu")]
        n_local = len(devs)
        world = topo.world
        self.control = None
        if world > 1:
            from . import control as CP
            self.control = CP.ControlPlane.for_topology(topo)
            CP.set_current(self.control)
        impl = communication if isinstance(communication, CommunicationImplementation) else \
            CommunicationImplementation(str(communication))
        if world * n_local == 1:
            comm = CM.NullCommunicator()
        elif use_gpu and impl in (CommunicationImplementation.AUTO, CommunicationImplementation.NCCL):
            comm = self._rccl(devs, topo, world, n_local, self.control)
        elif world > 1:
            comm = CM.StoreCommunicator(self.control, n_local)
        else:
            comm = CM.LocalCommunicator(n_local) if not use_gpu else CM.RcclCommunicator(devs)
        super().__init__(devs, comm, num_workers=world, worker_index=topo.rank, name="MultiWorkerMirroredStrategy")
        self.cluster_resolver = cluster_resolver or CL.TFConfigClusterResolver()
        # peer failure detection: heartbeats to the chief's native store + watchdog
        from . import health
        self.health = health.maybe_start(topo.rank, world, comm, self.control)

    @staticmethod
    def _rccl(devs, topo, world, n_local, control):
        if world == 1:
            return _local_gpu_comm(devs)
        if os.environ.get("TDE_RCCL", "1") == "0":
            # no RCCL clique (e.g. several ranks sharing one GPU in a rehearsal): the control-plane store
            # carries the non-gradient collectives, the xGMI kernel the gradient bucket
            base = CM.StoreCommunicator(control, n_local)
        else:
            import sys
            # the chief's ncclUniqueId travels through the native store
            uid = control.broadcast_bytes(CM.RcclCommunicator.unique_id() if topo.rank == 0 else None, 0,
                                          "rccl_uid")
            base, err = None, None
            try:
                base = CM.RcclCommunicator(devs, rank0=topo.rank * n_local, nranks=world * n_local, unique_id=uid)
            except Exception as e:  # keep every rank on the same backend: agree before using it
                err = f"rank {topo.rank}: {e}"
            errs = control.agree(err, "rccl_init")
            if errs:
                if base is not None:
                    base.abort()
                print(f"[tde] RCCL communicator init failed ({'; '.join(errs)}); collectives fall back to "
                      "the control-plane store", file=sys.stderr, flush=True)
                base = CM.StoreCommunicator(control, n_local)
        if n_local == 1:
            # one GPU per process on one xGMI node: the gradient bucket takes the peer-memory kernel
            return CM.maybe_xgmi(base, devs[0], topo.rank, world, control)
        # K GPUs per worker on one node: the same kernel over direct (in-process) and IPC (other
        # workers) windows, one graph per local replica
        if os.environ.get("TDE_MIRRORED_XGMI", "1") != "0" and CM.same_node(control):
            return CM.peer_xgmi(devs, base, rank0=topo.rank * n_local, world=world * n_local, control=control)
        return base

    def barrier(self):
        if self.num_workers > 1:
            self.control.barrier()


class _Experimental:
    MultiWorkerMirroredStrategy = MultiWorkerMirroredStrategy
    CommunicationImplementation = CommunicationImplementation
    CommunicationOptions = CommunicationOptions

    @property
    def ParameterServerStrategy(self):
        from .ps import ParameterServerStrategy
        return ParameterServerStrategy


experimental = _Experimental()
