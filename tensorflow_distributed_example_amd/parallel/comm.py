"""Cross-replica communicators.

``RcclCommunicator``   GPU data plane: our C++ RCCL wrapper (csrc/comm/rccl_comm.cpp)
                       over xGMI.  Multi-process (ncclCommInitRank; one or several
                       GPUs per process, grouped init) or in-process
                       (ncclCommInitAll).  Collectives are enqueued on each device's
                       current stream and are hipGraph-capturable.
``TorchDistCommunicator`` torch.distributed (gloo on CPU — the CPU plumbing
                       config's collective path; also a GPU fallback).
``LocalCommunicator``  several replicas in one process without RCCL (CPU).
``NullCommunicator``   a single replica.

All communicators reduce a *list* of tensors, one per local replica, in place.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5,
       torch.float64: 6}
_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "mean": 4}


class Communicator:
    world_size = 1      # total replicas across all processes
    capturable = False  # collectives may be captured into a hipGraph

    def all_reduce_(self, tensors, op="sum"):
        raise NotImplementedError

    def broadcast_(self, tensors, root=0):
        raise NotImplementedError

    def barrier(self):
        pass

    def check_health(self):
        return True

    def close(self):
        pass


class NullCommunicator(Communicator):
    capturable = True

    def all_reduce_(self, tensors, op="sum"):
        if op == "mean":
            return
        return

    def broadcast_(self, tensors, root=0):
        return


class LocalCommunicator(Communicator):
    """In-process replicas reduced with torch ops (CPU Mirrored)."""

    def __init__(self, n):
        self.world_size = n

    def all_reduce_(self, tensors, op="sum"):
        acc = tensors[0].clone()
        for t in tensors[1:]:
            acc = _combine(acc, t.to(acc.device), op)
        if op == "mean":
            acc = acc / len(tensors)
        for t in tensors:
            t.copy_(acc.to(t.device))

    def broadcast_(self, tensors, root=0):
        for i, t in enumerate(tensors):
            if i != root:
                t.copy_(tensors[root].to(t.device))


def _combine(a, b, op):
    if op in ("sum", "mean"):
        return a + b
    if op == "max":
        return torch.maximum(a, b)
    if op == "min":
        return torch.minimum(a, b)
    if op == "prod":
        return a * b
    raise ValueError(op)


class TorchDistCommunicator(Communicator):
    """torch.distributed process group (one or more local replicas per process)."""

    def __init__(self, n_local, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.n_local = n_local
        self.world_size = dist.get_world_size(group) * n_local

    def all_reduce_(self, tensors, op="sum"):
        d = self.dist
        t0 = tensors[0]
        if len(tensors) > 1:
            acc = t0.clone()
            for t in tensors[1:]:
                acc = _combine(acc, t.to(acc.device), op)
        else:
            acc = t0
        dop = {"sum": d.ReduceOp.SUM, "mean": d.ReduceOp.SUM, "max": d.ReduceOp.MAX, "min": d.ReduceOp.MIN,
               "prod": d.ReduceOp.PRODUCT}[op]
        d.all_reduce(acc, op=dop, group=self.group)
        if op == "mean":
            acc /= self.world_size
        for t in tensors:
            if t is not acc:
                t.copy_(acc.to(t.device))

    def broadcast_(self, tensors, root=0):
        d = self.dist
        src_rank, local = divmod(root, self.n_local)
        t0 = tensors[local] if d.get_rank(self.group) == src_rank else tensors[0]
        d.broadcast(t0, src=src_rank, group=self.group)
        for t in tensors:
            if t is not t0:
                t.copy_(t0.to(t.device))

    def barrier(self):
        self.dist.barrier(group=self.group)


class RcclError(RuntimeError):
    pass


class RcclCommunicator(Communicator):
    """RCCL over xGMI via the in-tree C ABI (csrc/comm/rccl_comm.cpp)."""

    capturable = True

    def __init__(self, devices, rank0=0, nranks=None, unique_id: bytes | None = None):
        from .. import _native as N
        self.N = N
        self.lib = N.hip()
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        self.nranks = nranks or n
        self.world_size = self.nranks
        self.rank0 = rank0
        self.comms = (C.c_void_p * n)()
        devs = (C.c_int * n)(*[d.index for d in self.devices])
        if self.nranks == n and unique_id is None:
            rc = self.lib.tde_nccl_comm_init_all(self.comms, n, devs)
            what = "ncclCommInitAll"
        else:
            if unique_id is None:
                raise ValueError("multi-process RCCL init needs the chief's unique id")
            if n == 1:
                c = C.c_void_p()
                rc = self.lib.tde_nccl_comm_init_rank(C.byref(c), self.nranks, unique_id, rank0, devs[0])
                self.comms[0] = c
            else:
                rc = self.lib.tde_nccl_comm_init_ranks_grouped(self.comms, self.nranks, unique_id, rank0, devs, n)
            what = "ncclCommInitRank"
        self._check(rc, what)
        self.capturable = n == 1  # grouped multi-device launches are issued eagerly

    @staticmethod
    def unique_id() -> bytes:
        from .. import _native as N
        lib = N.hip()
        nb = lib.tde_nccl_unique_id_bytes()
        buf = C.create_string_buffer(nb)
        rc = lib.tde_nccl_get_unique_id(buf)
        if rc != 0:
            raise RcclError(f"ncclGetUniqueId failed: {rc}")
        return buf.raw

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.tde_nccl_error_string(rc)
            raise RcclError(f"{what} failed: {rc} ({msg.decode() if msg else '?'})")

    def _each(self, fn):
        n = len(self.devices)
        if n > 1:
            self._check(self.lib.tde_nccl_group_start(), "ncclGroupStart")
        try:
            for i, dev in enumerate(self.devices):
                with torch.cuda.device(dev):
                    fn(i, torch.cuda.current_stream(dev).cuda_stream)
        finally:
            if n > 1:
                self._check(self.lib.tde_nccl_group_end(), "ncclGroupEnd")

    def all_reduce_(self, tensors, op="sum"):
        dt = _DT[tensors[0].dtype]
        o = _OP[op]

        def f(i, s):
            t = tensors[i]
            self._check(self.lib.tde_nccl_all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), dt, o, self.comms[i], s),
                        "ncclAllReduce")
        self._each(f)

    def broadcast_(self, tensors, root=0):
        dt = _DT[tensors[0].dtype]

        def f(i, s):
            t = tensors[i]
            self._check(self.lib.tde_nccl_broadcast(t.data_ptr(), t.data_ptr(), t.numel(), dt, root, self.comms[i], s),
                        "ncclBroadcast")
        self._each(f)

    def all_gather(self, send, recv):
        dt = _DT[send[0].dtype]

        def f(i, s):
            self._check(self.lib.tde_nccl_all_gather(send[i].data_ptr(), recv[i].data_ptr(), send[i].numel(), dt,
                                                     self.comms[i], s), "ncclAllGather")
        self._each(f)

    def check_health(self):
        for c in self.comms:
            rc = self.lib.tde_nccl_comm_async_error(c)
            if rc != 0:
                raise RcclError(f"RCCL async error {rc}: {self.lib.tde_nccl_error_string(rc).decode()}")
        return True

    def abort(self):
        for c in self.comms:
            if c:
                self.lib.tde_nccl_comm_abort(c)
        self.comms = (C.c_void_p * len(self.devices))()

    def close(self):
        for c in self.comms:
            if c:
                self.lib.tde_nccl_comm_destroy(c)
        self.comms = (C.c_void_p * len(self.devices))()
