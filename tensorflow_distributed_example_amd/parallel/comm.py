"""Cross-replica communicators.

``RcclCommunicator``   GPU data plane: our C++ RCCL wrapper (csrc/comm/rccl_comm.cpp)
                       over xGMI.  Multi-process (ncclCommInitRank; one or several
                       GPUs per process, grouped init) or in-process
                       (ncclCommInitAll).  Collectives are enqueued on each device's
                       current stream and are hipGraph-capturable.
``StoreCommunicator``  CPU collectives over the native control-plane store
                       (parallel/control.py; the CPU plumbing config's collective
                       path across worker processes; also the fallback when no RCCL
                       clique exists).
``LocalCommunicator``  several replicas in one process without RCCL (CPU).
``NullCommunicator``   a single replica.

All communicators reduce a *list* of tensors, one per local replica, in place.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

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


class StoreCommunicator(Communicator):
    """Collectives of one or more local replicas per process through the native control-plane store
    (``parallel/control.ControlPlane``): every rank publishes its (locally reduced) tensor and reduces
    all of them in rank order, so every rank ends with bit-identical results.  Host-staged: the CPU
    plumbing path and the non-gradient collectives of GPU jobs that have no RCCL clique."""

    def __init__(self, control, n_local):
        self.cp = control
        self.n_local = n_local
        self.world_size = control.world * n_local

    def all_reduce_(self, tensors, op="sum"):
        t0 = tensors[0]
        acc = t0.detach().clone()
        for t in tensors[1:]:
            acc = _combine(acc, t.to(acc.device), op)
        host = acc.cpu()
        wide = host.dtype in (torch.bfloat16, torch.float16)
        arr = (host.float() if wide else host).numpy()
        red = self.cp.all_reduce_array(arr, "sum" if op == "mean" else op)
        out = torch.from_numpy(red)
        if op == "mean":
            out = out / self.world_size
        for t in tensors:
            t.copy_(out.to(device=t.device, dtype=t.dtype).view_as(t))

    def broadcast_(self, tensors, root=0):
        src_rank, local = divmod(root, self.n_local)
        src = tensors[local] if self.cp.rank == src_rank else None
        data = None
        if src is not None:
            data = src.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes()
        raw = self.cp.broadcast_bytes(data, src_rank)
        t0 = tensors[0]
        val = torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(t0.dtype).view(t0.shape)
        for t in tensors:
            if t is not src:
                t.copy_(val.to(t.device))

    def barrier(self):
        self.cp.barrier()


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



def _device_key(d):
    """Node-wide identity of a GPU (host + PCI location): equal keys = the same physical device."""
    import socket
    p = torch.cuda.get_device_properties(d)
    return (f"{socket.gethostname()}/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}/"
            f"{getattr(p, 'uuid', '')}")


GPU_SHARED = {}   # spin_chunk_cap tag -> some GPU of the world runs more than one process's all-reduce


def spin_chunk_cap(control, devices, tag):
    """The most chunks (workgroups per rank) ONE all-reduce launch may use, the same number on every rank
    of the world, or None (no limit beyond the kernel's own).

    Why a limit exists (the round-3 eager MWMS 2x2 timeouts, scripts/diag/diag_xgmi_hang.sh): a waiting
    all-reduce workgroup holds a VGPR slice of its CU (4 waves x 80 VGPRs, one per SIMD).  The fused
    MNIST-CNN backward runs 1024-thread workgroups at 128 VGPRs — the whole register file of a CU — so it
    can only be dispatched onto a CU with no other wave on it.  When another PROCESS shares the GPU, its
    all-reduce grid can be spinning on every CU while this process's backward (which precedes this
    process's arrival at that very all-reduce) waits for a free CU: neither progresses until the peer
    wait times out.  Measured (profiles/r4_xgmi_hang/): without a limit, 2 workers x 2 replicas on one
    GPU time out in eager AND graph mode with the MNIST CNN, while Model B, whose kernels fit beside a
    spinning wave, runs clean; with the limit every mode runs clean.  One process per GPU (a real N-GPU
    node) never shares CUs with its peers' kernels, so there is no limit then.  With ``co`` processes on
    one device, the other ``co - 1`` may all be spinning while this one needs whole CUs: each process
    keeps its grid within (CUs - CUs/4) / (co - 1), leaving a quarter of the chip free for whole-CU
    kernels; a process launching ``nloc`` ranks of that device in one grid gives each rank 1/nloc of it.

    The kernel's slice length, chunking and per-chunk flags assume EVERY rank launches the same number of
    chunks (``xg_slice(M, nranks, nblocks)``; ``push_spec``'s L), so the cap is one world-wide number: the
    minimum over every shared device of its grid cap divided by the largest replica group any process
    launches on it (per-rank caps disagreed under uneven co-location, e.g. 3 processes on 2
    GPUs).  ``TDE_XGMI_SPIN_CAP=0`` disables the limit (diagnostics)."""
    mine = {}
    for d in devices:
        if d.type != "cuda":
            continue
        k = _device_key(d)
        if k not in mine:
            mine[k] = [0, torch.cuda.get_device_properties(d).multi_processor_count]
        mine[k][0] += 1
    per_proc = [mine] if control is None else control.all_gather_json(mine, tag)
    cap = chunk_cap_of(per_proc)
    GPU_SHARED[tag] = cap is not None   # before the diagnostics override: wide launches need an unshared GPU
    if os.environ.get("TDE_XGMI_SPIN_CAP", "1") == "0":
        cap = None
    if control is not None:
        caps = control.all_gather_json(cap, tag + "_agree")
        if any(c != cap for c in caps):
            raise RuntimeError(f"xGMI all-reduce chunk caps differ across ranks: {caps} (TDE_XGMI_SPIN_CAP set on "
                               "some ranks only?)")
    return cap


def chunk_cap_of(per_proc):
    """``spin_chunk_cap``'s rule on the gathered layouts: per_proc[i] = {device key: [replicas process i
    launches on it, CUs]}."""
    devs = {}
    for mine in per_proc:
        for k, (nloc, cus) in mine.items():
            co, mx, c = devs.get(k, (0, 0, cus))
            devs[k] = (co + 1, max(mx, int(nloc)), int(cus))
    cap = None
    for k, (co, nloc, cus) in sorted(devs.items()):
        if co <= 1:
            continue
        per_rank = max(1, max(8, (cus - cus // 4) // (co - 1)) // max(1, nloc))
        cap = per_rank if cap is None else min(cap, per_rank)
    return cap


class XgmiCommunicator(Communicator):
    """Single-node fp32 SUM all-reduce over IPC-mapped peer windows (csrc/comm/xgmi_allreduce.hip).

    One process per GPU, all ranks on one xGMI-connected node.  The gradient bucket all-reduce
     runs as one two-shot kernel that writes straight into the peers' HBM over
    all 7 links at once; every other collective (broadcast, metrics, other dtypes/ops, buckets
    larger than the window) goes to ``fallback`` (RCCL).  Stream-ordered and hipGraph-capturable:
    the call epoch lives on the device, so graph replays need no host bookkeeping.

    ``control`` is the native control plane (parallel/control.py) that exchanges the IPC handles and
    agrees on the setup outcome across ranks.
    """

    capturable = True
    plain_ok = True   # False: the fallback measured faster for a plain (unfused) gradient all-reduce

    def __init__(self, device, rank, world, fallback, control, max_elems=None, uncached=None, nblocks=None,
                 timeout_s=None):
        from .. import _native as N
        self.lib = N.hip()
        self.device = torch.device(device)
        self.rank, self.world = int(rank), int(world)
        self.world_size = self.world
        self.fallback = fallback
        self.cp = control
        if self.world > self.lib.tde_xgmi_max_ranks():
            raise ValueError(f"xGMI all-reduce supports at most {self.lib.tde_xgmi_max_ranks()} ranks")
        self.max_elems = int(max_elems or os.environ.get("TDE_XGMI_MAX_ELEMS", 8 << 20))
        self.uncached = int(os.environ.get("TDE_XGMI_UNCACHED", "1") if uncached is None else uncached)
        self.nblocks_override = int(nblocks or os.environ.get("TDE_XGMI_BLOCKS", 0))
        timeout_s = float(timeout_s or os.environ.get("TDE_XGMI_TIMEOUT", 300))
        self.timeout_ticks = int(timeout_s * 1e8)   # s_memrealtime: 100 MHz
        self.window, self.epoch, self.err = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._opened = []
        # every step below that can fail on one rank is followed by an agreement among all ranks, so a
        # failure anywhere makes EVERY rank raise (no rank is left waiting in a collective)
        hb = C.create_string_buffer(self.lib.tde_xgmi_ipc_handle_bytes())
        rc = self.lib.tde_xgmi_alloc(self.device.index, self.max_elems, self.uncached, C.byref(self.window),
                                     C.byref(self.epoch), C.byref(self.err), hb)
        if os.environ.get("TDE_XGMI_FAIL_RANK") == str(self.rank):   # fault injection (tests)
            rc = -999
        handles = [h if h else None for h in control.all_gather_bytes(hb.raw if rc == 0 else b"", "xgmi_handles")]
        if any(h is None for h in handles):
            self._free()
            raise RuntimeError(f"xGMI window allocation failed on rank(s) "
                               f"{[r for r, h in enumerate(handles) if h is None]} (local rc {rc})")
        peers, err = [], None
        for r, h in enumerate(handles):
            if r == self.rank:
                peers.append(self.window.value)
                continue
            m = C.c_void_p()
            rc = self.lib.tde_xgmi_open(self.device.index, h, C.byref(m))
            if rc != 0:
                err = f"hipIpcOpenMemHandle of rank {r}'s window failed ({rc})"
                break
            self._opened.append(m.value)
            peers.append(m.value)
        errs = control.agree(err, "xgmi_open")
        if errs:
            self._free()
            raise RuntimeError(f"xGMI peer mapping failed: {errs}")
        self.peers = (C.c_void_p * self.world)(*peers)
        self.chunk_cap = spin_chunk_cap(control, [self.device], "xgmi_spin")
        # 1024-thread workgroups only when no other process shares this GPU (csrc/comm/xgmi_allreduce.hip)
        self.lib.tde_xgmi_set_wide(int(not GPU_SHARED.get("xgmi_spin", True)))
        tc = int(os.environ.get("TDE_XGMI_TRACE", "0") or 0)
        self.trace = [_xg_trace_alloc(self.lib, self.device, self.epoch.value, tc)] if tc > 0 else None

    def nblocks(self, M):
        """Chunks (= workgroups) of a call: ~512 elements of the slice each, within the kernel maximum and
        the world-wide co-located-process spin limit (``spin_chunk_cap``): the same on every rank."""
        if self.nblocks_override:
            return self.nblocks_override
        L = -(-M // self.world)
        nb = max(8, min(self.lib.tde_xgmi_max_blocks(), L // 512))
        return min(nb, self.chunk_cap) if self.chunk_cap else nb

    def handles(self, t, op):
        return (op == "sum" and t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
                and t.numel() <= self.max_elems and t.data_ptr() % 16 == 0 and t.device == self.device)

    def all_reduce_(self, tensors, op="sum"):
        if len(tensors) != 1 or not self.handles(tensors[0], op):
            return self.fallback.all_reduce_(tensors, op)
        t = tensors[0]
        M = t.numel()
        with torch.cuda.device(self.device):
            s = torch.cuda.current_stream(self.device).cuda_stream
            rc = self.lib.tde_xgmi_all_reduce(t.data_ptr(), M, self.max_elems, self.peers, self.epoch, self.err,
                                              self.rank, self.world, self.nblocks(M), self.uncached,
                                              self.timeout_ticks, s)
        if rc != 0:
            raise RuntimeError(f"tde_xgmi_all_reduce failed ({rc})")

    def all_reduce_apply_(self, grad, spec):
        """SUM all-reduce of the flat gradient bucket fused with the optimizer step on every rank
        (``spec``: ``ops.kernels.XgApply``): weights, slots and the bf16 shadow are updated from the
        reduced sums and the bucket is left zeroed."""
        if not self.handles(grad, "sum"):
            raise ValueError("xGMI fused all-reduce: fp32 contiguous bucket within the window required")
        import ctypes as C
        M = grad.numel()
        with torch.cuda.device(self.device):
            s = torch.cuda.current_stream(self.device).cuda_stream
            rc = self.lib.tde_xgmi_all_reduce_apply(grad.data_ptr(), M, self.max_elems, self.peers, self.epoch,
                                                    self.err, self.rank, self.world, self.nblocks(M), self.uncached,
                                                    self.timeout_ticks, C.byref(spec), s)
        if rc != 0:
            raise RuntimeError(f"tde_xgmi_all_reduce_apply failed ({rc})")

    def push_spec(self, M, off):
        """``XgPush`` for a producer kernel that stores bucket elements [off, ...) of an M-element bucket
        straight into the owners' contribution areas of the next ``all_reduce_apply_`` call."""
        return _push_spec(self.lib, M, self.max_elems, self.peers, self.epoch.value, self.rank, self.world,
                          self.nblocks(M), off)

    def broadcast_(self, tensors, root=0):
        return self.fallback.broadcast_(tensors, root)

    def all_gather(self, send, recv):
        return self.fallback.all_gather(send, recv)

    def barrier(self):
        self.fallback.barrier()

    def calls(self):
        return int(self.lib.tde_xgmi_epoch(self.epoch))

    def check_health(self):
        e = self.lib.tde_xgmi_error(self.err) if self.err else 0
        if e:
            raise RcclError(f"xGMI all-reduce: a peer never arrived (error bits {e:#x}); a rank died or hung")
        return self.fallback.check_health()

    def abort(self):
        if hasattr(self.fallback, "abort"):
            self.fallback.abort()

    def _free(self):
        for m in getattr(self, "_opened", []):
            self.lib.tde_xgmi_close(m)
        self._opened = []
        if getattr(self, "trace", None) and self.epoch:
            self.lib.tde_xgmi_set_trace(self.epoch.value, None, 0)
        if self.window:
            self.lib.tde_xgmi_free(self.window, self.epoch, self.err)
        self.window = self.epoch = self.err = C.c_void_p()

    def close(self):
        self._free()
        if self.fallback is not None:
            self.fallback.close()

    # ------------------------------------------------------------------ selection
    def self_test(self, n=None):
        """Bitwise check against the rank-ordered fp32 sum on every rank (3 calls: both parities)."""
        n = n or min(self.max_elems, 347_146 + 37)
        idx = torch.arange(n, device=self.device, dtype=torch.float32)
        ok = True
        # a broken fabric path must not park the test for the production timeout: 10 s per wait here
        saved, self.timeout_ticks = self.timeout_ticks, int(10 * 1e8)
        for it in range(3):
            parts = [((idx * 0.37 + r * 1.91 + it) % 7.0) - 3.0 for r in range(self.world)]
            want = parts[0].clone()
            for p in parts[1:]:
                want += p
            t = parts[self.rank].clone()
            self.all_reduce_([t])
            torch.cuda.synchronize(self.device)
            ok = ok and bool(torch.equal(t, want))
        ok = ok and self.lib.tde_xgmi_error(self.err) == 0
        self.timeout_ticks = saved
        return ok


def _push_spec(lib, M, max_elems, peers, epoch, rank, world, nblocks, off):
    from ..ops.kernels import XgPush
    sp = XgPush()
    rc = lib.tde_xgmi_push_spec(int(M), int(max_elems), peers, epoch, int(rank), int(world), int(nblocks), int(off),
                                C.byref(sp))
    if rc != 0:
        raise RuntimeError(f"tde_xgmi_push_spec failed ({rc})")
    return sp


def _xg_trace_alloc(lib, device, epoch_ptr, calls):
    """Diagnostics (TDE_XGMI_TRACE=<calls>): a device buffer in which every launch of the rank whose
    epoch word is ``epoch_ptr`` records per-block phase timestamps (csrc/comm/xgmi_allreduce.hip,
    XgArgs::trace), ring-indexed by call.  Returned tensor: [calls, max_blocks, words] int64."""
    words = lib.tde_xgmi_trace_words()
    buf = torch.zeros((calls, lib.tde_xgmi_max_blocks(), words), dtype=torch.int64, device=device)
    lib.tde_xgmi_set_trace(epoch_ptr, buf.data_ptr(), calls)
    return buf


def xg_trace_records(buf, nblocks):
    """Decode a trace buffer into per-call dicts (host copy; call after a device sync).  Blocks of a
    launch with ``nblocks`` chunks occupy slots [0, nblocks) of their call."""
    t = buf.cpu().numpy().view(np.uint64)
    out = []
    for c in range(t.shape[0]):
        rec = t[c, :nblocks]
        if not rec[:, 0].any():
            continue
        info = rec[:, 7]
        out.append({
            "epoch": int((rec[:, 0] & 0xFFFFFFFF).max()),
            "start": [int(v) for v in rec[:, 1]], "pub1": [int(v) for v in rec[:, 2]],
            "arr1": [int(v) for v in rec[:, 3]], "pub2": [int(v) for v in rec[:, 4]],
            "arr2": [int(v) for v in rec[:, 5]], "end": [int(v) for v in rec[:, 6]],
            "miss1": [int(v) & 0xFF for v in info], "miss2": [(int(v) >> 8) & 0xFF for v in info],
            "xcc": [(int(v) >> 16) & 0xFF for v in info], "cu": [(int(v) >> 24) & 0xF for v in info],
            "se": [(int(v) >> 28) & 0x7 for v in info],
            # value the flag held when a wait timed out (0: the wait completed)
            "seen1": [int(v) >> 32 for v in rec[:, 0]], "seen2": [int(v) >> 32 for v in info]})
    return sorted(out, key=lambda r: r["epoch"])


class PeerXgmiCommunicator(Communicator):
    """The xGMI two-shot all-reduce (csrc/comm/xgmi_allreduce.hip) for SEVERAL replicas per process:
    ``MirroredStrategy`` over the GPUs of one process (``control=None``) or MWMS with K GPUs per worker.

    Each local replica owns a window on its device.  The windows of the other local replicas are
    plain device pointers (peer access enabled between the local devices, no IPC); the windows of other
    processes' replicas are IPC-mapped once per (local device, remote rank).  Replica ``i`` is global
    rank ``rank0 + i`` of the kernel's ``world``.

    Replicas are grouped by device.  Each group's parts of the all-reduce run as ONE launch (grid.y =
    local rank) that only waits, on the device, for the other groups' launches, so a group's step (fwd,
    bwd, all-reduce[+optimizer]) is captured into a hipGraph of its own, on its own stream, and the host
    replays one graph per device per execution (``train/runner.Program``).  On an N-GPU node every group
    is one replica; several replicas mapped onto one device (the 1-GPU rehearsal) share a group, so their
    mutual waits never depend on two streams of one device running concurrently.  Non-gradient
    collectives (broadcast, other dtypes/ops) go to ``fallback``."""

    capturable = True
    per_replica = True   # all_reduce_one_ / all_reduce_apply_one_: one replica's launch on its stream
    plain_ok = True

    def __init__(self, devices, fallback, rank0=0, world=None, control=None, max_elems=None, uncached=None,
                 timeout_s=None):
        from .. import _native as N
        self.lib = N.hip()
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        self.n_local = n
        self.rank0 = int(rank0)
        self.world = int(world or n)
        self.world_size = self.world
        self.fallback = fallback
        self.cp = control
        if self.world > self.lib.tde_xgmi_max_ranks():
            raise ValueError(f"xGMI all-reduce supports at most {self.lib.tde_xgmi_max_ranks()} ranks")
        if control is None and (self.rank0 != 0 or self.world != n):
            raise ValueError("a multi-process PeerXgmiCommunicator needs the control plane")
        self.max_elems = int(max_elems or os.environ.get("TDE_XGMI_MAX_ELEMS", 16 << 20))  # ResNet-18 (11.7 M) fits: per-device graphs
        self.uncached = int(os.environ.get("TDE_XGMI_UNCACHED", "1") if uncached is None else uncached)
        self.nblocks_override = int(os.environ.get("TDE_XGMI_BLOCKS", 0))
        timeout_s = float(timeout_s or os.environ.get("TDE_XGMI_TIMEOUT", 300))
        self.timeout_ticks = int(timeout_s * 1e8)
        self.windows, self.epochs, self.errs = [], [], []
        self._opened = []
        err = None
        idx = sorted({d.index for d in self.devices})
        for a in idx:   # before any window exists (allocations made later are mapped to the peers)
            for b in idx:
                rc = self.lib.tde_enable_peer_access(a, b)
                if rc != 0 and err is None:
                    err = f"peer access cuda:{a} -> cuda:{b} failed ({rc})"
        handles = []
        if err is None:
            for d in self.devices:
                w, e, x = C.c_void_p(), C.c_void_p(), C.c_void_p()
                hb = C.create_string_buffer(self.lib.tde_xgmi_ipc_handle_bytes())
                rc = self.lib.tde_xgmi_alloc(d.index, self.max_elems, self.uncached, C.byref(w), C.byref(e),
                                             C.byref(x), hb)
                if rc != 0:
                    err = f"xGMI window allocation on {d} failed ({rc})"
                    break
                self.windows.append(w.value)
                self.epochs.append(e.value)
                self.errs.append(x.value)
                handles.append(hb.raw)
        peers = [[None] * self.world for _ in range(n)]
        if control is not None:
            # every process publishes its replicas' handles; a failure anywhere fails everywhere
            allh = control.all_gather_json([h.hex() for h in handles] if err is None else None, "pxg_handles")
            if any(h is None for h in allh):
                err = err or "xGMI window setup failed on another worker"
            else:
                flat = [bytes.fromhex(h) for hs in allh for h in hs]
                if len(flat) != self.world:
                    err = f"xGMI: {len(flat)} windows for {self.world} ranks"
        if err is None:
            mapped = {}   # (device index, remote rank) -> pointer mapped on that device
            for i, d in enumerate(self.devices):
                for r in range(self.world):
                    j = r - self.rank0
                    if 0 <= j < n:
                        peers[i][r] = self.windows[j]   # same process: the device pointer itself
                        continue
                    key = (d.index, r)
                    if key not in mapped:
                        m = C.c_void_p()
                        rc = self.lib.tde_xgmi_open(d.index, flat[r], C.byref(m))
                        if rc != 0:
                            err = f"hipIpcOpenMemHandle of rank {r}'s window on {d} failed ({rc})"
                            break
                        self._opened.append(m.value)
                        mapped[key] = m.value
                    peers[i][r] = mapped[key]
                if err is not None:
                    break
            if err is None and len({d.index for d in self.devices}) > 1:
                # one IPC mapping per device: a runtime that hands every device the same mapping has not
                # mapped it for the others, so refuse instead of faulting
                for r in range(self.world):
                    ptrs = {mapped[(d.index, r)] for d in self.devices if (d.index, r) in mapped}
                    if len(ptrs) not in (0, len({d.index for d in self.devices})):
                        err = f"IPC window of rank {r} mapped at one address for several devices"
                        break
        if control is not None:
            errs = control.agree(err, "pxg_open")
            if errs:
                self._free()
                raise RuntimeError(f"xGMI peer setup failed: {errs}")
        elif err is not None:
            self._free()
            raise RuntimeError(err)
        self.peers = [(C.c_void_p * self.world)(*p) for p in peers]
        # groups of local replicas by device (order of first appearance), and their launch arrays
        self.groups = []
        for i, d in enumerate(self.devices):
            for grp in self.groups:
                if self.devices[grp[0]] == d:
                    grp.append(i)
                    break
            else:
                self.groups.append([i])
        # a group launch gives its j-th replica kernel rank rank0 + grp[0] + j: every group must be a
        # contiguous run of replicas (gpu:0,gpu:1,gpu:0,gpu:1 would give two replicas one rank)
        if any(grp != list(range(grp[0], grp[0] + len(grp))) for grp in self.groups):
            self._free()
            raise RuntimeError(f"xGMI replica groups must be contiguous runs of one device, got {self.groups}")
        self._gargs = []
        for grp in self.groups:
            flat = [p for i in grp for p in peers[i]]
            self._gargs.append(((C.c_void_p * len(flat))(*flat), (C.c_void_p * len(grp))(*[self.epochs[i] for i in grp]),
                                (C.c_void_p * len(grp))(*[self.errs[i] for i in grp])))
        self._side = [torch.cuda.Stream(self.devices[grp[0]]) for grp in self.groups]
        self.chunk_cap = spin_chunk_cap(control, self.devices, "pxg_spin")
        self.lib.tde_xgmi_set_wide(int(not GPU_SHARED.get("pxg_spin", True)))
        tc = int(os.environ.get("TDE_XGMI_TRACE", "0") or 0)
        self.trace = [_xg_trace_alloc(self.lib, d, e, tc) for d, e in zip(self.devices, self.epochs)] \
            if tc > 0 else None

    def nblocks(self, M, nloc=1, gi=0):
        """Chunks per rank of group ``gi``'s launches (``nloc`` ranks in one grid): ~512 elements of the
        slice each, within the kernel maximum and the world-wide co-located-process spin limit
        (``spin_chunk_cap``, which already divides each shared device's grid by its largest group; none
        when no process shares a GPU) — the same number on every rank, whatever its group."""
        cap = self.lib.tde_xgmi_max_blocks()
        if self.chunk_cap:
            cap = max(1, min(cap, self.chunk_cap))
        if self.nblocks_override:
            return min(self.nblocks_override, cap)
        return max(min(8, cap), min(cap, -(-M // self.world) // 512))

    def handles(self, t, op, i):
        return (op == "sum" and t.dtype == torch.float32 and t.is_cuda and t.is_contiguous()
                and t.numel() <= self.max_elems and t.data_ptr() % 16 == 0 and t.device == self.devices[i])

    def all_reduce_group_(self, gi, grads, specs=None):
        """Group ``gi``'s parts of the SUM all-reduce (``grads``: one flat fp32 bucket per replica of the
        group, in group order) as ONE launch on the current stream of the group's device; with ``specs``
        (one ``ops.kernels.XgApply`` per replica) the optimizer step is fused in
        (``XgmiCommunicator.all_reduce_apply_``)."""
        grp = self.groups[gi]
        if len(grads) != len(grp) or not all(self.handles(t, "sum", i) for t, i in zip(grads, grp)):
            raise ValueError("xGMI all-reduce: one fp32 contiguous bucket per group replica within the window")
        M = grads[0].numel()
        if any(t.numel() != M for t in grads):
            raise ValueError("xGMI all-reduce: buckets of one group differ in length")
        dev = self.devices[grp[0]]
        sp = None
        if specs is not None:
            sp = (type(specs[0]) * len(specs))(*specs)
        peers, epochs, errs = self._gargs[gi]
        with torch.cuda.device(dev):
            s = torch.cuda.current_stream(dev).cuda_stream
            rc = self.lib.tde_xgmi_all_reduce_group(
                len(grp), (C.c_void_p * len(grp))(*[t.data_ptr() for t in grads]), M, self.max_elems, peers, epochs,
                errs, self.rank0 + grp[0], self.world, self.nblocks(M, len(grp), gi), self.uncached, self.timeout_ticks,
                sp, s)
        if rc != 0:
            raise RuntimeError(f"tde_xgmi_all_reduce_group failed ({rc})")

    def push_spec(self, i, M, off):
        """``XgPush`` of local replica ``i`` (see ``XgmiCommunicator.push_spec``)."""
        gi = next(j for j, g in enumerate(self.groups) if i in g)
        return _push_spec(self.lib, M, self.max_elems, self.peers[i], self.epochs[i], self.rank0 + i, self.world,
                          self.nblocks(M, len(self.groups[gi]), gi), off)

    def all_reduce_(self, tensors, op="sum"):
        if len(tensors) != self.n_local or not all(self.handles(t, op, i) for i, t in enumerate(tensors)) or \
                len({t.numel() for t in tensors}) != 1:
            return self.fallback.all_reduce_(tensors, op)
        # every group's launch on a side stream of its device, joined back into the callers' streams
        cur = [torch.cuda.current_stream(self.devices[grp[0]]) for grp in self.groups]
        for gi, grp in enumerate(self.groups):
            self._side[gi].wait_stream(cur[gi])
            with torch.cuda.device(self.devices[grp[0]]), torch.cuda.stream(self._side[gi]):
                self.all_reduce_group_(gi, [tensors[i] for i in grp])
        for gi in range(len(self.groups)):
            cur[gi].wait_stream(self._side[gi])

    def broadcast_(self, tensors, root=0):
        return self.fallback.broadcast_(tensors, root)

    def all_gather(self, send, recv):
        return self.fallback.all_gather(send, recv)

    def barrier(self):
        self.fallback.barrier()

    def calls(self, i=0):
        return int(self.lib.tde_xgmi_epoch(self.epochs[i]))

    def error_bits(self):
        return [self.lib.tde_xgmi_error(e) for e in self.errs]

    def check_health(self):
        bits = self.error_bits()
        if any(bits):
            raise RcclError(f"xGMI all-reduce: a peer never arrived (error bits {bits}); a replica died or hung")
        return self.fallback.check_health()

    def abort(self):
        if hasattr(self.fallback, "abort"):
            self.fallback.abort()

    def _free(self):
        for m in self._opened:
            self.lib.tde_xgmi_close(m)
        self._opened = []
        if getattr(self, "trace", None):
            for e in self.epochs:
                self.lib.tde_xgmi_set_trace(e, None, 0)
        for w, e, x in zip(self.windows, self.epochs, self.errs):
            self.lib.tde_xgmi_free(w, e, x)
        self.windows, self.epochs, self.errs = [], [], []

    def close(self):
        self._free()
        if self.fallback is not None:
            self.fallback.close()

    def self_test(self, n=None):
        """Bitwise check against the rank-ordered fp32 sum on every replica (3 calls: both parities)."""
        n = n or min(self.max_elems, 347_146 + 37)
        ok = True
        saved, self.timeout_ticks = self.timeout_ticks, int(10 * 1e8)
        try:
            for it in range(3):
                ts, wants = [], []
                for i, d in enumerate(self.devices):
                    idx = torch.arange(n, device=d, dtype=torch.float32)
                    parts = [((idx * 0.37 + r * 1.91 + it) % 7.0) - 3.0 for r in range(self.world)]
                    want = parts[0].clone()
                    for p in parts[1:]:
                        want += p
                    ts.append(parts[self.rank0 + i].clone())
                    wants.append(want)
                self.all_reduce_(ts)
                for d in self.devices:
                    torch.cuda.synchronize(d)
                ok = ok and all(bool(torch.equal(t, w)) for t, w in zip(ts, wants))
            ok = ok and not any(self.error_bits())
        finally:
            self.timeout_ticks = saved
        return ok


def peer_xgmi(devices, fallback, rank0=0, world=None, control=None):
    """``PeerXgmiCommunicator`` over ``devices`` when it sets up and passes its bitwise self-test on every
    replica (agreed across workers), else ``fallback``.  ``TDE_ALLREDUCE=rccl`` keeps the fallback."""
    import warnings
    if os.environ.get("TDE_ALLREDUCE", "auto").lower() == "rccl" or not torch.cuda.is_available():
        return fallback
    err, xg, ok = None, None, False
    try:
        xg = PeerXgmiCommunicator(devices, fallback, rank0=rank0, world=world, control=control)
        ok = xg.self_test()
    except Exception as e:  # noqa: BLE001 - raised consistently on every worker (agreed in the constructor)
        err = e
    if control is not None:
        ok = all(control.all_gather_json(bool(ok), "pxg_selftest"))
    if not ok:
        if xg is not None:
            xg.fallback = None
            xg.close()
        warnings.warn(f"in-process xGMI all-reduce unavailable ({err or 'self-test failed'}); using "
                      f"{type(fallback).__name__}")
        return fallback
    return xg


def _time_allreduce(comm, t, iters, control):
    import time
    for _ in range(3):
        comm.all_reduce_([t])
    torch.cuda.synchronize(t.device)
    control.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.all_reduce_([t])
    torch.cuda.synchronize(t.device)
    return (time.perf_counter() - t0) / iters


def maybe_xgmi(fallback, device, rank, world, control, bucket_hint=None):
    """Wrap ``fallback`` with the xGMI peer-memory all-reduce when every rank is one GPU of this node.

    ``TDE_ALLREDUCE`` = ``auto`` (default: self-test, then keep whichever of xGMI / RCCL is faster on
    a gradient-sized bucket — decided on rank 0's numbers so all ranks agree), ``xgmi`` (self-test
    only) or ``rccl`` (never wrap)."""
    import warnings
    mode = os.environ.get("TDE_ALLREDUCE", "auto").lower()
    if mode == "rccl" or world < 2 or not torch.cuda.is_available():
        return fallback
    if not same_node(control):
        return fallback   # multi-node: RCCL handles the inter-node path
    err = None
    xg = None
    try:
        xg = XgmiCommunicator(device, rank, world, fallback, control)
    except Exception as e:  # noqa: BLE001 - raised consistently on every rank; keeps RCCL
        xg, err = None, e
    ok = False
    if xg is not None:
        try:
            ok = xg.self_test()
        except Exception as e:  # noqa: BLE001
            ok, err = False, e
    flags = control.all_gather_json(bool(ok), "xgmi_selftest")
    if not all(flags):
        if xg is not None:
            xg.fallback = None
            xg.close()
        if rank == 0:
            warnings.warn(f"xGMI all-reduce self-test failed ({err or flags}); using RCCL")
        return fallback
    if mode == "auto":
        n = int(bucket_hint or 347_146)
        t = torch.zeros(min(n, xg.max_elems), device=device)
        tx = _time_allreduce(xg, t, 20, control)
        tr = _time_allreduce(fallback, t, 20, control)
        # the xGMI kernel can also carry the optimizer update (one launch fewer per step, see
        # XgmiCommunicator.all_reduce_apply_): it keeps the bucket unless RCCL is faster by more than that
        # (the margin only applies to plans that fuse the update into it: Program re-decides the plain
        # all-reduce with plain_ok)
        margin = float(os.environ.get("TDE_XGMI_MARGIN_US", "3")) * 1e-6
        dec = control.broadcast_json([tx <= tr + margin, tx <= tr], src=0, tag="xgmi_pick")
        xg.plain_ok = bool(dec[1])
        if rank == 0:
            import sys
            print(f"[tde.comm] all-reduce of {t.numel()} fp32: xGMI {tx * 1e6:.1f} us, RCCL {tr * 1e6:.1f} us "
                  f"-> {'xGMI' if dec[0] else 'RCCL'}", file=sys.stderr, flush=True)
        if not dec[0]:
            xg.fallback = None
            xg.close()
            return fallback
    return xg


def same_node(control):
    """True when every worker of the control plane runs on this host (same hostname and boot id)."""
    import socket
    hosts = control.all_gather_json([socket.gethostname(), _boot_id()], "hosts")
    return all(h == hosts[0] for h in hosts)


def _boot_id():
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()
    except OSError:
        return ""
