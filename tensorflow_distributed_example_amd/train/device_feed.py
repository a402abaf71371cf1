"""HBM-resident input pipeline for ``Model.fit``.

The reference's pipelines cache the whole (mapped) training set in memory and then shuffle / repeat /
batch it (``distributed_with_keras.py:30,54``: ``map(scale).cache().shuffle(10000)...batch(128)``;
``mnist_keras_distributed.py:142-145``).  With 288 GB of HBM per GPU that cache belongs on the device:
``DeviceFeed`` uploads the cached columns once per device (x in the program's input dtype, y as
int32), keeps the shuffle / repeat / shard / rebatch algebra on host index streams
(``Dataset.device_source``: the same semantics as iterating the dataset, native shuffle engine), and per
execution ships only S x B int32 row indices per replica; the HIP gather kernel
(``csrc/kernels/gather.hip``) fills the program's input ring.  The host no longer gathers or copies image
bytes, so ``fit()`` runs at the device step rate instead of the host gather rate.

Used when the training dataset is batches of rows of in-memory numeric (x, y) columns and every replica is
a GPU; ``TDE_DEVICE_DATA=0`` keeps the host gather + pinned staging path (``runner._Stager``).
"""
from __future__ import annotations

import os

import numpy as np
import torch


class DeviceFeed:
    @staticmethod
    def try_make(dds, prog):
        if os.environ.get("TDE_DEVICE_DATA", "1") == "0":
            return None
        if not prog.devices or not all(d.type == "cuda" for d in prog.devices):
            return None
        src = dds.device_source() if hasattr(dds, "device_source") else None
        if src is None:
            return None
        cols, tup, index_iter = src
        if not tup or len(cols) != 2:
            return None
        x, y = cols
        if not (isinstance(x, np.ndarray) and isinstance(y, np.ndarray)):
            return None
        if x.dtype.kind not in "fiu" or y.dtype.kind not in "iu" or len(x) == 0:
            return None
        n = len(x)
        per = int(np.prod(prog.x_shape))
        if len(y) != n or x.size != n * per or y.size != n or n >= 2 ** 31:
            return None
        if not DeviceFeed.row_ok(per, prog.x_ring[0].dtype):
            return None
        return DeviceFeed(prog, x, y, index_iter)

    @staticmethod
    def row_ok(per, ring_dtype):
        """The HIP row gather moves whole 4-byte words (gather.hip): a row of ``per`` elements of the ring
        dtype must be a multiple of 4 bytes (an odd feature count in a bf16 ring is not), else the
        host gather + pinned staging path feeds the program."""
        return (per * torch.empty((), dtype=ring_dtype).element_size()) % 4 == 0

    def __init__(self, prog, x, y, index_iter):
        from .. import _native as N
        from ..ops import layer_ops as O
        self.N, self.lib = N, N.hip()
        self.prog = prog
        self.index_iter = index_iter
        self.it = None
        self.n = len(x)
        self.per = int(np.prod(prog.x_shape))
        self.x_host, self.y_host = x, y      # host copies for partial batches
        SB = prog.S * prog.B
        # the uploaded columns stay with the program: a later fit() over the same cached arrays reuses them
        cached = getattr(prog, "_device_cache", None)
        if cached is not None and cached[0] is x and cached[1] is y:
            cols = cached[2]
        else:
            prog._device_cache = None
            xf = np.ascontiguousarray(x.reshape(self.n, self.per), dtype=np.float32)
            yi = np.ascontiguousarray(y.reshape(-1), dtype=np.int32)
            cols = []
            for r, d in enumerate(prog.devices):
                with torch.cuda.device(d):
                    xd = torch.from_numpy(xf).to(d)
                    ring_dt = prog.x_ring[r].dtype
                    if ring_dt == torch.bfloat16:
                        xb = torch.empty(self.n * self.per, dtype=torch.bfloat16, device=d)
                        O.cast_bf16(xd.view(-1), xb)          # the staging cast, once for the whole cache
                        xd = xb
                    elif ring_dt != torch.float32:
                        xd = xd.to(ring_dt)
                    cols.append((xd, torch.from_numpy(yi).to(d)))
            prog._device_cache = (x, y, cols)
        self.dev = []
        for r, d in enumerate(prog.devices):
            xd, yd = cols[r]
            with torch.cuda.device(d):
                self.dev.append(dict(
                    x=xd, y=yd, idx=torch.empty(SB, dtype=torch.int32, device=d),
                    bad=torch.zeros(1, dtype=torch.int32, device=d),
                    pin=[torch.empty(SB, dtype=torch.int32, pin_memory=True) for _ in range(2)],
                    ev=[None, None], k=0))
            torch.cuda.synchronize(d)

    # ------------------------------------------------------------------ index stream
    def reset(self):
        self.it = None

    def next(self):
        """Per-replica row-index arrays of the next global batch, or None at the end of the stream."""
        if self.it is None:
            self.it = iter(self.index_iter())
        try:
            return next(self.it)
        except StopIteration:
            self.it = None
            return None

    def host_batch(self, per_replica_idx):
        """(x, y) per replica gathered on the host (partial batches run eagerly through run_single)."""
        return [(self.x_host[i].reshape((len(i),) + tuple(self.prog.x_shape)), self.y_host[i].reshape(-1))
                for i in per_replica_idx]

    # ------------------------------------------------------------------ device staging
    def stage(self, group):
        """group: S global batches, each a list of per-replica index arrays of exactly B rows."""
        prog = self.prog
        S, B = prog.S, prog.B
        for r, d in enumerate(prog.devices):
            st = self.dev[r]
            buf = st["pin"][st["k"]]
            ev = st["ev"][st["k"]]
            if ev is not None:
                ev.synchronize()           # the H2D that last read this pinned buffer is done
            flat = buf.numpy()
            for s in range(S):
                flat[s * B:(s + 1) * B] = group[s][r]
            with torch.cuda.device(d):
                stream = torch.cuda.current_stream(d)
                st["idx"].copy_(buf, non_blocking=True)
                e = torch.cuda.Event()
                e.record(stream)
                st["ev"][st["k"]] = e
                st["k"] ^= 1
                sp = self.N.stream_ptr()
                xr, yr = prog.x_ring[r], prog.y_ring[r]
                rc = self.lib.tde_gather_rows_dev(st["x"].data_ptr(), self.per * st["x"].element_size(), self.n,
                                                  st["idx"].data_ptr(), S * B, xr.data_ptr(), st["bad"].data_ptr(),
                                                  sp)
                self.N.check(rc, "tde_gather_rows_dev (x)")
                rc = self.lib.tde_gather_rows_dev(st["y"].data_ptr(), 4, self.n, st["idx"].data_ptr(), S * B,
                                                  yr.data_ptr(), st["bad"].data_ptr(), sp)
                self.N.check(rc, "tde_gather_rows_dev (y)")

    def check(self):
        """Raise if any gathered index was outside the cache (a bug in the index algebra)."""
        for st in self.dev:
            if int(st["bad"].item()):
                raise IndexError("device feed: row index outside the cached dataset")
