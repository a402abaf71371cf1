"""Same-node GPU data plane of ``ParameterServerStrategy`` (csrc/kernels/ps_device.hip; SURVEY.md F07 /
§5.8 "optional same-node fast path"; reference mnist_keras_distributed.py:242, tf2_mnist_distributed.py:189).

Every ps task owns ONE device window holding its round-robin shard of the variables (the placement of the
TCP plane, TF's replica_device_setter) — plus the momentum slots of its variables under SGD with momentum
/ Nesterov — and ps 0's window also carries the PS counters.  Windows are sized per training session: the
chief asks each ps task for the bytes its shard needs (``REQ_VAR`` on that task's TCP table); the ps task
checks its GPU's free memory, allocates (or re-arms, zeroed) a window and publishes its IPC handle
(``HANDLE_VAR``, tagged with the session).  Trainers map every window and run each async step's exchange
as one kernel over a segment table (push with f32 atomics / momentum compare-and-swap, BN moving averages
by compare-and-swap, pull, counter advance); the host only reads two host-mapped words after the step's
stream sync.  TCP keeps the control plane (the chief's plane decision, requests, handles) — no variable
bytes cross it.

Enabled with ``TDE_PS_DEVICE=1`` (ps tasks and trainers on one node with GPUs); the optimizer must be SGD
(plain, momentum or Nesterov); Adam runs on the host-staged TCP plane (``PSClient.step``).
"""
from __future__ import annotations

import ctypes as C
import os
import random
import time

import numpy as np
import torch

from .. import _native as N

_vp, _i, _i64, _f = C.c_void_p, C.c_int, C.c_longlong, C.c_float
N.register_hip({
    "tde_psdev_counters": (_i, []),
    "tde_psdev_alloc": (_i, [_i, _i64, C.POINTER(_vp), C.c_char_p]),
    "tde_psdev_free": (_i, [_vp]),
    "tde_psdev_zero": (_i, [_vp, _i64]),
    "tde_psdev_seg_bytes": (_i, []),
    "tde_host_mapped_alloc": (_i, [_i64, C.POINTER(_vp), C.POINTER(_vp)]),
    "tde_host_mapped_free": (_i, [_vp]),
    # windows, nwin, segs, beg, nseg, total, w, g, s, sp, mom, lr, mmt, kind, dstep, dticket, done, out, claim,
    # limit, stream
    "tde_psdev_step": (_i, [_vp, _i, _vp, _vp, _i, _i64, _vp, _vp, _vp, _vp, _vp, _f, _f, _i, _i64, _i64, _vp, _vp,
                            _vp, _i64, _vp]),
    "tde_psdev_copy": (_i, [_vp, _i, _vp, _i, _i64, _vp, _vp, _i, _vp]),
    "tde_psdev_set_counter": (_i, [_vp, _i, _i64]),
    "tde_psdev_get_counter": (_i64, [_vp, _i]),
})

HANDLE_VAR = "__tde_psdev_handle__"     # per ps task: [session, ok, bytes_mib, IPC handle as float32 words]
REQ_VAR = "__tde_psdev_request__"       # per ps task: [session, mib] asked by the chief
PLANE_VAR = "__tde_ps_plane__"          # ps 0: the chief's decision [1.0 device | 0.0 TCP, session]
INIT_CTR = 2
MAX_SEGS = 512                         # the exchange kernel stages the segment table in LDS (kPsMaxSegsLds)
MAX_SHARDS = 16
COUNTER_BYTES = 16 * 8
SEG_DTYPE = np.dtype([("woff", "<i8"), ("loff", "<i8"), ("n", "<i8"), ("moff", "<i8"), ("win", "<i4"),
                      ("state", "<i4")])


class NoWindow(RuntimeError):
    """A ps task publishes no device window for this session (yet)."""


def enabled() -> bool:
    return os.environ.get("TDE_PS_DEVICE", "0") == "1" and torch.cuda.is_available()


def layout(store, placement: dict, nshards: int, slots: bool):
    """Shard layouts of ``store``'s variables: ``placement`` maps a variable name to its ps task.  Returns
    (segments: SEG_DTYPE array, data elements per shard).  Shard k's data area holds its trainable
    variables, then (``slots``) one momentum slot per trainable element, then its BN moving statistics."""
    names = [n for n in store.order if n in placement]
    tr = [[n for n in names if placement[n] == k and store.segments[n].trainable] for k in range(nshards)]
    st = [[n for n in names if placement[n] == k and not store.segments[n].trainable] for k in range(nshards)]
    segs, sizes = [], []
    for k in range(nshards):
        off = 0
        woffs = {}
        for n in tr[k]:
            woffs[n] = off
            off += store.segments[n].numel
        ntr = off
        if slots:
            off += ntr
        for n in tr[k]:
            seg = store.segments[n]
            segs.append((woffs[n], seg.offset, seg.numel, ntr + woffs[n] if slots else -1, k, 0))
        for n in st[k]:
            seg = store.segments[n]
            segs.append((off, seg.offset, seg.numel, -1, k, 1))
            off += seg.numel
        sizes.append(off)
    return np.array(segs, dtype=SEG_DTYPE), sizes


def shard_bytes(n_elems: int) -> int:
    return COUNTER_BYTES + 4 * int(n_elems)


# ---------------------------------------------------------------------------------------- ps task side
class WindowServer:
    """ps task side: serves this task's window on the chief's request (polled from the run loop)."""

    def __init__(self, ps_port: int, device: int = 0, index: int = 0):
        from . import ps as PS
        self.lib = N.hip()
        self.device = int(device)
        self.index = index
        self.conn = PS._Conn(f"127.0.0.1:{ps_port}")
        self.ptr = None
        self.bytes = 0
        self.session = None

    def poll(self):
        from . import ps as PS
        req = np.zeros(2, np.float32)
        names = PS._arr([REQ_VAR])
        c = self.conn
        if c.lib.tde_ps_pull(c.h, 1, names, (C.c_void_p * 1)(req.ctypes.data), (C.c_longlong * 1)(2)) != 0:
            return
        session, mib = float(req[0]), float(req[1])
        if session == self.session:
            return
        need = int(mib * 2 ** 20)
        ok = self._ensure(need)
        hb = C.create_string_buffer(self.lib.tde_xgmi_ipc_handle_bytes())
        if ok:
            rc = self._handle(hb)
            ok = rc == 0
        raw = hb.raw + b"\0" * (-len(hb.raw) % 4)
        vals = np.concatenate([np.array([session, 1.0 if ok else 0.0, self.bytes / 2 ** 20], np.float32),
                               np.frombuffer(raw, dtype=np.float32)])
        c.lib.tde_ps_init(c.h, HANDLE_VAR.encode(), vals.ctypes.data, vals.size)
        c.lib.tde_ps_assign(c.h, HANDLE_VAR.encode(), vals.ctypes.data, vals.size)
        self.session = session
        print(f"[ps] device data plane: session {int(session)}: "
              f"{'%.1f MiB window on cuda:%d' % (self.bytes / 2 ** 20, self.device) if ok else 'no window'}",
              flush=True)

    def _ensure(self, need: int) -> bool:
        """A zeroed window of >= need bytes (re-armed if the current one is big enough)."""
        if self.ptr is not None and self.bytes >= need:
            return self.lib.tde_psdev_zero(self.ptr, self.bytes) == 0
        free, _ = torch.cuda.mem_get_info(self.device)
        if need > 0.9 * free:
            print(f"[ps] device window of {need >> 20} MiB exceeds the free memory of cuda:{self.device} "
                  f"({free >> 20} MiB)", flush=True)
            return False
        if self.ptr is not None:
            self.lib.tde_psdev_free(self.ptr)
            self.ptr, self.bytes = None, 0
        p = C.c_void_p()
        self._hb = C.create_string_buffer(self.lib.tde_xgmi_ipc_handle_bytes())
        rc = self.lib.tde_psdev_alloc(self.device, need, C.byref(p), self._hb)
        if rc != 0:
            return False
        self.ptr, self.bytes = p.value, need
        return True

    def _handle(self, hb) -> int:
        C.memmove(hb, self._hb, len(self._hb.raw))
        return 0

    def close(self):
        if self.ptr is not None:
            self.lib.tde_psdev_free(self.ptr)
            self.ptr = None
        self.conn.close()


# ---------------------------------------------------------------------------------------- trainer side
def new_session() -> float:
    """A session tag that survives the float32 round trip exactly."""
    return float(random.randint(1, 2 ** 23))


def request_windows(client, sizes, session: float):
    """Chief: ask every ps task for a window of its shard's bytes, tagged ``session``."""
    for k, c in enumerate(client.conns):
        req = np.array([session, shard_bytes(sizes[k]) / 2 ** 20 + 1e-3], np.float32)
        c.lib.tde_ps_init(c.h, REQ_VAR.encode(), req.ctypes.data, 2)
        c.lib.tde_ps_assign(c.h, REQ_VAR.encode(), req.ctypes.data, 2)


class DevicePlane:
    """Trainer side of the sharded windows for one ParamStore (flat ``w`` / ``state`` / ``g``).

    ``kind``: 0 SGD, 1 momentum, 2 Nesterov (``momentum`` = the optimizer's).  ``session``: the tag of the
    windows to map (the chief's ``request_windows``); waits up to ``timeout`` s for every ps task's handle."""

    def __init__(self, client, store, bn_momentum: dict, lr: float, kind: int = 0, momentum: float = 0.0,
                 session: float | None = None, timeout: float = 30.0):
        from . import ps as PS
        self.lib = N.hip()
        self.store = store
        dev = store.device
        if dev.type != "cuda":
            raise RuntimeError("the device data plane needs the model on a GPU")
        if kind not in (0, 1, 2):
            raise RuntimeError("the device data plane applies SGD / momentum / Nesterov only")
        if len(client.conns) > MAX_SHARDS:
            raise RuntimeError(f"the device data plane supports at most {MAX_SHARDS} ps tasks")
        self.kind, self.mmt, self.lr = int(kind), float(momentum), float(lr)
        segs, sizes = layout(store, client.placement, len(client.conns), slots=self.kind != 0)
        if len(segs) > MAX_SEGS:
            # raised before any window is mapped: the chief falls back to the TCP plane
            raise RuntimeError(f"{len(segs)} variable segments; the device exchange stages at most {MAX_SEGS}")
        if segs.dtype.itemsize != self.lib.tde_psdev_seg_bytes():
            raise RuntimeError("segment table layout differs from the kernel's PsSeg")
        self.sizes = sizes
        nbytes = self.lib.tde_xgmi_ipc_handle_bytes()
        nh = 3 + (-(-nbytes // 4))
        self.wins, self._opened = [], []
        try:
            for k, c in enumerate(client.conns):
                buf = np.zeros(nh, np.float32)
                names = PS._arr([HANDLE_VAR])
                t0 = time.time()
                while True:
                    got = c.lib.tde_ps_pull(c.h, 1, names, (C.c_void_p * 1)(buf.ctypes.data),
                                            (C.c_longlong * 1)(nh)) == 0
                    if got and (session is None or float(buf[0]) == session):
                        break
                    if time.time() - t0 > timeout:
                        raise NoWindow(f"ps task {k} publishes no device window for session {session} "
                                       "(TDE_PS_DEVICE unset on the ps task?)")
                    time.sleep(0.02)
                if buf[1] != 1.0:
                    raise NoWindow(f"ps task {k} could not allocate its {shard_bytes(sizes[k]) >> 20} MiB window")
                if shard_bytes(sizes[k]) > float(buf[2]) * 2 ** 20 + 1:
                    raise RuntimeError(f"ps task {k}'s window ({buf[2]:.1f} MiB) is smaller than its shard")
                m = C.c_void_p()
                rc = self.lib.tde_xgmi_open(dev.index, buf[3:].tobytes()[:nbytes], C.byref(m))
                if rc != 0:
                    raise RuntimeError(f"hipIpcOpenMemHandle of ps task {k}'s window failed ({rc})")
                self._opened.append(m.value)
                self.wins.append(m.value)
        except Exception:
            self.close()
            raise
        self.win = self.wins[0]           # ps 0's window: the counters
        self._wins = (C.c_void_p * len(self.wins))(*self.wins)
        self.segs_host = segs
        self.nseg = len(segs)
        self.maxn = int(segs["n"].max()) if len(segs) else 0
        self.segs = torch.from_numpy(segs.view(np.uint8).copy()).to(dev)
        beg = np.zeros(len(segs) + 1, np.int64)
        beg[1:] = np.cumsum(segs["n"]) if len(segs) else []
        self.total = int(beg[-1])
        self.beg = torch.from_numpy(beg).to(dev)   # the exchange's flat element index -> segment
        self.nw, self.ns = store.w.numel(), store.state.numel()
        mom = np.zeros(max(self.ns, 1), np.float32)
        for name, mm in bn_momentum.items():
            seg = store.segments[name]
            mom[seg.offset: seg.offset + seg.numel] = mm
        self.mom = torch.from_numpy(mom).to(dev)
        self.sp = torch.zeros(max(self.ns, 1), dtype=torch.float32, device=dev)
        self.done = torch.zeros(1, dtype=torch.int32, device=dev)
        self._claim = torch.zeros(1, dtype=torch.int64, device=dev)   # pipelined loop: this step's ticket
        h, d = C.c_void_p(), C.c_void_p()
        if self.lib.tde_host_mapped_alloc(16, C.byref(h), C.byref(d)) != 0:
            raise RuntimeError("host-mapped result words")
        self._out_h, self._out_d = h.value, d.value
        self._out = (C.c_longlong * 2).from_address(self._out_h)

    def close(self):
        for m in getattr(self, "_opened", []):
            self.lib.tde_xgmi_close(m)
        self._opened = []
        self.win = None
        if getattr(self, "_out_h", None):
            self.lib.tde_host_mapped_free(self._out_h)
            self._out_h = None

    # ------------------------------------------------------------------ control
    def initialized(self) -> bool:
        return self.lib.tde_psdev_get_counter(self.win, INIT_CTR) == 1

    def initialize(self, global_step: int, tickets: int):
        """Chief: the store's values (fresh or restored) and the counters become the PS state; the
        "initialised" counter goes to 1 only after every shard holds them."""
        st = self.store
        self.lib.tde_psdev_set_counter(self.win, INIT_CTR, 0)
        with torch.cuda.device(st.device):
            N.check(self.lib.tde_psdev_copy(self._wins, len(self.wins), N.ptr(self.segs), self.nseg, self.maxn,
                                            N.ptr(st.w), N.ptr(st.state), 0, N.stream_ptr()), "tde_psdev_copy")
            torch.cuda.synchronize(st.device)
        self.lib.tde_psdev_set_counter(self.win, 0, int(global_step))
        self.lib.tde_psdev_set_counter(self.win, 1, int(tickets))
        self.lib.tde_psdev_set_counter(self.win, INIT_CTR, 1)

    def end_session(self):
        """Chief, at session end: the windows stop counting as initialised, so a trainer of a later session
        that maps them before that session's chief re-arms them waits instead of claiming stale tickets."""
        if self.win is not None:
            self.lib.tde_psdev_set_counter(self.win, INIT_CTR, 0)

    def wait_initialized(self, timeout=120.0):
        t0 = time.time()
        while not self.initialized():
            if time.time() - t0 > timeout:
                raise TimeoutError("the chief never initialised the PS device windows")
            time.sleep(0.02)

    def global_step(self) -> int:
        return int(self.lib.tde_psdev_get_counter(self.win, 0))

    def tickets(self) -> int:
        return int(self.lib.tde_psdev_get_counter(self.win, 1))

    def counter_add(self, idx: int, d: int) -> int:
        """Host-side counter add (a 1-block exchange with nothing to push): returns the new value."""
        self._launch(push=False, dstep=d if idx == 0 else 0, dticket=d if idx == 1 else 0, pull=False)
        return self._out[idx]

    # ------------------------------------------------------------------ data
    def pull(self):
        """The PS's current values into the local store (and the BN reference copy)."""
        self._launch(push=False, dstep=0, dticket=0)

    def step(self, dstep=1, dticket=0):
        """Push this step's gradients / BN statistics, pull fresh values, advance the counters.
        Returns (global step, tickets) after this step."""
        self._launch(push=True, dstep=dstep, dticket=dticket)
        return int(self._out[0]), int(self._out[1])

    def set_claim(self, ticket: int):
        """Pipelined loop: the ticket the next pushed step was computed under (stream-ordered write)."""
        self._claim.fill_(int(ticket))

    def step_async(self, max_steps: int):
        """Pipelined loop: push + pull + counters WITHOUT waiting.  The kernel drops a push whose ticket
        (``set_claim``, then the one each live push claims) exceeds ``max_steps``, so the host may run ahead
        of the counters it has seen.  Returns the (global step, this trainer's next ticket) of the latest
        exchange the device has finished (host-mapped words, possibly a few steps old)."""
        self._launch(push=True, dstep=1, dticket=1, sync=False, limit=int(max_steps))
        return self.observed()

    def observed(self):
        return int(self._out[0]), int(self._out[1])

    def _launch(self, push, dstep, dticket, pull=True, sync=True, limit=0):
        st = self.store
        with torch.cuda.device(st.device):
            s = N.stream_ptr()
            nseg = self.nseg if pull else 0
            rc = self.lib.tde_psdev_step(self._wins, len(self.wins), N.ptr(self.segs) if nseg else None,
                                         N.ptr(self.beg) if nseg else None, nseg, self.total if nseg else 0,
                                         N.ptr(st.w), N.ptr(st.g) if push else None,
                                         N.ptr(st.state) if self.ns else None, N.ptr(self.sp), N.ptr(self.mom),
                                         self.lr, self.mmt, self.kind, int(dstep), int(dticket), N.ptr(self.done),
                                         self._out_d, N.ptr(self._claim) if limit > 0 else None, int(limit), s)
            N.check(rc, "tde_psdev_step")
            if sync:
                torch.cuda.current_stream(st.device).synchronize()
