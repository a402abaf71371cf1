"""Same-node GPU data plane of ``ParameterServerStrategy`` (csrc/kernels/ps_device.hip; SURVEY.md F07 /
§5.8 "optional same-node fast path"; reference mnist_keras_distributed.py:242, tf2_mnist_distributed.py:189).

ps task 0 allocates ONE device window holding the model's flat variable buffers and the PS counters and
publishes its IPC handle through its own TCP variable table.  Trainers map the window and run each async
step's exchange as one kernel (push with f32 atomics, BN moving averages by compare-and-swap, pull, counter
advance); the host only reads two host-mapped words after the step's stream sync.  TCP keeps the control
plane (initialisation flag of the TCP tables, the handle) — no variable bytes cross it.

Enabled with ``TDE_PS_DEVICE=1`` (ps task and trainers on one node with GPUs); the optimizer must be plain
SGD (the PS update is an atomic add); otherwise the host-staged TCP plane (``PSClient.step``) runs.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np
import torch

from .. import _native as N

_vp, _i, _i64, _f = C.c_void_p, C.c_int, C.c_longlong, C.c_float
N.register_hip({
    "tde_psdev_counters": (_i, []),
    "tde_psdev_alloc": (_i, [_i, _i64, C.POINTER(_vp), C.c_char_p]),
    "tde_psdev_free": (_i, [_vp]),
    "tde_host_mapped_alloc": (_i, [_i64, C.POINTER(_vp), C.POINTER(_vp)]),
    "tde_host_mapped_free": (_i, [_vp]),
    "tde_psdev_step": (_i, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _f, _i64, _i64, _vp, _vp, _vp]),
    "tde_psdev_copy": (_i, [_vp, _i64, _i64, _vp, _vp, _i, _vp]),
    "tde_psdev_set_counter": (_i, [_vp, _i, _i64]),
    "tde_psdev_get_counter": (_i64, [_vp, _i]),
})

HANDLE_VAR = "__tde_psdev_handle__"     # TCP variable of ps task 0 carrying the window's IPC handle
PLANE_VAR = "__tde_ps_plane__"          # the chief's decision: 1.0 device plane, 0.0 TCP plane
INIT_CTR = 2


class NoWindow(RuntimeError):
    """ps task 0 publishes no device window (yet)."""


def enabled() -> bool:
    return os.environ.get("TDE_PS_DEVICE", "0") == "1" and torch.cuda.is_available()


def window_bytes() -> int:
    return int(float(os.environ.get("TDE_PS_WINDOW_MB", "64")) * 2 ** 20)


def serve_window(ps_port: int, device: int = 0):
    """ps task side: allocate the window and publish its handle as a float32 variable of this ps task's own
    TCP table.  Returns the window pointer (kept for the life of the ps process) or None."""
    from . import ps as PS
    lib = N.hip()
    ptr = C.c_void_p()
    hb = C.create_string_buffer(N.hip().tde_xgmi_ipc_handle_bytes())
    rc = lib.tde_psdev_alloc(int(device), window_bytes(), C.byref(ptr), hb)
    if rc != 0:
        print(f"[ps] device data plane unavailable (alloc rc {rc}); TCP plane only", flush=True)
        return None
    raw = hb.raw + b"\0" * (-len(hb.raw) % 4)
    vals = np.frombuffer(raw, dtype=np.float32).copy()
    conn = PS._Conn(f"127.0.0.1:{ps_port}")
    conn.lib.tde_ps_init(conn.h, HANDLE_VAR.encode(), vals.ctypes.data, vals.size)
    conn.close()
    print(f"[ps] device data plane: {window_bytes() >> 20} MiB window on cuda:{device}", flush=True)
    return ptr


class DevicePlane:
    """Trainer side of the window for one ParamStore (flat ``w`` / ``state`` / ``g``)."""

    def __init__(self, client, store, bn_momentum: dict, lr: float):
        from . import ps as PS
        self.lib = N.hip()
        self.store = store
        dev = store.device
        if dev.type != "cuda":
            raise RuntimeError("the device data plane needs the model on a GPU")
        nbytes = self.lib.tde_xgmi_ipc_handle_bytes()
        n = -(-nbytes // 4)
        buf = np.zeros(n, np.float32)
        c0 = client.conns[0]
        names = PS._arr([HANDLE_VAR])
        ok = c0.lib.tde_ps_pull(c0.h, 1, names, (C.c_void_p * 1)(buf.ctypes.data), (C.c_longlong * 1)(n)) == 0
        if not ok:
            raise NoWindow("ps task 0 publishes no device window (TDE_PS_DEVICE unset on the ps task?)")
        self.nw, self.ns = store.w.numel(), store.state.numel()
        ncnt = self.lib.tde_psdev_counters()
        if (ncnt * 8 + 4 * (self.nw + self.ns)) > window_bytes():
            raise RuntimeError(f"model ({self.nw + self.ns} floats) exceeds the device window (TDE_PS_WINDOW_MB)")
        m = C.c_void_p()
        rc = self.lib.tde_xgmi_open(dev.index, buf.tobytes()[:nbytes], C.byref(m))
        if rc != 0:
            raise RuntimeError(f"hipIpcOpenMemHandle of the PS window failed ({rc})")
        self.win = m.value
        mom = np.zeros(max(self.ns, 1), np.float32)
        for name, mm in bn_momentum.items():
            seg = store.segments[name]
            mom[seg.offset: seg.offset + seg.numel] = mm
        self.mom = torch.from_numpy(mom).to(dev)
        self.sp = torch.zeros(max(self.ns, 1), dtype=torch.float32, device=dev)
        self.done = torch.zeros(1, dtype=torch.int32, device=dev)
        h, d = C.c_void_p(), C.c_void_p()
        if self.lib.tde_host_mapped_alloc(16, C.byref(h), C.byref(d)) != 0:
            raise RuntimeError("host-mapped result words")
        self._out_h, self._out_d = h.value, d.value
        self._out = (C.c_longlong * 2).from_address(self._out_h)
        self.lr = float(lr)

    def close(self):
        if getattr(self, "win", None):
            self.lib.tde_xgmi_close(self.win)
            self.win = None
        if getattr(self, "_out_h", None):
            self.lib.tde_host_mapped_free(self._out_h)
            self._out_h = None

    # ------------------------------------------------------------------ control
    def initialized(self) -> bool:
        return self.lib.tde_psdev_get_counter(self.win, INIT_CTR) == 1

    def initialize(self, global_step: int, tickets: int):
        """Chief: the store's values (fresh or restored) and the counters become the PS state."""
        st = self.store
        with torch.cuda.device(st.device):
            N.check(self.lib.tde_psdev_copy(self.win, self.nw, self.ns, N.ptr(st.w), N.ptr(st.state), 0,
                                            N.stream_ptr()), "tde_psdev_copy")
            torch.cuda.synchronize(st.device)
        self.lib.tde_psdev_set_counter(self.win, 0, int(global_step))
        self.lib.tde_psdev_set_counter(self.win, 1, int(tickets))
        self.lib.tde_psdev_set_counter(self.win, INIT_CTR, 1)

    def wait_initialized(self, timeout=120.0):
        t0 = time.time()
        while not self.initialized():
            if time.time() - t0 > timeout:
                raise TimeoutError("the chief never initialised the PS device window")
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

    def _launch(self, push, dstep, dticket, pull=True):
        st = self.store
        with torch.cuda.device(st.device):
            s = N.stream_ptr()
            if pull:
                rc = self.lib.tde_psdev_step(self.win, self.nw, self.ns, N.ptr(st.w), N.ptr(st.g) if push else None,
                                             N.ptr(st.state) if self.ns else None, N.ptr(self.sp), N.ptr(self.mom),
                                             self.lr, int(dstep), int(dticket), N.ptr(self.done), self._out_d, s)
            else:   # counters only
                rc = self.lib.tde_psdev_step(self.win, 0, 0, N.ptr(st.w), None, None, None, None, 0.0, int(dstep),
                                             int(dticket), N.ptr(self.done), self._out_d, s)
            N.check(rc, "tde_psdev_step")
            torch.cuda.current_stream(st.device).synchronize()
