"""Python binding of the native TCP key-value store (csrc/comm/tcp_store.cpp):
rendezvous, barriers, heartbeat-based failure detection.

    server = TCPStoreServer(port=0)            # chief
    st = TCPStore("127.0.0.1", server.port)    # everyone
    st.set("rccl_id", uid); st.get("rccl_id", timeout=30)
    st.barrier("init", world)
    hb = Heartbeat(st, "worker:1", interval=0.5).start()
    st.dead_members(timeout=3.0)               # -> ["worker:2"] if it stopped beating
"""
from __future__ import annotations

import ctypes as C
import re
import threading
import time

from .. import _native as N

N.register_host({
    "tde_store_server_start": (C.c_void_p, [C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
    "tde_store_server_stop": (None, [C.c_void_p]),
    "tde_store_connect": (C.c_void_p, [C.c_char_p, C.c_int, C.c_int]),
    "tde_store_close": (None, [C.c_void_p]),
    "tde_store_set": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int]),
    "tde_store_get": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "tde_store_wait": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "tde_store_add": (C.c_longlong, [C.c_void_p, C.c_char_p, C.c_longlong]),
    "tde_store_check": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tde_store_delete": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tde_store_heartbeat": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tde_store_dead": (C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_int]),
    "tde_store_num_keys": (C.c_longlong, [C.c_void_p]),
    "tde_store_barrier": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.c_int]),
})


class StoreTimeout(TimeoutError):
    pass


class StoreError(ConnectionError):
    pass


class TCPStoreServer:
    def __init__(self, host="0.0.0.0", port=0):
        lib = N.host()
        p = C.c_int()
        self._h = lib.tde_store_server_start(host.encode(), int(port), C.byref(p))
        if not self._h:
            raise OSError(f"cannot listen on {host}:{port}")
        self.port = p.value

    def stop(self):
        if self._h:
            N.host().tde_store_server_stop(self._h)
            self._h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


class TCPStore:
    def __init__(self, host, port, timeout=60.0):
        self._lib = N.host()
        self._h = self._lib.tde_store_connect(host.encode(), int(port), int(timeout * 1000))
        if not self._h:
            raise StoreError(f"cannot connect to store {host}:{port}")
        self._lock = threading.Lock()

    def close(self):
        if self._h:
            self._lib.tde_store_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set(self, key: str, value):
        b = value if isinstance(value, (bytes, bytearray)) else str(value).encode()
        if self._lib.tde_store_set(self._h, key.encode(), bytes(b), len(b)) != 0:
            raise StoreError("set failed")

    def get(self, key: str, timeout=60.0) -> bytes:
        # the value is fetched whole into a buffer of the last size seen for keys of the same family (the key
        # with its digits masked: round / rank counters vary, the payload kind does not), so large values such
        # as CPU all-reduce parts take one round trip each while small control-plane values (barrier, agree,
        # broadcast_json) keep a 64 KiB buffer
        fam = re.sub(r"\d+", "#", key)
        caps = self.__dict__.setdefault("_caps", {})
        cap = caps.get(fam, 1 << 16)
        while True:
            buf = C.create_string_buffer(cap)
            n = self._lib.tde_store_get(self._h, key.encode(), buf, cap, int(timeout * 1000) if timeout else -1)
            if n == -2:
                raise StoreTimeout(f"timed out waiting for key {key!r}")
            if n < 0:
                raise StoreError("get failed")
            if n <= cap:
                return buf.raw[:n]
            cap = caps[fam] = n

    def wait(self, key: str, timeout=60.0):
        rc = self._lib.tde_store_wait(self._h, key.encode(), int(timeout * 1000))
        if rc == -2:
            raise StoreTimeout(f"timed out waiting for key {key!r}")
        if rc != 0:
            raise StoreError("wait failed")

    def add(self, key: str, delta: int = 1) -> int:
        v = self._lib.tde_store_add(self._h, key.encode(), int(delta))
        if v == -(2 ** 63):
            raise StoreError("add failed")
        return v

    def check(self, key: str) -> bool:
        return self._lib.tde_store_check(self._h, key.encode()) == 1

    def delete(self, key: str) -> bool:
        return self._lib.tde_store_delete(self._h, key.encode()) == 1

    def num_keys(self) -> int:
        return self._lib.tde_store_num_keys(self._h)

    def barrier(self, name: str, world: int, timeout=120.0):
        rc = self._lib.tde_store_barrier(self._h, name.encode(), int(world), int(timeout * 1000))
        if rc == -2:
            raise StoreTimeout(f"barrier {name!r} timed out")
        if rc != 0:
            raise StoreError("barrier failed")

    def heartbeat(self, member_id: str):
        if self._lib.tde_store_heartbeat(self._h, member_id.encode()) != 0:
            raise StoreError("heartbeat failed: store unreachable")

    def dead_members(self, timeout: float) -> list:
        buf = C.create_string_buffer(1 << 16)
        n = self._lib.tde_store_dead(self._h, int(timeout * 1000), buf, 1 << 16)
        if n < 0:
            raise StoreError("dead query failed")
        return [s for s in buf.raw[:n].decode().split("\n") if s]


class Heartbeat:
    """Background thread beating ``member_id`` into the store every ``interval`` s."""

    def __init__(self, host, port, member_id, interval=0.5):
        self.store = TCPStore(host, port)
        self.member_id = member_id
        self.interval = interval
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name=f"tde-heartbeat-{member_id}")

    def _run(self):
        while not self._stop.is_set():
            try:
                self.store.heartbeat(self.member_id)
            except Exception:
                return
            self._stop.wait(self.interval)

    def start(self):
        self.store.heartbeat(self.member_id)
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        self._t.join(timeout=2)
        self.store.close()
