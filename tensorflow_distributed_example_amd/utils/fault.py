"""Fault injection for the failure-detection tests.

``TDE_FAULT="task=worker:1,step=7,kind=exit"`` (or ``rank=1`` instead of ``task=``) makes the
matching process fail when its training loop reaches ``step``:

* ``exit``  — ``os._exit(code)`` (default code 13): a crashed worker;
* ``hang``  — stop heartbeating and block forever: a wedged worker;
* ``raise`` — raise ``InjectedFault`` from the training loop (a Python-level error).

The reference has no fault handling of its own; TF's runtime surfaces a dead peer as an
error in the next collective (or a PS ``Unavailable`` retried by MonitoredTrainingSession).
"""
from __future__ import annotations

import os
import sys
import threading
import time


class InjectedFault(RuntimeError):
    pass


_lock = threading.Lock()
_fired = False
_hooks = []          # callables run before a hang (e.g. stop the heartbeat thread)


def on_hang(fn):
    _hooks.append(fn)


def parse(spec: str) -> dict:
    out = {}
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip()
    return out


def _me():
    from ..parallel import cluster as CL
    cfg = CL.tf_config()
    task = cfg.get("task") if cfg else None
    ttype = task.get("type") if task else None
    tidx = int(task.get("index", 0)) if task else 0
    rank = int(os.environ.get("RANK", "-1"))
    if rank < 0:
        try:
            rank = CL.worker_topology().rank
        except ValueError:
            rank = -1
    return ttype, tidx, rank


def matches(cfg: dict) -> bool:
    ttype, tidx, rank = _me()
    if "task" in cfg:
        job, _, idx = cfg["task"].partition(":")
        return job == ttype and int(idx or 0) == tidx
    if "rank" in cfg:
        return int(cfg["rank"]) == rank
    return True


def maybe_inject(step: int):
    """Called by the training loops after each executed step (group)."""
    global _fired
    spec = os.environ.get("TDE_FAULT")
    if not spec or _fired:
        return
    cfg = parse(spec)
    if step < int(cfg.get("step", 0)) or not matches(cfg):
        return
    with _lock:
        if _fired:
            return
        _fired = True
    kind = cfg.get("kind", "exit")
    print(f"[tde.fault] injecting '{kind}' at step {step} ({spec})", file=sys.stderr, flush=True)
    if kind == "exit":
        os._exit(int(cfg.get("code", 13)))
    if kind == "hang":
        for fn in _hooks:
            try:
                fn()
            except Exception:
                pass
        while True:
            time.sleep(3600)
    raise InjectedFault(f"injected fault at step {step}")
