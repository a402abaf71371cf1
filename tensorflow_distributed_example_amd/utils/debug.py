"""Race / divergence detection for data-parallel training.

* ``replica_fingerprints(model)`` / ``check_replicas(model)`` — the replica-consistency checker:
  every replica's flat weight bucket is hashed on its device (a 64-bit fold of the raw float bits —
  bitwise, not approximate) and the fingerprints of ALL replicas of ALL workers are compared; data
  parallelism keeps replicas bit-identical, so any difference means a missing stream/event
  dependency between compute and the gradient all-reduce, a non-deterministic update, or a
  corrupted collective.  ``ReplicaConsistencyCheck`` runs it from ``fit`` every N epochs, and
  ``TDE_CHECK_REPLICAS=N`` does so every N executions.
* ``TDE_DEBUG_SYNC=1`` — serialised-kernel debugging: ``AMD_SERIALIZE_KERNEL=3`` /
  ``HIP_LAUNCH_BLOCKING=1`` for the HIP runtime (set before the first HIP call), hipGraph capture
  off and a device synchronisation after every plan call, so an asynchronous fault surfaces at the
  launch that caused it.
"""
from __future__ import annotations

import os

import torch


class ReplicaDivergence(RuntimeError):
    pass


def debug_sync_enabled() -> bool:
    return os.environ.get("TDE_DEBUG_SYNC", "0") not in ("", "0")


def apply_debug_env():
    """Called at package import (before any HIP call) when TDE_DEBUG_SYNC is set."""
    if debug_sync_enabled():
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
        os.environ["TDE_GRAPH"] = "0"


def _fold(t: torch.Tensor) -> int:
    """64-bit fingerprint of the raw bits of a float32 tensor (position-weighted, order-sensitive)."""
    bits = t.detach().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    idx = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64)
    mixed = (bits * (idx * 2654435761 + 97)) ^ (bits << 13)
    return int(mixed.sum().item()) & ((1 << 63) - 1)


def replica_fingerprints(model) -> list:
    """[(worker, local replica, weights fp, BN-state fp)] for every replica of every worker."""
    st = model._strategy
    stores = model._stores.get(id(st)) if st is not None else None
    stores = stores or [model._store]
    local = [(_fold(s.w), _fold(s.state)) for s in stores]
    if st is None or st.num_workers == 1:
        return [(0, i, w, b) for i, (w, b) in enumerate(local)]
    allv = st.control.all_gather_json(local, "fingerprints")
    return [(r, i, w, b) for r, lst in enumerate(allv) for i, (w, b) in enumerate(lst)]


def check_replicas(model, what="weights"):
    """Raise unless every replica holds bit-identical trainable variables.  BN moving statistics are
    not compared: they are SyncOnRead (MEAN) variables that each replica updates from its own slice of
    the batch (mnist_keras_distributed.py:86 under a strategy), so they legitimately differ."""
    fps = replica_fingerprints(model)
    ref = fps[0]
    bad = [f for f in fps if f[2] != ref[2]]
    if bad:
        raise ReplicaDivergence(
            f"replicas diverged ({what}): reference worker {ref[0]}/replica {ref[1]} "
            f"fp={ref[2]:#x}/{ref[3]:#x}; differing: " +
            ", ".join(f"worker {w}/replica {r} fp={a:#x}/{b:#x}" for w, r, a, b in bad))
    return fps


from ..train.callbacks import Callback  # noqa: E402


class ReplicaConsistencyCheck(Callback):
    """Keras callback: assert all replicas are bit-identical every ``every_n_epochs`` epochs."""

    def __init__(self, every_n_epochs=1):
        super().__init__()
        self.n = max(1, int(every_n_epochs))

    def on_epoch_end(self, epoch, logs=None):
        if (epoch + 1) % self.n == 0:
            check_replicas(self.model, f"after epoch {epoch + 1}")
