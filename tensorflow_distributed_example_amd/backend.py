"""Global framework state: devices, dtype policy, learning phase, layer uids, seeds.

Keras-backend equivalents used by the reference:
  * ``set_learning_phase`` — mnist_keras_distributed.py:116, tf2_mnist_distributed.py:142
    (quirk Q4: a global training-phase override that also affects eval/export).
  * layer auto-naming (``conv2d``, ``conv2d_1``, ...) — used for checkpoint keys.
  * dtype policy: ``float32`` by default, the reference's precision (Keras default;
    distributed_with_keras.py:21 casts the images to float32): the fused GPU plans then
    run their exact-f32 MFMA kernel forms.  ``mixed_bfloat16`` (fp32 master weights,
    bf16 MFMA compute) is the opt-in fast path the bf16 BASELINE configs ask for.
"""
from __future__ import annotations

import collections
import os
import random

import numpy as np
import torch

_uids = collections.defaultdict(int)
_learning_phase = None  # None = follow `training` argument; True/False = forced (Q4)
_policy = None
_seed = None


# ----------------------------------------------------------------------------- naming
def get_uid(prefix: str) -> int:
    n = _uids[prefix]
    _uids[prefix] += 1
    return n


def unique_name(prefix: str) -> str:
    n = get_uid(prefix)
    return prefix if n == 0 else f"{prefix}_{n}"


def clear_session():
    global _learning_phase
    _uids.clear()
    _learning_phase = None


# ----------------------------------------------------------------------------- phase
def set_learning_phase(value):
    """Force training (1/True) or inference (0/False) behaviour globally (Q4)."""
    global _learning_phase
    _learning_phase = None if value is None else bool(value)


def learning_phase():
    return _learning_phase


def resolve_training(training: bool) -> bool:
    return training if _learning_phase is None else _learning_phase


# ----------------------------------------------------------------------------- devices
def gpu_available() -> bool:
    return torch.cuda.is_available()


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


_default_devices = None   # --devices: what a strategy built without devices uses


def set_default_devices(devices):
    """Devices strategies use when constructed without an explicit list (``--devices``): a list of
    ``"cpu"`` / ``"gpu:N"`` / ``"cuda:N"`` strings or torch devices, or None for all local GPUs (else CPU)."""
    global _default_devices
    _default_devices = None if devices is None else [str(d).strip() for d in devices if str(d).strip()]


def default_devices():
    return _default_devices


def parse_device(spec: str) -> torch.device:
    """``cpu`` / ``/cpu:0`` / ``gpu:N`` / ``/gpu:N`` / ``cuda:N`` (``--devices`` entries) -> torch device."""
    d = str(spec).strip().lower().lstrip("/")
    if d.startswith("device:"):
        d = d[len("device:"):]
    if d.startswith("cpu"):
        return torch.device("cpu")
    for pre in ("gpu", "cuda"):
        if d.startswith(pre):
            rest = d[len(pre):].lstrip(":")
            return torch.device("cuda", int(rest) if rest else 0)
    raise ValueError(f"unknown device {spec!r} (cpu, gpu:N, cuda:N)")


def default_device() -> torch.device:
    if _default_devices:
        # the first --devices entry (the Estimator paths build OneDeviceStrategy(default_device()))
        return parse_device(_default_devices[0])
    if gpu_available():
        n = torch.cuda.device_count()
        return torch.device("cuda", local_rank() % max(n, 1))
    return torch.device("cpu")


# ----------------------------------------------------------------------------- policy
class Policy:
    def __init__(self, name: str):
        if name not in ("float32", "mixed_bfloat16"):
            raise ValueError(f"unsupported policy {name!r}")
        self.name = name
        self.variable_dtype = torch.float32
        self.compute_dtype = torch.bfloat16 if name == "mixed_bfloat16" else torch.float32

    def __repr__(self):
        return f"<Policy {self.name}>"


def set_global_policy(name):
    """``"float32"`` | ``"mixed_bfloat16"`` | a Policy | None (back to the default, float32)."""
    global _policy
    _policy = Policy(name) if isinstance(name, str) else name


def global_policy() -> Policy:
    if _policy is None:
        return Policy(os.environ.get("TDE_POLICY", "float32"))
    return _policy


# ----------------------------------------------------------------------------- seeds
def set_random_seed(seed: int):
    global _seed
    _seed = int(seed)
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


def get_seed():
    return _seed


def make_generator(offset: int = 0) -> torch.Generator:
    g = torch.Generator()
    base = _seed if _seed is not None else int.from_bytes(os.urandom(4), "little")
    g.manual_seed(base + offset)
    return g


def floatx():
    return "float32"
