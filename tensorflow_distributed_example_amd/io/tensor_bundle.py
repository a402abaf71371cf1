"""TensorFlow TensorBundle checkpoints via the native C++ writer/reader
(csrc/io/tensor_bundle.cpp) + the ``checkpoint`` state file (text proto).

Variable names are the TF1/Keras graph names (``conv2d/kernel``, ``dense_1/bias``,
``batch_normalization/moving_mean``, ``global_step``) that an Estimator built by
``model_to_estimator`` writes; layouts are Keras-native
(HWIO conv kernels, [in, out] dense kernels), so no transposes are needed.
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

import numpy as np

from .. import _native as N

_DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3, np.dtype("uint8"): 4,
       np.dtype("int64"): 9, np.dtype("float16"): 19}
_DT_INV = {v: k for k, v in _DT.items()}
DT_BFLOAT16 = 14
DT_STRING = 7

N.register_host({
    "tde_bundle_write": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.POINTER(C.c_longlong), C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_longlong)]),
    "tde_bundle_open": (C.c_void_p, [C.c_char_p]),
    "tde_bundle_close": (None, [C.c_void_p]),
    "tde_bundle_count": (C.c_int, [C.c_void_p]),
    "tde_bundle_entry": (C.c_int, [C.c_void_p, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "tde_bundle_read": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_longlong]),
})


def write_bundle(prefix: str, tensors: dict):
    """Write {name: ndarray} as <prefix>.index + <prefix>.data-00000-of-00001."""
    lib = N.host()
    Path(prefix).parent.mkdir(parents=True, exist_ok=True)
    names = list(tensors)
    # a ``bytes`` value is a scalar DT_STRING tensor (TensorBundle string encoding, io/object_graph.py)
    strs = {n for n in names if isinstance(tensors[n], (bytes, bytearray))}
    from .object_graph import encode_string_tensor
    arrs = [np.frombuffer(encode_string_tensor([tensors[n]]), dtype=np.uint8) if n in strs else
            np.require(np.asarray(tensors[n]), requirements="C") for n in names]
    n = len(names)
    c_names = (C.c_char_p * n)(*[s.encode() for s in names])
    dtypes = (C.c_int * n)(*[DT_STRING if nm in strs else _DT[a.dtype] for nm, a in zip(names, arrs)])
    ranks = (C.c_int * n)(*[0 if nm in strs else a.ndim for nm, a in zip(names, arrs)])
    flat = [d for nm, a in zip(names, arrs) if nm not in strs for d in a.shape]
    shapes = (C.c_longlong * max(len(flat), 1))(*flat)
    datas = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
    nbytes = (C.c_longlong * n)(*[a.nbytes for a in arrs])
    rc = lib.tde_bundle_write(str(prefix).encode(), n, c_names, dtypes, ranks, shapes, datas, nbytes)
    if rc != 0:
        raise IOError(f"tde_bundle_write({prefix}) failed: {rc}")


def list_variables(prefix: str):
    lib = N.host()
    h = lib.tde_bundle_open(str(prefix).encode())
    if not h:
        raise IOError(f"cannot open TensorBundle {prefix}")
    out = []
    try:
        for i in range(lib.tde_bundle_count(h)):
            name = C.create_string_buffer(1024)
            dt, rank = C.c_int(), C.c_int()
            shape = (C.c_longlong * 16)()
            nb = C.c_longlong()
            lib.tde_bundle_entry(h, i, name, 1024, C.byref(dt), C.byref(rank), shape, C.byref(nb))
            out.append((name.value.decode(), tuple(shape[:rank.value]), dt.value, nb.value))
    finally:
        lib.tde_bundle_close(h)
    return out


def read_bundle(prefix: str, skip_bad_strings: bool | None = None) -> dict:
    """Every tensor of the bundle at ``prefix`` ({key: array}; scalar string tensors decoded).  A string
    tensor that fails its checksum or does not parse raises — except, by default (``None``), the TF2 object
    graph (``_CHECKPOINTABLE_OBJECT_GRAPH``: metadata only, restore matches variables by key without it),
    which is skipped with a warning naming it.  ``True`` skips (with the warning) every unreadable string
    tensor, ``False`` skips none."""
    import warnings

    from .object_graph import GRAPH_KEY
    lib = N.host()
    entries = list_variables(prefix)
    h = lib.tde_bundle_open(str(prefix).encode())
    out = {}
    try:
        for name, shape, dt, nb in entries:
            if dt == DT_STRING and not shape:
                raw = (C.c_char * nb)()
                rc = lib.tde_bundle_read(h, name.encode(), raw, nb)
                from .object_graph import decode_string_tensor
                try:
                    if rc != 0:
                        raise IOError(f"{prefix}: reading {name} failed ({'crc mismatch' if rc == -3 else rc})")
                    out[name] = decode_string_tensor(bytes(raw))[0]
                except (IOError, ValueError, IndexError) as e:
                    if not (skip_bad_strings or (skip_bad_strings is None and name == GRAPH_KEY)):
                        raise IOError(f"{prefix}: string tensor {name!r} is unreadable ({e})") from e
                    warnings.warn(f"{prefix}: skipping unreadable string tensor {name!r} ({e})")
                continue
            if dt not in _DT_INV:
                continue
            a = np.empty(shape, dtype=_DT_INV[dt])
            rc = lib.tde_bundle_read(h, name.encode(), a.ctypes.data, a.nbytes)
            if rc != 0:
                raise IOError(f"{prefix}: reading {name} failed ({'crc mismatch' if rc == -3 else rc})")
            out[name] = a
    finally:
        lib.tde_bundle_close(h)
    return out


# ------------------------------------------------------------------ checkpoint state file
def write_checkpoint_state(directory, latest_path, all_paths, timestamps=None):
    """The TF ``checkpoint`` CheckpointState text proto (atomic replace)."""
    d = Path(directory)
    lines = [f'model_checkpoint_path: "{latest_path}"']
    lines += [f'all_model_checkpoint_paths: "{p}"' for p in all_paths]
    if timestamps:
        lines += [f"all_model_checkpoint_timestamps: {t}" for t in timestamps]
        lines.append(f"last_preserved_timestamp: {timestamps[0]}")
    tmp = d / f"checkpoint.tmp{os.getpid()}"
    tmp.write_text("\n".join(lines) + "\n")
    os.replace(tmp, d / "checkpoint")


def read_checkpoint_state(directory):
    f = Path(directory) / "checkpoint"
    if not f.exists():
        return None
    latest, allp = None, []
    for line in f.read_text().splitlines():
        m = re.match(r'\s*(\w+):\s*"(.*)"', line)
        if not m:
            continue
        if m.group(1) == "model_checkpoint_path":
            latest = m.group(2)
        elif m.group(1) == "all_model_checkpoint_paths":
            allp.append(m.group(2))
    return {"model_checkpoint_path": latest, "all_model_checkpoint_paths": allp}


def latest_checkpoint(directory):
    st = read_checkpoint_state(directory)
    if not st or not st["model_checkpoint_path"]:
        return None
    p = st["model_checkpoint_path"]
    if not os.path.isabs(p):
        p = str(Path(directory) / p)
    return p if Path(p + ".index").exists() else None
