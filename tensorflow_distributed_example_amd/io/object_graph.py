"""TF2 object-based checkpoint layout: what Keras ``model.save_weights(prefix)`` (TF format) writes and
``model_to_estimator`` stores under ``model_dir/keras/`` (SURVEY.md §5.4 "optional TF2 object-graph
naming"; reference mnist_keras_distributed.py:118-119).

Keys follow the trackable object graph of a Keras model::

    layer_with_weights-<i>/<attr>/.ATTRIBUTES/VARIABLE_VALUE                  variables of the i-th layer
                                                                              that has weights
    layer_with_weights-<i>/<attr>/.OPTIMIZER_SLOT/optimizer/<slot>/.ATTRIBUTES/VARIABLE_VALUE
    optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE                                 the step counter (int64)
    _CHECKPOINTABLE_OBJECT_GRAPH                                              serialized TrackableObjectGraph

The object graph is a ``TrackableObjectGraph`` protobuf (tensorflow/core/protobuf/
trackable_object_graph.proto) encoded here by hand in the protobuf wire format — nodes with their
children (``layer_with_weights-i``, ``layer-j``, ``optimizer``, attribute names), the variables'
``SerializedTensor`` (``VARIABLE_VALUE``, the TF1 ``full_name``, the checkpoint key) and the optimizer's
slot references — and stored as a scalar DT_STRING tensor in the TensorBundle string encoding
([varint64 length][masked crc32c of the lengths][bytes]).  Restoring matches variables by their
position in the object graph (``layer_with_weights-i`` / attribute), as TF does — not by the
session-unique layer names; ``restore_map`` reads the graph's ``full_name`` fields for tools.  TensorFlow is not installed here: byte compatibility with TF's reader is
parity-unpinned (tests/test_io.py checks the round trip and the encodings against the format spec).
"""
from __future__ import annotations

import numpy as np

GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
VAR = "/.ATTRIBUTES/VARIABLE_VALUE"


# ------------------------------------------------------------------ protobuf wire format
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fv(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(v)


def _fb(field: int, b) -> bytes:
    if isinstance(b, str):
        b = b.encode()
    return _varint((field << 3) | 2) + _varint(len(b)) + b


def _read_varint(buf, i):
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _fields(buf):
    """(field, wire type, value) of a serialized message (varint and length-delimited fields)."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v = bytes(buf[i:i + ln])
            i += ln
        elif wt == 5:
            v = bytes(buf[i:i + 4])
            i += 4
        elif wt == 1:
            v = bytes(buf[i:i + 8])
            i += 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, wt, v


# ------------------------------------------------------------------ TensorBundle DT_STRING encoding
def _masked_crc(b: bytes) -> int:
    """The TensorBundle masked crc32c of ``b`` (native csrc/io/crc32c.cpp)."""
    import ctypes as C

    from .. import _native as N
    lib = N.host()
    buf = C.create_string_buffer(bytes(b), len(b))
    return int(lib.tde_crc32c_masked(C.cast(buf, C.c_void_p), len(b)))


def _len_words(lengths) -> bytes:
    """The bytes TF checksums for string lengths: each length as a little-endian uint32 (uint64 when it
    does not fit), kept for backward compatibility in TF's WriteStringTensor — not the varint bytes."""
    return b"".join(n.to_bytes(4 if n <= 0xFFFFFFFF else 8, "little") for n in lengths)


def encode_string_tensor(values) -> bytes:
    """TensorBundle data bytes of a DT_STRING tensor: [varint64 len]* [masked crc32c of the lengths
    as uint32 words, little endian] [bytes]*.  The entry checksum (computed natively when the bundle is
    written) covers the uint32 lengths, this 4-byte checksum and the string bytes."""
    vals = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
    lens = b"".join(_varint(len(v)) for v in vals)
    return lens + _masked_crc(_len_words([len(v) for v in vals])).to_bytes(4, "little") + b"".join(vals)


def decode_string_tensor(raw: bytes, n: int = 1):
    i, lens = 0, []
    for _ in range(n):
        ln, i = _read_varint(raw, i)
        lens.append(ln)
    want = int.from_bytes(raw[i:i + 4], "little")
    if want != _masked_crc(_len_words(lens)):
        raise IOError("string tensor: length checksum mismatch")
    i += 4
    out = []
    for ln in lens:
        out.append(bytes(raw[i:i + ln]))
        i += ln
    return out


# ------------------------------------------------------------------ the model's object graph
def _weighted_layers(model):
    return [layer for layer in model.layers if getattr(layer, "weight_specs", None)]


def variable_keys(model) -> dict:
    """{TF1 variable name: TF2 object-graph checkpoint key} of every model variable."""
    out = {}
    for i, layer in enumerate(_weighted_layers(model)):
        for s in layer.weight_specs:
            out[s.full_name] = f"layer_with_weights-{i}/{s.name}{VAR}"
    return out


def build(model, values: dict, slots: dict | None = None, iterations: int | None = None) -> dict:
    """{checkpoint key: array | bytes} of ``values`` ({TF1 name: array}), the optimizer ``slots``
    ({slot name: {TF1 name: array}}) and the step counter, plus the serialized object graph."""
    nodes = [dict(children=[], attrs=[], slots=[])]          # node 0: the model
    out = {}
    var_node = {}

    def new_node():
        nodes.append(dict(children=[], attrs=[], slots=[]))
        return len(nodes) - 1

    layer_node = {}
    for i, layer in enumerate(_weighted_layers(model)):
        ln = new_node()
        layer_node[id(layer)] = ln
        nodes[0]["children"].append((ln, f"layer_with_weights-{i}"))
        for s in layer.weight_specs:
            if s.full_name not in values:
                continue
            vn = new_node()
            key = f"layer_with_weights-{i}/{s.name}{VAR}"
            nodes[ln]["children"].append((vn, s.name))
            nodes[vn]["attrs"].append(("VARIABLE_VALUE", s.full_name, key))
            out[key] = np.asarray(values[s.full_name])
            var_node[s.full_name] = (vn, f"layer_with_weights-{i}/{s.name}")
    for j, layer in enumerate(model.layers):   # every layer is also reachable as layer-<j>
        ln = layer_node.get(id(layer))
        if ln is None:
            ln = new_node()
        nodes[0]["children"].append((ln, f"layer-{j}"))
    if slots is not None or iterations is not None:
        on = new_node()
        nodes[0]["children"].append((on, "optimizer"))
        if iterations is not None:
            it = new_node()
            key = f"optimizer/iter{VAR}"
            nodes[on]["children"].append((it, "iter"))
            nodes[it]["attrs"].append(("VARIABLE_VALUE", "iter", key))
            out[key] = np.asarray(iterations, dtype=np.int64)
        for sname, per_var in (slots or {}).items():
            for vname, arr in per_var.items():
                if vname not in var_node:
                    continue
                vn, path = var_node[vname]
                sn = new_node()
                key = f"{path}/.OPTIMIZER_SLOT/optimizer/{sname}{VAR}"
                nodes[sn]["attrs"].append(("VARIABLE_VALUE", f"{vname}/{sname}", key))
                nodes[on]["slots"].append((vn, sname, sn))
                out[key] = np.asarray(arr)
    graph = b""
    for nd in nodes:
        body = b"".join(_fb(1, _fv(1, c) + _fb(2, name)) for c, name in nd["children"])
        body += b"".join(_fb(2, _fb(1, n) + _fb(2, full) + _fb(3, key)) for n, full, key in nd["attrs"])
        body += b"".join(_fb(3, _fv(1, o) + _fb(2, sname) + _fv(3, sn)) for o, sname, sn in nd["slots"])
        graph += _fb(1, body)
    out[GRAPH_KEY] = graph
    return out


def parse_graph(graph: bytes):
    """[(full_name, checkpoint_key)] of every SerializedTensor in a TrackableObjectGraph."""
    out = []
    for f, wt, node in _fields(graph):
        if f != 1 or wt != 2:
            continue
        for g, wt2, att in _fields(node):
            if g != 2 or wt2 != 2:
                continue
            d = {h: v for h, _, v in _fields(att)}
            out.append((d.get(2, b"").decode(), d.get(3, b"").decode()))
    return out


def restore_map(bundle: dict) -> dict:
    """{TF1 name (or "<var>/<slot>", "iter"): array} of an object-graph checkpoint read as a dict."""
    graph = bundle.get(GRAPH_KEY)
    if graph is None:
        return {}
    out = {}
    for full, key in parse_graph(graph):
        if key in bundle:
            out[full] = bundle[key]
    return out
