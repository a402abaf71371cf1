"""``saved_model.pb``: the TF1 SavedModel protobuf of a model's serving graph (SURVEY.md F22 / §7.5;
FinalExporter at mnist_keras_distributed.py:264 with serving_input_fn :151-162 — a float32 ``[None, 784]``
placeholder), encoded by hand in the protobuf wire format (tensorflow/core/protobuf/saved_model.proto,
meta_graph.proto, saver.proto; tensorflow/core/framework/graph.proto, node_def.proto, attr_value.proto,
tensor.proto, tensor_shape.proto, versions.proto).

One MetaGraphDef tagged ``serve``:
* GraphDef — the inference graph with TensorFlow's standard ops: ``Placeholder`` for the serving input,
  resource variables (``VarHandleOp`` + ``ReadVariableOp``, shared names = the TF1 variable names of the
  exported TensorBundle), ``Reshape`` / ``Conv2D`` / ``BiasAdd`` / ``Relu`` / ``MaxPool`` /
  ``FusedBatchNormV3`` (4-D, ``is_training=false``) or the Keras 2-D batchnorm arithmetic / ``MatMul`` /
  ``Softmax`` / ``AddV2`` / ``Mean`` / ``Pad`` / ``Identity`` (Dropout at inference);
* the ``save/`` subgraph (``SaveV2`` / ``RestoreV2`` + ``AssignVariableOp`` → ``save/restore_all``) and a
  ``SaverDef`` pointing at it, so a TF1 loader restores ``variables/variables`` by running the restore op;
* ``SignatureDef`` ``serving_default`` (``tensorflow/serving/predict``) from the serving input to the model
  output.
TensorFlow is not installed here: loading by TF is parity-unpinned.  ``tests/test_io.py`` parses the file
with protobuf descriptors built from those .proto field numbers and EXECUTES the parsed graph with a small
numpy interpreter (``run_graph``) against the model's own forward.
"""
from __future__ import annotations

import numpy as np

from .object_graph import _fb, _fv, _varint

DT_FLOAT, DT_INT32, DT_STRING, DT_RESOURCE = 1, 3, 7, 20
GRAPH_PRODUCER = 1395     # VersionDef.producer of the graph (TF 2.x era); min_consumer 12


# ------------------------------------------------------------------ wire helpers
def _msg(field, payload: bytes) -> bytes:
    return _fb(field, payload)


def _f32(field, v) -> bytes:
    return _varint((field << 3) | 5) + np.float32(v).tobytes()


def _shape(dims) -> bytes:
    """TensorShapeProto (dim = 2 {size = 1}); None -> -1."""
    return b"".join(_msg(2, _fv(1, -1 if d is None else int(d)) if (d is None or int(d) != 0) else b"")
                    for d in dims)


def _tensor(arr: np.ndarray) -> bytes:
    """TensorProto: dtype = 1, tensor_shape = 2, tensor_content = 4 (little-endian raw) / string_val = 8."""
    if arr.dtype.kind in "SUO":
        vals = [v if isinstance(v, bytes) else str(v).encode() for v in arr.reshape(-1)]
        return _fv(1, DT_STRING) + _msg(2, _shape(arr.shape)) + b"".join(_fb(8, v) for v in vals)
    dt = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.int32): DT_INT32}[arr.dtype]
    return _fv(1, dt) + _msg(2, _shape(arr.shape)) + _fb(4, np.ascontiguousarray(arr).tobytes())


class A:
    """AttrValue encoders: list = 1, s = 2, i = 3, f = 4, b = 5, type = 6, shape = 7, tensor = 8."""

    @staticmethod
    def s(v):
        return _fb(2, v)

    @staticmethod
    def i(v):
        return _fv(3, int(v))

    @staticmethod
    def f(v):
        return _f32(4, v)

    @staticmethod
    def b(v):
        return _fv(5, 1 if v else 0)

    @staticmethod
    def type(v):
        return _fv(6, v)

    @staticmethod
    def shape(dims):
        return _msg(7, _shape(dims))

    @staticmethod
    def tensor(arr):
        return _msg(8, _tensor(arr))

    @staticmethod
    def ints(vs):   # ListValue.i (packed)
        return _msg(1, _fb(3, b"".join(_varint(int(v) & ((1 << 64) - 1)) for v in vs)) if vs else b"")

    @staticmethod
    def types(vs):  # ListValue.type (packed)
        return _msg(1, _fb(6, b"".join(_varint(v) for v in vs)) if vs else b"")

    @staticmethod
    def empty_list():
        return _msg(1, b"")


class GraphBuilder:
    def __init__(self):
        self.nodes = []
        self.names = set()

    def unique(self, name):
        base, k = name, 0
        while name in self.names:
            k += 1
            name = f"{base}_{k}"
        return name

    def node(self, name, op, inputs=(), **attrs):
        name = self.unique(name)
        self.names.add(name)
        body = _fb(1, name) + _fb(2, op) + b"".join(_fb(3, i) for i in inputs)
        for k in sorted(attrs):
            body += _msg(5, _fb(1, k) + _msg(2, attrs[k]))   # map<string, AttrValue> entry
        self.nodes.append(body)
        return name

    def const(self, name, arr):
        arr = np.asarray(arr)
        dt = DT_STRING if arr.dtype.kind in "SUO" else {np.dtype(np.float32): DT_FLOAT, np.dtype(np.int32): DT_INT32}[arr.dtype]
        return self.node(name, "Const", dtype=A.type(dt), value=A.tensor(arr))

    def graph_def(self):
        return b"".join(_msg(1, n) for n in self.nodes) + _msg(4, _fv(1, GRAPH_PRODUCER) + _fv(2, 12))


def _float_attrs():
    return dict(T=A.type(DT_FLOAT))


def build_graph(model, input_name="Placeholder", input_shape=None):
    """GraphDef bytes, the signature input / output tensor names, the (name, shape) of every variable."""
    from ..models import layers as L
    g = GraphBuilder()
    store = model._store
    var_shapes = [(n, tuple(store.segments[n].shape)) for n in store.order]
    handles = {}
    for n, shape in var_shapes:
        handles[n] = g.node(n, "VarHandleOp", dtype=A.type(DT_FLOAT), shape=A.shape(shape), shared_name=A.s(n),
                            container=A.s(""), allowed_devices=A.empty_list())

    def read(var, scope):
        return g.node(f"{scope}/ReadVariableOp", "ReadVariableOp", [handles[var]], dtype=A.type(DT_FLOAT))

    ishape = list(input_shape) if input_shape is not None else [None] + list(model.input_shape[1:])
    x_in = g.node(input_name, "Placeholder", dtype=A.type(DT_FLOAT), shape=A.shape(ishape))
    tensors = {0: x_in}
    in_rank = len(ishape)
    model_rank = 1 + len(model.input_shape[1:])
    if in_rank != model_rank:   # e.g. a [None, 784] serving input for a [28, 28, 1] model
        shp = g.const("serving/Reshape/shape", np.array([-1] + list(model.input_shape[1:]), np.int32))
        tensors[0] = g.node("serving/Reshape", "Reshape", [x_in, shp], T=A.type(DT_FLOAT), Tshape=A.type(DT_INT32))
    for layer, ins, out in model._nodes():
        nm = layer.name
        xs = [tensors[i] for i in ins]
        x = xs[0]
        if isinstance(layer, L.InputLayer):
            y = x
        elif isinstance(layer, (L.Reshape, L.Flatten)):
            tgt = layer.target_shape if isinstance(layer, L.Reshape) else (int(np.prod(layer.input_shape)),)
            shp = g.const(f"{nm}/Reshape/shape", np.array([-1] + list(tgt), np.int32))
            y = g.node(f"{nm}/Reshape", "Reshape", [x, shp], T=A.type(DT_FLOAT), Tshape=A.type(DT_INT32))
        elif isinstance(layer, L.Conv2D):
            y = g.node(f"{nm}/Conv2D", "Conv2D", [x, read(f"{nm}/kernel", f"{nm}/Conv2D")],
                       strides=A.ints([1, layer.strides[0], layer.strides[1], 1]),
                       padding=A.s(layer.padding.upper()), data_format=A.s("NHWC"), dilations=A.ints([1, 1, 1, 1]),
                       use_cudnn_on_gpu=A.b(True), explicit_paddings=A.empty_list(), **_float_attrs())
            if layer.use_bias:
                y = g.node(f"{nm}/BiasAdd", "BiasAdd", [y, read(f"{nm}/bias", f"{nm}/BiasAdd")],
                           data_format=A.s("NHWC"), **_float_attrs())
            y = _activation(g, nm, y, layer.activation)
        elif isinstance(layer, L.Dense):
            y = g.node(f"{nm}/MatMul", "MatMul", [x, read(f"{nm}/kernel", f"{nm}/MatMul")], transpose_a=A.b(False),
                       transpose_b=A.b(False), **_float_attrs())
            if layer.use_bias:
                y = g.node(f"{nm}/BiasAdd", "BiasAdd", [y, read(f"{nm}/bias", f"{nm}/BiasAdd")],
                           data_format=A.s("NHWC"), **_float_attrs())
            y = _activation(g, nm, y, layer.activation)
        elif isinstance(layer, L.Activation):
            y = _activation(g, nm, x, layer.activation)
        elif isinstance(layer, L.MaxPooling2D):
            y = g.node(f"{nm}/MaxPool", "MaxPool", [x], ksize=A.ints([1, *layer.pool_size, 1]),
                       strides=A.ints([1, *layer.strides, 1]), padding=A.s(layer.padding.upper()),
                       data_format=A.s("NHWC"), **_float_attrs())
        elif isinstance(layer, L.BatchNormalization):
            y = _batchnorm(g, layer, x, read)
        elif isinstance(layer, L.Dropout):
            y = g.node(f"{nm}/Identity", "Identity", [x], **_float_attrs())   # inference: no mask
        elif isinstance(layer, L.Add):
            y = x
            for k, other in enumerate(xs[1:]):
                y = g.node(f"{nm}/add" + (f"_{k}" if k else ""), "AddV2", [y, other], **_float_attrs())
        elif isinstance(layer, L.GlobalAveragePooling2D):
            ax = g.const(f"{nm}/Mean/reduction_indices", np.array([1, 2], np.int32))
            y = g.node(f"{nm}/Mean", "Mean", [x, ax], keep_dims=A.b(False), Tidx=A.type(DT_INT32), **_float_attrs())
        elif isinstance(layer, L.ZeroPadding2D):
            (t, b), (l, r) = layer.padding
            pads = g.const(f"{nm}/Pad/paddings", np.array([[0, 0], [t, b], [l, r], [0, 0]], np.int32))
            y = g.node(f"{nm}/Pad", "Pad", [x, pads], Tpaddings=A.type(DT_INT32), **_float_attrs())
        else:
            raise NotImplementedError(f"saved_model.pb: no TensorFlow op mapping for {type(layer).__name__}")
        tensors[out] = y
    out_node = tensors[model._nodes()[-1][2]]
    return g, f"{x_in}:0", f"{out_node}:0", var_shapes, handles


def _activation(g, nm, y, act):
    if act in (None, "linear"):
        return y
    op = {"relu": "Relu", "softmax": "Softmax", "sigmoid": "Sigmoid", "tanh": "Tanh"}.get(act)
    if op is None:
        raise NotImplementedError(f"saved_model.pb: activation {act!r}")
    return g.node(f"{nm}/{op}", op, [y], **_float_attrs())


def _batchnorm(g, layer, x, read):
    nm = layer.name
    C = layer.input_shape[-1]
    gamma = read(f"{nm}/gamma", f"{nm}/gamma") if layer.scale else g.const(f"{nm}/Const", np.ones(C, np.float32))
    beta = read(f"{nm}/beta", f"{nm}/beta") if layer.center else g.const(f"{nm}/Const_1", np.zeros(C, np.float32))
    mean = read(f"{nm}/moving_mean", f"{nm}/moving_mean")
    var = read(f"{nm}/moving_variance", f"{nm}/moving_variance")
    if layer.fused:   # 4-D input: FusedBatchNormV3 in inference mode
        return g.node(f"{nm}/FusedBatchNormV3", "FusedBatchNormV3", [x, gamma, beta, mean, var],
                      epsilon=A.f(layer.epsilon), exponential_avg_factor=A.f(1.0), data_format=A.s("NHWC"),
                      is_training=A.b(False), U=A.type(DT_FLOAT), **_float_attrs())
    # 2-D input (Keras' non-fused path): x * (gamma * rsqrt(var + eps)) + (beta - mean * gamma * rsqrt(var + eps))
    eps = g.const(f"{nm}/batchnorm/add/y", np.array(layer.epsilon, np.float32))
    a = g.node(f"{nm}/batchnorm/add", "AddV2", [var, eps], **_float_attrs())
    rs = g.node(f"{nm}/batchnorm/Rsqrt", "Rsqrt", [a], **_float_attrs())
    m = g.node(f"{nm}/batchnorm/mul", "Mul", [rs, gamma], **_float_attrs())
    m1 = g.node(f"{nm}/batchnorm/mul_1", "Mul", [x, m], **_float_attrs())
    m2 = g.node(f"{nm}/batchnorm/mul_2", "Mul", [mean, m], **_float_attrs())
    sb = g.node(f"{nm}/batchnorm/sub", "Sub", [beta, m2], **_float_attrs())
    return g.node(f"{nm}/batchnorm/add_1", "AddV2", [m1, sb], **_float_attrs())


def _saver(g: GraphBuilder, var_shapes, handles, dtypes=None):
    """The TF1 ``save/`` subgraph over the variables (V2 checkpoint format); returns the SaverDef.
    ``dtypes``: per-variable DataType (default all DT_FLOAT)."""
    dtypes = list(dtypes) if dtypes is not None else [DT_FLOAT] * len(var_shapes)
    names = np.array([n.encode() for n, _ in var_shapes], dtype=object)
    slices = np.array([b""] * len(var_shapes), dtype=object)
    fname = g.const("save/filename/input", np.array(b"model", dtype=object))
    fph = g.node("save/filename", "PlaceholderWithDefault", [fname], dtype=A.type(DT_STRING), shape=A.shape([]))
    prefix = g.node("save/Const", "PlaceholderWithDefault", [fph], dtype=A.type(DT_STRING), shape=A.shape([]))
    tn = g.const("save/SaveV2/tensor_names", names)
    sl = g.const("save/SaveV2/shape_and_slices", slices)
    reads = [g.node(f"save/Read_{i}/ReadVariableOp", "ReadVariableOp", [handles[n]], dtype=A.type(dtypes[i]))
             for i, (n, _) in enumerate(var_shapes)]
    save = g.node("save/SaveV2", "SaveV2", [prefix, tn, sl] + reads, dtypes=A.types(dtypes))
    dep = g.node("save/control_dependency", "Identity", [prefix, f"^{save}"], T=A.type(DT_STRING),
                 _class=_msg(1, _fb(2, f"loc:@{prefix}".encode())))
    rtn = g.const("save/RestoreV2/tensor_names", names)
    rsl = g.const("save/RestoreV2/shape_and_slices", slices)
    rst = g.node("save/RestoreV2", "RestoreV2", [prefix, rtn, rsl], dtypes=A.types(dtypes))
    assigns = []
    for i, (n, _) in enumerate(var_shapes):
        idn = g.node(f"save/Identity_{i}", "Identity", [f"{rst}:{i}"], T=A.type(dtypes[i]))
        assigns.append(g.node(f"save/AssignVariableOp_{i}", "AssignVariableOp", [handles[n], idn],
                              dtype=A.type(dtypes[i]), validate_shape=A.b(False)))
    g.node("save/restore_all", "NoOp", [f"^{a}" for a in assigns])
    # SaverDef: filename_tensor_name = 1, save_tensor_name = 2, restore_op_name = 3, max_to_keep = 4,
    # sharded = 5, keep_checkpoint_every_n_hours = 6, version = 7 (V2)
    return (_fb(1, f"{prefix}:0") + _fb(2, f"{dep}:0") + _fb(3, "save/restore_all") + _fv(4, 5) + _fv(5, 0)
            + _f32(6, 10000.0) + _fv(7, 2))


def _tensor_info(name, shape):
    # TensorInfo: name = 1, dtype = 2, tensor_shape = 3
    return _fb(1, name) + _fv(2, DT_FLOAT) + _msg(3, _shape(shape))


def saved_model_bytes(model, input_shape=None, input_key="input", output_key=None, tags=("serve",)):
    """Serialized SavedModel (schema version 1, one MetaGraphDef)."""
    g, in_t, out_t, var_shapes, handles = build_graph(model, input_shape=input_shape)
    saver_def = _saver(g, var_shapes, handles)
    ishape = list(input_shape) if input_shape is not None else [None] + list(model.input_shape[1:])
    oshape = [None] + list(model.output_shape[1:])
    output_key = output_key or model.layers[-1].name
    sig = (_msg(1, _fb(1, input_key) + _msg(2, _tensor_info(in_t, ishape)))
           + _msg(2, _fb(1, output_key) + _msg(2, _tensor_info(out_t, oshape)))
           + _fb(3, "tensorflow/serving/predict"))
    # MetaInfoDef: meta_graph_version = 1, tags = 4, tensorflow_version = 5
    meta_info = _fb(1, "v1") + b"".join(_fb(4, t) for t in tags) + _fb(5, "tensorflow_distributed_example_amd")
    meta = (_msg(1, meta_info) + _msg(2, g.graph_def()) + _msg(3, saver_def)
            + _msg(5, _fb(1, "serving_default") + _msg(2, sig)))
    return _fv(1, 1) + _msg(2, meta)


# ------------------------------------------------------------------ Estimator checkpoint metadata
_NP_DT = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): 2, np.dtype(np.int32): DT_INT32,
          np.dtype(np.uint8): 4, np.dtype(np.int64): 9, np.dtype(np.bool_): 10}


def checkpoint_meta_graph_bytes(model, tensors: dict) -> bytes:
    """``model.ckpt-N.meta``: the MetaGraphDef a TF1 Saver writes next to each checkpoint (RunConfig(model_dir,
    save_checkpoints_steps), mnist_keras_distributed.py:245,248).  Its GraphDef is the model's inference graph
    (build_graph) plus a resource variable for every other tensor of the bundle (``global_step`` int64,
    optimizer slots, iterator state), and its SaverDef points at a ``save/`` subgraph whose SaveV2 /
    RestoreV2 name EVERY tensor of the TensorBundle ``tensors`` {name: array} with its dtype and shape, so a
    TF1 ``tf.train.import_meta_graph`` + ``saver.restore`` pair would find the checkpoint's variables.  (The
    reference's meta graph also holds the training ops; ours carries the forward only: parity of the
    training subgraph is not claimed.)"""
    g, _in, _out, var_shapes, handles = build_graph(model)
    dt = {n: DT_FLOAT for n, _ in var_shapes}
    shapes = dict(var_shapes)
    for name in sorted(tensors):
        if name in handles:
            continue
        arr = np.asarray(tensors[name])
        d = _NP_DT.get(arr.dtype)
        if d is None:
            continue
        handles[name] = g.node(name, "VarHandleOp", dtype=A.type(d), shape=A.shape(arr.shape), shared_name=A.s(name),
                               container=A.s(""), allowed_devices=A.empty_list())
        dt[name], shapes[name] = d, tuple(arr.shape)
    saved = [(n, shapes[n]) for n in sorted(tensors) if n in handles]
    saver_def = _saver(g, saved, handles, [dt[n] for n, _ in saved])
    meta_info = _fb(1, "v1") + _fb(5, "tensorflow_distributed_example_amd")
    return _msg(1, meta_info) + _msg(2, g.graph_def()) + _msg(3, saver_def)


def graph_pbtxt(model) -> str:
    """``graph.pbtxt``: the text-format GraphDef an Estimator writes into ``model_dir`` (the model's graph)."""
    from .tf_proto import graph_def_text
    g, *_ = build_graph(model)
    return graph_def_text(g.graph_def())


# ------------------------------------------------------------------ a numpy interpreter of the graph
def run_graph(graph_nodes, feeds: dict, variables: dict, fetch: str):
    """Evaluate ``fetch`` ("node:0") of a parsed GraphDef (``graph_nodes``: [(name, op, inputs, attrs)] with
    decoded attrs) given ``feeds`` {placeholder name: array} and ``variables`` {shared_name: array} — the
    ops ``build_graph`` emits, in numpy float64 (a semantics check of the exported graph)."""
    by = {n[0]: n for n in graph_nodes}
    cache = {}

    def val(ref):
        ref = ref.split("^")[-1]
        name, _, idx = ref.partition(":")
        k = (name, int(idx or 0))
        if k not in cache:
            cache[k] = _eval(by[name])
        return cache[k]

    def _eval(node):
        name, op, ins, at = node
        xs = [val(i) for i in ins if not i.startswith("^")]
        if op == "Placeholder":
            return np.asarray(feeds[name], np.float64)
        if op == "Const":
            return at["value"]
        if op == "VarHandleOp":
            return at["shared_name"]
        if op == "ReadVariableOp":
            return np.asarray(variables[xs[0]], np.float64)
        if op == "Identity":
            return xs[0]
        if op == "Reshape":
            return xs[0].reshape([int(d) for d in xs[1]])
        if op == "Conv2D":
            return _conv2d(xs[0], xs[1], at["strides"][1:3], at["padding"])
        if op == "BiasAdd":
            return xs[0] + xs[1]
        if op == "Relu":
            return np.maximum(xs[0], 0)
        if op == "Softmax":
            e = np.exp(xs[0] - xs[0].max(-1, keepdims=True))
            return e / e.sum(-1, keepdims=True)
        if op == "MatMul":
            return xs[0] @ xs[1]
        if op == "MaxPool":
            return _maxpool(xs[0], at["ksize"][1:3], at["strides"][1:3], at["padding"])
        if op == "FusedBatchNormV3":
            x, sc, of, mu, var = xs
            return (x - mu) / np.sqrt(var + at["epsilon"]) * sc + of
        if op == "AddV2":
            return xs[0] + xs[1]
        if op == "Mul":
            return xs[0] * xs[1]
        if op == "Sub":
            return xs[0] - xs[1]
        if op == "Rsqrt":
            return 1.0 / np.sqrt(xs[0])
        if op == "Mean":
            return xs[0].mean(axis=tuple(int(a) for a in xs[1]))
        if op == "Pad":
            return np.pad(xs[0], [tuple(int(v) for v in p) for p in xs[1]])
        raise NotImplementedError(op)

    return val(fetch)


def _same_pads(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


def _conv2d(x, w, strides, padding):
    B, H, W, C = x.shape
    kh, kw, _, Co = w.shape
    sh, sw = strides
    if padding == "SAME":
        (pt, pb), (pl, pr) = _same_pads(H, kh, sh), _same_pads(W, kw, sw)
        x = np.pad(x, [(0, 0), (pt, pb), (pl, pr), (0, 0)])
    Ho, Wo = (x.shape[1] - kh) // sh + 1, (x.shape[2] - kw) // sw + 1
    out = np.zeros((B, Ho, Wo, Co))
    for i in range(kh):
        for j in range(kw):
            patch = x[:, i: i + sh * (Ho - 1) + 1: sh, j: j + sw * (Wo - 1) + 1: sw, :]
            out += patch @ w[i, j]
    return out


def _maxpool(x, ksize, strides, padding):
    B, H, W, C = x.shape
    kh, kw = ksize
    sh, sw = strides
    if padding == "SAME":
        (pt, pb), (pl, pr) = _same_pads(H, kh, sh), _same_pads(W, kw, sw)
        x = np.pad(x, [(0, 0), (pt, pb), (pl, pr), (0, 0)], constant_values=-np.inf)
    Ho, Wo = (x.shape[1] - kh) // sh + 1, (x.shape[2] - kw) // sw + 1
    out = np.full((B, Ho, Wo, C), -np.inf)
    for i in range(kh):
        for j in range(kw):
            out = np.maximum(out, x[:, i: i + sh * (Ho - 1) + 1: sh, j: j + sw * (Wo - 1) + 1: sw, :])
    return out
