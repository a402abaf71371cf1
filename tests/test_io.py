"""T2: native host I/O — crc32c golden values, TensorBundle round trip + an
independent pure-Python SSTable/proto parse of the native writer's bytes, and
TensorBoard event files."""
import ctypes as C
import struct

import numpy as np
import pytest

from tensorflow_distributed_example_amd import _native as N
from tensorflow_distributed_example_amd.io import events as EV
from tensorflow_distributed_example_amd.io import tensor_bundle as TB


def _crc(b: bytes):
    return N.host().tde_crc32c(b, len(b))


def test_crc32c_golden():
    assert _crc(b"123456789") == 0xE3069283
    assert _crc(b"") == 0
    assert _crc(b"\x00" * 32) == 0x8A9136AA
    lib = N.host()
    for v in (0, 1, 0xDEADBEEF, 0xE3069283):
        assert lib.tde_crc32c_unmask(lib.tde_crc32c_mask(v)) == v
    assert lib.tde_crc32c_mask(0xE3069283) == (((0xE3069283 >> 15) | (0xE3069283 << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        if x < 0x80:
            return r, i
        s += 7


def _block(buf, off, size):
    """Independent LevelDB block parser (prefix-compressed keys)."""
    data = buf[off: off + size]
    typ = buf[off + size]
    (stored,) = struct.unpack("<I", buf[off + size + 1: off + size + 5])
    lib = N.host()
    raw = bytes(data) + bytes([typ])
    assert lib.tde_crc32c_unmask(stored) == _crc(raw)
    assert typ == 0
    (nres,) = struct.unpack("<I", data[-4:])
    end = len(data) - 4 - 4 * nres
    i, key, out = 0, b"", []
    while i < end:
        shared, i = _varint(data, i)
        nonshared, i = _varint(data, i)
        vlen, i = _varint(data, i)
        key = key[:shared] + data[i:i + nonshared]
        i += nonshared
        out.append((key, data[i:i + vlen]))
        i += vlen
    return out


def _sstable(path):
    buf = open(path, "rb").read()
    assert struct.unpack("<Q", buf[-8:])[0] == 0xDB4775248B80FB57
    i = len(buf) - 48
    moff, i = _varint(buf, i)
    msize, i = _varint(buf, i)
    ioff, i = _varint(buf, i)
    isize, i = _varint(buf, i)
    rows = []
    for _, h in _block(buf, ioff, isize):
        bo, j = _varint(h, 0)
        bs, j = _varint(h, j)
        rows += _block(buf, bo, bs)
    return rows


def test_tensor_bundle_roundtrip_and_independent_parse(tmp_path):
    rng = np.random.default_rng(0)
    tensors = {"dense/kernel": rng.random((5408, 64), dtype=np.float32),
               "conv2d/kernel": rng.random((3, 3, 1, 32), dtype=np.float32),
               "conv2d/bias": np.zeros(32, np.float32),
               "global_step": np.array(469, dtype=np.int64)}
    for i in range(40):  # > 16 keys: exercises restart points
        tensors[f"extra/v{i:02d}"] = np.full((i + 1,), i, np.float32)
    prefix = str(tmp_path / "model.ckpt-469")
    TB.write_bundle(prefix, tensors)
    back = TB.read_bundle(prefix)
    assert set(back) == set(tensors)
    for k in tensors:
        assert back[k].shape == tensors[k].shape and np.array_equal(back[k], tensors[k])
    rows = _sstable(prefix + ".index")
    keys = [k for k, _ in rows]
    assert keys[0] == b"" and keys[1:] == sorted(k.encode() for k in tensors)
    # header proto: num_shards=1 (field 1), version{producer=1} (field 3)
    assert rows[0][1] == bytes([0x08, 0x01, 0x1A, 0x02, 0x08, 0x01])
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    ent = dict(rows)[b"dense/kernel"]
    # BundleEntryProto: dtype DT_FLOAT (08 01), shape dims 5408, 64, offset, size, crc (fixed32 field 6)
    assert ent[:2] == bytes([0x08, 0x01])
    fields = {}
    i = 0
    while i < len(ent):
        tag, i = _varint(ent, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(ent, i)
        elif wt == 2:
            n, i = _varint(ent, i)
            v = ent[i:i + n]
            i += n
        else:
            v = struct.unpack("<I", ent[i:i + 4])[0]
            i += 4
        fields[f] = v
    off, size = fields.get(4, 0), fields[5]
    assert size == 5408 * 64 * 4
    blob = data[off: off + size]
    assert np.array_equal(np.frombuffer(blob, np.float32).reshape(5408, 64), tensors["dense/kernel"])
    assert N.host().tde_crc32c_unmask(fields[6]) == _crc(blob)


def _entry_fields(ent):
    fields, i = {}, 0
    while i < len(ent):
        tag, i = _varint(ent, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(ent, i)
        elif wt == 2:
            n, i = _varint(ent, i)
            v = ent[i:i + n]
            i += n
        else:
            v = struct.unpack("<I", ent[i:i + 4])[0]
            i += 4
        fields[f] = v
    return fields


def test_string_tensor_checksums_follow_tf_layout(tmp_path):
    """TF's WriteStringTensor checksums each string length as a little-endian uint32 (not the
    varint bytes); the stored 4-byte length checksum is that crc masked; the BundleEntryProto crc covers the
    uint32 lengths, the 4-byte length checksum and the string bytes (masked).  A bundle whose string
    tensor fails its checksum still restores its numeric tensors (the object graph is metadata)."""
    from tensorflow_distributed_example_amd.io import object_graph as OG
    lib = N.host()
    payload = b"x" * 300                      # 300 needs a 2-byte varint: the layouts differ
    enc = OG.encode_string_tensor([payload])
    assert enc[:2] == bytes([0xAC, 0x02])
    want_len_crc = lib.tde_crc32c_mask(_crc(struct.pack("<I", 300)))
    assert struct.unpack("<I", enc[2:6])[0] == want_len_crc
    prefix = str(tmp_path / "s")
    TB.write_bundle(prefix, {"_CHECKPOINTABLE_OBJECT_GRAPH": payload, "v": np.ones(3, np.float32)})
    fields = _entry_fields(dict(_sstable(prefix + ".index"))[b"_CHECKPOINTABLE_OBJECT_GRAPH"])
    assert fields[1] == 7                       # DT_STRING
    c = lib.tde_crc32c_extend(_crc(struct.pack("<I", 300)), enc[2:6], 4)
    c = lib.tde_crc32c_extend(c, payload, len(payload))
    assert fields[6] == lib.tde_crc32c_mask(c)
    back = TB.read_bundle(prefix)
    assert back["_CHECKPOINTABLE_OBJECT_GRAPH"] == payload
    # corrupt one string byte: the numeric tensor still restores, the string tensor is skipped
    d = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    off = fields.get(4, 0)
    d[off + 10] ^= 0x01
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(d))
    back = TB.read_bundle(prefix)
    assert "_CHECKPOINTABLE_OBJECT_GRAPH" not in back and np.array_equal(back["v"], np.ones(3, np.float32))
    with pytest.raises(IOError, match="crc"):
        TB.read_bundle(prefix, skip_bad_strings=False)


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path / "c")
    TB.write_bundle(prefix, {"a": np.arange(100, dtype=np.float32)})
    d = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    d[10] ^= 0xFF
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(d))
    with pytest.raises(IOError, match="crc"):
        TB.read_bundle(prefix)


def test_checkpoint_state_file(tmp_path):
    TB.write_bundle(str(tmp_path / "model.ckpt-10"), {"x": np.ones(3, np.float32)})
    TB.write_checkpoint_state(tmp_path, "model.ckpt-10", ["model.ckpt-0", "model.ckpt-10"])
    st = TB.read_checkpoint_state(tmp_path)
    assert st["model_checkpoint_path"] == "model.ckpt-10"
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-0", "model.ckpt-10"]
    assert TB.latest_checkpoint(tmp_path) == str(tmp_path / "model.ckpt-10")
    assert 'model_checkpoint_path: "model.ckpt-10"' in (tmp_path / "checkpoint").read_text()


def test_event_file_roundtrip(tmp_path):
    w = EV.EventFileWriter(tmp_path)
    w.add_scalars(100, {"loss": 0.5, "accuracy": 0.875})
    w.add_scalar("global_step/sec", 1234.5, 100)
    w.close()
    evs = EV.read_events(w.path)
    assert evs[0]["file_version"] == "brain.Event:2"
    assert evs[1]["step"] == 100 and evs[1]["scalars"] == {"loss": 0.5, "accuracy": 0.875}
    assert abs(evs[2]["scalars"]["global_step/sec"] - 1234.5) < 1e-3
    # TFRecord framing: first 8 bytes = length, then masked crc32c of the length
    raw = open(w.path, "rb").read()
    (ln,) = struct.unpack("<Q", raw[:8])
    (lc,) = struct.unpack("<I", raw[8:12])
    assert N.host().tde_crc32c_unmask(lc) == _crc(raw[:8])
    assert ln == len(raw[12:12 + ln])


def test_tf2_object_graph_checkpoint_round_trip(tmp_path):
    """model.save_weights(prefix) writes the TF2 object-based layout (layer_with_weights-i/<attr>/
    .ATTRIBUTES/VARIABLE_VALUE, optimizer slots and iter, _CHECKPOINTABLE_OBJECT_GRAPH as a DT_STRING
    tensor); the graph parses as a TrackableObjectGraph protobuf (descriptor built from the field numbers
    of tensorflow/core/protobuf/trackable_object_graph.proto) and load_weights restores weights, slots and
    the step counter into a fresh model."""
    import torch
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.io import object_graph as OG
    from tensorflow_distributed_example_amd.io import tensor_bundle as TB

    # the DT_STRING encoding: [varint len][masked crc32c of the uint32 length][bytes]
    enc = OG.encode_string_tensor([b"abc"])
    assert enc[0] == 3 and enc[5:] == b"abc" and OG.decode_string_tensor(enc) == [b"abc"]

    def make():
        tde.backend.set_random_seed(3)
        m = tde.zoo.mnist_bn_cnn()
        m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01, momentum=0.9))
        m.build()
        return m

    m = make()
    st = m._store
    st.slot("momentum").copy_(torch.arange(st.slot("momentum").numel(), dtype=torch.float32) * 1e-3)
    m._set_iterations(17)
    prefix = str(tmp_path / "w" / "ckpt")
    m.save_weights(prefix)
    b = TB.read_bundle(prefix)
    assert "layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE" in b
    assert "layer_with_weights-1/beta/.ATTRIBUTES/VARIABLE_VALUE" in b
    assert "layer_with_weights-0/kernel/.OPTIMIZER_SLOT/optimizer/momentum/.ATTRIBUTES/VARIABLE_VALUE" in b
    assert int(b["optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE"]) == 17
    graph = b[OG.GRAPH_KEY]
    assert isinstance(graph, bytes)

    fd = descriptor_pb2.FileDescriptorProto(name="tog_test.proto", package="tog")
    msg = fd.message_type.add(name="TrackableObjectGraph")
    obj = msg.nested_type.add(name="TrackableObject")
    F = descriptor_pb2.FieldDescriptorProto
    for name, fields in [("ObjectReference", [("node_id", 1, F.TYPE_INT32), ("local_name", 2, F.TYPE_STRING)]),
                         ("SerializedTensor", [("name", 1, F.TYPE_STRING), ("full_name", 2, F.TYPE_STRING),
                                               ("checkpoint_key", 3, F.TYPE_STRING)]),
                         ("SlotVariableReference", [("original_variable_node_id", 1, F.TYPE_INT32),
                                                    ("slot_name", 2, F.TYPE_STRING),
                                                    ("slot_variable_node_id", 3, F.TYPE_INT32)])]:
        nt = obj.nested_type.add(name=name)
        for fname, num, typ in fields:
            nt.field.add(name=fname, number=num, type=typ, label=F.LABEL_OPTIONAL)
    for fname, num, tname in [("children", 1, "ObjectReference"), ("attributes", 2, "SerializedTensor"),
                              ("slot_variables", 3, "SlotVariableReference")]:
        obj.field.add(name=fname, number=num, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                      type_name=f".tog.TrackableObjectGraph.TrackableObject.{tname}")
    msg.field.add(name="nodes", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                  type_name=".tog.TrackableObjectGraph.TrackableObject")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    cls = message_factory.GetMessageClass(pool.FindMessageTypeByName("tog.TrackableObjectGraph"))
    g = cls()
    g.ParseFromString(graph)
    root = {c.local_name: c.node_id for c in g.nodes[0].children}
    assert "layer_with_weights-0" in root and "optimizer" in root and "layer-0" in root
    kern = {c.local_name: c.node_id for c in g.nodes[root["layer_with_weights-0"]].children}["kernel"]
    att = g.nodes[kern].attributes[0]
    assert att.name == "VARIABLE_VALUE" and att.full_name == "conv2d/kernel"
    assert att.checkpoint_key == "layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE"
    sv = g.nodes[root["optimizer"]].slot_variables
    assert any(s.original_variable_node_id == kern and s.slot_name == "momentum" for s in sv)

    m2 = make()
    m2.load_weights(prefix)
    for a, c in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, c)
    for n in st.names(trainable=True):
        sg = st.segments[n]
        assert torch.equal(m2._store.slot("momentum")[sg.offset: sg.offset + sg.numel],
                           st.slot("momentum")[sg.offset: sg.offset + sg.numel]), n
    assert int(m2.optimizer.iterations) == 17
    # the TF1-name layout stays available
    m.save_weights(str(tmp_path / "tf1" / "ckpt"), save_format="tf1")
    assert "conv2d/kernel" in TB.read_bundle(str(tmp_path / "tf1" / "ckpt"))


def _saved_model_classes():
    """Protobuf classes for the SavedModel subset, built from the field numbers of tensorflow/core/
    protobuf/{saved_model,meta_graph,saver}.proto and framework/{graph,node_def,attr_value,tensor,
    tensor_shape,versions}.proto (TF is not installed: the descriptors are the format spec)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="tf_sm_test.proto", package="tfsm")

    def msg(name, fields, parent=None):
        m = (parent.nested_type if parent is not None else fd.message_type).add(name=name)
        for fname, num, typ, lab, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=lab)
            if tname:
                f.type_name = tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("Dim", [("size", 1, F.TYPE_INT64, O, None), ("name", 2, F.TYPE_STRING, O, None)])
    msg("TensorShapeProto", [("dim", 2, F.TYPE_MESSAGE, R, ".tfsm.Dim"), ("unknown_rank", 3, F.TYPE_BOOL, O, None)])
    msg("TensorProto", [("dtype", 1, F.TYPE_INT32, O, None), ("tensor_shape", 2, F.TYPE_MESSAGE, O, ".tfsm.TensorShapeProto"),
                        ("tensor_content", 4, F.TYPE_BYTES, O, None), ("string_val", 8, F.TYPE_BYTES, R, None)])
    msg("ListValue", [("s", 2, F.TYPE_BYTES, R, None), ("i", 3, F.TYPE_INT64, R, None), ("f", 4, F.TYPE_FLOAT, R, None),
                      ("b", 5, F.TYPE_BOOL, R, None), ("type", 6, F.TYPE_INT32, R, None)])
    msg("AttrValue", [("list", 1, F.TYPE_MESSAGE, O, ".tfsm.ListValue"), ("s", 2, F.TYPE_BYTES, O, None),
                      ("i", 3, F.TYPE_INT64, O, None), ("f", 4, F.TYPE_FLOAT, O, None), ("b", 5, F.TYPE_BOOL, O, None),
                      ("type", 6, F.TYPE_INT32, O, None), ("shape", 7, F.TYPE_MESSAGE, O, ".tfsm.TensorShapeProto"),
                      ("tensor", 8, F.TYPE_MESSAGE, O, ".tfsm.TensorProto")])
    nd = msg("NodeDef", [("name", 1, F.TYPE_STRING, O, None), ("op", 2, F.TYPE_STRING, O, None),
                         ("input", 3, F.TYPE_STRING, R, None), ("device", 4, F.TYPE_STRING, O, None),
                         ("attr", 5, F.TYPE_MESSAGE, R, ".tfsm.NodeDef.AttrEntry")])
    e = msg("AttrEntry", [("key", 1, F.TYPE_STRING, O, None), ("value", 2, F.TYPE_MESSAGE, O, ".tfsm.AttrValue")], nd)
    e.options.map_entry = True
    msg("VersionDef", [("producer", 1, F.TYPE_INT32, O, None), ("min_consumer", 2, F.TYPE_INT32, O, None)])
    msg("GraphDef", [("node", 1, F.TYPE_MESSAGE, R, ".tfsm.NodeDef"), ("versions", 4, F.TYPE_MESSAGE, O, ".tfsm.VersionDef")])
    msg("SaverDef", [("filename_tensor_name", 1, F.TYPE_STRING, O, None), ("save_tensor_name", 2, F.TYPE_STRING, O, None),
                     ("restore_op_name", 3, F.TYPE_STRING, O, None), ("max_to_keep", 4, F.TYPE_INT32, O, None),
                     ("sharded", 5, F.TYPE_BOOL, O, None), ("keep_checkpoint_every_n_hours", 6, F.TYPE_FLOAT, O, None),
                     ("version", 7, F.TYPE_INT32, O, None)])
    msg("TensorInfo", [("name", 1, F.TYPE_STRING, O, None), ("dtype", 2, F.TYPE_INT32, O, None),
                       ("tensor_shape", 3, F.TYPE_MESSAGE, O, ".tfsm.TensorShapeProto")])
    sd = msg("SignatureDef", [("inputs", 1, F.TYPE_MESSAGE, R, ".tfsm.SignatureDef.InputsEntry"),
                              ("outputs", 2, F.TYPE_MESSAGE, R, ".tfsm.SignatureDef.OutputsEntry"),
                              ("method_name", 3, F.TYPE_STRING, O, None)])
    for en in ("InputsEntry", "OutputsEntry"):
        e = msg(en, [("key", 1, F.TYPE_STRING, O, None), ("value", 2, F.TYPE_MESSAGE, O, ".tfsm.TensorInfo")], sd)
        e.options.map_entry = True
    msg("MetaInfoDef", [("meta_graph_version", 1, F.TYPE_STRING, O, None), ("tags", 4, F.TYPE_STRING, R, None),
                        ("tensorflow_version", 5, F.TYPE_STRING, O, None)])
    mg = msg("MetaGraphDef", [("meta_info_def", 1, F.TYPE_MESSAGE, O, ".tfsm.MetaInfoDef"),
                              ("graph_def", 2, F.TYPE_MESSAGE, O, ".tfsm.GraphDef"),
                              ("saver_def", 3, F.TYPE_MESSAGE, O, ".tfsm.SaverDef"),
                              ("signature_def", 5, F.TYPE_MESSAGE, R, ".tfsm.MetaGraphDef.SignatureDefEntry")])
    e = msg("SignatureDefEntry", [("key", 1, F.TYPE_STRING, O, None), ("value", 2, F.TYPE_MESSAGE, O, ".tfsm.SignatureDef")], mg)
    e.options.map_entry = True
    msg("SavedModel", [("saved_model_schema_version", 1, F.TYPE_INT64, O, None),
                       ("meta_graphs", 2, F.TYPE_MESSAGE, R, ".tfsm.MetaGraphDef")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tfsm.SavedModel"))


def _decode_attr(a):
    import numpy as np_
    if a.HasField("tensor"):
        t = a.tensor
        shape = [d.size for d in t.tensor_shape.dim]
        if t.dtype == 7:
            vals = list(t.string_val)
            return vals[0] if not shape else vals
        return np_.frombuffer(t.tensor_content, {1: np_.float32, 3: np_.int32}[t.dtype]).reshape(shape)
    if a.HasField("list"):
        return list(a.list.i) or [bytes(s).decode() for s in a.list.s] or list(a.list.type)
    if a.HasField("shape"):
        return [d.size for d in a.shape.dim]
    for f in ("s", "i", "f", "b", "type"):
        if a.HasField(f):
            v = getattr(a, f)
            return v.decode() if isinstance(v, bytes) else v
    return None


@pytest.mark.parametrize("which", ["model_a", "model_b", "mini_resnet"])
def test_saved_model_pb_parses_and_executes(tmp_path, which):
    """The exported saved_model.pb parses as a SavedModel (descriptors from the TF .proto field numbers):
    one 'serve' MetaGraphDef, a serving_default predict signature from the [None, 784] / image placeholder,
    a V2 SaverDef whose save/restore subgraph names every variable of the TensorBundle; and the graph,
    EXECUTED by a numpy interpreter of its ops with the exported variables, reproduces the model's own
    inference forward (loading by TensorFlow itself is parity-unpinned: TF is not installed)."""
    import torch

    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.io import export as EX
    from tensorflow_distributed_example_amd.io import saved_model_pb as SM
    tde.backend.set_random_seed(0)
    if which == "model_a":
        m, serve_shape = tde.zoo.mnist_cnn(), [None, 784]
    elif which == "model_b":
        m, serve_shape = tde.zoo.mnist_bn_cnn(), [None, 784]
    else:
        m = tde.zoo.resnet((1, 1), (8, 16), input_shape=(16, 16, 3), classes=10, name="mini_resnet")
        serve_shape = [None, 16, 16, 3]
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01))
    m.build()
    g = torch.Generator().manual_seed(1)
    for n in m._store.names():   # non-trivial BN statistics / betas
        v = m._store.view(n)
        if "moving_variance" in n:
            v.copy_(torch.rand(v.shape, generator=g) + 0.5)
        elif "moving_mean" in n or n.endswith("/beta") or n.endswith("/gamma"):
            v.copy_(torch.rand(v.shape, generator=g) * 0.4 - 0.2 + (1.0 if n.endswith("/gamma") else 0.0))
    path = EX.export_saved_model(m, str(tmp_path / "exp"), lambda: EX.TensorServingInputReceiver(
        EX.placeholder("float32", serve_shape), {}))
    path = path.decode() if isinstance(path, bytes) else path
    SavedModel = _saved_model_classes()
    sm = SavedModel()
    sm.ParseFromString(open(f"{path}/saved_model.pb", "rb").read())
    assert sm.saved_model_schema_version == 1 and len(sm.meta_graphs) == 1
    mg = sm.meta_graphs[0]
    assert list(mg.meta_info_def.tags) == ["serve"]
    sig = mg.signature_def["serving_default"]
    assert sig.method_name == "tensorflow/serving/predict"
    (ik, iv), = sig.inputs.items()
    (ok, ov), = sig.outputs.items()
    assert [d.size for d in iv.tensor_shape.dim] == [-1] + serve_shape[1:] and iv.dtype == 1
    assert mg.saver_def.restore_op_name == "save/restore_all" and mg.saver_def.version == 2
    nodes = [(n.name, n.op, list(n.input), {k: _decode_attr(v) for k, v in n.attr.items()}) for n in mg.graph_def.node]
    names = {n[0] for n in nodes}
    assert len(names) == len(nodes) and mg.graph_def.versions.producer > 0
    for n in nodes:   # every input refers to an existing node
        for i in n[2]:
            assert i.lstrip("^").split(":")[0] in names, (n[0], i)
    bundle = TB.read_bundle(f"{path}/variables/variables")
    restore = next(n for n in nodes if n[0] == "save/RestoreV2/tensor_names")
    assert sorted(v.decode() for v in restore[3]["value"]) == sorted(bundle)
    handles = {n[3]["shared_name"] for n in nodes if n[1] == "VarHandleOp"}
    assert handles == set(bundle)
    rng = np.random.default_rng(2)
    x = rng.random([5] + serve_shape[1:], dtype=np.float32)
    got = SM.run_graph(nodes, {iv.name.split(":")[0]: x}, bundle, ov.name)
    want = m.predict(x.reshape((5,) + tuple(m.input_shape[1:])), verbose=0)
    assert np.allclose(got, want, rtol=1e-4, atol=1e-5), np.abs(got - want).max()
