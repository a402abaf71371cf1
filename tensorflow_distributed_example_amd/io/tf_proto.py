"""Protobuf message classes for the TensorFlow graph / checkpoint-metadata subset this package writes, built at
run time from the field numbers of tensorflow/core/framework/{graph,node_def,attr_value,tensor,tensor_shape,
types,versions}.proto and tensorflow/core/protobuf/{meta_graph,saver,saved_model}.proto (TensorFlow is not
installed: the .proto field numbers are the format spec).

Used to render ``graph.pbtxt`` (the text-format GraphDef an Estimator writes into ``model_dir``,
mnist_keras_distributed.py:245) from the binary GraphDef of ``io/saved_model_pb.py`` with protobuf's own
text printer, and by the tests to parse ``saved_model.pb`` / ``model.ckpt-N.meta`` back.
"""
from __future__ import annotations

import functools

# tensorflow/core/framework/types.proto DataType (the values this package emits)
DATA_TYPES = {"DT_INVALID": 0, "DT_FLOAT": 1, "DT_DOUBLE": 2, "DT_INT32": 3, "DT_UINT8": 4, "DT_STRING": 7,
              "DT_INT64": 9, "DT_BOOL": 10, "DT_RESOURCE": 20}


@functools.lru_cache(maxsize=1)
def classes() -> dict:
    """{message name: class} for GraphDef, MetaGraphDef, SavedModel and their parts (package ``tfpb``)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="tde_tf_subset.proto", package="tfpb")
    en = fd.enum_type.add(name="DataType")
    for k, v in sorted(DATA_TYPES.items(), key=lambda kv: kv[1]):
        en.value.add(name=k, number=v)

    def msg(name, fields, parent=None):
        m = (parent.nested_type if parent is not None else fd.message_type).add(name=name)
        for fname, num, typ, lab, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=lab)
            if tname:
                f.type_name = tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    DT = (F.TYPE_ENUM, ".tfpb.DataType")
    msg("Dim", [("size", 1, F.TYPE_INT64, O, None), ("name", 2, F.TYPE_STRING, O, None)])
    msg("TensorShapeProto", [("dim", 2, F.TYPE_MESSAGE, R, ".tfpb.Dim"), ("unknown_rank", 3, F.TYPE_BOOL, O, None)])
    msg("TensorProto", [("dtype", 1, DT[0], O, DT[1]),
                        ("tensor_shape", 2, F.TYPE_MESSAGE, O, ".tfpb.TensorShapeProto"),
                        ("tensor_content", 4, F.TYPE_BYTES, O, None), ("string_val", 8, F.TYPE_BYTES, R, None)])
    msg("ListValue", [("s", 2, F.TYPE_BYTES, R, None), ("i", 3, F.TYPE_INT64, R, None),
                      ("f", 4, F.TYPE_FLOAT, R, None), ("b", 5, F.TYPE_BOOL, R, None), ("type", 6, DT[0], R, DT[1])])
    msg("AttrValue", [("list", 1, F.TYPE_MESSAGE, O, ".tfpb.ListValue"), ("s", 2, F.TYPE_BYTES, O, None),
                      ("i", 3, F.TYPE_INT64, O, None), ("f", 4, F.TYPE_FLOAT, O, None), ("b", 5, F.TYPE_BOOL, O, None),
                      ("type", 6, DT[0], O, DT[1]), ("shape", 7, F.TYPE_MESSAGE, O, ".tfpb.TensorShapeProto"),
                      ("tensor", 8, F.TYPE_MESSAGE, O, ".tfpb.TensorProto")])
    nd = msg("NodeDef", [("name", 1, F.TYPE_STRING, O, None), ("op", 2, F.TYPE_STRING, O, None),
                         ("input", 3, F.TYPE_STRING, R, None), ("device", 4, F.TYPE_STRING, O, None),
                         ("attr", 5, F.TYPE_MESSAGE, R, ".tfpb.NodeDef.AttrEntry")])
    e = msg("AttrEntry", [("key", 1, F.TYPE_STRING, O, None), ("value", 2, F.TYPE_MESSAGE, O, ".tfpb.AttrValue")], nd)
    e.options.map_entry = True
    msg("VersionDef", [("producer", 1, F.TYPE_INT32, O, None), ("min_consumer", 2, F.TYPE_INT32, O, None)])
    msg("GraphDef", [("node", 1, F.TYPE_MESSAGE, R, ".tfpb.NodeDef"),
                     ("versions", 4, F.TYPE_MESSAGE, O, ".tfpb.VersionDef")])
    msg("SaverDef", [("filename_tensor_name", 1, F.TYPE_STRING, O, None), ("save_tensor_name", 2, F.TYPE_STRING, O, None),
                     ("restore_op_name", 3, F.TYPE_STRING, O, None), ("max_to_keep", 4, F.TYPE_INT32, O, None),
                     ("sharded", 5, F.TYPE_BOOL, O, None), ("keep_checkpoint_every_n_hours", 6, F.TYPE_FLOAT, O, None),
                     ("version", 7, F.TYPE_INT32, O, None)])
    msg("TensorInfo", [("name", 1, F.TYPE_STRING, O, None), ("dtype", 2, DT[0], O, DT[1]),
                       ("tensor_shape", 3, F.TYPE_MESSAGE, O, ".tfpb.TensorShapeProto")])
    sd = msg("SignatureDef", [("inputs", 1, F.TYPE_MESSAGE, R, ".tfpb.SignatureDef.InputsEntry"),
                              ("outputs", 2, F.TYPE_MESSAGE, R, ".tfpb.SignatureDef.OutputsEntry"),
                              ("method_name", 3, F.TYPE_STRING, O, None)])
    for name in ("InputsEntry", "OutputsEntry"):
        e = msg(name, [("key", 1, F.TYPE_STRING, O, None), ("value", 2, F.TYPE_MESSAGE, O, ".tfpb.TensorInfo")], sd)
        e.options.map_entry = True
    msg("MetaInfoDef", [("meta_graph_version", 1, F.TYPE_STRING, O, None), ("tags", 4, F.TYPE_STRING, R, None),
                        ("tensorflow_version", 5, F.TYPE_STRING, O, None)])
    mg = msg("MetaGraphDef", [("meta_info_def", 1, F.TYPE_MESSAGE, O, ".tfpb.MetaInfoDef"),
                              ("graph_def", 2, F.TYPE_MESSAGE, O, ".tfpb.GraphDef"),
                              ("saver_def", 3, F.TYPE_MESSAGE, O, ".tfpb.SaverDef"),
                              ("signature_def", 5, F.TYPE_MESSAGE, R, ".tfpb.MetaGraphDef.SignatureDefEntry")])
    e = msg("SignatureDefEntry", [("key", 1, F.TYPE_STRING, O, None),
                                  ("value", 2, F.TYPE_MESSAGE, O, ".tfpb.SignatureDef")], mg)
    e.options.map_entry = True
    msg("SavedModel", [("saved_model_schema_version", 1, F.TYPE_INT64, O, None),
                       ("meta_graphs", 2, F.TYPE_MESSAGE, R, ".tfpb.MetaGraphDef")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    out = {}
    for name in ("GraphDef", "MetaGraphDef", "SavedModel", "NodeDef", "AttrValue"):
        out[name] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"tfpb.{name}"))
    return out


def graph_def_text(graph_def_bytes: bytes) -> str:
    """Text-format rendering of a binary GraphDef (what TensorFlow's ``graph.pbtxt`` holds)."""
    from google.protobuf import text_format
    g = classes()["GraphDef"]()
    g.ParseFromString(graph_def_bytes)
    return text_format.MessageToString(g)


def parse_graph_def_text(text: str):
    from google.protobuf import text_format
    return text_format.Parse(text, classes()["GraphDef"]())
