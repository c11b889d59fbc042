"""Protobuf message classes for ``prediction.proto`` built at import time.

No protoc / grpc_tools exist on this platform, so the descriptors of
``proto/prediction.proto`` (wire-compatible with the reference
proto/prediction.proto:14-128) and of the TensorFlow ``TensorProto`` it
depends on are assembled with ``descriptor_pb2`` and turned into message
classes with the protobuf runtime.  ``prediction_pb2`` exposes the same names
as a protoc-generated module (SeldonMessage, DefaultData, Tensor, Meta, Metric,
Status, Feedback, SeldonMessageList, RequestResponse).
"""
from __future__ import annotations

from types import SimpleNamespace

from google.protobuf import descriptor_pb2, descriptor_pool, struct_pb2  # noqa: F401

try:
    from google.protobuf.message_factory import GetMessageClass as _get_class
except ImportError:  # protobuf < 4.21
    from google.protobuf.message_factory import MessageFactory as _MF

    _mf = _MF()

    def _get_class(desc):
        return _mf.GetPrototype(desc)

F = descriptor_pb2.FieldDescriptorProto
T_DOUBLE, T_FLOAT, T_INT64, T_UINT64, T_INT32, T_BOOL, T_STRING, T_MESSAGE, T_BYTES, T_UINT32, T_ENUM = (
    F.TYPE_DOUBLE, F.TYPE_FLOAT, F.TYPE_INT64, F.TYPE_UINT64, F.TYPE_INT32, F.TYPE_BOOL, F.TYPE_STRING,
    F.TYPE_MESSAGE, F.TYPE_BYTES, F.TYPE_UINT32, F.TYPE_ENUM)
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED


def _field(msg, name, number, ftype, label=OPT, type_name=None, oneof=None, packed=None):
    f = msg.field.add(name=name, number=number, type=ftype, label=label)
    if type_name:
        f.type_name = type_name
    if oneof is not None:
        f.oneof_index = oneof
    if packed is not None:
        f.options.packed = packed
    return f


def _map(msg, name, number, key_type, val_type, val_type_name=None):
    entry = msg.nested_type.add(name="".join(p.capitalize() for p in name.split("_")) + "Entry")
    entry.options.map_entry = True
    _field(entry, "key", 1, key_type)
    _field(entry, "value", 2, val_type, type_name=val_type_name)
    _field(msg, name, number, T_MESSAGE, REP, f".{_map.pkg}.{msg.name}.{entry.name}")


def _build():
    pool = descriptor_pool.Default()
    try:
        pool.FindMessageTypeByName("seldon.protos.SeldonMessage")
        return pool
    except KeyError:
        pass
    # ---- tensorflow/core/framework/types.proto
    fd = descriptor_pb2.FileDescriptorProto(name="tensorflow/core/framework/types.proto", package="tensorflow",
                                            syntax="proto3")
    e = fd.enum_type.add(name="DataType")
    for i, n in enumerate(["DT_INVALID", "DT_FLOAT", "DT_DOUBLE", "DT_INT32", "DT_UINT8", "DT_INT16", "DT_INT8",
                           "DT_STRING", "DT_COMPLEX64", "DT_INT64", "DT_BOOL", "DT_QINT8", "DT_QUINT8", "DT_QINT32",
                           "DT_BFLOAT16", "DT_QINT16", "DT_QUINT16", "DT_UINT16", "DT_COMPLEX128", "DT_HALF",
                           "DT_RESOURCE", "DT_VARIANT", "DT_UINT32", "DT_UINT64"]):
        e.value.add(name=n, number=i)
    pool.Add(fd)
    # ---- resource_handle.proto
    fd = descriptor_pb2.FileDescriptorProto(name="tensorflow/core/framework/resource_handle.proto",
                                            package="tensorflow", syntax="proto3")
    m = fd.message_type.add(name="ResourceHandleProto")
    for i, n in enumerate(["device", "container", "name"], 1):
        _field(m, n, i, T_STRING)
    _field(m, "hash_code", 4, T_UINT64)
    _field(m, "maybe_type_name", 5, T_STRING)
    pool.Add(fd)
    # ---- tensor_shape.proto
    fd = descriptor_pb2.FileDescriptorProto(name="tensorflow/core/framework/tensor_shape.proto",
                                            package="tensorflow", syntax="proto3")
    m = fd.message_type.add(name="TensorShapeProto")
    d = m.nested_type.add(name="Dim")
    _field(d, "size", 1, T_INT64)
    _field(d, "name", 2, T_STRING)
    _field(m, "dim", 2, T_MESSAGE, REP, ".tensorflow.TensorShapeProto.Dim")
    _field(m, "unknown_rank", 3, T_BOOL)
    pool.Add(fd)
    # ---- tensor.proto
    fd = descriptor_pb2.FileDescriptorProto(name="tensorflow/core/framework/tensor.proto", package="tensorflow",
                                            syntax="proto3",
                                            dependency=["tensorflow/core/framework/resource_handle.proto",
                                                        "tensorflow/core/framework/tensor_shape.proto",
                                                        "tensorflow/core/framework/types.proto"])
    m = fd.message_type.add(name="TensorProto")
    _field(m, "dtype", 1, T_ENUM, type_name=".tensorflow.DataType")
    _field(m, "tensor_shape", 2, T_MESSAGE, type_name=".tensorflow.TensorShapeProto")
    _field(m, "version_number", 3, T_INT32)
    _field(m, "tensor_content", 4, T_BYTES)
    _field(m, "half_val", 13, T_INT32, REP, packed=True)
    _field(m, "float_val", 5, T_FLOAT, REP, packed=True)
    _field(m, "double_val", 6, T_DOUBLE, REP, packed=True)
    _field(m, "int_val", 7, T_INT32, REP, packed=True)
    _field(m, "string_val", 8, T_BYTES, REP)
    _field(m, "scomplex_val", 9, T_FLOAT, REP, packed=True)
    _field(m, "int64_val", 10, T_INT64, REP, packed=True)
    _field(m, "bool_val", 11, T_BOOL, REP, packed=True)
    _field(m, "dcomplex_val", 12, T_DOUBLE, REP, packed=True)
    _field(m, "resource_handle_val", 14, T_MESSAGE, REP, ".tensorflow.ResourceHandleProto")
    _field(m, "variant_val", 15, T_MESSAGE, REP, ".tensorflow.VariantTensorDataProto")
    _field(m, "uint32_val", 16, T_UINT32, REP, packed=True)
    _field(m, "uint64_val", 17, T_UINT64, REP, packed=True)
    v = fd.message_type.add(name="VariantTensorDataProto")
    _field(v, "type_name", 1, T_STRING)
    _field(v, "metadata", 2, T_BYTES)
    _field(v, "tensors", 3, T_MESSAGE, REP, ".tensorflow.TensorProto")
    pool.Add(fd)
    # ---- prediction.proto
    _map.pkg = "seldon.protos"
    fd = descriptor_pb2.FileDescriptorProto(name="prediction.proto", package="seldon.protos", syntax="proto3",
                                            dependency=["google/protobuf/struct.proto",
                                                        "tensorflow/core/framework/tensor.proto"])
    m = fd.message_type.add(name="SeldonMessage")
    m.oneof_decl.add(name="data_oneof")
    _field(m, "status", 1, T_MESSAGE, type_name=".seldon.protos.Status")
    _field(m, "meta", 2, T_MESSAGE, type_name=".seldon.protos.Meta")
    _field(m, "data", 3, T_MESSAGE, type_name=".seldon.protos.DefaultData", oneof=0)
    _field(m, "binData", 4, T_BYTES, oneof=0)
    _field(m, "strData", 5, T_STRING, oneof=0)
    _field(m, "jsonData", 6, T_MESSAGE, type_name=".google.protobuf.Value", oneof=0)
    m = fd.message_type.add(name="DefaultData")
    m.oneof_decl.add(name="data_oneof")
    _field(m, "names", 1, T_STRING, REP)
    _field(m, "tensor", 2, T_MESSAGE, type_name=".seldon.protos.Tensor", oneof=0)
    _field(m, "ndarray", 3, T_MESSAGE, type_name=".google.protobuf.ListValue", oneof=0)
    _field(m, "tftensor", 4, T_MESSAGE, type_name=".tensorflow.TensorProto", oneof=0)
    m = fd.message_type.add(name="Tensor")
    _field(m, "shape", 1, T_INT32, REP, packed=True)
    _field(m, "values", 2, T_DOUBLE, REP, packed=True)
    m = fd.message_type.add(name="Meta")
    _field(m, "puid", 1, T_STRING)
    _map(m, "tags", 2, T_STRING, T_MESSAGE, ".google.protobuf.Value")
    _map(m, "routing", 3, T_STRING, T_INT32)
    m.nested_type.add().CopyFrom(descriptor_pb2.DescriptorProto(name="RequestPathEntry"))
    rp = m.nested_type[-1]
    rp.options.map_entry = True
    _field(rp, "key", 1, T_STRING)
    _field(rp, "value", 2, T_STRING)
    _field(m, "requestPath", 4, T_MESSAGE, REP, ".seldon.protos.Meta.RequestPathEntry")
    _field(m, "metrics", 5, T_MESSAGE, REP, ".seldon.protos.Metric")
    m = fd.message_type.add(name="Metric")
    en = m.enum_type.add(name="MetricType")
    for i, n in enumerate(["COUNTER", "GAUGE", "TIMER"]):
        en.value.add(name=n, number=i)
    _field(m, "key", 1, T_STRING)
    _field(m, "type", 2, T_ENUM, type_name=".seldon.protos.Metric.MetricType")
    _field(m, "value", 3, T_FLOAT)
    _map(m, "tags", 4, T_STRING, T_STRING)
    m = fd.message_type.add(name="SeldonMessageList")
    _field(m, "seldonMessages", 1, T_MESSAGE, REP, ".seldon.protos.SeldonMessage")
    m = fd.message_type.add(name="Status")
    en = m.enum_type.add(name="StatusFlag")
    en.value.add(name="SUCCESS", number=0)
    en.value.add(name="FAILURE", number=1)
    _field(m, "code", 1, T_INT32)
    _field(m, "info", 2, T_STRING)
    _field(m, "reason", 3, T_STRING)
    _field(m, "status", 4, T_ENUM, type_name=".seldon.protos.Status.StatusFlag")
    m = fd.message_type.add(name="Feedback")
    _field(m, "request", 1, T_MESSAGE, type_name=".seldon.protos.SeldonMessage")
    _field(m, "response", 2, T_MESSAGE, type_name=".seldon.protos.SeldonMessage")
    _field(m, "reward", 3, T_FLOAT)
    _field(m, "truth", 4, T_MESSAGE, type_name=".seldon.protos.SeldonMessage")
    m = fd.message_type.add(name="RequestResponse")
    _field(m, "request", 1, T_MESSAGE, type_name=".seldon.protos.SeldonMessage")
    _field(m, "response", 2, T_MESSAGE, type_name=".seldon.protos.SeldonMessage")
    for svc, methods in SERVICES.items():
        s = fd.service.add(name=svc)
        for meth, (inp, out) in methods.items():
            s.method.add(name=meth, input_type=f".seldon.protos.{inp}", output_type=f".seldon.protos.{out}")
    pool.Add(fd)
    return pool


SERVICES = {
    "Generic": {"TransformInput": ("SeldonMessage", "SeldonMessage"), "TransformOutput": ("SeldonMessage", "SeldonMessage"),
                "Route": ("SeldonMessage", "SeldonMessage"), "Aggregate": ("SeldonMessageList", "SeldonMessage"),
                "SendFeedback": ("Feedback", "SeldonMessage")},
    "Model": {"Predict": ("SeldonMessage", "SeldonMessage"), "SendFeedback": ("Feedback", "SeldonMessage")},
    "Router": {"Route": ("SeldonMessage", "SeldonMessage"), "SendFeedback": ("Feedback", "SeldonMessage")},
    "Transformer": {"TransformInput": ("SeldonMessage", "SeldonMessage")},
    "OutputTransformer": {"TransformOutput": ("SeldonMessage", "SeldonMessage")},
    "Combiner": {"Aggregate": ("SeldonMessageList", "SeldonMessage")},
    "Seldon": {"Predict": ("SeldonMessage", "SeldonMessage"), "SendFeedback": ("Feedback", "SeldonMessage")},
}

def _build_tfserving(pool):
    """``tensorflow_serving/apis/{model,predict,prediction_service}.proto``:
    the subset the TF-Serving gRPC proxy speaks (Predict)."""
    try:
        pool.FindMessageTypeByName("tensorflow.serving.PredictRequest")
        return
    except KeyError:
        pass
    from google.protobuf import wrappers_pb2  # noqa: F401  (registers wrappers.proto in the default pool)

    _map.pkg = "tensorflow.serving"
    fd = descriptor_pb2.FileDescriptorProto(name="tensorflow_serving/apis/predict.proto",
                                            package="tensorflow.serving", syntax="proto3",
                                            dependency=["google/protobuf/wrappers.proto",
                                                        "tensorflow/core/framework/tensor.proto"])
    m = fd.message_type.add(name="ModelSpec")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_MESSAGE, type_name=".google.protobuf.Int64Value")
    _field(m, "signature_name", 3, T_STRING)
    m = fd.message_type.add(name="PredictRequest")
    _field(m, "model_spec", 1, T_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    _map(m, "inputs", 2, T_STRING, T_MESSAGE, ".tensorflow.TensorProto")
    _field(m, "output_filter", 3, T_STRING, REP)
    m = fd.message_type.add(name="PredictResponse")
    _field(m, "model_spec", 2, T_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    _map(m, "outputs", 1, T_STRING, T_MESSAGE, ".tensorflow.TensorProto")
    s = fd.service.add(name="PredictionService")
    s.method.add(name="Predict", input_type=".tensorflow.serving.PredictRequest",
                 output_type=".tensorflow.serving.PredictResponse")
    pool.Add(fd)


_pool = _build()
_build_tfserving(_pool)


def _cls(full_name: str):
    return _get_class(_pool.FindMessageTypeByName(full_name))


prediction_pb2 = SimpleNamespace(
    SeldonMessage=_cls("seldon.protos.SeldonMessage"),
    DefaultData=_cls("seldon.protos.DefaultData"),
    Tensor=_cls("seldon.protos.Tensor"),
    Meta=_cls("seldon.protos.Meta"),
    Metric=_cls("seldon.protos.Metric"),
    SeldonMessageList=_cls("seldon.protos.SeldonMessageList"),
    Status=_cls("seldon.protos.Status"),
    Feedback=_cls("seldon.protos.Feedback"),
    RequestResponse=_cls("seldon.protos.RequestResponse"),
    DESCRIPTOR=_pool.FindFileByName("prediction.proto"),
)
tensor_pb2 = SimpleNamespace(TensorProto=_cls("tensorflow.TensorProto"))
predict_pb2 = SimpleNamespace(ModelSpec=_cls("tensorflow.serving.ModelSpec"),
                              PredictRequest=_cls("tensorflow.serving.PredictRequest"),
                              PredictResponse=_cls("tensorflow.serving.PredictResponse"))
TFSERVING_PREDICT = "/tensorflow.serving.PredictionService/Predict"

__all__ = ["prediction_pb2", "tensor_pb2", "predict_pb2", "SERVICES", "TFSERVING_PREDICT"]
