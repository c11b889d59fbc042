"""seldon_core.proto.prediction_pb2 -> seldon_core_amd.proto.prediction_pb2."""
from seldon_core_amd.proto import prediction_pb2 as _p

DefaultData, Feedback, Meta, Metric = _p.DefaultData, _p.Feedback, _p.Meta, _p.Metric
RequestResponse, SeldonMessage, SeldonMessageList = _p.RequestResponse, _p.SeldonMessage, _p.SeldonMessageList
Status, Tensor, DESCRIPTOR = _p.Status, _p.Tensor, _p.DESCRIPTOR
