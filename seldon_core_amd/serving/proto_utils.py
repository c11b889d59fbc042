"""Protobuf-side helpers of the reference's ``seldon_core.utils``
(python/seldon_core/utils.py: json <-> SeldonMessage / Feedback /
SeldonMessageList, DefaultData <-> numpy, request/response construction on
proto messages) over this package's ``prediction_pb2``.

The JSON-side helpers live in :mod:`seldon_core_amd.serving.codec`; these
functions reuse them so a proto request and its JSON form are handled by one
set of rules: a proto message is converted to its JSON dict
(``json_format.MessageToDict``), processed, and parsed back where a proto is
returned.  ``tftensor`` payloads are decoded with the codec's TensorProto
reader (no TensorFlow).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
from google.protobuf import json_format, struct_pb2

from ..proto import prediction_pb2
from .codec import (array_to_rest_datadef, construct_response_json, datadef_to_array, extract_request_parts_json,
                    get_data_from_json)
from .errors import SeldonMicroserviceException


def _parse(message_json: Dict, msg) -> Any:
    if not isinstance(message_json, dict):
        raise SeldonMicroserviceException(f"Invalid JSON: expected an object, got {type(message_json).__name__}")
    try:
        json_format.ParseDict(message_json, msg)
    except json_format.ParseError as e:
        raise SeldonMicroserviceException(f"Invalid JSON: {e}")
    return msg


def json_to_seldon_message(message_json: Dict) -> "prediction_pb2.SeldonMessage":
    return _parse(message_json or {}, prediction_pb2.SeldonMessage())


def json_to_feedback(message_json: Dict) -> "prediction_pb2.Feedback":
    return _parse(message_json or {}, prediction_pb2.Feedback())


def json_to_seldon_messages(message_json: Dict) -> "prediction_pb2.SeldonMessageList":
    return _parse(message_json or {}, prediction_pb2.SeldonMessageList())


def _to_json(msg) -> Dict:
    return json_format.MessageToDict(msg)


seldon_message_to_json = _to_json
seldon_messages_to_json = _to_json
feedback_to_json = _to_json


def get_meta_from_proto(request) -> Dict:
    return json_format.MessageToDict(request.meta) if request.HasField("meta") else {}


def grpc_datadef_to_array(datadef) -> np.ndarray:
    """``DefaultData`` (tensor / ndarray / tftensor) -> numpy."""
    return datadef_to_array(json_format.MessageToDict(datadef))


def get_data_from_proto(request) -> Union[np.ndarray, str, bytes, Dict]:
    """The request's payload: a numpy array for ``data``, else ``binData``
    bytes, ``strData`` text or the ``jsonData`` object."""
    which = request.WhichOneof("data_oneof")
    if which == "data":
        return grpc_datadef_to_array(request.data)
    if which == "binData":
        return request.binData
    if which == "strData":
        return request.strData
    if which == "jsonData":
        return json_format.MessageToDict(request.jsonData)
    raise SeldonMicroserviceException("Unknown data in SeldonMessage")


def array_to_list_value(array: np.ndarray, lv: Optional[struct_pb2.ListValue] = None) -> struct_pb2.ListValue:
    lv = struct_pb2.ListValue() if lv is None else lv
    lv.extend(np.asarray(array).tolist())
    return lv


def array_to_grpc_datadef(data_type: str, array: np.ndarray, names: Optional[List[str]] = None):
    """numpy -> ``DefaultData`` of ``data_type`` (tensor / ndarray / tftensor)."""
    dd = prediction_pb2.DefaultData()
    json_format.ParseDict(array_to_rest_datadef(data_type, np.asarray(array), names), dd)
    return dd


def extract_request_parts(request) -> Tuple[Any, Dict, Any, str]:
    """(features, meta, datadef, data_type) of a proto SeldonMessage -- the
    datadef as the request's ``DefaultData`` (None for non-``data`` payloads)."""
    features, meta, _, data_type = extract_request_parts_json(seldon_message_to_json(request))
    datadef = request.data if request.WhichOneof("data_oneof") == "data" else None
    return features, meta or {}, datadef, data_type


def extract_feedback_request_parts(request) -> Tuple[Any, np.ndarray, Optional[np.ndarray], float]:
    """(request datadef, request features, truth, reward) of a proto Feedback."""
    features = grpc_datadef_to_array(request.request.data)
    truth = grpc_datadef_to_array(request.truth.data) if request.HasField("truth") else None
    return request.request.data, features, truth, request.reward


def construct_response(user_model: Any, is_request: bool, client_request, client_raw_response) -> Any:
    """The proto form of :func:`codec.construct_response_json`: same data type
    as the request, the component's class names, tags and metrics in meta."""
    out = construct_response_json(user_model, is_request, seldon_message_to_json(client_request),
                                  client_raw_response)
    return json_to_seldon_message(out)


def get_data_from_json_message(message: Dict):
    """JSON counterpart kept next to the proto reader for symmetry."""
    return get_data_from_json(message)
