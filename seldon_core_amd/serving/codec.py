"""SeldonMessage payload codecs for Python components (JSON-dict form).

Behaviour parity with the reference wrapper's REST path
(python/seldon_core/utils.py: extract_request_parts_json 472-525,
construct_response_json 306-407, array_to_rest_datadef 202-236): numeric
results keep the request's DefaultData kind (tensor / ndarray / tftensor),
non-numeric results become ndarray, strings -> strData, bytes -> binData
(base64), dict payloads echo as jsonData.  ``tftensor`` is handled without
TensorFlow: TensorProto JSON <-> numpy is implemented here directly.
"""
from __future__ import annotations

import base64
import json
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np

from .errors import SeldonMicroserviceException
from .user_model import (client_class_names, client_custom_metrics, client_custom_tags,
                         client_feature_names)

# -------------------------------------------------------------- tftensor
_TF_DTYPES = {
    "DT_FLOAT": np.float32, "DT_DOUBLE": np.float64, "DT_INT32": np.int32, "DT_UINT8": np.uint8,
    "DT_INT16": np.int16, "DT_INT8": np.int8, "DT_STRING": object, "DT_INT64": np.int64,
    "DT_BOOL": np.bool_, "DT_UINT16": np.uint16, "DT_HALF": np.float16, "DT_UINT32": np.uint32,
    "DT_UINT64": np.uint64, "DT_COMPLEX64": np.complex64, "DT_COMPLEX128": np.complex128,
}
_TF_ENUM = ["DT_INVALID", "DT_FLOAT", "DT_DOUBLE", "DT_INT32", "DT_UINT8", "DT_INT16", "DT_INT8", "DT_STRING",
            "DT_COMPLEX64", "DT_INT64", "DT_BOOL", "DT_QINT8", "DT_QUINT8", "DT_QINT32", "DT_BFLOAT16", "DT_QINT16",
            "DT_QUINT16", "DT_UINT16", "DT_COMPLEX128", "DT_HALF", "DT_RESOURCE", "DT_VARIANT", "DT_UINT32",
            "DT_UINT64"]
_TF_VALS = {
    "DT_FLOAT": "floatVal", "DT_DOUBLE": "doubleVal", "DT_INT32": "intVal", "DT_UINT8": "intVal",
    "DT_INT16": "intVal", "DT_INT8": "intVal", "DT_UINT16": "intVal", "DT_INT64": "int64Val",
    "DT_BOOL": "boolVal", "DT_STRING": "stringVal", "DT_HALF": "halfVal", "DT_UINT32": "uint32Val",
    "DT_UINT64": "uint64Val",
}
_NP_TO_TF = {np.dtype(np.float32): "DT_FLOAT", np.dtype(np.float64): "DT_DOUBLE", np.dtype(np.int32): "DT_INT32",
             np.dtype(np.uint8): "DT_UINT8", np.dtype(np.int16): "DT_INT16", np.dtype(np.int8): "DT_INT8",
             np.dtype(np.int64): "DT_INT64", np.dtype(np.bool_): "DT_BOOL", np.dtype(np.uint16): "DT_UINT16",
             np.dtype(np.float16): "DT_HALF", np.dtype(np.uint32): "DT_UINT32", np.dtype(np.uint64): "DT_UINT64"}


def _camel_get(d: Dict, camel: str):
    snake = "".join("_" + c.lower() if c.isupper() else c for c in camel)
    return d.get(camel, d.get(snake))


def tftensor_to_array(t: Dict) -> np.ndarray:
    dtype_name = t.get("dtype", "DT_FLOAT")
    if isinstance(dtype_name, int):  # enum number (tensorflow/core/framework/types.proto)
        dtype_name = _TF_ENUM[dtype_name] if 0 <= dtype_name < len(_TF_ENUM) else "DT_INVALID"
    np_dtype = _TF_DTYPES.get(dtype_name)
    if np_dtype is None:
        raise SeldonMicroserviceException(f"Unsupported tftensor dtype {dtype_name}")
    shape_d = _camel_get(t, "tensorShape") or {}
    shape = [int(d.get("size", 0)) for d in shape_d.get("dim", [])]
    n = int(np.prod(shape)) if shape else 1
    content = _camel_get(t, "tensorContent")
    if content:
        raw = base64.b64decode(content)
        return np.frombuffer(raw, dtype=np_dtype).reshape(shape).copy()
    vals = _camel_get(t, _TF_VALS.get(dtype_name, "floatVal")) or []
    if dtype_name == "DT_STRING":
        arr = np.array([base64.b64decode(v) for v in vals], dtype=object)
    elif dtype_name == "DT_HALF":
        arr = np.array([int(v) for v in vals], dtype=np.uint16).view(np.float16)
    else:
        arr = np.array([float(v) if np_dtype in (np.float32, np.float64) else v for v in vals]).astype(np_dtype)
    if arr.size == n:
        return arr.reshape(shape)
    if arr.size == 1 or (arr.size == 0 and n > 0):
        return np.full(shape, arr[0] if arr.size else 0, dtype=arr.dtype if arr.size else np_dtype)
    raise SeldonMicroserviceException("tftensor value count does not match shape")


def array_to_tftensor(arr: np.ndarray) -> Dict:
    arr = np.asarray(arr)
    shape = {"dim": [{"size": str(s)} for s in arr.shape]}
    if arr.dtype.kind in ("U", "S", "O"):
        vals = [base64.b64encode(x if isinstance(x, bytes) else str(x).encode()).decode() for x in arr.ravel()]
        return {"dtype": "DT_STRING", "tensorShape": shape, "stringVal": vals}
    name = _NP_TO_TF.get(arr.dtype)
    if name is None:
        arr = arr.astype(np.float64)
        name = "DT_DOUBLE"
    return {"dtype": name, "tensorShape": shape,
            "tensorContent": base64.b64encode(np.ascontiguousarray(arr).tobytes()).decode()}


# -------------------------------------------------------------- helpers
def is_numeric(arr: np.ndarray) -> bool:
    return np.issubdtype(arr.dtype, np.number)


class NumpyJSONEncoder(json.JSONEncoder):
    def default(self, o):  # noqa: D401
        if isinstance(o, np.ndarray):
            return o.tolist()
        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, (bytes, bytearray)):
            return base64.b64encode(o).decode()
        return super().default(o)


def dumps(obj: Any) -> str:
    return json.dumps(_wire_arrays(obj), cls=NumpyJSONEncoder)


def _wire_arrays(obj: Any) -> Any:
    """A reply whose ``data.tensor`` / ``data.tftensor`` is a numpy array (a raw
    hook may return one: inside an engine graph it travels densely, see
    PythonUnit.call_json) in its wire form: ``{"shape", "values"}`` / a
    TensorProto JSON."""
    if not isinstance(obj, dict) or not isinstance(obj.get("data"), dict):
        return obj
    data = obj["data"]
    t, tf = data.get("tensor"), data.get("tftensor")
    if not isinstance(t, np.ndarray) and not isinstance(tf, np.ndarray):
        return obj
    data = dict(data)
    if isinstance(t, np.ndarray):
        data["tensor"] = {"shape": list(t.shape), "values": t.ravel().tolist()}
    if isinstance(tf, np.ndarray):
        data["tftensor"] = array_to_tftensor(tf)
    return dict(obj, data=data)


def array_to_rest_datadef(data_type: str, array: np.ndarray, names: Optional[List[str]] = None) -> Dict:
    names = [] if names is None else list(names)
    dd: Dict[str, Any] = {"names": names}
    if data_type == "tensor":
        dd["tensor"] = {"shape": list(array.shape), "values": array.ravel().tolist()}
    elif data_type == "tftensor":
        dd["tftensor"] = array_to_tftensor(array)
    else:
        dd["ndarray"] = array.tolist()
    return dd


def datadef_to_array(datadef: Optional[Dict]) -> np.ndarray:
    if not datadef:
        return np.array([])
    if "tensor" in datadef:
        t = datadef["tensor"]
        return np.array(t.get("values", [])).reshape(t.get("shape", [-1]))
    if "ndarray" in datadef:
        return np.array(datadef["ndarray"])
    if "tftensor" in datadef:
        return tftensor_to_array(datadef["tftensor"])
    return np.array([])


def extract_request_parts_json(request: Any) -> Tuple[Any, Optional[Dict], Optional[Dict], str]:
    if not isinstance(request, dict):
        raise SeldonMicroserviceException(f"Invalid request data type: {request}")
    meta = request.get("meta", None)
    datadef = None
    if "data" in request:
        data_type = "data"
        datadef = request["data"]
        features = datadef_to_array(datadef)
    elif "jsonData" in request:
        data_type = "jsonData"
        features = request["jsonData"]
    elif "strData" in request:
        data_type = "strData"
        features = request["strData"]
    elif "binData" in request:
        data_type = "binData"
        features = bytes(request["binData"], "utf8")
    else:
        raise SeldonMicroserviceException(f"Invalid request data type: {request}")
    return features, meta, datadef, data_type


def construct_response_json(user_model: Any, is_request: bool, client_request_raw: Dict,
                            client_raw_response: Any) -> Dict:
    response: Dict[str, Any] = {}
    if "jsonData" in client_request_raw:
        response["jsonData"] = client_raw_response
    elif isinstance(client_raw_response, (bytes, bytearray)):
        response["binData"] = base64.b64encode(client_raw_response).decode("utf-8")
    elif isinstance(client_raw_response, str):
        response["strData"] = client_raw_response
    else:
        if isinstance(client_raw_response, np.ndarray):
            arr, lst = client_raw_response, client_raw_response.tolist()
        elif isinstance(client_raw_response, list):
            arr, lst = np.array(client_raw_response), client_raw_response
        else:
            raise SeldonMicroserviceException(
                "Unknown data type returned as payload (must be list or np array):" + str(client_raw_response))
        data: Dict[str, Any] = {}
        req_data = client_request_raw.get("data") if isinstance(client_request_raw, dict) else None
        if "data" in client_request_raw:
            if is_numeric(arr):
                if "tensor" in req_data:
                    data["tensor"] = {"values": arr.ravel().tolist(), "shape": list(arr.shape)}
                elif "tftensor" in req_data:
                    data["tftensor"] = array_to_tftensor(arr)
                else:
                    data["ndarray"] = lst
            else:
                data["ndarray"] = lst
        else:
            if is_numeric(arr):
                data["tensor"] = {"values": arr.ravel().tolist(), "shape": list(arr.shape)}
            else:
                data["ndarray"] = lst
        if is_request:
            req_names = (req_data or {}).get("names", [])
            names = client_feature_names(user_model, req_names)
        else:
            names = client_class_names(user_model, arr)
        data["names"] = list(names)
        response["data"] = data
    meta: Dict[str, Any] = {}
    tags = client_custom_tags(user_model)
    if tags:
        meta["tags"] = tags
    metrics = client_custom_metrics(user_model)
    if metrics:
        meta["metrics"] = metrics
    puid = (client_request_raw.get("meta") or {}).get("puid") if isinstance(client_request_raw, dict) else None
    if puid:
        meta["puid"] = puid
    response["meta"] = meta
    return response


def get_data_from_json(message: Dict) -> Union[np.ndarray, str, bytes, Dict]:
    """Payload of a SeldonMessage dict (numpy for DefaultData)."""
    if "data" in message:
        return datadef_to_array(message["data"])
    if "binData" in message:
        return base64.b64decode(message["binData"])
    if "strData" in message:
        return message["strData"]
    if "jsonData" in message:
        return message["jsonData"]
    raise SeldonMicroserviceException("Unknown data in SeldonMessage")
