"""Proxies to external inference services.

The reference ships thin Python components that forward a Seldon request to
another server: TF Serving REST ``/v1/models/<m>:predict``
(integrations/tfserving/TfServingProxy.py:20-125), NVIDIA TensorRT Inference
Server HTTP inference (integrations/nvidia-inference-server/TRTProxy.py:31-81),
TF Serving gRPC ``PredictionService/Predict`` (TfServingProxy.py:39-90)
and an AWS SageMaker endpoint (integrations/sagemaker/SagemakerProxy.py:13-33).
On MI355X the models themselves are served in-process; these proxies remain
for graphs that mix in an external endpoint, using the engine's pooled HTTP
client semantics (keep-alive, timeout) from the standard library.
"""
from __future__ import annotations

import json
import urllib.request
from typing import Any, Dict, List, Optional

import numpy as np


class _HttpProxy:
    def __init__(self, timeout: float = 5.0):
        self.timeout = float(timeout)

    def _post(self, url: str, body: bytes, content_type: str = "application/json",
              headers: Optional[Dict[str, str]] = None) -> bytes:
        req = urllib.request.Request(url, data=body, headers={"Content-Type": content_type, **(headers or {})})
        with urllib.request.urlopen(req, timeout=self.timeout) as r:
            return r.read()


class TfServingRestProxy(_HttpProxy):
    """Forward to TF Serving's REST API (row format ``{"instances": X}``)."""

    def __init__(self, rest_endpoint: str, model_name: str, signature_name: str = "serving_default",
                 model_input: Optional[str] = None, model_output: Optional[str] = None, timeout: float = 5.0):
        super().__init__(timeout)
        self.url = f"http://{rest_endpoint}/v1/models/{model_name}:predict"
        self.signature_name = signature_name
        self.model_input = model_input
        self.model_output = model_output

    def predict(self, X, names, meta=None):
        inst = np.asarray(X).tolist()
        if self.model_input:
            inst = [{self.model_input: row} for row in inst]
        body = {"signature_name": self.signature_name, "instances": inst}
        out = json.loads(self._post(self.url, json.dumps(body).encode()))["predictions"]
        if self.model_output and out and isinstance(out[0], dict):
            out = [o[self.model_output] for o in out]
        return np.asarray(out)


class TfServingGrpcProxy:
    """Forward to TF Serving's gRPC ``PredictionService/Predict``.

    Behaviour of the reference's grpc branch (TfServingProxy.py:55-90): only
    ``data`` payloads are accepted (strData / binData / jsonData raise); a
    ``tftensor`` input is passed through untouched, any other DefaultData kind
    is converted to a TensorProto (``dtype``, DT_FLOAT by default as TF's
    ``make_tensor_proto`` infers from Python floats) and the response is the
    ``model_output`` tensor returned as ``tftensor``.  The channel is opened
    lazily so the component can be shipped to pool worker processes.
    """

    _MAX_MSG = 1_000_000_000

    def __init__(self, grpc_endpoint: str, model_name: str, signature_name: str = "serving_default",
                 model_input: str = "inputs", model_output: Optional[str] = None, dtype: str = "DT_FLOAT",
                 timeout: float = 5.0):
        self.grpc_endpoint = grpc_endpoint
        self.model_name = model_name
        self.signature_name = signature_name
        self.model_input = model_input
        self.model_output = model_output
        self.dtype = dtype
        self.timeout = float(timeout)
        self._call = None

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_call"] = None
        return st

    def _rpc(self):
        if self._call is None:
            import grpc

            from ..proto import TFSERVING_PREDICT, predict_pb2

            opts = [("grpc.max_send_message_length", self._MAX_MSG),
                    ("grpc.max_receive_message_length", self._MAX_MSG)]
            self._channel = grpc.insecure_channel(self.grpc_endpoint, opts)
            self._call = self._channel.unary_unary(TFSERVING_PREDICT,
                                                   request_serializer=lambda m: m.SerializeToString(),
                                                   response_deserializer=predict_pb2.PredictResponse.FromString)
        return self._call

    def _tensor(self, arr: np.ndarray):
        from ..proto import tensor_pb2

        np_dtype = {"DT_FLOAT": np.float32, "DT_DOUBLE": np.float64, "DT_INT32": np.int32,
                    "DT_INT64": np.int64}.get(self.dtype)
        if np_dtype is None:
            raise ValueError(f"TfServingGrpcProxy: unsupported dtype {self.dtype}")
        arr = np.ascontiguousarray(arr, dtype=np_dtype)
        t = tensor_pb2.TensorProto()
        t.dtype = tensor_pb2.TensorProto.DESCRIPTOR.fields_by_name["dtype"].enum_type.values_by_name[self.dtype].number
        for d in arr.shape:
            t.tensor_shape.dim.add(size=int(d))
        t.tensor_content = arr.tobytes()
        return t

    def _predict_tensor(self, tensor):
        from ..proto import predict_pb2

        req = predict_pb2.PredictRequest()
        req.model_spec.name = self.model_name
        req.model_spec.signature_name = self.signature_name
        req.inputs[self.model_input].CopyFrom(tensor)
        resp = self._rpc()(req, timeout=self.timeout)
        if self.model_output is not None:
            if self.model_output not in resp.outputs:
                raise KeyError(f"TF Serving response has no output {self.model_output!r} "
                               f"(got {sorted(resp.outputs)})")
            return resp.outputs[self.model_output]
        if len(resp.outputs) != 1:
            raise KeyError(f"model_output not set and TF Serving returned {sorted(resp.outputs)}")
        return next(iter(resp.outputs.values()))

    def predict_raw(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        from google.protobuf import json_format

        from ..proto import tensor_pb2
        from ..serving.codec import datadef_to_array

        if "data" not in msg:
            raise ValueError("strData, binData and jsonData not supported.")
        data = msg["data"]
        if "tftensor" in data:
            tensor = json_format.ParseDict(data["tftensor"], tensor_pb2.TensorProto())
        else:
            tensor = self._tensor(datadef_to_array(data))
        out = self._predict_tensor(tensor)
        return {"data": {"tftensor": json_format.MessageToDict(out)}}

    def predict(self, X, names, meta=None):
        from google.protobuf import json_format

        from ..serving.codec import tftensor_to_array

        out = self._predict_tensor(self._tensor(np.asarray(X)))
        return tftensor_to_array(json_format.MessageToDict(out))

    def close(self):
        if self._call is not None:
            self._channel.close()
            self._call = None


class InferenceServerProxy(_HttpProxy):
    """Forward to an inference server speaking the v2 (KServe/Triton) HTTP
    protocol -- the successor of the TRTIS HTTP API the reference targets."""

    def __init__(self, url: str, model_name: str, input_name: str = "input", output_name: Optional[str] = None,
                 datatype: str = "FP32", timeout: float = 5.0):
        super().__init__(timeout)
        self.url = f"http://{url}/v2/models/{model_name}/infer"
        self.input_name = input_name
        self.output_name = output_name
        self.datatype = datatype

    def predict(self, X, names, meta=None):
        arr = np.asarray(X)
        body = {"inputs": [{"name": self.input_name, "shape": list(arr.shape), "datatype": self.datatype,
                            "data": arr.ravel().tolist()}]}
        if self.output_name:
            body["outputs"] = [{"name": self.output_name}]
        outs: List[Dict[str, Any]] = json.loads(self._post(self.url, json.dumps(body).encode()))["outputs"]
        o = next((x for x in outs if self.output_name in (None, x.get("name"))), outs[0])
        return np.asarray(o["data"]).reshape(o["shape"])


class SagemakerProxy(_HttpProxy):
    """Forward to a SageMaker-style invocations endpoint (CSV rows in, CSV or
    JSON predictions out)."""

    def __init__(self, endpoint_url: str, timeout: float = 5.0, headers: Optional[Dict[str, str]] = None):
        super().__init__(timeout)
        self.url = endpoint_url if endpoint_url.startswith("http") else f"http://{endpoint_url}"
        self.headers = dict(headers or {})

    def predict(self, X, names, meta=None):
        arr = np.atleast_2d(np.asarray(X))
        body = "\n".join(",".join(repr(float(v)) for v in row) for row in arr).encode()
        raw = self._post(self.url, body, "text/csv", self.headers).decode().strip()
        try:
            return np.asarray(json.loads(raw), dtype=float)
        except ValueError:
            return np.asarray([[float(v) for v in line.split(",")] for line in raw.splitlines() if line.strip()])
