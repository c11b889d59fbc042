"""Proxies to external inference services.

The reference ships thin Python components that forward a Seldon request to
another server: TF Serving REST ``/v1/models/<m>:predict``
(integrations/tfserving/TfServingProxy.py:20-125), NVIDIA TensorRT Inference
Server HTTP inference (integrations/nvidia-inference-server/TRTProxy.py:31-81)
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
