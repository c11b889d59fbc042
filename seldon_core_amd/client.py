"""Python client for the engine (reference python/seldon_core/seldon_client.py:
SeldonClient predict / feedback / explain / microservice / microservice_feedback).

Transports: ``rest`` (JSON over HTTP/1.1) and ``grpc`` (``seldon.protos.Seldon``
or the per-node services for microservices).  Gateways: ``ambassador`` /
``istio`` build the reference's ``/seldon/<namespace>/<deployment>/api/v0.1/...``
paths (the native front end accepts them directly); ``seldon`` talks to the
engine endpoint (OAuth token flow when keys are given).  Responses are
``prediction_pb2.SeldonMessage`` objects (``client_return_type="proto"``) or
dicts (``"dict"``).
"""
from __future__ import annotations

import base64
import json
import logging
import urllib.error
import urllib.request
from typing import Any, Dict, Iterable, List, Optional

import numpy as np
from google.protobuf import json_format

from .proto import prediction_pb2
from .serving.codec import array_to_rest_datadef

logger = logging.getLogger(__name__)


class SeldonClientException(Exception):
    status_code = 400

    def __init__(self, message: str):
        super().__init__(message)
        self.message = message


class SeldonChannelCredentials:
    """TLS for the gateway connection (reference seldon_client.py:27-39).

    Field meanings follow the reference exactly, so existing client code keeps
    working: ``certificate_chain_file`` is the CA bundle the server is checked
    against (REST ``verify=``; gRPC ``root_certificates``), ``verify=False``
    skips server verification (REST), and ``root_certificates_file`` +
    ``private_key_file`` are the client's own certificate and key (mutual TLS;
    REST ``cert=(root_certificates_file, private_key_file)``, gRPC
    ``certificate_chain`` / ``private_key``)."""

    def __init__(self, verify: bool = True, root_certificates_file: Optional[str] = None,
                 private_key_file: Optional[str] = None, certificate_chain_file: Optional[str] = None):
        self.verify = verify
        self.root_certificates_file = root_certificates_file
        self.private_key_file = private_key_file
        self.certificate_chain_file = certificate_chain_file


class SeldonCallCredentials:
    """Per-call credentials: a token sent as ``X-Auth-Token`` (REST header /
    gRPC metadata) on TLS connections (reference seldon_client.py:42-48)."""

    def __init__(self, token: Optional[str] = None):
        self.token = token


def _ssl_context(cc: SeldonChannelCredentials):
    import ssl

    if cc.certificate_chain_file:
        ctx = ssl.create_default_context(cafile=cc.certificate_chain_file)
    else:
        ctx = ssl.create_default_context()
        if not cc.verify:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
    if cc.private_key_file:
        ctx.load_cert_chain(certfile=cc.root_certificates_file, keyfile=cc.private_key_file)
    return ctx


def _read(path: Optional[str]) -> Optional[bytes]:
    if not path:
        return None
    with open(path, "rb") as f:
        return f.read()


class SeldonClientPrediction:
    def __init__(self, request, response, success: bool = True, msg: str = ""):
        self.request, self.response, self.success, self.msg = request, response, success, msg

    def __repr__(self):
        return f"Success:{self.success} message:{self.msg}\nRequest:\n{self.request}\nResponse:\n{self.response}"


class SeldonClientFeedback(SeldonClientPrediction):
    pass


class SeldonClientCombine(SeldonClientPrediction):
    pass


def _payload(data, bin_data, str_data, json_data, names, payload_type, shape, meta) -> Dict:
    msg: Dict[str, Any] = {}
    if bin_data is not None:
        msg["binData"] = base64.b64encode(bin_data).decode()
    elif str_data is not None:
        msg["strData"] = str_data
    elif json_data is not None:
        msg["jsonData"] = json_data
    else:
        arr = np.random.rand(*shape) if data is None else np.asarray(data)
        msg["data"] = array_to_rest_datadef(payload_type, arr, list(names or []))
    if meta:
        msg["meta"] = meta
    return msg


def _to_proto(d: Dict, cls=None):
    m = (cls or prediction_pb2.SeldonMessage)()
    json_format.ParseDict(d, m, ignore_unknown_fields=True)
    return m


class SeldonClient:
    def __init__(self, gateway: str = "ambassador", transport: str = "rest", namespace: Optional[str] = None,
                 deployment_name: Optional[str] = None, payload_type: str = "tensor",
                 oauth_key: Optional[str] = None, oauth_secret: Optional[str] = None,
                 seldon_rest_endpoint: str = "localhost:8002", seldon_grpc_endpoint: str = "localhost:8004",
                 gateway_endpoint: str = "localhost:8003", microservice_endpoint: str = "localhost:5000",
                 grpc_max_send_message_length: int = 4 * 1024 * 1024,
                 grpc_max_receive_message_length: int = 4 * 1024 * 1024,
                 client_return_type: str = "proto", timeout: float = 30.0,
                 channel_credentials: Optional[SeldonChannelCredentials] = None,
                 call_credentials: Optional[SeldonCallCredentials] = None):
        self.config = dict(locals())
        del self.config["self"]

    def _cfg(self, kw: Dict) -> Dict:
        c = dict(self.config)
        c.update({k: v for k, v in kw.items() if v is not None})
        if c["transport"] not in ("rest", "grpc"):
            raise SeldonClientException("Valid values for transport are rest or grpc")
        if c["gateway"] not in ("ambassador", "istio", "seldon"):
            raise SeldonClientException("Valid values for gateway are ambassador, istio or seldon")
        if c["payload_type"] not in ("tensor", "ndarray", "tftensor"):
            raise SeldonClientException("Valid values for payload_type are tensor, ndarray or tftensor")
        return c

    # ------------------------------------------------------------- plumbing
    def _ret(self, c, d: Dict, cls=None):
        return d if c["client_return_type"] == "dict" else _to_proto(d, cls)

    def _rest(self, url: str, body: Dict, headers: Optional[Dict] = None, form: bool = False, timeout=30.0,
              c: Optional[Dict] = None) -> Dict:
        if form:
            data = ("json=" + urllib.request.quote(json.dumps(body))).encode()
            ctype = "application/x-www-form-urlencoded"
        else:
            data = json.dumps(body).encode()
            ctype = "application/json"
        hdrs = {"Content-Type": ctype, **self._token_headers(c), **(headers or {})}
        req = urllib.request.Request(url, data=data, headers=hdrs)
        cc = (c or {}).get("channel_credentials")
        try:
            with urllib.request.urlopen(req, timeout=timeout, context=_ssl_context(cc) if cc else None) as r:
                return json.loads(r.read())
        except urllib.error.HTTPError as e:
            raise SeldonClientException(e.read().decode())
        except urllib.error.URLError as e:
            raise SeldonClientException(f"{url}: {e.reason}")

    @staticmethod
    def _token_headers(c: Optional[Dict]) -> Dict[str, str]:
        # the reference sends the call token only on TLS connections
        if c and c.get("channel_credentials") is not None and c.get("call_credentials") is not None \
                and c["call_credentials"].token is not None:
            return {"X-Auth-Token": c["call_credentials"].token}
        return {}

    def _grpc(self, c, endpoint: str, path: str, req_bytes: bytes, metadata=None) -> bytes:
        import grpc

        opts = [("grpc.max_send_message_length", c["grpc_max_send_message_length"]),
                ("grpc.max_receive_message_length", c["grpc_max_receive_message_length"])]
        cc = c.get("channel_credentials")
        if cc is None:
            ch = grpc.insecure_channel(endpoint, options=opts)
        else:  # reference seldon_client.py:1380-1395 (secure channel + X-Auth-Token metadata)
            creds = grpc.ssl_channel_credentials(root_certificates=_read(cc.certificate_chain_file),
                                                 private_key=_read(cc.private_key_file),
                                                 certificate_chain=_read(cc.root_certificates_file))
            call = c.get("call_credentials")
            if call is not None and call.token is not None:
                tok = call.token
                creds = grpc.composite_channel_credentials(creds, grpc.metadata_call_credentials(
                    lambda context, callback: callback((("x-auth-token", tok),), None)))
            ch = grpc.secure_channel(endpoint, creds, options=opts)
        with ch:
            try:
                return ch.unary_unary(path)(req_bytes, timeout=c["timeout"], metadata=metadata)
            except grpc.RpcError as e:
                raise SeldonClientException(f"{e.code()}: {e.details()}")

    @staticmethod
    def _scheme(c) -> str:
        return "https://" if c.get("channel_credentials") is not None else "http://"

    def _gateway_base(self, c) -> str:
        sch = self._scheme(c)
        if c["gateway"] == "seldon":
            return sch + c["seldon_rest_endpoint"]
        dep, ns = c.get("deployment_name"), c.get("namespace")
        prefix = c.get("gateway_prefix")
        if prefix:
            return sch + c["gateway_endpoint"] + prefix
        if not dep:
            return sch + c["gateway_endpoint"]
        return sch + c["gateway_endpoint"] + ("/seldon/" + (ns + "/" if ns else "") + dep)

    def _oauth_headers(self, c) -> Dict[str, str]:
        if c["gateway"] != "seldon" or not c.get("oauth_key"):
            return {}
        tok = get_token(c["oauth_key"], c["oauth_secret"], c["seldon_rest_endpoint"])
        return {"Authorization": "Bearer " + tok}

    # ------------------------------------------------------------- API
    def predict(self, data: Optional[np.ndarray] = None, shape=(1, 1), names: Optional[Iterable[str]] = None,
                bin_data: Optional[bytes] = None, str_data: Optional[str] = None, json_data: Any = None,
                meta: Optional[Dict] = None, headers: Optional[Dict] = None, http_path: Optional[str] = None,
                **kw) -> SeldonClientPrediction:
        c = self._cfg(kw)
        req = _payload(data, bin_data, str_data, json_data, names, c["payload_type"], shape, meta)
        try:
            if c["transport"] == "rest":
                url = self._gateway_base(c) + (http_path or "/api/v0.1/predictions")
                resp = self._rest(url, req, {**self._oauth_headers(c), **(headers or {})}, timeout=c["timeout"], c=c)
            else:
                endpoint = c["seldon_grpc_endpoint"] if c["gateway"] == "seldon" else c["gateway_endpoint"]
                md = [("seldon", c.get("deployment_name") or ""), ("namespace", c.get("namespace") or "")]
                raw = self._grpc(c, endpoint, "/seldon.protos.Seldon/Predict",
                                 _to_proto(req).SerializeToString(), md)
                m = prediction_pb2.SeldonMessage()
                m.ParseFromString(raw)
                resp = json_format.MessageToDict(m)
            return SeldonClientPrediction(self._ret(c, req), self._ret(c, resp), True, "")
        except SeldonClientException as e:
            return SeldonClientPrediction(self._ret(c, req), None, False, e.message)

    def feedback(self, prediction_request=None, prediction_response=None, reward: float = 0.0, truth=None,
                 **kw) -> SeldonClientFeedback:
        c = self._cfg(kw)
        fb = {"reward": reward}
        for key, v in (("request", prediction_request), ("response", prediction_response), ("truth", truth)):
            if v is not None:
                fb[key] = v if isinstance(v, dict) else json_format.MessageToDict(v)
        try:
            if c["transport"] == "rest":
                resp = self._rest(self._gateway_base(c) + "/api/v0.1/feedback", fb, self._oauth_headers(c),
                                  timeout=c["timeout"], c=c)
            else:
                endpoint = c["seldon_grpc_endpoint"] if c["gateway"] == "seldon" else c["gateway_endpoint"]
                raw = self._grpc(c, endpoint, "/seldon.protos.Seldon/SendFeedback",
                                 _to_proto(fb, prediction_pb2.Feedback).SerializeToString())
                m = prediction_pb2.SeldonMessage()
                m.ParseFromString(raw)
                resp = json_format.MessageToDict(m)
            return SeldonClientFeedback(self._ret(c, fb, prediction_pb2.Feedback), self._ret(c, resp), True, "")
        except SeldonClientException as e:
            return SeldonClientFeedback(self._ret(c, fb, prediction_pb2.Feedback), None, False, e.message)

    def explain(self, data=None, shape=(1, 1), names=None, bin_data=None, str_data=None, headers=None,
                http_path=None, gateway_prefix=None, **kw) -> Dict:
        """REST explain call through the gateway to ``<dep>-explainer``
        (reference seldon_client.py:353-425, 1223-1321): returns the
        explanation JSON, or ``{"success": False, "response_code": code}``."""
        c = self._cfg(kw)
        if c["transport"] == "grpc":
            raise SeldonClientException("gRPC not supported for explain")
        req = _payload(data, bin_data, str_data, None, names, c["payload_type"], shape, None)
        dep, ns = c.get("deployment_name"), c.get("namespace")
        base = self._scheme(c) + c["gateway_endpoint"]
        if http_path is not None:
            url = f"{base}/seldon/{ns}/{dep}{http_path}"
        elif gateway_prefix is not None:
            url = f"{base}{gateway_prefix}/models/{dep}:explain"
        else:
            url = base + "/seldon/" + (ns + "/" if ns else "") + f"{dep}-explainer/models/{dep}:explain"
        body = json.dumps(req).encode()
        r = urllib.request.Request(url, data=body, headers={"Content-Type": "application/json",
                                                            **self._token_headers(c), **(headers or {})})
        cc = c.get("channel_credentials")
        try:
            with urllib.request.urlopen(r, timeout=c["timeout"], context=_ssl_context(cc) if cc else None) as resp:
                return json.loads(resp.read())
        except urllib.error.HTTPError as e:
            return {"success": False, "response_code": e.code}

    def microservice(self, method: str = "predict", data=None, shape=(1, 1), names=None, datas: Optional[List] = None,
                     ndatas: Optional[int] = None, bin_data=None, str_data=None, json_data=None, meta=None,
                     **kw):
        c = self._cfg(kw)
        ep = c["microservice_endpoint"]
        if method == "aggregate":
            n = ndatas or (len(datas) if datas else 2)
            msgs = [_payload(datas[i] if datas else None, None, None, None, names, c["payload_type"], shape, meta)
                    for i in range(n)]
            req = {"seldonMessages": msgs}
            try:
                if c["transport"] == "rest":
                    resp = self._rest(f"http://{ep}/aggregate", req, form=True, timeout=c["timeout"])
                else:
                    raw = self._grpc(c, ep, "/seldon.protos.Combiner/Aggregate",
                                     _to_proto(req, prediction_pb2.SeldonMessageList).SerializeToString())
                    m = prediction_pb2.SeldonMessage()
                    m.ParseFromString(raw)
                    resp = json_format.MessageToDict(m)
                return SeldonClientCombine(self._ret(c, req, prediction_pb2.SeldonMessageList), self._ret(c, resp))
            except SeldonClientException as e:
                return SeldonClientCombine(req, None, False, e.message)
        req = _payload(data, bin_data, str_data, json_data, names, c["payload_type"], shape, meta)
        grpc_path = {"predict": "/seldon.protos.Model/Predict", "route": "/seldon.protos.Router/Route",
                     "transform-input": "/seldon.protos.Transformer/TransformInput",
                     "transform-output": "/seldon.protos.OutputTransformer/TransformOutput"}
        if method not in grpc_path:
            raise SeldonClientException(f"Unknown method {method}")
        try:
            if c["transport"] == "rest":
                resp = self._rest(f"http://{ep}/{method}", req, form=True, timeout=c["timeout"])
            else:
                raw = self._grpc(c, ep, grpc_path[method], _to_proto(req).SerializeToString())
                m = prediction_pb2.SeldonMessage()
                m.ParseFromString(raw)
                resp = json_format.MessageToDict(m)
            return SeldonClientPrediction(self._ret(c, req), self._ret(c, resp), True, "")
        except SeldonClientException as e:
            return SeldonClientPrediction(self._ret(c, req), None, False, e.message)

    def microservice_feedback(self, prediction_request=None, prediction_response=None, reward: float = 0.0,
                              truth=None, **kw) -> SeldonClientFeedback:
        c = self._cfg(kw)
        fb = {"reward": reward}
        for key, v in (("request", prediction_request), ("response", prediction_response), ("truth", truth)):
            if v is not None:
                fb[key] = v if isinstance(v, dict) else json_format.MessageToDict(v)
        try:
            if c["transport"] == "rest":
                resp = self._rest(f"http://{c['microservice_endpoint']}/send-feedback", fb, form=True,
                                  timeout=c["timeout"])
            else:
                raw = self._grpc(c, c["microservice_endpoint"], "/seldon.protos.Model/SendFeedback",
                                 _to_proto(fb, prediction_pb2.Feedback).SerializeToString())
                m = prediction_pb2.SeldonMessage()
                m.ParseFromString(raw)
                resp = json_format.MessageToDict(m)
            return SeldonClientFeedback(fb, self._ret(c, resp), True, "")
        except SeldonClientException as e:
            return SeldonClientFeedback(fb, None, False, e.message)


def get_token(oauth_key: str, oauth_secret: str, endpoint: str) -> str:
    """OAuth client-credentials token (reference apife flow, seldon_client.py:931-966)."""
    auth = base64.b64encode(f"{oauth_key}:{oauth_secret}".encode()).decode()
    req = urllib.request.Request("http://" + endpoint + "/oauth/token", data=b"grant_type=client_credentials",
                                 headers={"Authorization": "Basic " + auth})
    with urllib.request.urlopen(req, timeout=10) as r:
        return json.loads(r.read())["access_token"]
