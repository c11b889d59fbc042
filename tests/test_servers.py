"""Native front ends: external REST/gRPC API of the engine and the internal
component API of microservice mode.

Mirrors engine/src/test/java/io/seldon/engine/api/rest/TestRestClientController.java
(health endpoints, JSON + multipart predictions, feedback, errors) and the
reference wrapper tests python/tests/test_model_microservice.py (form ``json=``,
query ``?json=``, error payloads, gRPC servicers).
"""
import base64
import json
import urllib.error
import urllib.parse
import urllib.request

import numpy as np
import pytest

import seldon_core_amd as sca


def http(port, path, data=None, ctype="application/json", method=None):
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, method=method)
    if data is not None:
        req.add_header("Content-Type", ctype)
    try:
        r = urllib.request.urlopen(req, timeout=20)
        return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


@pytest.fixture(scope="module")
def engine_server():
    d = sca.Deployment(None, device=-1)
    h = d.serve(http_port=0, grpc_port=0, threads=2, host="127.0.0.1")
    yield d, h
    d.close()


def test_health_endpoints(engine_server):
    _, h = engine_server
    p = h.http_port
    assert http(p, "/ping") == (200, "pong")
    assert http(p, "/live") == (200, "live")
    assert http(p, "/ready") == (200, "ready")
    assert http(p, "/pause") == (200, "paused")
    assert http(p, "/ready")[0] == 503
    assert http(p, "/unpause") == (200, "unpaused")
    assert http(p, "/ready") == (200, "ready")
    assert http(p, "/")[1] == "Hello World!!"
    assert http(p, "/nope")[0] == 404


def test_rest_predict_json(engine_server):
    _, h = engine_server
    st, body = http(h.http_port, "/api/v0.1/predictions", json.dumps({"data": {"ndarray": [[1.0]]}}).encode())
    assert st == 200
    out = json.loads(body)
    assert out["data"]["tensor"]["values"] == [0.1, 0.9, 0.5]


def test_rest_invalid_json(engine_server):
    _, h = engine_server
    st, body = http(h.http_port, "/api/v0.1/predictions", b'{"data": ')
    assert st == 500
    out = json.loads(body)
    assert out["code"] == 201 and out["reason"] == "Invalid JSON" and out["status"] == "FAILURE"


def test_rest_multipart(engine_server):
    _, h = engine_server
    boundary = "XyZ123"
    parts = [
        ("strData", None, b"hello multipart"),
    ]
    body = b""
    for name, fname, content in parts:
        body += f"--{boundary}\r\n".encode()
        disp = f'Content-Disposition: form-data; name="{name}"' + (f'; filename="{fname}"' if fname else "")
        body += disp.encode() + b"\r\n\r\n" + content + b"\r\n"
    body += f"--{boundary}--\r\n".encode()
    st, resp = http(h.http_port, "/api/v0.1/predictions", body, f"multipart/form-data; boundary={boundary}")
    assert st == 200 and json.loads(resp)["strData"] == "hello multipart"
    # file part -> binData
    body = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"binData\"; filename=\"x.bin\"\r\n"
            f"Content-Type: application/octet-stream\r\n\r\n").encode() + bytes([0, 1, 2, 255]) + \
           f"\r\n--{boundary}--\r\n".encode()
    st, resp = http(h.http_port, "/api/v0.1/predictions", body, f"multipart/form-data; boundary={boundary}")
    assert st == 200 and base64.b64decode(json.loads(resp)["binData"]) == bytes([0, 1, 2, 255])


def test_feedback_and_prometheus(engine_server):
    _, h = engine_server
    # one prediction of its own: the predictions series must not depend on
    # which other tests of this module ran first on this worker
    st, _ = http(h.http_port, "/api/v0.1/predictions", json.dumps({"data": {"ndarray": [[1.0]]}}).encode())
    assert st == 200
    st, body = http(h.http_port, "/api/v0.1/feedback", json.dumps({"reward": 1.0, "request": {"data": {"ndarray": [[1]]}}}).encode())
    assert (st, body) == (200, "{}")
    st, text = http(h.http_port, "/prometheus")
    assert st == 200
    assert "seldon_api_engine_server_requests_seconds_count" in text
    assert 'uri="/api/v0.1/predictions"' in text and 'quantile="0.99"' in text
    assert "seldon_api_model_feedback_total" in text


def test_grpc_external_api(engine_server, C):
    grpc = pytest.importorskip("grpc")
    _, h = engine_server
    ch = grpc.insecure_channel(f"127.0.0.1:{h.grpc_port}")
    predict = ch.unary_unary("/seldon.protos.Seldon/Predict")
    req = C.json_to_pb(json.dumps({"data": {"tensor": {"shape": [3, 2], "values": [1, 2, 3, 4, 5, 6]}}}))
    resp = predict(req, timeout=10)
    out = json.loads(C.pb_to_json(resp))
    assert out["data"]["tensor"]["values"] == [0.1, 0.9, 0.5]
    fb = ch.unary_unary("/seldon.protos.Seldon/SendFeedback")
    fb(C.feedback_json_to_pb(json.dumps({"reward": 0.5})), timeout=10)
    with pytest.raises(grpc.RpcError) as e:
        ch.unary_unary("/seldon.protos.Seldon/Nope")(req, timeout=10)
    assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
    ch.close()


def test_grpc_with_generated_style_messages(engine_server):
    """Python protobuf classes (seldon_core_amd.proto) interoperate with the native server."""
    grpc = pytest.importorskip("grpc")
    from seldon_core_amd.proto import prediction_pb2 as pb

    _, h = engine_server
    ch = grpc.insecure_channel(f"127.0.0.1:{h.grpc_port}")
    call = ch.unary_unary("/seldon.protos.Seldon/Predict", request_serializer=pb.SeldonMessage.SerializeToString,
                          response_deserializer=pb.SeldonMessage.FromString)
    msg = pb.SeldonMessage(data=pb.DefaultData(tensor=pb.Tensor(shape=[1, 2], values=[1.0, 2.0])))
    resp = call(msg, timeout=10)
    assert list(resp.data.tensor.values) == [0.1, 0.9, 0.5]
    assert resp.meta.requestPath["basic-pu"] == ""
    ch.close()


# ------------------------------------------------------------------ microservice mode
class UserObject:
    def __init__(self, metrics_ok=True):
        self.metrics_ok = metrics_ok

    def predict(self, X, features_names):
        return X

    def transform_input(self, X, names):
        return X * 2

    def route(self, X, names):
        return 22

    def aggregate(self, Xs, names):
        return Xs[0] + Xs[1]

    def send_feedback(self, features, names, reward, truth, routing=None):
        self.last_reward = reward

    def tags(self):
        return {"mytag": 1}

    def metrics(self):
        return [{"type": "COUNTER", "key": "mycounter", "value": 1}] if self.metrics_ok else [{"type": "BAD", "key": "k", "value": 1}]


@pytest.fixture
def micro():
    from seldon_core_amd.microservice import build_microservice
    from seldon_core_amd.serving.openapi import wrapper_spec_json

    obj = UserObject()
    d = build_microservice(obj, "MODEL", name="mymodel", device=-1)
    srv = d.C.HttpServer(d.engine, "127.0.0.1", [0], 2, "mymodel", True, wrapper_spec_json())
    srv.start()
    yield obj, d, srv.ports[0]
    srv.stop()
    d.close()


def test_micro_predict_form_query_and_body(micro):
    obj, d, port = micro
    payload = json.dumps({"data": {"names": ["a", "b"], "ndarray": [[1, 2]]}})
    st, body = http(port, "/predict", ("json=" + urllib.parse.quote(payload)).encode(), "application/x-www-form-urlencoded")
    assert st == 200
    out = json.loads(body)
    assert out["data"]["ndarray"] == [[1.0, 2.0]] and out["data"]["names"] == ["t:0", "t:1"]
    assert out["meta"]["tags"] == {"mytag": 1.0}
    assert out["meta"]["metrics"][0]["key"] == "mycounter"
    st, body = http(port, "/predict?json=" + urllib.parse.quote(payload))
    assert st == 200 and json.loads(body)["data"]["ndarray"] == [[1.0, 2.0]]
    st, body = http(port, "/predict", payload.encode())
    assert st == 200


def test_micro_routes(micro):
    obj, d, port = micro
    m = json.dumps({"data": {"ndarray": [[1, 2]]}})
    st, body = http(port, "/transform-input", m.encode())
    assert st == 200 and json.loads(body)["data"]["ndarray"] == [[2.0, 4.0]]
    st, body = http(port, "/route", m.encode())
    assert st == 200 and json.loads(body)["data"]["ndarray"] == [[22.0]]
    st, body = http(port, "/aggregate", json.dumps({"seldonMessages": [json.loads(m), json.loads(m)]}).encode())
    assert st == 200 and json.loads(body)["data"]["ndarray"] == [[2.0, 4.0]]
    st, body = http(port, "/send-feedback", json.dumps({"request": json.loads(m), "reward": 0.4}).encode())
    assert st == 200 and obj.last_reward == pytest.approx(0.4)
    st, body = http(port, "/seldon.json")
    assert st == 200 and "/predict" in json.loads(body)["paths"]


def test_micro_bad_data(micro):
    obj, d, port = micro
    st, body = http(port, "/predict", b"json=%7Bbad")
    assert st == 400
    out = json.loads(body)
    assert out["status"]["status"] == 1 and out["status"]["code"] == -1
    assert out["status"]["reason"] == "MICROSERVICE_BAD_DATA"
    obj.metrics_ok = False
    st, body = http(port, "/predict", json.dumps({"data": {"ndarray": [[1]]}}).encode())
    assert st == 400


def test_micro_grpc_servicers(C):
    grpc = pytest.importorskip("grpc")
    from seldon_core_amd.microservice import build_microservice

    obj = UserObject()
    d = build_microservice(obj, "MODEL", name="m", device=-1)
    g = d.C.GrpcServer(d.engine, "127.0.0.1", 0, 2, "m")
    g.start()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{g.port}")
        req = C.json_to_pb(json.dumps({"data": {"tensor": {"shape": [1, 2], "values": [1, 2]}}}))
        out = json.loads(C.pb_to_json(ch.unary_unary("/seldon.protos.Model/Predict")(req, timeout=10)))
        assert out["data"]["tensor"]["values"] == [1.0, 2.0]
        out = json.loads(C.pb_to_json(ch.unary_unary("/seldon.protos.Generic/TransformInput")(req, timeout=10)))
        assert out["data"]["tensor"]["values"] == [2.0, 4.0]
        lst = C.list_json_to_pb(json.dumps({"seldonMessages": [{"data": {"tensor": {"shape": [1, 1], "values": [3]}}}] * 2}))
        out = json.loads(C.pb_to_json(ch.unary_unary("/seldon.protos.Combiner/Aggregate")(lst, timeout=10)))
        assert out["data"]["tensor"]["values"] == [6.0]
        ch.close()
    finally:
        g.stop()
        d.close()


def test_microservice_cli_subprocess(tmp_path):
    """`python -m seldon_core_amd.microservice` serves a user class from cwd."""
    import os
    import socket
    import subprocess
    import sys
    import time

    (tmp_path / "MyModel.py").write_text(
        "class MyModel:\n    def __init__(self, scale=1.0):\n        self.scale = scale\n"
        "    def predict(self, X, names):\n        return X * self.scale\n")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PREDICTIVE_UNIT_SERVICE_PORT=str(port),
               PREDICTIVE_UNIT_PARAMETERS='[{"name":"scale","value":"3","type":"FLOAT"}]',
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.microservice", "MyModel", "REST", "--device", "-1"],
                         cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        for _ in range(200):
            try:
                st, body = http(port, "/predict", json.dumps({"data": {"ndarray": [[1, 2]]}}).encode())
                break
            except (urllib.error.URLError, ConnectionError):
                time.sleep(0.1)
        assert st == 200 and json.loads(body)["data"]["ndarray"] == [[3.0, 6.0]]
    finally:
        p.terminate()
        p.wait(timeout=20)


@pytest.mark.parametrize("proto", ["REST", "GRPC"])
def test_remote_microservice_node(proto):
    """A graph node served by an out-of-process microservice (REST or gRPC)."""
    from seldon_core_amd.microservice import build_microservice

    class Doubler:
        def predict(self, X, names):
            return X * 2

    md = build_microservice(Doubler(), "MODEL", name="remote", device=-1)
    if proto == "REST":
        srv = md.C.HttpServer(md.engine, "127.0.0.1", [0], 2, "remote", True, "")
        srv.start()
        port = srv.ports[0]
    else:
        srv = md.C.GrpcServer(md.engine, "127.0.0.1", 0, 2, "remote")
        srv.start()
        port = srv.port
    try:
        spec = {"name": "p", "componentSpecs": [{"spec": {"containers": [{"name": "remote", "image": "me/doubler:1.2"}]}}],
                "graph": {"name": "t", "implementation": "SIMPLE_ROUTER", "children": [
                    {"name": "remote", "type": "MODEL",
                     "endpoint": {"type": proto, "service_host": "127.0.0.1", "service_port": port}}]}}
        d = sca.Deployment(spec, device=-1)
        out = d.predict({"data": {"ndarray": [[1.5, 2.0]]}})
        assert out["data"]["ndarray"] == [[3.0, 4.0]]
        assert out["meta"]["requestPath"] == {"t": "", "remote": "me/doubler:1.2"}
        assert d.engine.unit_kind("remote").startswith(proto.lower())
        import time
        for _ in range(100):
            if d.ready():
                break
            time.sleep(0.05)
        assert d.ready()
        d.close()
    finally:
        srv.stop()
        md.close()
