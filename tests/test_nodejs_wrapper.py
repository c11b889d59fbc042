"""NodeJS component wrapper (wrappers/nodejs; SURVEY P1, reference
wrappers/s2i/nodejs/microservice.js): the internal REST and gRPC API of a
user JS class, called directly and as a remote node of the native engine.
Skipped when no `node` binary is on PATH."""
import json
import os
import shutil
import socket
import subprocess
import time
import urllib.parse
import urllib.request

import pytest

import seldon_core_amd as sca

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")
WRAPPER = os.path.join(ROOT, "wrappers", "nodejs", "microservice.js")
MODEL = os.path.join(ROOT, "tests", "fixtures", "nodejs", "model.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


def _free_port():
    from portutil import free_port

    return free_port()


def _start(api, service="MODEL", params=None):
    port = _free_port()
    env = dict(os.environ)
    if params is not None:
        env["PREDICTIVE_UNIT_PARAMETERS"] = json.dumps(params)
    p = subprocess.Popen([NODE, WRAPPER, "--model", MODEL, "--api", api, "--service", service, "--port", str(port),
                          "--host", "127.0.0.1"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
    deadline = time.time() + 20
    while time.time() < deadline:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.2).close()
            return p, port
        except OSError:
            if p.poll() is not None:
                raise RuntimeError(p.stdout.read())
            time.sleep(0.05)
    p.kill()
    raise RuntimeError("node wrapper did not start")


@pytest.fixture(scope="module")
def rest_server():
    p, port = _start("REST", params=[{"name": "scale", "value": "3", "type": "FLOAT"}])
    yield port
    p.terminate()
    p.wait(10)


@pytest.fixture(scope="module")
def grpc_server():
    p, port = _start("GRPC")
    yield port
    p.terminate()
    p.wait(10)


def _post(port, path, body, form=True):
    if form:
        data = urllib.parse.urlencode({"json": json.dumps(body)}).encode()
        ctype = "application/x-www-form-urlencoded"
    else:
        data, ctype = json.dumps(body).encode(), "application/json"
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, headers={"Content-Type": ctype})
    try:
        with urllib.request.urlopen(req, timeout=10) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def test_rest_predict_ndarray_and_tensor(rest_server):
    st, out = _post(rest_server, "/predict", {"data": {"names": ["a", "b"], "ndarray": [[1.0, 2.0]]},
                                              "meta": {"puid": "abc"}})
    assert st == 200
    assert out["data"] == {"names": ["t:0", "t:1"], "ndarray": [[3.0, 6.0]]}  # scale parameter 3
    assert out["meta"]["puid"] == "abc" and out["meta"]["tags"]["ready"] is True
    assert out["meta"]["metrics"] == [{"type": "COUNTER", "key": "node_requests", "value": 1}]
    st, out = _post(rest_server, "/predict", {"data": {"tensor": {"shape": [2, 2], "values": [1, 2, 3, 4]}}}, form=False)
    assert st == 200 and out["data"]["tensor"] == {"shape": [2, 2], "values": [3, 6, 9, 12]}


def test_rest_other_methods(rest_server):
    st, out = _post(rest_server, "/route", {"data": {"ndarray": [[5.0]]}})
    assert st == 200 and out["data"]["ndarray"] == [[1]]
    st, out = _post(rest_server, "/transform-input", {"data": {"ndarray": [[5.0]]}})
    assert st == 200 and out["data"]["ndarray"] == [[5.0]]  # identity when the class has no transform_input
    st, out = _post(rest_server, "/transform-output", {"data": {"ndarray": [[5.0]]}})
    assert st == 200 and out["data"]["ndarray"] == [[6.0]]  # promise-returning method
    st, out = _post(rest_server, "/aggregate", {"seldonMessages": [{"data": {"ndarray": [[1.0, 3.0]]}},
                                                                   {"data": {"ndarray": [[3.0, 5.0]]}}]})
    assert st == 200 and out["data"]["ndarray"] == [[2.0, 4.0]]
    st, out = _post(rest_server, "/send-feedback", {"request": {"data": {"ndarray": [[1.0]]}}, "reward": 1.0})
    assert st == 200
    _, out = _post(rest_server, "/predict", {"data": {"ndarray": [[1.0]]}})
    assert out["meta"]["tags"]["feedback"] >= 1


def test_rest_errors_and_health(rest_server):
    st, out = _post(rest_server, "/predict", {"nothing": 1})
    assert st == 400 and out["status"]["status"] == "FAILURE"
    req = urllib.request.Request(f"http://127.0.0.1:{rest_server}/predict", data=b"{not json",
                                 headers={"Content-Type": "application/json"})
    with pytest.raises(urllib.error.HTTPError) as ei:
        urllib.request.urlopen(req, timeout=10)
    assert ei.value.code == 400
    with urllib.request.urlopen(f"http://127.0.0.1:{rest_server}/health/ping", timeout=10) as r:
        assert r.read() == b"pong"
    q = urllib.parse.quote(json.dumps({"data": {"ndarray": [[2.0]]}}))
    with urllib.request.urlopen(f"http://127.0.0.1:{rest_server}/predict?json={q}", timeout=10) as r:
        assert json.loads(r.read())["data"]["ndarray"] == [[6.0]]


def test_grpc_predict_route_aggregate(grpc_server):
    import grpc
    from google.protobuf import json_format

    from seldon_core_amd.proto import prediction_pb2 as pb

    ch = grpc.insecure_channel(f"127.0.0.1:{grpc_server}")
    grpc.channel_ready_future(ch).result(timeout=10)
    call = lambda svc, m, req_t: ch.unary_unary(f"/seldon.protos.{svc}/{m}", request_serializer=req_t.SerializeToString,
                                                response_deserializer=pb.SeldonMessage.FromString)
    req = json_format.ParseDict({"data": {"names": ["x"], "tensor": {"shape": [1, 3], "values": [1, 2, -3.5]}},
                                 "meta": {"puid": "p1", "tags": {"t": "v"}}}, pb.SeldonMessage())
    out = call("Model", "Predict", pb.SeldonMessage)(req, timeout=10)
    assert list(out.data.tensor.shape) == [1, 3] and list(out.data.tensor.values) == [2, 4, -7]
    assert out.meta.puid == "p1" and out.meta.tags["ready"].bool_value
    assert out.meta.metrics[0].key == "node_requests"
    nd = json_format.ParseDict({"data": {"ndarray": [[-1.0, "s", True]]}}, pb.SeldonMessage())
    r = call("Router", "Route", pb.SeldonMessage)(json_format.ParseDict({"data": {"ndarray": [[-2.0]]}},
                                                                       pb.SeldonMessage()), timeout=10)
    assert json_format.MessageToDict(r)["data"]["ndarray"] == [[0]]
    lst = pb.SeldonMessageList(seldonMessages=[json_format.ParseDict({"data": {"ndarray": [[1.0]]}}, pb.SeldonMessage()),
                                               json_format.ParseDict({"data": {"ndarray": [[5.0]]}}, pb.SeldonMessage())])
    a = call("Combiner", "Aggregate", pb.SeldonMessageList)(lst, timeout=10)
    assert json_format.MessageToDict(a)["data"]["ndarray"] == [[3.0]]
    fb = pb.Feedback(request=nd, reward=0.5)
    call("Model", "SendFeedback", pb.Feedback)(fb, timeout=10)
    with pytest.raises(grpc.RpcError) as ei:
        call("Model", "Nope", pb.SeldonMessage)(req, timeout=10)
    assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
    ch.close()


@pytest.mark.parametrize("proto", ["REST", "GRPC"])
def test_engine_remote_node_is_a_nodejs_component(proto, rest_server, grpc_server):
    """The native engine calls the JS component as a remote MODEL node, over
    the internal REST (form json=) and gRPC APIs (csrc/server/remote_unit.cc)."""
    port = rest_server if proto == "REST" else grpc_server
    scale = 3.0 if proto == "REST" else 2.0
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": [{"name": "js", "image": "me/js-doubler:0.1"}]}}],
            "graph": {"name": "js", "type": "MODEL",
                                   "endpoint": {"type": proto, "service_host": "127.0.0.1", "service_port": port}}}
    d = sca.Deployment(spec, device=-1)
    try:
        out = d.predict({"data": {"ndarray": [[1.5, 2.0]]}})
        assert out["data"]["ndarray"] == [[1.5 * scale, 2.0 * scale]]
        out = d.predict({"data": {"tensor": {"shape": [1, 2], "values": [1.0, -1.0]}}})
        assert out["data"]["tensor"]["values"] == [scale, -scale]
    finally:
        d.close()


def test_builder_nodejs_context_and_run_argv(tmp_path):
    """LANGUAGE=nodejs: the s2i build context carries the wrapper and a Node
    base image; the run command is the wrapper's CLI (reference
    wrappers/s2i/nodejs/s2i/bin/run)."""
    from seldon_core_amd import builder

    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(MODEL, src / "model.js")
    (src / ".s2i").mkdir()
    (src / ".s2i" / "environment").write_text(
        "MODEL_NAME=model.js\nAPI_TYPE=REST\nSERVICE_TYPE=MODEL\nPERSISTENCE=0\nLANGUAGE=nodejs\n")
    ctx = builder.build(str(src), "me/js:0.1", context=str(tmp_path / "ctx"), docker=False)
    df = open(os.path.join(ctx, "Dockerfile")).read()
    assert df.startswith("# generated") and "FROM node:" in df and "COPY wrapper /wrapper" in df
    assert 'exec node /wrapper/microservice.js --model \\"$MODEL_NAME\\"' in df
    assert os.path.exists(os.path.join(ctx, "wrapper", "microservice.js"))
    assert os.path.exists(os.path.join(ctx, "microservice", "model.js"))
    env = builder.read_environment(str(src))
    argv = builder.node_argv(env)
    assert argv[1].endswith("microservice.js") and argv[2:6] == ["--model", "model.js", "--api", "REST"]
    with pytest.raises(builder.BuildError):
        builder.check_environment(dict(env, LANGUAGE="cobol"))
    # the command serves the component from the source directory
    port = _free_port()
    p = subprocess.Popen(argv + ["--port", str(port), "--host", "127.0.0.1"], cwd=str(src), stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True)
    try:
        for _ in range(200):
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.2).close()
                break
            except OSError:
                time.sleep(0.05)
        st, out = _post(port, "/predict", {"data": {"ndarray": [[1.0]]}})
        assert st == 200 and out["data"]["ndarray"] == [[2.0]]
    finally:
        p.terminate()
        p.wait(10)
