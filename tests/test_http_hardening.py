"""Malformed-input hardening of the native REST front end and codec
(an oversized chunk size used to wrap the bounds check and abort
the process; negative tensor dims used to reach the batcher)."""
import json
import socket
import urllib.request

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression


@pytest.fixture(scope="module")
def server():
    clf = iris_logistic_regression()
    dep = sca.Deployment({"name": "p", "graph": {"name": "clf", "type": "MODEL"}}, components={"clf": clf},
                         device=-1, batcher={"cpu_batching": True, "slots": 1})
    h = dep.serve(http_port=0, grpc_port=0, threads=2, host="127.0.0.1")
    yield dep, h
    h.stop()
    dep.close()


def _raw(port: int, data: bytes, timeout: float = 5.0) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=timeout) as s:
        s.sendall(data)
        out = b""
        try:
            while True:
                b = s.recv(65536)
                if not b:
                    break
                out += b
                if b"\r\n\r\n" in out:
                    head, _, body = out.partition(b"\r\n\r\n")
                    for line in head.split(b"\r\n"):
                        if line.lower().startswith(b"content-length:") and len(body) >= int(line.split(b":")[1]):
                            return out
        except socket.timeout:
            pass
        return out


def _post(port: int, body: dict):
    req = urllib.request.Request(f"http://127.0.0.1:{port}/api/v0.1/predictions", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=10) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read() or b"{}")


def _ok(port: int):
    st, out = _post(port, {"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}})
    assert st == 200 and len(out["data"]["ndarray"][0]) == 3


@pytest.mark.parametrize("size", [b"ffffffffffffffff", b"fffffffffffffff0", b"zz", b"-1", b"123456789abcdef0"])
def test_bad_chunk_size_is_rejected_not_fatal(server, size):
    _, h = server
    req = (b"POST /api/v0.1/predictions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
           b"Transfer-Encoding: chunked\r\n\r\n" + size + b"\r\nxx\r\n0\r\n\r\n")
    out = _raw(h.http_port, req)
    assert out.startswith(b"HTTP/1.1 4"), out[:80]
    _ok(h.http_port)  # the server is still alive


def test_valid_chunked_body_still_works(server):
    _, h = server
    body = json.dumps({"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}}).encode()
    a, b = body[:10], body[10:]
    req = (b"POST /api/v0.1/predictions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
           b"Transfer-Encoding: chunked\r\n\r\n" + b"%x\r\n" % len(a) + a + b"\r\n" + b"%x;ext=1\r\n" % len(b) + b +
           b"\r\n0\r\n\r\n")
    out = _raw(h.http_port, req)
    assert out.startswith(b"HTTP/1.1 200"), out[:200]
    assert b"ndarray" in out


@pytest.mark.parametrize("payload", [
    {"data": {"tensor": {"shape": [-2, -1], "values": [1, 2]}}},
    {"data": {"tensor": {"shape": [-1, 4], "values": [1, 2, 3, 4]}}},
    {"data": {"tftensor": {"dtype": "DT_DOUBLE", "tensorShape": {"dim": [{"size": "-1"}, {"size": "-4"}]},
                           "doubleVal": [1, 2, 3, 4]}}},
])
def test_negative_shape_is_a_client_error(server, payload):
    dep, h = server
    st, out = _post(h.http_port, payload)
    assert st in (400, 500), (st, out)
    status = out.get("status")
    assert status == "FAILURE" or (isinstance(status, dict) and status.get("status") in (1, "FAILURE")), out
    _ok(h.http_port)


def test_negative_shape_protobuf_rejected():
    C = sca.native()
    ok = C.json_to_pb(json.dumps({"data": {"tensor": {"shape": [1, 4], "values": [1, 2, 3, 4]}}}))
    assert C.pb_to_json(ok)
    # hand-craft DefaultData.tensor.shape = [-1] (int32 varint, 10-byte two's complement)
    neg = b"\x08" + b"\xff" * 9 + b"\x01"
    tensor = b"\x0a" + bytes([len(neg)]) + neg
    dd = b"\x12" + bytes([len(tensor)]) + tensor
    msg = b"\x1a" + bytes([len(dd)]) + dd
    with pytest.raises(Exception):
        C.pb_to_json(msg)


def test_distinct_gateway_paths_do_not_grow_metric_series_without_bound(server):
    """Gateway-prefixed predict paths are client-chosen: the per-uri request
    timer keeps at most 64 distinct uri labels per front-end worker (the rest
    are counted under uri="other")."""
    dep, h = server
    body = json.dumps({"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}}).encode()
    for i in range(300):
        req = urllib.request.Request(f"http://127.0.0.1:{h.http_port}/seldon/ns{i}/p/api/v0.1/predictions", data=body,
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=10) as r:
            assert r.status == 200
    with urllib.request.urlopen(f"http://127.0.0.1:{h.http_port}/prometheus", timeout=10) as r:
        text = r.read().decode()
    uris = {line.split('uri="')[1].split('"')[0] for line in text.splitlines()
            if line.startswith("seldon_api_engine_server_requests") and 'uri="' in line}
    assert any(u.startswith("/seldon/ns") for u in uris)
    assert len([u for u in uris if u.startswith("/seldon/ns")]) <= 2 * 64  # two front-end threads
    assert "other" in uris
    _ok(h.http_port)
