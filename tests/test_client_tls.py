"""SeldonClient TLS + call credentials (reference python/seldon_core/
seldon_client.py:27-49 SeldonChannelCredentials / SeldonCallCredentials,
1170-1196 https + X-Auth-Token, 1380-1395 secure gRPC channel), against local
HTTPS and TLS gRPC servers with a self-signed certificate."""
import http.server
import json
import shutil
import ssl
import subprocess
import threading

import pytest

from seldon_core_amd.client import SeldonCallCredentials, SeldonChannelCredentials, SeldonClient

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI needed to make a test cert")


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    key, crt = d / "key.pem", d / "cert.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                    "-days", "1", "-subj", "/CN=localhost", "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost"],
                   check=True, capture_output=True)
    return str(crt), str(key)


class _Handler(http.server.BaseHTTPRequestHandler):
    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length", 0))
        self.rfile.read(n)
        body = json.dumps({"data": {"ndarray": [[1.0]]},
                           "meta": {"tags": {"token": self.headers.get("X-Auth-Token"), "path": self.path}}}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.fixture()
def https_server(cert):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(cert[0], cert[1])
    srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    yield srv.server_address[1]
    srv.shutdown()


def test_rest_https_with_ca_and_token(cert, https_server):
    sc = SeldonClient(gateway="ambassador", transport="rest", gateway_endpoint=f"127.0.0.1:{https_server}",
                      deployment_name="mymodel", namespace="ns", client_return_type="dict",
                      channel_credentials=SeldonChannelCredentials(certificate_chain_file=cert[0]),
                      call_credentials=SeldonCallCredentials(token="secret-token"))
    r = sc.predict(shape=(1, 4))
    assert r.success, r.msg
    tags = r.response["meta"]["tags"]
    assert tags["token"] == "secret-token" and tags["path"] == "/seldon/ns/mymodel/api/v0.1/predictions"
    fb = sc.feedback(prediction_request={"data": {"ndarray": [[1.0]]}}, reward=1.0)
    assert fb.success and fb.response["meta"]["tags"]["path"] == "/seldon/ns/mymodel/api/v0.1/feedback"


def test_rest_https_verification(cert, https_server):
    base = dict(gateway="ambassador", transport="rest", gateway_endpoint=f"127.0.0.1:{https_server}",
                deployment_name="m", client_return_type="dict")
    bad = SeldonClient(**base, channel_credentials=SeldonChannelCredentials())  # system CAs: self-signed fails
    r = bad.predict()
    assert not r.success and "CERTIFICATE_VERIFY_FAILED" in r.msg.upper().replace(" ", "_")
    ok = SeldonClient(**base, channel_credentials=SeldonChannelCredentials(verify=False))
    r = ok.predict()
    assert r.success and r.response["meta"]["tags"]["token"] is None  # no call credentials, no token


def test_no_credentials_means_plain_http_and_no_token():
    sc = SeldonClient(gateway="ambassador", deployment_name="m", call_credentials=SeldonCallCredentials(token="t"))
    c = sc._cfg({})
    assert sc._gateway_base(c).startswith("http://") and sc._token_headers(c) == {}


def test_grpc_secure_channel_sends_token(cert):
    import grpc
    from concurrent import futures

    from seldon_core_amd.proto import prediction_pb2

    seen = {}

    def predict(req_bytes, context):
        seen.update({k: v for k, v in context.invocation_metadata()})
        m = prediction_pb2.SeldonMessage()
        m.strData = "ok"
        return m.SerializeToString()

    handler = grpc.method_handlers_generic_handler(
        "seldon.protos.Seldon", {"Predict": grpc.unary_unary_rpc_method_handler(predict)})
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    server.add_generic_rpc_handlers((handler,))
    key = open(cert[1], "rb").read()
    crt = open(cert[0], "rb").read()
    port = server.add_secure_port("127.0.0.1:0", grpc.ssl_server_credentials([(key, crt)]))
    server.start()
    try:
        sc = SeldonClient(gateway="ambassador", transport="grpc", gateway_endpoint=f"127.0.0.1:{port}",
                          deployment_name="mymodel", namespace="ns", client_return_type="dict",
                          channel_credentials=SeldonChannelCredentials(certificate_chain_file=cert[0]),
                          call_credentials=SeldonCallCredentials(token="grpc-token"))
        r = sc.predict(shape=(1, 2))
        assert r.success, r.msg
        assert r.response["strData"] == "ok"
        assert seen["x-auth-token"] == "grpc-token" and seen["seldon"] == "mymodel" and seen["namespace"] == "ns"
    finally:
        server.stop(0)
