"""SeldonClient against the native front ends (reference python/tests/test_seldon_client.py
uses mocks; here the calls hit a real in-process engine)."""
import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.client import SeldonClient


@pytest.fixture(scope="module")
def server():
    d = sca.Deployment(None, device=-1)
    h = d.serve(http_port=0, grpc_port=0, threads=2, host="127.0.0.1")
    yield h
    d.close()


@pytest.mark.parametrize("transport", ["rest", "grpc"])
@pytest.mark.parametrize("payload_type", ["tensor", "ndarray", "tftensor"])
def test_predict_via_gateway_paths(server, transport, payload_type):
    ep = f"127.0.0.1:{server.http_port if transport == 'rest' else server.grpc_port}"
    sc = SeldonClient(deployment_name="mymodel", namespace="seldon", gateway_endpoint=ep, transport=transport,
                      payload_type=payload_type)
    r = sc.predict(data=np.array([[1.0, 2.0]]), names=["a", "b"])
    assert r.success, r.msg
    assert list(r.response.data.tensor.values) == [0.1, 0.9, 0.5]
    f = sc.feedback(prediction_request=r.request, prediction_response=r.response, reward=1.0)
    assert f.success, f.msg


def test_predict_strdata_dict_return(server):
    sc = SeldonClient(gateway="seldon", seldon_rest_endpoint=f"127.0.0.1:{server.http_port}",
                      client_return_type="dict")
    r = sc.predict(str_data="hello")
    assert r.success and r.response["strData"] == "hello"


def test_microservice_calls():
    from seldon_core_amd.microservice import build_microservice

    class M:
        def predict(self, X, names):
            return X + 1

        def aggregate(self, Xs, names):
            return np.sum(Xs, axis=0)

        def send_feedback(self, X, names, reward, truth, routing=None):
            return None

    d = build_microservice(M(), "MODEL", name="m", device=-1)
    h = d.C.HttpServer(d.engine, "127.0.0.1", [0], 2, "m", True, "")
    h.start()
    g = d.C.GrpcServer(d.engine, "127.0.0.1", 0, 2, "m")
    g.start()
    try:
        for transport, port in (("rest", h.ports[0]), ("grpc", g.port)):
            sc = SeldonClient(microservice_endpoint=f"127.0.0.1:{port}", transport=transport)
            r = sc.microservice(method="predict", data=np.array([[1.0, 2.0]]))
            assert r.success, r.msg
            assert list(r.response.data.tensor.values) == [2.0, 3.0]
            a = sc.microservice(method="aggregate", datas=[np.array([[1.0]]), np.array([[2.0]])])
            assert a.success, a.msg
            fb = sc.microservice_feedback(prediction_request=r.request, prediction_response=r.response, reward=1.0)
            assert fb.success, fb.msg
    finally:
        h.stop()
        g.stop()
        d.close()
