"""External-service proxies against local fake servers, and
the MLflow sklearn flavour on the native path."""
import http.server
import json
import os
import threading

import joblib
import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.servers import MLFlowServer
from seldon_core_amd.servers.proxies import InferenceServerProxy, SagemakerProxy, TfServingRestProxy


class _Fake(http.server.BaseHTTPRequestHandler):
    def do_POST(self):
        body = self.rfile.read(int(self.headers["Content-Length"]))
        if self.path.startswith("/v1/models/m:predict"):
            inst = json.loads(body)["instances"]
            out = {"predictions": [[sum(r)] for r in inst]}
            data = json.dumps(out).encode()
        elif self.path.startswith("/v2/models/m/infer"):
            inp = json.loads(body)["inputs"][0]
            out = {"outputs": [{"name": "y", "shape": inp["shape"], "datatype": "FP32",
                                "data": [2 * v for v in inp["data"]]}]}
            data = json.dumps(out).encode()
        else:  # sagemaker invocations: CSV in, CSV out
            rows = [list(map(float, line.split(","))) for line in body.decode().splitlines()]
            data = "\n".join(str(max(r)) for r in rows).encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def log_message(self, *a):
        pass


@pytest.fixture(scope="module")
def fake():
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Fake)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield f"127.0.0.1:{srv.server_port}"
    srv.shutdown()


def test_tfserving_rest_proxy(fake):
    p = TfServingRestProxy(fake, "m")
    np.testing.assert_allclose(p.predict(np.array([[1.0, 2.0], [3.0, 4.0]]), []), [[3.0], [7.0]])


def test_inference_server_proxy(fake):
    p = InferenceServerProxy(fake, "m", output_name="y")
    np.testing.assert_allclose(p.predict(np.array([[1.0, 2.0]]), []), [[2.0, 4.0]])


def test_sagemaker_proxy(fake):
    p = SagemakerProxy(f"http://{fake}/endpoints/e/invocations")
    np.testing.assert_allclose(p.predict(np.array([[1.0, 5.0], [7.0, 2.0]]), []).ravel(), [5.0, 7.0])


def test_tensorflow_server_node_forwards(fake):
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "tf", "type": "MODEL", "implementation": "TENSORFLOW_SERVER", "modelUri": "unused",
                      "parameters": [{"name": "rest_endpoint", "value": fake, "type": "STRING"},
                                     {"name": "model_name", "value": "m", "type": "STRING"}]}}
    dep = sca.Deployment(spec, device=-1)
    try:
        out = dep.predict({"data": {"ndarray": [[1.0, 2.0, 3.0]]}})
        assert out["data"]["ndarray"] == [[6.0]]
    finally:
        dep.close()


def test_mlflow_sklearn_flavour_native(tmp_path):
    from sklearn.linear_model import LinearRegression

    rng = np.random.default_rng(0)
    X = rng.normal(size=(50, 3))
    m = LinearRegression().fit(X, X @ [1.0, 2.0, 3.0] + 0.5)
    joblib.dump(m, tmp_path / "model.joblib")
    s = MLFlowServer(str(tmp_path))
    s.load()
    rm = s.row_model()
    assert rm is not None
    np.testing.assert_allclose(rm.run_cpu(X[:4]).ravel(), m.predict(X[:4]), rtol=1e-12)


# ------------------------------------------------------------ TF Serving gRPC
@pytest.fixture(scope="module")
def fake_tfs():
    """A TF Serving ``PredictionService/Predict`` stand-in: output ``y`` is
    2*input (same dtype, same shape), output ``n`` the element count."""
    from concurrent import futures

    import grpc
    from google.protobuf import json_format

    from seldon_core_amd.proto import predict_pb2, tensor_pb2
    from seldon_core_amd.serving.codec import array_to_tftensor, tftensor_to_array

    seen = []

    def predict(req, ctx):
        seen.append(req)
        x = tftensor_to_array(json_format.MessageToDict(req.inputs["x"]))
        resp = predict_pb2.PredictResponse()
        resp.model_spec.CopyFrom(req.model_spec)
        resp.outputs["y"].CopyFrom(json_format.ParseDict(array_to_tftensor(x * 2), tensor_pb2.TensorProto()))
        resp.outputs["n"].CopyFrom(json_format.ParseDict(array_to_tftensor(np.array([x.size], dtype=np.int64)),
                                                         tensor_pb2.TensorProto()))
        return resp

    handler = grpc.method_handlers_generic_handler("tensorflow.serving.PredictionService", {
        "Predict": grpc.unary_unary_rpc_method_handler(predict, request_deserializer=predict_pb2.PredictRequest.FromString,
                                                       response_serializer=lambda m: m.SerializeToString())})
    srv = grpc.server(futures.ThreadPoolExecutor(4))
    srv.add_generic_rpc_handlers((handler,))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    yield f"127.0.0.1:{port}", seen
    srv.stop(0)


def test_tfserving_grpc_proxy_converts_dense_input(fake_tfs):
    from seldon_core_amd.serving.codec import datadef_to_array
    from seldon_core_amd.servers.proxies import TfServingGrpcProxy

    ep, seen = fake_tfs
    p = TfServingGrpcProxy(ep, "m", model_input="x", model_output="y")
    try:
        out = p.predict_raw({"data": {"ndarray": [[1.0, 2.0], [3.0, 4.5]]}})
        req = seen[-1]
        assert req.model_spec.name == "m" and req.model_spec.signature_name == "serving_default"
        assert req.inputs["x"].dtype == 1  # DT_FLOAT, as TF's make_tensor_proto infers from Python floats
        t = out["data"]["tftensor"]
        assert t["dtype"] == "DT_FLOAT"
        np.testing.assert_allclose(datadef_to_array(out["data"]), [[2.0, 4.0], [6.0, 9.0]])
        # plain predict (REST ingress / dense path) returns the numpy array
        np.testing.assert_allclose(p.predict(np.array([[1.0, 1.0]]), []), [[2.0, 2.0]])
    finally:
        p.close()


def test_tfserving_grpc_proxy_passes_tftensor_through(fake_tfs):
    from seldon_core_amd.serving.codec import datadef_to_array
    from seldon_core_amd.servers.proxies import TfServingGrpcProxy

    ep, seen = fake_tfs
    p = TfServingGrpcProxy(ep, "m", signature_name="sig", model_input="x", model_output="n")
    tft = {"dtype": "DT_DOUBLE", "tensorShape": {"dim": [{"size": "1"}, {"size": "3"}]}, "doubleVal": [1.0, 2.0, 3.0]}
    try:
        out = p.predict_raw({"data": {"tftensor": tft}})
        req = seen[-1]
        assert req.model_spec.signature_name == "sig"
        assert req.inputs["x"].dtype == 2 and list(req.inputs["x"].double_val) == [1.0, 2.0, 3.0]  # untouched
        assert datadef_to_array(out["data"]).tolist() == [3]
        with pytest.raises(ValueError, match="not supported"):
            p.predict_raw({"strData": "hi"})
    finally:
        p.close()


def test_tensorflow_server_node_over_grpc(fake_tfs):
    from seldon_core_amd.serving.codec import datadef_to_array

    ep, _ = fake_tfs
    params = [{"name": "grpc_endpoint", "value": ep, "type": "STRING"},
              {"name": "model_name", "value": "m", "type": "STRING"},
              {"name": "model_input", "value": "x", "type": "STRING"},
              {"name": "model_output", "value": "y", "type": "STRING"}]
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "tf", "type": "MODEL", "implementation": "TENSORFLOW_SERVER", "modelUri": "unused",
                      "parameters": params}}
    dep = sca.Deployment(spec, device=-1)
    try:
        out = dep.predict({"data": {"ndarray": [[1.0, 2.0, 3.0]]}})
        np.testing.assert_allclose(datadef_to_array(out["data"]), [[2.0, 4.0, 6.0]])
    finally:
        dep.close()
