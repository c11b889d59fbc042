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
