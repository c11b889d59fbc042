"""Contract testers (reference python/tests/test_microservice_tester.py,
test_api_tester.py, test_serving_test_gen.py)."""
import json

import numpy as np
import pandas as pd
import pytest

import seldon_core_amd as sca
from seldon_core_amd import testers

CONTRACT = {
    "features": [
        {"name": "sepal_length", "dtype": "FLOAT", "ftype": "continuous", "range": [4, 8]},
        {"name": "petal", "dtype": "INT", "ftype": "continuous", "range": [0, 10], "repeat": 2},
        {"name": "free", "dtype": "FLOAT", "ftype": "continuous", "range": ["inf", "inf"]},
    ],
    "targets": [{"name": "class", "dtype": "FLOAT", "ftype": "continuous", "range": [0, 1], "repeat": 3}],
}


def test_unfold_and_generate():
    c = testers.unfold_contract(CONTRACT)
    assert [f["name"] for f in c["features"]] == ["sepal_length", "petal1", "petal2", "free"]
    assert [t["name"] for t in c["targets"]] == ["class:0", "class:1", "class:2"]
    b = testers.generate_batch(c, 50)
    assert b.shape == (50, 4)
    assert ((b[:, 0] >= 4) & (b[:, 0] <= 8)).all()
    assert (b[:, 1] == np.round(b[:, 1])).all()


def test_categorical_mixed_batch():
    c = {"features": [{"name": "a", "ftype": "categorical", "values": ["x", "y"]},
                      {"name": "b", "ftype": "continuous", "dtype": "FLOAT", "range": [0, 1]}], "targets": []}
    b = testers.generate_batch(c, 7)
    assert b.shape == (7, 2) and set(b[:, 0]) <= {"x", "y"}


def test_serving_test_gen(tmp_path):
    df = pd.DataFrame({"f": [1.0, 2.5, 3.0], "i": [1, 5, 3], "cat": ["a", "b", "a"], "y": [0, 1, 0]})
    out = tmp_path / "contract.json"
    assert testers.create_seldon_api_testing_file(df, "y", str(out))
    c = json.loads(out.read_text())
    feats = {f["name"]: f for f in c["features"]}
    assert feats["f"] == {"name": "f", "ftype": "continuous", "dtype": "FLOAT", "range": [1.0, 3.0]}
    assert feats["i"]["dtype"] == "INTEGER" and feats["i"]["range"] == [1, 5]
    assert feats["cat"]["values"] == ["a", "b"]
    assert c["targets"][0]["name"] == "y"


@pytest.fixture(scope="module")
def server():
    d = sca.Deployment(None, device=-1)
    h = d.serve(http_port=0, grpc_port=0, threads=2, host="127.0.0.1")
    yield h
    d.close()


@pytest.mark.parametrize("grpc", [False, True])
def test_api_tester_against_engine(server, tmp_path, grpc):
    path = tmp_path / "c.json"
    path.write_text(json.dumps(CONTRACT))
    port = server.grpc_port if grpc else server.http_port
    argv = ["api", str(path), "127.0.0.1", str(port), "mymodel", "--namespace", "seldon", "-n", "3", "-b", "2",
            "--endpoint", "send-feedback"] + (["--grpc"] if grpc else [])
    assert testers.main(argv) == 0


def test_microservice_tester(tmp_path):
    from seldon_core_amd.microservice import build_microservice

    class M:
        def predict(self, X, names):
            return np.asarray(X, float).sum(axis=1, keepdims=True)

    d = build_microservice(M(), "MODEL", name="m", device=-1)
    h = d.C.HttpServer(d.engine, "127.0.0.1", [0], 2, "m", True, "")
    h.start()
    try:
        path = tmp_path / "c.json"
        path.write_text(json.dumps(CONTRACT))
        assert testers.main(["micro", str(path), "127.0.0.1", str(h.ports[0]), "-n", "2", "-t"]) == 0
    finally:
        h.stop()
        d.close()


def test_loadtester_predict_and_feedback(server):
    from seldon_core_amd import loadtester

    out = loadtester.run_predict_load("127.0.0.1", server.http_port, "rest", users=8, threads=1, steps=1, warmup=0,
                                      step_requests=200)
    assert out["errors"] == 0 and out["ok"] >= 200
    g = loadtester.run_predict_load("127.0.0.1", server.grpc_port, "grpc", users=8, threads=1, steps=1, warmup=0,
                                    step_requests=200, data_size=6)
    assert g["errors"] == 0
    fb = loadtester.run_feedback_load("127.0.0.1", server.http_port, "none", [1.0], requests=20, workers=4,
                                      namespace="seldon")
    assert fb["requests"] == 20
