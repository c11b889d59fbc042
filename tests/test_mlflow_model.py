"""MLFLOW_SERVER reads ``MLmodel`` (reference servers/mlflowserver/mlflowserver/
MLFlowServer.py:23-27 -> ``mlflow.pyfunc.load_model``).  mlflow is not
importable, so parity with mlflow itself is unpinned: the ``MLmodel`` files here
are hand-written in the layouts mlflow 1.x writes (sklearn + python_function,
xgboost, pytorch, signature blocks) and predictions are checked against the
estimator / booster / module they were written from."""
import json
import pickle

import numpy as np
import pytest
import yaml

from seldon_core_amd.servers import MLFlowServer, load_prepackaged
from seldon_core_amd.servers.mlflow_model import MLmodelError, MLModel, parse_signature

WINE = ["fixed_acidity", "volatile_acidity", "citric_acid", "residual_sugar", "chlorides", "free_sulfur",
        "total_sulfur", "density", "ph", "sulphates", "alcohol"]  # servers/mlflowserver/test/contract.json


def _write_mlmodel(root, flavors, signature=None):
    doc = {"artifact_path": "model", "flavors": flavors, "run_id": "0" * 32}
    if signature is not None:
        doc["signature"] = {"inputs": json.dumps(signature)}
    (root / "MLmodel").write_text(yaml.safe_dump(doc))


@pytest.fixture()
def wine_dir(tmp_path):
    from sklearn.linear_model import ElasticNet

    rng = np.random.default_rng(0)
    X = rng.uniform(0, 3, size=(200, len(WINE)))
    y = X @ np.linspace(-1, 1, len(WINE)) + 5.0
    m = ElasticNet(alpha=0.01, l1_ratio=0.5).fit(X, y)
    with open(tmp_path / "model.pkl", "wb") as f:
        pickle.dump(m, f)
    _write_mlmodel(tmp_path, {
        "python_function": {"data": "model.pkl", "env": "conda.yaml", "loader_module": "mlflow.sklearn",
                            "python_version": "3.6.8"},
        "sklearn": {"pickled_model": "model.pkl", "serialization_format": "cloudpickle",
                    "sklearn_version": "0.19.1"},
    }, signature=[{"name": n, "type": "double"} for n in WINE])
    return tmp_path, m, X


def test_sklearn_flavour_from_mlmodel(wine_dir):
    root, m, X = wine_dir
    s = MLFlowServer(str(root))
    s.load()
    assert s.flavour == "sklearn"
    assert s.signature.names == WINE
    np.testing.assert_allclose(s.predict(X[:5], WINE), m.predict(X[:5]), rtol=1e-12)
    rm = s.row_model()
    assert rm is not None  # ElasticNet -> native linear kernel
    np.testing.assert_allclose(rm.run_cpu(X[:5]).ravel(), m.predict(X[:5]), rtol=1e-12)


def test_signature_reorders_named_columns(wine_dir):
    root, m, X = wine_dir
    s = load_prepackaged("MLFLOW_SERVER", str(root), {})
    perm = np.random.default_rng(1).permutation(len(WINE))
    names = [WINE[i] for i in perm]
    np.testing.assert_allclose(s.predict(X[:3][:, perm], names), m.predict(X[:3]), rtol=1e-12)
    with pytest.raises(MLmodelError, match="missing"):
        s.predict(X[:1], ["bogus"] + WINE[1:])
    with pytest.raises(MLmodelError, match="columns|column"):
        s.predict(X[:1, :5], [])


def test_native_node_permutes_named_columns(wine_dir):
    """The MLflow node served natively (linear kernel behind the batcher)
    honours the signature too: permuted names are gathered back into
    signature order, a missing column is rejected."""
    import seldon_core_amd as sca

    root, m, X = wine_dir
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "wine", "type": "MODEL", "implementation": "MLFLOW_SERVER", "modelUri": str(root)}}
    dep = sca.Deployment(spec, device=-1)
    try:
        assert dep.engine.unit_kind("wine") == "gpu:linear"
        perm = np.random.default_rng(1).permutation(len(WINE))
        names = [WINE[i] for i in perm]
        for payload in ({"ndarray": X[:4][:, perm].tolist()},
                        {"tensor": {"shape": [4, len(WINE)], "values": X[:4][:, perm].ravel().tolist()}}):
            out = dep.predict({"data": {"names": names, **payload}})
            got = np.asarray(out["data"]["ndarray"] if "ndarray" in out["data"] else out["data"]["tensor"]["values"])
            np.testing.assert_allclose(got.ravel(), m.predict(X[:4]), rtol=1e-12)
        status, body = dep.predict_raw({"data": {"names": ["bogus"] + WINE[1:], "ndarray": X[:1].tolist()}})
        assert status != 200 and "missing signature column" in json.dumps(body), body
        # unnamed requests are taken in signature order
        out = dep.predict({"data": {"ndarray": X[:2].tolist()}})
        np.testing.assert_allclose(np.asarray(out["data"]["ndarray"]).ravel(), m.predict(X[:2]), rtol=1e-12)
    finally:
        dep.close()


def test_python_function_only_maps_loader_module(tmp_path):
    from sklearn.linear_model import LinearRegression

    X = np.random.default_rng(2).normal(size=(30, 3))
    m = LinearRegression().fit(X, X.sum(1))
    with open(tmp_path / "m.pkl", "wb") as f:
        pickle.dump(m, f)
    _write_mlmodel(tmp_path, {"python_function": {"data": "m.pkl", "loader_module": "mlflow.sklearn"}})
    s = MLFlowServer(str(tmp_path))
    s.load()
    assert s.flavour == "sklearn" and s.signature is None
    np.testing.assert_allclose(s.predict(X[:4]), m.predict(X[:4]), rtol=1e-12)


def test_xgboost_flavour(tmp_path):
    from test_xgboost_formats import _model, _oracle

    model = _model("reg:squarederror", n_trees=6, n_features=5)
    (tmp_path / "model.xgb").write_text(json.dumps(model))
    _write_mlmodel(tmp_path, {"xgboost": {"data": "model.xgb", "xgb_version": "1.7.6"},
                              "python_function": {"data": "model.xgb", "loader_module": "mlflow.xgboost"}})
    s = MLFlowServer(str(tmp_path))
    s.load()
    assert s.flavour == "xgboost"
    X = np.random.default_rng(4).normal(size=(8, 5))
    np.testing.assert_allclose(np.asarray(s.predict(X)).reshape(8, -1), _oracle(model, X), rtol=1e-6, atol=1e-6)
    assert s.row_model() is not None  # tree kernel


def test_pytorch_flavour_torchscript(tmp_path):
    import torch

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Tanh())
    (tmp_path / "data").mkdir()
    torch.jit.save(torch.jit.script(net), str(tmp_path / "data" / "model.pth"))
    _write_mlmodel(tmp_path, {"pytorch": {"model_data": "data", "pytorch_version": "2.0"}},
                   signature=[{"type": "tensor", "tensor-spec": {"dtype": "float32", "shape": [-1, 4]}}])
    s = MLFlowServer(str(tmp_path), device="cpu")
    s.load()
    assert s.flavour == "pytorch"
    X = np.random.default_rng(5).normal(size=(6, 4))
    with torch.no_grad():
        want = net(torch.as_tensor(X, dtype=torch.float32)).numpy()
    np.testing.assert_allclose(s.predict(X), want, rtol=1e-6)
    with pytest.raises(MLmodelError, match="shape"):
        s.predict(X[:, :3])


def test_unsupported_and_hostile_mlmodels(tmp_path):
    _write_mlmodel(tmp_path, {"python_function": {"loader_module": "my_custom.loader", "code": "code"}})
    with pytest.raises(MLmodelError, match="mlflow package"):
        MLModel.read(str(tmp_path)).choose()
    _write_mlmodel(tmp_path, {"onnx": {"data": "model.onnx"}})
    with pytest.raises(MLmodelError, match="no supported flavour"):
        MLModel.read(str(tmp_path)).choose()
    _write_mlmodel(tmp_path, {"sklearn": {"pickled_model": "../../etc/passwd"}})
    with pytest.raises(MLmodelError, match="escapes"):
        MLModel.read(str(tmp_path)).choose()
    _write_mlmodel(tmp_path, {"sklearn": {"pickled_model": "absent.pkl"}})
    with pytest.raises(MLmodelError, match="does not exist"):
        MLModel.read(str(tmp_path)).choose()
    (tmp_path / "MLmodel").write_text("just a string\n")
    with pytest.raises(MLmodelError, match="flavors"):
        MLModel.read(str(tmp_path))


def test_parse_signature_forms():
    assert parse_signature(None) is None
    sig = parse_signature({"inputs": '[{"name": "a", "type": "long"}, {"name": "b", "type": "long"}]'})
    out = sig.enforce(np.array([[1.0, 2.0]]), [])
    assert out.dtype == np.int64
    with pytest.raises(MLmodelError, match="unsupported"):
        parse_signature({"inputs": [{"name": "a", "type": "binary"}]})


@pytest.mark.gpu
def test_pytorch_flavour_on_gpu_replays_hip_graphs(tmp_path):
    """On a GPU the pytorch flavour serves through GraphedModule: one captured
    HIP graph per batch bucket; outputs equal eager torch at fp32 rounding for
    batches that hit, pad into and span buckets."""
    import torch

    torch.manual_seed(1)
    net = torch.nn.Sequential(torch.nn.Linear(8, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64), torch.nn.GELU(),
                              torch.nn.Linear(64, 5), torch.nn.Softmax(dim=1))
    (tmp_path / "data").mkdir()
    torch.jit.save(torch.jit.script(net), str(tmp_path / "data" / "model.pth"))
    _write_mlmodel(tmp_path, {"pytorch": {"model_data": "data", "pytorch_version": "2.0"}})
    s = MLFlowServer(str(tmp_path), device="cuda:0")
    s.load()
    gm = s._fn.graphed
    for n in (1, 3, 64, 300):
        X = np.random.default_rng(n).normal(size=(n, 8))
        with torch.no_grad():
            want = net(torch.as_tensor(X, dtype=torch.float32)).numpy()
        np.testing.assert_allclose(s.predict(X), want, rtol=1e-5, atol=1e-6)
    assert gm.graph_error is None and gm.replays >= 5 and gm.eager_calls == 0  # 300 rows: 2 pieces


@pytest.mark.gpu
def test_graphed_module_falls_back_when_capture_is_refused():
    import torch

    from seldon_core_amd.models.graphed import GraphedModule

    class HostSync(torch.nn.Module):  # .item() synchronises the host: not capturable
        def forward(self, x):
            return x * float(x.abs().max().item())

    gm = GraphedModule(HostSync(), device=0)
    X = np.arange(12, dtype=np.float32).reshape(3, 4)
    np.testing.assert_allclose(gm(X), X * 11.0)
    assert gm.graph_error is not None and gm.eager_calls >= 1
    np.testing.assert_allclose(gm(X), X * 11.0)  # keeps serving eagerly
