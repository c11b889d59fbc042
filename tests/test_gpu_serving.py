"""End-to-end serving on the GPU: native front ends -> executor -> micro-batcher
-> HIP kernels, checked against scikit-learn / the CPU reference path."""
import json
import threading
import urllib.request

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _iris_dep(device=0, **batcher):
    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.servers import SKLearnServer

    clf = iris_logistic_regression()
    spec = {"name": "iris", "graph": {"name": "classifier", "type": "MODEL", "implementation": "SKLEARN_SERVER",
                                      "modelUri": "memory://iris"}}
    dep = sca.Deployment(spec, components={"classifier": SKLearnServer(model=clf)}, device=device,
                         batcher=batcher or None)
    return dep, clf


def test_gpu_unit_is_native():
    dep, _ = _iris_dep()
    try:
        assert dep.engine.unit_kind("classifier") == "gpu:linear"
    finally:
        dep.close()


@pytest.mark.parametrize("kind", ["ndarray", "tensor"])
def test_iris_parity(kind):
    dep, clf = _iris_dep()
    try:
        X = np.random.default_rng(0).uniform(0, 8, (33, 4))
        if kind == "ndarray":
            payload = {"data": {"ndarray": X.tolist()}}
        else:
            payload = {"data": {"tensor": {"shape": [33, 4], "values": X.ravel().tolist()}}}
        out = dep.predict(payload)
        if kind == "ndarray":
            got = np.array(out["data"]["ndarray"])
        else:
            got = np.array(out["data"]["tensor"]["values"]).reshape(out["data"]["tensor"]["shape"])
        np.testing.assert_allclose(got, clf.predict_proba(X), rtol=1e-12, atol=1e-13)
        assert out["data"]["names"] == ["t:0", "t:1", "t:2"]
        assert out["meta"]["requestPath"] == {"classifier": ""}
    finally:
        dep.close()


def test_concurrent_requests_batch_together():
    dep, clf = _iris_dep(max_batch=512)
    h = dep.serve(http_port=0, grpc_port=None, threads=4, host="127.0.0.1")
    errors = []
    rng = np.random.default_rng(1)
    rows = rng.uniform(0, 8, (64, 4))

    def worker(i):
        try:
            for j in range(20):
                x = rows[(i + j) % 64]
                req = urllib.request.Request(f"http://127.0.0.1:{h.http_port}/api/v0.1/predictions",
                                             data=json.dumps({"data": {"ndarray": [x.tolist()]}}).encode(),
                                             headers={"Content-Type": "application/json"})
                out = json.loads(urllib.request.urlopen(req, timeout=30).read())
                got = np.array(out["data"]["ndarray"])
                np.testing.assert_allclose(got, clf.predict_proba(x[None, :]), rtol=1e-12, atol=1e-13)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(32)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    h.stop()
    stats = dep.batcher_stats()["classifier"]
    dep.close()
    assert not errors, errors[:3]
    assert stats["requests"] == 32 * 20
    assert stats["batches"] <= stats["requests"]


def test_xgboost_1000_tree_graph_gpu():
    import seldon_core_amd as sca
    from seldon_core_amd.models import synthetic_xgboost
    from seldon_core_amd.servers import XGBoostServer

    ens = synthetic_xgboost(1000, 8, 32, seed=0)
    spec = {"name": "xgb", "graph": {"name": "xgb", "type": "MODEL", "implementation": "XGBOOST_SERVER",
                                     "modelUri": "memory://xgb"}}
    dep = sca.Deployment(spec, components={"xgb": XGBoostServer(ensemble=ens)}, device=0)
    try:
        assert dep.engine.unit_kind("xgb") == "gpu:tree_perfect"
        X = np.random.default_rng(2).standard_normal((256, 32))
        out = dep.predict({"data": {"tensor": {"shape": [256, 32], "values": X.ravel().tolist()}}})
        assert out["data"]["tensor"]["shape"] == [256]
        got = np.array(out["data"]["tensor"]["values"])
        np.testing.assert_allclose(got, ens.predict(X), rtol=1e-4, atol=1e-4)
    finally:
        dep.close()


def test_gpu_abtest_two_devices_or_one():
    """seldon-abtest graph: RANDOM_ABTEST over two GPU model replicas."""
    import torch

    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.servers import SKLearnServer

    ndev = torch.cuda.device_count()
    clf = iris_logistic_regression()
    spec = {"name": "ab", "graph": {"name": "ab", "implementation": "RANDOM_ABTEST",
                                    "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
                                    "children": [
                                        {"name": "a", "type": "MODEL", "device": 0},
                                        {"name": "b", "type": "MODEL", "device": 1 % ndev}]}}
    dep = sca.Deployment(spec, components={"a": SKLearnServer(model=clf), "b": SKLearnServer(model=clf)})
    try:
        seen = set()
        for _ in range(40):
            out = dep.predict({"data": {"ndarray": [[5.0, 3.0, 1.5, 0.3]]}})
            seen.add(out["meta"]["routing"]["ab"])
        assert seen == {0, 1}
    finally:
        dep.close()


def test_python_api_graph_with_a_device_call_inside_a_python_node():
    """Deployment.predict (no front-end thread): the Python OUTPUT_TRANSFORMER
    after the GPU model calls a device Mahalanobis detector synchronously; that
    detector's batcher shares GPU 0's pump with the model.  The request's
    continuations run on the shared pool (csrc/core/pool_executor.h) and the
    Python node on its own unit thread, so the pump stays free to run the
    nested device call."""
    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.servers import SKLearnServer

    C = sca.native()
    det = C.MahalanobisDevice(3, 2, 3.0, 50.0, -1.0, 1e-8, 0)

    class Post:
        def transform_output(self, X, names):
            X = np.asarray(X, dtype=np.float64)
            det.step(X)  # synchronous device call (run_ptr) on GPU 0's pump
            return X

    clf = iris_logistic_regression()
    spec = {"name": "p", "graph": {"name": "post", "type": "OUTPUT_TRANSFORMER", "children": [
        {"name": "classifier", "type": "MODEL", "implementation": "SKLEARN_SERVER", "modelUri": "memory://iris"}]}}
    dep = sca.Deployment(spec, components={"classifier": SKLearnServer(model=clf), "post": Post()}, device=0)
    try:
        assert dep.engine.unit_kind("classifier") == "gpu:linear"
        out, err = {}, []

        def call():
            try:
                for i in range(20):
                    X = np.random.default_rng(i).normal(loc=4.0, scale=1.0, size=(1 + i % 3, 4))
                    r = dep.predict({"data": {"ndarray": X.tolist()}})
                    np.testing.assert_allclose(np.asarray(r["data"]["ndarray"]), clf.predict_proba(X),
                                               rtol=0, atol=1e-12)
                out["ok"] = True
            except Exception as e:  # noqa: BLE001
                err.append(repr(e))

        th = threading.Thread(target=call, daemon=True)
        th.start()
        th.join(60)
        assert not th.is_alive(), "Deployment.predict did not finish"
        assert err == [] and out.get("ok"), err
    finally:
        dep.close()


@pytest.mark.parametrize("model", ["iris", "xgb1000"])
def test_bar_staged_rows_match_the_cpu_oracle(monkeypatch, model):
    """SCA_BATCH_INPUT=bar: the CPU writes each zero-copy batch into
    fine-grained HBM through the PCIe BAR (csrc/gpu/batcher.cc) and the
    kernel reads it there.  Answers must match the CPU oracle under
    concurrency (slots and their BAR buffers reused)."""
    import seldon_core_amd as sca
    from seldon_core_amd.utils import benchkit as bk

    monkeypatch.setenv("SCA_BATCH_INPUT", "bar")
    wl = bk.Workload(model)
    dep = sca.Deployment({"name": "p", "graph": {"name": "m", "type": "MODEL"}}, components={"m": wl.comp},
                         device=0)
    try:
        errs, worst = [], [0.0]
        cols = len(wl.row)

        def client(t):
            rng = np.random.default_rng(100 + t)
            for i in range(40):
                X = np.asarray(wl.row) + rng.normal(scale=0.5, size=(1 + (i + t) % 5, cols))
                try:
                    out = np.asarray(dep.predict({"data": {"ndarray": X.tolist()}})["data"]["ndarray"], dtype=float)
                    worst[0] = max(worst[0], float(np.abs(out.reshape(len(X), -1) - wl.oracle(X)).max()))
                except Exception as e:  # noqa: BLE001
                    errs.append(repr(e))

        th = [threading.Thread(target=client, args=(t,)) for t in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert errs == [], errs[:3]
        assert worst[0] < 1e-9, worst[0]
    finally:
        dep.close()
