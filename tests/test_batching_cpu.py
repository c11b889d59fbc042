"""The micro-batcher's device thread + executor hand-off, exercised on the CPU
(``cpu_batching``: same queue / device-thread / continuation-posting path as
a GPU unit, with the reference CPU kernels).  Concurrent REST and gRPC
clients must all get their own answers, and requests must share batches."""
import concurrent.futures as cf
import json
import urllib.request

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.client import SeldonClient
from seldon_core_amd.models import iris_logistic_regression


def _spec(graph):
    return {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}


@pytest.fixture(scope="module")
def served():
    clf = iris_logistic_regression()
    dep = sca.Deployment(_spec({"name": "clf", "type": "MODEL"}), components={"clf": clf}, device=-1,
                         batcher={"cpu_batching": True, "slots": 2, "max_wait_us": 100})
    h = dep.serve(http_port=0, grpc_port=0, threads=3, host="127.0.0.1")
    yield dep, h, clf
    dep.close()


def test_concurrent_rest_requests_share_batches(served):
    dep, h, clf = served
    rng = np.random.default_rng(0)
    rows = rng.uniform(0, 8, (64, 4))
    dep.batched["clf"].reset_stats()

    def call(i):
        x = rows[i % 64]
        req = urllib.request.Request(f"http://127.0.0.1:{h.http_port}/api/v0.1/predictions",
                                     data=json.dumps({"data": {"ndarray": [x.tolist()]}}).encode(),
                                     headers={"Content-Type": "application/json"})
        out = json.loads(urllib.request.urlopen(req, timeout=30).read())
        np.testing.assert_allclose(out["data"]["ndarray"], clf.predict_proba(x[None, :]), rtol=1e-12)
        return True

    with cf.ThreadPoolExecutor(32) as ex:
        assert all(ex.map(call, range(640)))
    st = dep.batched["clf"].stats()
    assert st["requests"] == 640 and st["batches"] < 640


def test_concurrent_grpc_requests(served):
    dep, h, clf = served
    sc = SeldonClient(gateway="ambassador", transport="grpc", gateway_endpoint=f"127.0.0.1:{h.grpc_port}",
                      deployment_name="d", namespace="n")
    rng = np.random.default_rng(1)

    def call(i):
        x = rng.uniform(0, 8, (1 + i % 3, 4))
        r = sc.predict(data=x)
        assert r.success, r.msg
        got = np.array(r.response.data.tensor.values).reshape(x.shape[0], 3)
        np.testing.assert_allclose(got, clf.predict_proba(x), rtol=1e-12)
        return True

    with cf.ThreadPoolExecutor(16) as ex:
        assert all(ex.map(call, range(200)))


def test_device_graph_through_batched_cpu_path():
    C = sca.native()
    rng = np.random.default_rng(2)
    comps = {"t": C.linear_model(rng.normal(size=(4, 4)), rng.normal(size=4), 0),
             "a": C.linear_model(rng.normal(size=(3, 4)), rng.normal(size=3), 1),
             "b": C.linear_model(rng.normal(size=(3, 4)), rng.normal(size=3), 1)}
    graph = {"name": "t", "type": "TRANSFORMER", "children": [
        {"name": "c", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
         "children": [{"name": "a", "type": "MODEL"}, {"name": "b", "type": "MODEL"}]}]}
    fused = sca.Deployment(_spec(graph), components=comps, device=-1, batcher={"cpu_batching": True})
    plain = sca.Deployment(_spec(graph), components=comps, device=-1, fuse=False)
    h = fused.serve(http_port=0, grpc_port=None, threads=2, host="127.0.0.1")
    try:
        X = rng.normal(size=(3, 4))

        def call(_):
            req = urllib.request.Request(f"http://127.0.0.1:{h.http_port}/api/v0.1/predictions",
                                         data=json.dumps({"data": {"ndarray": X.tolist()}}).encode(),
                                         headers={"Content-Type": "application/json"})
            return json.loads(urllib.request.urlopen(req, timeout=30).read())

        want = plain.predict({"data": {"ndarray": X.tolist()}})
        with cf.ThreadPoolExecutor(8) as ex:
            for out in ex.map(call, range(40)):
                np.testing.assert_allclose(out["data"]["ndarray"], want["data"]["ndarray"], rtol=1e-12)
                assert out["meta"]["requestPath"] == want["meta"]["requestPath"]
    finally:
        fused.close()
        plain.close()


def test_batch_device_time_histogram_exported(served):
    """Per-unit kernel-time histogram + batch-size quantiles on /prometheus."""
    dep, h, clf = served
    for _ in range(3):
        dep.predict({"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}})
    body = urllib.request.urlopen(f"http://127.0.0.1:{h.http_port}/prometheus", timeout=10).read().decode()
    assert "# TYPE seldon_gpu_batch_device_seconds histogram" in body
    assert 'seldon_gpu_batch_device_seconds_bucket{' in body and "seldon_gpu_batch_rows_p99" in body


def test_loadgen_storm_through_shards_handoff_and_parcels():
    """Closed-loop storm (native load generator, 128 users over 4 front-end
    threads) through the sharded submission queue, the hand-off thread and
    the recycled response parcels: no failed request, every request counted
    once, batches shared, and answers still correct afterwards."""
    import os
    import subprocess

    clf = iris_logistic_regression()
    dep = sca.Deployment(_spec({"name": "clf", "type": "MODEL"}), components={"clf": clf}, device=-1,
                         batcher={"cpu_batching": True, "slots": 3})
    h = dep.serve(http_port=0, grpc_port=0, threads=4, host="127.0.0.1")
    try:
        lg = os.path.join(os.path.dirname(sca.__file__), "bin", "sca_loadgen")
        body = json.dumps({"data": {"names": ["a", "b", "c", "d"], "ndarray": [[5.1, 3.5, 1.4, 0.2]]}})
        dep.batched["clf"].reset_stats()
        res = subprocess.run([lg, "--host", "127.0.0.1", "--port", str(h.http_port), "--users", "128", "--threads", "2",
                              "--steps", "2", "--warmup", "0", "--step-requests", "3000", "--mode", "rest",
                              "--path", "/api/v0.1/predictions", "--body", body],
                             capture_output=True, text=True, timeout=240)
        out = json.loads(res.stdout.strip().splitlines()[-1])
        assert out["errors"] == 0 and out["ok"] == 6000, out
        st = dep.batched["clf"].stats()
        assert st["requests"] == 6000 and st["rows"] == 6000, st
        assert st["batches"] < st["requests"]  # concurrent requests shared batches
        X = np.random.default_rng(7).uniform(0, 8, (5, 4))
        got = dep.predict({"data": {"ndarray": X.tolist()}})
        np.testing.assert_allclose(np.array(got["data"]["ndarray"]), clf.predict_proba(X), rtol=1e-12)
    finally:
        h.stop()
        dep.close()


def test_python_api_nested_predictions():
    """A Python node that synchronously calls ANOTHER deployment's predict,
    from 8 concurrent Python-API callers; both models are CPU-batched units
    whose completions are posted to the shared continuation pool
    (csrc/core/pool_executor.h).  Every answer matches sklearn."""
    import threading

    import numpy as np

    import seldon_core_amd as sca
    from seldon_core_amd.models import iris_logistic_regression
    from seldon_core_amd.servers import SKLearnServer

    clf = iris_logistic_regression()
    inner = sca.Deployment({"name": "inner", "graph": {"name": "m", "type": "MODEL"}},
                           components={"m": SKLearnServer(model=clf)}, device=-1,
                           batcher={"cpu_batching": True, "slots": 2})

    def pad(P):  # 3 class probabilities -> 4 iris-scale features
        P = np.asarray(P, dtype=np.float64)
        return np.hstack([P * 5.0, np.ones((P.shape[0], 1))])

    class Post:
        def transform_output(self, X, names):
            r = inner.predict({"data": {"ndarray": pad(X).tolist()}})
            return np.asarray(r["data"]["ndarray"])

    outer = sca.Deployment({"name": "outer", "graph": {"name": "post", "type": "OUTPUT_TRANSFORMER", "children": [
        {"name": "m", "type": "MODEL"}]}}, components={"m": SKLearnServer(model=clf), "post": Post()}, device=-1,
        batcher={"cpu_batching": True, "slots": 4, "max_batch": 2})  # one request per batch: parallel continuations
    try:
        errs, done = [], []

        def call(t):
            try:
                for i in range(10):
                    X = np.random.default_rng(t * 100 + i).normal(loc=4.0, size=(2, 4))
                    out = outer.predict({"data": {"ndarray": X.tolist()}})
                    want = clf.predict_proba(pad(clf.predict_proba(X)))
                    np.testing.assert_allclose(np.asarray(out["data"]["ndarray"]), want, rtol=0, atol=1e-12)
                done.append(t)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=call, args=(t,), daemon=True) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert not any(t.is_alive() for t in th), "nested Python-API predictions deadlocked"
        assert errs == [] and len(done) == 8, errs[:3]
    finally:
        outer.close()
        inner.close()
