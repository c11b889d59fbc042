"""Traffic splitting across predictors and shadow mirroring (SURVEY X4;
reference: PredictorSpec.traffic + Istio/Ambassador weights,
operator/controllers/seldondeployment_controller.go:180-215, ambassador.go:88,119-122;
webhook rule seldondeployment_webhook.go:372-386)."""
import threading

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.serving.spec import SpecError


class Const:
    def __init__(self, v):
        self.v = v
        self.calls = 0
        self.fb = 0
        self.lock = threading.Lock()

    def predict(self, X, names):
        with self.lock:
            self.calls += 1
        return np.full((len(X), 1), self.v)

    def send_feedback(self, X, names, reward, truth, routing=None):
        with self.lock:
            self.fb += 1


def _sdep(preds):
    return {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": "ab"}, "spec": {"name": "ab", "predictors": preds}}


def _pred(name, traffic, node, **extra):
    p = {"name": name, "traffic": traffic, "componentSpecs": [{"spec": {"containers": [{"name": node, "image": f"img/{node}:1"}]}}],
         "graph": {"name": node, "type": "MODEL", "children": []}}
    p.update(extra)
    return p


def test_weighted_split_and_shadow():
    a, b, s = Const(1.0), Const(2.0), Const(3.0)
    spec = _sdep([_pred("main", 70, "ma"), _pred("canary", 30, "mb"), _pred("mirror", 0, "ms", shadow=True)])
    dep = sca.Deployment(spec, components={"ma": a, "mb": b, "ms": s}, device=-1)
    try:
        assert set(dep.peers) == {"canary", "mirror"}
        seen = {1.0: 0, 2.0: 0}
        n = 2000
        for _ in range(n):
            out = dep.predict({"data": {"ndarray": [[0.0]]}})
            seen[out["data"]["ndarray"][0][0]] += 1
        assert 0.65 * n < seen[1.0] < 0.75 * n
        assert seen[1.0] + seen[2.0] == n
        # the shadow saw every request; its answers were discarded
        import time
        for _ in range(100):
            if s.calls == n:
                break
            time.sleep(0.01)
        assert s.calls == n
        # one /prometheus for all predictors, labelled by predictor
        text = dep.metrics()
        assert 'predictor_name="canary"' in text and 'predictor_name="main"' in text
        assert text.count("# TYPE seldon_api_engine_client_requests_seconds ") <= 1
    finally:
        dep.close()


def test_feedback_goes_to_serving_predictor():
    a, b = Const(1.0), Const(2.0)
    spec = _sdep([_pred("main", 50, "ma"), _pred("canary", 50, "mb")])
    dep = sca.Deployment(spec, components={"ma": a, "mb": b}, device=-1)
    try:
        for _ in range(40):
            req = {"data": {"ndarray": [[0.0]]}}
            out = dep.predict(req)
            before = (a.fb, b.fb)
            dep.feedback({"request": req, "response": out, "reward": 1.0})
            if out["data"]["ndarray"][0][0] == 1.0:
                assert (a.fb, b.fb) == (before[0] + 1, before[1])
            else:
                assert (a.fb, b.fb) == (before[0], before[1] + 1)
    finally:
        dep.close()


def test_predictor_scoped_components():
    spec = _sdep([_pred("main", 50, "m"), _pred("canary", 50, "m")])
    dep = sca.Deployment(spec, components={"main/m": Const(1.0), "canary/m": Const(2.0)}, device=-1)
    try:
        vals = {dep.predict({"data": {"ndarray": [[0.0]]}})["data"]["ndarray"][0][0] for _ in range(200)}
        assert vals == {1.0, 2.0}
    finally:
        dep.close()


def test_header_routing_python_and_http():
    import urllib.request

    a, b, c = Const(1.0), Const(2.0), Const(3.0)
    spec = _sdep([_pred("main", 100, "ma"),
                  _pred("london", 0, "mb", annotations={"seldon.io/header": "location:london"}),
                  _pred("beta", 0, "mc", annotations={"seldon.io/regex-header": "x-user:beta-.*"})])
    dep = sca.Deployment(spec, components={"ma": a, "mb": b, "mc": c}, device=-1)
    try:
        v = lambda out: out["data"]["ndarray"][0][0]  # noqa: E731
        req = {"data": {"ndarray": [[0.0]]}}
        assert {v(dep.predict(req)) for _ in range(50)} == {1.0}  # weights: main only
        assert v(dep.predict(req, headers={"Location": "london"})) == 2.0
        assert v(dep.predict(req, headers={"location": "paris"})) == 1.0
        assert v(dep.predict(req, headers={"X-User": "beta-42"})) == 3.0
        h = dep.serve(http_port=0, grpc_port=None, threads=1, host="127.0.0.1")
        r = urllib.request.Request(f"http://127.0.0.1:{h.http_port}/api/v0.1/predictions",
                                   data=b'{"data":{"ndarray":[[0.0]]}}',
                                   headers={"Content-Type": "application/json", "location": "london"})
        import json as _json

        assert _json.loads(urllib.request.urlopen(r, timeout=5).read())["data"]["ndarray"][0][0] == 2.0
    finally:
        dep.close()


def test_traffic_must_sum_to_100():
    spec = _sdep([_pred("main", 60, "ma"), _pred("canary", 30, "mb")])
    with pytest.raises(SpecError, match="Traffic must sum to 100"):
        sca.Deployment(spec, components={"ma": Const(1.0), "mb": Const(2.0)}, device=-1)


def test_single_predictor_selectable():
    spec = _sdep([_pred("main", 60, "ma"), _pred("canary", 40, "mb")])
    dep = sca.Deployment(spec, components={"ma": Const(1.0), "mb": Const(2.0)}, device=-1, predictor="canary")
    try:
        assert not dep.peers
        assert dep.predict({"data": {"ndarray": [[0.0]]}})["data"]["ndarray"][0][0] == 2.0
    finally:
        dep.close()
