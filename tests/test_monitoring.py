"""Dashboards / alert rules vs the live /prometheus endpoint (SURVEY P3;
reference helm-charts/seldon-core-analytics/files/grafana/configs/*.json).

Every metric series a generated dashboard or rule queries must be emitted by a
running engine: a deployment with an outlier detector in front of a
micro-batched classifier is driven with predictions + labelled feedback and
scraped."""
import json
import os
import re
import urllib.request

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components import outlier as od
from seldon_core_amd.monitoring import dashboards as db

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SERIES = re.compile(r"([a-zA-Z_:][a-zA-Z0-9_:]*)\s*[{\[]")


def _queried(obj):
    out = set()
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k in ("expr", "query") and isinstance(v, str):
                v = re.sub(r"label_values\(([a-zA-Z0-9_:]+)", r"\1{", v)
                out |= {m for m in _SERIES.findall(v) if m not in ("by", "ignoring", "on", "without")}
            else:
                out |= _queried(v)
    elif isinstance(obj, list):
        for v in obj:
            out |= _queried(v)
    return out


@pytest.fixture(scope="module")
def scrape():
    spec = json.load(open(os.path.join(ROOT, "examples", "outlier_transformer.json")))
    dep = sca.Deployment(spec, device=-1, batcher={"cpu_batching": True})
    h = dep.serve(http_port=0, grpc_port=None, threads=2, host="127.0.0.1")
    base = f"http://127.0.0.1:{h.http_port}"

    def post(path, body):
        r = urllib.request.Request(base + path, data=json.dumps(body).encode(),
                                   headers={"Content-Type": "application/json"})
        return json.loads(urllib.request.urlopen(r, timeout=30).read())

    try:
        rng = np.random.default_rng(0)
        for i in range(6):
            x = rng.normal(size=(1, 4)).tolist()
            out = post("/api/v0.1/predictions", {"data": {"ndarray": x}})
            post("/api/v0.1/feedback", {"request": {"data": {"ndarray": x}}, "response": out, "reward": float(i % 2),
                                        "truth": {"data": {"ndarray": [[i % 2]]}}})
        txt = urllib.request.urlopen(base + "/prometheus", timeout=10).read().decode()
    finally:
        dep.close()
    return {ln.split("{")[0].split(" ")[0] for ln in txt.splitlines() if ln and not ln.startswith("#")}


def test_prediction_gpu_and_mab_dashboards_query_emitted_series(scrape):
    for name in ("prediction-analytics", "gpu-serving", "multi-armed-bandit", "outlier-detection-md"):
        q = _queried(db.all_dashboards()[name])
        assert q, name
        missing = q - scrape
        assert not missing, f"{name} queries series the engine does not emit: {missing}"


def test_outlier_dashboards_match_detector_score_keys():
    for name, cls in (("outlier-detection-md", od.OutlierMahalanobis), ("outlier-detection-vae", od.OutlierVAE),
                      ("outlier-detection-if", od.OutlierIsolationForest)):
        q = _queried(db.all_dashboards()[name])
        assert cls.score_key in q
        assert set(db.OUTLIER_GAUGES) <= q


def test_rules_reference_emitted_series(scrape):
    rules = db.prometheus_rules()
    exprs = re.findall(r'expr: (".*")', rules)
    assert len(exprs) == 4
    q = _queried({"expr": " ".join(json.loads(e) for e in exprs)})
    assert q and not (q - scrape), q - scrape


def test_committed_assets_are_current(tmp_path):
    """monitoring/ in the repo is the generator's output (regenerate with
    python -m seldon_core_amd.monitoring.dashboards --out monitoring)."""
    db.write(str(tmp_path), ["127.0.0.1:8000"])
    for sub in ("grafana", "prometheus"):
        for f in os.listdir(tmp_path / sub):
            assert open(os.path.join(ROOT, "monitoring", sub, f)).read() == open(tmp_path / sub / f).read(), f
