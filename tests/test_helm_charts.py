"""Helm charts (reference helm-charts/seldon-single-model,
seldon-abtest, seldon-mab, seldon-od-model, seldon-core-operator,
seldon-core-loadtesting) rendered with tools/helm_lite.py: every
SeldonDeployment they produce passes the schema + webhook validation, renders
to cluster objects, and -- for the in-process graphs -- serves predictions on
the CPU path."""
import os
import sys

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd import k8s
from seldon_core_amd.serving.spec import apply_defaults, validate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import helm_lite  # noqa: E402

CHARTS = os.path.join(ROOT, "helm-charts")


def _render(chart, **kw):
    return helm_lite.render_chart(os.path.join(CHARTS, chart), "rel", "seldon", **kw)


@pytest.mark.parametrize("chart", ["seldon-single-model", "seldon-abtest", "seldon-mab", "seldon-od-model"])
def test_serving_charts_valid(chart):
    sdep, = _render(chart)
    assert sdep["kind"] == "SeldonDeployment" and sdep["metadata"]["name"] == "rel"
    assert validate(apply_defaults(sdep)) == []
    kinds = {o["kind"] for o in k8s.render(sdep)}
    assert {"Deployment", "Service"} <= kinds


@pytest.mark.parametrize("chart", ["seldon-abtest", "seldon-mab", "seldon-od-model"])
def test_in_process_charts_serve(chart):
    sdep, = _render(chart)
    dep = sca.Deployment(sdep, device=-1)
    try:
        X = np.random.default_rng(0).uniform(size=(3, 4))
        out = dep.predict({"data": {"ndarray": X.tolist()}})
        assert "data" in out, out
    finally:
        dep.close()


def test_single_model_external_image_and_env():
    sdep, = _render("seldon-single-model", sets=["model.image=me/model:1", "model.env.LOG_LEVEL=DEBUG",
                                                  "gpusPerPod=4"])
    c, = sdep["spec"]["predictors"][0]["componentSpecs"][0]["spec"]["containers"]
    assert c["image"] == "me/model:1" and c["env"] == [{"name": "LOG_LEVEL", "value": "DEBUG"}]
    assert "implementation" not in sdep["spec"]["predictors"][0]["graph"]
    assert validate(apply_defaults(sdep)) == []
    eng = [o for o in k8s.render(sdep) if o["kind"] == "Deployment" and "engine" in str(o)][0]
    limits = eng["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert limits["amd.com/gpu"] == "4"


def test_mab_thompson_drops_epsilon():
    sdep, = _render("seldon-mab", sets=["mab.implementation=THOMPSON_SAMPLING"])
    names = [p["name"] for p in sdep["spec"]["predictors"][0]["graph"]["parameters"]]
    assert names == ["n_branches", "verbose"]


def test_operator_chart():
    docs = _render("seldon-core-amd-operator")
    kinds = [d["kind"] for d in docs]
    for k in ("CustomResourceDefinition", "ServiceAccount", "ClusterRole", "ClusterRoleBinding", "Deployment",
              "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration", "Service"):
        assert k in kinds, k
    from seldon_core_amd import operator as op

    hooks = [d for d in docs if d["kind"].endswith("WebhookConfiguration")]
    assert {h["webhooks"][0]["clientConfig"]["service"]["path"] for h in hooks} == set(op.WEBHOOK_PATHS)
    mgr = next(d for d in docs if d["kind"] == "Deployment")
    c = mgr["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["python", "-m", "seldon_core_amd.operator"]
    role = next(d for d in docs if d["kind"] == "ClusterRole")
    granted = {r for rule in role["rules"] for r in rule["resources"]}
    assert {op.KINDS[k][1] for k in op.KINDS} <= granted
    off = _render("seldon-core-amd-operator", sets=["webhook.enabled=false", "crd.create=false"])
    assert not any(d["kind"].endswith("WebhookConfiguration") or d["kind"] == "CustomResourceDefinition"
                   for d in off)


def test_loadtesting_chart_args_parse():
    job, = _render("seldon-core-amd-loadtesting", sets=["feedback=true"])
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][-1] == "seldon_core_amd.loadtester" and "--feedback" in c["args"]


@pytest.mark.parametrize("od", ["mahalanobis", "isolationforest", "vae", "seq2seq"])
def test_od_transformer_chart_valid(od):
    sdep, = _render("seldon-od-transformer", sets=[f"outlierDetection.type={od}"])
    g = sdep["spec"]["predictors"][0]["graph"]
    assert g["type"] == "TRANSFORMER" and g["name"] == "outlier-detector"
    assert g["implementation"].endswith("_OD") and g["children"][0]["name"] == "classifier"
    assert validate(apply_defaults(sdep)) == []
    off, = _render("seldon-od-transformer", sets=["outlierDetection.enabled=false"])
    assert off["spec"]["predictors"][0]["graph"]["name"] == "classifier"


def test_od_transformer_chart_serves():
    """Mahalanobis detector in front of the iris classifier, in-process: the
    request is scored and tagged by the detector, then classified."""
    from seldon_core_amd.models import iris_logistic_regression

    sdep, = _render("seldon-od-transformer")
    lr = iris_logistic_regression()
    dep = sca.Deployment(sdep, components={"classifier": lr}, device=-1)
    try:
        X = np.random.default_rng(0).normal(loc=4.0, size=(3, 4))
        out = dep.predict({"data": {"ndarray": X.tolist()}})
        np.testing.assert_allclose(np.asarray(out["data"]["ndarray"]), lr.predict_proba(X), rtol=1e-12)
        assert out["meta"]["requestPath"].keys() >= {"outlier-detector", "classifier"}
    finally:
        dep.close()


def test_openvino_chart():
    sdep, = _render("seldon-openvino")
    pred = sdep["spec"]["predictors"][0]
    g = pred["graph"]
    assert g["implementation"] == "TENSORFLOW_SERVER"
    params = {p["name"]: p["value"] for p in g["parameters"]}
    assert params["rest_endpoint"] == "http://localhost:8001" and params["model_name"] == "squeezenet1.1"
    c, = pred["componentSpecs"][0]["spec"]["containers"]
    assert c["image"].startswith("intelaipg/openvino-model-server") and c["ports"][0]["containerPort"] == 8001
    assert validate(apply_defaults(sdep)) == []


def test_kafka_chart():
    docs = _render("seldon-core-kafka")
    kinds = sorted(d["kind"] for d in docs)
    assert kinds == ["Deployment", "Service", "Service", "StatefulSet"]
    sts = next(d for d in docs if d["kind"] == "StatefulSet")
    env = {e["name"]: e["value"] for e in sts["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["KAFKA_PROCESS_ROLES"] == "broker,controller"
    assert env["KAFKA_ADVERTISED_LISTENERS"] == "PLAINTEXT://rel-kafka.seldon.svc.cluster.local:9092"
    logger = next(d for d in docs if d["kind"] == "Deployment")
    args = logger["spec"]["template"]["spec"]["containers"][0]["args"]
    assert args[args.index("--kafka") + 1] == "rel-kafka.seldon.svc.cluster.local:9092"
    from seldon_core_amd import request_logger

    request_logger.main.__code__  # the module the container runs exists
    persistent = _render("seldon-core-kafka", sets=["kafka.persistence=true", "requestLogger.enabled=false"])
    assert [d["kind"] for d in persistent] == ["Service", "StatefulSet"]
    assert "volumeClaimTemplates" in persistent[1]["spec"]


def test_analytics_chart_ships_the_monitoring_dashboards():
    import json

    import yaml

    docs = _render("seldon-core-analytics")
    kinds = {d["kind"] for d in docs}
    assert {"ConfigMap", "Deployment", "Service", "Secret", "ClusterRole", "ServiceAccount"} <= kinds
    dash = next(d for d in docs if d["metadata"]["name"] == "rel-grafana-dashboards")
    mon = os.path.join(ROOT, "monitoring", "grafana")
    assert set(dash["data"]) == set(os.listdir(mon))
    for name, text in dash["data"].items():
        with open(os.path.join(mon, name)) as f:
            assert json.loads(text) == json.load(f), name  # chart copies == monitoring/ sources
    prom = next(d for d in docs if d["metadata"]["name"] == "rel-prometheus-config")
    cfg = yaml.safe_load(prom["data"]["prometheus.yml"])
    assert cfg["scrape_configs"][0]["kubernetes_sd_configs"] == [{"role": "pod"}]
    with open(os.path.join(ROOT, "monitoring", "prometheus", "rules.yml")) as f:
        assert yaml.safe_load(prom["data"]["rules.yml"]) == yaml.safe_load(f)
