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
