"""Kubernetes manifest rendering (reference
operator/controllers/seldondeployment_controller.go, seldondeployment_engine.go,
ambassador.go + ambassador_test.go, seldondeployment_explainers.go)."""
import base64
import json
import os

import yaml

from seldon_core_amd import k8s

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _by_kind(objs, kind):
    return [o for o in objs if o["kind"] == kind]


def _sdep(predictors, annotations=None, name="mymodel"):
    return {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": name}, "spec": {"name": name, "annotations": annotations or {},
                                                 "predictors": predictors}}


def _pred(name="p", traffic=None, graph=None, **kw):
    p = {"name": name, "graph": graph or {"name": "clf", "type": "MODEL", "implementation": "SIMPLE_MODEL"},
         "componentSpecs": [{"spec": {"containers": []}}]}
    if traffic is not None:
        p["traffic"] = traffic
    p.update(kw)
    return p


def test_engine_deployment_and_service():
    objs = k8s.render(_sdep([_pred()]))
    dep, = _by_kind(objs, "Deployment")
    svc, = _by_kind(objs, "Service")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["name"] == "seldon-container-engine"
    env = {e["name"]: e["value"] for e in c["env"]}
    pred = json.loads(base64.b64decode(env["ENGINE_PREDICTOR"]))
    assert pred["traffic"] == 0 and pred["graph"]["name"] == "clf"
    assert env["DEPLOYMENT_NAME"] == "mymodel" and env["ENGINE_SERVER_PORT"] == "8000"
    assert c["readinessProbe"]["httpGet"]["path"] == "/ready" and c["livenessProbe"]["httpGet"]["port"] == "admin"
    assert "/pause" in c["lifecycle"]["preStop"]["exec"]["command"][-1]
    assert c["resources"]["limits"]["amd.com/gpu"] == "1"
    assert dep["spec"]["template"]["spec"]["terminationGracePeriodSeconds"] == 20
    assert dep["spec"]["strategy"]["rollingUpdate"]["maxUnavailable"] == "10%"
    assert dep["spec"]["template"]["metadata"]["annotations"]["prometheus.io/path"] == "/prometheus"
    assert {p["name"]: p["port"] for p in svc["spec"]["ports"]} == {"http": 8000, "grpc": 5001}
    assert svc["spec"]["selector"] == {"seldon-app": dep["metadata"]["labels"]["seldon-app"]}
    for o in objs:
        assert len(o["metadata"]["name"]) <= 63


def test_ambassador_mappings_like_reference():
    """ambassador_test.go: two configs (REST + gRPC), namespaced prefix,
    no headers, ambassador_id when annotated."""
    objs = k8s.render(_sdep([_pred()], {"seldon.io/ambassador-id": "myinstance_id"}))
    svc, = _by_kind(objs, "Service")
    docs = [d for d in yaml.safe_load_all(svc["metadata"]["annotations"]["getambassador.io/config"]) if d]
    assert len(docs) == 2
    rest, grpc = docs
    assert rest["prefix"] == "/seldon/default/mymodel/" and "headers" not in rest and rest["weight"] == 100
    assert grpc["grpc"] is True and grpc["headers"] == {"seldon": "mymodel", "namespace": "default"}
    assert rest["ambassador_id"] == grpc["ambassador_id"] == "myinstance_id"
    # canary weights, shadow, header routing
    objs = k8s.render(_sdep([_pred("a", 75), _pred("b", 25, annotations={"seldon.io/ambassador-header": "x:y"}),
                             _pred("s", shadow=True)]), namespace="ns1")
    maps = {}
    for s in _by_kind(objs, "Service"):
        for d in yaml.safe_load_all(s["metadata"]["annotations"]["getambassador.io/config"]):
            if d and not d.get("grpc"):
                maps[d["name"]] = d
    assert maps["seldon_ns1_mymodel_a_rest_mapping"]["weight"] == 75
    assert maps["seldon_ns1_mymodel_b_rest_mapping"]["headers"] == {"x": "y"}
    assert maps["seldon_ns1_mymodel_s_rest_mapping"]["shadow"] is True


def test_external_container_node_gets_deployment_service_and_hpa():
    graph = {"name": "step", "type": "TRANSFORMER", "endpoint": {"type": "GRPC", "service_port": 9500},
             "children": [{"name": "clf", "type": "MODEL", "implementation": "SKLEARN_SERVER",
                           "modelUri": "gs://b/m"}]}
    cs = [{"spec": {"containers": [{"name": "step", "image": "me/step:1.0"}]},
           "hpaSpec": {"minReplicas": 1, "maxReplicas": 4,
                       "metrics": [{"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 50}}]}}]
    objs = k8s.render(_sdep([_pred(graph=graph, componentSpecs=cs)]))
    deps = {d["spec"]["template"]["spec"]["containers"][0]["name"]: d for d in _by_kind(objs, "Deployment")}
    assert set(deps) == {"seldon-container-engine", "step"}
    c = deps["step"]["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["PREDICTIVE_UNIT_SERVICE_PORT"] == "9500" and env["PREDICTIVE_UNIT_ID"] == "step"
    assert c["readinessProbe"]["tcpSocket"]["port"] == 9500
    svcs = {s["metadata"]["name"]: s for s in _by_kind(objs, "Service")}
    step_svc = [s for n, s in svcs.items() if "step" in n][0]
    assert step_svc["spec"]["ports"][0] == {"protocol": "TCP", "port": 9500, "targetPort": 9500, "name": "grpc"}
    hpa, = _by_kind(objs, "HorizontalPodAutoscaler")
    assert hpa["spec"]["maxReplicas"] == 4 and hpa["spec"]["scaleTargetRef"]["name"] == deps["step"]["metadata"]["name"]


def test_gpu_requests_follow_graph_placement():
    g = {"name": "c", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
        {"name": "a", "type": "MODEL", "implementation": "SIMPLE_MODEL", "device": 3},
        {"name": "b", "type": "MODEL", "implementation": "SIMPLE_MODEL", "devices": [0, 5]}]}
    dep = _by_kind(k8s.render(_sdep([_pred(graph=g)])), "Deployment")[0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == "6" and c["command"][-1] == "1"
    dep = _by_kind(k8s.render(_sdep([_pred(annotations={"seldon.io/gpus-per-pod": "8"})])), "Deployment")[0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == "8" and c["command"][-1] == "8"


def test_explainer_deployment():
    p = _pred(explainer={"type": "anchor_tabular", "modelUri": "s3://b/explainer",
                         "config": {"threshold": "0.9", "feature_names": "a,b"}})
    objs = k8s.render(_sdep([p]), namespace="seldon")
    x = [d for d in _by_kind(objs, "Deployment") if d["metadata"]["name"].endswith("-explainer")][0]
    c = x["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][-1] == "seldon_core_amd.explainers.server"
    a = c["args"]
    assert a[a.index("--predictor_host") + 1].endswith(".seldon:8000") and "anchor_tabular" in a
    assert "--threshold=0.9" in a and "--storage_uri" in a
    xs = [s for s in _by_kind(objs, "Service") if s["metadata"]["name"] == x["metadata"]["name"]][0]
    rest = next(yaml.safe_load_all(xs["metadata"]["annotations"]["getambassador.io/config"]))
    assert rest["prefix"] == "/seldon/seldon/mymodel-explainer/"


def test_examples_render_and_cli(capsys):
    for f in sorted(os.listdir(os.path.join(ROOT, "examples"))):
        if f.endswith(".json"):
            objs = k8s.render(os.path.join(ROOT, "examples", f))
            assert _by_kind(objs, "Deployment") and _by_kind(objs, "Service")
    assert k8s.main([os.path.join(ROOT, "examples", "abtest.json"), "--namespace", "x"]) == 0
    docs = [d for d in yaml.safe_load_all(capsys.readouterr().out) if d]
    assert all(d["metadata"]["namespace"] == "x" for d in docs)


def test_istio_virtual_services_split_traffic(monkeypatch):
    """createIstioResources (seldondeployment_controller.go:111-225): one REST
    and one gRPC VirtualService, a weighted route per predictor, one
    ISTIO_MUTUAL DestinationRule per predictor Service selecting its version."""
    sd = _sdep([_pred("a", 75, labels={"version": "v1"}), _pred("b", 25, labels={"version": "v2"})])
    assert not _by_kind(k8s.render(sd), "VirtualService")  # ISTIO_ENABLED unset
    monkeypatch.setenv("ISTIO_ENABLED", "true")
    objs = k8s.render(sd, namespace="ns1")
    vs = {v["metadata"]["name"]: v["spec"] for v in _by_kind(objs, "VirtualService")}
    assert set(vs) == {"mymodel-mymodel-http", "mymodel-mymodel-grpc"}  # seldonId + suffix
    http, grpc = vs["mymodel-mymodel-http"], vs["mymodel-mymodel-grpc"]
    assert http["gateways"] == ["seldon-gateway"] and http["hosts"] == ["*"]
    assert http["http"][0]["match"][0]["uri"]["prefix"] == "/seldon/ns1/mymodel/"
    assert http["http"][0]["rewrite"] == {"uri": "/"}
    assert grpc["http"][0]["match"][0]["headers"] == {"seldon": {"exact": "mymodel"}, "namespace": {"exact": "ns1"}}
    svcs = {s["metadata"]["name"] for s in _by_kind(objs, "Service")}
    for rt, port in ((http, 8000), (grpc, 5001)):
        r = rt["http"][0]["route"]
        assert [(d["destination"]["subset"], d["weight"]) for d in r] == [("a", 75), ("b", 25)]
        assert all(d["destination"]["port"]["number"] == port and d["destination"]["host"] in svcs for d in r)
    drs = _by_kind(objs, "DestinationRule")
    assert sorted(d["spec"]["subsets"][0]["labels"]["version"] for d in drs) == ["v1", "v2"]
    assert all(d["spec"]["trafficPolicy"]["tls"]["mode"] == "ISTIO_MUTUAL" for d in drs)
    # the subset's version label is what the engine pods carry
    deps = {d["metadata"]["name"]: d for d in _by_kind(objs, "Deployment")}
    versions = {d["spec"]["template"]["metadata"]["labels"].get("version") for d in deps.values()}
    assert {"v1", "v2"} <= versions


def test_istio_gateway_annotation_and_explainer(monkeypatch):
    monkeypatch.setenv("ISTIO_ENABLED", "true")
    monkeypatch.setenv("ISTIO_GATEWAY", "envgw")
    p = _pred(explainer={"type": "anchor_tabular"})
    objs = k8s.render(_sdep([p]), namespace="s")
    vs = {v["metadata"]["name"]: v["spec"] for v in _by_kind(objs, "VirtualService")}
    assert vs["mymodel-mymodel-http"]["gateways"] == ["envgw"]
    assert vs["mymodel-mymodel-http"]["http"][0]["route"][0]["weight"] == 100  # single predictor
    xhttp = [v for n, v in vs.items() if "explainer" in n and n.endswith("-http")][0]
    assert xhttp["http"][0]["match"][0]["uri"]["prefix"] == "/seldon/s/mymodel/p/explainer/"
    xdr = [d for d in _by_kind(objs, "DestinationRule") if "explainer" in d["metadata"]["name"]][0]
    assert "trafficPolicy" not in xdr["spec"]
    objs = k8s.render(_sdep([_pred()], {"seldon.io/istio-gateway": "ns/gw"}), istio=True)
    assert _by_kind(objs, "VirtualService")[0]["spec"]["gateways"] == ["ns/gw"]
