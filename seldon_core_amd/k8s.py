"""Kubernetes manifests for a SeldonDeployment on MI355X nodes (SURVEY O4/O5,
P2; reference operator/controllers/seldondeployment_controller.go:253-636 --
createComponents / createContainerService / createDeploymentWithoutEngine --,
seldondeployment_engine.go:101-214 (engine container), ambassador.go:50-260
(Mapping annotations), seldondeployment_explainers.go:32-184 and, with
``ISTIO_ENABLED=true`` / ``--istio``, the Istio VirtualServices +
DestinationRules of seldondeployment_controller.go:111-225 and
seldondeployment_explainers.go:196-290).

    python -m seldon_core_amd.k8s sdep.json [--namespace ns] > manifests.yaml

The reference reconciler turns a SeldonDeployment into one Deployment per
componentSpec plus an injected Java engine container that calls every model
over HTTP/gRPC.  Here the engine *hosts* the GPU graph: every node with an
in-process implementation (built-ins, prepackaged servers, registered
components, fused device graphs) runs inside the engine pod, which requests
``amd.com/gpu`` for the devices its graph is placed on and serves REST +
gRPC + admin.  Only nodes whose implementation is an external container keep
the reference layout (a Deployment per componentSpec + a Service per
container, the engine reaching them through ``endpoint.service_host``).

Generated per predictor: engine Deployment (``ENGINE_PREDICTOR`` base64 with
traffic zeroed, probes ``/ready`` / ``/live`` on the admin port, preStop
``/pause``, downward-API annotations at ``/etc/podinfo``, Prometheus scrape
annotations, 10% maxUnavailable, 20 s grace), predictor Service with the
Ambassador REST + gRPC Mappings (weight, shadow, header / regex-header,
ambassador-id, custom config), component Deployments / Services, HPAs from
``hpaSpec``, explainer Deployment + Service; with Istio one ``-http`` and
one ``-grpc`` VirtualService per deployment whose routes split traffic over
the predictors (weight = ``traffic``, destination subset = predictor name on
the engine's REST / gRPC port) and an ISTIO_MUTUAL DestinationRule per
predictor Service selecting its ``version`` label; explainers get their own
unsplit pair under ``/seldon/<ns>/<name>/<predictor>/explainer/``.
"""
from __future__ import annotations

import argparse
import base64
import copy
import json
import os
import sys
from typing import Any, Dict, List, Optional

import yaml

from .serving import naming
from .serving.spec import BUILTIN_IMPLEMENTATIONS, PREPACKAGED_SERVERS, apply_defaults, is_shadow, iter_nodes, \
    load_spec, predictors

ENGINE_CONTAINER = "seldon-container-engine"
HTTP_PORT, GRPC_PORT, ADMIN_PORT = 8000, 5001, 8082
LABEL_APP, LABEL_ID = "seldon-app", "seldon-deployment-id"
PODINFO = ("podinfo", "/etc/podinfo")
AMBASSADOR_ANNOTATION = "getambassador.io/config"
AMBASSADOR_IDLE_TIMEOUT = 300000


def _engine_image() -> str:
    return os.environ.get("ENGINE_CONTAINER_IMAGE_AND_VERSION", "seldon-core-amd/engine:0.1.0")


def _annotations(sdep: Dict, predictor: Optional[Dict] = None) -> Dict[str, str]:
    a = dict((sdep.get("spec") or {}).get("annotations") or {})
    a.update((sdep.get("metadata") or {}).get("annotations") or {})
    if predictor is not None:
        a.update(predictor.get("annotations") or {})
    return a


def _external_nodes(predictor: Dict, bound: Optional[set] = None) -> List[str]:
    """Graph nodes served by their own container (not hosted in the engine)."""
    bound = bound or set()
    out = []
    for node, _ in iter_nodes(predictor["graph"]):
        impl = node.get("implementation", "UNKNOWN_IMPLEMENTATION")
        if impl in BUILTIN_IMPLEMENTATIONS or impl in PREPACKAGED_SERVERS or node["name"] in bound:
            continue
        if impl != "UNKNOWN_IMPLEMENTATION":  # registered in-process component implementation
            continue
        out.append(node["name"])
    return out


def gpus_for(predictor: Dict) -> int:
    """GPUs one engine pod needs: highest device ordinal the graph pins (+1),
    replica fan-out, or 1 when any node is GPU-resident by default."""
    need = 0
    for node, _ in iter_nodes(predictor["graph"]):
        if node.get("device") is not None and int(node["device"]) >= 0:
            need = max(need, int(node["device"]) + 1)
        devs = [int(d) for d in node.get("devices") or [] if int(d) >= 0]
        if devs:
            need = max(need, max(devs) + 1)
        elif int(node.get("replicas", 1) or 1) > 1:
            need = max(need, int(node["replicas"]))
    return max(1, need)


def _ambassador(sdep: Dict, predictor: Dict, svc: str, ns: str) -> str:
    ann = _annotations(sdep, predictor)
    if ann.get("seldon.io/ambassador-config"):
        return ann["seldon.io/ambassador-config"]
    name = sdep["metadata"]["name"]
    ext = ann.get("seldon.io/ambassador-service-name", name)
    weight = 100 if len(predictors(sdep)) <= 1 else int(predictor.get("traffic", 0) or 0)
    docs = []
    for grpc in (False, True):
        timeout = int(ann.get("seldon.io/grpc-read-timeout" if grpc else "seldon.io/rest-read-timeout", "3000"))
        m: Dict[str, Any] = {"apiVersion": "ambassador/v1", "kind": "Mapping",
                             "name": f"seldon_{ns}_{name}_{predictor['name']}_{'grpc' if grpc else 'rest'}_mapping",
                             "service": f"{svc}.{ns}:{GRPC_PORT if grpc else HTTP_PORT}", "timeout_ms": timeout,
                             "retry_policy": {"retry_on": "connect-failure", "num_retries": 3}, "weight": weight}
        if grpc:
            m.update({"grpc": True, "prefix": "/seldon.protos.Seldon/", "rewrite": "/seldon.protos.Seldon/",
                      "headers": {"seldon": ext, "namespace": ns}})
        else:
            m["prefix"] = f"/seldon/{ns}/{ext}/"
        if timeout > AMBASSADOR_IDLE_TIMEOUT:
            m["idle_timeout_ms"] = timeout
        for key, field in (("seldon.io/ambassador-header", "headers"), ("seldon.io/ambassador-regex-header",
                                                                        "regex_headers")):
            if ann.get(key):
                parts = [p.strip() for p in ann[key].split(":")]
                m.setdefault(field, {}).update(dict(zip(parts[0::2], parts[1::2])))
        if ann.get("seldon.io/ambassador-shadow") or is_shadow(predictor):
            m["shadow"] = True
        if ann.get("seldon.io/ambassador-id"):
            m["ambassador_id"] = ann["seldon.io/ambassador-id"]
        docs.append(yaml.safe_dump(m, sort_keys=True))
    return "".join("---\n" + d for d in docs)


def istio_enabled() -> bool:
    return os.environ.get("ISTIO_ENABLED", "false") == "true"


def _vs_name(name: str) -> str:
    return name[:63].rstrip("-")


def _istio(sdep: Dict, ns: str, seldon_id: str, targets: List[Dict], prefix: str, mtls: bool = True) -> List[Dict]:
    """VirtualServices (REST + gRPC) routing ``prefix`` / the Seldon gRPC
    service to ``targets`` (``{"host", "subset", "weight", "version"}``), and
    one DestinationRule per target host."""
    ann = _annotations(sdep)
    gateway = ann.get("seldon.io/istio-gateway", os.environ.get("ISTIO_GATEWAY", "seldon-gateway"))
    name = sdep["metadata"]["name"]
    base = targets[0]["vs"]

    def route(port: int) -> List[Dict]:
        return [{"destination": {"host": t["host"], "subset": t["subset"], "port": {"number": port}},
                 "weight": t["weight"]} for t in targets]

    http = {"match": [{"uri": {"prefix": prefix}}], "rewrite": {"uri": "/"}, "route": route(HTTP_PORT)}
    grpc = {"match": [{"uri": {"prefix": "/seldon.protos.Seldon/"},
                       "headers": {"seldon": {"exact": name}, "namespace": {"exact": ns}}}],
            "route": route(GRPC_PORT)}
    out = []
    for suffix, rt in (("http", http), ("grpc", grpc)):
        out.append({"apiVersion": "networking.istio.io/v1alpha3", "kind": "VirtualService",
                    "metadata": _meta(_vs_name(f"{base}-{suffix}"), ns, {LABEL_ID: seldon_id}),
                    "spec": {"hosts": ["*"], "gateways": [gateway], "http": [rt]}})
    for t in targets:
        spec = {"host": t["host"], "subsets": [{"name": t["subset"], "labels": {"version": t["version"]}}]}
        if mtls:
            spec["trafficPolicy"] = {"tls": {"mode": "ISTIO_MUTUAL"}}
        out.append({"apiVersion": "networking.istio.io/v1alpha3", "kind": "DestinationRule",
                    "metadata": _meta(t["host"], ns, {LABEL_ID: seldon_id}), "spec": spec})
    return out


def _meta(name: str, ns: str, labels: Dict[str, str], annotations: Optional[Dict[str, str]] = None) -> Dict:
    m = {"name": name, "namespace": ns, "labels": dict(labels)}
    if annotations:
        m["annotations"] = dict(annotations)
    return m


def _deployment(name: str, ns: str, labels: Dict[str, str], pod: Dict, replicas: int,
                pod_annotations: Optional[Dict[str, str]] = None) -> Dict:
    pod = copy.deepcopy(pod)
    pod.setdefault("terminationGracePeriodSeconds", 20)
    vols = pod.setdefault("volumes", [])
    if not any(v.get("name") == PODINFO[0] for v in vols):
        vols.append({"name": PODINFO[0], "downwardAPI": {"items": [
            {"path": "annotations", "fieldRef": {"fieldPath": "metadata.annotations"}}]}})
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": _meta(name, ns, labels),
            "spec": {"replicas": replicas, "selector": {"matchLabels": {LABEL_APP: labels[LABEL_APP]}},
                     "strategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "10%"}},
                     "template": {"metadata": {"labels": dict(labels), "annotations": dict(pod_annotations or {})},
                                  "spec": pod}}}


def _service(name: str, ns: str, labels: Dict[str, str], selector: str, ports: List[Dict],
             annotations: Optional[Dict[str, str]] = None, headless: bool = False) -> Dict:
    spec: Dict[str, Any] = {"selector": {LABEL_APP: selector}, "ports": ports, "type": "ClusterIP",
                            "sessionAffinity": "None"}
    if headless:
        spec["clusterIP"] = "None"
    return {"apiVersion": "v1", "kind": "Service", "metadata": _meta(name, ns, labels, annotations), "spec": spec}


def _engine_container(sdep: Dict, predictor: Dict, ns: str, n_gpus: int, workers: int) -> Dict:
    p = copy.deepcopy(predictor)
    p["traffic"] = 0  # no diff in the generated Deployment when only traffic changes
    p.pop("explainer", None)
    b64 = base64.b64encode(json.dumps(p, sort_keys=True).encode()).decode()
    env = [{"name": "ENGINE_PREDICTOR", "value": b64},
           {"name": "DEPLOYMENT_NAME", "value": sdep["spec"].get("name", "")},
           {"name": "DEPLOYMENT_NAMESPACE", "value": ns},
           {"name": "ENGINE_SERVER_PORT", "value": str(HTTP_PORT)},
           {"name": "ENGINE_SERVER_GRPC_PORT", "value": str(GRPC_PORT)},
           {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]
    orch = predictor.get("svcOrchSpec") or {}
    have = {e["name"] for e in env}
    for e in orch.get("env") or []:
        env = [x for x in env if x["name"] != e["name"]] + [e]
        have.add(e["name"])
    for k, v in sorted(_annotations(sdep, predictor).items()):  # seldon.io/engine-* -> env (controller_utils.go:49-69)
        if k.startswith("seldon.io/engine-"):
            name = k[len("seldon.io/engine-"):].upper().replace("-", "_")
            if name not in have:
                env.append({"name": name, "value": str(v)})
                have.add(name)
    resources = copy.deepcopy(orch.get("resources") or predictor.get("engineResources") or {})
    resources.setdefault("requests", {}).setdefault("cpu", "4")
    resources.setdefault("limits", {})["amd.com/gpu"] = str(n_gpus)
    resources["requests"]["amd.com/gpu"] = str(n_gpus)
    probe = lambda path: {"httpGet": {"port": "admin", "path": path, "scheme": "HTTP"},  # noqa: E731
                          "initialDelaySeconds": 20, "periodSeconds": 5, "failureThreshold": 3,
                          "successThreshold": 1, "timeoutSeconds": 60}
    return {"name": ENGINE_CONTAINER, "image": _engine_image(),
            "imagePullPolicy": os.environ.get("ENGINE_CONTAINER_IMAGE_PULL_POLICY", "IfNotPresent"),
            "command": ["python", "-m", "seldon_core_amd.serve", "--gpus", str(workers)],
            "env": env, "resources": resources,
            "ports": [{"containerPort": HTTP_PORT, "name": "http", "protocol": "TCP"},
                      {"containerPort": GRPC_PORT, "name": "grpc", "protocol": "TCP"},
                      {"containerPort": ADMIN_PORT, "name": "admin", "protocol": "TCP"}],
            "readinessProbe": probe("/ready"), "livenessProbe": probe("/live"),
            "lifecycle": {"preStop": {"exec": {"command": [
                "/bin/sh", "-c", f"curl 127.0.0.1:{HTTP_PORT}/pause; /bin/sleep 10"]}}},
            "volumeMounts": [{"name": PODINFO[0], "mountPath": PODINFO[1]}],
            "terminationMessagePath": "/dev/termination-log", "terminationMessagePolicy": "File"}


def _unit_env(sdep: Dict, predictor: Dict, node: Dict, port: int) -> List[Dict]:
    return [{"name": "PREDICTIVE_UNIT_SERVICE_PORT", "value": str(port)},
            {"name": "PREDICTIVE_UNIT_PARAMETERS", "value": json.dumps(node.get("parameters") or [])},
            {"name": "PREDICTIVE_UNIT_ID", "value": node["name"]},
            {"name": "PREDICTOR_ID", "value": predictor["name"]},
            {"name": "SELDON_DEPLOYMENT_ID", "value": sdep["metadata"]["name"]}]


def render(sdep_in: Any, namespace: Optional[str] = None, bound: Optional[set] = None,
           istio: Optional[bool] = None) -> List[Dict]:
    """All objects for a SeldonDeployment (dict / JSON / YAML path).
    ``istio`` defaults to the operator's ``ISTIO_ENABLED`` environment flag."""
    sdep = apply_defaults(copy.deepcopy(load_spec(sdep_in)))
    ns = namespace or (sdep.get("metadata") or {}).get("namespace") or "default"
    seldon_id = naming.sdep_name(sdep)
    istio = istio_enabled() if istio is None else istio
    out: List[Dict] = []
    routes: List[Dict] = []
    n_pred = len(predictors(sdep))
    for p in predictors(sdep):
        ann = _annotations(sdep, p)
        version = (p.get("labels") or {}).get("version", p["name"])
        ext = _external_nodes(p, bound)
        # ---- engine pod (hosts every in-process node of the graph)
        eng_name = naming.service_orchestrator_name(sdep, p)
        # One engine process owning every GPU its graph is placed on; or, with
        # seldon.io/gpus-per-pod on a single-device graph, that many
        # data-parallel worker processes (one per GPU) sharing the pod's ports.
        n_gpus, workers = gpus_for(p), 1
        per_pod = int(ann.get("seldon.io/gpus-per-pod", "0") or 0)
        if per_pod > 1 and n_gpus == 1:
            n_gpus = workers = per_pod
        labels = {LABEL_APP: naming.predictor_key(sdep, p), LABEL_ID: seldon_id, "version": version,
                  "app.kubernetes.io/managed-by": "seldon-core-amd"}
        pod = {"containers": [_engine_container(sdep, p, ns, n_gpus, workers)],
               "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]}
        prom = {"prometheus.io/scrape": "true", "prometheus.io/path": "/prometheus",
                "prometheus.io/port": str(HTTP_PORT)}
        out.append(_deployment(eng_name, ns, labels, pod, int(p.get("replicas", 1) or 1), prom))
        svc = naming.predictor_key(sdep, p)
        svc_ann = {AMBASSADOR_ANNOTATION: _ambassador(sdep, p, svc, ns)}
        out.append(_service(svc, ns, {LABEL_APP: svc, LABEL_ID: seldon_id}, svc,
                            [{"protocol": "TCP", "port": HTTP_PORT, "targetPort": HTTP_PORT, "name": "http"},
                             {"protocol": "TCP", "port": GRPC_PORT, "targetPort": GRPC_PORT, "name": "grpc"}],
                            svc_ann, headless=ann.get("seldon.io/headless-svc", "false") != "false"))
        routes.append({"vs": seldon_id, "host": svc, "subset": p["name"], "version": version,
                       "weight": 100 if n_pred <= 1 else int(p.get("traffic", 0) or 0)})
        # ---- external component containers (reference layout)
        for cs in p.get("componentSpecs") or []:
            containers = [c for c in ((cs.get("spec") or {}).get("containers") or []) if c.get("name") in ext]
            if not containers:
                continue
            dname = naming.deployment_name(sdep, p, cs)
            clabels = {LABEL_APP: dname, LABEL_ID: seldon_id, "version": version,
                       "app.kubernetes.io/managed-by": "seldon-core-amd"}
            cpod = copy.deepcopy(cs.get("spec") or {})
            cpod["containers"] = []
            for c in (cs.get("spec") or {}).get("containers") or []:
                c = copy.deepcopy(c)
                node = next((n for n, _ in iter_nodes(p["graph"]) if n["name"] == c.get("name")), None)
                if node is not None and c["name"] in ext:
                    ep = node.get("endpoint") or {}
                    port = int(ep.get("service_port") or 9000)
                    ptype = "grpc" if ep.get("type") == "GRPC" else "http"
                    c.setdefault("ports", [{"name": ptype, "containerPort": port, "protocol": "TCP"}])
                    have = {e.get("name") for e in c.get("env") or []}
                    c["env"] = list(c.get("env") or []) + [e for e in _unit_env(sdep, p, node, port)
                                                           if e["name"] not in have]
                    tcp = {"tcpSocket": {"port": port}, "periodSeconds": 5, "timeoutSeconds": 1,
                           "successThreshold": 1}
                    c.setdefault("readinessProbe", dict(tcp, initialDelaySeconds=20, failureThreshold=3))
                    c.setdefault("livenessProbe", dict(tcp, initialDelaySeconds=60, failureThreshold=3))
                    c.setdefault("lifecycle", {"preStop": {"exec": {"command": ["/bin/sh", "-c", "/bin/sleep 10"]}}})
                    cname = naming.container_service_name(sdep, p, c)
                    out.append(_service(cname, ns, {LABEL_APP: cname, LABEL_ID: seldon_id}, dname,
                                        [{"protocol": "TCP", "port": port, "targetPort": port, "name": ptype}]))
                cpod["containers"].append(c)
            out.append(_deployment(dname, ns, clabels, cpod, int(cs.get("replicas", p.get("replicas", 1)) or 1)))
            if cs.get("hpaSpec"):
                h = cs["hpaSpec"]
                out.append({"apiVersion": "autoscaling/v2beta1", "kind": "HorizontalPodAutoscaler",
                            "metadata": _meta(dname, ns, {LABEL_ID: seldon_id}),
                            "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": dname},
                                     "minReplicas": h.get("minReplicas", 1), "maxReplicas": h["maxReplicas"],
                                     "metrics": h.get("metrics", [])}})
        # ---- explainer
        ex = p.get("explainer") or {}
        if ex.get("type"):
            xname = naming.explainer_deployment_name(sdep["metadata"]["name"], p)
            port = int((ex.get("endpoint") or {}).get("service_port") or 9000)
            args = ["--model_name", sdep["metadata"]["name"], "--predictor_host", f"{svc}.{ns}:{HTTP_PORT}",
                    "--protocol", "seldon.http", "--http_port", str(port)]
            if ex.get("modelUri"):
                args += ["--storage_uri", ex["modelUri"]]
            args.append(ex["type"].lower())
            args += [f"--{k}={v}" for k, v in sorted((ex.get("config") or {}).items())]
            c = copy.deepcopy(ex.get("containerSpec") or {})
            c.setdefault("name", xname)
            c.setdefault("image", _engine_image())
            c["command"] = ["python", "-m", "seldon_core_amd.explainers.server"]
            c["args"] = args
            c.setdefault("ports", [{"name": "http", "containerPort": port, "protocol": "TCP"}])
            tcp = {"tcpSocket": {"port": port}, "periodSeconds": 5, "timeoutSeconds": 1, "successThreshold": 1}
            c.setdefault("readinessProbe", dict(tcp, initialDelaySeconds=20, failureThreshold=7))
            c.setdefault("livenessProbe", dict(tcp, initialDelaySeconds=60, failureThreshold=5))
            xl = {LABEL_APP: xname, LABEL_ID: seldon_id, "version": version,
                  "app.kubernetes.io/managed-by": "seldon-core-amd"}
            out.append(_deployment(xname, ns, xl, {"containers": [c]}, 1))
            out.append(_service(xname, ns, {LABEL_APP: xname, LABEL_ID: seldon_id}, xname,
                                [{"protocol": "TCP", "port": port, "targetPort": port, "name": "http"}],
                                {AMBASSADOR_ANNOTATION: _ambassador(
                                    {**sdep, "metadata": {**sdep["metadata"], "name": sdep["metadata"]["name"] +
                                                          "-explainer"}}, p, xname, ns)}))
            if istio:
                out += _istio(sdep, ns, seldon_id,
                              [{"vs": xname, "host": xname, "subset": p["name"], "version": version, "weight": 100}],
                              f"/seldon/{ns}/{sdep['metadata']['name']}/{p['name']}/explainer/", mtls=False)
    if istio and routes:
        out += _istio(sdep, ns, seldon_id, routes, f"/seldon/{ns}/{sdep['metadata']['name']}/")
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-k8s")
    ap.add_argument("spec")
    ap.add_argument("--namespace", default=None)
    ap.add_argument("--istio", action="store_true", default=None,
                    help="also render Istio VirtualServices / DestinationRules (default: $ISTIO_ENABLED)")
    a = ap.parse_args(argv)
    sys.stdout.write(yaml.safe_dump_all(render(a.spec, a.namespace, istio=a.istio), sort_keys=False))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
