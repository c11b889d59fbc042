"""In-cluster operator (reference operator/controllers/
seldondeployment_controller.go Reconcile, seldondeployment_webhook.go)
against a fake Kubernetes API server: server-side apply of the rendered
objects with owner references, status, pruning, failed specs, webhooks."""
import base64
import copy
import json
import re
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from seldon_core_amd import operator as op

PATH = re.compile(r"^/(?:api/v1|apis/[^/]+/[^/]+)(?:/namespaces/(?P<ns>[^/]+))?/(?P<plural>[^/]+)"
                  r"(?:/(?P<name>[^/]+))?(?P<status>/status)?$")


class FakeApi:
    def __init__(self):
        self.objs = {}  # (plural, ns, name) -> obj
        self.calls = []
        self.lock = threading.Lock()

    def handle(self, method, url, body):
        u = urllib.parse.urlparse(url)
        m = PATH.match(u.path)
        q = urllib.parse.parse_qs(u.query)
        plural, ns, name = m["plural"], m["ns"], m["name"]
        with self.lock:
            self.calls.append((method, plural, ns, name, bool(m["status"]), q))
            if method == "GET" and name is None:
                items = [o for (p, n, _), o in self.objs.items() if p == plural and (ns is None or n == ns)]
                if "labelSelector" in q:
                    k, v = q["labelSelector"][0].split("=")
                    items = [o for o in items if o["metadata"].get("labels", {}).get(k) == v]
                return 200, {"items": copy.deepcopy(items)}
            key = (plural, ns, name)
            if method == "GET":
                return (200, copy.deepcopy(self.objs[key])) if key in self.objs else (404, {"reason": "NotFound"})
            if method == "DELETE":
                return (200, self.objs.pop(key)) if key in self.objs else (404, {})
            if method == "PATCH" and m["status"]:
                if key not in self.objs:
                    return 404, {}
                self.objs[key]["status"] = body["status"]
                return 200, self.objs[key]
            if method == "PATCH":  # server-side apply: create or replace
                assert q.get("fieldManager") == ["seldon-core-amd"] and q.get("force") == ["true"]
                if key in self.objs and "status" in self.objs[key]:
                    body["status"] = self.objs[key]["status"]  # apply never touches status
                self.objs[key] = body
                return 200, body
        return 405, {}

    def serve(self):
        api = self

        class H(BaseHTTPRequestHandler):
            def _do(self):
                n = int(self.headers.get("Content-Length", 0))
                body = json.loads(self.rfile.read(n)) if n else None
                if self.command == "PATCH" and "/status" not in self.path:
                    assert self.headers["Content-Type"] == "application/apply-patch+yaml"
                code, out = api.handle(self.command, self.path, body)
                data = json.dumps(out).encode()
                self.send_response(code)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            do_GET = do_PATCH = do_DELETE = _do

            def log_message(self, *a):
                pass

        srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        return srv


@pytest.fixture
def api():
    fa = FakeApi()
    srv = fa.serve()
    yield fa, op.KubeClient(f"http://127.0.0.1:{srv.server_port}")
    srv.shutdown()


def _sdep(preds, name="mymodel", ns="ns1"):
    return {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": name, "namespace": ns, "uid": "uid-1"},
            "spec": {"name": name, "predictors": preds}}


def _pred(name, traffic=50):
    return {"name": name, "traffic": traffic, "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "clf", "type": "MODEL", "implementation": "SIMPLE_MODEL"}}


def test_reconcile_applies_status_and_prunes(api):
    fa, client = api
    sd = _sdep([_pred("a"), _pred("b")])
    fa.objs[("seldondeployments", "ns1", "mymodel")] = copy.deepcopy(sd)
    r = op.Reconciler(client, istio=False)
    out = r.reconcile_all()
    st = out["ns1/mymodel"]
    deps = {k[2]: o for k, o in fa.objs.items() if k[0] == "deployments"}
    svcs = {k[2]: o for k, o in fa.objs.items() if k[0] == "services"}
    assert len(deps) == 2 and len(svcs) == 2
    for o in list(deps.values()) + list(svcs.values()):
        ref, = o["metadata"]["ownerReferences"]
        assert ref["kind"] == "SeldonDeployment" and ref["uid"] == "uid-1" and ref["controller"]
        assert o["metadata"]["namespace"] == "ns1"
    assert st["state"] == "Creating" and set(st["deploymentStatus"]) == set(deps)
    assert all(s["grpcEndpoint"].endswith(":5001") for s in st["serviceStatus"].values())
    assert fa.objs[("seldondeployments", "ns1", "mymodel")]["status"]["state"] == "Creating"
    # the cluster brings the pods up -> Available
    for d in deps.values():
        d["status"] = {"replicas": 1, "availableReplicas": 1}
    assert r.reconcile_all()["ns1/mymodel"]["state"] == "Available"
    # drop predictor b -> its Deployment and Service are pruned
    sd2 = _sdep([_pred("a", 100)])
    sd2["status"] = fa.objs[("seldondeployments", "ns1", "mymodel")]["status"]
    fa.objs[("seldondeployments", "ns1", "mymodel")] = sd2
    r.reconcile_all()
    deps2 = {k[2] for k in fa.objs if k[0] == "deployments"}
    assert len(deps2) == 1 and deps2 < set(deps)
    assert sum(1 for k in fa.objs if k[0] == "services") == 1
    assert any(c[0] == "DELETE" for c in fa.calls)


def test_reconcile_istio_objects(api):
    fa, client = api
    fa.objs[("seldondeployments", "ns1", "m")] = _sdep([_pred("a", 60), _pred("b", 40)], name="m")
    op.Reconciler(client, istio=True).reconcile_all()
    assert sum(1 for k in fa.objs if k[0] == "virtualservices") == 2
    assert sum(1 for k in fa.objs if k[0] == "destinationrules") == 2


def test_invalid_spec_is_failed(api):
    fa, client = api
    bad = _sdep([_pred("a", 30), _pred("b", 30)])  # traffic must sum to 100
    fa.objs[("seldondeployments", "ns1", "mymodel")] = bad
    st = op.Reconciler(client, istio=False).reconcile_all()["ns1/mymodel"]
    assert st["state"] == "Failed" and "traffic" in st["description"].lower()
    assert not any(k[0] == "deployments" for k in fa.objs)


def test_webhooks():
    sd = _sdep([_pred("a", 100)])
    del sd["spec"]["predictors"][0]["graph"]["type"]
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
              "request": {"uid": "r1", "object": sd}}
    out = op.mutate(review)["response"]
    assert out["uid"] == "r1" and out["allowed"] and out["patchType"] == "JSONPatch"
    patch = json.loads(base64.b64decode(out["patch"]))
    assert patch[0]["path"] == "/spec" and patch[0]["value"]["predictors"][0]["graph"]["type"] == "UNKNOWN_TYPE"  # webhook Default()
    bad = _sdep([_pred("a", 30), _pred("b", 30)])
    res = op.admit({"request": {"uid": "r2", "object": bad}})["response"]
    assert not res["allowed"] and res["status"]["code"] == 400
    ok = op.admit({"request": {"uid": "r3", "object": _sdep([_pred("a", 100)])}})["response"]
    assert ok["allowed"]


def test_webhook_server_paths():
    import urllib.request

    srv = op.webhook_server("127.0.0.1", 0)
    try:
        body = json.dumps({"request": {"uid": "x", "object": _sdep([_pred("a", 100)])}}).encode()
        for path in op.WEBHOOK_PATHS:
            req = urllib.request.Request(f"http://127.0.0.1:{srv.server_port}{path}", data=body,
                                         headers={"Content-Type": "application/json"})
            assert json.loads(urllib.request.urlopen(req, timeout=10).read())["response"]["uid"] == "x"
    finally:
        srv.shutdown()


def test_usage_report_spartakus_format(api):
    import http.server

    from seldon_core_amd.usage import UsageReporter

    fa, client = api
    fa.objs[("nodes", None, "n1")] = {"metadata": {"name": "n1", "uid": "u1"},
                                      "status": {"nodeInfo": {"operatingSystem": "linux", "architecture": "amd64",
                                                              "kernelVersion": "6.8"},
                                                 "capacity": {"cpu": "256", "memory": "2Ti", "amd.com/gpu": "8",
                                                              "pods": "110"}}}
    fa.objs[("seldondeployments", "ns1", "m")] = _sdep([_pred("a", 100)], name="m")
    got = []

    class Collector(http.server.BaseHTTPRequestHandler):
        def do_POST(self):
            got.append(json.loads(self.rfile.read(int(self.headers["Content-Length"]))))
            self.send_response(201)
            self.send_header("Content-Length", "0")
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = http.server.HTTPServer(("127.0.0.1", 0), Collector)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        r = UsageReporter(client, f"http://127.0.0.1:{srv.server_port}")
        assert r.report_once()
    finally:
        srv.shutdown()
    rep, = got
    assert rep["version"] == "v1" and rep["clusterID"] == r.cluster_id
    node, = rep["nodes"]
    assert node["architecture"] == "amd64" and {"resource": "amd.com/gpu", "value": "8"} in node["capacity"]
    assert "n1" not in json.dumps(rep) and "ns1" not in json.dumps(rep)  # anonymous
    assert {"name": "seldondeployments", "value": "1"} in rep["extensions"]
    assert not UsageReporter(client, "http://127.0.0.1:9").report_once()  # unreachable: no exception
