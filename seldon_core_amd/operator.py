"""In-cluster SeldonDeployment operator (reference
operator/main.go, operator/controllers/seldondeployment_controller.go:
860-1150 -- the Reconcile loop --, operator/api/v1alpha2/
seldondeployment_webhook.go:417-460 -- defaulting and validating webhooks).

    python -m seldon_core_amd.operator [--namespace NS] [--resync 10] [--webhook-port 9443 --cert C --key K]

Reconcile, per SeldonDeployment:

1. validate the spec (``serving.spec.validate``); invalid -> ``status.state =
   Failed`` with the messages as ``description``;
2. render the objects (``k8s.render``: engine Deployments that request
   ``amd.com/gpu``, predictor Services with Ambassador mappings, external
   component Deployments / Services / HPAs, explainer, Istio objects when
   ``ISTIO_ENABLED``), stamp an owner reference to the SeldonDeployment so the
   garbage collector removes them with it, and server-side apply each one
   (``PATCH application/apply-patch+yaml``, field manager ``seldon-core-amd``)
   -- create and update are one idempotent call;
3. prune objects labelled ``seldon-deployment-id=<id>`` that the current spec
   no longer renders (a removed predictor, a renamed component);
4. write ``status``: ``deploymentStatus`` (replicas / availableReplicas of every
   owned Deployment), ``serviceStatus`` (REST / gRPC endpoints of the predictor
   and explainer Services) and ``state`` = Available when every Deployment has
   all replicas available, else Creating.

The loop lists every SeldonDeployment each ``resync`` seconds (level-triggered
reconciliation; the reference's watch/requeue gives the same fixed point).
The API client is stdlib HTTPS with the pod's service-account token, so the
operator image is the engine image.  The webhooks serve AdmissionReview v1
(mutating: JSON patch replacing ``spec`` with the defaulted spec; validating:
``allowed`` + the validation messages).
"""
from __future__ import annotations

import argparse
import base64
import copy
import json
import logging
import os
import ssl
import threading
import urllib.error
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, Iterable, List, Optional, Tuple

from . import k8s
from .serving import naming
from .serving.spec import apply_defaults, validate

logger = logging.getLogger(__name__)

GROUP, VERSION, PLURAL = "machinelearning.seldon.io", "v1alpha2", "seldondeployments"
FIELD_MANAGER = "seldon-core-amd"
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

# kind -> (api prefix, plural) for every kind k8s.render emits
KINDS: Dict[str, Tuple[str, str]] = {
    "Deployment": ("/apis/apps/v1", "deployments"),
    "Service": ("/api/v1", "services"),
    "HorizontalPodAutoscaler": ("/apis/autoscaling/v2beta1", "horizontalpodautoscalers"),
    "VirtualService": ("/apis/networking.istio.io/v1alpha3", "virtualservices"),
    "DestinationRule": ("/apis/networking.istio.io/v1alpha3", "destinationrules"),
}


class ApiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{code}: {msg}")
        self.code = code


class KubeClient:
    """Minimal Kubernetes REST client (JSON over HTTPS, bearer token)."""

    def __init__(self, base_url: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 insecure: bool = False, timeout: float = 30.0):
        self.base = base_url.rstrip("/")
        self.token = token
        self.timeout = timeout
        self.ctx = None
        if self.base.startswith("https"):
            self.ctx = ssl.create_default_context(cafile=ca_file)
            if insecure:
                self.ctx.check_hostname = False
                self.ctx.verify_mode = ssl.CERT_NONE

    @classmethod
    def in_cluster(cls) -> "KubeClient":
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        with open(os.path.join(SA_DIR, "token")) as f:
            token = f.read().strip()
        return cls(f"https://{host}:{port}", token, os.path.join(SA_DIR, "ca.crt"))

    def request(self, method: str, path: str, body: Any = None, content_type: str = "application/json") -> Any:
        data = None if body is None else json.dumps(body).encode()
        req = urllib.request.Request(self.base + path, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self.ctx) as r:
                raw = r.read()
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        return json.loads(raw) if raw else None

    def get(self, path: str) -> Any:
        return self.request("GET", path)

    def apply(self, path: str, obj: Dict) -> Any:
        return self.request("PATCH", f"{path}?fieldManager={FIELD_MANAGER}&force=true", obj,
                            "application/apply-patch+yaml")

    def merge_patch(self, path: str, patch: Dict) -> Any:
        return self.request("PATCH", path, patch, "application/merge-patch+json")

    def delete(self, path: str) -> Any:
        return self.request("DELETE", path, {"kind": "DeleteOptions", "apiVersion": "v1",
                                             "propagationPolicy": "Background"})


def _sdep_path(ns: Optional[str], name: Optional[str] = None) -> str:
    p = f"/apis/{GROUP}/{VERSION}"
    if ns:
        p += f"/namespaces/{ns}"
    p += f"/{PLURAL}"
    return p + (f"/{name}" if name else "")


def _obj_path(kind: str, ns: str, name: Optional[str] = None) -> str:
    prefix, plural = KINDS[kind]
    return f"{prefix}/namespaces/{ns}/{plural}" + (f"/{name}" if name else "")


class Reconciler:
    def __init__(self, client: KubeClient, namespace: Optional[str] = None, istio: Optional[bool] = None):
        self.client = client
        self.namespace = namespace
        self.istio = k8s.istio_enabled() if istio is None else istio
        self.reconciles = 0

    # ------------------------------------------------------------ one SDep
    def reconcile(self, sdep: Dict) -> Dict:
        meta = sdep["metadata"]
        ns = meta.get("namespace") or self.namespace or "default"
        name = meta["name"]
        self.reconciles += 1
        errs = validate(apply_defaults(sdep))
        if errs:
            status = {"state": "Failed", "description": "; ".join(errs)}
            self._write_status(ns, name, status)
            return status
        try:
            objs = k8s.render(sdep, ns, istio=self.istio)
        except (KeyError, ValueError, TypeError) as e:
            status = {"state": "Failed", "description": f"render: {e}"}
            self._write_status(ns, name, status)
            return status
        seldon_id = naming.sdep_name(apply_defaults(copy.deepcopy(sdep)))
        owner = {"apiVersion": f"{GROUP}/{VERSION}", "kind": "SeldonDeployment", "name": name,
                 "uid": meta.get("uid", ""), "controller": True, "blockOwnerDeletion": True}
        wanted = set()
        for o in objs:
            o = copy.deepcopy(o)
            o["metadata"]["namespace"] = ns
            o["metadata"].setdefault("labels", {})[k8s.LABEL_ID] = seldon_id
            o["metadata"]["ownerReferences"] = [owner]
            self.client.apply(_obj_path(o["kind"], ns, o["metadata"]["name"]), o)
            wanted.add((o["kind"], o["metadata"]["name"]))
        self._prune(ns, seldon_id, wanted)
        status = self._status(ns, sdep, objs)
        self._write_status(ns, name, status)
        return status

    def _owned(self, ns: str, seldon_id: str, kinds: Iterable[str]) -> List[Tuple[str, Dict]]:
        out = []
        for kind in kinds:
            try:
                lst = self.client.get(f"{_obj_path(kind, ns)}?labelSelector={k8s.LABEL_ID}%3D{seldon_id}")
            except ApiError as e:
                if e.code == 404 and kind in ("VirtualService", "DestinationRule"):
                    continue  # Istio CRDs not installed
                raise
            out += [(kind, item) for item in (lst or {}).get("items", [])]
        return out

    def _prune(self, ns: str, seldon_id: str, wanted: set) -> None:
        kinds = [k for k in KINDS if self.istio or k not in ("VirtualService", "DestinationRule")]
        for kind, item in self._owned(ns, seldon_id, kinds):
            n = item["metadata"]["name"]
            if (kind, n) not in wanted:
                logger.info("pruning %s %s/%s", kind, ns, n)
                try:
                    self.client.delete(_obj_path(kind, ns, n))
                except ApiError as e:
                    if e.code != 404:
                        raise

    def _status(self, ns: str, sdep: Dict, objs: List[Dict]) -> Dict:
        dep_status: Dict[str, Dict] = {}
        ready = True
        for o in objs:
            if o["kind"] != "Deployment":
                continue
            n = o["metadata"]["name"]
            try:
                live = self.client.get(_obj_path("Deployment", ns, n))
            except ApiError:
                live = {}
            st = (live or {}).get("status") or {}
            want = int(o["spec"].get("replicas", 1))
            avail = int(st.get("availableReplicas", 0) or 0)
            ds = {"name": n, "replicas": int(st.get("replicas", 0) or 0), "availableReplicas": avail,
                  "status": "Available" if avail >= want else "Creating"}
            if n.endswith("-explainer"):
                ds["explainerFor"] = n[: -len("-explainer")]
            dep_status[n] = ds
            ready &= avail >= want
        svc_status: Dict[str, Dict] = {}
        for o in objs:
            if o["kind"] != "Service":
                continue
            ports = {p["name"]: p["port"] for p in o["spec"].get("ports", [])}
            n = o["metadata"]["name"]
            ss = {"svcName": n}
            if "http" in ports:
                ss["httpEndpoint"] = f"{n}.{ns}:{ports['http']}"
            if "grpc" in ports:
                ss["grpcEndpoint"] = f"{n}.{ns}:{ports['grpc']}"
            svc_status[n] = ss
        return {"state": "Available" if ready else "Creating", "deploymentStatus": dep_status,
                "serviceStatus": svc_status}

    def _write_status(self, ns: str, name: str, status: Dict) -> None:
        try:
            self.client.merge_patch(_sdep_path(ns, name) + "/status", {"status": status})
        except ApiError as e:
            logger.warning("status update of %s/%s failed: %s", ns, name, e)

    # ------------------------------------------------------------ loop
    def reconcile_all(self) -> Dict[str, Dict]:
        out = {}
        for sdep in (self.client.get(_sdep_path(self.namespace)) or {}).get("items", []):
            key = f"{sdep['metadata'].get('namespace', 'default')}/{sdep['metadata']['name']}"
            if sdep["metadata"].get("deletionTimestamp"):
                continue  # owner references let the garbage collector finish it
            try:
                out[key] = self.reconcile(sdep)
            except ApiError as e:
                logger.error("reconcile %s failed: %s", key, e)
                out[key] = {"state": "Failed", "description": str(e)}
        return out

    def run(self, resync: float = 10.0, stop: Optional[threading.Event] = None) -> None:
        stop = stop or threading.Event()
        while not stop.is_set():
            try:
                self.reconcile_all()
            except (ApiError, OSError) as e:
                logger.error("list failed: %s", e)
            stop.wait(resync)


# ---------------------------------------------------------------- webhooks
def _review_response(review: Dict, allowed: bool, message: str = "", patch: Optional[List] = None) -> Dict:
    resp: Dict[str, Any] = {"uid": (review.get("request") or {}).get("uid", ""), "allowed": allowed}
    if message:
        resp["status"] = {"message": message, "code": 200 if allowed else 400}
    if patch is not None:
        resp["patchType"] = "JSONPatch"
        resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
    return {"apiVersion": review.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview",
            "response": resp}


def mutate(review: Dict) -> Dict:
    """Defaulting webhook (seldondeployment_webhook.go Default())."""
    obj = (review.get("request") or {}).get("object") or {}
    defaulted = apply_defaults(obj)
    patch = [] if defaulted.get("spec") == obj.get("spec") else [
        {"op": "replace" if "spec" in obj else "add", "path": "/spec", "value": defaulted["spec"]}]
    return _review_response(review, True, patch=patch)


def admit(review: Dict) -> Dict:
    """Validating webhook (ValidateCreate / ValidateUpdate)."""
    obj = (review.get("request") or {}).get("object") or {}
    errs = validate(apply_defaults(obj))
    return _review_response(review, not errs, "; ".join(errs))


WEBHOOK_PATHS = {f"/mutate-{GROUP.replace('.', '-')}-{VERSION}-seldondeployment": mutate,
                 f"/validate-{GROUP.replace('.', '-')}-{VERSION}-seldondeployment": admit}


class _WebhookHandler(BaseHTTPRequestHandler):
    def do_POST(self):
        fn = WEBHOOK_PATHS.get(self.path.split("?")[0])
        if fn is None:
            self.send_error(404)
            return
        try:
            review = json.loads(self.rfile.read(int(self.headers.get("Content-Length", 0))))
            body = json.dumps(fn(review)).encode()
        except (ValueError, KeyError, TypeError) as e:
            self.send_error(400, str(e))
            return
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


def webhook_server(host: str = "0.0.0.0", port: int = 9443, cert: Optional[str] = None,
                   key: Optional[str] = None) -> ThreadingHTTPServer:
    srv = ThreadingHTTPServer((host, port), _WebhookHandler)
    if cert:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(cert, key)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    threading.Thread(target=srv.serve_forever, daemon=True, name="sdep-webhook").start()
    return srv


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-operator")
    ap.add_argument("--namespace", default=os.environ.get("WATCH_NAMESPACE") or None)
    ap.add_argument("--resync", type=float, default=10.0)
    ap.add_argument("--api", default=None, help="API server URL (default: in-cluster config)")
    ap.add_argument("--webhook-port", type=int, default=0)
    ap.add_argument("--cert", default=None)
    ap.add_argument("--key", default=None)
    ap.add_argument("--usage-database", default=None,
                    help="opt-in anonymous usage reports (spartakus format) to this URL")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    client = KubeClient(a.api) if a.api else KubeClient.in_cluster()
    if a.webhook_port:
        webhook_server(port=a.webhook_port, cert=a.cert, key=a.key)
    if a.usage_database:
        from .usage import UsageReporter

        UsageReporter(client, a.usage_database).start()
    Reconciler(client, a.namespace).run(a.resync)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
