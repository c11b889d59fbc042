"""Explainer server (reference operator/controllers/
seldondeployment_explainers.go:32-184 starts ``seldonio/alibiexplainer`` with
``--model_name --predictor_host --protocol seldon.http|seldon.grpc
--http_port <type> --<config key>=<value>...`` and exposes it as
``<sdep>-explainer``; python/seldon_core/seldon_client.py:1223-1321 posts a
SeldonMessage JSON to ``/seldon/<ns>/<sdep>-explainer/models/<sdep>:explain``).

    python -m seldon_core_amd.explainers.server --model_name income \
        --predictor_host 127.0.0.1:8000 --protocol seldon.http --http_port 9000 \
        anchor_tabular --training_data=/mnt/models/train.npy --feature_names=Age,Workclass,...

Routes (POST): ``.../models/<name>:explain`` (any gateway prefix),
``/v1/models/<name>:explain`` and ``/api/v0.1/explain``; GET ``/health``.
The body is a SeldonMessage (``data.ndarray`` / ``data.tensor`` / ``strData``)
or ``{"instances": [...]}``; the reply is the explanation JSON.

Perturbation batches are labelled by the predictor over REST (``seldon.http``)
or gRPC (``seldon.grpc``), or in-process through a ``Deployment`` when the
engine hosts the explainer itself (``serve`` with an ``explainer`` section):
each batch is one request, micro-batched onto the GPU like any other.

Explainer state comes from ``--storage_uri`` / the config, never from pickles:
``training_data`` is ``.npy`` (``allow_pickle=False``) or ``.csv``;
``feature_names`` a comma list or JSON list; ``categorical_names`` JSON
``{"<col>": ["name0", ...]}``; an ``explainer.json`` in the storage directory
may hold the same keys.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import re
import threading
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from .anchor import AnchorImage, AnchorTabular, AnchorText

log = logging.getLogger("seldon_core_amd.explainer")

EXPLAINER_TYPES = ("anchor_tabular", "anchor_text", "anchor_images")
_EXPLAIN_PATH = re.compile(r"(/models/[^/:]+:explain|/api/v0\.1/explain)$")


# ---------------------------------------------------------------- predictor
def _response_array(resp: Dict) -> np.ndarray:
    from ..serving.codec import datadef_to_array

    if "data" in resp:
        return np.asarray(datadef_to_array(resp["data"]))
    if "jsonData" in resp:
        return np.asarray(resp["jsonData"])
    raise RuntimeError(f"predictor returned no data: {str(resp)[:200]}")


def _request(batch) -> Dict:
    if isinstance(batch, list) and batch and isinstance(batch[0], str):
        return {"data": {"ndarray": batch}}
    arr = np.asarray(batch)
    if arr.dtype.kind in "fiub":
        return {"data": {"tensor": {"shape": list(arr.shape), "values": arr.astype(np.float64).ravel().tolist()}}}
    return {"data": {"ndarray": arr.tolist()}}


def rest_predictor(host: str, timeout: float = 60.0) -> Callable:
    url = f"http://{host}/api/v0.1/predictions"

    def predict(batch):
        body = json.dumps(_request(batch)).encode()
        req = urllib.request.Request(url, data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return _response_array(json.loads(r.read()))

    return predict


def grpc_predictor(host: str) -> Callable:
    from ..client import SeldonClient

    sc = SeldonClient(gateway="seldon", transport="grpc", seldon_grpc_endpoint=host)

    def predict(batch):
        if isinstance(batch, list) and batch and isinstance(batch[0], str):
            r = sc.predict(data=np.array(batch, dtype=object), payload_type="ndarray")
        else:
            r = sc.predict(data=np.asarray(batch, dtype=np.float64))
        if not r.success:
            raise RuntimeError(r.msg)
        from google.protobuf import json_format

        return _response_array(json_format.MessageToDict(r.response))

    return predict


def deployment_predictor(dep) -> Callable:
    def predict(batch):
        return _response_array(dep.predict(_request(batch)))

    return predict


# ---------------------------------------------------------------- explainer
def _load_matrix(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False)
    return np.loadtxt(path, delimiter=",", dtype=np.float64, ndmin=2)


def _config(cfg: Dict[str, Any], storage_uri: Optional[str]) -> Dict[str, Any]:
    cfg = dict(cfg)
    if storage_uri:
        from ..utils.storage import Storage

        root = Storage.download(storage_uri)
        meta = os.path.join(root, "explainer.json")
        if os.path.exists(meta):
            with open(meta) as f:
                cfg = {**json.load(f), **cfg}
        for k in ("training_data",):
            if k in cfg and not os.path.isabs(str(cfg[k])):
                cfg[k] = os.path.join(root, cfg[k])
        if "training_data" not in cfg:
            for cand in ("training_data.npy", "train.npy", "training_data.csv"):
                if os.path.exists(os.path.join(root, cand)):
                    cfg["training_data"] = os.path.join(root, cand)
                    break
    return cfg


def _list(v) -> List[str]:
    if isinstance(v, list):
        return [str(x) for x in v]
    v = str(v).strip()
    return [str(x) for x in json.loads(v)] if v.startswith("[") else [x.strip() for x in v.split(",") if x.strip()]


_EXPLAIN_KW = {"threshold": float, "delta": float, "tau": float, "batch_size": int, "coverage_samples": int,
               "beam_size": int, "max_anchor_size": int, "sample_proba": float, "p_sample": float,
               "min_samples_start": int, "max_samples": int}


class Explainer:
    def __init__(self, kind: str, predict_fn: Callable, config: Optional[Dict[str, Any]] = None,
                 storage_uri: Optional[str] = None):
        if kind not in EXPLAINER_TYPES:
            raise ValueError(f"unknown explainer type {kind}; supported: {', '.join(EXPLAINER_TYPES)}")
        cfg = _config(config or {}, storage_uri)
        self.kind = kind
        self.explain_kw = {k: t(cfg[k]) for k, t in _EXPLAIN_KW.items() if k in cfg}
        seed = int(cfg.get("seed", 0))
        self.lock = threading.Lock()  # explainers keep an RNG; one explanation at a time
        if kind == "anchor_tabular":
            if "training_data" not in cfg:
                raise ValueError("anchor_tabular needs training_data (config or storage_uri)")
            train = _load_matrix(str(cfg["training_data"]))
            names = _list(cfg["feature_names"]) if "feature_names" in cfg else [f"f{i}" for i in
                                                                                 range(train.shape[1])]
            cats = cfg.get("categorical_names") or {}
            if isinstance(cats, str):
                cats = json.loads(cats)
            cats = {int(k): list(v) for k, v in cats.items()}
            disc = [float(x) for x in _list(cfg["disc_perc"])] if "disc_perc" in cfg else (25, 50, 75)
            self.impl = AnchorTabular(predict_fn, names, cats, seed=seed).fit(train, disc)
        elif kind == "anchor_text":
            self.impl = AnchorText(predict_fn, seed=seed)
        else:
            shape = [int(x) for x in _list(cfg.get("image_shape", "32,32,3"))]
            seg_kw = {"n_segments": int(cfg.get("n_segments", 16))}
            if "compactness" in cfg:
                seg_kw["compactness"] = float(cfg["compactness"])
            self.impl = AnchorImage(predict_fn, shape, segmentation_kwargs=seg_kw, seed=seed)

    def explain(self, payload: Dict) -> Dict:
        inst = _instance(payload)
        with self.lock:
            if self.kind == "anchor_text":
                text = inst if isinstance(inst, str) else str(np.asarray(inst).ravel()[0])
                return _jsonable(self.impl.explain(text, **self.explain_kw))
            arr = np.asarray(inst, dtype=np.float64)
            if self.kind == "anchor_tabular":
                return _jsonable(self.impl.explain(arr.reshape(-1, arr.shape[-1])[0], **self.explain_kw))
            return _jsonable(self.impl.explain(arr.reshape(self.impl.image_shape), **self.explain_kw))


def _instance(payload: Dict):
    if "instances" in payload:
        return payload["instances"][0] if isinstance(payload["instances"], list) else payload["instances"]
    if "strData" in payload:
        return payload["strData"]
    if "data" in payload:
        from ..serving.codec import datadef_to_array

        arr = datadef_to_array(payload["data"])
        if arr.dtype.kind in "OUS":
            return str(arr.ravel()[0])
        return arr[0] if arr.ndim > 1 and arr.shape[0] == 1 else arr
    raise ValueError("request has no data / strData / instances")


def _jsonable(o):
    if isinstance(o, dict):
        return {str(k): _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, np.ndarray):
        return _jsonable(o.tolist())
    if isinstance(o, np.generic):
        return o.item()
    return o


# ---------------------------------------------------------------- HTTP
class ExplainerServer:
    def __init__(self, explainer: Explainer, model_name: str, host: str = "0.0.0.0", port: int = 9000):
        ex, name = explainer, model_name

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # noqa: D401
                log.debug(*a)

            def _send(self, code: int, obj: Dict) -> None:
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path.rstrip("/").endswith(("/health", "/ready", "/live", "/ping")):
                    return self._send(200, {"status": "ok", "model": name, "explainer": ex.kind})
                self._send(404, {"error": f"no route {self.path}"})

            def do_POST(self):
                n = int(self.headers.get("Content-Length", "0") or 0)
                raw = self.rfile.read(n)
                path = self.path.split("?", 1)[0]
                m = _EXPLAIN_PATH.search(path)
                if not m:
                    return self._send(404, {"error": f"no route {self.path}"})
                if m.group(1).startswith("/models/") and m.group(1)[len("/models/"):-len(":explain")] != name:
                    return self._send(404, {"error": f"model {m.group(1)[8:-8]} not found (serving {name})"})
                try:
                    payload = json.loads(raw or b"{}")
                    if isinstance(payload, str):  # form-style double encoding
                        payload = json.loads(payload)
                    self._send(200, ex.explain(payload))
                except Exception as e:  # explanation errors are client-visible, server stays up
                    log.exception("explain failed")
                    self._send(400 if isinstance(e, (ValueError, KeyError)) else 500, {"error": str(e)})

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.thread: Optional[threading.Thread] = None

    def start(self) -> "ExplainerServer":
        self.thread = threading.Thread(target=self.httpd.serve_forever, name="explainer", daemon=True)
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def from_spec(predictor: Dict, predict_fn: Callable, model_name: str, host: str = "0.0.0.0",
              port: Optional[int] = None) -> Optional[ExplainerServer]:
    """Explainer for a PredictorSpec's ``explainer`` section (None if absent)."""
    spec = predictor.get("explainer") or {}
    if not spec.get("type"):
        return None
    ep = spec.get("endpoint") or {}
    port = port if port is not None else int(ep.get("service_port") or 9000)
    ex = Explainer(spec["type"].lower(), predict_fn, spec.get("config") or {}, spec.get("modelUri"))
    return ExplainerServer(ex, model_name, host, port)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-explainer")
    ap.add_argument("--model_name", required=True)
    ap.add_argument("--predictor_host", required=True)
    ap.add_argument("--protocol", default="seldon.http", choices=["seldon.http", "seldon.grpc"])
    ap.add_argument("--http_port", type=int, default=9000)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--storage_uri", default=None)
    ap.add_argument("--use_grpc", action="store_true", help="accepted for compatibility (protocol decides)")
    ap.add_argument("--tf_data_type", default=None, help="accepted for compatibility")
    ap.add_argument("type", choices=EXPLAINER_TYPES)
    args, rest = ap.parse_known_args(argv)
    cfg: Dict[str, str] = {}
    for r in rest:
        if not r.startswith("--") or "=" not in r:
            ap.error(f"explainer config must be --key=value, got {r}")
        k, _, v = r[2:].partition("=")
        cfg[k] = v
    logging.basicConfig(level=logging.INFO)
    pf = grpc_predictor(args.predictor_host) if args.protocol == "seldon.grpc" else rest_predictor(args.predictor_host)
    srv = ExplainerServer(Explainer(args.type, pf, cfg, args.storage_uri), args.model_name, args.host, args.http_port)
    log.info("explainer %s for %s on :%d -> %s (%s)", args.type, args.model_name, srv.port, args.predictor_host,
             args.protocol)
    try:
        srv.httpd.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
