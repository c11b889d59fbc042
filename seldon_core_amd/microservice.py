"""``seldon-core-microservice``-compatible launcher (reference
python/seldon_core/microservice.py:177-322).

    python -m seldon_core_amd.microservice <Interface> REST|GRPC \
        [--service-type MODEL|ROUTER|TRANSFORMER|COMBINER|OUTLIER_DETECTOR] \
        [--persistence] [--parameters '<json list>'] [--log-level INFO] \
        [--tracing] [--workers N] [--batching ROWS]

The user class is imported exactly as the reference does (``Module`` ->
``Module.Module``, ``pkg.mod.Class`` -> ``pkg.mod.Class``), built from the
typed ``PREDICTIVE_UNIT_PARAMETERS`` and served by the native HTTP/1.1 server
(internal API: /predict /transform-input /transform-output /route /aggregate
/send-feedback /seldon.json, plus /ping /ready /live /prometheus) or the native
gRPC server (Generic / Model / Router / Transformer / OutputTransformer /
Combiner services) on ``PREDICTIVE_UNIT_SERVICE_PORT`` (default 5000).
"""
from __future__ import annotations

import argparse
import importlib
import json
import logging
import os
import sys
import threading
from typing import Any, Dict, List

logger = logging.getLogger(__name__)

PARAMETERS_ENV_NAME = "PREDICTIVE_UNIT_PARAMETERS"
SERVICE_PORT_ENV_NAME = "PREDICTIVE_UNIT_SERVICE_PORT"
LOG_LEVEL_ENV = "SELDON_LOG_LEVEL"
DEFAULT_PORT = 5000
ANNOTATIONS_FILE = "/etc/podinfo/annotations"

SERVICE_TO_NODE_TYPE = {"MODEL": "MODEL", "ROUTER": "ROUTER", "TRANSFORMER": "TRANSFORMER",
                        "COMBINER": "COMBINER", "OUTLIER_DETECTOR": "TRANSFORMER"}


def parse_parameters(parameters: List[Dict]) -> Dict[str, Any]:
    casts = {"INT": int, "FLOAT": float, "DOUBLE": float, "STRING": str,
             "BOOL": lambda v: str(v).lower() in ("1", "true")}
    out = {}
    for p in parameters:
        t = p.get("type", "STRING")
        if t not in casts:
            raise ValueError(f"Bad parameter type {t} for {p.get('name')}")
        try:
            out[p["name"]] = casts[t](p["value"])
        except ValueError as e:
            raise ValueError(f"Bad value {p['value']!r} for {t} parameter {p['name']}") from e
    return out


def load_annotations(path: str = ANNOTATIONS_FILE) -> Dict[str, str]:
    """Downward-API annotations file: ``key="value"`` per line."""
    out: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                line = line.strip()
                if "=" not in line:
                    continue
                k, v = line.split("=", 1)
                out[k] = v.strip().strip('"')
    except OSError:
        pass
    return out


def import_user_class(interface_name: str):
    parts = interface_name.rsplit(".", 1)
    if len(parts) == 1:
        mod = importlib.import_module(interface_name)
        return getattr(mod, interface_name)
    mod = importlib.import_module(parts[0])
    return getattr(mod, parts[1])


def build_microservice(user_object: Any, service_type: str = "MODEL", name: str = None, device: int = None,
                       workers: int = 0, batching: int = 0):
    """A one-node deployment wrapping the component (graph-equivalent).
    ``workers`` > 0 runs the component in that many worker processes (the
    reference's gunicorn workers); ``batching`` stacks concurrent requests."""
    from .serving.deployment import Deployment

    name = name or os.environ.get("PREDICTIVE_UNIT_ID", "model")
    node_type = SERVICE_TO_NODE_TYPE.get(service_type, "MODEL")
    spec = {"name": os.environ.get("PREDICTOR_ID", "microservice"),
            "graph": {"name": name, "type": node_type, "children": []}}
    if node_type == "ROUTER":  # a router needs children to be a valid graph node type; keep methods explicit
        spec["graph"] = {"name": name, "type": "UNKNOWN_TYPE", "methods": ["ROUTE", "SEND_FEEDBACK"]}
    elif node_type == "COMBINER":
        spec["graph"] = {"name": name, "type": "UNKNOWN_TYPE", "methods": ["AGGREGATE"]}
    if workers > 0:
        spec["graph"]["workers"] = int(workers)
    if batching > 0:
        spec["graph"]["batching"] = int(batching)
    return Deployment(spec, components={name: user_object}, device=device)


class _Response:
    """What a Flask test client returns, as far as component tests use it."""

    def __init__(self, status: int, data: bytes, headers: Dict[str, str]):
        self.status_code = status
        self.data = data
        self.headers = headers

    @property
    def status(self) -> str:
        return str(self.status_code)

    def get_json(self):
        return json.loads(self.data)

    def get_data(self, as_text: bool = False):
        return self.data.decode() if as_text else self.data


class _TestClient:
    """``app.test_client()``: real HTTP requests to the app's native server on
    a loopback port, with Flask's call shapes -- ``get(path_with_query)``,
    ``post(path, data={...}, content_type=...)`` where a value may be a
    ``(path, filename)`` file tuple (multipart) -- so component tests written
    for the reference's Flask wrapper keep running."""

    def __init__(self, app: "MicroserviceApp"):
        self.app = app

    def _send(self, method: str, path: str, body: bytes = None, content_type: str = None) -> _Response:
        import urllib.error
        import urllib.parse
        import urllib.request

        base, _, query = path.partition("?")
        if query:  # Flask's client percent-encodes the query; so do we
            query = urllib.parse.urlencode(urllib.parse.parse_qsl(query, keep_blank_values=True))
        url = f"http://127.0.0.1:{self.app.port}{base}" + (f"?{query}" if query else "")
        req = urllib.request.Request(url, data=body, method=method)
        if content_type:
            req.add_header("Content-Type", content_type)
        try:
            with urllib.request.urlopen(req, timeout=60) as r:
                return _Response(r.status, r.read(), dict(r.headers))
        except urllib.error.HTTPError as e:
            return _Response(e.code, e.read(), dict(e.headers))

    def get(self, path: str, **_kw) -> _Response:
        return self._send("GET", path)

    def post(self, path: str, data=None, json_body=None, content_type: str = None, **kw) -> _Response:
        import urllib.parse

        if "json" in kw:
            json_body = kw["json"]
        if json_body is not None:
            return self._send("POST", path, json.dumps(json_body).encode(), "application/json")
        if isinstance(data, (bytes, str)):
            return self._send("POST", path, data.encode() if isinstance(data, str) else data,
                              content_type or "application/json")
        data = data or {}
        if content_type and content_type.startswith("multipart/form-data"):
            body, ctype = _multipart(data)
            return self._send("POST", path, body, ctype)
        return self._send("POST", path, urllib.parse.urlencode(data).encode(), "application/x-www-form-urlencoded")


def _multipart(fields: Dict[str, Any]):
    import uuid

    boundary = uuid.uuid4().hex
    out = []
    for k, v in fields.items():
        if isinstance(v, tuple):  # (path or file object, filename)
            src, fname = v[0], v[1] if len(v) > 1 else "file"
            content = open(src, "rb").read() if isinstance(src, str) else src.read()
            out.append(f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"; filename="{fname}"\r\n'
                       f"Content-Type: application/octet-stream\r\n\r\n".encode() + content + b"\r\n")
        else:
            out.append(f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n{v}\r\n'.encode())
    out.append(f"--{boundary}--\r\n".encode())
    return b"".join(out), f"multipart/form-data; boundary={boundary}"


class MicroserviceApp:
    """``get_rest_microservice(user_object)``: the component behind the native
    internal-API server (what ``python -m seldon_core_amd.microservice``
    serves), with the reference's Flask-app surface for tests and embedding:
    ``test_client()`` and ``run(host, port)``.  The server starts on first use
    on an ephemeral loopback port; ``close()`` stops it."""

    def __init__(self, user_object: Any, service_type: str = "MODEL"):
        self.user_object = user_object
        self.service_type = service_type
        self._dep = None
        self._http = None

    def _start(self, host: str = "127.0.0.1", port: int = 0, threads: int = 4):
        if self._http is None:
            from .serving.openapi import wrapper_spec_json

            self._dep = build_microservice(self.user_object, self.service_type, device=-1)
            node = self._dep.predictor["graph"]["name"]
            self._http = self._dep.C.HttpServer(self._dep.engine, host, [port], threads, node, True,
                                                wrapper_spec_json())
            self._http.start()
        return self

    @property
    def port(self) -> int:
        return self._start()._http.ports[0]

    def test_client(self) -> _TestClient:
        self._start()
        return _TestClient(self)

    def run(self, host: str = "0.0.0.0", port: int = DEFAULT_PORT, **_kw) -> None:
        from .utils.shutdown import StopSignal

        self._start(host, port)
        StopSignal().install().wait()
        self.close()

    def close(self) -> None:
        if self._http is not None:
            self._http.stop()
            self._http = None
        if self._dep is not None:
            self._dep.close()
            self._dep = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  interpreter shutdown
            pass


def get_rest_microservice(user_object: Any, service_type: str = "MODEL") -> MicroserviceApp:
    """The reference's ``seldon_core.wrapper.get_rest_microservice`` (wrapper.py:22-31)."""
    return MicroserviceApp(user_object, service_type)


def main(argv=None) -> None:
    logging.basicConfig(level=logging.INFO,
                        format="%(asctime)s - %(name)s:%(funcName)s:%(lineno)s - %(levelname)s:  %(message)s")
    sys.path.append(os.getcwd())
    ap = argparse.ArgumentParser(prog="seldon-core-microservice")
    ap.add_argument("interface_name", type=str)
    ap.add_argument("api_type", type=str, choices=["REST", "GRPC", "FBS"])
    ap.add_argument("--service-type", type=str, default="MODEL",
                    choices=["MODEL", "ROUTER", "TRANSFORMER", "COMBINER", "OUTLIER_DETECTOR"])
    ap.add_argument("--persistence", nargs="?", default=0, const=1, type=int)
    ap.add_argument("--parameters", type=str, default=os.environ.get(PARAMETERS_ENV_NAME, "[]"))
    ap.add_argument("--log-level", type=str, default="INFO")
    ap.add_argument("--tracing", nargs="?", default=int(os.environ.get("TRACING", "0")), const=1, type=int)
    ap.add_argument("--workers", type=int, default=int(os.environ.get("GUNICORN_WORKERS", "4")),
                    help="component worker processes when > 1 (the reference's gunicorn workers); "
                         "the native front end uses max(workers, 4) I/O threads")
    ap.add_argument("--batching", type=int, default=int(os.environ.get("SELDON_BATCHING", "0")),
                    help="stack concurrent requests to a row-wise component, up to this many rows (0 = off)")
    ap.add_argument("--port", type=int, default=int(os.environ.get(SERVICE_PORT_ENV_NAME, DEFAULT_PORT)))
    ap.add_argument("--device", type=int, default=None, help="GPU for native units (-1 = CPU)")
    args = ap.parse_args(argv)

    level = getattr(logging, os.environ.get(LOG_LEVEL_ENV, args.log_level.upper()), None)
    if not isinstance(level, int):
        raise ValueError(f"Invalid log level: {args.log_level}")
    logging.getLogger().setLevel(level)
    if args.api_type == "FBS":
        raise SystemExit("FBS (FlatBuffers) API is not supported (vestigial in the reference too)")

    parameters = parse_parameters(json.loads(args.parameters))
    annotations = load_annotations()
    logger.info("Annotations: %s", annotations)
    user_class = import_user_class(args.interface_name)
    persister = None
    if args.persistence:
        from .utils import persistence

        user_object = persistence.restore(user_class, parameters)
        persister = persistence.persist(user_object, parameters.get("push_frequency"))
    else:
        user_object = user_class(**parameters)
    try:
        user_object.load()
    except (NotImplementedError, AttributeError):
        pass
    if args.tracing:
        from .utils.tracing import configure_tracing

        configure_tracing(args.interface_name)

    workers = args.workers if args.workers > 1 else 0
    if workers and args.persistence:
        logger.warning("--persistence keeps one copy of the component: running it in-process, not in %d workers",
                       workers)
        workers = 0
    dep = build_microservice(user_object, args.service_type, device=args.device, workers=workers,
                             batching=args.batching)
    io_threads = max(args.workers, 4)
    node = dep.predictor["graph"]["name"]
    from .serving.openapi import wrapper_spec_json

    if args.api_type == "REST":
        http = dep.C.HttpServer(dep.engine, "0.0.0.0", [args.port], io_threads, node, True, wrapper_spec_json())
        http.start()
        servers = [http]
        logger.info("REST microservice running on port %i", http.ports[0])
    else:
        max_msg = int(annotations.get("seldon.io/grpc-max-message-size", 64 << 20))
        grpc = dep.C.GrpcServer(dep.engine, "0.0.0.0", args.port, io_threads, node, max_msg)
        grpc.start()
        servers = [grpc]
        logger.info("GRPC microservice running on port %i", grpc.port)
    if callable(getattr(user_object, "custom_service", None)):
        threading.Thread(target=user_object.custom_service, daemon=True).start()

    from .utils.shutdown import StopSignal

    # the handlers only flip a flag: a lock taken inside a handler (Event.set)
    # deadlocks when a second SIGTERM/SIGINT lands in it
    StopSignal().install().wait()
    for s in servers:
        s.stop()
    if persister is not None:
        persister.push()
        persister.stop()
    dep.close()


if __name__ == "__main__":
    main()
