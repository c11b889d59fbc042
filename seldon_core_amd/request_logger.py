"""Request-logger sink (reference seldon-request-logger/app/app.py).

Receives the engine's CloudEvents ``seldon.message.pair`` POSTs
(csrc/core/msglog.cc; reference PredictionService.java:140-191), splits each
{request, response} pair into one JSON document per row with per-feature
``request_elements`` / ``response_elements`` dicts and a ``dataType``
(tabular / text / image), and prints one line per row to stdout for a log
shipper (fluentd / Elasticsearch in the reference setup).

    python -m seldon_core_amd.request_logger --port 8080
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, TextIO, Tuple

import numpy as np

from .serving.codec import array_to_rest_datadef, extract_request_parts_json


def _elements(X: Any, names: List[str]) -> Optional[List[Dict[str, Any]]]:
    if not isinstance(X, np.ndarray):
        return None
    if X.ndim == 1:
        return [{n: (X[i].decode() if isinstance(X[i], bytes) else X[i].item() if hasattr(X[i], "item") else X[i])
                 for i, n in enumerate(names)}]
    return [{n: [X[r, i].item() if hasattr(X[r, i], "item") else X[r, i]] for i, n in enumerate(names)}
            for r in range(X.shape[0])]


def _row(i: int, msg: Dict, X: np.ndarray, names: List[str]) -> Dict:
    if X.ndim == 2:
        data_type, part = "tabular", X[i:i + 1]
    elif X.ndim > 2:
        data_type, part = "image", X
    else:
        data_type, part = "text", X
    out: Dict[str, Any] = {"data": array_to_rest_datadef("ndarray", part, names)}
    if msg.get("meta"):
        out["meta"] = msg["meta"]
    out["dataType"] = data_type
    return out


def _parts(msg: Optional[Dict]) -> Tuple[Optional[Dict], Any, List[str], Optional[List]]:
    if msg is None:
        return None, None, [], None
    m = {k: v for k, v in msg.items() if k != "date"}
    X, _, datadef, _ = extract_request_parts_json(m)
    names = list((datadef or {}).get("names", []))
    if isinstance(X, np.ndarray) and X.ndim >= 1 and not names:
        width = X.shape[1] if X.ndim >= 2 else X.shape[0]
        names = [f"t:{i}" for i in range(width)]  # positional names when the message carries none
    return m, X, names, _elements(X, names)


def flatten_pair(content: Dict) -> List[Dict]:
    """One document per row of the request/response pair."""
    req, Xq, nq, eq = _parts(content.get("request"))
    res, Xr, nr, er = _parts(content.get("response"))
    docs = []
    if eq is not None and er is not None:
        for i, (a, b) in enumerate(zip(eq, er)):
            d = dict(content, request_elements=a, response_elements=b)
            rq, rs = _row(i, req, Xq, nq), _row(i, res, Xr, nr)
            d["request"] = {"dataType": rq["dataType"], rq["dataType"]: rq}
            d["response"] = {"dataType": rs["dataType"], rs["dataType"]: rs}
            docs.append(d)
    elif eq is not None:
        for i, a in enumerate(eq):
            rq = _row(i, req, Xq, nq)
            docs.append(dict(content, request_elements=a, request={"dataType": rq["dataType"], rq["dataType"]: rq}))
    elif er is not None:
        for i, b in enumerate(er):
            rs = _row(i, res, Xr, nr)
            docs.append(dict(content, response_elements=b, response={"dataType": rs["dataType"], rs["dataType"]: rs}))
    else:
        docs.append(content)
    return docs


class _Handler(BaseHTTPRequestHandler):
    out: TextIO = sys.stdout
    lock = threading.Lock()

    def _handle(self):
        n = int(self.headers.get("Content-Length") or 0)
        try:
            content = json.loads(self.rfile.read(n) or b"{}")
            docs = flatten_pair(content)
            with self.lock:
                for d in docs:
                    self.out.write(json.dumps(d, default=str) + "\n")
                self.out.flush()
            body, code = b"{}", 200
        except Exception as e:  # malformed event: report, keep serving
            body, code = json.dumps({"error": str(e)}).encode(), 400
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    do_POST = _handle
    do_GET = _handle

    def log_message(self, *a):
        pass


def serve(host: str = "0.0.0.0", port: int = 8080, out: TextIO = sys.stdout) -> ThreadingHTTPServer:
    handler = type("Handler", (_Handler,), {"out": out})
    srv = ThreadingHTTPServer((host, port), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-request-logger")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    args = ap.parse_args(argv)
    srv = serve(args.host, args.port)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
