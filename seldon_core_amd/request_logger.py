"""Request-logger sink (reference seldon-request-logger/app/app.py).

Receives the engine's CloudEvents ``seldon.message.pair`` POSTs
(csrc/core/msglog.cc; reference PredictionService.java:140-191), splits each
{request, response} pair into one JSON document per row with per-feature
``request_elements`` / ``response_elements`` dicts and a ``dataType``
(tabular / text / image), and prints one line per row to stdout for a log
shipper (fluentd / Elasticsearch in the reference setup).

With ``--kafka host:port --kafka-topic T`` every pair is also published as a
``RequestResponse`` proto to the legacy prediction stream (the
reference reader is kafka/tests/src/read_predictions.py), batched off the
request thread by :class:`KafkaSink`.

    python -m seldon_core_amd.request_logger --port 8080 [--kafka localhost:9093 --kafka-topic predictions]
"""
from __future__ import annotations

import argparse
import json
import logging
import queue
import sys
import threading
import time
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


logger = logging.getLogger(__name__)


def pair_to_proto(content: Dict) -> bytes:
    """CloudEvents pair content -> serialized seldon.protos.RequestResponse."""
    from google.protobuf import json_format

    from .proto import prediction_pb2

    m = prediction_pb2.RequestResponse()
    for k in ("request", "response"):
        if isinstance(content.get(k), dict):
            json_format.ParseDict(content[k], getattr(m, k), ignore_unknown_fields=True)
    return m.SerializeToString()


class KafkaSink:
    """Publishes pairs to a topic from one background thread.

    Records queued while a produce is in flight go out together as one
    RecordBatch (``linger_s`` bounds how long the first one waits)."""

    def __init__(self, bootstrap: str, topic: str, linger_s: float = 0.02, max_batch: int = 500, producer=None):
        from .utils.kafka import KafkaProducer

        self.topic, self.linger_s, self.max_batch = topic, linger_s, max_batch
        self.producer = producer or KafkaProducer(bootstrap, client_id="seldon-request-logger")
        self.q: "queue.Queue" = queue.Queue()
        self.sent = self.dropped = 0
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def publish(self, content: Dict) -> None:
        puid = ((content.get("response") or {}).get("meta") or {}).get("puid") or content.get("id")
        self.q.put(((puid or "").encode() or None, pair_to_proto(content)))

    def _run(self) -> None:
        while True:
            first = self.q.get()
            if first is None:
                return
            batch, stop = [first], False
            deadline = time.monotonic() + self.linger_s
            while len(batch) < self.max_batch:
                try:
                    item = self.q.get(timeout=max(0.0, deadline - time.monotonic()))
                except queue.Empty:
                    break
                if item is None:
                    stop = True
                    break
                batch.append(item)
            try:
                self.producer.send_batch(self.topic, [(k, v, [("content-type", b"application/x-protobuf")])
                                                      for k, v in batch])
                self.sent += len(batch)
            except Exception as e:  # broker down: drop, keep the HTTP sink alive
                self.dropped += len(batch)
                logger.warning("kafka publish of %d pairs failed: %s", len(batch), e)
            if stop:
                return

    def close(self, timeout: float = 5.0) -> None:
        self.q.put(None)
        self._t.join(timeout)
        self.producer.close()


class _Handler(BaseHTTPRequestHandler):
    out: TextIO = sys.stdout
    lock = threading.Lock()
    sink: Optional[KafkaSink] = None

    def _handle(self):
        n = int(self.headers.get("Content-Length") or 0)
        try:
            content = json.loads(self.rfile.read(n) or b"{}")
            docs = flatten_pair(content)
            with self.lock:
                for d in docs:
                    self.out.write(json.dumps(d, default=str) + "\n")
                self.out.flush()
            if self.sink is not None:
                self.sink.publish(content)
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


def serve(host: str = "0.0.0.0", port: int = 8080, out: TextIO = sys.stdout,
          sink: Optional[KafkaSink] = None) -> ThreadingHTTPServer:
    handler = type("Handler", (_Handler,), {"out": out, "sink": sink})
    srv = ThreadingHTTPServer((host, port), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="seldon-amd-request-logger")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--kafka", default=None, help="also publish RequestResponse protos to this broker")
    ap.add_argument("--kafka-topic", default="predictions")
    args = ap.parse_args(argv)
    sink = KafkaSink(args.kafka, args.kafka_topic) if args.kafka else None
    srv = serve(args.host, args.port, sink=sink)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
