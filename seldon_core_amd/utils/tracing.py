"""Distributed tracing (reference engine/.../tracing/TracingProvider.java:25-40,
python/seldon_core/microservice.py:116-151: Jaeger/OpenTracing).

A dependency-free tracer: spans carry W3C trace-context ids
(``traceparent``), are sampled by ``JAEGER_SAMPLER_PARAM`` / const sampling and
exported as Zipkin v2 JSON (Jaeger accepts it on its Zipkin collector port) to
``JAEGER_COLLECTOR_URL`` / ``ZIPKIN_URL``, or appended to
``SELDON_TRACE_FILE``.  When ``SELDON_ROCTX=1`` every span also opens a
``roctx`` range so ``rocprofv3 --marker-trace`` shows graph structure next to
the HIP kernels.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import logging
import os
import random
import threading
import time
import urllib.request
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

_tracer: Optional["Tracer"] = None


def _rand_hex(nbytes: int) -> str:
    return "%0*x" % (nbytes * 2, random.getrandbits(nbytes * 8))


class _Roctx:
    def __init__(self):
        self.lib = None
        if os.environ.get("SELDON_ROCTX") == "1":
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    self.lib = ctypes.CDLL(name)
                    break
                except OSError:
                    continue

    def push(self, name: str) -> None:
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def pop(self) -> None:
        if self.lib is not None:
            self.lib.roctxRangePop()


class Span:
    def __init__(self, tracer: "Tracer", name: str, trace_id: str, parent_id: Optional[str], tags: Dict[str, str]):
        self.tracer = tracer
        self.name = name
        self.trace_id = trace_id
        self.span_id = _rand_hex(8)
        self.parent_id = parent_id
        self.tags = dict(tags)
        self.start_us = int(time.time() * 1e6)
        self.duration_us = 0

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-01"

    def set_tag(self, k: str, v) -> None:
        self.tags[k] = str(v)

    def finish(self) -> None:
        self.duration_us = int(time.time() * 1e6) - self.start_us
        self.tracer._finished(self)

    def to_zipkin(self) -> Dict:
        d = {"traceId": self.trace_id, "id": self.span_id, "name": self.name, "timestamp": self.start_us,
             "duration": max(1, self.duration_us), "localEndpoint": {"serviceName": self.tracer.service},
             "tags": self.tags}
        if self.parent_id:
            d["parentId"] = self.parent_id
        return d


class Tracer:
    def __init__(self, service: str, sample_rate: float = 1.0, collector: Optional[str] = None,
                 trace_file: Optional[str] = None, extra_tags: Optional[Dict[str, str]] = None):
        self.service = service
        self.sample_rate = sample_rate
        self.collector = collector
        self.trace_file = trace_file
        self.extra_tags = extra_tags or {}
        self._buf: List[Span] = []
        self._lock = threading.Lock()
        self._roctx = _Roctx()
        self.finished: List[Span] = []  # kept for inspection/tests (bounded)

    def start_span(self, name: str, parent: Optional[Span] = None, traceparent: Optional[str] = None,
                   tags: Optional[Dict[str, str]] = None) -> Optional[Span]:
        trace_id, parent_id = None, None
        if parent is not None:
            trace_id, parent_id = parent.trace_id, parent.span_id
        elif traceparent:
            parts = traceparent.split("-")
            if len(parts) == 4:
                trace_id, parent_id = parts[1], parts[2]
        if trace_id is None:
            if random.random() >= self.sample_rate:
                return None
            trace_id = _rand_hex(16)
        t = dict(self.extra_tags)
        t.update(tags or {})
        self._roctx.push(name)
        return Span(self, name, trace_id, parent_id, t)

    @contextlib.contextmanager
    def span(self, name: str, parent: Optional[Span] = None, **tags):
        s = self.start_span(name, parent, tags={k: str(v) for k, v in tags.items()})
        try:
            yield s
        finally:
            if s is not None:
                s.finish()

    def _finished(self, s: Span) -> None:
        self._roctx.pop()
        with self._lock:
            self._buf.append(s)
            self.finished.append(s)
            if len(self.finished) > 10000:
                del self.finished[:5000]
            flush = len(self._buf) >= 64
        if flush:
            self.flush()

    def flush(self) -> None:
        with self._lock:
            spans, self._buf = self._buf, []
        if not spans:
            return
        payload = [s.to_zipkin() for s in spans]
        if self.trace_file:
            with open(self.trace_file, "a") as f:
                for p in payload:
                    f.write(json.dumps(p) + "\n")
        if self.collector:
            try:
                req = urllib.request.Request(self.collector, data=json.dumps(payload).encode(),
                                             headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=2).read()
            except Exception as e:  # never fail a request because tracing is down
                logger.debug("trace export failed: %s", e)


def configure_tracing(service: str) -> Tracer:
    global _tracer
    rate = float(os.environ.get("JAEGER_SAMPLER_PARAM", "1"))
    collector = os.environ.get("JAEGER_COLLECTOR_URL") or os.environ.get("ZIPKIN_URL")
    extra = {}
    for t in filter(None, (x.strip() for x in os.environ.get("JAEGER_EXTRA_TAGS", "").split(","))):
        extra[t] = os.environ.get(t, "")
    _tracer = Tracer(service, rate, collector, os.environ.get("SELDON_TRACE_FILE"), extra)
    return _tracer


def get_tracer() -> Optional[Tracer]:
    return _tracer


class NativeSpanExporter:
    """Drains the native engine's span buffer (per-request root span +
    one span per node method call, csrc/core/engine.cc) and exports it through
    a :class:`Tracer` (Zipkin v2 JSON to the collector / trace file)."""

    def __init__(self, engine, tracer: Tracer, interval_s: float = 0.2):
        self.engine = engine
        self.tracer = tracer
        self.interval_s = interval_s
        self._stop = threading.Event()
        engine.enable_tracing(tracer.sample_rate)
        self._th = threading.Thread(target=self._run, name="span-exporter", daemon=True)
        self._th.start()

    def export_once(self) -> int:
        spans = self.engine.drain_spans()
        if not spans:
            return 0
        for s in spans:
            s["localEndpoint"] = {"serviceName": self.tracer.service}
            s["tags"].update(self.tracer.extra_tags)
        if self.tracer.trace_file:
            with open(self.tracer.trace_file, "a") as f:
                for s in spans:
                    f.write(json.dumps(s) + "\n")
        if self.tracer.collector:
            try:
                req = urllib.request.Request(self.tracer.collector, data=json.dumps(spans).encode(),
                                             headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=2).read()
            except Exception as e:
                logger.debug("trace export failed: %s", e)
        return len(spans)

    def _run(self):
        while not self._stop.wait(self.interval_s):
            self.export_once()

    def close(self):
        self._stop.set()
        self._th.join(timeout=5)
        self.export_once()
