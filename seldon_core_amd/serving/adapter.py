"""Bridge between the native executor and a Python component.

The native unit (csrc/bindings/py_unit.h) calls this adapter two ways:

* ``call_dense(method, X, names, meta, kind)`` -- the fast path for numeric
  DefaultData payloads when the component has no low-level hook for the
  method: ``X`` is a numpy view over the request's fp64 values, and a numeric
  result goes back as an array (the native side rebuilds the message with the
  request's data kind, as the reference's ``construct_response_json`` does,
  python/seldon_core/utils.py:306-407).  Any other result is returned as the
  full response JSON text.
* ``transform_input / transform_output / route / aggregate / send_feedback /
  predict`` with SeldonMessage JSON text -- exactly what the reference engine
  POSTs to a microservice (engine/.../InternalPredictionService.java:186-350)
  -- for raw hooks, strData / binData / jsonData and the list / feedback
  methods.  A MODEL node's transform-input is the component's ``predict``
  (InternalPredictionService.java:255-256).

``start_pool(n)`` starts ``n`` worker processes (the reference's gunicorn
``--workers``, python/seldon_core/microservice.py:153-174): fresh Python
interpreters (``python -m seldon_core_amd.serving.pyworker``), each holding a
copy of the component, fed binary frames over a Unix socketpair.
"""
from __future__ import annotations

import inspect
import json
import logging
import pickle
import socket
import struct
import subprocess
import sys
import threading
from typing import Any, List, Optional

import numpy as np

from . import dispatch
from .codec import construct_response_json, dumps
from .errors import SeldonMicroserviceException, SeldonNotImplementedError, component_error_reply
from .user_model import (SeldonComponent, client_class_names, client_custom_metrics, client_custom_tags,
                         client_predict, client_route, client_transform_input, client_transform_output)

logger = logging.getLogger(__name__)

DENSE_METHODS = ("predict", "transform_input", "transform_output", "route")
FRAME = struct.Struct("<IIII8qQQ")  # PoolFrame in py_unit.h
MAGIC = 0x57414353
OP_INIT = 100


def _has_hook(obj: Any, name: str) -> bool:
    """A user-defined low-level hook (``*_rest`` / ``*_raw``); SeldonComponent's
    stubs that only raise SeldonNotImplementedError do not count."""
    if hasattr(obj, f"{name}_rest"):
        return True
    raw = getattr(type(obj), f"{name}_raw", None)
    if raw is None:
        return hasattr(obj, f"{name}_raw")  # instance attribute
    return raw is not getattr(SeldonComponent, f"{name}_raw", None)


def _dense_reply(out: Any):
    if not isinstance(out, dict) or not isinstance(out.get("data"), dict):
        return None
    data = out["data"]
    for kind in ("tensor", "tftensor", "ndarray"):
        v = data.get(kind)
        if isinstance(v, np.ndarray) and v.dtype.kind in "iuf" and v.ndim >= 1:
            meta = out.get("meta")
            return (np.ascontiguousarray(v, dtype=np.float64), [str(n) for n in data.get("names") or []], kind,
                    json.dumps(meta, default=_json_default) if meta else None)
    return None


class PythonUnit:
    def __init__(self, user_model: Any, unit_type: str = "MODEL", name: str = "", lock: bool = True):
        self.user_model = user_model
        self.unit_type = unit_type or "MODEL"
        self.name = name
        # The native unit runs one call at a time on its own thread; the lock
        # only serialises direct Python callers (tests, tools) with it.
        self._lock = threading.Lock() if lock else None
        self._procs: List[subprocess.Popen] = []

    def _run(self, fn, *args):
        if self._lock is None:
            return fn(*args)
        with self._lock:
            return fn(*args)

    # ------------------------------------------------------------ dense path
    def dense_methods(self) -> List[str]:
        return [m for m in DENSE_METHODS if not _has_hook(self.user_model, m)]

    def call_dense(self, method: str, X: np.ndarray, names: List[str], meta: Optional[str], kind: str = "tensor"):
        """-> (0, float64 array, class names, meta-for-all json|None, meta-for-first json|None)
        or (1, response json text)."""
        return self._run(self._call_dense, method, X, names, meta, kind)

    def _meta_arity(self, method: str) -> Optional[bool]:
        """Does the user's method take ``meta``?  (None: unknown -> the generic
        client_* helper, which retries without meta on TypeError.)"""
        cache = self.__dict__.setdefault("_arity", {})
        if method not in cache:
            fn = getattr(self.user_model, method, None)
            try:
                ps = inspect.signature(fn).parameters.values() if fn is not None else ()
                cache[method] = any(p.name == "meta" or p.kind == p.VAR_KEYWORD for p in ps)
            except (TypeError, ValueError):
                cache[method] = None
        return cache[method]

    def _call_dense(self, method, X, names, meta, kind):
        m = self.user_model
        takes_meta = self._meta_arity(method)
        meta_d = json.loads(meta) if takes_meta is not False and meta and meta != "null" else None
        if method == "route":
            branch = client_route(m, X, names)
            if not isinstance(branch, (int, np.integer)) or isinstance(branch, bool):
                raise SeldonMicroserviceException("Routing response must be int but got " + str(branch))
            resp: Any = np.array([[int(branch)]])
        elif takes_meta is False and callable(getattr(m, method, None)):
            try:  # the common plain signature: no TypeError round trip per call
                resp = getattr(m, method)(X, names)
            except SeldonNotImplementedError:
                resp = X if method != "predict" else []
        elif method == "predict":
            resp = client_predict(m, X, names, meta=meta_d)
        elif method == "transform_input":
            resp = client_transform_input(m, X, names, meta=meta_d)
        elif method == "transform_output":
            resp = client_transform_output(m, X, names, meta=meta_d)
        else:
            raise ValueError(method)
        arr = resp if isinstance(resp, np.ndarray) else (np.asarray(resp) if isinstance(resp, list) else None)
        if arr is not None and arr.dtype.kind in "iuf" and arr.ndim >= 1:
            y = np.ascontiguousarray(arr, dtype=np.float64)
            cn = [str(c) for c in client_class_names(m, arr)]
            tags = client_custom_tags(m)
            metrics = client_custom_metrics(m)
            meta_all = json.dumps({"tags": tags}, default=_json_default) if tags else None
            meta_first = (json.dumps({"tags": tags or {}, "metrics": metrics}, default=_json_default)
                          if metrics else None)
            return 0, y, cn, meta_all, meta_first
        # anything else (strings, dicts, bytes, object arrays): the reference's
        # full response construction
        request = {"data": {kind: {}}, "meta": meta_d or {}}
        return 1, dumps(construct_response_json(m, False, request, resp))

    # ------------------------------------------------------------ JSON path
    def call_json(self, method: str, text: str, node: str):
        """The native unit's entry to the JSON path: the method's JSON reply,
        or -- when a raw hook put a numeric numpy array in its reply's
        ``data`` (``tensor`` / ``tftensor`` / ``ndarray``) -- the tuple
        ``(float64 array, names, kind, meta json | None)``, which the native
        side turns into a dense message without a JSON round trip (an image
        transformer's [1, 3, 224, 224] reply is 0.8 MB of base64 otherwise)."""
        if method in ("predict", "transform_input", "transform_output"):
            out = self._run(getattr(dispatch, method), self.user_model, json.loads(text))
            d = _dense_reply(out)
            return d if d is not None else dumps(out)
        return getattr(self, method)(text, node)

    def predict(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.predict, self.user_model, json.loads(text)))

    def transform_input(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.transform_input, self.user_model, json.loads(text)))

    def transform_output(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.transform_output, self.user_model, json.loads(text)))

    def route(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.route, self.user_model, json.loads(text)))

    def aggregate(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.aggregate, self.user_model, json.loads(text)))

    def send_feedback(self, text: str, node: str) -> str:
        return dumps(self._run(dispatch.send_feedback, self.user_model, json.loads(text), node or self.name))

    def error_reply(self, exc: BaseException):
        """(http status, JSON body, info) for an exception the component's
        error contract covers (its model_error_handler, or a
        SeldonMicroserviceException), else None -- see errors.component_error_reply."""
        try:
            return component_error_reply(self.user_model, exc, self.__dict__.setdefault("_err_cache", {}))
        except Exception:  # noqa: BLE001  a broken handler must not take the request path down
            logger.exception("model_error_handler failed for %r", exc)
            return None

    def ready(self) -> bool:
        if self._procs and all(p.poll() is not None for p in self._procs):
            return False
        r = getattr(self.user_model, "ready", True)
        return bool(r() if callable(r) else r)

    # persistence (reference python/seldon_core/persistence.py pickles the user object)
    def snapshot(self) -> bytes:
        st = getattr(self.user_model, "state_dict", None)
        if callable(st):
            return pickle.dumps(("state_dict", st()))
        return pickle.dumps(("object", self.user_model))

    def restore(self, blob: bytes) -> None:
        kind, payload = pickle.loads(blob)
        if kind == "state_dict" and hasattr(self.user_model, "load_state_dict"):
            self.user_model.load_state_dict(payload)
        elif kind == "object":
            self.user_model = payload

    # ------------------------------------------------------------ process pool
    def start_pool(self, n: int, timeout: float = 120.0) -> List[int]:
        """Start ``n`` worker processes; returns the parent-side socket fds
        (ownership passes to the native unit)."""
        import os

        blob = _pickle_component(self.user_model, self.unit_type, self.name)
        # the component's class must import in the worker as it does here
        env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in sys.path if p and os.path.isdir(p)))
        fds = []
        try:
            for _ in range(n):
                parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
                proc = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serving.pyworker", str(child.fileno())],
                                        pass_fds=[child.fileno()], close_fds=True, env=env)
                child.close()
                self._procs.append(proc)
                parent.settimeout(timeout)
                send_frame(parent, OP_INIT, b"", blob)
                code, _, _, _, text = recv_frame(parent)
                if code != 0:
                    raise RuntimeError(f"python worker failed to start: {text.decode(errors='replace')}")
                parent.settimeout(None)
                fds.append(parent.detach())
        except BaseException:
            for fd in fds:
                os.close(fd)
            self.stop_pool()
            raise
        return fds

    def stop_pool(self, timeout: float = 10.0) -> None:
        for p in self._procs:
            try:
                p.wait(timeout=timeout)  # the native unit's shutdown closes the sockets -> EOF -> exit
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        self._procs = []

    @property
    def worker_pids(self) -> List[int]:
        return [p.pid for p in self._procs]


def _json_default(o):
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(type(o))


def _pickle_component(obj: Any, unit_type: str, name: str) -> bytes:
    payload = {"obj": obj, "unit_type": unit_type, "name": name}
    try:
        import cloudpickle  # classes defined in __main__ / test modules

        return cloudpickle.dumps(payload)
    except ImportError:
        return pickle.dumps(payload)


# ------------------------------------------------------------ frames
def send_frame(sock: socket.socket, op: int, x: bytes, text: bytes, shape=(), flags: int = 0) -> None:
    shp = list(shape) + [0] * (8 - len(shape))
    hdr = FRAME.pack(MAGIC, op, len(shape), flags, *shp, len(x), len(text))
    sock.sendall(hdr + bytes(x) + text if len(x) + len(text) < 65536 else hdr)
    if len(x) + len(text) >= 65536:
        if len(x):
            sock.sendall(x)
        if len(text):
            sock.sendall(text)


def _recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        r = sock.recv_into(view[got:], n - got)
        if r == 0:
            raise EOFError("socket closed")
        got += r
    return buf


def recv_frame(sock: socket.socket):
    """-> (op, flags, shape tuple, x bytearray, text bytes)."""
    hdr = _recv_exact(sock, FRAME.size)
    f = FRAME.unpack(bytes(hdr))
    if f[0] != MAGIC:
        raise ValueError("bad frame magic")
    op, ndim, flags = f[1], f[2], f[3]
    shape = tuple(f[4:4 + ndim])
    x_bytes, t_bytes = f[12], f[13]
    x = _recv_exact(sock, x_bytes) if x_bytes else bytearray()
    text = bytes(_recv_exact(sock, t_bytes)) if t_bytes else b""
    return op, flags, shape, x, text
