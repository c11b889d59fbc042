"""Bridge between the native executor and a Python component.

The engine calls ``transform_input / transform_output / route / aggregate /
send_feedback`` with SeldonMessage JSON text (exactly what the reference engine
POSTs to a microservice, engine/.../InternalPredictionService.java:186-350) and
gets SeldonMessage JSON text back.  A MODEL node's transform-input is the
component's ``predict`` (the reference maps MODEL -> ``/predict``,
InternalPredictionService.java:255-256).
"""
from __future__ import annotations

import json
import pickle
import threading
from typing import Any

from . import dispatch
from .codec import dumps


class PythonUnit:
    def __init__(self, user_model: Any, unit_type: str = "MODEL", name: str = "", lock: bool = True):
        self.user_model = user_model
        self.unit_type = unit_type or "MODEL"
        self.name = name
        # One request at a time per component (the reference runs one Flask
        # worker per process unless --workers is set).
        self._lock = threading.Lock() if lock else None

    def _run(self, fn, *args):
        if self._lock is None:
            return fn(*args)
        with self._lock:
            return fn(*args)

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

    def ready(self) -> bool:
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
