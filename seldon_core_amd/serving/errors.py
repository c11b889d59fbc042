"""Error types of the component API.

Behaviour mirrors the reference wrapper (python/seldon_core/flask_utils.py:67-82,
python/seldon_core/user_model.py:12-16): a bad request from a component is a
400 with body ``{"status": {"status": 1, "info": msg, "code": -1, "reason": ...}}``.
"""
from __future__ import annotations

from typing import Any, Dict, Optional


class SeldonMicroserviceException(Exception):
    status_code = 400

    def __init__(self, message: str, status_code: Optional[int] = None, payload: Optional[Dict[str, Any]] = None,
                 reason: str = "MICROSERVICE_BAD_DATA"):
        super().__init__(message)
        self.message = message
        if status_code is not None:
            self.status_code = status_code
        self.payload = payload
        self.reason = reason

    def to_dict(self) -> Dict[str, Any]:
        body = dict(self.payload or {})
        body["status"] = {"status": 1, "info": self.message, "code": -1, "reason": self.reason}
        return body


class SeldonNotImplementedError(SeldonMicroserviceException):
    """Raised by the optional methods of :class:`SeldonComponent`."""

    status_code = 400

    def __init__(self, message: str):
        super().__init__(message)


class EngineError(RuntimeError):
    """A native-engine error (``Status{code 20x, reason, info}``)."""

    def __init__(self, http_status: int, body: Dict[str, Any]):
        self.http_status = http_status
        self.body = body
        super().__init__(f"{http_status}: {body}")
