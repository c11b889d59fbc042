"""Method dispatch for Python components (REST / JSON-dict path).

Precedence per method, as in the reference wrapper
(python/seldon_core/seldon_methods.py:17-302):

1. deprecated low-level ``<method>_rest`` hook (called with the raw request),
2. ``<method>_raw`` (skipped if it raises ``SeldonNotImplementedError``),
3. the high-level numpy API via the ``client_*`` helpers, with the response
   packaged by :func:`construct_response_json`.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

import numpy as np

from .codec import construct_response_json, datadef_to_array, extract_request_parts_json
from .errors import SeldonMicroserviceException, SeldonNotImplementedError
from .user_model import (client_aggregate, client_predict, client_route, client_send_feedback,
                         client_transform_input, client_transform_output)

logger = logging.getLogger(__name__)


def _low_level(user_model: Any, name: str, request: Any):
    """Return (handled, result) for the *_rest and *_raw hooks."""
    if hasattr(user_model, f"{name}_rest"):
        logger.warning("%s_rest is deprecated. Please use %s_raw", name, name)
        return True, getattr(user_model, f"{name}_rest")(request)
    if hasattr(user_model, f"{name}_raw"):
        try:
            return True, getattr(user_model, f"{name}_raw")(request)
        except SeldonNotImplementedError:
            pass
    return False, None


def _names(datadef: Optional[Dict]) -> List[str]:
    return list(datadef["names"]) if datadef and "names" in datadef else []


def predict(user_model: Any, request: Dict) -> Dict:
    handled, out = _low_level(user_model, "predict", request)
    if handled:
        return out
    features, meta, datadef, _ = extract_request_parts_json(request)
    resp = client_predict(user_model, features, _names(datadef), meta=meta)
    return construct_response_json(user_model, False, request, resp)


def transform_input(user_model: Any, request: Dict) -> Dict:
    handled, out = _low_level(user_model, "transform_input", request)
    if handled:
        return out
    features, meta, datadef, _ = extract_request_parts_json(request)
    resp = client_transform_input(user_model, features, _names(datadef), meta=meta)
    return construct_response_json(user_model, False, request, resp)


def transform_output(user_model: Any, request: Dict) -> Dict:
    handled, out = _low_level(user_model, "transform_output", request)
    if handled:
        return out
    features, meta, datadef, _ = extract_request_parts_json(request)
    resp = client_transform_output(user_model, features, _names(datadef), meta=meta)
    return construct_response_json(user_model, False, request, resp)


def route(user_model: Any, request: Dict) -> Dict:
    handled, out = _low_level(user_model, "route", request)
    if handled:
        return out
    features, _, datadef, _ = extract_request_parts_json(request)
    branch = client_route(user_model, features, _names(datadef))
    if not isinstance(branch, (int, np.integer)) or isinstance(branch, bool):
        raise SeldonMicroserviceException("Routing response must be int but got " + str(branch))
    return construct_response_json(user_model, False, request, np.array([[int(branch)]]))


def aggregate(user_model: Any, request: Dict) -> Dict:
    handled, out = _low_level(user_model, "aggregate", request)
    if handled:
        return out
    if not isinstance(request, dict) or not isinstance(request.get("seldonMessages"), list):
        raise SeldonMicroserviceException(f"Invalid request data type: {request}")
    features_list, names_list = [], []
    for msg in request["seldonMessages"]:
        features, _, datadef, _ = extract_request_parts_json(msg)
        features_list.append(features)
        names_list.append(_names(datadef))
    resp = client_aggregate(user_model, features_list, names_list)
    return construct_response_json(user_model, False, request["seldonMessages"][0], resp)


def send_feedback(user_model: Any, request: Dict, predictive_unit_id: str) -> Dict:
    handled, out = _low_level(user_model, "send_feedback", request)
    if handled:
        return out if out is not None else {}
    req = request.get("request") or {}
    truth_msg = request.get("truth") or {}
    features = datadef_to_array(req.get("data"))
    truth = datadef_to_array(truth_msg.get("data"))
    reward = float(request.get("reward", 0.0))
    routing = ((request.get("response") or {}).get("meta") or {}).get("routing", {}).get(predictive_unit_id)
    if routing is not None:
        routing = int(routing)
    resp = client_send_feedback(user_model, features, _names(req.get("data")), reward, truth, routing)
    resp = np.array([]) if resp is None else np.array(resp)
    return construct_response_json(user_model, False, req, resp)
