"""The duck-typed component interface and the ``client_*`` call helpers.

Same contract as the reference's ``SeldonComponent`` (python/seldon_core/
user_model.py:18-361): every method is optional; the helpers decide what a
missing method means (identity transforms, ``t:i`` class names, no tags...).
Existing user classes run unchanged.

One deliberate fix: ``send_feedback`` is called with
``reward``/``truth``/``routing`` as keywords when the user's signature names
them, so both the documented ``(features, names, reward, truth, routing)``
order and the bundled routers' ``(features, names, routing, reward, truth)``
order work.
"""
from __future__ import annotations

import inspect
import json
import logging
from typing import Any, Dict, Iterable, List, Optional, Union

import numpy as np

from .errors import SeldonMicroserviceException, SeldonNotImplementedError
from .metrics import validate_metrics

logger = logging.getLogger(__name__)

Payload = Union[np.ndarray, List, str, bytes, Dict]


class SeldonComponent:
    """Base class documenting the optional component API."""

    def __init__(self, **kwargs):
        pass

    def tags(self) -> Dict:
        raise SeldonNotImplementedError("tags is not implemented")

    def class_names(self) -> Iterable[str]:
        raise SeldonNotImplementedError("class_names is not implemented")

    def load(self):
        pass

    def predict(self, X, names: Iterable[str], meta: Dict = None) -> Payload:
        raise SeldonNotImplementedError("predict is not implemented")

    def predict_raw(self, msg):
        raise SeldonNotImplementedError("predict_raw is not implemented")

    def send_feedback_raw(self, feedback):
        raise SeldonNotImplementedError("send_feedback_raw is not implemented")

    def transform_input(self, X, names: Iterable[str], meta: Dict = None) -> Payload:
        raise SeldonNotImplementedError("transform_input is not implemented")

    def transform_input_raw(self, msg):
        raise SeldonNotImplementedError("transform_input_raw is not implemented")

    def transform_output(self, X, names: Iterable[str], meta: Dict = None) -> Payload:
        raise SeldonNotImplementedError("transform_output is not implemented")

    def transform_output_raw(self, msg):
        raise SeldonNotImplementedError("transform_output_raw is not implemented")

    def metrics(self) -> List[Dict]:
        raise SeldonNotImplementedError("metrics is not implemented")

    def feature_names(self) -> Iterable[str]:
        raise SeldonNotImplementedError("feature_names is not implemented")

    def send_feedback(self, features, feature_names, reward, truth, routing=None):
        raise SeldonNotImplementedError("send_feedback is not implemented")

    def route(self, features, feature_names) -> int:
        raise SeldonNotImplementedError("route is not implemented")

    def route_raw(self, msg):
        raise SeldonNotImplementedError("route_raw is not implemented")

    def aggregate(self, features_list: List, feature_names_list: List) -> Payload:
        raise SeldonNotImplementedError("aggregate is not implemented")

    def aggregate_raw(self, msgs):
        raise SeldonNotImplementedError("aggregate_raw is not implemented")


def client_custom_tags(user_model: Any) -> Dict:
    if hasattr(user_model, "tags"):
        try:
            return user_model.tags()
        except SeldonNotImplementedError:
            pass
    return {}


def client_class_names(user_model: Any, predictions: np.ndarray) -> Iterable[str]:
    if len(predictions.shape) <= 1:
        return []
    if hasattr(user_model, "class_names"):
        attr = getattr(user_model, "class_names")
        if inspect.ismethod(attr):
            try:
                return user_model.class_names()
            except SeldonNotImplementedError:
                pass
        else:
            return attr  # deprecated attribute form
    return [f"t:{i}" for i in range(predictions.shape[1])]


def _call_with_meta(fn, features, names, kwargs):
    try:
        return fn(features, names, **kwargs)
    except TypeError:
        return fn(features, names)


def client_predict(user_model: Any, features, feature_names: Iterable[str], **kwargs) -> Payload:
    if hasattr(user_model, "predict"):
        try:
            return _call_with_meta(user_model.predict, features, feature_names, kwargs)
        except SeldonNotImplementedError:
            pass
    return []


def client_transform_input(user_model: Any, features, feature_names: Iterable[str], **kwargs) -> Payload:
    if hasattr(user_model, "transform_input"):
        try:
            return _call_with_meta(user_model.transform_input, features, feature_names, kwargs)
        except SeldonNotImplementedError:
            pass
    return features


def client_transform_output(user_model: Any, features, feature_names: Iterable[str], **kwargs) -> Payload:
    if hasattr(user_model, "transform_output"):
        try:
            return _call_with_meta(user_model.transform_output, features, feature_names, kwargs)
        except SeldonNotImplementedError:
            pass
    return features


def client_custom_metrics(user_model: Any) -> List[Dict]:
    if hasattr(user_model, "metrics"):
        try:
            metrics = user_model.metrics()
        except SeldonNotImplementedError:
            return []
        if not validate_metrics(metrics):
            raise SeldonMicroserviceException("Bad metric created during request: " + json.dumps(metrics, default=str),
                                              reason="MICROSERVICE_BAD_METRIC")
        return metrics
    return []


def client_feature_names(user_model: Any, original: Iterable[str]) -> Iterable[str]:
    if hasattr(user_model, "feature_names"):
        try:
            return user_model.feature_names()
        except SeldonNotImplementedError:
            pass
    return original


def client_send_feedback(user_model: Any, features, feature_names: Iterable[str], reward: float, truth,
                         routing: Optional[int]) -> Optional[Payload]:
    if not hasattr(user_model, "send_feedback"):
        return None
    fn = user_model.send_feedback
    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        params = {}
    try:
        if "reward" in params and "truth" in params:
            kw = {"reward": reward, "truth": truth}
            if "routing" in params:
                kw["routing"] = routing
            return fn(features, feature_names, **kw)
        return fn(features, feature_names, reward, truth, routing=routing)
    except SeldonNotImplementedError:
        return None


def client_route(user_model: Any, features, feature_names: Iterable[str]) -> int:
    if hasattr(user_model, "route"):
        return user_model.route(features, feature_names)
    raise SeldonNotImplementedError("Route not defined")


def client_aggregate(user_model: Any, features_list: List, feature_names_list: List) -> Payload:
    if hasattr(user_model, "aggregate"):
        return user_model.aggregate(features_list, feature_names_list)
    raise SeldonNotImplementedError("Aggregate not defined")
