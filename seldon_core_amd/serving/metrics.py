"""Custom-metric helpers for components (reference python/seldon_core/metrics.py:8-89).

A component's ``metrics()`` returns a list of ``{"key", "type", "value"[, "tags"]}``
dicts; the engine turns them into Prometheus counters / gauges / timers tagged
with the model labels (engine CustomMetricsManager semantics).
"""
from __future__ import annotations

from numbers import Number
from typing import Dict, List, Optional

COUNTER = "COUNTER"
GAUGE = "GAUGE"
TIMER = "TIMER"


def _metric(key: str, kind: str, value: float, tags: Optional[Dict[str, str]]) -> Dict:
    m = {"key": key, "type": kind, "value": value}
    if tags:
        m["tags"] = dict(tags)
    return m


def create_counter(key: str, value: float, tags: Optional[Dict[str, str]] = None) -> Dict:
    return _metric(key, COUNTER, value, tags)


def create_gauge(key: str, value: float, tags: Optional[Dict[str, str]] = None) -> Dict:
    return _metric(key, GAUGE, value, tags)


def create_timer(key: str, value: float, tags: Optional[Dict[str, str]] = None) -> Dict:
    """``value`` is in milliseconds."""
    return _metric(key, TIMER, value, tags)


def validate_metrics(metrics: List[Dict]) -> bool:
    if not isinstance(metrics, list):
        return False
    for m in metrics:
        if not isinstance(m, dict):
            return False
        if "key" not in m or "value" not in m or "type" not in m:
            return False
        if m["type"] not in (COUNTER, GAUGE, TIMER):
            return False
        if isinstance(m["value"], bool) or not isinstance(m["value"], Number):
            return False
    return True
