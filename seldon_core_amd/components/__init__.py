"""Engine-native components: routers and outlier detectors.

``NATIVE_IMPLEMENTATIONS`` maps a graph node's ``implementation`` string to a
component factory (node parameters become constructor kwargs), so specs can
use them without a container image.
"""
from __future__ import annotations

from typing import Callable, Dict

NATIVE_IMPLEMENTATIONS: Dict[str, Callable] = {}


def register(name: str):
    def deco(cls):
        NATIVE_IMPLEMENTATIONS[name] = cls
        return cls

    return deco


from . import routers  # noqa: E402,F401  (registers EPSILON_GREEDY / THOMPSON_SAMPLING)
from . import examples  # noqa: E402,F401  (MEAN_TRANSFORMER, MEAN_CLASSIFIER, IMAGENET_*, ...)
from . import outlier  # noqa: E402,F401  (MAHALANOBIS_OD, ISOLATION_FOREST_OD, VAE_OD, SEQ2SEQ_OD)
