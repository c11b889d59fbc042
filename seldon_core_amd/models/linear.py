"""Linear / logistic model import (scikit-learn -> GPU ``linear_f64`` kernel).

The reference SKLearnServer (servers/sklearnserver/sklearnserver/
SKLearnServer.py:32-42) calls ``predict_proba`` (default) or ``predict`` on a
joblib-loaded estimator per request on the CPU.  For linear estimators the
parameters are pulled out once and the per-request math runs in
csrc/kernels/linear.hip (fp64, bit-compatible with sklearn up to summation
order).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

# activations (csrc/kernels/kernels.h LinearAct)
ACT_IDENTITY, ACT_SOFTMAX, ACT_BINARY_LOGISTIC, ACT_OVR, ACT_SIGMOID = range(5)


@dataclass
class LinearSpec:
    W: np.ndarray  # [C, K]
    b: np.ndarray  # [C]
    act: int
    class_names: Optional[List[str]] = None
    flat_output: bool = False

    def predict(self, X: np.ndarray) -> np.ndarray:
        z = np.asarray(X, dtype=np.float64) @ self.W.T + self.b
        if self.act == ACT_SOFTMAX:
            e = np.exp(z - z.max(axis=1, keepdims=True))
            out = e / e.sum(axis=1, keepdims=True)
        elif self.act == ACT_BINARY_LOGISTIC:
            p = 1.0 / (1.0 + np.exp(-z[:, 0]))
            out = np.stack([1 - p, p], axis=1)
        elif self.act == ACT_OVR:
            s = 1.0 / (1.0 + np.exp(-z))
            out = s / s.sum(axis=1, keepdims=True)
        elif self.act == ACT_SIGMOID:
            out = 1.0 / (1.0 + np.exp(-z))
        else:
            out = z
        return out[:, 0] if self.flat_output else out


def from_sklearn_linear(est, method: str = "predict_proba") -> Optional[LinearSpec]:
    """LogisticRegression (predict_proba) and linear regressors (predict)."""
    from sklearn.base import is_classifier
    from sklearn.linear_model import LogisticRegression

    if not hasattr(est, "coef_") or not hasattr(est, "intercept_"):
        return None
    coef = np.atleast_2d(np.asarray(est.coef_, dtype=np.float64))
    inter = np.atleast_1d(np.asarray(est.intercept_, dtype=np.float64))
    if inter.size == 1 and coef.shape[0] > 1:
        inter = np.repeat(inter, coef.shape[0])
    if is_classifier(est):
        if method != "predict_proba" or not isinstance(est, LogisticRegression):
            return None
        names = None  # SKLearnServer defines no class_names -> the wrapper reports t:0..t:C-1
        if coef.shape[0] == 1:
            return LinearSpec(coef, inter, ACT_BINARY_LOGISTIC, names)
        multi = getattr(est, "multi_class", "auto")
        ovr = multi == "ovr" or (multi in ("auto", "deprecated") and est.solver == "liblinear")
        return LinearSpec(coef, inter, ACT_OVR if ovr else ACT_SOFTMAX, names)
    flat = np.asarray(est.coef_).ndim == 1
    return LinearSpec(coef, inter, ACT_IDENTITY, None, flat_output=flat)
