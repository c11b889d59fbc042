"""Model families served natively on the GPU and their importers.

``to_row_model(obj)`` turns a supported model description into a native
``RowModel`` (parameters resident in HBM once ``BatchedUnit`` uploads them):

* :class:`~seldon_core_amd.models.linear.LinearSpec` / sklearn linear estimators
* :class:`~seldon_core_amd.models.trees.TreeEnsemble` / XGBoost JSON /
  sklearn trees, forests, gradient boosting, isolation forest
"""
from __future__ import annotations

from typing import Any, Optional

from .linear import LinearSpec, from_sklearn_linear
from .trees import TreeEnsemble, from_sklearn_trees, from_xgboost_json, synthetic_xgboost

__all__ = ["LinearSpec", "TreeEnsemble", "from_sklearn_linear", "from_sklearn_trees", "from_xgboost_json",
           "synthetic_xgboost", "to_row_model", "iris_logistic_regression"]


def to_row_model(obj: Any, method: str = "predict_proba"):
    """Return a native RowModel for ``obj`` or ``None`` if unsupported."""
    from .._native import native

    C = native()
    spec: Any = obj
    from .mlp import from_sklearn_mlp, from_torch

    for conv in (from_sklearn_mlp, lambda o, m: from_torch(o) if _is_torch_module(o) else None):
        try:
            rm = conv(obj, method)
        except Exception:
            rm = None
        if rm is not None:
            return rm
    if not isinstance(obj, (LinearSpec, TreeEnsemble)):
        try:
            spec = from_sklearn_linear(obj, method)
        except Exception:
            spec = None
        # tree classifiers import as predict_proba; regressors as predict
        if spec is None and (method == "predict_proba" or not _is_classifier(obj)):
            try:
                spec = from_sklearn_trees(obj)
            except (TypeError, AttributeError):
                spec = None
    if spec is None:
        return None
    if isinstance(spec, LinearSpec):
        m = C.linear_model(spec.W, spec.b, int(spec.act))
    else:
        m = C.tree_model(spec.device_spec())
    if spec.class_names:
        m.set_class_names(list(spec.class_names))
    m.flat_output = bool(spec.flat_output)
    return m


def _is_torch_module(obj: Any) -> bool:
    try:
        import torch.nn as nn

        return isinstance(obj, nn.Module)
    except Exception:
        return False


def _is_classifier(obj: Any) -> bool:
    try:
        from sklearn.base import is_classifier

        return bool(is_classifier(obj))
    except Exception:
        return False


def iris_logistic_regression(seed: int = 0):
    """The reference's sklearn iris example model
    (examples/models/sklearn_iris/train_iris.py:9-18): LogisticRegression fit
    on the iris dataset bundled with scikit-learn (no network access needed)."""
    from sklearn.datasets import load_iris
    from sklearn.linear_model import LogisticRegression

    X, y = load_iris(return_X_y=True)
    clf = LogisticRegression(max_iter=1000, random_state=seed)
    clf.fit(X, y)
    return clf
