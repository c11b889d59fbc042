"""Dense networks -> native fused-MLP row models (csrc/kernels/mlp.hip).

Converters:
* sklearn ``MLPClassifier`` / ``MLPRegressor`` (``coefs_``, ``intercepts_``,
  ``activation``, ``out_activation_``) -- what SKLearnServer would run with
  ``predict_proba`` / ``predict`` (servers/sklearnserver/SKLearnServer.py:32-42),
* torch ``nn.Sequential`` of ``Linear`` + ``ReLU``/``Sigmoid``/``Tanh``/``Softmax``,
* plain Keras-style lists ``[(W [in, out], b, "relu"), ...]``.

Numerics: fp32 weights/activations with exact fp32 MFMA products (the
precision Keras / torch / sklearn-float32 compute in); sklearn fits in fp64,
so its outputs agree to ~1e-6 relative rather than bit-for-bit.
"""
from __future__ import annotations

from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np

ACTS = {"identity": 0, "linear": 0, None: 0, "relu": 1, "logistic": 2, "sigmoid": 2, "tanh": 3}
OUT_PLAIN, OUT_SOFTMAX, OUT_BINARY = 0, 1, 2


def layer(W_out_in, b, act="identity") -> dict:
    W = np.ascontiguousarray(W_out_in, dtype=np.float32)
    return {"W": W, "b": np.ascontiguousarray(b, dtype=np.float32).reshape(-1), "act": ACTS[act]}


def mlp_row_model(layers: Sequence[dict], out_mode: int = OUT_PLAIN, class_names: Optional[List[str]] = None,
                  precision: str = "fp32"):
    """Native dense network.  ``precision="bf16"`` is an explicit per-model
    opt-in: bf16 operands with fp32 accumulation on v_mfma_f32_16x16x32_bf16
    (expect ~1e-2 relative error on the logits vs float32; tests/test_mlp.py
    states the tolerance), the default keeps exact fp32 products."""
    from .._native import native

    m = native().mlp_model(list(layers), out_mode, precision)
    if class_names:
        m.set_class_names([str(c) for c in class_names])
    return m


def from_sklearn_mlp(est: Any, method: str = "predict_proba"):
    """Row model for a fitted sklearn MLPClassifier / MLPRegressor, or None."""
    try:
        from sklearn.neural_network import MLPClassifier, MLPRegressor
    except ImportError:  # pragma: no cover
        return None
    if not isinstance(est, (MLPClassifier, MLPRegressor)):
        return None
    hidden = ACTS[est.activation]
    n = len(est.coefs_)
    layers = []
    for i, (W, b) in enumerate(zip(est.coefs_, est.intercepts_)):
        last = i == n - 1
        act = hidden if not last else (ACTS["logistic"] if est.out_activation_ == "logistic" else 0)
        layers.append({"W": np.ascontiguousarray(np.asarray(W).T, dtype=np.float32),
                       "b": np.asarray(b, dtype=np.float32), "act": act})
    if isinstance(est, MLPClassifier):
        if method != "predict_proba":
            return None
        if est.out_activation_ == "softmax":
            return mlp_row_model(layers, OUT_SOFTMAX, list(est.classes_))
        if est.out_activation_ == "logistic" and layers[-1]["W"].shape[0] == 1:
            return mlp_row_model(layers, OUT_BINARY, list(est.classes_))
        return None  # multilabel logistic: independent sigmoids (plain)
    m = mlp_row_model(layers, OUT_PLAIN)
    if layers[-1]["W"].shape[0] == 1:
        m.flat_output = True  # MLPRegressor.predict returns a 1-D array
    return m


def from_torch(module: Any):
    """Row model for a torch ``nn.Sequential`` of Linear layers and
    element-wise activations (final Softmax -> row softmax), or None."""
    try:
        import torch.nn as nn
    except ImportError:  # pragma: no cover
        return None
    mods = list(module) if isinstance(module, nn.Sequential) else [module]
    layers: List[dict] = []
    out_mode = OUT_PLAIN
    for i, m in enumerate(mods):
        if isinstance(m, nn.Linear):
            b = m.bias.detach().cpu().numpy() if m.bias is not None else np.zeros(m.out_features)
            layers.append({"W": m.weight.detach().cpu().float().numpy(), "b": b.astype(np.float32), "act": 0})
        elif isinstance(m, (nn.ReLU, nn.Sigmoid, nn.Tanh)) and layers and layers[-1]["act"] == 0:
            layers[-1]["act"] = {nn.ReLU: 1, nn.Sigmoid: 2, nn.Tanh: 3}[type(m)]
        elif isinstance(m, nn.Softmax) and i == len(mods) - 1 and layers and layers[-1]["act"] == 0:
            out_mode = OUT_SOFTMAX
        elif isinstance(m, (nn.Identity, nn.Dropout)):
            continue
        else:
            return None
    return mlp_row_model(layers, out_mode) if layers else None


def from_keras_style(spec: Iterable[Tuple[Any, Any, str]], softmax: bool = False):
    """``[(W [in, out], b, act), ...]`` (Keras Dense kernel layout)."""
    layers = [layer(np.asarray(W).T, b, act) for W, b, act in spec]
    return mlp_row_model(layers, OUT_SOFTMAX if softmax else OUT_PLAIN)


def random_dense_stack(dims: Sequence[int], acts: Sequence[str], seed: int = 0) -> List[dict]:
    """Glorot-uniform random layers (synthetic weights for benchmarks/tests)."""
    rng = np.random.default_rng(seed)
    out = []
    for (k, n), a in zip(zip(dims[:-1], dims[1:]), acts):
        lim = np.sqrt(6.0 / (k + n))
        out.append(layer(rng.uniform(-lim, lim, size=(n, k)), rng.uniform(-0.1, 0.1, size=n), a))
    return out
