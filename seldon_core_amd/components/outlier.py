"""Outlier detectors: same classes, parameters, predictions,
tags and metrics as the reference components/outlier-detection/*, with the
scoring on the MI355X:

* ``OutlierMahalanobis`` -- mahalanobis/CoreMahalanobis.py:68-151 (online mean /
  covariance, top-k PCA via ``eigh``, Sherman-Morrison inverse updates,
  Mahalanobis score).  On a GPU the state (mean, covariance, clip bounds, n)
  stays in HBM and each request is one single-workgroup kernel launch that
  runs the whole step -- clip, running moments, top-k eigenpairs by one
  wave in LDS (tridiagonalisation, Sturm multisection, twisted-factorisation
  eigenvectors), projections, Sherman-Morrison recurrence, state update (``MahalanobisDevice``, csrc/kernels/mahalanobis.hip); on the
  CPU it is fp64 numpy (the parity oracle).
* ``OutlierIsolationForest`` -- isolation-forest/CoreIsolationForest.py:62-76:
  ``decision_function < threshold``; the forest runs on the tree-ensemble HIP
  kernel (isolation transform: 2^(-mean path / c(n)) - offset).
* ``OutlierVAE`` -- vae/CoreVAE.py:106-141: clip, reservoir sampling, scaling,
  10 MC reconstructions -> row MSE; the whole VAE + MC loop + MSE is one fused
  MFMA kernel launch (csrc/kernels/mlp.hip, ``vae_model``).
* ``OutlierSeq2SeqLSTM`` -- seq2seq-lstm/CoreSeq2SeqLSTM.py:107-174: BiLSTM
  encoder, step-by-step LSTM decoder fed its own outputs, row MSE; on a GPU the
  whole model + T-1 step decode + MSE is one persistent MFMA kernel per batch
  (csrc/kernels/lstm.hip), on the CPU torch eager.
"""
from __future__ import annotations

import copy
import json
import logging
import math
import os
import random
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import register

logger = logging.getLogger(__name__)


def _default_device(device: Optional[int]) -> int:
    if device is not None:
        return int(device)
    try:
        from .._native import gpu_count

        return 0 if gpu_count() > 0 else -1
    except Exception:
        return -1


class _NativeScorer:
    """Runs a native row model on the GPU through a micro-batcher (concurrent
    requests share launches), or its CPU reference path with device -1."""

    def __init__(self, row_model, device: int):
        self.rm = row_model
        self.device = device
        self._unit = None

    def __call__(self, X: np.ndarray) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float64)
        if self.device < 0:
            return self.rm.run_cpu(X)
        if self._unit is None:
            from .._native import native

            self._unit = native().BatchedUnit(self.rm, self.device)
        return self._unit.run(X)

    def close(self):
        if self._unit is not None:
            self._unit.stop()
            self._unit = None


# ------------------------------------------------------------ feedback stats
def _flatten(x) -> list:
    if isinstance(x, (list, tuple, np.ndarray)):
        return [a for i in x for a in _flatten(i)]
    return [x]


def performance(y_true, y_pred, roll_window: int = 100) -> List[float]:
    """[tn, fp, fn, tp, acc, prec, rec, f1, f2] total + rolling (utils.py:106-132)."""
    from sklearn.metrics import (accuracy_score, confusion_matrix, f1_score, fbeta_score, precision_score,
                                 recall_score)

    y_true, y_pred = np.asarray(y_true, int), np.asarray(y_pred, int)
    tn, fp, fn, tp = confusion_matrix(y_true, y_pred, labels=[0, 1]).ravel()

    def scores(t, p):
        return [accuracy_score(t, p), precision_score(t, p, zero_division=0), recall_score(t, p, zero_division=0),
                f1_score(t, p, zero_division=0), fbeta_score(t, p, beta=2, zero_division=0)]

    return [tn, fp, fn, tp, *scores(y_true, y_pred), *scores(y_true[-roll_window:], y_pred[-roll_window:])]


def outlier_stats(y_true, y_pred, roll_window: int = 100) -> List[float]:
    return [np.sum(y_pred[-roll_window:]), np.sum(y_true[-roll_window:]), np.sum(y_pred), np.sum(y_true)]


class _FeedbackMetrics:
    """Labels arrive through send_feedback; metrics lag one prediction."""
    roll_window = 100
    score_key = "score"
    # Online state checkpointed by state_dict() (the reference
    # pickles the whole detector into Redis, persistence.py:21-85).  Model
    # weights and device handles are construction inputs, not state.
    _STATE = ("_predictions", "_labels", "_scores", "metric", "label", "nb_outliers")

    def state_dict(self) -> Dict[str, Any]:
        keys: List[str] = []
        for cls in type(self).__mro__:
            keys += [k for k in cls.__dict__.get("_STATE", ()) if k not in keys]
        return {k: copy.deepcopy(getattr(self, k)) for k in keys if hasattr(self, k)}

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        for k, v in state.items():
            setattr(self, k, copy.deepcopy(v))

    def _init_feedback(self):
        self._predictions: List[int] = []
        self._labels: List[int] = []
        self._scores: List[float] = []
        self.metric = [float("nan")] * 18
        self.label = None

    def _last_scores(self) -> np.ndarray:
        raise NotImplementedError

    def send_feedback(self, X, feature_names, reward, truth, routing=None):
        self._scores = _flatten([self._scores, list(np.asarray(self._last_scores()).ravel())])
        self._predictions = _flatten([self._predictions, list(np.asarray(self.prediction).ravel())])
        self.label = np.asarray(truth).ravel() if truth is not None else np.array([])
        self._labels = _flatten([self._labels, list(self.label)])
        if len(self._labels) == len(self._predictions) and self._labels:
            conv = _flatten([performance(self._labels, self._predictions, self.roll_window),
                             outlier_stats(np.asarray(self._labels), np.asarray(self._predictions), self.roll_window)])
            self.metric = [float(np.asarray(c)) for c in conv]
        return []

    def _feedback_metrics(self, n_obs: int) -> List[Dict[str, Any]]:
        if n_obs <= 1 or not self._predictions:
            pred = err = y_true = float("nan")
        else:
            pred = int(self._predictions[-1])
            err = float(self._scores[-1])
            y_true = int(self.label[0]) if self.label is not None and len(self.label) else float("nan")
        g = lambda k, v: {"type": "GAUGE", "key": k, "value": v}  # noqa: E731
        m = self.metric
        names = ["accuracy_tot", "precision_tot", "recall_tot", "f1_tot", "f2_tot", "accuracy_roll",
                 "precision_roll", "recall_roll", "f1_roll", "f2_roll"]
        out = [g("is_outlier", pred), g(self.score_key, err), g("observation", n_obs - 1),
               g("threshold", self.threshold), g("label", y_true)]
        out += [g(n, m[4 + i]) for i, n in enumerate(names)]
        out += [g("true_negative", m[0]), g("false_positive", m[1]), g("false_negative", m[2]),
                g("true_positive", m[3]), g("nb_outliers_roll", m[14]), g("nb_labels_roll", m[15]),
                g("nb_outliers_tot", m[16]), g("nb_labels_tot", m[17])]
        return out

    def _batch_metrics(self, n_total: int) -> List[Dict[str, Any]]:
        """Core* metrics (batch averages) -- used for multi-row requests, for
        which the reference wrappers raise 'Metrics can only handle single
        observations'."""
        g = lambda k, v: {"type": "GAUGE", "key": k, "value": v}  # noqa: E731
        return [g("is_outlier", float(np.mean(self.prediction))), g(self.score_key, float(np.mean(self._last_scores()))),
                g("nb_outliers", int(self.nb_outliers)), g("fraction_outliers", int(self.nb_outliers) / max(1, n_total)),
                g("observation", n_total), g("threshold", self.threshold)]

    def tags(self):
        try:
            return {"outlier-predictions": self.prediction_meta.tolist()}
        except AttributeError:
            return {}

    def transform_input(self, X, feature_names):
        self.prediction_meta = self._get_preds(np.asarray(X, dtype=float))
        return X

    def predict(self, X, feature_names):
        return self._get_preds(np.asarray(X, dtype=float))


class _Reservoir:
    """Reservoir sampling + scaling statistics (CoreVAE.py:59-77)."""
    _STATE = ("batch", "N", "mu", "sigma", "xmin", "xmax")

    def _init_scaling(self, preprocess: Optional[Dict], reservoir_size: int, n_features: int):
        self.reservoir_size = reservoir_size
        self.batch: List[np.ndarray] = []
        self.N = 0
        pp = dict(preprocess or {})
        self.preprocess = pp.get("method", "standardized")
        self.clip = np.asarray(pp.get("clip", [np.inf] * n_features), dtype=float)
        self.axis = pp.get("axis", 0)
        if self.preprocess == "minmax":
            self.xmin = np.asarray(pp.get("xmin", np.zeros(n_features)), float)
            self.xmax = np.asarray(pp.get("xmax", np.ones(n_features)), float)
            self.min, self.max = float(pp.get("min", 0.0)), float(pp.get("max", 1.0))
        else:
            self.mu = np.asarray(pp.get("mu", np.zeros(n_features)), float)
            self.sigma = np.asarray(pp.get("sigma", np.ones(n_features)), float)

    def reservoir_sampling(self, X, update_stand=False):
        for item in X:
            self.N += 1
            if len(self.batch) < self.reservoir_size:
                self.batch.append(item)
            else:
                s = int(random.random() * self.N)
                if s < self.reservoir_size:
                    self.batch[s] = item
        if update_stand:
            b = np.array(self.batch)
            if self.preprocess == "minmax":
                self.xmin, self.xmax = b.min(axis=self.axis), b.max(axis=self.axis)
            else:
                self.mu, self.sigma = b.mean(axis=self.axis), b.std(axis=self.axis)

    def _scale(self, X):
        if self.preprocess == "minmax":
            return ((X - self.xmin) / (self.xmax - self.xmin)) * (self.max - self.min) + self.min
        return (X - self.mu) / (self.sigma + 1e-10)


# --------------------------------------------------------------- Mahalanobis
@register("MAHALANOBIS_OD")
class OutlierMahalanobis(_FeedbackMetrics):
    score_key = "outlier_score"
    _STATE = ("mean", "C", "n", "clip")
    _EPSILON = 1e-8

    def __init__(self, threshold=25, n_components=3, n_stdev=3, start_clip=50, max_n=-1, device=None,
                 gpu_min_rows: int = 0, n_features: Optional[int] = None):
        self.threshold = threshold
        self.n_components = n_components
        self.max_n = max_n
        self.n_stdev = n_stdev
        self.start_clip = start_clip
        self.clip = None
        self.mean = 0
        self.C = 0
        self.n = 0
        self.nb_outliers = 0
        self.device = _default_device(device)
        self.n_features = int(n_features) if n_features else None
        self._dev = None  # native MahalanobisDevice: state resident in HBM (created at the first request)
        self._init_feedback()

    def _last_scores(self):
        return self.score

    # ------------------------------------------------------------ device path
    def _device_for(self, p: int):
        """The whole _get_preds runs on the GPU through the native micro-batcher
        (csrc/gpu/maha_device.cc): concurrent requests share one
        single-workgroup launch that steps the HBM-resident state through them
        in order (csrc/kernels/mahalanobis.hip: maha_step_segments); p <= 64,
        k <= 16."""
        if self.device < 0 or p > 64 or min(self.n_components, p) > 16:
            return None  # CPU placement: the numpy / scipy-eigh path (the parity oracle)
        if self._dev is not None and self._dev.p == p:
            return self._dev
        return self._make_device(p, self.device)

    def _make_device(self, p: int, device: int):
        from .._native import native

        self._dev = native().MahalanobisDevice(p, min(self.n_components, p), float(self.n_stdev),
                                               float(self.start_clip), float(self.max_n), self._EPSILON, device)
        if self.n:  # state restored / accumulated on the host before the device existed
            self._push_state(p)
        return self._dev

    def row_model(self):
        """Native graph node (MODEL): predictions ``score > threshold`` -- the
        reference's predict() output (CoreMahalanobis.py:148-151) -- served by
        the micro-batcher with no Python per request.  Needs ``n_features``
        (the reference learns p from the first request; a native unit is bound
        before any arrives).  The node shares this object's detector state, so
        state_dict()/load_state_dict() checkpoint it.  Served natively, the
        per-request Python bookkeeping (``n``, ``nb_outliers``, the feedback
        metrics) is not updated -- no Python runs per request;
        state_dict() pulls ``n`` and the state from the device."""
        p = self.n_features
        if not p or p > 64 or min(self.n_components, p) > 16:
            return None
        dev = self._dev if (self._dev is not None and self._dev.p == p) else self._make_device(p, self.device)
        return dev.predict_view(float(self.threshold))

    def _push_state(self, p: int) -> None:
        c_zero = isinstance(self.C, int) and self.C == 0
        mean = np.broadcast_to(np.asarray(self.mean, float), (p,))
        C = np.zeros((p, p)) if c_zero else np.asarray(self.C, float)
        lo, hi = (np.zeros(p), np.zeros(p)) if self.clip is None else (np.asarray(self.clip[0], float),
                                                                        np.asarray(self.clip[1], float))
        st = np.concatenate([mean, C.ravel(), lo, hi, [float(self.n), 1.0 if c_zero else 0.0,
                                                      0.0 if self.clip is None else 1.0]])
        self._dev.set_state(st.tolist())

    def _pull_state(self) -> None:
        if self._dev is None:
            return
        p = self._dev.p
        st = np.asarray(self._dev.state())
        self.mean = st[:p].copy()
        self.C = 0 if st[-2] != 0 else st[p:p + p * p].reshape(p, p).copy()
        self.clip = [st[p + p * p:2 * p + p * p].copy(), st[2 * p + p * p:3 * p + p * p].copy()] if st[-1] else None
        self.n = int(st[-3])

    def state_dict(self):
        self._pull_state()
        return super().state_dict()

    def load_state_dict(self, state):
        super().load_state_dict(state)
        if self._dev is not None:
            self._push_state(self._dev.p)

    def _sm_scores(self, B, proj_cov, x_diff, n):
        """Sherman-Morrison inverse recurrence over the batch rows + quadratic
        forms (CoreMahalanobis.py:118-146) -- host path."""
        nb, k = x_diff.shape
        all_C_inv = np.zeros_like(B)
        c_inv = None
        for i, b in enumerate(B):
            if c_inv is None:
                if abs(np.linalg.det(proj_cov)) > self._EPSILON:
                    c_inv = np.linalg.inv(proj_cov)
                    all_C_inv[i] = c_inv
                    continue
                if n + i == 0:
                    continue
                proj_cov = (n + i - 1.0) / (n + i) * proj_cov + b
                continue
            c_inv = (n + i - 1.0) / float(n + i - 2.0) * all_C_inv[i - 1]
            BC1 = np.matmul(B[i - 1], c_inv)
            all_C_inv[i] = c_inv - 1.0 / (1.0 + np.trace(BC1)) * np.matmul(c_inv, BC1)
        return np.matmul(x_diff[:, None, :], np.matmul(all_C_inv, x_diff[:, :, None])).reshape(nb)

    def _get_preds(self, X):
        X = np.asarray(X, dtype=float)
        if X.ndim == 2 and self._device_for(X.shape[1]) is not None:
            self.score = np.asarray(self._dev.step(X))
            self.n += X.shape[0]
            self.prediction = (self.score > self.threshold).astype(int)
            return self.prediction
        shared = self._dev is not None and X.ndim == 2 and self._dev.p == X.shape[1]
        if not shared:
            return self._get_preds_host(X)
        # A native node (row_model) holds the state: one detector, two entry
        # points.  Pull -> host step -> push runs under the state's lock, so a
        # native step cannot land in between and be overwritten by the push.
        self._dev.lock_state()
        try:
            self._pull_state()
            out = self._get_preds_host(X)
            self._push_state(self._dev.p)
        finally:
            self._dev.unlock_state()
        return out

    def _get_preds_host(self, X):
        """numpy path (CPU placement; the parity oracle of the device kernel)."""
        from scipy.linalg import eigh

        nb, p = X.shape
        k = min(self.n_components, p)
        n = min(self.n, self.max_n) if self.max_n > 0 else self.n
        Xc = np.clip(X, self.clip[0], self.clip[1]) if self.n > self.start_clip else X
        # running mean / covariance over the batch
        steps = np.arange(nb)
        roll = Xc.cumsum(axis=0) / (steps + 1).reshape(nb, 1)
        new_means = self.mean + ((steps + 1.0) / (steps + n + 1.0)).reshape(nb, 1) * (roll - self.mean)
        means_off = np.empty_like(new_means)
        means_off[0] = self.mean
        means_off[1:] = new_means[:-1]
        d = Xc - means_off
        coefs = ((n + steps) / (n + steps + 1.0)).reshape(nb, 1, 1)
        B = coefs * np.matmul(d[:, :, None], d[:, None, :])
        cov = (n - 1.0) / (n + max(1, nb - 1.0)) * self.C + 1.0 / (n + max(1, nb - 1.0)) * B.sum(axis=0)
        # top-k principal subspace
        _, V = eigh(cov, subset_by_index=[p - k, p - 1])
        proj_x, proj_xc, proj_m = X @ V, Xc @ V, means_off @ V
        proj_cov = np.zeros((k, k)) if (isinstance(self.C, int) and self.C == 0) else V.T @ self.C @ V
        dpc = proj_xc - proj_m
        Bp = (1.0 / (n + steps + 1.0)).reshape(nb, 1, 1) * np.matmul(dpc[:, :, None], dpc[:, None, :])
        self.score = self._sm_scores(Bp, proj_cov, proj_x - proj_m, n)
        # state updates
        self.mean = new_means[-1]
        self.C = cov
        std = np.sqrt(np.diag(cov))
        self.n += nb
        if self.n > self.start_clip:
            self.clip = [self.mean - self.n_stdev * std, self.mean + self.n_stdev * std]
        self.prediction = (self.score > self.threshold).astype(int)
        return self.prediction

    def metrics(self):
        self.nb_outliers += int(np.sum(self.prediction))
        if np.asarray(self.score).shape[0] > 1:
            return self._batch_metrics(self.n)
        return self._feedback_metrics(self.n)


# ----------------------------------------------------------- isolation forest
@register("ISOLATION_FOREST_OD")
class OutlierIsolationForest(_FeedbackMetrics):
    score_key = "anomaly_score"
    _STATE = ("N",)

    def __init__(self, threshold=0.0, model=None, model_name="if", load_path="./models/", train_data=None,
                 n_estimators=100, max_samples="auto", contamination="auto", random_state=0, device=None):
        from sklearn.ensemble import IsolationForest

        self.threshold = threshold
        self.N = 0
        self.nb_outliers = 0
        if model is None:
            path = train_data or os.path.join(load_path, model_name + ".npz")
            if not os.path.exists(path):
                raise FileNotFoundError(f"IsolationForest needs model= or training data at {path}")
            Xtr = np.load(path, allow_pickle=False)["X"]
            model = IsolationForest(n_estimators=n_estimators, max_samples=max_samples, contamination=contamination,
                                    random_state=random_state).fit(Xtr)
        self.clf = model
        from ..models import to_row_model

        self._scorer = _NativeScorer(to_row_model(model), _default_device(device))
        self._init_feedback()

    def _last_scores(self):
        return self.decision_val

    def decision_function(self, X):
        return self._scorer(np.asarray(X, dtype=float))[:, 0]

    def _get_preds(self, X):
        self.decision_val = self.decision_function(X)
        self.prediction = (self.decision_val < self.threshold).astype(int)
        self.N += self.prediction.shape[0]
        return self.prediction

    def metrics(self):
        self.nb_outliers += int(np.sum(self.prediction))
        if self.prediction.shape[0] > 1:
            return self._batch_metrics(self.N)
        return self._feedback_metrics(self.N)


# ------------------------------------------------------------------------ VAE
def _vae_hidden_dims(n_features: int, hidden_layers: int) -> List[int]:
    """vae/model.py:38-45 default hidden widths."""
    dims, dim = [], float(n_features)
    for _ in range(hidden_layers):
        dims.append(int(np.max([dim / 2, 2])))
        dim /= 2
    return dims


@register("VAE_OD")
class OutlierVAE(_FeedbackMetrics, _Reservoir):
    score_key = "mse"

    def __init__(self, threshold=10, reservoir_size=50000, model_name="vae", load_path="./models/", weights=None,
                 preprocess=None, samples: int = 10, seed: int = 0, device=None, precision: str = "fp32"):
        self.threshold = threshold
        self.nb_outliers = 0
        if weights is None:
            weights = load_vae_weights(os.path.join(load_path, model_name + ".npz"))
        self.weights = weights
        n_features = int(np.asarray(weights["encoder"][0]["W"]).shape[1])
        if preprocess is None and os.path.exists(os.path.join(load_path, "preprocess_" + model_name + ".json")):
            with open(os.path.join(load_path, "preprocess_" + model_name + ".json")) as f:
                preprocess = json.load(f)
        self._init_scaling(preprocess, reservoir_size, n_features)
        from .._native import native

        # precision="bf16": bf16 MFMA operands, fp32 accumulation (opt-in; scores within ~1e-2 relative)
        rm = native().vae_model(weights["encoder"], int(weights["latent"]), weights["decoder"], samples, seed,
                                precision)
        self._scorer = _NativeScorer(rm, _default_device(device))
        self._init_feedback()

    @classmethod
    def random(cls, n_features: int, hidden_layers: int = 1, latent_dim: int = 2, hidden_dim=None,
               output_activation: str = "sigmoid", weight_seed: int = 0, **kw) -> "OutlierVAE":
        """Random-init VAE of the reference architecture (vae/model.py:23-91)."""
        return cls(weights=random_vae_weights(n_features, hidden_layers, latent_dim, hidden_dim, output_activation,
                                              weight_seed), **kw)

    def _last_scores(self):
        return self.mse

    def _get_preds(self, X):
        X = np.clip(np.asarray(X, dtype=float), -self.clip, self.clip)
        self.reservoir_sampling(X, update_stand=self.N >= self.reservoir_size)
        self.mse = self._scorer(self._scale(X))[:, 0]
        self.prediction = (self.mse > self.threshold).astype(int)
        return self.prediction

    def metrics(self):
        self.nb_outliers += int(np.sum(self.prediction))
        if self.mse.shape[0] > 1:
            return self._batch_metrics(self.N)
        return self._feedback_metrics(self.N)


def random_vae_weights(n_features, hidden_layers=1, latent_dim=2, hidden_dim=None, output_activation="sigmoid",
                       seed=0) -> Dict:
    from ..models.mlp import layer, random_dense_stack

    hd = list(hidden_dim) if hidden_dim else _vae_hidden_dims(n_features, hidden_layers)
    enc = random_dense_stack([n_features, *hd], ["relu"] * len(hd), seed)
    rng = np.random.default_rng(seed + 1)
    lim = np.sqrt(6.0 / (hd[-1] + 2 * latent_dim))
    enc.append(layer(rng.uniform(-lim, lim, size=(2 * latent_dim, hd[-1])), np.zeros(2 * latent_dim), "identity"))
    dec = random_dense_stack([latent_dim, *hd[::-1], n_features], ["relu"] * len(hd) + [output_activation],
                             seed + 2)
    return {"encoder": enc, "latent": latent_dim, "decoder": dec}


def save_vae_weights(path: str, weights: Dict) -> None:
    arrays = {"latent": np.array(weights["latent"])}
    for part in ("encoder", "decoder"):
        for i, L in enumerate(weights[part]):
            arrays[f"{part}_{i}_W"] = np.asarray(L["W"], np.float32)
            arrays[f"{part}_{i}_b"] = np.asarray(L["b"], np.float32)
            arrays[f"{part}_{i}_act"] = np.array(L["act"])
    np.savez(path, **arrays)


def load_vae_weights(path: str) -> Dict:
    """Weights saved by :func:`save_vae_weights` (npz, no pickle)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"VAE weights not found at {path}; pass weights= or use OutlierVAE.random()")
    z = np.load(path, allow_pickle=False)
    out: Dict[str, Any] = {"latent": int(z["latent"])}
    for part in ("encoder", "decoder"):
        layers, i = [], 0
        while f"{part}_{i}_W" in z:
            layers.append({"W": z[f"{part}_{i}_W"], "b": z[f"{part}_{i}_b"], "act": int(z[f"{part}_{i}_act"])})
            i += 1
        out[part] = layers
    return out


# --------------------------------------------------------------- Seq2Seq LSTM
class Seq2SeqLSTMNet:
    """BiLSTM encoder (stack), LSTM decoder (stack) initialised with the
    concatenated final encoder states, Dense output (seq2seq-lstm/model.py:6-92).
    Weights live in torch modules (random-init or a state_dict from safetensors);
    on a GPU the scoring runs as the native MFMA kernel (``native_model``), on
    the CPU as torch eager."""

    def __init__(self, n_features: int, encoder_dim=(20,), decoder_dim=(20,), output_activation="sigmoid",
                 device: int = -1, seed: int = 0):
        import torch
        import torch.nn as nn

        if any(d != encoder_dim[-1] * 2 for d in decoder_dim):
            raise ValueError(f"Decoder units should be equal to {encoder_dim[-1] * 2}")
        torch.manual_seed(seed)
        self.dev = torch.device(f"cuda:{device}") if device >= 0 else torch.device("cpu")
        self.enc = nn.ModuleList()
        d_in = n_features
        for u in encoder_dim:
            self.enc.append(nn.LSTM(d_in, u, batch_first=True, bidirectional=True))
            d_in = 2 * u
        self.dec = nn.ModuleList()
        d_in = n_features
        for u in decoder_dim:
            self.dec.append(nn.LSTMCell(d_in, u))
            d_in = u
        self.out = nn.Linear(d_in, n_features)
        self.act = {"sigmoid": torch.sigmoid, "linear": lambda t: t, "tanh": torch.tanh,
                    "relu": torch.relu}[output_activation]
        self.act_name = output_activation
        self.modules = nn.ModuleList([self.enc, self.dec, self.out]).to(self.dev).eval()
        self._units: Dict[int, Any] = {}  # timesteps -> native BatchedUnit (GPU)

    def load_state_dict(self, sd):
        self.modules.load_state_dict(sd)

    def _decode(self, x):
        import torch

        h = x
        for i, lstm in enumerate(self.enc):
            h, (hn, cn) = lstm(h)
        state_h = torch.cat([hn[0], hn[1]], dim=1)
        state_c = torch.cat([cn[0], cn[1]], dim=1)
        states = [(state_h, state_c) for _ in self.dec]
        T = x.shape[1]
        out = torch.empty_like(x)
        out[:, 0] = x[:, 0]
        target = x[:, 0]
        for t in range(1, T):
            inp = target
            new_states = []
            for cell, (hs, cs) in zip(self.dec, states):
                hs, cs = cell(inp, (hs, cs))
                new_states.append((hs, cs))
                inp = hs
            states = new_states
            target = self.act(self.out(inp))
            out[:, t] = target
        return out

    def reconstruct(self, X: np.ndarray) -> np.ndarray:
        """Greedy T-1 step decode (torch, eager) -- the CPU path and the test
        oracle of the native kernel."""
        import torch

        x = torch.as_tensor(np.ascontiguousarray(X), dtype=torch.float32, device=self.dev)
        with torch.no_grad():
            return self._decode(x).double().cpu().numpy()

    # ------------------------------------------------------------ native
    _ACTS = {"linear": 0, "sigmoid": 1, "tanh": 2, "relu": 3}

    def native_model(self, timesteps: int):
        """The same network as a native RowModel: one row = a flattened [T, F]
        sequence -> its reconstruction MSE, computed on the GPU by one
        persistent MFMA kernel per batch (csrc/kernels/lstm.hip)."""
        from .._native import native

        def cell(w_ih, w_hh, b_ih, b_hh):
            t = lambda v: v.detach().float().cpu().numpy()  # noqa: E731
            return {"W_ih": t(w_ih), "W_hh": t(w_hh), "b": t(b_ih) + t(b_hh)}

        enc = []
        for m in self.enc:
            enc.append((cell(m.weight_ih_l0, m.weight_hh_l0, m.bias_ih_l0, m.bias_hh_l0),
                        cell(m.weight_ih_l0_reverse, m.weight_hh_l0_reverse, m.bias_ih_l0_reverse,
                             m.bias_hh_l0_reverse)))
        dec = [cell(c.weight_ih, c.weight_hh, c.bias_ih, c.bias_hh) for c in self.dec]
        W = self.out.weight.detach().float().cpu().numpy()
        b = self.out.bias.detach().float().cpu().numpy()
        return native().lstm_seq2seq_model(int(timesteps), int(W.shape[0]), enc, dec, W, b,
                                           self._ACTS[self.act_name])

    def mse(self, X: np.ndarray) -> np.ndarray:
        """Per-sequence reconstruction MSE of X [B, T, F]."""
        B, T, F = X.shape
        if self.dev.type == "cuda":
            unit = self._units.get(T)
            if unit is None:
                from .._native import native

                unit = self._units[T] = native().BatchedUnit(self.native_model(T), self.dev.index or 0,
                                                             max_batch=4096)
            return np.asarray(unit.run(np.ascontiguousarray(X, dtype=np.float64).reshape(B, T * F)))[:, 0]
        rec = self.reconstruct(X)
        return np.mean((X - rec) ** 2, axis=(1, 2))

    def close(self) -> None:
        for u in self._units.values():
            u.stop()
        self._units = {}


@register("SEQ2SEQ_OD")
class OutlierSeq2SeqLSTM(_FeedbackMetrics, _Reservoir):
    score_key = "mse"

    def __init__(self, threshold=0.003, reservoir_size=50000, model_name="seq2seq", load_path="./models/",
                 timesteps: int = 0, n_features: int = 0, encoder_dim=(20,), decoder_dim=(40,),
                 output_activation="sigmoid", preprocess=None, device=None, seed: int = 0):
        self.threshold = threshold
        self.nb_outliers = 0
        cfg_path = os.path.join(load_path, model_name + ".json")
        if (not timesteps or not n_features) and os.path.exists(cfg_path):
            with open(cfg_path) as f:
                cfg = json.load(f)
            timesteps, n_features = cfg["timesteps"], cfg["n_features"]
            encoder_dim, decoder_dim = cfg.get("encoder_dim", encoder_dim), cfg.get("decoder_dim", decoder_dim)
            output_activation = cfg.get("output_activation", output_activation)
        if not timesteps or not n_features:
            raise ValueError("Seq2SeqLSTM needs timesteps and n_features (arguments or <model>.json)")
        self.timesteps, self.n_features = int(timesteps), int(n_features)
        dev = _default_device(device)
        self.net = Seq2SeqLSTMNet(self.n_features, tuple(encoder_dim), tuple(decoder_dim), output_activation, dev, seed)
        wpath = os.path.join(load_path, model_name + ".safetensors")
        if os.path.exists(wpath):
            from safetensors.torch import load_file

            self.net.load_state_dict(load_file(wpath))
        self._init_scaling(preprocess, reservoir_size, self.n_features)

    def _last_scores(self):
        return self.mse

    def _get_preds(self, X):
        X = np.array(X, dtype=float).reshape(-1, self.timesteps, self.n_features)
        for col, c in enumerate(self.clip):
            X[:, :, col] = np.clip(X[:, :, col], -c, c)
        self.reservoir_sampling(X, update_stand=self.N >= self.reservoir_size)
        X = self._scale(X)
        self.mse = self.net.mse(X)
        self.prediction = (self.mse > self.threshold).astype(int)
        return self.prediction

    def metrics(self):
        self.nb_outliers += int(np.sum(self.prediction))
        if self.mse.shape[0] > 1:
            return self._batch_metrics(self.N)
        return self._feedback_metrics(self.N)
