"""Tree-ensemble model import: XGBoost JSON, scikit-learn trees / forests /
gradient boosting / isolation forest -> the engine's GPU tree kernels.

Two device layouts (csrc/kernels/tree.hip):

* **perfect** -- every tree padded to a complete binary tree of depth D and
  stored breadth-first as 8-byte ``{thr, feat|default_left}`` nodes; child of
  node i is 2i+1 (left) / 2i+2 (right).  Used when the deepest tree has
  depth <= ``MAX_PERFECT_DEPTH`` (XGBoost-style boosted trees).
* **sparse** -- explicit ``{thr, feat, left, right}`` nodes for deep trees
  (random forests grown to purity).

Decision semantics: XGBoost goes left iff ``x < thr`` (missing -> default
direction); scikit-learn goes left iff ``x <= thr`` with fp32 features and
fp64 thresholds, reproduced exactly by rounding each threshold *down* to the
largest float32 <= thr.

Reference servers: servers/xgboostserver/xgboostserver/XGBoostServer.py:10-26,
servers/sklearnserver/sklearnserver/SKLearnServer.py:15-44,
components/outlier-detection/isolation-forest/CoreIsolationForest.py:62-76.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import numpy as np

MAX_PERFECT_DEPTH = 10
DEFAULT_LEFT = np.int32(-(2 ** 31))  # bit 31

# transforms (csrc/kernels/kernels.h TreeTransform)
T_IDENTITY, T_SIGMOID, T_SOFTMAX, T_BINARY_PROBA, T_MEAN, T_ISOLATION = range(6)


@dataclass
class Tree:
    """One binary tree in explicit (sparse) form; leaves have left == -1."""
    left: np.ndarray
    right: np.ndarray
    feature: np.ndarray
    threshold: np.ndarray  # float32 (already rounded for cmp semantics); leaf value for leaves
    default_left: np.ndarray
    group: int = 0

    def depth(self) -> int:
        d = np.zeros(len(self.left), dtype=np.int64)
        best = 0
        stack = [0]
        while stack:
            i = stack.pop()
            if self.left[i] >= 0:
                for c in (self.left[i], self.right[i]):
                    d[c] = d[i] + 1
                    stack.append(int(c))
            else:
                best = max(best, int(d[i]))
        return best


@dataclass
class TreeEnsemble:
    trees: List[Tree]
    n_features: int
    groups: int = 1
    out_cols: int = 1
    transform: int = T_IDENTITY
    cmp_le: int = 0
    scale: float = 1.0
    base_margin: List[float] = field(default_factory=lambda: [0.0])
    flat_output: bool = False
    class_names: Optional[List[str]] = None

    # ----------------------------------------------------------- layouts
    def max_depth(self) -> int:
        return max(t.depth() for t in self.trees)

    def _sorted(self) -> List[Tree]:
        return sorted(self.trees, key=lambda t: t.group)  # stable: keeps round order per group

    def to_perfect(self, depth: Optional[int] = None) -> Dict:
        D = max(1, depth or self.max_depth())
        ni, nl = (1 << D) - 1, 1 << D
        trees = self._sorted()
        T = len(trees)
        thr = np.full((T, ni), np.inf, dtype=np.float32)
        feat = np.full((T, ni), DEFAULT_LEFT, dtype=np.int32)  # feature 0, default-left
        leaves = np.zeros((T, nl), dtype=np.float32)
        for t, tr in enumerate(trees):
            # (sparse node, perfect index, depth)
            stack = [(0, 0, 0)]
            while stack:
                s, p, d = stack.pop()
                if tr.left[s] >= 0:
                    if d >= D:
                        raise ValueError("tree deeper than layout depth")
                    thr[t, p] = tr.threshold[s]
                    f = np.int32(tr.feature[s])
                    feat[t, p] = f | DEFAULT_LEFT if tr.default_left[s] else f
                    stack.append((int(tr.left[s]), 2 * p + 1, d + 1))
                    stack.append((int(tr.right[s]), 2 * p + 2, d + 1))
                else:
                    # leaf at depth d: fill every leaf of the padded subtree
                    span = 1 << (D - d)
                    first = p
                    for _ in range(D - d):
                        first = 2 * first + 1
                    first -= ni
                    leaves[t, first:first + span] = tr.threshold[s]
        return dict(n_trees=T, n_features=self.n_features, groups=self.groups, out_cols=self.out_cols,
                    transform=self.transform, cmp_le=self.cmp_le, scale=float(self.scale),
                    base_margin=[float(x) for x in self.base_margin], tree_group=[t.group for t in trees],
                    depth=D, thr=thr.ravel(), feat=feat.ravel(), leaves=leaves.ravel())

    def to_sparse(self) -> Dict:
        trees = self._sorted()
        thr, feat, left, right, roots = [], [], [], [], []
        off = 0
        for tr in trees:
            n = len(tr.left)
            roots.append(off)
            f = tr.feature.astype(np.int32).copy()
            f[tr.left < 0] = 0
            f = np.where(tr.default_left.astype(bool), f | DEFAULT_LEFT, f).astype(np.int32)
            l = np.where(tr.left >= 0, tr.left + off, -1).astype(np.int32)
            r = np.where(tr.left >= 0, tr.right + off, -1).astype(np.int32)
            thr.append(tr.threshold.astype(np.float32))
            feat.append(f)
            left.append(l)
            right.append(r)
            off += n
        return dict(n_trees=len(trees), n_features=self.n_features, groups=self.groups, out_cols=self.out_cols,
                    transform=self.transform, cmp_le=self.cmp_le, scale=float(self.scale),
                    base_margin=[float(x) for x in self.base_margin], tree_group=[t.group for t in trees], depth=0,
                    thr=np.concatenate(thr), feat=np.concatenate(feat), left=np.concatenate(left),
                    right=np.concatenate(right), tree_root=roots)

    def device_spec(self) -> Dict:
        d = self.max_depth()
        return self.to_perfect(d) if d <= MAX_PERFECT_DEPTH else self.to_sparse()

    # ---------------------------------------------------- CPU reference
    def margins(self, X: np.ndarray) -> np.ndarray:
        X = np.asarray(X, dtype=np.float32)
        out = np.zeros((X.shape[0], self.groups), dtype=np.float64)
        for tr in self.trees:
            for r in range(X.shape[0]):
                i = 0
                while tr.left[i] >= 0:
                    x = X[r, tr.feature[i]]
                    if np.isnan(x):
                        go_left = bool(tr.default_left[i])
                    else:
                        go_left = x <= tr.threshold[i] if self.cmp_le else x < tr.threshold[i]
                    i = tr.left[i] if go_left else tr.right[i]
                out[r, tr.group] += tr.threshold[i]
        return out * self.scale + np.asarray(self.base_margin, dtype=np.float64)

    def predict(self, X: np.ndarray) -> np.ndarray:
        m = self.margins(X)
        if self.transform == T_SIGMOID:
            out = 1.0 / (1.0 + np.exp(-m[:, :1]))
        elif self.transform == T_BINARY_PROBA:
            p = 1.0 / (1.0 + np.exp(-m[:, 0]))
            out = np.stack([1 - p, p], axis=1)
        elif self.transform == T_SOFTMAX:
            e = np.exp(m - m.max(axis=1, keepdims=True))
            out = e / e.sum(axis=1, keepdims=True)
        elif self.transform == T_ISOLATION:
            base = self.base_margin[0]
            out = -np.exp2(-(m[:, :1] - base)) - base
        else:
            out = m
        return out[:, 0] if self.flat_output else out


# ------------------------------------------------------------------ helpers
def f32_le_threshold(t: np.ndarray) -> np.ndarray:
    """Largest float32 <= t (exact `x <= t` for float32 x against fp64 t)."""
    t = np.asarray(t, dtype=np.float64)
    f = t.astype(np.float32)
    too_big = f.astype(np.float64) > t
    f[too_big] = np.nextafter(f[too_big], np.float32(-np.inf))
    return f


def _avg_path_length(n: np.ndarray) -> np.ndarray:
    """c(n) of the isolation-forest paper (sklearn _average_path_length)."""
    n = np.asarray(n, dtype=np.float64)
    out = np.zeros_like(n)
    m1 = n <= 1
    m2 = n == 2
    mo = ~(m1 | m2)
    out[m2] = 1.0
    out[mo] = 2.0 * (np.log(n[mo] - 1.0) + np.euler_gamma) - 2.0 * (n[mo] - 1.0) / n[mo]
    return out


# ------------------------------------------------------------------ XGBoost
def from_xgboost_json(model: Union[str, Path, bytes, Dict]) -> TreeEnsemble:
    """Import an XGBoost model: JSON (``Booster.save_model('model.json')``),
    or -- decoded to the same schema by :mod:`.xgb_binary` -- UBJSON
    (``model.ubj``) and the legacy binary ``model.bst``."""
    if not isinstance(model, dict):
        from .xgb_binary import load_xgboost_model

        model = load_xgboost_model(model)
    learner = model["learner"]
    lmp = learner.get("learner_model_param", {})
    n_features = int(lmp.get("num_feature", 0))
    num_class = int(lmp.get("num_class", 0) or 0)
    bs = lmp.get("base_score", 0.5)
    base_score = float(bs.strip("[]").split(",")[0]) if isinstance(bs, str) else float(bs)  # 2.x: "[5E-1]"
    objective = learner.get("objective", {}).get("name", "reg:squarederror")
    gb = learner["gradient_booster"]
    if gb.get("name") not in ("gbtree", "dart"):
        raise ValueError(f"unsupported booster {gb.get('name')}")
    gm = gb["model"]
    tree_info = gm.get("tree_info", [0] * len(gm["trees"]))
    trees: List[Tree] = []
    for tj, g in zip(gm["trees"], tree_info):
        left = np.asarray(tj["left_children"], dtype=np.int64)
        right = np.asarray(tj["right_children"], dtype=np.int64)
        split = np.asarray(tj["split_conditions"], dtype=np.float32)
        feat = np.asarray(tj["split_indices"], dtype=np.int64)
        dl = np.asarray(tj.get("default_left", [0] * len(left)), dtype=np.int64)
        feat = np.where(left >= 0, feat, 0)
        trees.append(Tree(left, right, feat, split, dl, int(g)))
        n_features = max(n_features, int(feat.max()) + 1 if len(feat) else 1)
    if gb.get("name") == "dart":
        w = gb.get("weight_drop", [1.0] * len(trees))
        for t, wt in zip(trees, w):
            t.threshold = np.where(t.left >= 0, t.threshold, t.threshold * np.float32(wt)).astype(np.float32)
    groups = max(1, num_class)
    if objective in ("binary:logistic", "reg:logistic"):
        margin = math.log(base_score / (1.0 - base_score)) if 0 < base_score < 1 else 0.0
        return TreeEnsemble(trees, n_features, 1, 1, T_SIGMOID, 0, 1.0, [margin], flat_output=True)
    if objective == "binary:logitraw":
        return TreeEnsemble(trees, n_features, 1, 1, T_IDENTITY, 0, 1.0, [base_score], flat_output=True)
    if objective in ("multi:softprob", "multi:softmax"):
        return TreeEnsemble(trees, n_features, groups, groups, T_SOFTMAX, 0, 1.0, [base_score] * groups)
    # regression family (reg:squarederror, reg:linear, ...): identity link
    return TreeEnsemble(trees, n_features, 1, 1, T_IDENTITY, 0, 1.0, [base_score], flat_output=True)


def synthetic_xgboost(n_trees: int = 1000, depth: int = 8, n_features: int = 32, seed: int = 0,
                      objective: str = "reg:squarederror") -> TreeEnsemble:
    """Random perfect trees of the given depth (random-init weights for the
    ``xgboostserver 1000-tree depth-8 regressor`` benchmark config)."""
    rng = np.random.default_rng(seed)
    ni, nl = (1 << depth) - 1, 1 << depth
    trees = []
    for _ in range(n_trees):
        n = ni + nl
        left = np.full(n, -1, dtype=np.int64)
        right = np.full(n, -1, dtype=np.int64)
        idx = np.arange(ni)
        left[:ni] = 2 * idx + 1
        right[:ni] = 2 * idx + 2
        feat = np.zeros(n, dtype=np.int64)
        feat[:ni] = rng.integers(0, n_features, ni)
        thr = np.zeros(n, dtype=np.float32)
        thr[:ni] = rng.standard_normal(ni).astype(np.float32) * 0.8
        thr[ni:] = (rng.standard_normal(nl) * 0.05).astype(np.float32)
        dl = np.zeros(n, dtype=np.int64)
        dl[:ni] = rng.integers(0, 2, ni)
        trees.append(Tree(left, right, feat, thr, dl, 0))
    if objective == "binary:logistic":
        return TreeEnsemble(trees, n_features, 1, 1, T_SIGMOID, 0, 1.0, [0.0], flat_output=True)
    return TreeEnsemble(trees, n_features, 1, 1, T_IDENTITY, 0, 1.0, [0.5], flat_output=True)


# ------------------------------------------------------------------ sklearn
def _sk_tree(est_tree, group: int, value_fn, feature_map: Optional[np.ndarray] = None) -> Tree:
    t = est_tree.tree_
    left = t.children_left.astype(np.int64)
    right = t.children_right.astype(np.int64)
    feat = np.where(left >= 0, t.feature, 0).astype(np.int64)
    if feature_map is not None:
        feat = np.where(left >= 0, np.asarray(feature_map)[feat], 0)
    thr = f32_le_threshold(t.threshold)
    leafv = value_fn(t).astype(np.float32)
    thr = np.where(left >= 0, thr, leafv).astype(np.float32)
    # sklearn sends NaN to the side chosen at fit (missing_go_to_left, >=1.3)
    mgl = getattr(t, "missing_go_to_left", None)
    dl = np.asarray(mgl, dtype=np.int64) if mgl is not None else np.ones(len(left), dtype=np.int64)
    return Tree(left, right, feat, thr, dl, group)


def from_sklearn_trees(est) -> TreeEnsemble:
    """DecisionTree / RandomForest / ExtraTrees / GradientBoosting / IsolationForest."""
    from sklearn.ensemble import (ExtraTreesClassifier, ExtraTreesRegressor, GradientBoostingClassifier,
                                  GradientBoostingRegressor, IsolationForest, RandomForestClassifier,
                                  RandomForestRegressor)
    from sklearn.tree import DecisionTreeClassifier, DecisionTreeRegressor

    nf = int(est.n_features_in_)
    if isinstance(est, (DecisionTreeClassifier, RandomForestClassifier, ExtraTreesClassifier)):
        estimators = [est] if isinstance(est, DecisionTreeClassifier) else list(est.estimators_)
        C = len(est.classes_)
        trees = []
        for c in range(C):
            for e in estimators:
                def val(t, c=c):
                    v = t.value[:, 0, :]
                    return v[:, c] / np.maximum(v.sum(axis=1), 1e-300)
                trees.append(_sk_tree(e, c, val))
        return TreeEnsemble(trees, nf, C, C, T_MEAN, 1, 1.0 / len(estimators), [0.0] * C,
                            class_names=[str(x) for x in est.classes_])
    if isinstance(est, (DecisionTreeRegressor, RandomForestRegressor, ExtraTreesRegressor)):
        estimators = [est] if isinstance(est, DecisionTreeRegressor) else list(est.estimators_)
        trees = [_sk_tree(e, 0, lambda t: t.value[:, 0, 0]) for e in estimators]
        return TreeEnsemble(trees, nf, 1, 1, T_MEAN, 1, 1.0 / len(estimators), [0.0], flat_output=True)
    if isinstance(est, GradientBoostingRegressor):
        init = float(np.ravel(est._raw_predict_init(np.zeros((1, nf))))[0])
        trees = [_sk_tree(e, 0, lambda t: t.value[:, 0, 0]) for e in est.estimators_[:, 0]]
        return _gb_scaled(trees, nf, 1, T_IDENTITY, est.learning_rate, [init], True)
    if isinstance(est, GradientBoostingClassifier):
        init = np.ravel(est._raw_predict_init(np.zeros((1, nf)))).astype(np.float64)
        K = est.estimators_.shape[1]
        trees = []
        for k in range(K):
            trees += [_sk_tree(e, k, lambda t: t.value[:, 0, 0]) for e in est.estimators_[:, k]]
        if K == 1:
            return _gb_scaled(trees, nf, 1, T_BINARY_PROBA, est.learning_rate, [float(init[0])], False, out_cols=2,
                              class_names=[str(x) for x in est.classes_])
        return _gb_scaled(trees, nf, K, T_SOFTMAX, est.learning_rate, list(map(float, init)), False,
                          class_names=[str(x) for x in est.classes_])
    if isinstance(est, IsolationForest):
        trees = []
        feats = getattr(est, "estimators_features_", [None] * len(est.estimators_))
        for e, fmap in zip(est.estimators_, feats):
            t = e.tree_
            depth = np.zeros(t.node_count, dtype=np.float64)
            for i in range(t.node_count):
                if t.children_left[i] >= 0:
                    depth[t.children_left[i]] = depth[i] + 1
                    depth[t.children_right[i]] = depth[i] + 1
            pl = depth + _avg_path_length(t.n_node_samples)
            trees.append(_sk_tree(e, 0, lambda tt, pl=pl: pl, feature_map=fmap))
        c = float(_avg_path_length(np.array([est.max_samples_]))[0])
        scale = 1.0 / (len(est.estimators_) * c)
        return TreeEnsemble(trees, nf, 1, 1, T_ISOLATION, 1, scale, [float(est.offset_)], flat_output=True)
    raise TypeError(f"unsupported tree estimator {type(est).__name__}")


def _gb_scaled(trees, nf, groups, transform, lr, init, flat, out_cols=None, class_names=None) -> TreeEnsemble:
    # margin = init + lr * sum(tree)  ->  scale leaves by lr, base = init
    lr = float(lr)
    for t in trees:
        leaf = t.left < 0
        t.threshold = np.where(leaf, t.threshold * np.float32(lr), t.threshold).astype(np.float32)
    return TreeEnsemble(trees, nf, groups, out_cols or groups, transform, 1, 1.0, list(init), flat_output=flat,
                        class_names=class_names)
