"""Anchor explanations (the reference deploys ``seldonio/alibiexplainer``
next to a predictor -- operator/controllers/seldondeployment_explainers.go:32-184,
explainer types ``anchor_tabular`` / ``anchor_text`` / ``anchor_images`` -- whose
algorithm is Ribeiro, Singh & Guestrin, "Anchors: High-Precision Model-Agnostic
Explanations", AAAI 2018).

An anchor is a set of predicates on an instance (feature bins, words, image
segments) such that perturbed samples that keep the predicates get the same
prediction with probability >= ``threshold``.  The search is a beam search
over predicate sets of growing size; at each size the KL-LUCB best-arm
identification picks the ``beam_size`` most precise candidates, each is then
sampled until its precision is known to be above or below the threshold with
confidence ``1 - delta``, and the valid anchor with the largest coverage wins.

Written here from the paper: perturbation samples are produced in large
batches and labelled by one batched call of the predictor (one request to the
engine per batch, so a GPU-served model labels thousands of samples per
round trip).  Samples are shared between a candidate and its extensions: a
sample drawn for anchor A that also satisfies predicate p counts for A + {p}.
"""
from __future__ import annotations

import math
import re
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

# ----------------------------------------------------------------- bounds


def kl_bernoulli(p: float, q: float) -> float:
    p = min(1 - 1e-16, max(1e-7, p))
    q = min(1 - 1e-16, max(1e-7, q))
    return p * math.log(p / q) + (1 - p) * math.log((1 - p) / (1 - q))


def kl_upper(p: float, level: float) -> float:
    """Largest q >= p with KL(p || q) <= level (bisection)."""
    lo, hi = p, min(1.0, p + math.sqrt(level / 2.0))
    for _ in range(17):
        mid = (lo + hi) / 2.0
        if kl_bernoulli(p, mid) > level:
            hi = mid
        else:
            lo = mid
    return hi


def kl_lower(p: float, level: float) -> float:
    """Smallest q <= p with KL(p || q) <= level."""
    lo, hi = max(0.0, p - math.sqrt(level / 2.0)), p
    for _ in range(17):
        mid = (lo + hi) / 2.0
        if kl_bernoulli(p, mid) > level:
            lo = mid
        else:
            hi = mid
    return lo


def lucb_beta(n_arms: int, t: int, delta: float) -> float:
    # Exploration rate of KL-LUCB (Kaufmann & Kalyanakrishnan 2013), alpha = 1.1, k = 405.5.
    x = math.log(405.5 * n_arms * t ** 1.1 / delta)
    return x + math.log(x)


# ----------------------------------------------------------------- search


class AnchorSearch:
    """Beam search over predicate sets.

    ``sample(anchor, n)`` -> (raw_samples, present [n, n_predicates] bool,
    labels [n] bool) draws ``n`` perturbations that keep every predicate of
    ``anchor`` and labels them (prediction == the instance's prediction).
    ``coverage_present`` [m, n_predicates] are unconditional perturbations
    used for coverage.
    """

    def __init__(self, sample: Callable, n_predicates: int, coverage_present: np.ndarray):
        self.sample = sample
        self.n_pred = n_predicates
        self.cov = coverage_present
        self.present = np.zeros((0, n_predicates), dtype=bool)
        self.labels = np.zeros(0, dtype=bool)
        self.raw: List[np.ndarray] = []
        self.idx: Dict[Tuple[int, ...], np.ndarray] = {}   # samples usable for each anchor
        self.order: Dict[Tuple[int, ...], List[int]] = {(): []}
        self.n_sampled = 0

    # ---- bookkeeping
    def _draw(self, anchor: Tuple[int, ...], n: int) -> None:
        raw, present, labels = self.sample(list(self.order.get(anchor, anchor)), n)
        start = len(self.labels)
        self.present = np.concatenate([self.present, present])
        self.labels = np.concatenate([self.labels, labels.astype(bool)])
        self.raw.append(raw)
        self.n_sampled += n
        # Only the sampled anchor owns them: a sample conditioned on A is a
        # valid conditional sample of an extension A + {p} (taken over when
        # that extension is created, _track), not of an unrelated anchor.
        self.idx[anchor] = np.concatenate([self.idx[anchor], np.arange(start, start + n)])

    def stats(self, a: Tuple[int, ...]) -> Tuple[int, float]:
        ix = self.idx[a]
        return len(ix), float(self.labels[ix].mean()) if len(ix) else 0.0

    def coverage(self, a: Tuple[int, ...]) -> float:
        return float(self.cov[:, list(a)].all(axis=1).mean()) if a else 1.0

    def _track(self, parent: Tuple[int, ...], p: int) -> Tuple[int, ...]:
        a = tuple(sorted(parent + (p,)))
        if a not in self.idx:
            base = self.idx[parent]
            self.idx[a] = base[self.present[base, p]] if len(base) else base
            self.order[a] = self.order[parent] + [p]
        return a

    # ---- KL-LUCB best-arm identification of the top_n most precise anchors
    def lucb(self, arms: List[Tuple[int, ...]], top_n: int, epsilon: float, delta: float,
             batch: int) -> List[int]:
        n = len(arms)
        if n <= top_n:
            return list(range(n))
        for a in arms:  # at least one batch per arm
            if self.stats(a)[0] == 0:
                self._draw(a, batch)
        t = 1
        while True:
            ns = np.array([self.stats(a)[0] for a in arms], dtype=float)
            means = np.array([self.stats(a)[1] for a in arms])
            order = np.argsort(means, kind="stable")
            J, notJ = order[-top_n:], order[:-top_n]
            beta = lucb_beta(n, t, delta)
            ub = np.array([kl_upper(means[f], beta / ns[f]) for f in notJ])
            lb = np.array([kl_lower(means[f], beta / ns[f]) for f in J])
            ut, lt = notJ[int(np.argmax(ub))], J[int(np.argmin(lb))]
            if ub.max() - lb.min() < epsilon or self.n_sampled > self.max_samples:
                return [int(j) for j in J]
            self._draw(arms[ut], batch)
            self._draw(arms[lt], batch)
            t += 1

    def run(self, threshold: float = 0.95, delta: float = 0.1, epsilon: float = 0.15, batch_size: int = 100,
            beam_size: int = 1, max_anchor_size: Optional[int] = None, epsilon_stop: float = 0.05,
            min_samples_start: int = 100, stop_on_first: bool = False, max_samples: int = 200_000) -> Dict:
        self.max_samples = max_samples
        self.idx[()] = np.zeros(0, dtype=np.int64)
        self._draw((), max(1, min_samples_start))
        n, mean = self.stats(())
        beta = math.log(1.0 / delta)
        lb = kl_lower(mean, beta / n)
        while mean > threshold and lb < threshold - epsilon and self.n_sampled < max_samples:
            self._draw((), batch_size)
            n, mean = self.stats(())
            lb = kl_lower(mean, beta / n)
        if lb > threshold:
            return self._result((), mean)
        max_size = max_anchor_size or self.n_pred
        best_of: Dict[int, List[Tuple[int, ...]]] = {0: [()]}
        best_cov, best = -1.0, None
        for size in range(1, max_size + 1):
            cands = []
            for parent in best_of[size - 1]:
                for p in range(self.n_pred):
                    if p in parent:
                        continue
                    a = self._track(parent, p)
                    if a not in cands and self.coverage(a) > best_cov:
                        cands.append(a)
            if not cands:
                break
            chosen = self.lucb(cands, min(beam_size, len(cands)), epsilon, delta, batch_size)
            best_of[size] = [cands[i] for i in chosen]
            stop = False
            beta = math.log(1.0 / (delta / (1 + (beam_size - 1) * self.n_pred)))
            for a in best_of[size]:
                n, mean = self.stats(a)
                lb, ub = kl_lower(mean, beta / n), kl_upper(mean, beta / n)
                while ((mean >= threshold and lb < threshold - epsilon_stop) or
                       (mean < threshold and ub >= threshold + epsilon_stop)) and self.n_sampled < max_samples:
                    self._draw(a, batch_size)
                    n, mean = self.stats(a)
                    lb, ub = kl_lower(mean, beta / n), kl_upper(mean, beta / n)
                cov = self.coverage(a)
                if mean >= threshold and lb > threshold - epsilon_stop and cov > best_cov:
                    best_cov, best = cov, a
                    if best_cov == 1.0 or stop_on_first:
                        stop = True
            if stop or self.n_sampled >= max_samples:
                break
        if best is None:  # no anchor reached the threshold: most precise candidate seen
            pool = [a for s, lst in best_of.items() if s > 0 for a in lst]
            best = max(pool, key=lambda a: self.stats(a)[1]) if pool else ()
        return self._result(best, self.stats(best)[1] if best else mean)

    def _result(self, a: Tuple[int, ...], mean: float) -> Dict:
        seq = self.order.get(a, list(a))
        prec, cov, examples = [], [], []
        for k in range(1, len(seq) + 1):
            sub = tuple(sorted(seq[:k]))
            if sub not in self.idx:
                self._track(tuple(sorted(seq[:k - 1])), seq[k - 1])
            prec.append(self.stats(sub)[1])
            cov.append(self.coverage(sub))
            examples.append(self._examples(sub))
        return {"feature": list(seq), "mean": list(prec), "precision": prec, "coverage": cov, "examples": examples,
                "all_precision": mean if not seq else None, "num_preds": int(self.n_sampled),
                "final_precision": prec[-1] if prec else mean, "final_coverage": cov[-1] if cov else 1.0}

    def _examples(self, a: Tuple[int, ...], k: int = 5) -> Dict[str, list]:
        raw = np.concatenate(self.raw) if self.raw else np.zeros((0,))
        ix = self.idx.get(a, np.zeros(0, dtype=np.int64))
        pos, neg = ix[self.labels[ix]][:k], ix[~self.labels[ix]][:k]
        if not len(raw):
            return {"covered": [], "covered_true": [], "covered_false": []}
        return {"covered": raw[ix[:k]].tolist(), "covered_true": raw[pos].tolist(),
                "covered_false": raw[neg].tolist()}


def _labels_of(predictions: np.ndarray) -> np.ndarray:
    p = np.asarray(predictions)
    if p.ndim == 2 and p.shape[1] > 1:
        return p.argmax(axis=1)
    if p.ndim == 2:
        p = p[:, 0]
    if p.dtype.kind == "f" and np.all((p >= 0) & (p <= 1)) and not np.all(np.mod(p, 1) == 0):
        return (p > 0.5).astype(int)
    return p


# ----------------------------------------------------------------- tabular


class AnchorTabular:
    """Tabular anchors: ordinal features are discretised at the training data's
    percentiles (``disc_perc``); a predicate is "feature in the instance's
    bin" (categorical: "feature == value").  Perturbations take a random
    training row and, for each anchored feature, a training value from the
    instance's bin."""

    def __init__(self, predict_fn: Callable[[np.ndarray], np.ndarray], feature_names: Sequence[str],
                 categorical_names: Optional[Dict[int, Sequence[str]]] = None, seed: int = 0):
        self.predict_fn = predict_fn
        self.feature_names = list(feature_names)
        self.categorical_names = dict(categorical_names or {})
        self.rng = np.random.default_rng(seed)

    def fit(self, train_data: np.ndarray, disc_perc: Sequence[float] = (25, 50, 75)) -> "AnchorTabular":
        X = np.asarray(train_data, dtype=np.float64)
        self.train = X
        self.cuts: Dict[int, np.ndarray] = {}
        for f in range(X.shape[1]):
            if f in self.categorical_names:
                continue
            self.cuts[f] = np.unique(np.percentile(X[:, f], list(disc_perc)))
        self.train_bins = self._disc(X)
        return self

    def _disc(self, X: np.ndarray) -> np.ndarray:
        B = np.empty(X.shape, dtype=np.int64)
        for f in range(X.shape[1]):
            B[:, f] = np.searchsorted(self.cuts[f], X[:, f], side="left") if f in self.cuts else X[:, f]
        return B

    def _pred_name(self, f: int, b: int) -> str:
        name = self.feature_names[f]
        if f not in self.cuts:
            cats = self.categorical_names.get(f)
            return f"{name} = {cats[b] if cats is not None and 0 <= b < len(cats) else b}"
        c = self.cuts[f]
        if b == 0:
            return f"{name} <= {c[0]:.2f}"
        if b >= len(c):
            return f"{name} > {c[-1]:.2f}"
        return f"{c[b - 1]:.2f} < {name} <= {c[b]:.2f}"

    def explain(self, x: np.ndarray, threshold: float = 0.95, delta: float = 0.1, tau: float = 0.15,
                batch_size: int = 100, coverage_samples: int = 10000, **kw) -> Dict:
        x = np.asarray(x, dtype=np.float64).reshape(-1)
        F = x.shape[0]
        xb = self._disc(x[None, :])[0]
        target = _labels_of(self.predict_fn(x[None, :]))[0]
        T, TB, rng = self.train, self.train_bins, self.rng
        same_bin = [np.nonzero(TB[:, f] == xb[f])[0] for f in range(F)]

        def sample(anchor: List[int], n: int, label: bool = True):
            rows = T[rng.integers(0, len(T), n)].copy()
            for f in anchor:
                pool = same_bin[f]
                rows[:, f] = T[pool[rng.integers(0, len(pool), n)], f] if len(pool) else x[f]
            present = self._disc(rows) == xb[None, :]
            labels = (_labels_of(self.predict_fn(rows)) == target) if label else np.zeros(n, bool)
            return rows, present, labels

        cov_present = sample([], coverage_samples, label=False)[1]
        res = AnchorSearch(sample, F, cov_present).run(threshold=threshold, delta=delta, epsilon=tau,
                                                       batch_size=batch_size, **kw)
        names = [self._pred_name(f, int(xb[f])) for f in res["feature"]]
        return _explanation("AnchorTabular", names, res, instance=x.tolist(), prediction=int(target))


# ----------------------------------------------------------------- text

_TOKEN = re.compile(r"\w+|[^\w\s]")


class AnchorText:
    """Text anchors: predicates are the instance's words (by position); a
    perturbation replaces each unanchored word by ``UNK`` with probability
    ``sample_proba`` (alibi's ``use_unk`` mode; no language model here)."""

    def __init__(self, predict_fn: Callable[[List[str]], np.ndarray], seed: int = 0, unk: str = "UNK"):
        self.predict_fn = predict_fn
        self.rng = np.random.default_rng(seed)
        self.unk = unk

    def explain(self, text: str, threshold: float = 0.95, delta: float = 0.1, tau: float = 0.15,
                batch_size: int = 100, sample_proba: float = 0.5, coverage_samples: int = 1000, **kw) -> Dict:
        words = _TOKEN.findall(text)
        W = len(words)
        target = _labels_of(self.predict_fn([text]))[0]
        rng = self.rng

        def sample(anchor: List[int], n: int, label: bool = True):
            keep = rng.random((n, W)) >= sample_proba
            keep[:, anchor] = True
            texts = [" ".join(w if k else self.unk for w, k in zip(words, row)) for row in keep]
            labels = (_labels_of(self.predict_fn(texts)) == target) if label else np.zeros(n, bool)
            return np.array(texts, dtype=object), keep, labels

        cov_present = sample([], coverage_samples, label=False)[1]
        res = AnchorSearch(sample, W, cov_present).run(threshold=threshold, delta=delta, epsilon=tau,
                                                       batch_size=batch_size, **kw)
        names = [words[i] for i in res["feature"]]
        out = _explanation("AnchorText", names, res, instance=text, prediction=int(target))
        out["raw"]["positions"] = [sum(len(w) + 1 for w in words[:i]) for i in res["feature"]]
        return out


# ----------------------------------------------------------------- images


def grid_slic(image: np.ndarray, n_segments: int = 16, iters: int = 4, compactness: float = 10.0) -> np.ndarray:
    """Superpixels: a k-means in (colour, x, y) seeded on a regular grid
    (SLIC-style, restricted to a 2S window per centre)."""
    img = np.asarray(image, dtype=np.float64)
    if img.ndim == 2:
        img = img[:, :, None]
    H, W, C = img.shape
    g = max(1, int(round(math.sqrt(n_segments))))
    S = max(1.0, math.sqrt(H * W / float(g * g)))
    ys = (np.arange(g) + 0.5) * H / g
    xs = (np.arange(g) + 0.5) * W / g
    cy, cx = [a.ravel() for a in np.meshgrid(ys, xs, indexing="ij")]
    cc = np.stack([img[int(y), int(x)] for y, x in zip(cy, cx)])
    yy, xx = np.mgrid[0:H, 0:W]
    scale = (np.ptp(img) or 1.0)
    for _ in range(iters):
        dist = np.full((H, W), np.inf)
        lab = np.zeros((H, W), dtype=np.int64)
        for k in range(len(cy)):
            y0, y1 = int(max(0, cy[k] - 2 * S)), int(min(H, cy[k] + 2 * S + 1))
            x0, x1 = int(max(0, cx[k] - 2 * S)), int(min(W, cx[k] + 2 * S + 1))
            dc = ((img[y0:y1, x0:x1] - cc[k]) ** 2).sum(-1) / scale ** 2
            ds = ((yy[y0:y1, x0:x1] - cy[k]) ** 2 + (xx[y0:y1, x0:x1] - cx[k]) ** 2) / S ** 2
            d = dc + (compactness / 10.0) ** 2 * ds
            better = d < dist[y0:y1, x0:x1]
            dist[y0:y1, x0:x1][better] = d[better]
            lab[y0:y1, x0:x1][better] = k
        for k in range(len(cy)):
            m = lab == k
            if m.any():
                cy[k], cx[k] = yy[m].mean(), xx[m].mean()
                cc[k] = img[m].mean(0)
    _, lab = np.unique(lab, return_inverse=True)
    return lab.reshape(H, W)


class AnchorImage:
    """Image anchors over superpixels: a perturbation replaces each unanchored
    segment, with probability ``p_sample``, by the segment's mean colour
    (``fudged`` image); anchored segments keep the original pixels."""

    def __init__(self, predict_fn: Callable[[np.ndarray], np.ndarray], image_shape: Sequence[int],
                 segmentation_fn: Optional[Callable[[np.ndarray], np.ndarray]] = None,
                 segmentation_kwargs: Optional[Dict] = None, seed: int = 0):
        self.predict_fn = predict_fn
        self.image_shape = tuple(image_shape)
        kw = dict(segmentation_kwargs or {"n_segments": 16})
        self.segment = segmentation_fn or (lambda im: grid_slic(im, **kw))
        self.rng = np.random.default_rng(seed)

    def explain(self, image: np.ndarray, threshold: float = 0.95, delta: float = 0.1, tau: float = 0.15,
                batch_size: int = 100, p_sample: float = 0.5, coverage_samples: int = 1000, **kw) -> Dict:
        img = np.asarray(image, dtype=np.float64).reshape(self.image_shape)
        seg = np.unique(np.asarray(self.segment(img)), return_inverse=True)[1].reshape(img.shape[:2])
        nseg = int(seg.max()) + 1
        fudged = img.copy()
        for s in range(nseg):
            fudged[seg == s] = img[seg == s].mean(0)
        target = _labels_of(self.predict_fn(img[None]))[0]
        rng = self.rng
        onehot = np.stack([seg == s for s in range(nseg)])  # [nseg, H, W]

        def sample(anchor: List[int], n: int, label: bool = True):
            keep = rng.random((n, nseg)) >= p_sample
            keep[:, anchor] = True
            if not label:
                return None, keep, np.zeros(n, bool)
            mask = np.tensordot(keep.astype(np.float64), onehot, axes=1) > 0  # [n, H, W]
            m = mask.reshape(mask.shape + (1,) * (img.ndim - 2))
            batch = np.where(m, img[None], fudged[None])
            labels = _labels_of(self.predict_fn(batch)) == target
            return keep.astype(np.float64), keep, labels

        cov_present = sample([], coverage_samples, label=False)[1]
        res = AnchorSearch(sample, nseg, cov_present).run(threshold=threshold, delta=delta, epsilon=tau,
                                                          batch_size=batch_size, **kw)
        anchor_img = np.zeros_like(img)
        for s in res["feature"]:
            anchor_img[seg == s] = img[seg == s]
        out = _explanation("AnchorImage", [int(s) for s in res["feature"]], res, instance=None,
                           prediction=int(target))
        out["anchor"] = anchor_img.tolist()
        out["segments"] = seg.tolist()
        return out


def _explanation(name: str, names: list, res: Dict, instance, prediction: int) -> Dict:
    raw = dict(res)
    raw["names"] = names
    raw["instance"] = instance
    raw["prediction"] = prediction
    return {"names": names, "precision": float(res["final_precision"]), "coverage": float(res["final_coverage"]),
            "raw": raw, "meta": {"name": name}}
