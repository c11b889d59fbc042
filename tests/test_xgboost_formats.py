"""XGBoost model files (reference servers/xgboostserver/xgboostserver/
XGBoostServer.py:8-19 loads ``model.bst``): JSON, UBJSON and the legacy binary
layout decode to the same ensemble.  xgboost is not importable and the
reference ships no ``.bst`` fixture, so parity with files written by xgboost
itself is unpinned: the files here are written byte-by-byte from the documented
layout (models/xgb_binary.py) and predictions are checked against a direct
per-tree walk."""
import math
import struct

import numpy as np
import pytest

from seldon_core_amd.models import from_xgboost_json
from seldon_core_amd.models.xgb_binary import load_xgboost_model, parse_ubjson


def _rand_tree(rng, n_features, max_depth):
    left, right, feat, thr, dl = [], [], [], [], []

    def grow(d):
        i = len(left)
        for a in (left, right, feat, thr, dl):
            a.append(0)
        if d == max_depth or (d > 0 and rng.random() < 0.25):
            left[i] = right[i] = -1
            thr[i] = float(np.float32(rng.normal() * 0.3))
            return i
        feat[i] = int(rng.integers(0, n_features))
        thr[i] = float(np.float32(rng.normal()))
        dl[i] = int(rng.integers(0, 2))
        left[i] = grow(d + 1)
        right[i] = grow(d + 1)
        return i

    grow(0)
    return {"left_children": left, "right_children": right, "split_indices": feat, "split_conditions": thr,
            "default_left": dl}


def _model(objective, n_trees=12, n_features=5, num_class=0, base_score=0.5, seed=0, booster="gbtree"):
    rng = np.random.default_rng(seed)
    trees = [_rand_tree(rng, n_features, 4) for _ in range(n_trees)]
    groups = max(1, num_class)
    gb = {"name": booster, "model": {"trees": trees, "tree_info": [i % groups for i in range(n_trees)]}}
    if booster == "dart":
        gb["weight_drop"] = [float(np.float32(w)) for w in rng.uniform(0.5, 1.0, n_trees)]
    return {"learner": {"learner_model_param": {"num_feature": str(n_features), "num_class": str(num_class),
                                                "base_score": repr(base_score)},
                        "objective": {"name": objective}, "gradient_booster": gb}}


def _oracle(model, X):
    lr = model["learner"]
    gb = lr["gradient_booster"]
    trees, info = gb["model"]["trees"], gb["model"]["tree_info"]
    w = gb.get("weight_drop", [1.0] * len(trees))
    groups = max(1, int(lr["learner_model_param"]["num_class"]))
    bs = float(lr["learner_model_param"]["base_score"])
    obj = lr["objective"]["name"]
    out = np.zeros((len(X), groups))
    for r, x in enumerate(X):
        m = np.full(groups, bs if obj != "binary:logistic" else math.log(bs / (1 - bs)))
        for t, g, wt in zip(trees, info, w):
            i = 0
            while t["left_children"][i] >= 0:
                v = x[t["split_indices"][i]]
                go_left = bool(t["default_left"][i]) if np.isnan(v) else np.float32(v) < np.float32(
                    t["split_conditions"][i])
                i = t["left_children"][i] if go_left else t["right_children"][i]
            m[g] += np.float32(t["split_conditions"][i]) * np.float32(wt)
        if obj == "binary:logistic":
            out[r] = 1 / (1 + np.exp(-m))
        elif obj.startswith("multi:"):
            e = np.exp(m - m.max())
            out[r] = e / e.sum()
        else:
            out[r] = m
    return out


# ------------------------------------------------------------ writers (tests only)
def _str(s):
    b = s.encode()
    return struct.pack("<Q", len(b)) + b


def _legacy_binary(model, magic=True, attrs=None):
    lr = model["learner"]
    p = lr["learner_model_param"]
    gb = lr["gradient_booster"]
    trees = gb["model"]["trees"]
    out = bytearray(b"binf" if magic else b"")
    out += struct.pack("<fIiii", float(p["base_score"]), int(p["num_feature"]), int(p["num_class"]),
                       1 if attrs else 0, 0) + bytes(29 * 4)
    out += _str(lr["objective"]["name"]) + _str(gb["name"])
    out += struct.pack("<iiiiqii", len(trees), 1, int(p["num_feature"]), 0, 0, max(1, int(p["num_class"])), 0)
    out += bytes(32 * 4)
    for t in trees:
        n = len(t["left_children"])
        out += struct.pack("<iiiiii", 1, n, 0, 0, int(p["num_feature"]), 0) + bytes(31 * 4)
        for i in range(n):
            leaf = t["left_children"][i] < 0
            sidx = 0 if leaf else (t["split_indices"][i] | (int(t["default_left"][i]) << 31))
            out += struct.pack("<iiiIf", -1, t["left_children"][i], t["right_children"][i], sidx,
                               t["split_conditions"][i])
        out += bytes(16 * n)  # node statistics
    out += struct.pack(f"<{len(trees)}i", *gb["model"]["tree_info"])
    if gb["name"] == "dart":
        out += struct.pack("<Q", len(trees)) + struct.pack(f"<{len(trees)}f", *gb["weight_drop"])
    if attrs:
        out += struct.pack("<Q", len(attrs))
        for k, v in attrs.items():
            out += _str(k) + _str(v)
    return bytes(out)


def _ubj_key(k):
    b = k.encode()
    return b"U" + struct.pack(">B", len(b)) + b


def _ubj(v):
    if isinstance(v, dict):
        return b"{" + b"".join(_ubj_key(k) + _ubj(x) for k, x in v.items()) + b"}"
    if isinstance(v, list):
        if v and all(isinstance(x, float) for x in v):
            return b"[$d#L" + struct.pack(">q", len(v)) + struct.pack(f">{len(v)}f", *v)
        if v and all(isinstance(x, int) and not isinstance(x, bool) for x in v):
            return b"[$l#I" + struct.pack(">h", len(v)) + struct.pack(f">{len(v)}i", *v)
        return b"[" + b"".join(_ubj(x) for x in v) + b"]"  # generic, unsized
    if isinstance(v, str):
        b = v.encode()
        return b"Si" + struct.pack(">b", len(b)) + b
    if isinstance(v, bool):
        return b"T" if v else b"F"
    if isinstance(v, int):
        return b"L" + struct.pack(">q", v)
    if isinstance(v, float):
        return b"D" + struct.pack(">d", v)
    if v is None:
        return b"Z"
    raise TypeError(type(v))


CASES = [("reg:squarederror", 0, 0.5, "gbtree"), ("binary:logistic", 0, 0.3, "gbtree"),
         ("multi:softprob", 3, 0.5, "gbtree"), ("reg:squarederror", 0, 0.5, "dart")]


@pytest.mark.parametrize("objective,num_class,base_score,booster", CASES,
                         ids=["reg", "binary", "softprob", "dart"])
def test_three_formats_predict_identically(objective, num_class, base_score, booster):
    model = _model(objective, num_class=num_class, base_score=base_score, booster=booster)
    rng = np.random.default_rng(1)
    X = rng.normal(size=(64, 5))
    X[::7, 2] = np.nan  # default directions
    want = _oracle(model, X)
    for src in (model, _legacy_binary(model), _legacy_binary(model, magic=False, attrs={"best_iteration": "11"}),
                _ubj(model)):
        ens = from_xgboost_json(src if isinstance(src, dict) else load_xgboost_model(src))
        got = np.asarray(ens.predict(X), dtype=float).reshape(len(X), -1)
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-6)


def test_ubjson_decoder_types():
    doc = {"a": [1, 2, 3], "b": [0.5, 1.5], "c": "x", "d": {"e": None, "f": True, "g": [1, "two", 3.0]}, "h": -7}
    got = parse_ubjson(_ubj(doc))
    assert got["a"].tolist() == [1, 2, 3] and got["b"].tolist() == [0.5, 1.5]
    assert got["c"] == "x" and got["d"] == {"e": None, "f": True, "g": [1, "two", 3.0]} and got["h"] == -7
    # unsized, untyped array of int8 and a high-precision number
    assert parse_ubjson(b"[i\x01i\xffHi\x031.5]") == [1, -1, 1.5]


def test_server_loads_model_bst(tmp_path):
    from seldon_core_amd.servers import XGBoostServer

    model = _model("binary:logistic", base_score=0.5)
    (tmp_path / "model.bst").write_bytes(_legacy_binary(model))
    s = XGBoostServer(str(tmp_path))
    s.load()
    X = np.random.default_rng(2).normal(size=(8, 5))
    np.testing.assert_allclose(np.asarray(s.predict(X, [])).reshape(8, -1), _oracle(model, X), rtol=2e-6)


def test_deleted_nodes_and_base_score_vector_string():
    model = _model("reg:squarederror", n_trees=2)
    t = model["learner"]["gradient_booster"]["model"]["trees"][0]
    # append an orphan (deleted) node as the trainer leaves it: sindex all ones
    raw = bytearray(_legacy_binary(model))
    ens = from_xgboost_json(load_xgboost_model(bytes(raw)))
    assert ens.n_features == 5
    n = len(t["left_children"])
    # locate tree 0's node block and mark its last node deleted with a garbage split index
    off = 4 + 136 + len(_str("reg:squarederror")) + len(_str("gbtree")) + 160 + 148
    last = off + (n - 1) * 20
    parent, lft, rgt, sidx, val = struct.unpack_from("<iiiIf", raw, last)
    if lft < 0:  # only a leaf may become a deleted orphan without breaking the tree
        struct.pack_into("<iiiIf", raw, last, -1, -1, -1, 0xFFFFFFFF, val)
        ens = from_xgboost_json(load_xgboost_model(bytes(raw)))
        assert ens.n_features == 5
    model["learner"]["learner_model_param"]["base_score"] = "[5E-1]"  # xgboost 2.x vector form
    X = np.random.default_rng(3).normal(size=(4, 5))
    model_ref = _model("reg:squarederror", n_trees=2)
    np.testing.assert_allclose(np.asarray(from_xgboost_json(model).predict(X)).reshape(4, -1),
                               _oracle(model_ref, X), rtol=2e-6)


def test_truncated_binary_is_rejected():
    raw = _legacy_binary(_model("reg:squarederror"))
    with pytest.raises(ValueError, match="truncated"):
        load_xgboost_model(raw[: len(raw) // 2])
