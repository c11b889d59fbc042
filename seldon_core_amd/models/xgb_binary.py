"""XGBoost model files without the xgboost library: the legacy binary
``model.bst`` and the UBJSON ``model.ubj`` formats, decoded into the same
dict schema as ``Booster.save_model('model.json')`` so that
:func:`seldon_core_amd.models.trees.from_xgboost_json` builds the device
ensemble from any of the three.

The reference XGBoost server loads ``<modelUri>/model.bst`` through
``xgb.Booster(model_file=...)`` (servers/xgboostserver/xgboostserver/
XGBoostServer.py:8-19).  xgboost is not importable on this platform, so the
two binary layouts are parsed here directly.

Legacy binary (little-endian, what ``save_model('model.bst')`` wrote before
UBJSON became the default)::

    ["binf"]                                optional 4-byte magic
    LearnerModelParam                       136 B: f32 base_score, u32 num_feature,
                                            i32 num_class, i32 contain_extra_attrs,
                                            i32 contain_eval_metrics, 29 x i32 reserved
    str objective, str booster              u64 length + bytes each
    GBTreeModelParam                        160 B: i32 num_trees, i32 num_roots,
                                            i32 num_feature, i32 pad, i64 num_pbuffer,
                                            i32 num_output_group, i32 size_leaf_vector,
                                            32 x i32 reserved
    num_trees x RegTree:
        TreeParam                           148 B: i32 num_roots, i32 num_nodes,
                                            i32 num_deleted, i32 max_depth,
                                            i32 num_feature, i32 size_leaf_vector,
                                            31 x i32 reserved
        num_nodes x Node                    20 B: i32 parent, i32 left, i32 right,
                                            u32 sindex (bit 31 = default left),
                                            f32 split_cond | leaf_value
        num_nodes x NodeStat                16 B: f32 loss_chg, f32 sum_hess,
                                            f32 base_weight, i32 leaf_child_cnt
        [u64 n + n x f32 leaf_vector]       only when size_leaf_vector != 0
    num_trees x i32 tree_info               output group of each tree
    [u64 n + n x f32 weight_drop]           dart only
    [u64 n + n x (str, str) attributes]     when contain_extra_attrs

Parity with real xgboost files is unpinned (no xgboost and no ``.bst``
fixture in the reference); the tests build files byte-by-byte from the layout
above and check them against the JSON path.
"""
from __future__ import annotations

import struct
from pathlib import Path
from typing import Any, Dict, List, Tuple, Union

import numpy as np

_DELETED = 0xFFFFFFFF


class _Reader:
    def __init__(self, buf: bytes, endian: str = "<"):
        self.b = memoryview(buf)
        self.o = 0
        self.e = endian

    def take(self, n: int) -> memoryview:
        if n < 0 or self.o + n > len(self.b):
            raise ValueError(f"truncated XGBoost model: need {n} bytes at offset {self.o}, have {len(self.b) - self.o}")
        v = self.b[self.o:self.o + n]
        self.o += n
        return v

    def unpack(self, fmt: str) -> Tuple:
        s = struct.Struct(self.e + fmt)
        return s.unpack(self.take(s.size))

    def array(self, dtype: str, n: int) -> np.ndarray:
        dt = np.dtype(dtype).newbyteorder(self.e)
        return np.frombuffer(self.take(n * dt.itemsize), dtype=dt).astype(dt.newbyteorder("="))

    def string(self) -> str:
        (n,) = self.unpack("Q")
        return bytes(self.take(n)).decode()

    def done(self) -> bool:
        return self.o >= len(self.b)


# ------------------------------------------------------------------ legacy binary
def parse_legacy_binary(buf: bytes) -> Dict[str, Any]:
    r = _Reader(buf)
    if bytes(r.b[:4]) == b"binf":
        r.take(4)
    base_score, num_feature, num_class, extra_attrs, _eval_metrics = r.unpack("fIiii")
    r.take(29 * 4)
    objective = r.string()
    booster = r.string()
    if booster not in ("gbtree", "dart"):
        raise ValueError(f"unsupported booster {booster!r} in XGBoost binary model")
    num_trees, _roots, gb_features, _pad, _pbuffer, _groups, _leaf_vec = r.unpack("iiiiqii")
    r.take(32 * 4)
    if num_trees < 0:
        raise ValueError("corrupt XGBoost binary model: negative tree count")
    trees: List[Dict[str, Any]] = []
    node_t = np.dtype([("parent", "<i4"), ("left", "<i4"), ("right", "<i4"), ("sindex", "<u4"), ("value", "<f4")])
    for _ in range(num_trees):
        _nr, num_nodes, _ndel, _md, _nf, size_leaf_vector = r.unpack("iiiiii")
        r.take(31 * 4)
        if num_nodes <= 0:
            raise ValueError("corrupt XGBoost binary model: tree with no nodes")
        nodes = np.frombuffer(r.take(num_nodes * node_t.itemsize), dtype=node_t)
        r.take(num_nodes * 16)  # NodeStat: training statistics, unused for inference
        if size_leaf_vector:
            (n,) = r.unpack("Q")
            r.take(n * 4)
        left = nodes["left"].astype(np.int64)
        right = nodes["right"].astype(np.int64)
        sidx = nodes["sindex"].astype(np.int64)
        deleted = sidx == _DELETED
        left[deleted] = -1
        right[deleted] = -1
        leaf = left < 0
        trees.append({"left_children": left, "right_children": np.where(leaf, -1, right),
                      "split_indices": np.where(leaf, 0, sidx & 0x7FFFFFFF),
                      "split_conditions": np.where(deleted, np.float32(0), nodes["value"]).astype(np.float32),
                      "default_left": np.where(leaf, 0, sidx >> 31).astype(np.int64)})
    tree_info = r.array("i4", num_trees).tolist() if num_trees else []
    gb: Dict[str, Any] = {"name": booster, "model": {"trees": trees, "tree_info": tree_info}}
    if booster == "dart":
        (n,) = r.unpack("Q")
        gb["weight_drop"] = r.array("f4", n).tolist()
    attrs: Dict[str, str] = {}
    if extra_attrs and not r.done():
        (n,) = r.unpack("Q")
        for _ in range(n):
            k = r.string()
            attrs[k] = r.string()
    return {"learner": {"learner_model_param": {"num_feature": str(max(num_feature, gb_features)),
                                                "num_class": str(num_class), "base_score": repr(float(base_score))},
                        "objective": {"name": objective}, "gradient_booster": gb, "attributes": attrs},
            "version": [0, 0, 0]}


# ------------------------------------------------------------------ UBJSON
_UBJ_SCALARS = {b"i": ("b", 1), b"U": ("B", 1), b"I": ("h", 2), b"l": ("i", 4), b"L": ("q", 8),
                b"d": ("f", 4), b"D": ("d", 8)}
_UBJ_NP = {b"i": "i1", b"U": "u1", b"I": "i2", b"l": "i4", b"L": "i8", b"d": "f4", b"D": "f8"}


def parse_ubjson(buf: bytes) -> Any:
    """Universal Binary JSON (big-endian), including the optimized ``$type
    #count`` containers XGBoost uses for its node arrays (returned as numpy
    arrays)."""
    r = _Reader(buf, ">")
    v = _ubj_value(r, bytes(r.take(1)))
    return v


def _ubj_int(r: _Reader) -> int:
    m = bytes(r.take(1))
    if m not in (b"i", b"U", b"I", b"l", b"L"):
        raise ValueError(f"UBJSON: expected an integer length, got {m!r}")
    return int(r.unpack(_UBJ_SCALARS[m][0])[0])


def _ubj_value(r: _Reader, m: bytes) -> Any:
    if m in _UBJ_SCALARS:
        return r.unpack(_UBJ_SCALARS[m][0])[0]
    if m == b"S" or m == b"H":
        n = _ubj_int(r)
        s = bytes(r.take(n)).decode()
        return float(s) if m == b"H" else s
    if m == b"C":
        return bytes(r.take(1)).decode()
    if m == b"Z":
        return None
    if m == b"T":
        return True
    if m == b"F":
        return False
    if m == b"[":
        return _ubj_container(r, array=True)
    if m == b"{":
        return _ubj_container(r, array=False)
    raise ValueError(f"UBJSON: unknown marker {m!r} at offset {r.o - 1}")


def _ubj_container(r: _Reader, array: bool) -> Any:
    typ = count = None
    m = bytes(r.take(1))
    if m == b"$":
        typ = bytes(r.take(1))
        m = bytes(r.take(1))
    if m == b"#":
        count = _ubj_int(r)
        m = None
    elif typ is not None:
        raise ValueError("UBJSON: a typed container needs a count")
    if array:
        if typ in _UBJ_NP and count is not None:
            return r.array(_UBJ_NP[typ], count)
        out: List[Any] = []
        while True:
            if count is not None:
                if len(out) == count:
                    return out
                out.append(_ubj_value(r, typ if typ is not None else bytes(r.take(1))))
            else:
                if m == b"]":
                    return out
                out.append(_ubj_value(r, m))
                m = bytes(r.take(1))
    obj: Dict[str, Any] = {}
    while True:
        if count is not None:
            if len(obj) == count:
                return obj
            key = bytes(r.take(_ubj_int(r))).decode()
            obj[key] = _ubj_value(r, typ if typ is not None else bytes(r.take(1)))
        else:
            if m == b"}":
                return obj
            r.o -= 1  # m was the key's length marker
            key = bytes(r.take(_ubj_int(r))).decode()
            obj[key] = _ubj_value(r, bytes(r.take(1)))
            m = bytes(r.take(1))


# ------------------------------------------------------------------ dispatch
def load_xgboost_model(src: Union[str, Path, bytes]) -> Dict[str, Any]:
    """JSON, UBJSON or legacy binary -> the JSON-schema dict (format sniffed
    from the content, not the file name)."""
    import json

    buf = Path(src).read_bytes() if not isinstance(src, (bytes, bytearray)) else bytes(src)
    head = buf.lstrip()[:2]
    if head[:1] == b"{" and (len(head) < 2 or head[1:2] in b'"}\n\r\t '):
        return json.loads(buf)
    if buf[:1] == b"{":
        return parse_ubjson(buf)
    return parse_legacy_binary(buf)
