"""MLflow model-directory semantics without the ``mlflow`` package.

The reference's MLFLOW_SERVER hands the downloaded directory to
``mlflow.pyfunc.load_model`` (servers/mlflowserver/mlflowserver/MLFlowServer.py:23-27),
which reads the ``MLmodel`` YAML at the directory root, picks the flavour's
artifact and wraps it in a pyfunc whose ``predict`` enforces the logged input
signature.  mlflow is not importable here, so this module reads ``MLmodel``
itself (``yaml.safe_load``) and loads the artifact of the first flavour it can
run natively:

* ``sklearn``  -> ``pickled_model`` (pickle / cloudpickle-compatible pickle);
  the estimator also gets the native GPU row model (linear, trees, MLP).
* ``xgboost``  -> ``data`` (JSON, UBJSON or legacy binary booster) decoded by
  ``models.from_xgboost_json`` -> GPU tree kernel.
* ``pytorch``  -> ``model_data`` (a TorchScript file, or a directory holding
  ``model.pth``/``model.pt``) executed by PyTorch-ROCm on the GPU.
* ``python_function`` whose ``loader_module`` is one of ``mlflow.sklearn``,
  ``mlflow.xgboost`` or ``mlflow.pytorch`` -> the same loaders on its ``data``.

The ``signature`` block (column-based ``[{"name", "type"}]`` or tensor-based
``[{"type": "tensor", "tensor-spec": {...}}]``) is enforced the pyfunc way:
named request columns are reordered to the schema's order, the column count is
checked and values are cast to the schema's types.  Parity with mlflow itself is
unpinned (the library is absent); the tests pin the behaviour on hand-written
``MLmodel`` files of the layouts mlflow 1.x writes.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

MLMODEL_FILE = "MLmodel"

# pyfunc loader modules this server can stand in for -> native flavour name
_LOADER_MODULES = {"mlflow.sklearn": "sklearn", "mlflow.xgboost": "xgboost", "mlflow.pytorch": "pytorch"}
# preference order when several flavours are present: native kernels first
_FLAVOUR_ORDER = ("sklearn", "xgboost", "pytorch")

_COLUMN_TYPES = {
    "double": np.float64,
    "float": np.float32,
    "long": np.int64,
    "integer": np.int32,
    "boolean": np.bool_,
}
_TENSOR_TYPES = {
    "float64": np.float64, "float32": np.float32, "float16": np.float16,
    "int64": np.int64, "int32": np.int32, "int16": np.int16, "int8": np.int8,
    "uint8": np.uint8, "bool": np.bool_,
}


class MLmodelError(ValueError):
    pass


@dataclass
class Signature:
    """Parsed ``signature.inputs``: either named columns or one tensor spec."""

    columns: List[Dict[str, str]] = field(default_factory=list)
    tensor_dtype: Optional[Any] = None
    tensor_shape: Optional[List[int]] = None

    @property
    def names(self) -> List[str]:
        return [c.get("name", "") for c in self.columns]

    def enforce(self, X: np.ndarray, feature_names: Sequence[str] = ()) -> np.ndarray:
        X = np.asarray(X)
        if self.columns:
            if X.ndim == 1:
                X = X.reshape(1, -1)
            n = len(self.columns)
            names = self.names
            if feature_names and all(names) and len(feature_names) == X.shape[1]:
                idx = {f: i for i, f in enumerate(feature_names)}
                missing = [c for c in names if c not in idx]
                if missing:
                    raise MLmodelError(f"request is missing signature column(s) {missing}")
                X = X[:, [idx[c] for c in names]]
            if X.shape[1] != n:
                raise MLmodelError(f"signature expects {n} column(s), request has {X.shape[1]}")
            types = {c.get("type", "double") for c in self.columns}
            if len(types) == 1:
                t = _COLUMN_TYPES.get(types.pop())
                if t is not None:
                    X = X.astype(t, copy=False)
            return X
        if self.tensor_dtype is not None:
            X = X.astype(self.tensor_dtype, copy=False)
            if self.tensor_shape:
                want = self.tensor_shape
                if len(want) != X.ndim or any(w != -1 and w != s for w, s in zip(want, X.shape)):
                    raise MLmodelError(f"signature expects tensor shape {want}, request has {list(X.shape)}")
        return X


def parse_signature(sig: Any) -> Optional[Signature]:
    if not isinstance(sig, dict) or "inputs" not in sig:
        return None
    inputs = sig["inputs"]
    if isinstance(inputs, str):
        inputs = json.loads(inputs)
    if not isinstance(inputs, list) or not inputs:
        return None
    if all(isinstance(c, dict) and c.get("type") == "tensor" for c in inputs):
        spec = inputs[0].get("tensor-spec", {})
        dt = _TENSOR_TYPES.get(str(spec.get("dtype", "")))
        return Signature(tensor_dtype=dt, tensor_shape=list(spec.get("shape", [])) or None)
    cols = [c for c in inputs if isinstance(c, dict)]
    for c in cols:
        if c.get("type", "double") not in _COLUMN_TYPES:
            raise MLmodelError(f"unsupported signature column type {c.get('type')!r}")
    return Signature(columns=cols)


@dataclass
class MLModel:
    root: str
    flavors: Dict[str, Dict[str, Any]]
    signature: Optional[Signature]
    raw: Dict[str, Any]

    @classmethod
    def read(cls, root: str) -> "MLModel":
        import yaml

        path = os.path.join(root, MLMODEL_FILE)
        with open(path, "r", encoding="utf-8") as f:
            doc = yaml.safe_load(f) or {}
        if not isinstance(doc, dict) or not isinstance(doc.get("flavors"), dict):
            raise MLmodelError(f"{path}: no 'flavors' mapping")
        return cls(root=root, flavors=doc["flavors"], signature=parse_signature(doc.get("signature")), raw=doc)

    def choose(self) -> tuple:
        """-> (flavour name, artifact path) of the first flavour we can run."""
        for fl in _FLAVOUR_ORDER:
            conf = self.flavors.get(fl)
            if isinstance(conf, dict):
                key = {"sklearn": "pickled_model", "xgboost": "data", "pytorch": "model_data"}[fl]
                if key in conf:
                    return fl, self._artifact(conf[key])
        pf = self.flavors.get("python_function")
        if isinstance(pf, dict):
            fl = _LOADER_MODULES.get(str(pf.get("loader_module", "")))
            if fl and "data" in pf:
                return fl, self._artifact(pf["data"])
            raise MLmodelError(
                f"python_function loader_module {pf.get('loader_module')!r} needs the mlflow package; "
                f"supported: {sorted(_LOADER_MODULES)}")
        raise MLmodelError(f"no supported flavour in {sorted(self.flavors)}; supported: {list(_FLAVOUR_ORDER)}")

    def _artifact(self, rel: str) -> str:
        p = os.path.normpath(os.path.join(self.root, str(rel)))
        root = os.path.normpath(self.root)
        if os.path.commonpath([p, root]) != root:
            raise MLmodelError(f"artifact path {rel!r} escapes the model directory")
        if not os.path.exists(p):
            raise MLmodelError(f"artifact {rel!r} listed in MLmodel does not exist")
        return p


@dataclass
class LoadedFlavour:
    flavour: str
    predict: Callable[[np.ndarray], Any]
    model: Any = None  # sklearn estimator / tree ensemble (native row model source)


def load_sklearn(path: str) -> LoadedFlavour:
    import pickle

    if path.endswith(".joblib"):
        import joblib

        m = joblib.load(path)
    else:
        with open(path, "rb") as f:
            m = pickle.load(f)  # user-provided model artifact, as pyfunc does
    return LoadedFlavour("sklearn", m.predict, m)


def load_xgboost(path: str) -> LoadedFlavour:
    from ..models import from_xgboost_json

    if os.path.isdir(path):
        cands = [os.path.join(path, f) for f in sorted(os.listdir(path))
                 if f.endswith((".json", ".ubj", ".bst", ".xgb", ".model"))]
        if not cands:
            raise MLmodelError(f"no booster file in {path}")
        path = cands[0]
    ens = from_xgboost_json(path)
    return LoadedFlavour("xgboost", lambda X: ens.predict(np.asarray(X, dtype=np.float64)), ens)


def load_pytorch(path: str, device: Optional[str] = None) -> LoadedFlavour:
    import torch

    if os.path.isdir(path):
        for f in ("model.pth", "model.pt"):
            if os.path.exists(os.path.join(path, f)):
                path = os.path.join(path, f)
                break
        else:
            raise MLmodelError(f"no model.pth / model.pt in {path}")
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    try:
        mod = torch.jit.load(path, map_location=dev)
    except RuntimeError:
        # mlflow.pytorch pickles the whole nn.Module: a user artifact, loaded as pyfunc would
        mod = torch.load(path, map_location=dev, weights_only=False)
    mod.eval()
    if str(dev).startswith("cuda") and os.environ.get("SCA_TORCH_GRAPHS", "1") != "0":
        # one captured HIP graph per batch bucket instead of a launch per op
        from ..models.graphed import GraphedModule

        gm = GraphedModule(mod, device=torch.device(dev).index or 0)

        def graphed(X):
            return gm(np.asarray(X, dtype=np.float32))

        graphed.graphed = gm  # replay / eager counters for tests and stats
        return LoadedFlavour("pytorch", graphed, None)

    def fn(X):
        with torch.no_grad():
            t = torch.as_tensor(np.asarray(X, dtype=np.float32), device=dev)
            return mod(t).float().cpu().numpy()

    return LoadedFlavour("pytorch", fn, None)


def load_mlmodel(root: str, device: Optional[str] = None) -> tuple:
    """-> (MLModel, LoadedFlavour) for a directory holding an ``MLmodel`` file."""
    mm = MLModel.read(root)
    fl, path = mm.choose()
    if fl == "sklearn":
        lf = load_sklearn(path)
    elif fl == "xgboost":
        lf = load_xgboost(path)
    else:
        lf = load_pytorch(path, device)
    return mm, lf
