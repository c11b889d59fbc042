"""Prepackaged model servers (reference servers/sklearnserver, servers/
xgboostserver, servers/mlflowserver, integrations/tfserving; operator wiring
operator/controllers/seldondeployment_prepackaged_servers.go:30-303).

Each server is a regular component (``predict``) *and* exposes
``row_model()``: when the model family has a native kernel the deployment binds
the GPU micro-batched unit instead of calling ``predict`` per request.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Any, Dict, Optional

import numpy as np

from ..utils.storage import Storage

logger = logging.getLogger(__name__)

JOBLIB_FILE = "model.joblib"
XGB_JSON_FILES = ("model.json", "model.bst.json", "model.ubj", "model.bst")


class SKLearnServer:
    """sklearn estimator from ``<modelUri>/model.joblib``; method predict_proba|predict."""

    def __init__(self, model_uri: str = "", method: str = "predict_proba", model: Any = None):
        self.model_uri = model_uri
        self.method = method
        self._model = model
        self.ready = model is not None

    def load(self) -> None:
        if self._model is None:
            import joblib

            path = os.path.join(Storage.download(self.model_uri), JOBLIB_FILE)
            self._model = joblib.load(path)
        self.ready = True

    def predict(self, X, names, meta=None):
        if not self.ready:
            self.load()
        fn = self._model.predict_proba if self.method == "predict_proba" else self._model.predict
        return fn(X)

    def row_model(self):
        if not self.ready:
            self.load()
        from ..models import to_row_model

        return to_row_model(self._model, self.method)


class XGBoostServer:
    """XGBoost booster from ``<modelUri>/model.{json,ubj,bst}``: XGBoost JSON,
    UBJSON or the legacy binary format (decoded without the xgboost library,
    ``models/xgb_binary.py``)."""

    def __init__(self, model_uri: str = "", ensemble=None):
        self.model_uri = model_uri
        self._ens = ensemble
        self.ready = ensemble is not None

    def load(self) -> None:
        if self._ens is None:
            from ..models import from_xgboost_json

            root = Storage.download(self.model_uri)
            path = root
            if os.path.isdir(root):
                cands = [os.path.join(root, f) for f in XGB_JSON_FILES if os.path.exists(os.path.join(root, f))]
                if not cands:
                    raise FileNotFoundError(f"no XGBoost model ({', '.join(XGB_JSON_FILES)}) in {root}")
                path = cands[0]
            self._ens = from_xgboost_json(path)
        self.ready = True

    def predict(self, X, names, meta=None):
        if not self.ready:
            self.load()
        return self._ens.predict(np.asarray(X, dtype=np.float64))

    def row_model(self):
        if not self.ready:
            self.load()
        from ..models import to_row_model

        return to_row_model(self._ens)


class MLFlowServer:
    """MLflow model directory (reference servers/mlflowserver/mlflowserver/
    MLFlowServer.py:17-45).  With an ``MLmodel`` file the flavour and its
    artifact come from it and the logged input signature is enforced
    (``servers/mlflow_model.py``).  Directories without ``MLmodel`` fall back to
    ``model.pt`` (TorchScript on the GPU) or ``model.joblib``/``model.pkl``."""

    def __init__(self, model_uri: str = "", device: Optional[str] = None):
        self.model_uri = model_uri
        self.device = device
        self.ready = False
        self._fn = None
        self._model = None
        self.flavour: Optional[str] = None
        self.signature = None

    def load(self) -> None:
        from .mlflow_model import MLMODEL_FILE, load_mlmodel, load_pytorch, load_sklearn

        root = Storage.download(self.model_uri)
        if os.path.isfile(os.path.join(root, MLMODEL_FILE)):
            mm, lf = load_mlmodel(root, self.device)
            self.signature = mm.signature
        elif os.path.exists(os.path.join(root, "model.pt")):
            lf = load_pytorch(os.path.join(root, "model.pt"), self.device)
        else:
            lf = None
            for f in ("model.joblib", "model.pkl"):
                p = os.path.join(root, f)
                if os.path.exists(p):
                    lf = load_sklearn(p)
                    break
            if lf is None:
                raise FileNotFoundError(f"no MLmodel file and no supported model flavour in {root}")
        self.flavour, self._fn, self._model = lf.flavour, lf.predict, lf.model
        self.ready = True

    def predict(self, X, names=None, meta=None):
        if not self.ready:
            self.load()
        if self.signature is not None:
            X = self.signature.enforce(X, list(names or ()))
        return self._fn(X)

    def row_model(self):
        """sklearn / xgboost flavours with a native kernel (linear, trees, MLP):
        the pyfunc ``predict`` is served by the GPU micro-batcher."""
        m = self._model
        if m is None:
            return None
        from ..models import to_row_model

        sig = self.signature
        if sig is not None and sig.columns:
            types = {c.get("type", "double") for c in sig.columns}
            if not types <= {"double", "float"}:
                return None  # integer / string columns: the Python path casts them
        rm = to_row_model(m, "predict") if self.flavour == "sklearn" else to_row_model(m)
        if rm is not None and sig is not None and sig.columns and all(sig.names):
            # named signature: the native unit permutes requests that name the
            # columns in another order (and rejects ones missing a column)
            rm.input_names = list(sig.names)
        return rm


class TFServingProxy:
    """TENSORFLOW_SERVER: the reference proxies to a TF Serving sidecar
    (integrations/tfserving/TfServingProxy.py).  With ``rest_endpoint`` (and
    ``model_name``) requests are forwarded to a TF Serving REST server; without
    one the model directory is served in-process (TorchScript export on the GPU
    via PyTorch-ROCm, or a scikit-learn flavour on the native kernels)."""

    def __init__(self, model_uri: str = "", rest_endpoint: str = "", model_name: str = "", **kw):
        self.model_uri = model_uri
        if rest_endpoint:
            from .proxies import TfServingRestProxy

            self._inner = TfServingRestProxy(rest_endpoint, model_name or "model", **kw)
        else:
            self._inner = MLFlowServer(model_uri)

    def load(self) -> None:
        if hasattr(self._inner, "load"):
            self._inner.load()

    def predict(self, X, names, meta=None):
        return self._inner.predict(X, names, meta)

    def row_model(self):
        rm = getattr(self._inner, "row_model", None)
        return rm() if callable(rm) else None


def load_prepackaged(impl: str, model_uri: str, params: Dict[str, Any]):
    p = {k: v for k, v in params.items() if k not in ("model_uri",)}
    if impl == "SKLEARN_SERVER":
        s = SKLearnServer(model_uri, method=p.get("method", "predict_proba"))
    elif impl == "XGBOOST_SERVER":
        s = XGBoostServer(model_uri)
    elif impl == "MLFLOW_SERVER":
        s = MLFlowServer(model_uri)
    elif impl == "TENSORFLOW_SERVER" and p.get("grpc_endpoint"):
        from .proxies import TfServingGrpcProxy

        kw = {k: p[k] for k in ("signature_name", "model_input", "model_output") if k in p}
        return TfServingGrpcProxy(p["grpc_endpoint"], p.get("model_name", "model"), **kw)
    elif impl == "TENSORFLOW_SERVER":
        s = TFServingProxy(model_uri, rest_endpoint=p.get("rest_endpoint", ""), model_name=p.get("model_name", ""))
    else:
        raise ValueError(f"unknown prepackaged server {impl}")
    s.load()
    return s
