"""The reference's example transformers / models / combiners,
with the same class names, constructor parameters and method signatures, but
backed by the engine's GPU kernels when they sit in a graph:

* ``MeanTransformer`` -- examples/transformers/mean_transformer/MeanTransformer.py:8-12:
  per-request global min-max normalisation -> native ``minmax`` row model
  (``segment_minmax`` kernel: one workgroup per request of a micro-batch).
* ``MeanClassifier`` -- examples/models/mean_classifier/MeanClassifier.py:19-27:
  ``sigmoid(mean(row) - threshold)`` -> native ``mean_sigmoid`` row model.
* ``MnistCombiner`` -- examples/combiners/mnist_combiner/MnistCombiner.py:8-11.
* ``OutputTransformer`` -- examples/output_transformers/OutputTransformer.py:9-11.
* ``ImageNetTransformer`` / ``ImageNetCombiner`` / ``ImageNetOutputTransformer``
  -- examples/models/openvino_imagenet_ensemble/resources/{transformer,combiner}:
  JPEG decode on the host, centre crop / resize / HWC->CHW on the GPU
  (``crop_resize_chw`` kernel), average of two model outputs
  (``combine_mean_f64``), argmax -> class name (``argmax_rows_f64``).
"""
from __future__ import annotations

import base64
import io
import json
import logging
import os
from typing import List, Optional

import numpy as np

from . import register

logger = logging.getLogger(__name__)


def _native():
    from .._native import native

    return native()


@register("MEAN_TRANSFORMER")
class MeanTransformer:
    def transform_input(self, X, feature_names):
        X = np.asarray(X, dtype=float)
        if X.max() == X.min():
            return np.zeros_like(X)
        return (X - X.min()) / (X.max() - X.min())

    def row_model(self):
        return _native().minmax_model()


@register("MEAN_CLASSIFIER")
class MeanClassifier:
    def __init__(self, intValue: int = 0, model_path: str = "model.npy", threshold: Optional[float] = None):
        if not isinstance(intValue, int):
            raise TypeError("intValue parameters must be an integer")
        self.class_names = ["proba"]
        self.int_value = intValue
        if threshold is None:
            base = 0.0
            if os.path.exists(model_path):
                base = float(np.load(model_path, allow_pickle=False).mean())
            threshold = base + intValue
        self.threshold_ = float(threshold)

    def predict(self, X, feature_names):
        X = np.asarray(X, dtype=float)
        if X.ndim != 2:
            raise ValueError("Incorrect shape")
        return 1.0 / (1.0 + np.exp(-(X.mean(axis=1, keepdims=True) - self.threshold_)))

    def row_model(self):
        m = _native().mean_sigmoid_model(self.threshold_)
        m.set_class_names(self.class_names)
        return m


@register("MNIST_COMBINER")
class MnistCombiner:
    def __init__(self, metrics_ok: bool = True):
        pass

    def aggregate(self, Xs, features_names):
        return (np.asarray(Xs[0]) + np.asarray(Xs[1])) / 2.0


@register("APPEND_ONE_OUTPUT_TRANSFORMER")
class OutputTransformer:
    def transform_output(self, X, names):
        return np.vstack((X, np.array([1])))


def _tftensor_json(arr: np.ndarray) -> dict:
    return {"dtype": "DT_FLOAT", "tensorShape": {"dim": [{"size": str(int(d))} for d in arr.shape]},
            "tensorContent": base64.b64encode(np.ascontiguousarray(arr, dtype="<f4").tobytes()).decode()}


def _tftensor_array(t: dict) -> np.ndarray:
    shape = [int(d.get("size", 0)) for d in (t.get("tensorShape") or {}).get("dim", [])]
    if t.get("tensorContent"):
        dt = {"DT_FLOAT": "<f4", "DT_DOUBLE": "<f8"}.get(t.get("dtype", "DT_FLOAT"), "<f4")
        a = np.frombuffer(base64.b64decode(t["tensorContent"]), dtype=dt)
    else:
        a = np.asarray(t.get("floatVal") or t.get("doubleVal") or [], dtype=np.float64)
    return a.reshape(shape) if shape else a


@register("IMAGENET_TRANSFORMER")
class ImageNetTransformer:
    def __init__(self, metrics_ok: bool = True, size: int = 224, classes: int = 1000, device: Optional[int] = None):
        self.size = int(os.environ.get("SIZE", size))
        self.classes = int(os.environ.get("CLASSES", classes))
        self.device = device

    def _use_gpu(self) -> bool:
        try:
            import torch

            return torch.cuda.is_available() and self.device != -1
        except Exception:
            return False

    def preprocess(self, jpeg: bytes) -> np.ndarray:
        from PIL import Image

        img = np.asarray(Image.open(io.BytesIO(jpeg)).convert("RGB"))[:, :, ::-1]  # BGR, as cv2.imdecode
        img = np.ascontiguousarray(img)
        if self._use_gpu():
            import torch

            from .. import ops

            with _side_stream(self, self.device or 0):
                t = torch.from_numpy(img).cuda(self.device or 0)
                out = ops.crop_resize_chw(t, self.size).cpu().numpy()
        else:
            from ..ops import crop_resize_chw_ref

            out = crop_resize_chw_ref(img, self.size)
        return out.reshape(1, 3, self.size, self.size)

    def transform_input_raw(self, request: dict) -> dict:
        jpeg = base64.b64decode(request["binData"]) if isinstance(request.get("binData"), str) else request["binData"]
        X = self.preprocess(jpeg)
        # the array itself: inside an engine graph it becomes a dense tftensor
        # message with no JSON / base64 round trip (PythonUnit.call_json); a
        # JSON reply (dispatch path) encodes it as the reference's TensorProto
        return {"data": {"names": ["x"], "tftensor": X}}


def _side_stream(obj, dev: int):
    """The component's own (non-blocking) stream: its GPU work must not sit
    on the null stream, which orders it behind every other component's
    (e.g. the ensemble's CNN graphs) -- see models/cnn.py CompiledCnn.__call__."""
    import torch

    st = obj.__dict__.get("_stream")
    if st is None:
        st = obj.__dict__["_stream"] = torch.cuda.Stream(torch.device(f"cuda:{dev}"))
    return torch.cuda.stream(st)


def _gpu_device(device: Optional[int]) -> Optional[int]:
    """GPU ordinal for a component's kernels, or None (CPU placement / no GPU)."""
    if device is not None and device < 0:
        return None
    try:
        import torch

        return (device or 0) if torch.cuda.is_available() else None
    except Exception:
        return None


@register("IMAGENET_COMBINER")
class ImageNetCombiner:
    """Average of the two model outputs (resources/combiner: (Xs[0] + Xs[1]) / 2)
    -- on a GPU the ``combine_mean_f64`` kernel (csrc/kernels/combine.hip)."""

    def __init__(self, device: Optional[int] = None):
        self.device = device
        self.gpu_calls = 0

    def aggregate(self, Xs, features_names):
        dev = _gpu_device(self.device)
        if dev is not None:
            import torch

            from .. import ops

            with _side_stream(self, dev):
                ts = [torch.as_tensor(np.reshape(np.asarray(x, dtype=np.float64), (1, -1)), device=f"cuda:{dev}")
                      for x in Xs[:2]]
                self.gpu_calls += 1
                return ops.combine_mean(ts).cpu().numpy()
        return (np.reshape(Xs[0], (1, -1)) + np.reshape(Xs[1], (1, -1))) / 2.0


@register("IMAGENET_OUTPUT_TRANSFORMER")
class ImageNetOutputTransformer:
    def __init__(self, classes: int = 1000, class_names_path: str = "", device: Optional[int] = None):
        self.device = device
        self.gpu_calls = 0
        self.classes = int(os.environ.get("CLASSES", classes))
        self.cnames: List[str] = [str(i) for i in range(self.classes)]
        if class_names_path and os.path.exists(class_names_path):
            with open(class_names_path) as f:
                names = json.load(f)  # JSON list or {index: name}
            self.cnames = [names[str(i)] if isinstance(names, dict) else names[i] for i in range(self.classes)]

    def transform_output_raw(self, request: dict) -> dict:
        data = request.get("data") or {}
        if "tftensor" in data:
            result = _tftensor_array(data["tftensor"])
        elif "tensor" in data:
            result = np.asarray(data["tensor"]["values"], dtype=float)
        else:
            result = np.asarray(data.get("ndarray"), dtype=float)
        result = np.reshape(np.asarray(result, dtype=np.float64), (1, self.classes))
        dev = _gpu_device(self.device)
        if dev is not None:  # argmax_rows_f64 kernel (first maximum, as np.argmax)
            import torch

            from .. import ops

            self.gpu_calls += 1
            with _side_stream(self, dev):
                idx = int(ops.argmax_rows(torch.as_tensor(result, device=f"cuda:{dev}")).cpu()[0])
        else:
            idx = int(np.argmax(result[0]))
        return {"strData": self.cnames[idx]}


class IrisClassifier:
    """The reference's user-class example (examples/models/sklearn_iris/
    IrisClassifier.py:3-10): a plain Python class whose ``predict`` calls a
    scikit-learn LogisticRegression.  It stays a *Python* component (the
    wrapper-microservice workload), unlike ``SKLearnServer`` which compiles the
    model to a kernel.  ``model`` defaults to the iris fit from sklearn's
    bundled dataset (no joblib file or network needed)."""

    def __init__(self, model=None):
        if model is None:
            from ..models import iris_logistic_regression

            model = iris_logistic_regression()
        self.model = model

    def predict(self, X, features_names):
        return self.model.predict_proba(X)


class EchoModel:
    """No-op user component: returns its input (Python-runtime overhead probe)."""

    def predict(self, X, features_names):
        return X


@register("IMAGENET_MODEL")
class ImageNetModel:
    """The ensemble's two MODEL nodes (resources/model/Prediction.py:70-104:
    an OpenVINO DenseNet-169 / ResNet-50 ``exec_net.infer`` on ``[1, 3, 224,
    224]``, float64 probabilities back), here a :mod:`seldon_core_amd.models.cnn`
    network on PyTorch-ROCm: BN folded into the convolutions, bf16 NHWC on the
    matrix cores, one captured HIP graph per batch bucket.

    ``seldon_batching``: concurrent requests reach ``predict`` as one stacked
    ``[B, 3, H, W]`` batch (up to ``max_batch`` images), one graph launch.
    ``device=-1`` (or no GPU) runs the folded fp32 network on the CPU.
    """

    def __init__(self, arch: str = "resnet50", weights: str = "", device: Optional[int] = None, dtype: str = "bf16",
                 max_batch: int = 32, graphs: bool = True, seed: int = 0, image: int = 224, tune: bool = True):
        from ..models import cnn

        self.arch = arch
        self.image = int(image)
        self.seldon_batching = int(max_batch)
        net = cnn.build(arch, weights=weights, seed=int(seed))
        dev = _gpu_device(device)
        self.gpu = dev is not None
        if self.gpu:
            self.net = cnn.CompiledCnn(net, device=dev, dtype=dtype, max_batch=int(max_batch), graphs=bool(graphs),
                                       image=self.image, tune=bool(tune))
            if self.net.graph_error:
                logger.warning("%s: HIP graph capture failed (%s); serving eagerly", arch, self.net.graph_error)
        else:
            self.cpu_net = cnn.fold_for_inference(net).float()
        self.calls = 0
        self.images = 0

    def predict(self, X, feature_names):
        X = np.asarray(X)
        X = X.reshape(-1, 3, self.image, self.image)
        self.calls += 1
        self.images += X.shape[0]
        if self.gpu:
            return self.net(X)
        import torch

        with torch.no_grad():
            return torch.softmax(self.cpu_net(torch.from_numpy(X.astype(np.float32))), 1).double().numpy()
