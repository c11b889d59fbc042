"""Example components against numpy re-statements of the
reference classes (examples/transformers/mean_transformer, models/mean_classifier,
combiners/mnist_combiner, output_transformers, openvino_imagenet_ensemble)."""
import base64
import concurrent.futures as cf
import io
import json
import os

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components.examples import (ImageNetCombiner, ImageNetOutputTransformer, ImageNetTransformer,
                                                  MeanClassifier, MeanTransformer, MnistCombiner, OutputTransformer)
from seldon_core_amd.ops import crop_resize_chw_ref
from seldon_core_amd.serving.codec import dumps

REF_NPY = "/root/reference/examples/models/mean_classifier/model.npy"


def _spec(graph):
    return {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}


def _ref_minmax(X):
    X = np.asarray(X, float)
    return np.zeros_like(X) if X.max() == X.min() else (X - X.min()) / (X.max() - X.min())


def test_mean_transformer_python_api():
    X = np.array([[1.0, 2.0], [3.0, 5.0]])
    np.testing.assert_allclose(MeanTransformer().transform_input(X, []), _ref_minmax(X))
    assert (MeanTransformer().transform_input(np.ones((2, 2)), []) == 0).all()


@pytest.mark.skipif(not os.path.exists(REF_NPY), reason="reference fixture absent")
def test_mean_classifier_threshold_from_reference_fixture():
    m = MeanClassifier(intValue=1, model_path=REF_NPY)
    base = np.load(REF_NPY, allow_pickle=False).mean()
    assert m.threshold_ == pytest.approx(base + 1)
    X = np.array([[0.0, 1.0, 2.0]])
    want = [[1 / (1 + np.exp(-(x.mean() - m.threshold_)))] for x in X]
    np.testing.assert_allclose(m.predict(X, []), want)


@pytest.mark.parametrize("device", [-1])
def test_transformer_classifier_chain_native(device):
    graph = {"name": "mt", "type": "TRANSFORMER", "implementation": "MEAN_TRANSFORMER",
             "children": [{"name": "mc", "type": "MODEL", "implementation": "MEAN_CLASSIFIER",
                           "parameters": [{"name": "threshold", "value": "0.25", "type": "FLOAT"}]}]}
    dep = sca.Deployment(_spec(graph), device=device)
    try:
        assert dep.fused  # both are native row models -> one device graph
        X = np.array([[1.0, 4.0, 9.0], [2.0, 3.0, 5.0]])
        out = dep.predict({"data": {"names": ["a", "b", "c"], "ndarray": X.tolist()}})
        want = 1 / (1 + np.exp(-(_ref_minmax(X).mean(axis=1, keepdims=True) - 0.25)))
        np.testing.assert_allclose(out["data"]["ndarray"], want, rtol=1e-12)
        assert out["data"]["names"] == ["proba"]
    finally:
        dep.close()


def test_mnist_combiner_and_output_transformer():
    a, b = np.array([[0.2, 0.8]]), np.array([[0.4, 0.6]])
    np.testing.assert_allclose(MnistCombiner().aggregate([a, b], []), (a + b) / 2)
    np.testing.assert_array_equal(OutputTransformer().transform_output(np.array([[3]]), []), [[3], [1]])


def _jpeg(h, w, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    img = (rng.random((h, w, 3)) * 255).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG")  # lossless so the decode is exact
    return buf.getvalue(), img


@pytest.mark.parametrize("hw", [(256, 300), (180, 400), (100, 150)])
def test_imagenet_transformer_cpu(hw):
    data, img = _jpeg(*hw)
    t = ImageNetTransformer(device=-1, size=64)
    out = t.transform_input_raw({"binData": base64.b64encode(data).decode()})
    assert isinstance(out["data"]["tftensor"], np.ndarray)  # dense inside a graph (PythonUnit.call_json)
    tf = json.loads(dumps(out))["data"]["tftensor"]  # the reference's TensorProto JSON on the wire
    assert tf["dtype"] == "DT_FLOAT"
    arr = np.frombuffer(base64.b64decode(tf["tensorContent"]), dtype="<f4").reshape(1, 3, 64, 64)
    bgr = np.ascontiguousarray(img[:, :, ::-1])
    np.testing.assert_array_equal(arr[0], crop_resize_chw_ref(bgr, 64))
    if hw[0] >= 64 and hw[1] >= 64:  # pure crop: exact pixels
        y0, x0 = hw[0] // 2 - 32, hw[1] // 2 - 32
        np.testing.assert_array_equal(arr[0], bgr[y0:y0 + 64, x0:x0 + 64].transpose(2, 0, 1).astype(np.float32))


def test_imagenet_combiner_and_output():
    x0, x1 = np.zeros((1, 10)), np.zeros((1, 10))
    x0[0, 3], x1[0, 3] = 1.0, 0.5
    avg = ImageNetCombiner(device=-1).aggregate([x0, x1], [])
    assert avg.shape == (1, 10) and avg[0, 3] == 0.75
    o = ImageNetOutputTransformer(classes=10, device=-1)
    assert o.transform_output_raw({"data": {"ndarray": avg.tolist()}}) == {"strData": "3"}


@pytest.mark.gpu
def test_imagenet_combiner_and_output_on_kernels():
    rng = np.random.default_rng(1)
    x0, x1 = rng.normal(size=(1, 1000)), rng.normal(size=(1, 1000))
    comb = ImageNetCombiner(device=0)
    avg = comb.aggregate([x0, x1], [])
    np.testing.assert_allclose(avg, (x0 + x1) / 2, rtol=0, atol=1e-15)
    o = ImageNetOutputTransformer(classes=1000, device=0)
    out = o.transform_output_raw({"data": {"tensor": {"shape": [1, 1000], "values": avg.ravel().tolist()}}})
    assert out == {"strData": str(int(np.argmax(avg[0])))}
    assert comb.gpu_calls == 1 and o.gpu_calls == 1


@pytest.mark.gpu
def test_mean_transformer_gpu_per_request_segments():
    """Concurrent requests share micro-batches; each must be normalised by its
    own min/max (segment_minmax kernel)."""
    graph = {"name": "mt", "type": "TRANSFORMER", "implementation": "MEAN_TRANSFORMER"}
    dep = sca.Deployment(_spec(graph), device=0, batcher={"max_wait_us": 200})
    try:
        assert dep.engine.unit_kind("mt") == "gpu:minmax"
        rng = np.random.default_rng(0)
        reqs = [rng.normal(size=(1 + i % 5, 6)) * (i + 1) for i in range(64)]
        with cf.ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(lambda X: dep.predict({"data": {"ndarray": X.tolist()}}), reqs))
        for X, o in zip(reqs, outs):
            np.testing.assert_allclose(o["data"]["ndarray"], _ref_minmax(X), rtol=1e-12, atol=1e-15)
        assert dep.batcher_stats()["mt"]["batches"] < 64  # they really were batched together
    finally:
        dep.close()
