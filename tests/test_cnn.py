"""ImageNet CNNs for the reference's OpenVINO ensemble
(examples/models/openvino_imagenet_ensemble: DenseNet-169 + ResNet-50 MODEL
nodes, resources/model/Prediction.py:70-104) -- models/cnn.py and the
IMAGENET_MODEL component.

Parity is pinned where something public pins it: the parameter counts of the
two architectures (torchvision's published 25,557,032 and 14,149,480) and its
state_dict names.  No trained weights or OpenVINO runtime exist here, so
outputs are checked against the same network in fp32 on the CPU."""
import base64
import concurrent.futures as cf
import io

import numpy as np
import pytest
import torch

import seldon_core_amd as sca
from seldon_core_amd.components.examples import ImageNetModel
from seldon_core_amd.models import cnn


@pytest.mark.parametrize("arch,params", [("resnet50", 25_557_032), ("densenet169", 14_149_480),
                                         ("resnet101", 44_549_160), ("densenet121", 7_978_856)])
def test_architecture_parameter_counts(arch, params):
    m = cnn.ARCHS[arch]()
    assert sum(p.numel() for p in m.parameters()) == params


def test_torchvision_state_dict_names():
    r = cnn.ARCHS["resnet50"]().state_dict()
    for k in ("conv1.weight", "bn1.running_var", "layer1.0.downsample.0.weight", "layer4.2.bn3.bias", "fc.weight"):
        assert k in r
    d = cnn.ARCHS["densenet169"]().state_dict()
    for k in ("features.conv0.weight", "features.denseblock3.denselayer32.conv2.weight",
              "features.transition2.norm.running_mean", "features.norm5.weight", "classifier.bias"):
        assert k in d


@pytest.mark.parametrize("arch", ["resnet50", "densenet169"])
def test_batchnorm_folding_is_exact(arch):
    net = cnn.build(arch, seed=3)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(0)) * 255
    with torch.no_grad():
        a = net(x)
        b = cnn.fold_for_inference(cnn.build(arch, seed=3))(x)
    torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-4 * float(a.abs().max()))
    assert float(torch.softmax(a, 1).max()) < 0.9  # the random init is not degenerate


def test_weights_roundtrip_through_safetensors(tmp_path):
    from safetensors.torch import save_file

    src = cnn.build("resnet50", seed=7)
    path = str(tmp_path / "r50.safetensors")
    save_file({k: v.contiguous() for k, v in src.state_dict().items()}, path)
    pt = str(tmp_path / "r50.pt")
    torch.save(src.state_dict(), pt)
    x = torch.rand(1, 3, 64, 64)
    with torch.no_grad():
        want = src(x)
        for p in (path, pt):
            torch.testing.assert_close(cnn.build("resnet50", weights=p)(x), want, rtol=0, atol=0)
    bad = str(tmp_path / "bad.safetensors")
    save_file({"fc.weight": torch.zeros(3, 3)}, bad)
    with pytest.raises(Exception):
        cnn.build("resnet50", weights=bad)


def _png(h, w, seed):
    from PIL import Image

    img = (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="PNG")
    return b.getvalue()


def _P(n, v, t="INT"):
    return {"name": n, "value": str(v), "type": t}


def _ensemble(device, size):
    """The reference's seldon_ov_predict_ensemble.json graph: output
    transformer <- transformer <- combiner <- (DenseNet-169, ResNet-50)."""
    models = [{"name": n, "type": "MODEL", "implementation": "IMAGENET_MODEL",
               "parameters": [_P("arch", a, "STRING"), _P("image", size), _P("device", device)]}
              for n, a in (("prediction1", "densenet169"), ("prediction2", "resnet50"))]
    return {"name": "imagenet-otransformer", "type": "OUTPUT_TRANSFORMER",
            "implementation": "IMAGENET_OUTPUT_TRANSFORMER",
            "children": [{"name": "imagenet-itransformer", "type": "TRANSFORMER",
                          "implementation": "IMAGENET_TRANSFORMER", "parameters": [_P("size", size)],
                          "children": [{"name": "imagenet-combiner", "type": "COMBINER",
                                        "implementation": "IMAGENET_COMBINER", "children": models}]}]}


def test_ensemble_graph_on_cpu_matches_the_networks_and_batches_concurrent_images():
    size = 64
    comps = {"prediction1": ImageNetModel("densenet169", device=-1, image=size, max_batch=8),
             "prediction2": ImageNetModel("resnet50", device=-1, image=size, max_batch=8)}
    spec = {"name": "p", "graph": _ensemble(-1, size), "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=-1, components=comps)
    try:
        from seldon_core_amd.components.examples import ImageNetTransformer

        tr = ImageNetTransformer(device=-1, size=size)
        imgs = [_png(70 + i, 90, i) for i in range(12)]
        with cf.ThreadPoolExecutor(12) as ex:
            outs = list(ex.map(lambda b: dep.predict({"binData": base64.b64encode(b).decode()}), imgs))
        nets = [cnn.fold_for_inference(cnn.build(a)) for a in ("densenet169", "resnet50")]
        for b, o in zip(imgs, outs):
            x = torch.from_numpy(tr.preprocess(b).astype(np.float32))
            with torch.no_grad():
                p = sum(torch.softmax(n(x), 1) for n in nets) / 2
            assert o["strData"] == str(int(p.argmax()))
        assert comps["prediction1"].images == 12
        assert comps["prediction1"].calls < 12  # concurrent images were stacked into shared calls
    finally:
        dep.close()


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["resnet50", "densenet169"])
def test_compiled_cnn_bf16_graphs_match_fp32(arch):
    """bf16 NHWC through captured HIP graphs vs the fp32 network on the CPU:
    probabilities within 6% relative + 3e-4 absolute (bf16 through 169 layers;
    measured worst 3.3% on DenseNet's largest probability), top-1 equal on 90%
    of images, for batches that hit a bucket exactly, pad into one, and span
    several."""
    net = cnn.build(arch, seed=1)
    # tune=False keeps the test short (MIOpen's solver search is 44-128 s on a fresh box)
    m = cnn.CompiledCnn(cnn.build(arch, seed=1), device=0, dtype="bf16", max_batch=8, graphs=True,
                        tune=arch == "resnet50")
    assert m.graphs and m.graph_error is None, m.graph_error
    for n in (1, 3, 8, 11):
        x = torch.rand(n, 3, 224, 224, generator=torch.Generator().manual_seed(n)) * 255
        with torch.no_grad():
            ref = torch.softmax(net(x), 1).double().numpy()
        got = m(x.numpy().astype(np.float64))
        assert got.shape == (n, 1000)
        np.testing.assert_allclose(got, ref, rtol=0.06, atol=3e-4)
        assert (got.argmax(1) == ref.argmax(1)).mean() >= 0.9


@pytest.mark.gpu
def test_ensemble_graph_on_gpu():
    size = 224
    comps = {"prediction1": ImageNetModel("densenet169", device=0, max_batch=8, tune=False),
             "prediction2": ImageNetModel("resnet50", device=0, max_batch=8, tune=False)}
    assert comps["prediction1"].gpu and comps["prediction1"].net.graphs
    spec = {"name": "p", "graph": _ensemble(0, size), "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=0, components=comps)
    try:
        imgs = [_png(300, 260 + i, i) for i in range(16)]
        with cf.ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(lambda b: dep.predict({"binData": base64.b64encode(b).decode()}), imgs))
        assert all(o.get("strData", "").isdigit() for o in outs)
        assert comps["prediction2"].images == 16
    finally:
        dep.close()


def test_example_spec_serves_a_jpeg_on_cpu():
    """examples/imagenet/seldon_imagenet_ensemble.json: the reference's
    ensemble graph, node names and all, answering one binData request."""
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "imagenet",
                        "seldon_imagenet_ensemble.json")
    dep = sca.Deployment(path, device=-1)
    try:
        out = dep.predict({"binData": base64.b64encode(_png(240, 320, 5)).decode()})
        assert out["strData"].isdigit() and 0 <= int(out["strData"]) < 1000
        assert set(out["meta"]["requestPath"]) == {"imagenet-otransformer", "imagenet-itransformer",
                                                   "imagenet-combiner", "prediction1", "prediction2"}
    finally:
        dep.close()


def test_folding_twice_is_a_no_op():
    net = cnn.build("densenet121", seed=2)
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(1)) * 255
    with torch.no_grad():
        once = cnn.fold_for_inference(net)
        a = once(x)
        b = cnn.fold_for_inference(once)(x)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
