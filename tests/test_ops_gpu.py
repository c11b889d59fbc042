"""Numerics of the torch-facing HIP ops vs plain PyTorch / numpy fp64
references (GPU only)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def test_linear_softmax_matches_torch(torch):
    from seldon_core_amd import ops

    g = torch.Generator().manual_seed(0)
    X = torch.randn(1000, 37, dtype=torch.float64, generator=g)
    W = torch.randn(11, 37, dtype=torch.float64, generator=g)
    b = torch.randn(11, dtype=torch.float64, generator=g)
    out = ops.linear(X.cuda(), W.cuda(), b.cuda(), "softmax").cpu()
    ref = torch.softmax(X @ W.T + b, dim=1)
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-14)


def test_softmax_argmax_rows(torch):
    from seldon_core_amd import ops

    x = torch.randn(513, 1000, dtype=torch.float64)
    s = ops.softmax_rows(x.cuda()).cpu()
    assert torch.allclose(s, torch.softmax(x, 1), rtol=1e-12, atol=1e-15)
    a = ops.argmax_rows(x.cuda()).cpu()
    assert torch.equal(a.long(), x.argmax(1))


def test_combine_mean(torch):
    from seldon_core_amd import ops

    xs = [torch.randn(77, 13, dtype=torch.float64) for _ in range(5)]
    out = ops.combine_mean([x.cuda() for x in xs]).cpu()
    assert torch.allclose(out, torch.stack(xs).mean(0), rtol=1e-13, atol=1e-15)


def test_minmax_and_segments(torch):
    from seldon_core_amd import ops

    x = torch.randn(50, 7, dtype=torch.float64) * 3
    full = ops.minmax_normalize(x.cuda()).cpu()
    assert torch.allclose(full, (x - x.min()) / (x.max() - x.min()), rtol=1e-13)
    offs = [0, 3, 3 + 1, 20, 50]
    seg = ops.segment_minmax(x.cuda(), offs).cpu()
    for a, b in zip(offs[:-1], offs[1:]):
        part = x[a:b]
        want = torch.zeros_like(part) if part.max() == part.min() else (part - part.min()) / (part.max() - part.min())
        assert torch.allclose(seg[a:b], want, rtol=1e-13)


def test_mean_sigmoid(torch):
    from seldon_core_amd import ops

    x = torch.randn(300, 129, dtype=torch.float64)
    out = ops.mean_sigmoid(x.cuda(), 0.3).cpu()
    assert torch.allclose(out[:, 0], torch.sigmoid(x.mean(1) - 0.3), rtol=1e-13)


@pytest.mark.parametrize("hw", [(480, 640), (180, 400), (100, 150), (224, 224)])
def test_crop_resize_chw(torch, hw):
    from seldon_core_amd import ops

    rng = np.random.default_rng(1)
    img = (rng.random((*hw, 3)) * 255).astype(np.uint8)
    out = ops.crop_resize_chw(torch.from_numpy(img).cuda(), 224).cpu().numpy()
    ref = ops.crop_resize_chw_ref(img, 224)
    # pure crops are exact; resized axes may differ by one rounding step (fp32 fma order)
    assert np.abs(out - ref).max() <= (0 if hw[0] >= 224 and hw[1] >= 224 else 1)


@pytest.mark.parametrize("shape,cl", [((1, 256, 56, 56), True), ((3, 64, 28, 28), False), ((2, 1664, 7, 7), True),
                                      ((1, 128, 8, 8), False), ((4, 32, 3, 5), True)])
def test_bn_relu_bf16_matches_torch(shape, cl):
    """scale_shift_relu_bf16 (image.hip) == relu(batch_norm) in fp32 rounded to
    bf16: at most one bf16 ulp apart, NCHW and channels_last."""
    import torch

    from seldon_core_amd import ops

    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(shape, generator=g) * 3).to("cuda", torch.bfloat16)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    C = shape[1]
    scale = (torch.rand(C, generator=g) + 0.5).cuda()
    shift = torch.randn(C, generator=g).cuda()
    assert ops.bn_relu_bf16_applies(x)
    got = ops.bn_relu_bf16(x, scale, shift)
    assert got.is_contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)
    want = torch.relu(x.float() * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)).to(torch.bfloat16)
    torch.testing.assert_close(got.float(), want.float(), rtol=8e-3, atol=1e-6)


@pytest.mark.parametrize("shape,cl", [((1, 256, 56, 56), True), ((2, 2048, 7, 7), True), ((3, 64, 10, 8), False)])
def test_add_relu_bf16_matches_torch(shape, cl):
    import torch

    from seldon_core_amd import ops

    g = torch.Generator().manual_seed(sum(shape) + 1)
    a = torch.randn(shape, generator=g).to("cuda", torch.bfloat16)
    b = torch.randn(shape, generator=g).to("cuda", torch.bfloat16)
    if cl:
        a, b = a.contiguous(memory_format=torch.channels_last), b.contiguous(memory_format=torch.channels_last)
    assert ops.add_relu_bf16_applies(a, b)
    got = ops.add_relu_bf16(a, b)
    want = torch.relu(a.float() + b.float()).to(torch.bfloat16)
    torch.testing.assert_close(got.float(), want.float(), rtol=8e-3, atol=1e-6)
    assert not ops.add_relu_bf16_applies(a, b.contiguous()) or not cl  # mixed layouts go to torch
