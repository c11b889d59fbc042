"""Torch-facing wrappers over the engine's hand-written gfx950 kernels.

Each op takes/returns ``torch`` tensors resident on an MI355X and launches the
HIP kernel from ``seldon_core_amd._C.kernels`` on the current HIP stream (so it
orders with surrounding torch work and can be captured in a hipGraph).  There
is no silent fallback: calling an op on CPU tensors or without the native
extension raises.  CPU references for the tests live next to each op.

Kernel sources: csrc/kernels/{linear,combine,image,tree,bandit}.hip.
"""
from __future__ import annotations

from typing import List, Sequence

from .._native import native


def _k():
    return native().kernels


def _check(t, dtype=None, name="tensor"):
    import torch

    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    return t.contiguous()


def _stream(t) -> int:
    import torch

    return int(torch.cuda.current_stream(t.device).cuda_stream)


ACT = {"identity": 0, "softmax": 1, "binary_logistic": 2, "ovr": 3, "sigmoid": 4}


def linear(X, W, b, act: str = "softmax"):
    """act(X @ W.T + b), fp64 (sklearn linear models' predict_proba)."""
    import torch

    X = _check(X, torch.float64, "X")
    W = _check(W, torch.float64, "W")
    b = _check(b, torch.float64, "b")
    C, K = W.shape
    oc = 2 if act == "binary_logistic" else C
    out = torch.empty((X.shape[0], oc), dtype=torch.float64, device=X.device)
    _k().linear_f64(X.data_ptr(), X.shape[0], K, W.data_ptr(), b.data_ptr(), C, ACT[act], out.data_ptr(), _stream(X))
    return out


def bn_relu_bf16(x, scale, shift):
    """relu(x * scale[c] + shift[c]) over a bf16 [N, C, H, W] activation, NCHW
    or channels_last, in one pass (``scale_shift_relu_bf16``, image.hip).
    ``scale`` / ``shift`` are fp32 [C] on the same GPU."""
    import torch

    if not x.is_cuda or x.dtype != torch.bfloat16 or x.dim() != 4:
        raise ValueError("bn_relu_bf16 takes a 4-D bf16 GPU tensor")
    N, C, H, W = x.shape
    cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
    if not cl:
        x = x.contiguous()
    if x.data_ptr() % 16 or not _k().scale_shift_relu_bf16_ok(C, H * W, int(cl)):
        raise ValueError("bn_relu_bf16: activation not 16-byte aligned / 8-element divisible")
    out = torch.empty_like(x)
    _k().scale_shift_relu_bf16(x.data_ptr(), _check(scale, torch.float32, "scale").data_ptr(),
                               _check(shift, torch.float32, "shift").data_ptr(), N, C, H * W, int(cl),
                               out.data_ptr(), _stream(x))
    return out


def add_relu_bf16(a, b):
    """relu(a + b) for two bf16 GPU tensors of one shape and memory layout
    (ResNet's residual join) in one pass (``add_relu_bf16``, image.hip)."""
    if not add_relu_bf16_applies(a, b):
        raise ValueError("add_relu_bf16 takes two same-layout, 16-byte aligned bf16 GPU tensors, numel % 8 == 0")
    import torch

    out = torch.empty_like(a)
    _k().add_relu_bf16(a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), _stream(a))
    return out


def add_relu_bf16_applies(a, b) -> bool:
    import torch

    if not (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    if a.shape != b.shape or a.stride() != b.stride() or a.numel() % 8 or a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    fmt = torch.channels_last if a.dim() == 4 and not a.is_contiguous() else torch.contiguous_format
    return a.is_contiguous(memory_format=fmt) and b.is_contiguous(memory_format=fmt)


def bn_relu_bf16_applies(x) -> bool:
    """Whether :func:`bn_relu_bf16` takes ``x`` as it is (else use torch)."""
    import torch

    if not x.is_cuda or x.dtype != torch.bfloat16 or x.dim() != 4 or x.data_ptr() % 16:
        return False
    cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
    if not cl and not x.is_contiguous():
        return False
    return bool(_k().scale_shift_relu_bf16_ok(x.shape[1], x.shape[2] * x.shape[3], int(cl)))


def softmax_rows(x):
    import torch

    x = _check(x, torch.float64, "x")
    out = torch.empty_like(x)
    _k().softmax_rows_f64(x.data_ptr(), x.shape[0], x.shape[1], out.data_ptr(), _stream(x))
    return out


def argmax_rows(x):
    import torch

    x = _check(x, torch.float64, "x")
    out = torch.empty((x.shape[0],), dtype=torch.int32, device=x.device)
    _k().argmax_rows_f64(x.data_ptr(), x.shape[0], x.shape[1], out.data_ptr(), _stream(x))
    return out


def combine_mean(xs: Sequence):
    """Element-wise mean of same-shaped fp64 tensors (AVERAGE_COMBINER)."""
    import torch

    xs = [_check(x, torch.float64, "input") for x in xs]
    shape = xs[0].shape
    if any(x.shape != shape for x in xs):
        raise ValueError("combine_mean inputs must share a shape")
    ptrs = torch.tensor([x.data_ptr() for x in xs], dtype=torch.int64, device=xs[0].device)
    out = torch.empty_like(xs[0])
    _k().combine_mean_f64(ptrs.data_ptr(), len(xs), out.numel(), out.data_ptr(), _stream(out))
    return out


def minmax_normalize(x):
    import torch

    x = _check(x, torch.float64, "x")
    out = torch.empty_like(x)
    scratch = torch.empty(2, dtype=torch.float64, device=x.device)
    _k().minmax_normalize_f64(x.data_ptr(), x.numel(), out.data_ptr(), scratch.data_ptr(), _stream(x))
    return out


def segment_minmax(x, row_offsets: List[int]):
    """Per-segment min-max normalisation of the rows of a 2-D tensor."""
    import torch

    x = _check(x, torch.float64, "x")
    seg = torch.tensor(list(row_offsets), dtype=torch.int32, device=x.device)
    out = torch.empty_like(x)
    _k().segment_minmax_f64(x.data_ptr(), seg.data_ptr(), len(row_offsets) - 1, x.shape[1], out.data_ptr(),
                            _stream(x))
    return out


def mean_sigmoid(x, threshold: float):
    import torch

    x = _check(x, torch.float64, "x")
    out = torch.empty((x.shape[0], 1), dtype=torch.float64, device=x.device)
    _k().mean_sigmoid_rows_f64(x.data_ptr(), x.shape[0], x.shape[1], float(threshold), out.data_ptr(), _stream(x))
    return out


def crop_resize_chw(img, crop: int = 224):
    """Decoded HWC uint8 image -> [C, crop, crop] fp32 (centre crop; axes
    shorter than ``crop`` are bilinearly up-sized first, as cv2 does)."""
    import torch

    img = _check(img, torch.uint8, "img")
    H, W, C = img.shape
    out = torch.empty((C, crop, crop), dtype=torch.float32, device=img.device)
    _k().crop_resize_chw_u8(img.data_ptr(), H, W, C, crop, out.data_ptr(), _stream(img))
    return out


def mahalanobis_sm_scores(B, proj_cov, x_diff, n: float, device: int = 0):
    """Sherman-Morrison inverse recurrence + Mahalanobis scores for one batch
    (numpy in/out; None if k > 16 -- caller falls back to numpy)."""
    import numpy as np
    import torch

    nb, k = x_diff.shape
    if k > 16:
        return None
    dev = torch.device(f"cuda:{device}")
    tB = torch.as_tensor(np.ascontiguousarray(B, dtype=np.float64), device=dev)
    tC = torch.as_tensor(np.ascontiguousarray(proj_cov, dtype=np.float64), device=dev)
    tX = torch.as_tensor(np.ascontiguousarray(x_diff, dtype=np.float64), device=dev)
    out = torch.empty(nb, dtype=torch.float64, device=dev)
    ok = _k().mahalanobis_sm_scores(tB.data_ptr(), tC.data_ptr(), tX.data_ptr(), nb, k, float(n), out.data_ptr(),
                                    _stream(out))
    return out.cpu().numpy() if ok else None


# ------------------------------------------------------------ CPU references
def crop_resize_chw_ref(img, crop: int = 224):
    """numpy reference of :func:`crop_resize_chw` (same fused bilinear map)."""
    import numpy as np

    H, W, C = img.shape
    rh, rw = max(H, crop), max(W, crop)

    def axis(n_src, n_dst, idx):
        if n_src == n_dst:
            return idx, idx, np.zeros(len(idx), np.float32)
        s = (idx.astype(np.float32) + 0.5) * np.float32(n_src / n_dst) - 0.5
        s = np.maximum(s, 0)
        i0 = np.minimum(s.astype(np.int64), n_src - 1)
        i1 = np.minimum(i0 + 1, n_src - 1)
        return i0, i1, (s - i0).astype(np.float32)

    xs = rw // 2 - crop // 2 + np.arange(crop)
    ys = rh // 2 - crop // 2 + np.arange(crop)
    x0, x1, wx = axis(W, rw, xs)
    y0, y1, wy = axis(H, rh, ys)
    f = img.astype(np.float32)
    top = f[y0][:, x0] * (1 - wx)[None, :, None] + f[y0][:, x1] * wx[None, :, None]
    bot = f[y1][:, x0] * (1 - wx)[None, :, None] + f[y1][:, x1] * wx[None, :, None]
    v = top * (1 - wy)[:, None, None] + bot * wy[:, None, None]
    if rw != W or rh != H:
        v = np.rint(v)
    return v.transpose(2, 0, 1).astype(np.float32)
