"""bf16 GEMM kernels (csrc/kernels/gemm.hip) against torch fp32 on the same
bf16-rounded operands: the register-staged LDS kernel and the
global_load_lds ring kernel, with bias + activation epilogues and ragged
row counts.  Reference: the Dense layers of components/outlier-detection/vae/
model.py:23-91 and the MLP servers, which these kernels serve."""
import numpy as np
import pytest

import seldon_core_amd as sca

SHAPES = [  # rows, K (padded to 64), N (padded to 64)
    (8192, 784, 512),   # the MLP's first layer
    (8192, 512, 256),
    (4000, 256, 384),   # ragged rows: the last 128-row tile is partial
    (2048, 2048, 2048),
    (300, 64, 128),
]


def _pad(x, m):
    return (x + m - 1) // m * m


@pytest.mark.gpu
@pytest.mark.parametrize("rows,K,N", SHAPES)
@pytest.mark.parametrize("path", [1, 2, 3, 4, 5, 6, 9])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_bf16_matches_torch(rows, K, N, path, act):
    import torch

    C = sca.native()
    Kp, Np = _pad(K, 64), _pad(N, 64)
    g = torch.Generator(device="cpu").manual_seed(rows + K + N)
    A = torch.zeros(rows, Kp, dtype=torch.bfloat16)
    A[:, :K] = torch.randn(rows, K, generator=g).to(torch.bfloat16)
    W = torch.zeros(Np, Kp, dtype=torch.bfloat16)
    W[:N, :K] = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Np, generator=g).float()
    want = A.float() @ W.float().T + bias
    if act == 1:
        want = torch.relu(want)
    want = want[:, :N]
    dA, dW, db = A.cuda(), W.cuda(), bias.cuda()
    O = torch.full((rows, N), float("nan"), dtype=torch.float32, device="cuda")
    C.kernels.gemm_bf16(dA.data_ptr(), Kp, rows, dW.data_ptr(), Kp, Np, N, db.data_ptr(), act, O.data_ptr(), N, 1,
                        path)
    torch.cuda.synchronize()
    got = O.cpu()
    assert torch.isfinite(got).all()
    err = (got - want).abs().max().item()
    assert err <= 1e-3 * max(1.0, want.abs().max().item()), err
