"""MFMA vs wave-per-row linear_f64 at the VERDICT r5 K3 shapes (one process;
SCA_LINEAR_MFMA toggled per run).  Prints one JSON line per (shape, path)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from seldon_core_amd import native  # noqa: E402

K_ = native().kernels
SHAPES = [(4096, 784, 10, 1), (8192, 256, 1000, 1), (64, 30, 1, 2), (4096, 4, 3, 1), (16384, 64, 100, 1)]
for rows, K, C, act in SHAPES:
    X = torch.randn(rows, K, dtype=torch.float64, device="cuda")
    W = torch.randn(C, K, dtype=torch.float64, device="cuda") / K ** 0.5
    b = torch.randn(C, dtype=torch.float64, device="cuda")
    out = torch.empty(rows, 2 if act == 2 else C, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for path, env in (("wave_or_thread", "0"), ("mfma", "2")):
        os.environ["SCA_LINEAR_MFMA"] = env
        for _ in range(5):
            K_.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, act, out.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            K_.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, act, out.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / n
        z = X @ W.T + b
        ref = torch.softmax(z, 1) if act == 1 else torch.stack([1 - torch.sigmoid(z[:, 0]), torch.sigmoid(z[:, 0])], 1)
        err = float((out - ref).abs().max())
        flops = 2.0 * rows * K * C
        byts = 8.0 * (rows * K + C * K + rows * out.shape[1])
        print(json.dumps({"rows": rows, "K": K, "C": C, "path": path, "us": round(us, 2),
                          "tflops": round(flops / us / 1e6, 2), "gbs": round(byts / us / 1e3, 1),
                          "max_err": err}), flush=True)
os.environ.pop("SCA_LINEAR_MFMA", None)
