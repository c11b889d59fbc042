"""Narrow-model MFMA linear kernel: K-split / chunk-group variants
(SCA_LINEAR_MFMA_SPLIT=1..6) at memory-bound shapes.  One JSON line per
(shape, variant): us per call (HIP events, 50 launches) and effective GB/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from seldon_core_amd import native  # noqa: E402

K_ = native().kernels
SHAPES = [(4096, 784, 10), (512, 784, 10), (64, 784, 10), (32768, 784, 10), (4096, 3072, 10), (16384, 64, 10), (8192, 256, 20),
          (2048, 1024, 2), (8192, 256, 1000), (16384, 64, 100), (4096, 256, 200), (4096, 512, 1000), (32768, 128, 512), (8192, 784, 1000), (2048, 1024, 1000), (16384, 384, 300)]
os.environ["SCA_LINEAR_MFMA"] = "2"
for rows, K, C in SHAPES:
    X = torch.randn(rows, K, dtype=torch.float64, device="cuda")
    W = torch.randn(C, K, dtype=torch.float64, device="cuda") / K ** 0.5
    b = torch.randn(C, dtype=torch.float64, device="cuda")
    out = torch.empty(rows, C, dtype=torch.float64, device="cuda")
    ref = torch.softmax(X @ W.T + b, 1)
    s = torch.cuda.current_stream().cuda_stream
    for v in ((0,) + tuple(range(1, 7)) if C <= 32 else (0, "wide0", "wide1", "wide2") if C > 256 else (0,)):
        os.environ["SCA_LINEAR_MFMA_SPLIT"] = "0" if str(v).startswith("wide") else str(v)
        if str(v).startswith("wide"):
            os.environ["SCA_LINEAR_WIDE"] = str(v)[-1]
        else:
            os.environ.pop("SCA_LINEAR_WIDE", None)
        out.zero_()
        for _ in range(5):
            K_.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, 1, out.data_ptr(), s)
        torch.cuda.synchronize()
        err = float((out - ref).abs().max())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            K_.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, 1, out.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / n
        byts = 8.0 * (rows * K + C * K + rows * C)
        print(json.dumps({"rows": rows, "K": K, "C": C, "variant": v, "us": round(us, 2),
                          "gbs": round(byts / us / 1e3, 1), "tflops": round(2.0 * rows * K * C / us / 1e6, 2),
                          "max_err": err}), flush=True)
os.environ.pop("SCA_LINEAR_MFMA_SPLIT", None)
os.environ.pop("SCA_LINEAR_MFMA", None)
