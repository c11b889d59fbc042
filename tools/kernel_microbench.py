"""Hot serving kernels at throughput batch sizes, for timing and PMC passes (GPU only).

    python tools/kernel_microbench.py [--only tree,vae,mlp,linear] [--iters 50]

Each case launches its kernel `iters` times on one stream after a warmup and
prints one JSON line (microseconds per launch from HIP events for the raw
tree kernels; wall time per BatchedUnit.run and the batcher's GPU-busy time
for the model kernels, which includes the H2D/D2H of the batch).  Used under
`rocprofv3 --pmc ...` by tools/gpu_pmc.sh so every dispatch of the same
kernel reports the same counters; tools/pmc_summary.py turns the CSVs into
profiles/*/pmc_summary.md.

Cases (shapes are the serving configs of BASELINE.json, at a large batch):
  tree    xgboost 1000 trees x depth 8, 32 features, 4096 rows (tree_perfect_partial + tree_reduce)
  vae     VAE outlier detector 64 -> 256 -> 128 -> z16 -> 128 -> 256 -> 64, 10 MC decodes, 4096 rows
  mlp     MNIST-shaped classifier 784 -> 512 -> 256 -> 10 softmax, 8192 and 64 rows
  mlp_torch / vae_torch  the same networks in PyTorch eager fp32 (hipBLASLt GEMMs), as the library baseline
  linear  iris logistic regression 4 -> 3 softmax, 65536 rows
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time_unit(name, unit, X, iters, extra):
    unit.run(X[: min(len(X), 64)])
    unit.run(X)
    unit.reset_stats()
    t0 = time.perf_counter()
    for _ in range(iters):
        unit.run(X)
    dt = time.perf_counter() - t0
    st = unit.stats()
    rec = {"case": name, "rows": len(X), "iters": iters, "wall_us_per_run": round(dt / iters * 1e6, 1),
           "gpu_busy_us_per_run": round(st["gpu_busy_s"] / iters * 1e6, 1), "batches": st["batches"], **extra}
    print(json.dumps(rec), flush=True)
    return rec


def case_tree_small(iters):
    """Serving-size batches of the xgb1000 model: the two-kernel chunked plan
    (partial + reduce, the plan TreeEnsembleModel picks) vs the single-launch
    whole-ensemble kernel at every rows-per-block choice."""
    import torch

    from seldon_core_amd import native

    K = native().kernels
    T, D, F = 1000, 8, 32
    ni = (1 << D) - 1
    g = torch.Generator().manual_seed(0)
    thr = torch.randn(T * ni, generator=g)
    feat = torch.randint(0, F, (T * ni,), generator=g, dtype=torch.int32)
    nodes = torch.stack([thr.view(torch.int32), feat], 1).contiguous().cuda()
    leaves = (torch.randn(T * (ni + 1), generator=g) * 0.01).cuda()
    s = torch.cuda.current_stream().cuda_stream
    out_rec = []
    for rows in (1, 4, 10, 16, 64, 256):
        X = torch.randn(rows, F, dtype=torch.float64, generator=g).cuda()
        out = torch.empty(rows, dtype=torch.float64, device="cuda")
        rb = 1 if rows == 1 else 2
        while rb * 2 <= rows // 16 and rb < 64:
            rb *= 2
        chunk = max(256 // rb, (T * ((rows + rb - 1) // rb) + 2047) // 2048)
        chunk = next(c for c in (4, 8, 16, 32, 64, 128, 256, 512) if c >= chunk) if chunk <= 512 else 512
        begin = torch.unique_consecutive(torch.arange(0, T + chunk, chunk, dtype=torch.int32).clamp_(max=T)).cuda()
        nc = begin.numel() - 1
        group = torch.zeros(nc, dtype=torch.int32, device="cuda")
        partial = torch.empty(nc * rows, dtype=torch.float64, device="cuda")

        def two():
            K.tree_perfect_partial(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, begin.data_ptr(),
                                   nc, rb, partial.data_ptr(), s, 0)
            K.tree_reduce(partial.data_ptr(), rows, nc, group.data_ptr(), 1, 0, 1.0, 0, out.data_ptr(), 1, s)

        def timed(fn):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return round(e0.elapsed_time(e1) * 1000.0 / iters, 2)

        rec = {"case": "tree_small", "rows": rows, "two_kernel_us": timed(two), "chunks": nc, "chunk_rb": rb}
        ref = out.clone()
        for wrb in (1, 2, 4, 8, 16):
            if wrb > 1 and wrb >= 2 * rows:
                break

            def whole(wrb=wrb):
                K.tree_perfect_whole(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, T, wrb, 0, 1.0,
                                     0, out.data_ptr(), 1, s)

            rec[f"whole_rb{wrb}_us"] = timed(whole)
            rec[f"whole_rb{wrb}_maxdiff"] = float((out - ref).abs().max())
        print(json.dumps(rec), flush=True)
        out_rec.append(rec)
    return out_rec


def case_tree(iters):
    import torch

    from seldon_core_amd import native

    K = native().kernels
    T, D, F, rows = 1000, 8, 32, 4096
    ni = (1 << D) - 1
    g = torch.Generator().manual_seed(0)
    thr = torch.randn(T * ni, generator=g)
    feat = torch.randint(0, F, (T * ni,), generator=g, dtype=torch.int32)
    nodes = torch.stack([thr.view(torch.int32), feat], 1).contiguous().cuda()
    leaves = (torch.randn(T * (ni + 1), generator=g) * 0.01).cuda()
    X = torch.randn(rows, F, dtype=torch.float64, generator=g).cuda()
    rb, chunk = 64, 32  # measured best two-pass geometry at >= 2048 rows (profiles/r01g_tree_variants)
    begin = torch.unique_consecutive(torch.arange(0, T + chunk, chunk, dtype=torch.int32).clamp_(max=T)).cuda()
    nc = begin.numel() - 1
    group = torch.zeros(nc, dtype=torch.int32, device="cuda")
    partial = torch.empty(nc * rows, dtype=torch.float64, device="cuda")  # fp64 slab
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def launch():
        K.tree_perfect_partial(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0, begin.data_ptr(), nc,
                               rb, partial.data_ptr(), s, 0)
        K.tree_reduce(partial.data_ptr(), rows, nc, group.data_ptr(), 1, 0, 1.0, 0, out.data_ptr(), 1, s)

    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / iters
    # reference: the same ensemble on the CPU twin
    ref = torch.zeros(rows, dtype=torch.float64)
    Xc, thr_c, feat_c, leaves_c = X.cpu()[:256].float().double(), thr, feat, leaves.cpu()  # kernel compares in fp32
    for t in range(T):
        idx = torch.zeros(256, dtype=torch.long)
        for _ in range(D):
            n = t * ni + idx
            go_right = Xc[torch.arange(256), feat_c[n].long()] >= thr_c[n].double()
            idx = 2 * idx + 1 + go_right.long()
        ref[:256] += leaves_c[t * (ni + 1) + idx - ni].double()
    err = float((out.cpu()[:256] - ref[:256]).abs().max())
    visits = rows * T * D
    rec = {"case": "tree", "rows": rows, "trees": T, "depth": D, "iters": iters, "us_per_batch": round(us, 2),
           "rows_per_s": round(rows / us * 1e6), "node_visits_per_s": round(visits / us * 1e6),
           "max_err_vs_cpu": err}
    print(json.dumps(rec), flush=True)
    return rec


def case_vae(iters):
    from seldon_core_amd import native
    from seldon_core_amd.models.mlp import random_dense_stack

    C = native()
    F, latent, rows = 64, 16, 4096
    enc = random_dense_stack([F, 256, 128, 2 * latent], ["relu", "relu", "identity"], seed=1)
    dec = random_dense_stack([latent, 128, 256, F], ["relu", "relu", "sigmoid"], seed=2)
    unit = C.BatchedUnit(C.vae_model(enc, latent, dec, 10, 3), 0)
    X = np.random.default_rng(0).random(size=(rows, F))
    try:
        flops = 2 * rows * (F * 256 + 256 * 128 + 128 * 2 * latent + 10 * (latent * 128 + 128 * 256 + 256 * F))
        rec = _time_unit("vae", unit, X, iters, {"gflop_per_run": round(flops / 1e9, 3)})
        rec["tflops_gpu_busy"] = round(flops / (rec["gpu_busy_us_per_run"] * 1e-6) / 1e12, 2)
        print(json.dumps({"case": "vae_derived", "tflops_fp32_mfma": rec["tflops_gpu_busy"]}), flush=True)
    finally:
        unit.stop()


MLP_DIMS = [784, 512, 256, 10]


def case_mlp(iters, rows_list=(8192, 64)):
    from seldon_core_amd import native
    from seldon_core_amd.models.mlp import OUT_SOFTMAX, mlp_row_model, random_dense_stack

    C = native()
    dims = MLP_DIMS
    unit = C.BatchedUnit(mlp_row_model(random_dense_stack(dims, ["relu", "relu", "identity"], seed=4), OUT_SOFTMAX), 0)
    try:
        for rows in rows_list:
            X = np.random.default_rng(1).normal(size=(rows, dims[0]))
            flops = 2 * rows * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
            rec = _time_unit("mlp", unit, X, iters, {"gflop_per_run": round(flops / 1e9, 4),
                                                     "input_mb_fp64": round(X.nbytes / 2**20, 2)})
            print(json.dumps({"case": "mlp_derived", "rows": rows,
                              "tflops_fp32_mfma_incl_h2d": round(flops / (rec["gpu_busy_us_per_run"] * 1e-6) / 1e12, 2)}),
                  flush=True)
    finally:
        unit.stop()


def case_mlp_modes(iters):
    """Fused vs layer-wise MLP / VAE at serving batch sizes (GPU-busy time per batch incl. H2D)."""
    import os

    from seldon_core_amd import native
    from seldon_core_amd.models.mlp import OUT_SOFTMAX, mlp_row_model, random_dense_stack

    C = native()
    nets = {"mlp784": lambda: mlp_row_model(random_dense_stack(MLP_DIMS, ["relu", "relu", "identity"], seed=4),
                                            OUT_SOFTMAX),
            "vae64": lambda: C.vae_model(random_dense_stack([64, 256, 128, 32], ["relu", "relu", "identity"], seed=1), 16,
                                         random_dense_stack([16, 128, 256, 64], ["relu", "relu", "sigmoid"], seed=2),
                                         10, 3)}
    for net, make in nets.items():
        for rows in (1, 16, 64, 256, 1024, 4096):
            rec = {"case": "mlp_modes", "net": net, "rows": rows}
            for mode in ("fused", "layer", "auto"):
                os.environ["SCA_MLP_MODE"] = mode
                m = make()
                if mode == "auto":
                    rec["auto_layerwise"] = bool(C.mlp_layerwise(m, rows))
                unit = C.BatchedUnit(m, 0)
                X = np.random.default_rng(rows).random(size=(rows, 784 if net == "mlp784" else 64))
                try:
                    y = unit.run(X)
                    unit.reset_stats()
                    for _ in range(iters):
                        y2 = unit.run(X)
                    rec[mode + "_us"] = round(unit.stats()["gpu_busy_s"] / iters * 1e6, 1)
                    if mode == "fused":
                        ref = y2
                    else:
                        rec[mode + "_maxdiff"] = float(np.abs(y2 - ref).max()) if net == "mlp784" else None
                finally:
                    unit.stop()
            os.environ.pop("SCA_MLP_MODE", None)
            print(json.dumps(rec), flush=True)


def case_dense_prec(iters):
    """MLP 784-512-256-10 @ 8192 rows and VAE 64-256-128-z16 x10 @ 4096 rows:
    fused fp32 / layer-wise fp32 (register-tiled GEMM) / bf16 GEMM.  Kernel
    time comes from the rocprofv3 kernel trace (gpu-busy here includes the
    fp64 H2D of the batch); run with torch cases for the library baseline."""
    import os

    from seldon_core_amd import native
    from seldon_core_amd.models.mlp import OUT_SOFTMAX, mlp_row_model, random_dense_stack

    C = native()
    mlp_layers = random_dense_stack(MLP_DIMS, ["relu", "relu", "identity"], seed=4)
    enc = random_dense_stack([64, 256, 128, 32], ["relu", "relu", "identity"], seed=1)
    dec = random_dense_stack([16, 128, 256, 64], ["relu", "relu", "sigmoid"], seed=2)
    for net, rows in (("mlp784", 8192), ("vae64", 4096)):
        X = np.random.default_rng(0).random(size=(rows, 784 if net == "mlp784" else 64))
        ref = None
        for label, mode, prec in (("fused_fp32", "fused", "fp32"), ("layer_fp32", "layer", "fp32"),
                                  ("bf16", "layer", "bf16")):
            os.environ["SCA_MLP_MODE"] = mode
            m = (mlp_row_model(mlp_layers, OUT_SOFTMAX, precision=prec) if net == "mlp784"
                 else C.vae_model(enc, 16, dec, 10, 3, prec))
            unit = C.BatchedUnit(m, 0, max_batch=8192)
            try:
                y = unit.run(X)
                ref = y if ref is None else ref
                rec = _time_unit(f"dense_{net}_{label}", unit, X, iters,
                                 {"max_abs_diff_vs_fused_fp32": float(np.abs(y - ref).max())})
            finally:
                unit.stop()
        os.environ.pop("SCA_MLP_MODE", None)


def case_gemm(iters):
    """bf16 GEMM C = A . W^T (fp32 out) at the MLP layer shapes and square
    shapes: register-staged LDS kernel (path 1), glds ring kernel (path 2) and
    torch bf16 (hipBLASLt), interleaved in one process on the same random
    operands; TFLOP/s from HIP event time per launch."""
    import torch

    from seldon_core_amd import native

    C = native()
    shapes = ((8192, 832, 512), (8192, 512, 256), (4096, 4096, 4096), (8192, 8192, 8192))
    if os.environ.get("GEMM_SHAPES"):  # e.g. "8192x832x512,4096x4096x4096" (PMC passes)
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["GEMM_SHAPES"].split(",")]
    for rows, K, N in shapes:
        A = torch.randn(rows, K, device="cuda").to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device="cuda")
        O = torch.empty(rows, N, device="cuda")
        flops = 2.0 * rows * K * N
        n = iters if rows * K * N < 1e10 else max(3, iters // 5)

        Ob = torch.empty(rows, N, device="cuda", dtype=torch.bfloat16)

        def run(path):
            C.kernels.gemm_bf16(A.data_ptr(), K, rows, W.data_ptr(), K, N, N, b.data_ptr(), 0, O.data_ptr(), N, 1, path)

        def run_bf16_out(path):  # bf16 C, as torch.matmul writes it
            C.kernels.gemm_bf16(A.data_ptr(), K, rows, W.data_ptr(), K, N, N, b.data_ptr(), 0, Ob.data_ptr(), N, 0, path)

        def lib():
            torch.matmul(A, W.T, out=None)

        res = {}
        for _ in range(1 if os.environ.get("SCA_PMC") else 2):  # interleaved rounds
            for name, fn in (("reg", lambda: run(1)), ("glds", lambda: run(2)), ("glds256", lambda: run(3)),
                             ("8ph", lambda: run(4)), ("8ph_spread", lambda: run(6)),
                             ("8ph_ring", lambda: run(9)), ("8ph_spread_bf16out", lambda: run_bf16_out(6)), ("w4", lambda: run(5)),
                             ("torch", lib)) + ((("abl_no_mfma", lambda: run(7)), ("abl_no_reads", lambda: run(8)))
                                                if os.environ.get("GEMM_ABLATE") else ()):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / n
                res[name] = min(res.get(name, 1e30), us)
        errs = {}
        ref = (A.float() @ W.float().T)
        for pth, nm in ((3, "glds256"), (4, "8ph"), (6, "8ph_spread"), (9, "8ph_ring"), (5, "w4")):
            run(pth)
            errs[nm + "_rel_err"] = float((O - ref).abs().max() / ref.abs().max())
        print(json.dumps({"case": "gemm_bf16", "M": rows, "K": K, "N": N,
                          **{f"{k}_us": round(v, 2) for k, v in res.items()},
                          **{f"{k}_tflops": round(flops / (v * 1e-6) / 1e12, 1) for k, v in res.items()},
                          **errs}), flush=True)


def case_mlp_torch_bf16(iters, rows_list=(8192,)):
    """The MLP in PyTorch eager bf16 (hipBLASLt bf16 GEMMs)."""
    import torch

    from seldon_core_amd.models.mlp import random_dense_stack

    layers = random_dense_stack(MLP_DIMS, ["relu", "relu", "identity"], seed=4)
    Ws = [torch.tensor(L["W"], device="cuda", dtype=torch.bfloat16) for L in layers]
    bs = [torch.tensor(L["b"], device="cuda", dtype=torch.bfloat16) for L in layers]
    for rows in rows_list:
        x = torch.randn(rows, MLP_DIMS[0], device="cuda", dtype=torch.bfloat16)

        def fwd():
            h = x
            for i, (W, b) in enumerate(zip(Ws, bs)):
                h = torch.nn.functional.linear(h, W, b)
                if i + 1 < len(Ws):
                    h = torch.relu(h)
            return torch.softmax(h.float(), 1)

        us = _torch_time(fwd, iters)
        flops = 2 * rows * sum(a * b for a, b in zip(MLP_DIMS[:-1], MLP_DIMS[1:]))
        print(json.dumps({"case": "mlp_torch_bf16", "rows": rows, "us_per_run": round(us, 2),
                          "tflops": round(flops / (us * 1e-6) / 1e12, 2)}), flush=True)


def _torch_time(fn, iters):
    import torch

    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def case_mlp_torch(iters, rows_list=(8192, 64), fp64_io=False):
    """Same MLP in PyTorch eager fp32 (hipBLASLt GEMMs + elementwise), input already fp32 on device.
    fp64_io: the serving contract of our kernels -- fp64 rows in, fp64 probabilities out (the
    fp64 -> fp32 cast and the fp64 output are part of the timed work, as in mlp_kernel)."""
    import torch

    from seldon_core_amd.models.mlp import random_dense_stack

    layers = random_dense_stack(MLP_DIMS, ["relu", "relu", "identity"], seed=4)
    Ws = [torch.tensor(L["W"], device="cuda") for L in layers]
    bs = [torch.tensor(L["b"], device="cuda") for L in layers]
    for rows in rows_list:
        x = torch.randn(rows, MLP_DIMS[0], device="cuda", dtype=torch.float64 if fp64_io else torch.float32)

        def fwd():
            h = x.float() if fp64_io else x
            for i, (W, b) in enumerate(zip(Ws, bs)):
                h = torch.nn.functional.linear(h, W, b)
                if i + 1 < len(Ws):
                    h = torch.relu(h)
            out = torch.softmax(h, 1)
            return out.double() if fp64_io else out

        us = _torch_time(fwd, iters)
        flops = 2 * rows * sum(a * b for a, b in zip(MLP_DIMS[:-1], MLP_DIMS[1:]))
        print(json.dumps({"case": "mlp_torch_fp32" + ("_fp64io" if fp64_io else ""), "rows": rows,
                          "us_per_run": round(us, 2),
                          "tflops": round(flops / (us * 1e-6) / 1e12, 2)}), flush=True)


def case_vae_torch(iters):
    import torch

    from seldon_core_amd.models.mlp import random_dense_stack

    F, latent, rows = 64, 16, 4096
    enc = random_dense_stack([F, 256, 128, 2 * latent], ["relu", "relu", "identity"], seed=1)
    dec = random_dense_stack([latent, 128, 256, F], ["relu", "relu", "sigmoid"], seed=2)
    E = [(torch.tensor(L["W"], device="cuda"), torch.tensor(L["b"], device="cuda")) for L in enc]
    D = [(torch.tensor(L["W"], device="cuda"), torch.tensor(L["b"], device="cuda")) for L in dec]
    x = torch.rand(rows, F, device="cuda")
    F_ = torch.nn.functional

    def fwd():
        h = F_.relu(F_.linear(F_.relu(F_.linear(x, *E[0])), *E[1]))
        h = F_.linear(h, *E[2])
        mu, logvar = h[:, :latent], h[:, latent:]
        err = torch.zeros(rows, device="cuda")
        for _ in range(10):
            z = mu + torch.exp(0.5 * logvar) * torch.randn_like(mu)
            y = torch.sigmoid(F_.linear(F_.relu(F_.linear(F_.relu(F_.linear(z, *D[0])), *D[1])), *D[2]))
            err += ((y - x) ** 2).mean(1)
        return err / 10

    us = _torch_time(fwd, iters)
    print(json.dumps({"case": "vae_torch_fp32", "rows": rows, "us_per_run": round(us, 2)}), flush=True)


def case_linear(iters):
    from seldon_core_amd import native

    C = native()
    rows = 65536
    rng = np.random.default_rng(2)
    unit = C.BatchedUnit(C.linear_model(rng.normal(size=(3, 4)), rng.normal(size=3), 1), 0)
    X = rng.normal(size=(rows, 4))
    try:
        _time_unit("linear", unit, X, iters, {"bytes_in_out": rows * (4 + 3) * 8})
    finally:
        unit.stop()


def case_latency(iters):
    """Round trip of one micro-batch through BatchedUnit (submit -> launch ->
    completion seen -> response rows) for serving-size batches, spin vs
    blocking completion, next to torch's launch + synchronize floor."""
    import torch

    from seldon_core_amd import native

    C = native()
    rng = np.random.default_rng(2)
    n = max(iters, 2000)
    for spin in (True, False):
        unit = C.BatchedUnit(C.linear_model(rng.normal(size=(3, 4)), rng.normal(size=3), 1), 0, spin_wait=spin)
        try:
            for rows in (1, 20):
                _time_unit(f"latency_linear_spin{int(spin)}", unit, rng.normal(size=(rows, 4)), n, {})
        finally:
            unit.stop()
    x = torch.zeros(4, device="cuda")
    for _ in range(100):
        x.add_(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"case": "latency_torch_launch_sync", "iters": n, "wall_us_per_run": round(dt / n * 1e6, 2)}),
          flush=True)


def case_lstm(iters):
    """seq2seq LSTM detector (ECG-shaped: T=140, F=1, BiLSTM 20 -> LSTM 40 -> Dense),
    one persistent kernel per batch: the small-batch VALU kernel and the 16-row
    MFMA kernel at each batch size, vs the torch eager decode loop."""
    import torch

    from seldon_core_amd import native
    from seldon_core_amd.components.outlier import Seq2SeqLSTMNet

    C = native()
    T, F = 140, 1
    net = Seq2SeqLSTMNet(F, (20,), (40,), "sigmoid", 0, 0)
    for rows in (1, 16, 256, 1024, 4096):
        X = np.random.default_rng(3).random((rows, T, F))
        ref, torch_us = None, 0.0
        if rows in (16, 1024) and not os.environ.get("SCA_PMC"):
            ref = np.mean((X - net.reconstruct(X)) ** 2, axis=(1, 2))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                net.reconstruct(X)
            torch.cuda.synchronize()
            torch_us = (time.perf_counter() - t0) / 3 * 1e6
        for path in ("valu", "mfma"):
            if path == "valu" and rows > 1024:
                continue
            os.environ["SCA_LSTM_PATH"] = path
            unit = C.BatchedUnit(net.native_model(T), 0, max_batch=4096)
            try:
                got = np.asarray(unit.run(X.reshape(rows, -1)))[:, 0]
                err = float(np.max(np.abs(got - ref) / np.abs(ref))) if ref is not None else None
                _time_unit("lstm_" + path, unit, X.reshape(rows, -1), iters if rows <= 1024 else max(3, iters // 5),
                           {"T": T, "F": F, "enc": 20, "dec": 40, "torch_eager_us": round(torch_us, 1),
                            "max_rel_err_vs_torch": err})
            finally:
                unit.stop()
        os.environ.pop("SCA_LSTM_PATH", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="tree,vae,mlp,linear")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    cases = {"tree": case_tree, "tree_small": case_tree_small, "vae": case_vae, "mlp": case_mlp, "linear": case_linear,
             "mlp_torch": case_mlp_torch,
             "mlp_torch_fp64io": lambda it: case_mlp_torch(it, fp64_io=True), "vae_torch": case_vae_torch, "mlp_modes": case_mlp_modes,
             "lstm": case_lstm, "gemm": case_gemm, "latency": case_latency, "dense_prec": case_dense_prec, "mlp_torch_bf16": case_mlp_torch_bf16}
    for c in a.only.split(","):
        cases[c](a.iters)


if __name__ == "__main__":
    main()
