"""Per-request latency of the Mahalanobis outlier detector: numpy path
(reference semantics, CoreMahalanobis.py:68-151) vs the device path through the
micro-batcher (csrc/gpu/maha_device.cc), sequential and with concurrent
callers.  Run it under ``rocprofv3 --kernel-trace --stats`` for the kernel's
own duration (maha_step_kernel).

    python tools/maha_bench.py --p 9 64 --requests 2000 --threads 16
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from seldon_core_amd.components.outlier import OutlierMahalanobis  # noqa: E402


def pct(v, q):
    return float(np.percentile(np.asarray(v) * 1e6, q))


def dist_us(v):
    """p50 / p99 / p99.9 / max in microseconds (the periodic refresh shows
    only in the tail: 1 request in 1,024)."""
    return {"p50": pct(v, 50), "p99": pct(v, 99), "p99_9": pct(v, 99.9), "max": float(np.max(v) * 1e6)}


def seq_latency(fn, reqs):
    lat = []
    for X in reqs:
        t = time.perf_counter()
        fn(X)
        lat.append(time.perf_counter() - t)
    return lat


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, nargs="+", default=[9, 64])
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--requests", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from seldon_core_amd._native import native

    C = native()
    res = {}
    for p in a.p:
        rng = np.random.default_rng(p)
        reqs = [rng.normal(size=(1, p)) for _ in range(a.requests)]
        warm = [rng.normal(size=(1, p)) for _ in range(100)]
        host = OutlierMahalanobis(n_components=a.k, device=-1)
        for X in warm:
            host.predict(X, [])
        lat_np = seq_latency(lambda X: host.predict(X, []), reqs)
        print(f"p={p}: numpy done", file=sys.stderr, flush=True)
        dev = C.MahalanobisDevice(p, a.k, 3.0, 50.0, -1.0, 1e-8, 0)
        for X in warm:
            dev.step(X)
        print(f"p={p}: device warm-up done {dev.solver_stats()}", file=sys.stderr, flush=True)
        lat_dev = seq_latency(dev.step, reqs)
        print(f"p={p}: device sequential done {dev.solver_stats()}", file=sys.stderr, flush=True)
        # concurrent callers: requests share launches (segments)
        b0 = dev.batches()
        t0 = time.perf_counter()
        lat_c = [[] for _ in range(a.threads)]

        def worker(t):
            for X in reqs[t::a.threads]:
                s = time.perf_counter()
                dev.step(X)
                lat_c[t].append(time.perf_counter() - s)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        b1 = dev.batches()
        flat = [x for v in lat_c for x in v]
        jac = dev.solver_stats()
        res[p] = {
            "numpy_seq_us": dict(dist_us(lat_np), req_per_s=len(reqs) / sum(lat_np)),
            "device_seq_us": dict(dist_us(lat_dev), req_per_s=len(reqs) / sum(lat_dev)),
            "device_concurrent": {"threads": a.threads, "p50_us": pct(flat, 50), "p99_us": pct(flat, 99),
                                  "p99_9_us": pct(flat, 99.9), "max_us": float(np.max(flat) * 1e6),
                                  "req_per_s": len(reqs) / wall,
                                  "requests_per_launch": (b1["requests"] - b0["requests"]) /
                                  max(1, b1["batches"] - b0["batches"])},
            "kernel_phase_us": jac.get("phase_us_per_step"),
            "eigen_clock_mhz": jac.get("eigen_clock_mhz"),
            "rank1_steps": jac.get("rank1_steps"),
            "rank1_fallbacks": jac.get("rank1_fallbacks"),
            "solver_steps": jac.get("steps"),
            "jacobi_solves": jac.get("jacobi_solves"),
            "jacobi_sweeps_per_solve": jac.get("jacobi_sweeps_per_solve"),
        }
        print(json.dumps({"p": p, **res[p]}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
