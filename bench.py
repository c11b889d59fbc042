#!/usr/bin/env python3
"""Headline serving benchmark (BASELINE.json): predictions/sec + p50/p99
latency of a single-model inference graph, REST API, at N MI355X GPUs.

Reference numbers (doc/source/reference/benchmarking.md:31-64):
REST 12,088.95 req/s (p50 4 ms, p99 69 ms), gRPC 28,256.39 req/s (p50 1 ms,
p99 6 ms), 256 locust users, one engine replica.

Here: one process per GPU (torch.distributed over RCCL for the job-level
barrier / result gather).  Each rank serves one replica of the graph -- the
reference's sklearn-iris LogisticRegression model (BASELINE config
1) executed by the GPU micro-batcher + linear_softmax HIP kernel on its GPU --
through the native HTTP/1.1 front end, and drives it with the native
closed-loop load generator (256 concurrent users per rank, no think time, the
locust REST payload shape).  Weak scaling: per-GPU load is fixed as N grows.

A "step" is ``--step-requests`` completed predictions per rank.  W warmup steps
run untimed; K steps are timed between a barrier + device synchronize on both
sides; ms_per_step is the max over ranks; ``value`` is the whole-job
predictions/s.  ``--api grpc`` measures the gRPC front end instead
(``seldon.protos.Seldon/Predict``, Tensor [3,2]-style payload).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REST_BASELINE = 12088.95
GRPC_BASELINE = 28256.39


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--api", choices=["rest", "grpc"], default="rest")
    ap.add_argument("--model", choices=["iris", "xgb1000"], default="iris")
    ap.add_argument("--users", type=int, default=256, help="concurrent clients per GPU")
    ap.add_argument("--step-requests", type=int, default=40000, help="predictions per step per GPU")
    ap.add_argument("--server-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--client-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--slots", type=int, default=4, help="GPU batches in flight per unit")
    ap.add_argument("--no-spin", action="store_true", help="block on events instead of spinning")
    ap.add_argument("--graph", choices=["single", "abtest", "pipeline", "mab"], default="single",
                    help="graph shape (single = the headline single-model graph)")
    ap.add_argument("--extra-grpc", action="store_true", help="also report the gRPC API (untimed extra)")
    return ap.parse_args()


def cpu_budget() -> float:
    """CPUs this process may use: cgroup v2 quota (cpu.max) or affinity."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return float(quota) / float(period)
    except (OSError, ValueError):
        pass
    try:
        return float(len(os.sched_getaffinity(0)))
    except AttributeError:
        return float(os.cpu_count() or 8)


def size_threads(args, local_world: int) -> None:
    """Split the CPU share of one rank between the front end (~60%), the
    closed-loop load generator (~32%) and the GPU device thread (measured on
    a 16-CPU MI355X share: 10 front-end / 5 generator threads was the best
    split, profiles/r01f_sweep_executor)."""
    per_rank = max(2.0, cpu_budget() / max(1, local_world))
    if args.server_threads is None:
        args.server_threads = max(1, min(16, int(round(per_rank * 0.6))))
    if args.client_threads is None:
        args.client_threads = max(1, min(10, int(round(per_rank * 0.32))))


def build_deployment(model: str, device: int, graph_kind: str = "single", slots: int = 4, spin: bool = True):
    import numpy as np  # noqa: F401

    import seldon_core_amd as sca
    from seldon_core_amd.servers import SKLearnServer, XGBoostServer

    if model == "iris":
        from seldon_core_amd.models import iris_logistic_regression

        comp = SKLearnServer(model=iris_logistic_regression())
        names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
        row = [5.1, 3.5, 1.4, 0.2]
        label = "sklearn-iris-LogisticRegression (linear_softmax HIP kernel, fp64)"
    else:
        from seldon_core_amd.models import synthetic_xgboost

        ens = synthetic_xgboost(1000, 8, 32, seed=0)
        comp = XGBoostServer(ensemble=ens)
        names = [f"f{i}" for i in range(32)]
        row = [0.1 * ((i * 7) % 13 - 6) for i in range(32)]
        label = "xgboost-1000trees-depth8 regressor (tree_perfect HIP kernel, random-init)"
    impl = "SKLEARN_SERVER" if model == "iris" else "XGBOOST_SERVER"
    graph = {"name": "classifier", "type": "MODEL", "implementation": impl,
             "modelUri": "memory://bench", "children": [], "device": device}
    comps = {"classifier": comp}
    if graph_kind != "single":
        graph, comps, glabel = _graph_variant(graph_kind, comp, model, device, len(row))
        label = f"{glabel} [{label}]"
    spec = {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": "bench"},
            "spec": {"name": "bench", "predictors": [{
                "name": "default", "replicas": 1, "componentSpecs": [{"spec": {"containers": []}}],
                "graph": graph}]}}
    dep = sca.Deployment(spec, components=comps, device=device,
                         batcher={"max_batch": 4096, "slots": slots, "spin_wait": spin})
    return dep, names, row, label


def _graph_variant(kind: str, comp, model: str, device: int, n_features: int):
    """Multi-node graphs of BASELINE.json's other configs (extra measurements,
    not the headline): GPU placement spreads nodes over the visible GPUs."""
    import numpy as np

    import seldon_core_amd as sca
    from seldon_core_amd.models import to_row_model

    C = sca.native()
    ngpu = max(1, sca.gpu_count()) if device >= 0 else 1
    dev = (lambda i: (device + i) % ngpu) if device >= 0 else (lambda i: -1)
    rm_a = comp.row_model() if hasattr(comp, "row_model") else to_row_model(comp)
    rm_b = rm_a.clone()
    if kind == "abtest":  # seldon-abtest: RANDOM_ABTEST router over 2 model replicas on 2 GPUs
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST", "device": dev(0),
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "device": dev(0)},
                          {"name": "b", "type": "MODEL", "device": dev(1)}]}
        return g, {"a": rm_a, "b": rm_b}, "RANDOM_ABTEST(2 replicas)"
    if kind == "pipeline":  # transformer -> combiner over 2 models, one stage per GPU (device graph)
        rng = np.random.default_rng(0)
        scale = np.diag(1.0 + 0.01 * rng.random(n_features))
        tr = C.linear_model(scale, np.zeros(n_features), 0)  # standard-scaler-style affine transform
        g = {"name": "scaler", "type": "TRANSFORMER", "device": dev(0), "children": [
            {"name": "combiner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "device": dev(3),
             "children": [{"name": "a", "type": "MODEL", "device": dev(1)},
                          {"name": "b", "type": "MODEL", "device": dev(2)}]}]}
        return g, {"scaler": tr, "a": rm_a, "b": rm_b}, "TRANSFORMER->COMBINER(2 models) device graph"
    if kind == "mab":  # epsilon-greedy router over one model replica per GPU
        from seldon_core_amd.components.routers import EpsilonGreedy

        n = max(2, ngpu)
        kids = [{"name": f"m{i}", "type": "MODEL", "device": dev(i)} for i in range(n)]
        comps = {f"m{i}": (rm_a if i == 0 else rm_a.clone()) for i in range(n)}
        comps["mab"] = EpsilonGreedy(n_branches=n, epsilon=0.1, seed=1)
        g = {"name": "mab", "type": "ROUTER", "device": dev(0), "children": kids}
        return g, comps, f"EPSILON_GREEDY router over {n} replicas"
    raise ValueError(kind)


def run_loadgen(args, port: int, steps: int, warmup: int, api: str, body: bytes | str) -> dict:
    lg = os.path.join(ROOT, "seldon_core_amd", "bin", "sca_loadgen")
    cmd = [lg, "--host", "127.0.0.1", "--port", str(port), "--users", str(args.users),
           "--threads", str(args.client_threads), "--steps", str(steps), "--warmup", str(warmup),
           "--step-requests", str(args.step_requests)]
    if api == "rest":
        cmd += ["--mode", "rest", "--path", "/api/v0.1/predictions", "--body", body]
    else:
        path = f"/tmp/sca_bench_req_{os.getpid()}.pb"
        with open(path, "wb") as f:
            f.write(body)
        cmd += ["--mode", "grpc", "--path", "/seldon.protos.Seldon/Predict", "--body-file", path,
                "--streams-per-conn", "8"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
    if res.returncode not in (0, 1) or not res.stdout.strip():
        raise RuntimeError(f"loadgen failed rc={res.returncode}: {res.stderr[-2000:]}")
    out = json.loads(res.stdout.strip().splitlines()[-1])
    if out["errors"]:
        raise RuntimeError(f"loadgen saw {out['errors']} failed requests")
    return out


def main() -> None:
    args = parse_args()
    import torch

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    has_gpu = torch.cuda.is_available()
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        if has_gpu:
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl" if has_gpu else "gloo")
    device = local_rank if has_gpu else -1

    def barrier():
        if dist is not None:
            if has_gpu:
                dist.barrier(device_ids=[local_rank])
            else:
                dist.barrier()

    def sync():
        if has_gpu:
            torch.cuda.synchronize()

    size_threads(args, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    dep, names, row, label = build_deployment(args.model, device, args.graph, args.slots, not args.no_spin)
    handle = dep.serve(http_port=0, grpc_port=0, threads=args.server_threads, host="127.0.0.1")
    payload = json.dumps({"data": {"names": names, "ndarray": [row]}})
    C = dep.C
    if args.api == "rest":
        body, port = payload, handle.http_port
    else:
        body, port = C.json_to_pb(json.dumps({"data": {"names": names, "tensor": {"shape": [1, len(row)],
                                                                                   "values": row}}})), handle.grpc_port
    # warmup (untimed)
    if args.warmup > 0:
        run_loadgen(args, port, args.warmup, 0, args.api, body)
    for u in dep.batched.values():
        u.reset_stats()
    barrier()
    sync()
    t0 = time.perf_counter()
    lg = run_loadgen(args, port, args.steps, 0, args.api, body)
    sync()
    barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    stats = {k: v.stats() for k, v in dep.batched.items()}
    mine = {"ok": lg["ok"], "wall": wall, "rps": lg["ok"] / wall, "p50": lg["p50_ms"], "p99": lg["p99_ms"],
            "p90": lg["p90_ms"], "lg_rps": lg["rps"], "batch": stats}
    extra = None
    if args.extra_grpc and args.api == "rest":
        gbody = C.json_to_pb(json.dumps({"data": {"names": names, "tensor": {"shape": [1, len(row)], "values": row}}}))
        g = run_loadgen(args, handle.grpc_port, max(2, args.steps // 2), 1, "grpc", gbody)
        extra = {"rps": g["rps"], "p50": g["p50_ms"], "p99": g["p99_ms"]}
    results = [mine]
    extras = [extra]
    if dist is not None:
        results = [None] * world
        dist.all_gather_object(results, mine)
        extras = [None] * world
        dist.all_gather_object(extras, extra)
    handle.stop()
    dep.close()
    if rank == 0:
        # whole-job throughput: every rank's completed predictions over the
        # slowest rank's timed window
        wall_max = max(r["wall"] for r in results)
        value = sum(r["ok"] for r in results) / wall_max
        ms_per_step = wall_max / args.steps * 1000.0
        base = REST_BASELINE if args.api == "rest" else GRPC_BASELINE
        batch = next(iter(results[0]["batch"].values()), {}) if results[0]["batch"] else {}
        mean_rows = batch.get("rows", 0) / max(1, batch.get("batches", 1))
        line = {
            "metric": "predictions/sec (%s graph, %s)" % ("single-model" if args.graph == "single" else args.graph,
                                                          args.api.upper()),
            "value": round(value, 2), "unit": "predictions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / base, 3), "dtype": "fp64",
            "data": ("synthetic (locust-shaped JSON payload, iris feature row); model fit on sklearn's bundled iris"
                     if args.model == "iris" else
                     f"synthetic (locust-shaped JSON payload, {len(row)}-feature random row); random-init model"),
            "p50_ms": round(max(r["p50"] for r in results), 4), "p99_ms": round(max(r["p99"] for r in results), 4),
            "baseline": {"rest_rps": REST_BASELINE, "rest_p50_ms": 4, "rest_p99_ms": 69, "grpc_rps": GRPC_BASELINE,
                         "grpc_p50_ms": 1, "grpc_p99_ms": 6},
            "config": {"model": label, "global_batch": args.users * world, "seq_len": len(row),
                       "parallelism": f"dp{world}", "graph": args.graph, "api": args.api,
                       "users_per_gpu": args.users, "requests_per_step_per_gpu": args.step_requests,
                       "device": "gpu" if has_gpu else "cpu", "gpu_batches": batch.get("batches", 0),
                       "mean_rows_per_gpu_batch": round(mean_rows, 2),
                       "gpu_busy_frac_per_slot": round(batch.get("gpu_busy_s", 0.0) /
                                                       max(1e-9, results[0]["wall"] * args.slots), 3),
                       "slots": args.slots, "server_threads": args.server_threads,
                       "client_threads": args.client_threads, "host_cpus": os.cpu_count(),
                       "cpu_budget": round(cpu_budget(), 2)},
        }
        if extras[0] is not None:
            g_rps = sum(e["rps"] for e in extras if e)
            line["grpc"] = {"value": round(g_rps, 2), "vs_baseline": round(g_rps / GRPC_BASELINE, 3),
                            "p50_ms": max(e["p50"] for e in extras if e), "p99_ms": max(e["p99"] for e in extras if e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
