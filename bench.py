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

Launch: ``python bench.py --gpus N`` spawns N rank processes itself (fresh
processes, before anything touches a GPU); under ``torch.distributed.run`` the
ranks come from the environment and ``--gpus`` must equal ``WORLD_SIZE``.

A "step" is ``--step-requests`` completed predictions per rank.  W warmup steps
run untimed; K steps are timed between a barrier + device synchronize on both
sides; ms_per_step is the max over ranks; ``value`` is the whole-job
predictions/s.

After the timed headline (never inside it) every rank:

* checks a sample of responses, sent through the same front end, against a CPU
  oracle (scikit-learn for iris, the host tree walker for xgboost) and exits
  non-zero on a mismatch;
* measures the gRPC API (``seldon.protos.Seldon/Predict``, Tensor payload);
* with N >= 2, measures BASELINE.json's multi-GPU graph configs with their
  nodes placed on distinct GPUs of the rank's GPU group: ``abtest`` (RANDOM_ABTEST
  over 2 model replicas on 2 GPUs), ``pipeline`` (transformer -> combiner over 2
  models, 4 GPUs, N >= 4) and ``mab`` (epsilon-greedy router over one replica per
  GPU of the job, with concurrent feedback traffic so the bandit learns), each
  self-checked the same way and reporting its per-GPU batch counts.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REST_BASELINE = 12088.95
GRPC_BASELINE = 28256.39
VARIANT_SPAN = {"abtest": 2, "pipeline": 4}  # GPUs a variant's graph spans (mab: all of the job's)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--api", choices=["rest", "grpc"], default="rest")
    ap.add_argument("--model", choices=["iris", "xgb1000", "python-iris", "python-noop"], default="iris",
                    help="iris/xgb1000: prepackaged servers on HIP kernels; python-*: user Python classes "
                         "(the reference's wrapper-microservice workload)")
    ap.add_argument("--py-batching", type=int, default=4096,
                    help="python-* models: stack concurrent requests up to this many rows (0 = off)")
    ap.add_argument("--py-workers", type=int, default=0, help="python-* models: worker processes (0 = in-process)")
    ap.add_argument("--users", type=int, default=256, help="concurrent clients per GPU")
    ap.add_argument("--step-requests", type=int, default=40000, help="predictions per step per GPU")
    ap.add_argument("--server-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--client-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--slots", type=int, default=4, help="GPU batches in flight per unit")
    ap.add_argument("--no-spin", action="store_true", help="block on events instead of spinning")
    ap.add_argument("--graph", choices=["single", "abtest", "pipeline", "mab"], default="single",
                    help="graph of the timed region (single = the headline single-model graph)")
    ap.add_argument("--extras", choices=["auto", "none"], default="auto",
                    help="after the timed region: gRPC + multi-GPU graph variants (auto) or nothing")
    ap.add_argument("--extra-steps", type=int, default=2, help="steps per extra measurement")
    ap.add_argument("--cpu-profile", default=None,
                    help="write a sampling CPU profile of the serving process over the timed window to this JSON file")
    ap.add_argument("--cpu-profile-depth", type=int, default=1, help="frames per CPU-profile sample (>1: call paths)")
    ap.add_argument("--variants-child", default=None, help=argparse.SUPPRESS)  # internal: isolated variant runner
    ap.add_argument("--pin", choices=["auto", "none"], default="auto",
                    help="pin each rank (front end, device thread, load generator) to whole CCDs local to its GPU")
    ap.add_argument("--fabric-probe", choices=["auto", "none"], default="auto",
                    help="N >= 2: after everything else, run tools/fabric_probe.py in child processes "
                         "(rank-placed graph nodes over the RCCL p2p fabric) under a time limit")
    ap.add_argument("--extra-grpc", action="store_true", help="(kept for old command lines; gRPC is an auto extra)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launch
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Direct launch with --gpus N: start N fresh rank processes (no GPU has
    been touched in this one) and exit with the first failing rank's code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    pending = set(range(n))
    while pending:
        for r in list(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.discard(r)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # a failed rank would leave the others in a collective
                    procs[q].terminate()
        time.sleep(0.05)
    return rc


# ------------------------------------------------------------------ sizing
def cpu_budget() -> float:
    """CPUs this process may use: the smaller of the cgroup v2 quota (cpu.max)
    and the CPU affinity mask."""
    limits = []
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            limits.append(float(quota) / float(period))
    except (OSError, ValueError):
        pass
    try:
        limits.append(float(len(os.sched_getaffinity(0))))
    except AttributeError:
        limits.append(float(os.cpu_count() or 8))
    return min(limits)


def size_threads(args, per_rank: float) -> float:
    """Split the CPU share of one rank between the front end (~60%), the
    closed-loop load generator (~25%) and the GPU device / hand-off threads
    (measured on a 16-CPU MI355X share: 10 front-end / 5 generator threads
    was the best split unpinned, profiles/r01f_sweep_executor; pinned to one
    CCD, 10 / 4 serves 1.44M vs 1.38M REST pred/s with p99 0.29-0.35 vs
    0.46-1.08 ms, and gRPC 2.10M vs 1.99M, profiles/r02v_threads)."""
    per_rank = max(2.0, per_rank)
    if args.server_threads is None:
        args.server_threads = max(1, min(16, int(round(per_rank * 0.6))))
    if args.client_threads is None:
        args.client_threads = max(1, min(10, int(round(per_rank * 0.25))))
    return per_rank


def place_rank(args, d) -> tuple:
    """(per-rank CPU budget, pinned CPUs): with --pin auto each rank is pinned
    to whole CCDs local to its GPU (seldon_core_amd.utils.topology), so its
    front end, device thread and load generator share one L3."""
    per_rank = cpu_budget() / max(1, d.local_world)
    if args.pin != "auto" or not d.has_gpu:
        return per_rank, []
    from seldon_core_amd.utils import topology

    # One CCD (16 logical CPUs on MI355X hosts) is the measured sweet spot
    # (profiles/r02m_pinning): a rank with a larger share still takes one, so
    # N = 1 and N = 8 on an unconstrained node run the same per-rank setup.
    per_rank = min(per_rank, 16.0)
    cpus = topology.pin(d.local_rank, int(round(per_rank)))
    return per_rank, cpus


def cpu_ranges(cpus) -> str:
    out, i = [], 0
    cpus = sorted(cpus)
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


# ------------------------------------------------------------------ graphs
class Workload:
    """The benchmark model: component, payload row, names and a CPU oracle."""

    def __init__(self, model: str):
        from seldon_core_amd.servers import SKLearnServer, XGBoostServer

        self.model = model
        if model == "iris":
            from seldon_core_amd.models import iris_logistic_regression

            self.clf = iris_logistic_regression()
            self.comp = SKLearnServer(model=self.clf)
            self.names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
            self.row = [5.1, 3.5, 1.4, 0.2]
            self.label = "sklearn-iris-LogisticRegression (linear_softmax HIP kernel, fp64)"
            self.impl = "SKLEARN_SERVER"
        elif model in ("python-iris", "python-noop"):
            from seldon_core_amd.components.examples import EchoModel, IrisClassifier

            self.names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
            self.row = [5.1, 3.5, 1.4, 0.2]
            if model == "python-iris":
                self.comp = IrisClassifier()
                self.clf = self.comp.model
                self.label = "user Python class IrisClassifier (sklearn LogisticRegression.predict_proba)"
            else:
                self.comp = EchoModel()
                self.label = "user Python class EchoModel (no-op predict)"
            self.impl = None
        else:
            from seldon_core_amd.models import synthetic_xgboost

            self.ens = synthetic_xgboost(1000, 8, 32, seed=0)
            self.comp = XGBoostServer(ensemble=self.ens)
            self.names = [f"f{i}" for i in range(32)]
            self.row = [0.1 * ((i * 7) % 13 - 6) for i in range(32)]
            self.label = "xgboost-1000trees-depth8 regressor (tree_perfect HIP kernel, random-init)"
            self.impl = "XGBOOST_SERVER"

    def oracle(self, X):
        import numpy as np

        if self.model in ("iris", "python-iris"):
            return self.clf.predict_proba(X)
        if self.model == "python-noop":
            return np.asarray(X, dtype=np.float64)
        return np.asarray(self.ens.predict(X), dtype=np.float64).reshape(len(X), -1)

    def sample(self, n: int, seed: int):
        import numpy as np

        rng = np.random.default_rng(seed)
        base = np.asarray(self.row)
        return base + rng.normal(scale=0.5, size=(n, len(base)))


def group_devices(rank: int, span: int, ngpu: int):
    """GPUs of a variant graph on `rank`: the rank's group of `span` GPUs,
    rotated so the graph's first node sits on the rank's own GPU."""
    if ngpu <= 0:
        return [-1] * span
    base = (rank // span) * span
    return [(base + (rank + i) % span) % ngpu for i in range(span)]


def build_graph(wl: Workload, kind: str, devs):
    """SeldonDeployment graph + components for one graph kind on devices `devs`."""
    import numpy as np

    import seldon_core_amd as sca
    from seldon_core_amd.models import to_row_model

    if kind == "single":
        g = {"name": "classifier", "type": "MODEL", "children": [], "device": devs[0]}
        if wl.impl:
            g.update(implementation=wl.impl, modelUri="memory://bench")
        else:  # a user Python class
            g.update(batching=wl.py_batching, workers=wl.py_workers)
        label = wl.label
        if not wl.impl:
            label += f" [batching={wl.py_batching}, workers={wl.py_workers}]"
        return g, {"classifier": wl.comp}, wl.oracle, label
    C = sca.native()
    rm_a = wl.comp.row_model() if hasattr(wl.comp, "row_model") else to_row_model(wl.comp)
    if kind == "abtest":  # seldon-abtest: RANDOM_ABTEST router over 2 model replicas on 2 GPUs
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST", "device": devs[0],
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "device": devs[0]},
                          {"name": "b", "type": "MODEL", "device": devs[1]}]}
        return g, {"a": rm_a, "b": rm_a.clone()}, wl.oracle, f"RANDOM_ABTEST(2 replicas on GPUs {devs[:2]})"
    if kind == "pipeline":  # transformer -> combiner over 2 models, one stage per GPU (device graph)
        F = len(wl.row)
        scale = 1.0 + 0.01 * np.random.default_rng(0).random(F)
        tr = C.linear_model(np.diag(scale), np.zeros(F), 0)  # standard-scaler-style affine transform
        g = {"name": "scaler", "type": "TRANSFORMER", "device": devs[0], "children": [
            {"name": "combiner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "device": devs[3],
             "children": [{"name": "a", "type": "MODEL", "device": devs[1]},
                          {"name": "b", "type": "MODEL", "device": devs[2]}]}]}
        return (g, {"scaler": tr, "a": rm_a, "b": rm_a.clone()}, lambda X: wl.oracle(np.asarray(X) * scale),
                f"TRANSFORMER->COMBINER(2 models) device graph on GPUs {devs[:4]}")
    if kind == "mab":  # epsilon-greedy router over one model replica per GPU
        from seldon_core_amd.components.routers import EpsilonGreedy

        n = len(devs)
        kids = [{"name": f"m{i}", "type": "MODEL", "device": devs[i]} for i in range(n)]
        comps = {f"m{i}": (rm_a if i == 0 else rm_a.clone()) for i in range(n)}
        comps["mab"] = EpsilonGreedy(n_branches=n, epsilon=0.1, seed=1)
        g = {"name": "mab", "type": "ROUTER", "device": devs[0], "children": kids}
        return g, comps, wl.oracle, f"EPSILON_GREEDY router over {n} replicas on GPUs {devs}"
    raise ValueError(kind)


def make_deployment(wl: Workload, kind: str, devs, device: int, slots: int, spin: bool):
    import seldon_core_amd as sca

    graph, comps, oracle, label = build_graph(wl, kind, devs)
    spec = {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": "bench"},
            "spec": {"name": "bench", "predictors": [{
                "name": "default", "replicas": 1, "componentSpecs": [{"spec": {"containers": []}}],
                "graph": graph}]}}
    dep = sca.Deployment(spec, components=comps, device=device,
                         batcher={"max_batch": 4096, "slots": slots, "spin_wait": spin})
    return dep, oracle, label


# ------------------------------------------------------------------ load
def run_loadgen(args, port: int, steps: int, warmup: int, api: str, body, path: str = "/api/v0.1/predictions",
                users: int | None = None, step_requests: int | None = None, threads: int | None = None) -> dict:
    lg = os.path.join(ROOT, "seldon_core_amd", "bin", "sca_loadgen")
    cmd = [lg, "--host", "127.0.0.1", "--port", str(port), "--users", str(users or args.users),
           "--threads", str(threads or args.client_threads), "--steps", str(steps), "--warmup", str(warmup),
           "--step-requests", str(step_requests or args.step_requests)]
    if api == "rest":
        cmd += ["--mode", "rest", "--path", path, "--body", body]
    else:
        bpath = f"/tmp/sca_bench_req_{os.getpid()}.pb"
        with open(bpath, "wb") as f:
            f.write(body)
        cmd += ["--mode", "grpc", "--path", "/seldon.protos.Seldon/Predict", "--body-file", bpath,
                "--streams-per-conn", "8"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
    if res.returncode not in (0, 1) or not res.stdout.strip():
        raise RuntimeError(f"loadgen failed rc={res.returncode}: {res.stderr[-2000:]}")
    out = json.loads(res.stdout.strip().splitlines()[-1])
    if out["errors"]:
        raise RuntimeError(f"loadgen saw {out['errors']} failed requests")
    return out


def self_check(port: int, wl: Workload, oracle, seed: int, n: int = 24) -> dict:
    """Send distinct rows through the REST front end (one-row requests and one
    batch) and compare with the CPU oracle."""
    import numpy as np

    X = wl.sample(n, seed)
    got = []

    def post(rows):
        body = json.dumps({"data": {"names": wl.names, "ndarray": rows.tolist()}}).encode()
        req = urllib.request.Request(f"http://127.0.0.1:{port}/api/v0.1/predictions", data=body,
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=30) as r:
            out = np.asarray(json.loads(r.read())["data"]["ndarray"], dtype=np.float64)
            return out.reshape(len(rows), -1)  # regressors answer one flat value per row

    for i in range(n // 2):
        got.append(post(X[i:i + 1]))
    got.append(post(X[n // 2:]))
    got = np.vstack(got)
    ref = np.asarray(oracle(X), dtype=np.float64).reshape(got.shape)
    err = float(np.abs(got - ref).max())
    tol = 1e-4 * max(1.0, float(np.abs(ref).max())) if wl.model == "xgb1000" else 1e-9
    return {"rows": n, "max_abs_err": err, "tol": tol, "ok": bool(err <= tol)}


def unit_stats(dep) -> dict:
    per_dev: dict = {}
    total = {"batches": 0, "rows": 0, "gpu_busy_s": 0.0, "launch_cpu_s": 0.0, "complete_cpu_s": 0.0}
    for name, st in dep.batcher_stats().items():
        if not isinstance(st, dict):
            continue
        for k in total:
            total[k] += st.get(k, 0)
        entries = st.get("per_device") or [{"device": st.get("device", -1), "batches": st.get("batches", 0),
                                            "rows": st.get("rows", 0)}]
        for e in entries:
            d = per_dev.setdefault(str(e["device"]), {"batches": 0, "rows": 0, "units": []})
            d["batches"] += e["batches"]
            d["rows"] += e["rows"]
            d["units"].append(name)
    total["per_device"] = per_dev
    return total


class Dist:
    def __init__(self, backend: str | None = None):
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_world = int(os.environ.get("LOCAL_WORLD_SIZE", self.world))
        import torch

        self.torch = torch
        self.has_gpu = torch.cuda.is_available()
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist

            if self.has_gpu:
                torch.cuda.set_device(self.local_rank)
            self.backend = backend or ("nccl" if self.has_gpu else "gloo")
            dist.init_process_group(backend=self.backend)
            self.dist = dist
        self.device = self.local_rank if self.has_gpu else -1

    def barrier(self):
        if self.dist is not None:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.local_rank])
            else:
                self.dist.barrier()

    def sync(self):
        if self.has_gpu:
            self.torch.cuda.synchronize()

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def cpu_seconds() -> tuple:
    """(this process: front end + device thread + Python, reaped children:
    the load generator) user+sys CPU seconds."""
    import resource

    me = resource.getrusage(resource.RUSAGE_SELF)
    ch = resource.getrusage(resource.RUSAGE_CHILDREN)
    return me.ru_utime + me.ru_stime, ch.ru_utime + ch.ru_stime


def timed(d: Dist, fn, cpu: dict | None = None):
    d.barrier()
    d.sync()
    c0 = cpu_seconds()
    t0 = time.perf_counter()
    err = None
    try:
        out = fn()
    except Exception as e:  # still meet the closing barrier, or the other ranks would wait forever
        out, err = None, e
    d.sync()
    wall = time.perf_counter() - t0
    if cpu is not None:  # CPUs busy over the window, server side vs load generator
        c1 = cpu_seconds()
        cpu["server_cpus"] = round((c1[0] - c0[0]) / wall, 2)
        cpu["loadgen_cpus"] = round((c1[1] - c0[1]) / wall, 2)
    d.barrier()
    if err is not None:
        raise err
    return out, wall


def measure_variant(args, d: Dist, wl: Workload, kind: str, spin: bool) -> dict:
    """One multi-GPU graph config, untimed by the driver contract but timed the
    same way (barrier + sync around the loadgen window, max over ranks)."""
    import seldon_core_amd as sca

    ngpu = sca.gpu_count() if d.has_gpu else 0
    span = max(2, d.world) if kind == "mab" else VARIANT_SPAN[kind]
    devs = group_devices(d.rank, span, ngpu)
    body = json.dumps({"data": {"names": wl.names, "ndarray": [wl.row]}})
    sreq = max(1000, args.step_requests // 2)
    dep = h = None
    setup_error = None
    try:  # everything rank-local first: a rank that fails here must not skip a collective alone
        if os.environ.get("SCA_BENCH_FAULT") == f"{kind}:{d.rank}":  # fault injection (tests)
            raise RuntimeError(f"injected {kind} setup fault")
        dep, oracle, label = make_deployment(wl, kind, devs, d.device, args.slots, spin)
        h = dep.serve(http_port=0, grpc_port=0, threads=args.server_threads, host="127.0.0.1")
        run_loadgen(args, h.http_port, 1, 0, "rest", body, step_requests=sreq)  # warm every replica
    except Exception as e:
        setup_error = f"rank {d.rank}: {type(e).__name__}: {e}"[:400]
    errors = [e for e in d.gather(setup_error) if e]
    fb = None
    try:
        if errors:  # every rank skips the variant together
            raise RuntimeError("; ".join(errors))
        for u in dep.batched.values():
            u.reset_stats()
        fb_out = {}
        if kind == "mab":
            # feedback traffic next to the predictions (reference MAB loadtest:
            # util/loadtester/scripts/predict_rest_locust.py sends feedback):
            # branch 0 is rewarded, so the bandit must keep routing to it.
            fbody = json.dumps({"request": {"data": {"names": wl.names, "ndarray": [wl.row]}},
                                "response": {"meta": {"routing": {"mab": 0}}, "data": {"ndarray": [[0.0]]}},
                                "reward": 1.0})
            fb = threading.Thread(target=lambda: fb_out.update(run_loadgen(
                args, h.http_port, args.extra_steps, 0, "rest", fbody, path="/api/v0.1/feedback",
                users=max(4, args.users // 16), step_requests=max(200, sreq // 16),
                threads=max(1, args.client_threads // 4))))
            fb.start()
        lg, wall = timed(d, lambda: run_loadgen(args, h.http_port, args.extra_steps, 0, "rest", body,
                                                step_requests=sreq))
        if fb is not None:
            fb.join()
        check = self_check(h.http_port, wl, oracle, seed=100 + d.rank)
        st = unit_stats(dep)
        res = {"ok": lg["ok"], "wall": wall, "p50": lg["p50_ms"], "p99": lg["p99_ms"], "check": check,
               "devices": devs, "label": label, "stats": st}
        if fb_out:
            res["feedback_rps"] = fb_out.get("rps")
            routed = {k: v["rows"] for k, v in st["per_device"].items()}
            res["rows_per_device"] = routed
        return res
    finally:
        if h is not None:
            h.stop()
        if dep is not None:
            dep.close()


def child_env(d: "Dist", port: int) -> dict:
    """Environment of a per-rank child that forms its own process group on
    `port`.  Under torch.distributed.run the ranks carry
    TORCHELASTIC_USE_AGENT_STORE=True (connect to the launcher's store instead
    of hosting one): a child must not inherit that, or every rank would wait
    for a store nobody serves on the new port."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(RANK=str(d.rank), LOCAL_RANK=str(d.local_rank), WORLD_SIZE=str(d.world),
               LOCAL_WORLD_SIZE=str(d.local_world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def run_variants_isolated(args, d: Dist, argv, kinds, timeout_s: float = 900.0) -> dict:
    """Run the multi-GPU graph variants in a child process per rank (a fresh
    gloo process group on a new port): a device fault or hang while nodes of
    a graph talk across GPUs ends the child, which is recorded, instead of the
    rank that still has to print the headline line."""
    import signal

    box = [_free_port() if d.rank == 0 else None]
    if d.dist is not None:
        d.dist.broadcast_object_list(box, src=0)
    env = child_env(d, box[0])
    child_argv = [a for a in argv if a != "--variants-child"]
    cmd = [sys.executable, os.path.abspath(__file__), *child_argv, "--variants-child", ",".join(kinds),
           "--server-threads", str(args.server_threads), "--client-threads", str(args.client_threads)]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout_s)
        status = None if p.returncode == 0 else f"variant runner rc={p.returncode}: {(err or '')[-400:]}"
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        status = f"variant runner timed out after {timeout_s:.0f}s"
    res = {}
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if lines:
        try:
            res = json.loads(lines[-1])
        except ValueError:
            pass
    for kind in kinds:
        if kind not in res:
            res[kind] = {"error": status or "variant runner printed no result"}
    return res


def variants_child(args) -> None:
    """Entry of the isolated variant runner: measure each kind, print one JSON
    line {kind: result} for this rank."""
    d = Dist(backend="gloo")
    import seldon_core_amd  # noqa: F401

    wl = Workload(args.model)
    wl.py_batching, wl.py_workers = args.py_batching, args.py_workers
    out = {}
    for kind in args.variants_child.split(","):
        try:
            out[kind] = measure_variant(args, d, wl, kind, spin=False)
        except Exception as e:
            out[kind] = {"error": f"{type(e).__name__}: {e}"[:600]}
    print(json.dumps(out), flush=True)
    d.close()


def fabric_probe(d: Dist, timeout_s: float = 150.0, requests: int = 200):
    """Cross-process graph placement over the p2p fabric: every
    rank starts ``tools/fabric_probe.py`` as a child process in a fresh
    process group (rank 0 hosts an AVERAGE_COMBINER whose MODEL children live
    on every rank; batches and replies travel as RCCL send/recv on GPUs).  It
    runs after the measurements, in children under a time limit, so a hang or
    fault there is recorded instead of costing the benchmark line.  Returns
    rank 0's summary (None on other ranks)."""
    import signal

    box = [_free_port() if d.rank == 0 else None]
    if d.dist is not None:
        d.dist.broadcast_object_list(box, src=0)
    env = child_env(d, box[0])
    t0 = time.perf_counter()
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "fabric_probe.py"), "--requests", str(requests)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout_s)
        status = "ok" if p.returncode == 0 else f"rc={p.returncode}"
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        status = f"timeout after {timeout_s:.0f}s"
    res = {"rank": d.rank, "status": status, "wall_s": round(time.perf_counter() - t0, 2)}
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if lines:
        try:
            res["probe"] = json.loads(lines[-1])
        except ValueError:
            pass
    if status != "ok":
        res["stderr_tail"] = (err or "")[-600:]
    allr = d.gather(res)
    if d.rank != 0:
        return None
    top = allr[0].get("probe") or {}
    return {"ok": all(r["status"] == "ok" for r in allr), "world": d.world,
            "data_plane": top.get("data_plane"), "requests": top.get("requests"),
            "max_abs_err": top.get("max_abs_err"), "req_per_s": round(top.get("req_per_s", 0.0), 1),
            "units": top.get("units"), "ranks": [{k: r[k] for k in r if k != "probe"} for r in allr]}


def main() -> None:
    argv = sys.argv[1:]
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)

    if args.variants_child:
        variants_child(args)
        return
    d = Dist()
    per_rank_budget, pinned = place_rank(args, d)
    per_rank_cpus = size_threads(args, per_rank_budget)
    spin = not args.no_spin
    import seldon_core_amd as sca

    wl = Workload(args.model)
    wl.py_batching, wl.py_workers = args.py_batching, args.py_workers
    ngpu = sca.gpu_count() if d.has_gpu else 0
    devs = [d.device] if args.graph == "single" else group_devices(
        d.rank, max(2, d.world) if args.graph == "mab" else VARIANT_SPAN[args.graph], ngpu)
    dep, oracle, label = make_deployment(wl, args.graph, devs, d.device, args.slots, spin)
    if args.graph != "single":
        if not wl.impl:
            raise SystemExit("multi-node --graph variants use the kernel models (iris / xgb1000)")
        label = f"{label} [{wl.label}]"
    handle = dep.serve(http_port=0, grpc_port=0, threads=args.server_threads, host="127.0.0.1")
    C = dep.C
    payload = json.dumps({"data": {"names": wl.names, "ndarray": [wl.row]}})
    pb = C.json_to_pb(json.dumps({"data": {"names": wl.names,
                                           "tensor": {"shape": [1, len(wl.row)], "values": wl.row}}}))
    if args.api == "rest":
        body, port = payload, handle.http_port
    else:
        body, port = pb, handle.grpc_port
    if args.warmup > 0:  # untimed
        run_loadgen(args, port, args.warmup, 0, args.api, body)
    for u in dep.batched.values():
        u.reset_stats()
    cpu: dict = {}
    if args.cpu_profile:
        from seldon_core_amd.utils import cpuprof

        cpuprof.start(depth=args.cpu_profile_depth)
    lg, wall = timed(d, lambda: run_loadgen(args, port, args.steps, 0, args.api, body), cpu)
    if args.cpu_profile:
        prof = cpuprof.stop()
        prof.update(rps=round(lg["ok"] / wall, 1), server_cpus=cpu.get("server_cpus"), rank=d.rank)
        with open(args.cpu_profile if d.world == 1 else f"{args.cpu_profile}.rank{d.rank}", "w") as f:
            json.dump(prof, f, indent=1)
    st = unit_stats(dep)
    mine = {"rank": d.rank, "device": d.device, "ok": lg["ok"], "wall": wall, "p50": lg["p50_ms"],
            "p99": lg["p99_ms"], "stats": st, "cpu_budget": round(per_rank_cpus, 2), "cpu": cpu,
            "pinned_cpus": cpu_ranges(pinned) if pinned else None}
    extras: dict = {}
    failures = []
    # ---- after the timed region: correctness + extra configs
    chk = self_check(handle.http_port, wl, oracle, seed=d.rank)
    mine["check"] = chk
    if not chk["ok"]:
        failures.append(f"rank {d.rank} headline self-check: {chk}")
    if args.extras == "auto" and args.graph == "single":
        try:
            g, gwall = timed(d, lambda: run_loadgen(args, handle.grpc_port, args.extra_steps, 0, "grpc", pb))
            extras["grpc"] = {"ok": g["ok"], "wall": gwall, "p50": g["p50_ms"], "p99": g["p99_ms"]}
        except Exception as e:  # reported; the headline stands
            extras["grpc"] = {"error": f"{type(e).__name__}: {e}"[:600]}
    handle.stop()
    dep.close()
    if args.extras == "auto" and args.graph == "single" and d.world >= 2 and wl.impl:
        kinds = ["abtest"] + (["pipeline"] if d.world >= 4 else []) + ["mab"]
        for kind, r in run_variants_isolated(args, d, argv, kinds).items():
            if "error" not in r and not r["check"]["ok"]:
                failures.append(f"rank {d.rank} {kind} self-check: {r['check']}")
            extras[kind] = r
    results = d.gather({"mine": mine, "extras": extras, "failures": failures})
    fabric = None
    if args.extras == "auto" and args.fabric_probe == "auto" and d.world >= 2:
        fabric = fabric_probe(d)
    if d.rank == 0:
        line = summarize(args, d, results, label, wl)
        if fabric is not None:
            line["rccl_fabric"] = fabric
        print(json.dumps(line), flush=True)
    bad = [f for r in results for f in r["failures"]]
    d.close()
    if bad:
        print("bench.py: self-check FAILED: " + "; ".join(bad), file=sys.stderr)
        sys.exit(3)


def summarize(args, d: Dist, results, label: str, wl: Workload) -> dict:
    mines = [r["mine"] for r in results]
    # whole-job throughput: every rank's completed predictions over the
    # slowest rank's timed window
    wall_max = max(m["wall"] for m in mines)
    value = sum(m["ok"] for m in mines) / wall_max
    base = REST_BASELINE if args.api == "rest" else GRPC_BASELINE
    st0 = mines[0]["stats"]
    per_rank = [{"rank": m["rank"], "device": m["device"], "cpu_budget": m["cpu_budget"],
                 "pinned_cpus": m.get("pinned_cpus"), **m["cpu"],
                 "rps": round(m["ok"] / m["wall"], 1), "p50_ms": m["p50"], "p99_ms": m["p99"],
                 "gpu_batches": m["stats"]["batches"],
                 "mean_rows_per_batch": round(m["stats"]["rows"] / max(1, m["stats"]["batches"]), 2),
                 # share of the window the GPU device thread spent launching / handing off responses
                 "device_thread_launch_frac": round(m["stats"]["launch_cpu_s"] / m["wall"], 3),
                 "device_thread_complete_frac": round(m["stats"]["complete_cpu_s"] / m["wall"], 3),
                 "check_max_abs_err": m["check"]["max_abs_err"]} for m in mines]
    line = {
        "metric": "predictions/sec (%s graph, %s)" % ("single-model" if args.graph == "single" else args.graph,
                                                      args.api.upper()),
        "value": round(value, 2), "unit": "predictions/s", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1000.0, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": round(value / base, 3), "dtype": "fp64",
        "data": ("synthetic (locust-shaped JSON payload, iris feature row); model fit on sklearn's bundled iris"
                 if args.model in ("iris", "python-iris", "python-noop") else
                 f"synthetic (locust-shaped JSON payload, {len(wl.row)}-feature random row); random-init model"),
        "p50_ms": round(max(m["p50"] for m in mines), 4), "p99_ms": round(max(m["p99"] for m in mines), 4),
        "baseline": {"rest_rps": REST_BASELINE, "rest_p50_ms": 4, "rest_p99_ms": 69, "grpc_rps": GRPC_BASELINE,
                     "grpc_p50_ms": 1, "grpc_p99_ms": 6},
        "self_check": {"ok": all(m["check"]["ok"] for m in mines),
                       "max_abs_err": max(m["check"]["max_abs_err"] for m in mines)},
        "config": {"model": label, "global_batch": args.users * d.world, "seq_len": len(wl.row),
                   "parallelism": f"dp{d.world}", "graph": args.graph, "api": args.api,
                   "users_per_gpu": args.users, "requests_per_step_per_gpu": args.step_requests,
                   "device": "gpu" if d.has_gpu else "cpu", "gpu_batches": st0["batches"],
                   "mean_rows_per_gpu_batch": round(st0["rows"] / max(1, st0["batches"]), 2),
                   "gpu_busy_frac_per_slot": round(st0["gpu_busy_s"] / max(1e-9, mines[0]["wall"] * args.slots), 3),
                   "slots": args.slots, "server_threads": args.server_threads,
                   "client_threads": args.client_threads, "host_cpus": os.cpu_count(),
                   "cpu_budget": round(cpu_budget(), 2), "per_rank": per_rank},
    }
    ex = [r["extras"] for r in results]
    if any("error" in e.get("grpc", {}) for e in ex):
        line["grpc"] = {"error": next(e["grpc"]["error"] for e in ex if "error" in e.get("grpc", {}))}
    elif ex[0].get("grpc"):
        gw = max(e["grpc"]["wall"] for e in ex)
        g = sum(e["grpc"]["ok"] for e in ex) / gw
        line["grpc"] = {"value": round(g, 2), "vs_baseline": round(g / GRPC_BASELINE, 3),
                        "p50_ms": max(e["grpc"]["p50"] for e in ex), "p99_ms": max(e["grpc"]["p99"] for e in ex)}
    variants = {}
    for kind in ("abtest", "pipeline", "mab"):
        if kind not in ex[0]:
            continue
        rs = [e[kind] for e in ex]
        errs = [r["error"] for r in rs if "error" in r]
        if errs:
            variants[kind] = {"error": errs[0], "ranks_failed": len(errs)}
            continue
        w = max(r["wall"] for r in rs)
        v = sum(r["ok"] for r in rs) / w
        variants[kind] = {
            "graph": rs[0]["label"], "gpus_per_graph": len(rs[0]["devices"]), "n_gpus": d.world,
            "value": round(v, 2), "unit": "predictions/s", "vs_rest_baseline": round(v / REST_BASELINE, 3),
            "p50_ms": max(r["p50"] for r in rs), "p99_ms": max(r["p99"] for r in rs),
            "self_check": {"ok": all(r["check"]["ok"] for r in rs),
                           "max_abs_err": max(r["check"]["max_abs_err"] for r in rs)},
            "rank0_batches_per_device": {k: v2["batches"] for k, v2 in rs[0]["stats"]["per_device"].items()},
        }
        if "feedback_rps" in rs[0]:
            variants[kind]["feedback_rps"] = round(sum(r.get("feedback_rps") or 0 for r in rs), 1)
            variants[kind]["rank0_rows_per_device"] = rs[0].get("rows_per_device")
    if variants:
        line["variants"] = variants
    return line


if __name__ == "__main__":
    main()
