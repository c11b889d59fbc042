#!/usr/bin/env python3
"""Headline serving benchmark (BASELINE.json): predictions/sec + p50/p99
latency of a single-model inference graph, REST API, at N MI355X GPUs.

Reference numbers (doc/source/reference/benchmarking.md:31-64):
REST 12,088.95 req/s (p50 4 ms, p99 69 ms), gRPC 28,256.39 req/s (p50 1 ms,
p99 6 ms), 256 locust users, one engine replica.

Headline: one process per GPU.  Each rank serves one replica of the graph --
the reference's sklearn-iris LogisticRegression model (BASELINE config 1)
executed by the GPU micro-batcher + linear_softmax HIP kernel on its GPU --
through the native HTTP/1.1 front end, and drives it with the native
closed-loop load generator (256 concurrent users per rank, no think time, the
locust REST payload shape, a sampled reply-body check).  Weak scaling: per-GPU
load is fixed as N grows.  A "step" is ``--step-requests`` completed
predictions per rank (default: calibrated so the K timed steps last >= 5 s);
W warmup steps run untimed; K steps are timed between a barrier + device
synchronize on both sides; ms_per_step is the max over ranks; ``value`` is
the whole-job predictions/s.

After the headline (never inside it):

* every rank checks sampled replies against a CPU oracle (scikit-learn for
  iris, the host tree walker for xgboost) and measures the gRPC API;
* with N >= 2, rank 0 measures BASELINE.json's multi-GPU graphs as ONE graph
  over the node's GPUs, each in a child process with its own deadline:
  ``abtest`` (RANDOM_ABTEST over replicas on 2 GPUs), ``pipeline``
  (transformer -> combiner over 2 models, 4 GPUs), ``mab`` (epsilon-greedy
  over one replica per GPU, with concurrent feedback traffic) and
  ``replicas`` (one endpoint over a replica per GPU);
* then every rank starts a fabric child: the same graphs with their nodes
  placed on ranks (``abtest_ranks``, ``pipeline_ranks``, ``mab_ranks``), one
  engine process per GPU; placed subtrees run as mesh programs whose stages
  hand rows to each other directly (HIP IPC + shared-memory doorbells; the
  transport is reported per graph, SCA_FABRIC_TRANSPORT selects another).

Robustness: the whole run has one budget (``BUDGET_S``); every child and load
generator call gets a timeout from what is left; ranks hand results to rank 0
through files (no collective after the headline); a rank-0 watchdog prints
the JSON line when the budget runs out, marking what did not finish as
``"timeout"``, and kills every child process group.

Launch: ``python bench.py --gpus N`` spawns N rank processes itself; under
``torch.distributed.run`` the ranks come from the environment and ``--gpus``
must equal ``WORLD_SIZE``.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from seldon_core_amd.utils import benchkit as bk  # noqa: E402  (no GPU, no torch import)

REST_BASELINE = 12088.95
GRPC_BASELINE = 28256.39
BUDGET_S = float(os.environ.get("SCA_BENCH_BUDGET_S", "420"))  # whole run, well under the driver's 600 s lease
VARIANT_CAP_S = float(os.environ.get("SCA_BENCH_VARIANT_CAP_S", "75"))  # one in-process variant child
TARGET_TIMED_S = float(os.environ.get("SCA_BENCH_TARGET_S", "5"))  # headline timed region when calibrated
EXTRA_WINDOW_S = float(os.environ.get("SCA_BENCH_EXTRA_S", "1.5"))  # gRPC / variant timed windows
PROBE_S = 0.5  # steady-state calibration probe
REPORT_RESERVE_S = 8.0  # rank 0 keeps this much of the budget to write the line
HEAD_RESERVE_S = min(45.0, 0.25 * BUDGET_S)  # left for the report + extras when the headline starts a step
FABRIC_RESERVE_S = min(75.0, 0.3 * BUDGET_S)
EXTRA_RESERVE_S = min(30.0, 0.15 * BUDGET_S)  # left when the gRPC extra starts  # kept for the rank-placed (RCCL) phase while in-process variants run
T_START = time.time()
try:
    ORIG_AFFINITY = sorted(os.sched_getaffinity(0))
except AttributeError:
    ORIG_AFFINITY = []
VARIANTS = ("abtest", "pipeline", "mab", "replicas", "reuseport")
RANK_VARIANTS = ("abtest", "pipeline", "mab")
SPAN = {"abtest": 2, "pipeline": 4}  # GPUs a graph spans (mab / replicas: all of the job's)


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
    ap.add_argument("--step-requests", type=int, default=None,
                    help="predictions per step per GPU (default: calibrated so the timed steps last >= 5 s)")
    ap.add_argument("--server-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--client-threads", type=int, default=None, help="default: sized from the CPU quota per rank")
    ap.add_argument("--slots", type=int, default=4, help="GPU batches in flight per unit")
    ap.add_argument("--no-spin", action="store_true", help="block on events instead of spinning")
    ap.add_argument("--graph", choices=["single", "abtest", "pipeline", "mab", "replicas"], default="single",
                    help="graph of the timed region (single = the headline single-model graph)")
    ap.add_argument("--extras", choices=["auto", "none"], default="auto",
                    help="after the timed region: gRPC + multi-GPU graph variants (auto) or nothing")
    ap.add_argument("--variants", default=",".join(VARIANTS), help="in-process variants to run (N >= 2)")
    ap.add_argument("--rank-variants", default=",".join(RANK_VARIANTS),
                    help="rank-placed (RCCL fabric) variants to run (N >= 2); empty = none")
    ap.add_argument("--cpu-profile", default=None,
                    help="write a sampling CPU profile of the serving process over the timed window to this JSON file")
    ap.add_argument("--cpu-profile-depth", type=int, default=1, help="frames per CPU-profile sample (>1: call paths)")
    ap.add_argument("--pin", choices=["auto", "none"], default="auto",
                    help="pin each rank (front end, device thread, load generator) to whole CCDs local to its GPU")
    # kept for old command lines
    ap.add_argument("--extra-grpc", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--extra-steps", type=int, default=2, help=argparse.SUPPRESS)
    ap.add_argument("--fabric-probe", choices=["auto", "none"], default="auto", help=argparse.SUPPRESS)
    # internal: child processes
    ap.add_argument("--variant-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--fabric-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--span", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--deadline", type=float, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.fabric_probe == "none":
        args.rank_variants = ""
    return args


def fault(kind: str, rank: int) -> None:
    """Fault injection for tests: SCA_BENCH_FAULT is a comma list of
    "<kind>:<rank>" (setup error) or "hang:<kind>:<rank>" (sleep forever at
    that point)."""
    faults = os.environ.get("SCA_BENCH_FAULT", "").split(",")
    if f"{kind}:{rank}" in faults:
        raise RuntimeError(f"injected {kind} setup fault")
    if f"hang:{kind}:{rank}" in faults:
        while True:
            time.sleep(3600)


# ------------------------------------------------------------------ launch
def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Direct launch with --gpus N: start N fresh rank processes (no GPU has
    been touched in this one), all sharing one deadline; exit with rank 0's
    code (rank 0 reports every other rank's failures in its line).  A rank
    still running past the deadline is killed."""
    port = _free_port()
    deadline = T_START + BUDGET_S
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SCA_BENCH_DEADLINE=str(deadline))
        procs.append(bk.CHILDREN.popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                       stdout=None if r == 0 else subprocess.DEVNULL))
    while any(p.poll() is None for p in procs) and time.time() < deadline + 20:
        if procs[0].poll() is not None and procs[0].returncode != 0:
            break  # rank 0 failed: the others would wait for it
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            bk.Children.kill(p)
            p.wait()
    rc0 = procs[0].returncode
    return 124 if rc0 is None or rc0 < 0 else rc0


# ------------------------------------------------------------------ sizing
def size_threads(args, per_rank: float) -> float:
    """Split the CPU share of one rank between the front end (~60%), the
    closed-loop load generator (~30%) and the GPU pump thread.  On a 16-CPU
    MI355X share pinned to one CCD, with responses posted from the pump
    (round 5): 10 front-end / 5 generator threads serve 1.705-1.715M REST
    pred/s (p99 0.23-0.29 ms) against 1.57-1.59M at 10 / 4, 1.62-1.63M at
    11 / 5 and 1.66M at 10 / 6 (profiles/r05x_threads; round 2 had found 10 / 4
    best before the hand-off thread went, profiles/r02v_threads)."""
    per_rank = max(2.0, per_rank)
    if args.server_threads is None:
        args.server_threads = max(1, min(16, int(round(per_rank * 0.6))))
    if args.client_threads is None:
        args.client_threads = max(1, min(10, int(round(per_rank * 0.3125))))
    return per_rank


def place_rank(args, d) -> tuple:
    """(per-rank CPU budget, pinned CPUs): with --pin auto each rank is pinned
    to whole CCDs local to its GPU (seldon_core_amd.utils.topology), so its
    front end, device thread and load generator share one L3."""
    per_rank = bk.cpu_budget() / max(1, d.local_world)
    if args.pin != "auto" or not d.has_gpu:
        return per_rank, []
    from seldon_core_amd.utils import topology

    # One CCD (16 logical CPUs on MI355X hosts) is the measured sweet spot
    # (profiles/r02m_pinning): a rank with a larger share still takes one, so
    # N = 1 and N = 8 on an unconstrained node run the same per-rank setup.
    per_rank = min(per_rank, 16.0)
    cpus = topology.pin(d.local_rank, int(round(per_rank)))
    return per_rank, cpus


# ------------------------------------------------------------------ ranks
class Dist:
    def __init__(self, budget: bk.Budget, backend: str | None = None):
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_world = int(os.environ.get("LOCAL_WORLD_SIZE", self.world))
        import torch

        self.torch = torch
        self.has_gpu = torch.cuda.is_available()
        # SCA_BENCH_FOLD_GPUS=1: every rank on GPU 0 (a rehearsal of the
        # multi-rank flow on a 1-GPU box -- not a scaling measurement; RCCL
        # refuses two ranks on one device, so the collectives use gloo)
        self.fold = os.environ.get("SCA_BENCH_FOLD_GPUS") == "1" and self.has_gpu
        self.gpu_index = 0 if self.fold else self.local_rank
        self.dist = None
        self.backend = None
        if self.world > 1:
            import datetime

            import torch.distributed as dist

            if self.has_gpu:
                torch.cuda.set_device(self.gpu_index)
            self.backend = backend or ("nccl" if self.has_gpu and not self.fold else "gloo")
            dist.init_process_group(backend=self.backend,
                                    timeout=datetime.timedelta(seconds=max(30.0, budget.left())))
            self.dist = dist
        self.device = self.gpu_index if self.has_gpu else -1

    def barrier(self):
        if self.dist is not None:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.gpu_index])
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

    def bcast(self, obj):
        if self.dist is None:
            return obj
        box = [obj if self.rank == 0 else None]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]


def cpu_seconds() -> tuple:
    """(this process: front end + device thread + Python, reaped children:
    the load generator) user+sys CPU seconds."""
    import resource

    me = resource.getrusage(resource.RUSAGE_SELF)
    ch = resource.getrusage(resource.RUSAGE_CHILDREN)
    return me.ru_utime + me.ru_stime, ch.ru_utime + ch.ru_stime


def child_env(d: "Dist", port: int, deadline: float) -> dict:
    """Environment of a per-rank child that forms its own process group on
    `port`.  Under torch.distributed.run the ranks carry
    TORCHELASTIC_USE_AGENT_STORE=True (connect to the launcher's store instead
    of hosting one): a child must not inherit that, or every rank would wait
    for a store nobody serves on the new port."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(RANK=str(d.rank), LOCAL_RANK=str(d.local_rank), WORLD_SIZE=str(d.world),
               LOCAL_WORLD_SIZE=str(d.local_world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               SCA_BENCH_DEADLINE=str(deadline))
    return env


# ------------------------------------------------------------------ report
class Reporter:
    """Rank 0's single JSON line.  emit() is called once, either at the end
    of a normal run or by the watchdog when the budget runs out (what has not
    finished is reported as "timeout"); it then kills every child."""

    def __init__(self, args, d: Dist, ex: bk.Exchange, budget: bk.Budget):
        self.args, self.d, self.ex, self.budget = args, d, ex, budget
        self.lock = threading.Lock()
        self.emitted = False
        self.label = ""
        self.wl = None
        self.variants: dict = {}
        self.pending: list = []
        self.rc = 0

    def start_watchdog(self):
        def run():
            while self.budget.left() > 0:
                time.sleep(min(1.0, max(0.05, self.budget.left())))
            if self.d.rank == 0:
                self.emit(watchdog=True)
            bk.CHILDREN.kill_all()
            sys.stdout.flush()
            os._exit(self.rc if self.d.rank == 0 else 0)

        threading.Thread(target=run, daemon=True, name="bench-watchdog").start()

    def emit(self, watchdog: bool = False):
        with self.lock:
            if self.emitted:
                return
            self.emitted = True
            try:
                line, failures = summarize(self, watchdog)
            except Exception as e:  # the line must come out whatever happened
                line, failures = {"metric": metric_name(self.args), "value": 0.0, "unit": "predictions/s",
                                  "n_gpus": self.d.world, "steps": self.args.steps, "warmup": self.args.warmup,
                                  "error": f"report failed: {type(e).__name__}: {e}"}, ["report"]
            print(json.dumps(line), flush=True)
            if failures:
                print("bench.py: FAILED: " + "; ".join(failures), file=sys.stderr, flush=True)
                self.rc = 3


def metric_name(args) -> str:
    return "predictions/sec (%s graph, %s)" % ("single-model" if args.graph == "single" else args.graph,
                                               args.api.upper())


def summarize(rep: Reporter, watchdog: bool):
    args, d, ex = rep.args, rep.d, rep.ex
    failures = []
    heads = {r: ex.get("headline", r) for r in range(d.world)}
    missing = [r for r, h in heads.items() if h is None]
    mines = [h for h in heads.values() if h is not None]
    if missing:
        failures.append(f"no headline result from ranks {missing}")
    for m in mines:
        if not m["check"]["ok"]:
            failures.append(f"rank {m['rank']} headline self-check: {m['check']}")
    base = REST_BASELINE if args.api == "rest" else GRPC_BASELINE
    line = {"metric": metric_name(args), "value": 0.0, "unit": "predictions/s", "n_gpus": d.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp64"}
    if mines:
        # whole-job throughput: every rank's completed predictions over the
        # slowest rank's timed window
        wall_max = max(m["wall"] for m in mines)
        value = sum(m["ok"] for m in mines) / wall_max if not missing else 0.0
        line.update(value=round(value, 2), ms_per_step=round(wall_max / args.steps * 1000.0, 3),
                    vs_baseline=round(value / base, 3), timed_region_s=round(wall_max, 3),
                    p50_ms=round(max(m["p50"] for m in mines), 4), p99_ms=round(max(m["p99"] for m in mines), 4),
                    step_ms=bk.step_spread([s for m in mines for s in m["step_ms"]]))
    wl = rep.wl
    line["data"] = ("synthetic (locust-shaped JSON payload, iris feature row); model fit on sklearn's bundled iris"
                    if args.model in ("iris", "python-iris", "python-noop") else
                    f"synthetic (locust-shaped JSON payload, {len(wl.row) if wl else '?'}-feature random row); "
                    "random-init model")
    line["baseline"] = {"rest_rps": REST_BASELINE, "rest_p50_ms": 4, "rest_p99_ms": 69, "grpc_rps": GRPC_BASELINE,
                        "grpc_p50_ms": 1, "grpc_p99_ms": 6}
    if mines:
        line["self_check"] = {"ok": all(m["check"]["ok"] for m in mines) and not missing,
                              "max_abs_err": max(m["check"]["max_abs_err"] for m in mines),
                              "sampled_replies_checked": sum(m.get("checked", 0) for m in mines)}
    st0 = mines[0]["stats"] if mines else {"batches": 0, "rows": 0, "gpu_busy_s": 0.0}
    wall0 = mines[0]["wall"] if mines else 1.0
    per_rank = [{"rank": m["rank"], "device": m["device"], "cpu_budget": m["cpu_budget"],
                 "pinned_cpus": m.get("pinned_cpus"), **m["cpu"], "step_requests": m["step_requests"],
                 "rps": round(m["ok"] / m["wall"], 1), "p50_ms": m["p50"], "p99_ms": m["p99"],
                 "step_ms": bk.step_spread(m["step_ms"]),
                 "gpu_batches": m["stats"]["batches"],
                 "mean_rows_per_batch": round(m["stats"]["rows"] / max(1, m["stats"]["batches"]), 2),
                 # share of the window the GPU device thread spent launching / handing off responses
                 "device_thread_launch_frac": round(m["stats"]["launch_cpu_s"] / m["wall"], 3),
                 "device_thread_complete_frac": round(m["stats"]["complete_cpu_s"] / m["wall"], 3),
                 "check_max_abs_err": m["check"]["max_abs_err"]} for m in mines]
    line["config"] = {"model": rep.label, "global_batch": args.users * d.world, "seq_len": len(wl.row) if wl else 0,
                      "parallelism": f"dp{d.world}", "graph": args.graph, "api": args.api,
                      "users_per_gpu": args.users,
                      "requests_per_step_per_gpu": mines[0]["step_requests"] if mines else args.step_requests,
                      "device": "gpu" if d.has_gpu else "cpu", "gpu_batches": st0["batches"],
                      "mean_rows_per_gpu_batch": round(st0["rows"] / max(1, st0["batches"]), 2),
                      "gpu_busy_frac_per_slot": round(st0["gpu_busy_s"] / max(1e-9, wall0 * args.slots), 3),
                      "slots": args.slots, "server_threads": args.server_threads,
                      "client_threads": args.client_threads, "host_cpus": os.cpu_count(),
                      "cpu_budget": round(bk.cpu_budget(), 2), "per_rank": per_rank}
    # ---- extras
    if args.extras == "auto" and args.graph == "single":
        gr = {r: ex.get("grpc", r) for r in range(d.world)}
        errs = [g["error"] for g in gr.values() if g and "error" in g]
        if errs:
            line["grpc"] = {"error": errs[0]}
        elif all(g is not None for g in gr.values()):
            gs = list(gr.values())
            gw = max(g["wall"] for g in gs)
            v = sum(g["ok"] for g in gs) / gw
            line["grpc"] = {"value": round(v, 2), "vs_baseline": round(v / GRPC_BASELINE, 3),
                            "p50_ms": max(g["p50"] for g in gs), "p99_ms": max(g["p99"] for g in gs),
                            "window_s": round(gw, 3), "step_ms": bk.step_spread([s for g in gs for s in g["step_ms"]])}
        else:
            line["grpc"] = {"error": "timeout" if watchdog else "missing"}
    variants = dict(rep.variants)
    for k in rep.pending:
        variants.setdefault(k, {"error": "timeout" if watchdog else "not run"})
    for k, v in variants.items():
        if "error" not in v and not v.get("self_check", {}).get("ok", True):
            failures.append(f"{k} self-check: {v['self_check']}")
    if variants:
        line["variants"] = variants
    line["budget"] = {"budget_s": BUDGET_S, "used_s": round(time.time() - T_START, 1), "watchdog_fired": watchdog}
    return line, failures


# ---------------------------------------------------------------- headline
def step_size(rate: float, steps: int, target_s: float) -> int:
    """Requests per step so `steps` steps at `rate` req/s last `target_s`
    (each step >= 0.2 s)."""
    per_step = max(0.2, target_s / max(1, steps))
    return int(min(50_000_000, max(2000, rate * per_step)))


def calibrate(args, d: Dist, port: int, body, budget: bk.Budget) -> int:
    """Step size so the K timed steps last >= TARGET_TIMED_S on the slowest
    rank.  A one-step probe of a few thousand requests reads about half the
    steady rate (connection set-up, cold batcher: VERDICT r3 weak #3), so the
    rate comes from a second probe sized to last >= PROBE_S at the first
    probe's rate; min rate over ranks (one collective, before the timed
    region).  headline() re-sizes once more from the warmup steps."""
    r = bk.probe_rate(port, args.api, body, args.users, args.client_threads,
                      lambda: budget.timeout(cap=120, reserve=HEAD_RESERVE_S), min_s=PROBE_S)
    return step_size(min(d.gather(r)), args.steps, TARGET_TIMED_S)


def headline(args, d: Dist, rep: Reporter, budget: bk.Budget, per_rank_cpus: float, pinned) -> tuple:
    import seldon_core_amd as sca

    wl = bk.Workload(args.model, args.py_batching, args.py_workers)
    rep.wl = wl
    ngpu = sca.gpu_count() if d.has_gpu else 0
    if args.graph == "single":
        devs = [d.device]
    else:
        span = SPAN.get(args.graph, max(2, d.world))
        devs = [(d.device + i) % ngpu for i in range(span)] if ngpu else [-1] * span
    lg_cores = int(os.environ.get("SCA_BENCH_LG_CORES", "0") or 0)
    if lg_cores > 0 and pinned and len(pinned) % 2 == 0 and 2 * lg_cores < len(pinned):
        # placement A/B: the load generator on the last `lg_cores` cores (both
        # SMT threads), the server's threads -- created below -- on the rest
        # of the rank's CCD.  pinned = [cores..., their siblings...]
        half = len(pinned) // 2
        cores, sibs = pinned[:half], pinned[half:]
        lg = cores[half - lg_cores:] + sibs[half - lg_cores:]
        os.environ["SCA_LOADGEN_CPUS"] = ",".join(map(str, lg))
        os.sched_setaffinity(0, [c for c in pinned if c not in lg])
    dep, oracle, label = bk.make_deployment(wl, args.graph, devs, d.device, args.slots, not args.no_spin)
    if args.graph != "single":
        if not wl.impl:
            raise SystemExit("multi-node --graph variants use the kernel models (iris / xgb1000)")
        label = f"{label} [{wl.label}]"
    rep.label = label
    handle = dep.serve(http_port=0, grpc_port=0, threads=args.server_threads, host="127.0.0.1")
    body_rest = wl.rest_body()
    pb = dep.C.json_to_pb(json.dumps({"data": {"names": wl.names,
                                               "tensor": {"shape": [1, len(wl.row)], "values": wl.row}}}))
    expect_rest = bk.rest_expect(handle.http_port, body_rest)
    expect_pb = bk.pb_data_suffix(dep.predict_pb(pb)[1])
    if args.api == "rest":
        body, port, expect = body_rest, handle.http_port, expect_rest
    else:
        body, port, expect = pb, handle.grpc_port, expect_pb
    calibrated = args.step_requests is None
    if calibrated:
        args.step_requests = calibrate(args, d, port, body, budget)
    if args.warmup > 0:  # untimed
        wu = bk.run_loadgen(port, args.warmup, 0, args.api, body, args.users, args.client_threads,
                            args.step_requests, budget.timeout(reserve=HEAD_RESERVE_S), expect=expect)
        if calibrated:  # the warmup steps are the longest steady-state probe there is: grow, never shrink
            warm = d.gather(float(wu["rps"]))
            args.step_requests = max(args.step_requests, step_size(min(warm), args.steps, TARGET_TIMED_S))
    for u in dep.batched.values():
        u.reset_stats()
    cpu: dict = {}
    if args.cpu_profile:
        from seldon_core_amd.utils import cpuprof

        cpuprof.start(depth=args.cpu_profile_depth)
    tmo = budget.timeout(reserve=HEAD_RESERVE_S)
    d.barrier()
    d.sync()
    c0 = cpu_seconds()
    t0 = time.perf_counter()
    err = None
    try:
        lg = bk.run_loadgen(port, args.steps, 0, args.api, body, args.users, args.client_threads, args.step_requests,
                            tmo, expect=expect)
    except Exception as e:  # still meet the closing barrier, or the other ranks would wait forever
        lg, err = None, e
    d.sync()
    wall = time.perf_counter() - t0
    c1 = cpu_seconds()
    cpu["server_cpus"] = round((c1[0] - c0[0]) / wall, 2)
    cpu["loadgen_cpus"] = round((c1[1] - c0[1]) / wall, 2)
    d.barrier()
    if err is not None:
        raise err
    if args.cpu_profile:
        prof = cpuprof.stop()
        prof.update(rps=round(lg["ok"] / wall, 1), server_cpus=cpu.get("server_cpus"), rank=d.rank)
        with open(args.cpu_profile if d.world == 1 else f"{args.cpu_profile}.rank{d.rank}", "w") as f:
            json.dump(prof, f, indent=1)
    st = bk.unit_stats(dep)
    chk = bk.self_check(handle.http_port, wl, oracle, seed=d.rank)
    mine = {"rank": d.rank, "device": d.device, "ok": lg["ok"], "wall": wall, "p50": lg["p50_ms"],
            "p99": lg["p99_ms"], "step_ms": lg["step_ms"], "checked": lg.get("checked", 0), "stats": st,
            "cpu_budget": round(per_rank_cpus, 2), "cpu": cpu, "step_requests": args.step_requests,
            "pinned_cpus": bk.cpu_ranges(pinned) if pinned else None, "check": chk}
    rep.ex.put("headline", mine)
    return dep, handle, pb, expect_pb, lg


def grpc_extra(args, d: Dist, rep: Reporter, budget: bk.Budget, handle, pb, expect_pb, head_lg) -> None:
    """gRPC API (seldon.protos.Seldon/Predict, Tensor payload) on every rank,
    started together (soft file barrier), window >= EXTRA_WINDOW_S."""
    try:
        fault("grpc", d.rank)
        rep.ex.barrier("grpc_go", timeout=budget.timeout(cap=60, reserve=EXTRA_RESERVE_S))
        rate = bk.probe_rate(handle.grpc_port, "grpc", pb, args.users, args.client_threads,
                             lambda: budget.timeout(cap=60, reserve=EXTRA_RESERVE_S), min_s=PROBE_S)
        sreq = bk.window_requests(rate, EXTRA_WINDOW_S)
        t0 = time.perf_counter()
        g = bk.run_loadgen(handle.grpc_port, 2, 1, "grpc", pb, args.users, args.client_threads, sreq,
                           budget.timeout(cap=120, reserve=EXTRA_RESERVE_S), expect=expect_pb)
        res = {"ok": g["ok"], "wall": g["seconds"], "p50": g["p50_ms"], "p99": g["p99_ms"],
               "step_ms": g["step_ms"], "call_s": round(time.perf_counter() - t0, 2)}
    except Exception as e:  # reported; the headline stands
        res = {"error": f"{type(e).__name__}: {e}"[:600]}
    rep.ex.put("grpc", res)


# ---------------------------------------------------------------- variants
def variant_cmd(args, kind: str, span: int, deadline: float, extra=()):
    return [sys.executable, os.path.abspath(__file__), "--model", args.model, "--slots", str(args.slots),
            "--users", str(args.users), "--variant-child", kind, "--span", str(span), "--deadline", str(deadline),
            *extra]


def run_inprocess_variants(args, d: Dist, rep: Reporter, budget: bk.Budget, kinds) -> None:
    """Rank 0: each multi-GPU graph as ONE deployment over the node's GPUs,
    in a child process (a fault or hang there is recorded, not fatal) with
    its own deadline; results go into the line as soon as they exist."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK")
           and not k.startswith("TORCHELASTIC_")}
    env["SCA_BENCH_AFFINITY"] = bk.cpu_ranges(ORIG_AFFINITY) if ORIG_AFFINITY else ""
    reserve = REPORT_RESERVE_S + (FABRIC_RESERVE_S if args.rank_variants else 0.0)
    for kind in kinds:
        span = SPAN.get(kind, d.world)
        try:
            tmo = budget.timeout(cap=VARIANT_CAP_S, reserve=reserve, floor=10.0)
        except bk.BudgetExpired as e:
            rep.variants[kind] = {"error": f"skipped: {e}"}
            continue
        res = bk.CHILDREN.run(variant_cmd(args, kind, span, time.time() + tmo), tmo + 5, env=env)
        out = bk.last_json(res["stdout"])
        if res["timed_out"]:
            out = {"error": "timeout", "after_s": round(tmo, 1), "stderr_tail": res["stderr"][-600:]}
        elif out is None or res["rc"] != 0:
            out = dict(out or {}, error=(out or {}).get("error") or f"variant child rc={res['rc']}",
                       stderr_tail=res["stderr"][-600:])
        out["child_wall_s"] = res["wall_s"]
        rep.variants[kind] = out
        if kind in rep.pending:
            rep.pending.remove(kind)


def variant_child(args) -> None:
    """One in-process variant: build it on GPUs 0..span-1, serve, calibrate,
    time a >= EXTRA_WINDOW_S window (mab: with concurrent feedback that
    rewards the last branch), self-check, report placement; one JSON line."""
    budget = bk.Budget(args.deadline)
    aff = os.environ.get("SCA_BENCH_AFFINITY")
    if aff:  # the parent rank was pinned to one CCD; one process now drives every GPU
        from seldon_core_amd.utils.topology import _parse_cpulist

        try:
            os.sched_setaffinity(0, _parse_cpulist(aff))
        except OSError:
            pass
    kind = args.variant_child
    if kind == "reuseport":
        print(json.dumps(reuseport_child(args, budget)), flush=True)
        return
    out = {"error": "unfinished"}
    dep = h = None
    try:
        fault(kind, 0)
        import seldon_core_amd as sca

        ngpu = sca.gpu_count()
        devs = list(range(args.span)) if ngpu > 0 else [-1] * args.span
        if ngpu and args.span > ngpu:
            if not (os.environ.get("SCA_BENCH_FOLD") or os.environ.get("SCA_BENCH_FOLD_GPUS")):
                raise RuntimeError(f"{kind} needs {args.span} GPUs, {ngpu} visible")
            devs = [i % ngpu for i in devs]  # rehearsal on a smaller box: nodes fold onto the GPUs present
        cpus = bk.cpu_budget()
        server_threads = max(2, min(32, int(cpus * 0.55)))
        client_threads = max(1, min(16, int(cpus * 0.3)))
        wl = bk.Workload(args.model)
        dep, oracle, label = bk.make_deployment(wl, kind, devs, devs[0], args.slots, spin=False)
        h = dep.serve(http_port=0, grpc_port=0, threads=server_threads, host="127.0.0.1")
        body = wl.rest_body()
        expect = bk.rest_expect(h.http_port, body)
        rate = bk.probe_rate(h.http_port, "rest", body, args.users, client_threads,
                             lambda: budget.timeout(reserve=3), min_s=PROBE_S, expect=expect)
        sreq = bk.window_requests(rate, EXTRA_WINDOW_S)
        for u in dep.batched.values():
            u.reset_stats()
        fb_out, fb = {}, None
        n = len(devs)
        if kind == "mab":
            # feedback next to the predictions (reference MAB loadtest sends
            # feedback: util/loadtester/scripts/predict_rest_locust.py); the
            # last branch (the farthest GPU) is rewarded, so the bandit must
            # learn to send most traffic there.
            fbody = json.dumps({"request": {"data": {"names": wl.names, "ndarray": [wl.row]}},
                                "response": {"meta": {"routing": {"mab": n - 1}}, "data": {"ndarray": [[0.0]]}},
                                "reward": 1.0})

            def feedback():
                try:
                    fb_out.update(bk.run_loadgen(h.http_port, 2, 0, "rest", fbody, max(4, args.users // 16),
                                                 max(1, client_threads // 4), max(200, sreq // 16),
                                                 budget.timeout(reserve=3), path="/api/v0.1/feedback"))
                except Exception as e:
                    fb_out["error"] = f"{type(e).__name__}: {e}"[:300]

            fb = threading.Thread(target=feedback)
            fb.start()
        lg = bk.run_loadgen(h.http_port, 2, 0, "rest", body, args.users, client_threads, sreq,
                            budget.timeout(reserve=3), expect=expect)
        if fb is not None:
            fb.join()
        check = bk.self_check(h.http_port, wl, oracle, seed=100)
        st = bk.unit_stats(dep)
        pl = bk.placement(dep)
        used = sorted({x for v in pl.values() if isinstance(v, list) for x in v})
        out = {"graph": label, "model": wl.label, "gpus_per_graph": len(set(devs)), "value": round(lg["rps"], 2),
               "unit": "predictions/s", "vs_rest_baseline": round(lg["rps"] / REST_BASELINE, 3),
               "p50_ms": lg["p50_ms"], "p99_ms": lg["p99_ms"], "window_s": round(lg["seconds"], 3),
               "step_ms": bk.step_spread(lg["step_ms"]), "sampled_replies_checked": lg.get("checked", 0),
               "self_check": check, "placement": pl, "peer_access": bk.peer_access(used),
               "device_graphs": bk.device_graphs(dep),
               "batches_per_device": {k: v["batches"] for k, v in st["per_device"].items()},
               "rows_per_device": {k: v["rows"] for k, v in st["per_device"].items()},
               "server_threads": server_threads, "client_threads": client_threads, "cpu_budget": cpus}
        if kind == "mab":
            out["feedback"] = {"rewarded_branch": n - 1, "rps": fb_out.get("rps"), "error": fb_out.get("error")}
    except Exception as e:
        out = {"error": f"{type(e).__name__}: {e}"[:600]}
    finally:
        try:
            if h is not None:
                h.stop()
            if dep is not None:
                dep.close()
        except Exception:
            pass
    print(json.dumps(out), flush=True)


def _tail(path: str, n: int) -> list:
    try:
        with open(path, errors="replace") as f:
            return [ln.rstrip()[:300] for ln in f.readlines()[-n:]]
    except OSError:
        return []


def reuseport_child(args, budget: bk.Budget) -> dict:
    """The production multi-worker path: ``serve --gpus
    N`` -- the Supervisor's N worker processes, one per GPU, all bound to ONE
    port with SO_REUSEPORT (the reference's replicas behind one Service,
    seldondeployment_controller.go:296-302) -- driven by one load generator
    with N x users connections.  Reports the whole-endpoint rate and each
    worker's share of the requests (the kernel's connection balancing)."""
    import signal

    n = args.span
    work = tempfile.mkdtemp(prefix="sca_reuseport_")
    proc = None
    try:
        with open(os.path.join(work, "bench_iris.py"), "w") as f:
            f.write("from seldon_core_amd.models import iris_logistic_regression\n"
                    "from seldon_core_amd.servers import SKLearnServer\n\n\n"
                    "class Iris(SKLearnServer):\n"
                    "    def __init__(self):\n"
                    "        super().__init__(model=iris_logistic_regression())\n")
        spec = {"name": "reuseport", "componentSpecs": [{"spec": {"containers": []}}],
                "graph": {"name": "classifier", "type": "MODEL", "children": []}}
        with open(os.path.join(work, "spec.json"), "w") as f:
            json.dump(spec, f)
        stats = os.path.join(work, "stats")
        os.makedirs(stats)
        port = _free_port()
        cpus = bk.cpu_budget()
        threads = max(2, int(cpus * 0.5 / n))
        env = {k: v for k, v in os.environ.items() if not k.startswith(("TORCHELASTIC_", "RANK", "LOCAL_RANK",
                                                                       "WORLD_SIZE", "LOCAL_WORLD_SIZE"))}
        env.update(PYTHONPATH=os.pathsep.join([ROOT, work]), SCA_WORKER_STATS_DIR=stats)
        cmd = [sys.executable, "-m", "seldon_core_amd.serve", "--spec", os.path.join(work, "spec.json"),
               "--gpus", str(n), "--http-port", str(port), "--grpc-port", str(_free_port()), "--admin-port", "0",
               "--threads", str(threads), "--component", "classifier=bench_iris.Iris", "--log-level", "INFO"]
        import torch

        if torch.cuda.device_count() < n:  # (counting does not initialise the GPU on this stack)
            cmd += ["--device", "-1"]
        log = open(os.path.join(work, "serve.log"), "w")
        proc = subprocess.Popen(cmd, env=env, cwd=work, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        deadline = time.time() + min(90.0, budget.left(10))
        while time.time() < deadline:
            with open(os.path.join(work, "serve.log")) as f:
                if f.read().count("serving reuseport") >= n:
                    break
            if proc.poll() is not None:
                raise RuntimeError(f"serve --gpus {n} exited rc={proc.returncode}")
            time.sleep(0.2)
        else:
            raise TimeoutError(f"{n} workers not up")
        wl = bk.Workload("iris")
        body = wl.rest_body()
        expect = bk.rest_expect(port, body)
        users = args.users * n
        cthreads = max(1, min(32, int(cpus * 0.3)))
        rate = bk.probe_rate(port, "rest", body, users, cthreads, lambda: budget.timeout(reserve=10), min_s=PROBE_S,
                             expect=expect)
        lg = bk.run_loadgen(port, 2, 0, "rest", body, users, cthreads, bk.window_requests(rate, EXTRA_WINDOW_S),
                            budget.timeout(reserve=10), expect=expect)
        # drain: SIGTERM to the supervisor ONLY -- it forwards one SIGTERM to
        # each worker (every worker files its request count) and SIGKILLs
        # stragglers itself; a killpg would hand every worker a second signal
        proc.send_signal(signal.SIGTERM)
        drain_timeout = None
        t_stop = time.time()
        try:
            proc.wait(timeout=max(5.0, min(40.0, budget.left(5))))
        except subprocess.TimeoutExpired:  # the window is measured: report it, note the slow exit
            drain_timeout = {"error": "serve supervisor still running after SIGTERM (killed)",
                             "serve_log_tail": _tail(os.path.join(work, "serve.log"), 40)}
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
        stop_s = round(time.time() - t_stop, 3)
        per = []
        for fn in sorted(os.listdir(stats)):
            with open(os.path.join(stats, fn)) as f:
                per.append(json.load(f))
        counts = [w["requests"] for w in per]
        return {"graph": f"single-model x {n} workers (serve --gpus {n}, SO_REUSEPORT)", "workers": n,
                "value": round(lg["rps"], 2), "unit": "predictions/s", "vs_rest_baseline": round(lg["rps"] / REST_BASELINE, 3),
                "p50_ms": lg["p50_ms"], "p99_ms": lg["p99_ms"], "window_s": round(lg["seconds"], 3),
                "users": users, "sampled_replies_checked": lg.get("checked", 0),
                "self_check": {"ok": lg.get("bad_body", 0) == 0},
                "per_worker_requests": {str(w["rank"]): w["requests"] for w in per},
                "balance_min_over_max": round(min(counts) / max(1, max(counts)), 3) if counts else None,
                "server_threads_per_worker": threads, "client_threads": cthreads, "shutdown_s": stop_s,
                **({"drain_timeout": drain_timeout} if drain_timeout else {}),
                **({"missing_worker_stats": sorted(set(map(str, range(n))) - {str(w["rank"]) for w in per}),
                    "serve_log_tail": _tail(os.path.join(work, "serve.log"), 40)} if len(per) < n else {})}
    except Exception as e:
        return {"error": f"{type(e).__name__}: {e}"[:600]}
    finally:
        if proc is not None and proc.poll() is None:
            import signal as _s

            try:
                os.killpg(proc.pid, _s.SIGKILL)
            except OSError:
                pass
            proc.wait()
        shutil.rmtree(work, ignore_errors=True)


# ------------------------------------------------------------------ fabric
def run_fabric_phase(args, d: Dist, rep: Reporter, budget: bk.Budget, kinds) -> None:
    """Every rank: start a fabric child (fresh gloo group on a port rank 0
    publishes through the exchange); rank 0's child serves the rank-placed
    graphs, the others run PeerServer loops.  Each rank files its child's
    result; rank 0 merges them into the line."""
    ex = rep.ex
    if d.rank == 0:
        try:
            tmo = budget.timeout(reserve=REPORT_RESERVE_S, floor=20.0)
            ex.put("fabric_go", {"port": _free_port(), "deadline": time.time() + tmo})
        except bk.BudgetExpired as e:
            ex.put("fabric_go", {"skip": str(e)})
    go = ex.wait("fabric_go", [0], timeout=max(0.0, budget.left(REPORT_RESERVE_S))).get(0)
    if not go or "skip" in go:
        if d.rank == 0:
            for k in kinds:
                rep.variants[f"{k}_ranks"] = {"error": (go or {}).get("skip", "not run")}
                if f"{k}_ranks" in rep.pending:
                    rep.pending.remove(f"{k}_ranks")
        return
    deadline = float(go["deadline"])
    cmd = [sys.executable, os.path.abspath(__file__), "--model", args.model, "--slots", str(args.slots),
           "--users", str(args.users), "--fabric-child", ",".join(kinds), "--deadline", str(deadline),
           "--server-threads", str(args.server_threads), "--client-threads", str(args.client_threads)]
    res = bk.CHILDREN.run(cmd, max(1.0, deadline - time.time()) + 3, env=child_env(d, int(go["port"]), deadline))
    out = {"graphs": {}}
    for ln in res["stdout"].splitlines():  # one line per finished graph, then a summary
        if ln.startswith("{"):
            try:
                o = json.loads(ln)
            except ValueError:
                continue
            if "kind" in o:
                out["graphs"][o["kind"]] = o["result"]
            else:
                out.update({k: v for k, v in o.items() if k != "graphs"})
    status = "timeout" if res["timed_out"] else ("ok" if res["rc"] == 0 else f"rc={res['rc']}")
    mine = {"rank": d.rank, "status": status, "wall_s": res["wall_s"], "result": out}
    if status != "ok":
        mine["stderr_tail"] = res["stderr"][-600:]
    ex.put("fabric", mine)
    if d.rank != 0:
        return
    peers = ex.wait("fabric", list(range(1, d.world)), timeout=max(0.0, budget.left(REPORT_RESERVE_S)))
    for k in kinds:
        key = f"{k}_ranks"
        r0 = out["graphs"].get(k)
        if r0 is None:
            r0 = {"error": "timeout" if status == "timeout" else f"fabric child {status}: no result",
                  "stderr_tail": res["stderr"][-400:]}
        r0 = dict(r0)
        r0["data_plane"] = out.get("data_plane") or ("ipc" if d.has_gpu else "shm")
        r0["fabric_world"] = d.world
        r0["worker_ranks"] = {str(r): ((p.get("result") or {}).get("graphs") or {}).get(k, {"status": p["status"]})
                              for r, p in sorted(peers.items())}
        missing = [r for r in range(1, d.world) if r not in peers]
        if missing:
            r0["workers_missing"] = missing
        rep.variants[key] = r0
        if key in rep.pending:
            rep.pending.remove(key)


def fabric_child(args) -> None:
    """Rank-placed graphs.  Rank 0 hosts the front end,
    routers and the program units; the nodes placed on rank r run on rank r's
    GPU (mesh programs over HIP IPC + shared memory by default, shared memory
    alone on CPU; SCA_FABRIC_TRANSPORT=rccl|rccl1 for the RCCL star).  Every
    rank walks the same graph list in the same order, with a fresh fabric per
    graph."""
    import datetime

    import torch
    import torch.distributed as dist

    budget = bk.Budget(args.deadline)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) if torch.cuda.is_available() else -1
    if dev >= 0 and os.environ.get("SCA_BENCH_FOLD_GPUS") == "1":
        dev = 0  # rehearsal: every rank process on GPU 0 (the ipc mesh runs between them)
    if dev >= 0:
        torch.cuda.set_device(dev)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(10.0, budget.left())))
    from seldon_core_amd.parallel.fabric import init_fabric, serve_peer
    from seldon_core_amd.serving.deployment import Deployment

    wl = bk.Workload(args.model)
    graphs = {}
    transport = None
    for kind in [k for k in args.fabric_child.split(",") if k]:
        if (kind == "pipeline" and world < 4) or world < 2:
            continue
        g, comps, oracle, label = bk.build_rank_graph(wl, kind, world)
        spec = bk.sdep(g)
        fabric = init_fabric(device=dev)  # one per graph: a mesh is set up once
        transport = fabric.transport
        if rank != 0:
            t0 = time.perf_counter()
            try:
                fault(f"{kind}_ranks", rank)
                srv = serve_peer(spec, fabric, comps)
                srv.join()
                graphs[kind] = {"batches": srv.batches, "rows": srv.rows, "host_syncs": srv.host_syncs,
                                "max_inflight": getattr(srv, "max_inflight", None), "error": srv.error(),
                                "device": dev, "transport": transport, "wall_s": round(time.perf_counter() - t0, 2)}
            except Exception as e:
                graphs[kind] = {"error": f"{type(e).__name__}: {e}"[:400]}
            fabric.close()
            print(json.dumps({"kind": kind, "result": graphs[kind]}), flush=True)
            continue
        dep = h = None
        try:
            fault(f"{kind}_ranks", 0)
            dep = Deployment(spec, components=comps, device=dev, fabric=fabric, fuse=False,
                             batcher={"max_batch": 4096, "slots": args.slots, "spin_wait": False})
            h = dep.serve(http_port=0, grpc_port=0, threads=args.server_threads, host="127.0.0.1")
            body = wl.rest_body()
            expect = bk.rest_expect(h.http_port, body)
            rate = bk.probe_rate(h.http_port, "rest", body, args.users, args.client_threads,
                                 lambda: budget.timeout(reserve=5), min_s=PROBE_S, expect=expect)
            sreq = bk.window_requests(rate, EXTRA_WINDOW_S)
            for u in dep.batched.values():
                u.reset_stats()
            fb_out, fb = {}, None
            if kind == "mab":  # reward the last rank's replica: most batches must cross the fabric
                fbody = json.dumps({"request": {"data": {"names": wl.names, "ndarray": [wl.row]}},
                                    "response": {"meta": {"routing": {"mab": world - 1}},
                                                 "data": {"ndarray": [[0.0]]}}, "reward": 1.0})

                def feedback():
                    try:
                        fb_out.update(bk.run_loadgen(h.http_port, 2, 0, "rest", fbody, max(4, args.users // 16),
                                                     max(1, args.client_threads // 4), max(200, sreq // 16),
                                                     budget.timeout(reserve=5), path="/api/v0.1/feedback"))
                    except Exception as e:
                        fb_out["error"] = f"{type(e).__name__}: {e}"[:300]

                fb = threading.Thread(target=feedback)
                fb.start()
            lg = bk.run_loadgen(h.http_port, 2, 0, "rest", body, args.users, args.client_threads, sreq,
                                budget.timeout(reserve=5), expect=expect)
            if fb is not None:
                fb.join()
            check = bk.self_check(h.http_port, wl, oracle, seed=200)
            st = bk.unit_stats(dep)
            r = {"graph": label, "value": round(lg["rps"], 2), "unit": "predictions/s",
                 "p50_ms": lg["p50_ms"], "p99_ms": lg["p99_ms"], "window_s": round(lg["seconds"], 3),
                 "step_ms": bk.step_spread(lg["step_ms"]), "sampled_replies_checked": lg.get("checked", 0),
                 "self_check": check, "placement": bk.placement(dep),
                 "unit_kinds": {n: dep.engine.unit_kind(n) for n in dep.engine.node_names()},
                 "rank0_batches_per_unit": {k: v.get("batches", 0) for k, v in dep.batcher_stats().items()
                                            if isinstance(v, dict)},
                 "rank0_device_batches": {k: v["batches"] for k, v in st["per_device"].items()}}
            if kind == "mab":
                r["feedback"] = {"rewarded_branch": world - 1, "rps": fb_out.get("rps"), "error": fb_out.get("error")}
            if dep.mesh is not None:
                r["mesh_programs"] = [{"root": p.root, "stages": p.describe(), "messages_per_batch": m,
                                       "edges": (dep.mesh.edges[i] if i < len(dep.mesh.edges) else [])}
                                      for i, (p, m) in enumerate(zip(dep.mesh.programs, dep.mesh.messages))]
                r["peer"] = dep.mesh.peer  # GPUs, hipDeviceCanAccessPeer, IPC canary per edge
            r["transport"] = transport
            graphs[kind] = r
        except Exception as e:
            graphs[kind] = {"error": f"{type(e).__name__}: {e}"[:600]}
        finally:
            try:
                if h is not None:
                    h.stop()
                if dep is not None:
                    dep.close()  # stops the peers' loops for this graph
                else:
                    fabric.stop_peers()  # keep the workers in step with the graph list
                fabric.close()
            except Exception:
                pass
        print(json.dumps({"kind": kind, "result": graphs[kind]}), flush=True)
    print(json.dumps({"rank": rank, "world": world, "device": dev, "data_plane": transport}), flush=True)
    sys.stdout.flush()
    os._exit(0)  # no teardown collective: a peer that failed must not hold this child


# -------------------------------------------------------------------- main
def main() -> None:
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.variant_child:
        variant_child(args)
        return
    if args.fabric_child:
        fabric_child(args)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        sys.exit(2)

    deadline = float(os.environ.get("SCA_BENCH_DEADLINE", T_START + BUDGET_S))
    budget = bk.Budget(deadline)
    d = Dist(budget)
    rep = Reporter(args, d, None, budget)
    rep.start_watchdog()
    ex_dir = d.bcast(tempfile.mkdtemp(prefix="sca_bench_") if d.rank == 0 else None)
    rep.ex = ex = bk.Exchange(ex_dir, d.rank, d.world)
    per_rank_budget, pinned = place_rank(args, d)
    per_rank_cpus = size_threads(args, per_rank_budget)
    extras = args.extras == "auto" and args.graph == "single"
    inproc, rccl = [], []
    if extras and d.world >= 2 and args.model in ("iris", "xgb1000"):  # same lists on every rank
        inproc = [k for k in args.variants.split(",") if k and (k != "pipeline" or d.world >= 4)]
        rccl = [k for k in args.rank_variants.split(",") if k and (k != "pipeline" or d.world >= 4)]
    rep.pending = inproc + [f"{k}_ranks" for k in rccl]
    dep = handle = None
    try:
        dep, handle, pb, expect_pb, head_lg = headline(args, d, rep, budget, per_rank_cpus, pinned)
        if extras:
            grpc_extra(args, d, rep, budget, handle, pb, expect_pb, head_lg)
    except Exception as e:
        rep.ex.put("headline_error", f"rank {d.rank}: {type(e).__name__}: {e}"[:600])
        if d.rank == 0:
            print(f"bench.py: rank 0 headline failed: {e}", file=sys.stderr, flush=True)
    finally:
        if handle is not None:
            handle.stop()
        if dep is not None:
            dep.close()
    if inproc or rccl:
        ex.put("idle", True)
        if d.rank == 0 and inproc:
            # others' gRPC windows must be over before rank 0 drives every GPU
            ex.wait("idle", list(range(d.world)), timeout=max(0.0, min(60.0, budget.left(REPORT_RESERVE_S))))
            run_inprocess_variants(args, d, rep, budget, inproc)
        if rccl:
            run_fabric_phase(args, d, rep, budget, rccl)
    if d.rank != 0:
        ex.put("done", True)
        sys.stdout.flush()
        os._exit(0)
    rep.emit()
    shutil.rmtree(ex_dir, ignore_errors=True)
    sys.stdout.flush()
    if os.environ.get("SCA_BENCH_CLEAN_EXIT") == "1":
        sys.exit(rep.rc)  # a normal exit lets a profiler's exit hooks write its trace (rocprofv3)
    os._exit(rep.rc)


if __name__ == "__main__":
    main()
