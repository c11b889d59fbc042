"""Building blocks of the serving benchmark (``bench.py``).

The reference measures its engine with locust users against a deployed graph
(``util/loadtester/scripts/predict_rest_locust.py``,
``doc/source/reference/benchmarking.md:31-64``).  Here the same measurement is
one closed-loop native load generator (``sca_loadgen``) against the native
front end, plus the pieces ``bench.py`` needs to run it robustly on a node of
8 MI355X GPUs:

* :class:`Budget` -- one wall-clock deadline for the whole run; every child
  process and load-generator call gets a timeout taken from what is left;
* :class:`Exchange` -- rank results as files in a shared directory, so the
  report never waits in a collective on a rank that hung;
* :class:`Children` -- every child process in its own process group, killed
  as a group on timeout or when the watchdog fires;
* the workloads, graph builders (one process driving N GPUs, or nodes placed
  on worker ranks behind the fabric), the load generator wrapper with a sampled
  reply-body check, the CPU-oracle self check and placement reports.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import threading
import time
import urllib.request
from typing import Any, Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LOADGEN = os.path.join(ROOT, "seldon_core_amd", "bin", "sca_loadgen")


class BudgetExpired(RuntimeError):
    pass


# ------------------------------------------------------------------ budget
class Budget:
    """Absolute deadline (epoch seconds) shared by a rank and its children."""

    def __init__(self, deadline: float):
        self.deadline = float(deadline)

    def left(self, reserve: float = 0.0) -> float:
        return self.deadline - time.time() - reserve

    def timeout(self, cap: Optional[float] = None, reserve: float = 0.0, floor: float = 1.0) -> float:
        """Seconds a step may take: what is left minus `reserve`, at most
        `cap`.  Raises BudgetExpired when less than `floor` is left."""
        t = self.left(reserve)
        if cap is not None:
            t = min(t, cap)
        if t < floor:
            raise BudgetExpired(f"benchmark budget spent ({self.left():.0f}s left, {reserve:.0f}s reserved)")
        return t


# ---------------------------------------------------------------- exchange
class Exchange:
    """Per-rank result files in a directory all ranks of one node can see.
    Writes are atomic (temp file + rename); readers poll."""

    def __init__(self, path: str, rank: int, world: int):
        self.path, self.rank, self.world = path, rank, world

    def _file(self, name: str, rank: int) -> str:
        return os.path.join(self.path, f"{name}.{rank}.json")

    def put(self, name: str, obj: Any, rank: Optional[int] = None) -> None:
        f = self._file(name, self.rank if rank is None else rank)
        tmp = f + f".tmp{os.getpid()}"
        with open(tmp, "w") as fh:
            json.dump(obj, fh)
        os.replace(tmp, f)

    def get(self, name: str, rank: int) -> Any:
        try:
            with open(self._file(name, rank)) as fh:
                return json.load(fh)
        except (OSError, ValueError):
            return None

    def wait(self, name: str, ranks: List[int], timeout: float, poll: float = 0.05) -> Dict[int, Any]:
        """{rank: obj} for the ranks whose `name` appeared within `timeout`."""
        end = time.time() + max(0.0, timeout)
        out: Dict[int, Any] = {}
        while True:
            for r in ranks:
                if r not in out:
                    v = self.get(name, r)
                    if v is not None:
                        out[r] = v
            if len(out) == len(ranks) or time.time() >= end:
                return out
            time.sleep(poll)

    def barrier(self, name: str, timeout: float) -> bool:
        """Soft barrier: announce, then wait (bounded) for every rank."""
        self.put(name, True)
        return len(self.wait(name, list(range(self.world)), timeout)) == self.world


# ---------------------------------------------------------------- children
class Children:
    """Child processes, each in its own session (process group), so a
    timeout or the watchdog can kill a child together with everything it
    started (load generators, RCCL worker threads)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._procs: List[subprocess.Popen] = []

    def popen(self, cmd, **kw) -> subprocess.Popen:
        p = subprocess.Popen(cmd, start_new_session=True, **kw)
        with self._lock:
            self._procs.append(p)
        return p

    def forget(self, p: subprocess.Popen) -> None:
        with self._lock:
            if p in self._procs:
                self._procs.remove(p)

    @staticmethod
    def kill(p: subprocess.Popen) -> None:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass

    def kill_all(self) -> None:
        with self._lock:
            procs = list(self._procs)
        for p in procs:
            if p.poll() is None:
                self.kill(p)

    def run(self, cmd, timeout: float, env=None) -> Dict[str, Any]:
        """Run to completion or kill at `timeout`:
        {"rc", "stdout", "stderr", "timed_out", "wall_s"}."""
        t0 = time.time()
        p = self.popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        timed_out = False
        try:
            out, err = p.communicate(timeout=max(0.5, timeout))
        except subprocess.TimeoutExpired:
            timed_out = True
            self.kill(p)
            out, err = p.communicate()
        finally:
            self.forget(p)
        return {"rc": p.returncode, "stdout": out or "", "stderr": err or "", "timed_out": timed_out,
                "wall_s": round(time.time() - t0, 2)}


CHILDREN = Children()


def last_json(text: str) -> Optional[Dict]:
    for line in reversed((text or "").splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


# ------------------------------------------------------------------ CPUs
def cpu_budget() -> float:
    """CPUs this process may use: the smaller of the cgroup v2 quota
    (cpu.max) and the CPU affinity mask."""
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


# --------------------------------------------------------------- workloads
class Workload:
    """The benchmark model: component, payload row, names and a CPU oracle."""

    def __init__(self, model: str, py_batching: int = 4096, py_workers: int = 0):
        from ..servers import SKLearnServer, XGBoostServer

        self.model = model
        self.py_batching, self.py_workers = py_batching, py_workers
        if model == "iris":
            from ..models import iris_logistic_regression

            self.clf = iris_logistic_regression()
            self.comp = SKLearnServer(model=self.clf)
            self.names = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
            self.row = [5.1, 3.5, 1.4, 0.2]
            self.label = "sklearn-iris-LogisticRegression (linear_softmax HIP kernel, fp64)"
            self.impl = "SKLEARN_SERVER"
        elif model in ("python-iris", "python-noop"):
            from ..components.examples import EchoModel, IrisClassifier

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
        elif model == "xgb1000":
            from ..models import synthetic_xgboost

            self.ens = synthetic_xgboost(1000, 8, 32, seed=0)
            self.comp = XGBoostServer(ensemble=self.ens)
            self.names = [f"f{i}" for i in range(32)]
            self.row = [0.1 * ((i * 7) % 13 - 6) for i in range(32)]
            self.label = "xgboost-1000trees-depth8 regressor (tree_perfect HIP kernel, random-init)"
            self.impl = "XGBOOST_SERVER"
        else:
            raise ValueError(model)

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

    def tol(self, ref) -> float:
        import numpy as np

        return 1e-4 * max(1.0, float(np.abs(ref).max())) if self.model == "xgb1000" else 1e-9

    def rest_body(self) -> str:
        return json.dumps({"data": {"names": self.names, "ndarray": [self.row]}})

    def row_model(self):
        from ..models import to_row_model

        return self.comp.row_model() if hasattr(self.comp, "row_model") else to_row_model(self.comp)


def _scaler(C, width: int):
    """A standard-scaler-style affine TRANSFORMER (diag weights) and its scale."""
    import numpy as np

    scale = 1.0 + 0.01 * np.random.default_rng(0).random(width)
    return C.linear_model(np.diag(scale), np.zeros(width), 0), scale


def build_graph(wl: Workload, kind: str, devs: List[int], reward_branch: Optional[int] = None):
    """(graph, components, oracle, label) of one benchmark graph served by one
    process, node ``i`` of the graph on GPU ``devs[i]``:

    * ``single``   -- one MODEL node (the headline);
    * ``abtest``   -- RANDOM_ABTEST router over 2 replicas on 2 GPUs (BASELINE config 3);
    * ``pipeline`` -- TRANSFORMER -> AVERAGE_COMBINER over 2 models, one stage per GPU of 4
      (BASELINE config 4), fused into a device graph;
    * ``mab``      -- epsilon-greedy router over one replica per GPU (BASELINE config 5);
    * ``replicas`` -- one MODEL node served by a replica per GPU behind one endpoint
      (the reference's Deployment replicas behind a Service,
      ``operator/controllers/seldondeployment_controller.go:296-302``).
    """
    import numpy as np

    from .._native import native

    if kind == "single":
        g = {"name": "classifier", "type": "MODEL", "children": [], "device": devs[0]}
        if wl.impl:
            g.update(implementation=wl.impl, modelUri="memory://bench")
            label = wl.label
        else:  # a user Python class
            g.update(batching=wl.py_batching, workers=wl.py_workers)
            label = wl.label + f" [batching={wl.py_batching}, workers={wl.py_workers}]"
        return g, {"classifier": wl.comp}, wl.oracle, label
    C = native()
    rm = wl.row_model()
    if kind == "replicas":
        g = {"name": "classifier", "type": "MODEL", "devices": list(devs)}
        return g, {"classifier": rm}, wl.oracle, f"one endpoint over {len(devs)} GPU replicas {devs} (JSQ)"
    if kind == "abtest":
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST", "device": devs[0],
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "device": devs[0]},
                          {"name": "b", "type": "MODEL", "device": devs[1]}]}
        return g, {"a": rm, "b": rm.clone()}, wl.oracle, f"RANDOM_ABTEST(2 replicas on GPUs {devs[:2]})"
    if kind == "pipeline":
        tr, scale = _scaler(C, len(wl.row))
        g = {"name": "scaler", "type": "TRANSFORMER", "device": devs[0], "children": [
            {"name": "combiner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "device": devs[3],
             "children": [{"name": "a", "type": "MODEL", "device": devs[1]},
                          {"name": "b", "type": "MODEL", "device": devs[2]}]}]}
        return (g, {"scaler": tr, "a": rm, "b": rm.clone()}, lambda X: wl.oracle(np.asarray(X) * scale),
                f"TRANSFORMER->COMBINER(2 models) device graph on GPUs {devs[:4]}")
    if kind == "mab":
        from ..components.routers import EpsilonGreedy

        n = len(devs)
        kids = [{"name": f"m{i}", "type": "MODEL", "device": devs[i]} for i in range(n)]
        comps = {f"m{i}": (rm if i == 0 else rm.clone()) for i in range(n)}
        comps["mab"] = EpsilonGreedy(n_branches=n, epsilon=0.1, seed=1)
        g = {"name": "mab", "type": "ROUTER", "device": devs[0], "children": kids}
        return g, comps, wl.oracle, f"EPSILON_GREEDY router over {n} replicas on GPUs {devs}"
    raise ValueError(kind)


def build_rank_graph(wl: Workload, kind: str, world: int):
    """(graph, components, oracle, label) of a graph whose nodes are placed on
    torch.distributed ranks (``rank: r`` -- one engine process per GPU, the
    nodes of other ranks reached over the fabric: mesh programs by default):

    * ``abtest``   -- router + replica a on rank 0, replica b on rank 1;
    * ``pipeline`` -- scaler on rank 3 -> combiner on rank 0 over a (rank 1), b (rank 2);
    * ``mab``      -- epsilon-greedy router on rank 0 over replica m_r on every rank r.
    """
    import numpy as np

    from .._native import native

    C = native()
    rm = wl.row_model()
    if kind == "abtest":
        g = {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
             "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
             "children": [{"name": "a", "type": "MODEL", "rank": 0}, {"name": "b", "type": "MODEL", "rank": 1}]}
        return g, {"a": rm, "b": rm.clone()}, wl.oracle, "RANDOM_ABTEST: a on rank 0, b on rank 1 (mesh)"
    if kind == "pipeline":
        tr, scale = _scaler(C, len(wl.row))
        g = {"name": "scaler", "type": "TRANSFORMER", "rank": 3, "children": [
            {"name": "combiner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
             "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}]}
        return (g, {"scaler": tr, "a": rm, "b": rm.clone()}, lambda X: wl.oracle(np.asarray(X) * scale),
                "scaler (rank 3) -> AVERAGE_COMBINER (rank 0) over a (rank 1), b (rank 2) (mesh)")
    if kind == "mab":
        from ..components.routers import EpsilonGreedy

        kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(world)]
        comps = {f"m{r}": (rm if r == 0 else rm.clone()) for r in range(world)}
        comps["mab"] = EpsilonGreedy(n_branches=world, epsilon=0.1, seed=1)
        g = {"name": "mab", "type": "ROUTER", "children": kids}
        return g, comps, wl.oracle, f"EPSILON_GREEDY router (rank 0) over replicas on ranks 0..{world - 1} (mesh)"
    raise ValueError(kind)


def sdep(graph: Dict) -> Dict:
    return {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": "bench"},
            "spec": {"name": "bench", "predictors": [{
                "name": "default", "replicas": 1, "componentSpecs": [{"spec": {"containers": []}}],
                "graph": graph}]}}


def make_deployment(wl: Workload, kind: str, devs, device: int, slots: int, spin: bool, **kw):
    from ..serving.deployment import Deployment

    graph, comps, oracle, label = build_graph(wl, kind, devs)
    dep = Deployment(sdep(graph), components=comps, device=device,
                     batcher={"max_batch": 4096, "slots": slots, "spin_wait": spin}, **kw)
    return dep, oracle, label


# ------------------------------------------------------------------- load
def pb_data_suffix(msg: bytes) -> bytes:
    """Bytes of a serialized SeldonMessage from its `data` field (3) on: the
    part of a reply that does not change between requests (meta carries the
    per-request puid and routing)."""
    i = 0
    while i < len(msg):
        start = i
        tag, i = _varint(msg, i)
        field, wire = tag >> 3, tag & 7
        if field == 3:
            return msg[start:]
        if wire == 2:
            n, i = _varint(msg, i)
            i += n
        elif wire == 0:
            _, i = _varint(msg, i)
        elif wire == 1:
            i += 8
        elif wire == 5:
            i += 4
        else:
            break
    return b""


def _varint(b: bytes, i: int):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def rest_expect(port: int, body: str, path: str = "/api/v0.1/predictions") -> str:
    """The invariant tail of a reference REST reply (from ``"data":`` on)."""
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=body.encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        text = r.read().decode()
    k = text.rfind('"data":')
    if k < 0:
        raise RuntimeError(f"reference reply has no data: {text[:200]}")
    return text[k:]


def run_loadgen(port: int, steps: int, warmup: int, api: str, body, users: int, threads: int,
                step_requests: int, timeout: float, path: str = "/api/v0.1/predictions",
                expect=None, check_every: int = 16) -> Dict[str, Any]:
    """One sca_loadgen run (killed at `timeout`); raises on failed requests
    or on sampled replies whose body differs from `expect`."""
    cmd = [LOADGEN, "--host", "127.0.0.1", "--port", str(port), "--users", str(users), "--threads", str(threads),
           "--steps", str(steps), "--warmup", str(warmup), "--step-requests", str(step_requests)]
    spin = int(os.environ.get("SCA_LOADGEN_SPIN_US", "0") or 0)
    if spin > 0:
        cmd += ["--spin-us", str(spin)]
    if os.environ.get("SCA_LOADGEN_CPUS"):  # set by bench.py's SCA_BENCH_LG_CORES placement A/B
        cmd += ["--cpus", os.environ["SCA_LOADGEN_CPUS"]]
    tmp = []
    if api == "rest":
        cmd += ["--mode", "rest", "--path", path, "--body", body]
    else:
        bpath = f"/tmp/sca_bench_req_{os.getpid()}_{threading.get_ident()}.pb"
        with open(bpath, "wb") as f:
            f.write(body)
        tmp.append(bpath)
        cmd += ["--mode", "grpc", "--path", "/seldon.protos.Seldon/Predict", "--body-file", bpath,
                "--streams-per-conn", "8"]
    if expect:
        epath = f"/tmp/sca_bench_expect_{os.getpid()}_{threading.get_ident()}"
        with open(epath, "wb") as f:
            f.write(expect if isinstance(expect, bytes) else expect.encode())
        tmp.append(epath)
        cmd += ["--expect-file", epath, "--check-every", str(check_every)]
    try:
        res = CHILDREN.run(cmd, timeout)
    finally:
        for t in tmp:
            try:
                os.unlink(t)
            except OSError:
                pass
    if res["timed_out"]:
        raise TimeoutError(f"loadgen killed after {timeout:.0f}s")
    out = last_json(res["stdout"])
    if res["rc"] not in (0, 1) or out is None:
        raise RuntimeError(f"loadgen failed rc={res['rc']}: {res['stderr'][-2000:]}")
    if out.get("bad_body"):
        raise RuntimeError(f"loadgen: {out['bad_body']} of {out['checked']} sampled replies had a wrong body")
    if out["errors"]:
        raise RuntimeError(f"loadgen saw {out['errors']} failed requests")
    return out


def probe_rate(port: int, api: str, body, users: int, threads: int, timeout_fn, min_s: float = 0.5,
               expect=None) -> float:
    """Steady-state request rate of a server: a short warm probe, then one
    step sized to last about `min_s` at the short probe's rate (a one-step
    probe of a few thousand requests reads about half the steady rate).
    `timeout_fn()` gives each loadgen call's timeout."""
    first = run_loadgen(port, 1, 1, api, body, users, threads, max(2000, users * 16), timeout_fn(), expect=expect)
    r1 = float(first["rps"])
    second = run_loadgen(port, 1, 0, api, body, users, threads, int(max(2000, r1 * min_s)), timeout_fn(),
                         expect=expect)
    return max(r1, float(second["rps"]))


def window_requests(rate: float, window_s: float, steps: int = 2) -> int:
    """Requests per step so `steps` steps at `rate` fill `window_s` (10%
    headroom: the rate is a probe's, the window a floor)."""
    return int(max(2000, 1.1 * rate * window_s / max(1, steps)))


def step_spread(step_ms: List[float]) -> Dict[str, float]:
    if not step_ms:
        return {}
    s = sorted(step_ms)
    return {"min": round(s[0], 3), "median": round(s[len(s) // 2], 3), "max": round(s[-1], 3)}


def self_check(port: int, wl: Workload, oracle, seed: int, n: int = 24) -> Dict[str, Any]:
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
    tol = wl.tol(ref)
    return {"rows": n, "max_abs_err": err, "tol": tol, "ok": bool(err <= tol)}


# -------------------------------------------------------------- placement
def unit_stats(dep) -> Dict[str, Any]:
    per_dev: Dict[str, Any] = {}
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


def placement(dep) -> Dict[str, Any]:
    """{node: [HIP devices]} of a deployment's GPU-backed nodes (replicated
    nodes list every replica's device; fused device graphs list each stage's)."""
    from ..serving.spec import iter_nodes

    out: Dict[str, Any] = {}
    for node, _ in iter_nodes(dep.predictor["graph"]):
        name = node["name"]
        if node.get("rank") is not None and dep.fabric is not None:
            out[name] = {"rank": int(node["rank"])}
            continue
        out[name] = dep.replica_devices(node) if (node.get("devices") or node.get("replicas")) \
            else [dep._node_device(node)]
    return out


def device_graphs(dep) -> Dict[str, Any]:
    """Per fused device graph: devices, peer-direct or staged edges, the
    start-up peer canaries and whether it runs as one fused kernel."""
    out: Dict[str, Any] = {}
    C = dep.C
    for name, unit in getattr(dep, "batched", {}).items():
        try:
            info = dict(C.graph_info(unit.model))
        except Exception:  # noqa: BLE001  not a graph model
            continue
        out[name] = {k: info[k] for k in ("devices", "peer_direct", "peer_canary", "fused", "stages") if k in info}
    return out


def peer_access(devs) -> Dict[str, bool]:
    """hipDeviceCanAccessPeer between every ordered pair of distinct GPUs used."""
    from .._native import gpu_count, native

    ds = sorted({int(d) for d in devs if d is not None and int(d) >= 0})
    if gpu_count() <= 0 or len(ds) < 2:
        return {}
    C = native()
    return {f"{a}->{b}": bool(C.can_access_peer(a, b)) for a in ds for b in ds if a != b}
