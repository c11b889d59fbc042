"""Engine entry point and one-process-per-GPU replica supervisor.

    python -m seldon_core_amd.serve --spec sdep.json [--predictor NAME] \
        [--http-port 8000] [--grpc-port 5001] [--admin-port 8082] [--threads 4] \
        [--gpus 1|N|all] [--component node=module.Class ...] [--no-fuse]

Replaces the reference's engine container (``engine/.../App.java``: boot, serve
REST + gRPC, drain on shutdown) and the slice of the operator that keeps
``replicas`` copies of it running (``operator/controllers/
seldondeployment_controller.go:296-302,548-636``: Deployment replicas, rolling
restarts, ``terminationGracePeriodSeconds`` 20, preStop ``/pause``).

``--gpus N`` (N > 1) starts N worker processes, one per MI355X, each seeing
only its own GPU (``HIP_VISIBLE_DEVICES``).  All workers bind the same REST and
gRPC ports with ``SO_REUSEPORT``, so the kernel spreads connections across
them -- the in-host equivalent of a Service over N pods, with no proxy hop.
The supervisor never touches a GPU itself; it restarts a worker that dies
(bounded restart rate) and, on SIGTERM/SIGINT, forwards SIGTERM so every
worker drains: readiness off, wait for in-flight requests, stop.

SIGHUP is a rolling update (the Deployment's RollingUpdate strategy,
``seldondeployment_controller.go:565``, exercised upstream by
``testing/scripts/test_rolling_updates.py``): worker by worker, a new worker
is started from the current ``--spec`` file next to the old one (same GPU,
same ports through ``SO_REUSEPORT``), and only once it reports ready is the
old one drained -- one extra worker at a time, never fewer than N serving.
A new worker that fails to come up stops the rollout and the old one stays.

Rank-placed graphs: a spec whose nodes carry ``rank: r`` (the GPU / process
hosting that node, see ``seldon_core_amd.parallel.fabric``) runs as ONE graph
over ``--gpus N`` processes instead of N copies: the supervisor starts the N
rank processes as a gang (RANK / WORLD_SIZE / MASTER_* like torchrun, every
GPU visible), rank 0 serves the REST/gRPC front end and the graph, and ranks
1..N-1 run ``serve_peer`` -- placed subtrees run there as mesh programs (HIP
IPC + shared memory, or shared memory alone on CPU gangs; RCCL with
``SCA_FABRIC_TRANSPORT=rccl``).  ``--device D`` puts every rank on GPU D; by
default each rank gets its own GPU when there are enough, else the gang runs
on the CPU.  A rank that dies takes the gang down and the supervisor
restarts all of it (the communicators cannot be re-joined); SIGHUP restarts
the gang from the current spec.

Shared router state: with N replica workers, stateful routers (epsilon-greedy,
Thompson) keep their counters in one host-wide shared mapping
(``SCA_SHARED_STATE``), so feedback that SO_REUSEPORT hands to any worker
trains the one bandit every worker routes with -- the reference's single
router object per deployment (``EpsilonGreedy.py:87-130``).

Configuration precedence: defaults < ``/etc/podinfo/annotations`` < spec
annotations < environment (``ENGINE_SERVER_PORT``, ``SELDON_LOG_*``, ...) < flags.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

from .utils.shutdown import StopSignal

logger = logging.getLogger("seldon_core_amd.serve")


def parse_args(argv: Optional[List[str]] = None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="seldon-amd-engine")
    ap.add_argument("--spec", default=None, help="SeldonDeployment / PredictorSpec JSON or YAML (default: "
                                                  "ENGINE_PREDICTOR env, ./deploymentdef.json, SIMPLE_MODEL graph)")
    ap.add_argument("--predictor", default=None)
    ap.add_argument("--http-port", type=int, default=None)
    ap.add_argument("--grpc-port", type=int, default=None)
    ap.add_argument("--admin-port", type=int, default=None)
    ap.add_argument("--host", default=None)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--gpus", default="1", help="worker processes, one per GPU: N or 'all'")
    ap.add_argument("--device", type=int, default=None, help="GPU for a single worker (-1 = CPU)")
    ap.add_argument("--component", action="append", default=[], help="node=module.Class binding")
    ap.add_argument("--no-fuse", action="store_true", help="disable device-graph fusion")
    ap.add_argument("--max-restarts", type=int, default=5, help="per worker per minute")
    ap.add_argument("--log-level", default=os.environ.get("SELDON_LOG_LEVEL", "INFO"))
    ap.add_argument("--explainer-port", type=int, default=None,
                    help="port of the predictor's explainer (default: explainer.endpoint.service_port or 9000)")
    ap.add_argument("--persistence", nargs="?", default=0, const=1, type=int,
                    help="checkpoint stateful nodes (routers, detectors) and restore them at start "
                         "(SELDON_PERSISTENCE_BACKEND=file|redis)")
    ap.add_argument("--push-frequency", type=float, default=None, help="seconds between checkpoints (default 60)")
    ap.add_argument("--pin-cpus", type=int, default=0,
                    help="pin each worker to whole CCDs of its GPU's socket covering this many CPUs (0 = off)")
    ap.add_argument("--supervise", action="store_true",
                    help="run even a single worker under the supervisor (SIGHUP rolling updates, restarts)")
    ap.add_argument("--kill-after", type=float, default=30.0,
                    help="supervisor: SIGKILL workers still running this many seconds after the forwarded "
                         "SIGTERM (their own drain is seldon.io/engine-drain-seconds, default 20)")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _gpu_total() -> int:
    try:
        import torch

        return int(torch.cuda.device_count())  # does not initialise the GPU on this stack
    except Exception:
        return 0


def _n_workers(arg: str) -> int:
    if str(arg).lower() == "all":
        return max(1, _gpu_total())
    return max(1, int(arg))


def _placed_world(spec_path: Optional[str], predictor: Optional[str]) -> int:
    """1 + the highest ``rank:`` of the served predictor's graph (0 = no
    rank placement)."""
    from .parallel.fabric import rank_assignments
    from .serving.spec import load_spec, select_predictor

    try:
        pred = select_predictor(load_spec(spec_path), predictor)
    except Exception:  # the worker reports spec errors
        return 0
    ranks = rank_assignments(pred.get("graph") or {})
    return (max(ranks) + 1) if ranks and max(ranks) > 0 else 0


def run_fabric_worker(args: argparse.Namespace) -> int:
    """One rank of a rank-placed graph (see the module doc)."""
    import datetime

    import torch.distributed as dist

    from .parallel.fabric import gang_device, init_fabric, serve_peer
    from .serving.spec import load_spec

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    # one placement for the whole gang (never GPU and CPU ranks mixed):
    # --device D puts every rank on GPU D (ranks share it over the ipc mesh)
    device = gang_device(rank, world, args.device)
    fabric = init_fabric(device=device)
    if rank == 0:
        return run_worker(args, fabric=fabric)
    comps = {}
    for c in args.component:
        node, _, cls = c.partition("=")
        comps[node] = cls
    # SIGTERM: rank 0 drains first and then stops this loop; leave on our own
    # only if it never does.  The handler only flips a flag (utils/shutdown.py).
    stop_requested = StopSignal().install()
    _stack_dumps()
    srv = serve_peer(load_spec(args.spec), fabric, comps, predictor=args.predictor)
    logger.info("rank %d/%d serving its placed nodes on device %s (%s)", rank, world, device, fabric.transport)
    joiner = threading.Thread(target=srv.join, daemon=True)
    joiner.start()
    while joiner.is_alive():
        joiner.join(0.2)
        if stop_requested.is_set():
            deadline = time.monotonic() + 60.0
            while joiner.is_alive() and time.monotonic() < deadline:
                joiner.join(0.2)
            break
    err = srv.error()
    fabric.close()
    if err:
        logger.error("rank %d peer loop ended: %s", rank, err)
    logger.info("rank %d done: %d batches, %d rows, max in flight %d", rank, srv.batches, srv.rows,
                srv.max_inflight)
    os._exit(0 if not err or stop_requested.is_set() else 1)


# ------------------------------------------------------------------ worker
def _stack_dumps() -> None:
    """SIGUSR1 dumps every thread's Python stack to stderr (hang triage in
    production: ``kill -USR1 <worker pid>``)."""
    import faulthandler

    try:
        faulthandler.register(signal.SIGUSR1, all_threads=True, chain=False)
    except (AttributeError, ValueError, RuntimeError):
        pass


def run_worker(args: argparse.Namespace, fabric=None) -> int:
    # installed first: a SIGTERM during start-up becomes a drain as soon as
    # the servers are up instead of the default action killing the process
    stop = StopSignal().install()
    _stack_dumps()
    if args.pin_cpus > 0 and (args.device is None or args.device >= 0):
        # before the front end and the GPU units start their threads (they inherit it)
        from .utils.topology import pin

        cpus = pin(args.device or 0, args.pin_cpus)
        if cpus:
            logger.info("worker pinned to CPUs %s", cpus)
    from .serving.config import EngineConfig
    from .serving.deployment import Deployment
    from .serving.spec import load_spec, predictors

    sdep = load_spec(args.spec)
    spec_ann: Dict[str, str] = dict(((sdep.get("spec") or {}).get("annotations") or {}))
    for p in predictors(sdep):
        spec_ann.update(p.get("annotations") or {})
    cfg = EngineConfig.resolve(spec_annotations=spec_ann, http_port=args.http_port, grpc_port=args.grpc_port,
                               admin_port=args.admin_port, host=args.host, threads=args.threads)
    comps = {}
    for c in args.component:
        node, _, cls = c.partition("=")
        comps[node] = cls
    device = args.device if fabric is None else int(fabric.device)
    dep = Deployment(sdep, components=comps, predictor=args.predictor, deployment_name=cfg.deployment_name,
                     device=device, fuse=False if (args.no_fuse or fabric is not None) else None, config=cfg,
                     fabric=fabric)
    if args.persistence:
        dep.restore_checkpoint()
        dep.start_checkpointing(args.push_frequency)
    h = dep.serve(http_port=cfg.http_port, grpc_port=cfg.grpc_port, admin_port=cfg.admin_port,
                  threads=cfg.threads, grpc_threads=cfg.grpc_threads, host=cfg.host)
    rank = os.environ.get("SCA_WORKER_RANK", "0")
    ready_file = os.environ.get("SCA_READY_FILE")
    if ready_file:  # the supervisor's rolling update waits for this before draining the old worker
        with open(ready_file, "w") as f:
            f.write(str(os.getpid()))
    logger.info("worker %s serving %s: REST :%s gRPC :%s admin :%s (device %s, units %s)", rank,
                dep.predictor.get("name"), h.http_port, h.grpc_port, cfg.admin_port, dep.device,
                {n: dep.engine.unit_kind(n) for n in dep.engine.node_names()})
    explainer = None
    if rank == "0" and (dep.predictor.get("explainer") or {}).get("type"):
        # The reference runs the explainer as its own Deployment pointed at the
        # predictor (seldondeployment_explainers.go:32-184); here it shares the
        # worker process and labels perturbation batches through the engine.
        from .explainers.server import deployment_predictor, from_spec

        model_name = (sdep.get("metadata") or {}).get("name") or cfg.deployment_name
        explainer = from_spec(dep.predictor, deployment_predictor(dep), model_name, cfg.host, args.explainer_port)
        explainer.start()
        logger.info("explainer %s on :%d", dep.predictor["explainer"]["type"], explainer.port)
    def on_hup(signum, frame):  # noqa: ARG001
        # SIGHUP's default action would kill the only serving process: a
        # rolling update needs a supervisor to start the replacement first.
        if not os.environ.get("SCA_WORKER_RANK"):
            logger.warning("SIGHUP ignored: rolling updates need the supervisor (--supervise or --gpus > 1)")

    signal.signal(signal.SIGHUP, on_hup)
    stop.wait()
    if explainer is not None:
        explainer.stop()
    clean = h.drain(cfg.drain_seconds)
    stats_dir = os.environ.get("SCA_WORKER_STATS_DIR")
    if stats_dir:  # per-worker share of the traffic SO_REUSEPORT handed out (bench reuseport variant)
        served = 0.0
        for ln in dep.metrics().splitlines():
            if ln.startswith("seldon_api_engine_server_requests") and "_count" in ln.split(" ")[0]:
                served += float(ln.rsplit(" ", 1)[-1])
        with open(os.path.join(stats_dir, f"worker-{rank}.json"), "w") as f:
            json.dump({"rank": int(rank), "pid": os.getpid(), "requests": int(served),
                       "units": {k: v.get("requests", 0) for k, v in dep.batcher_stats().items()
                                 if isinstance(v, dict)}}, f)
    dep.engine.flush_message_log()
    dep.close()  # rank-placed graph: also stops the other ranks' peer loops
    if fabric is not None:
        fabric.close()
    logger.info("worker %s drained (%s)", rank, "clean" if clean else "timeout")
    return 0


# -------------------------------------------------------------- supervisor
class Supervisor:
    """Keeps one worker process per GPU alive."""

    def __init__(self, n: int, worker_argv: List[str], max_restarts: int = 5, ready_timeout: float = 120.0,
                 drain_timeout: float = 60.0, gang: bool = False, kill_after: float = 30.0):
        self.n = n
        self.gang = gang  # rank-placed graph: the N processes are ranks of ONE graph
        self.master_port = 0
        self.shared_prefix = f"/sca_state_{os.getpid()}"
        self.argv = worker_argv
        self.max_restarts = max_restarts
        self.ready_timeout = ready_timeout
        self.drain_timeout = drain_timeout
        self.procs: Dict[int, subprocess.Popen] = {}
        self.restarts: Dict[int, List[float]] = {i: [] for i in range(n)}
        self.stopping = False
        self.roll_requested = False
        self.generation = 0
        self.rollouts: List[Dict] = []
        self._surge: Optional[subprocess.Popen] = None  # the rollout's new worker before it is swapped in
        self.stop_signal = StopSignal()
        self.kill_after = kill_after       # SIGKILL workers this long after the forwarded SIGTERM
        self._forwarded_at: Optional[float] = None
        self._killed = False
        self.killed_pids: List[int] = []

    def _start(self, rank: int, ready_file: Optional[str] = None) -> subprocess.Popen:
        env = dict(os.environ)
        if self.gang:  # torchrun-style rank environment; every GPU visible (peer links between them)
            env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(self.n), LOCAL_WORLD_SIZE=str(self.n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.master_port), SCA_FABRIC_WORLD=str(self.n))
        else:
            env["HIP_VISIBLE_DEVICES"] = str(rank)
            env["SCA_SHARED_STATE"] = self.shared_prefix
        env["SCA_WORKER_RANK"] = str(rank)
        env["SCA_WORKERS"] = str(self.n)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if ready_file:
            env["SCA_READY_FILE"] = ready_file
        else:
            env.pop("SCA_READY_FILE", None)
        p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--worker", *self.argv], env=env)
        logger.info("started worker %d (pid %d) on GPU %d", rank, p.pid, rank)
        return p

    def spawn(self, rank: int) -> None:
        self.procs[rank] = self._start(rank)

    def spawn_gang(self) -> None:
        """(Re)start every rank of a rank-placed graph on a fresh rendezvous port."""
        import socket

        for p in self.procs.values():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in self.procs.values():
            try:
                p.wait(timeout=self.drain_timeout)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            self.master_port = sk.getsockname()[1]
        for r in range(self.n):
            self.spawn(r)

    def cleanup_shared(self) -> None:
        """Remove the shared router-state mappings the workers created."""
        base = "/dev/shm"
        tag = self.shared_prefix.lstrip("/") + "_"
        try:
            names = os.listdir(base)
        except OSError:
            return
        for n in names:
            if n.startswith(tag):
                try:
                    os.unlink(os.path.join(base, n))
                except OSError:
                    pass

    def rolling_update(self) -> bool:
        """Replace every worker, one at a time, surge 1: start the new one,
        wait for its ready marker, then drain the old one.  Returns False (and
        keeps the old worker) if a new worker does not come up.  A rank-placed
        gang cannot run two generations side by side: it restarts whole."""
        import tempfile

        if self.gang:
            self.generation += 1
            logger.warning("rollout %d: rank-placed graph restarts as a gang", self.generation)
            self.spawn_gang()
            self.rollouts.append({"generation": self.generation, "replaced": list(range(self.n)), "ok": True,
                                  "gang": True})
            return True

        self.generation += 1
        record = {"generation": self.generation, "replaced": [], "ok": True}
        with tempfile.TemporaryDirectory(prefix="sca-rollout-") as tmp:
            for rank in range(self.n):
                if self.stopping:
                    record["ok"] = False
                    break
                ready = os.path.join(tmp, f"worker-{rank}.ready")
                new = self._start(rank, ready)
                self._surge = new  # terminate() must reach it too
                deadline = time.monotonic() + self.ready_timeout
                while (not os.path.exists(ready) and new.poll() is None and time.monotonic() < deadline
                       and not self.stopping):
                    time.sleep(0.05)
                if self.stopping:  # SIGTERM arrived mid-rollout: stop the new worker, keep nothing half-done
                    self._stop_proc(new)
                    self._surge = None
                    record["ok"] = False
                    break
                if not os.path.exists(ready):
                    logger.error("rollout %d: new worker %d did not become ready; keeping the old one",
                                 self.generation, rank)
                    self._stop_proc(new)
                    self._surge = None
                    record["ok"] = False
                    break
                old = self.procs[rank]
                self.procs[rank] = new  # from here on the new one is the supervised worker
                self._surge = None
                if old.poll() is None:
                    old.send_signal(signal.SIGTERM)  # drain: readiness off, in-flight requests finish
                    try:
                        old.wait(timeout=self.drain_timeout)
                    except subprocess.TimeoutExpired:
                        old.kill()
                        old.wait()
                record["replaced"].append({"rank": rank, "old_pid": old.pid, "new_pid": new.pid})
                logger.info("rollout %d: worker %d replaced (pid %d -> %d)", self.generation, rank, old.pid, new.pid)
        self.rollouts.append(record)
        return record["ok"]

    def status(self) -> Dict:
        return {"workers": {r: {"pid": p.pid, "alive": p.poll() is None, "restarts": len(self.restarts[r])}
                            for r, p in self.procs.items()}}

    def _stop_proc(self, p: subprocess.Popen) -> None:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
            try:
                p.wait(timeout=self.drain_timeout)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def request_stop(self, signum=None, frame=None) -> None:  # noqa: ARG002
        """Signal handler: flips flags only (no lock, no Popen call -- see
        utils/shutdown.py); the main loop forwards and escalates."""
        self.stop_signal.handler(signum or 0)
        self.stopping = True

    def _children(self) -> List[subprocess.Popen]:
        return list(self.procs.values()) + ([self._surge] if self._surge is not None else [])

    def terminate(self) -> None:
        """Main-loop side, idempotent: forward ONE SIGTERM to every worker
        (they drain: readiness off, in-flight requests finish), then
        :meth:`_escalate` SIGKILLs whatever is still alive ``kill_after``
        seconds later -- the reference's forced stop after its 20 s drain
        (``App.java:89-92``)."""
        self.stopping = True
        if self._forwarded_at is not None:
            return
        self._forwarded_at = time.monotonic()
        for p in self._children():
            if p.poll() is None:
                try:
                    p.send_signal(signal.SIGTERM)
                except OSError:
                    pass

    def _escalate(self) -> None:
        if self._forwarded_at is None or self._killed:
            return
        if time.monotonic() - self._forwarded_at < self.kill_after:
            return
        self._killed = True
        for p in self._children():
            if p.poll() is None:
                logger.error("worker pid %d still running %.0f s after SIGTERM: SIGKILL", p.pid, self.kill_after)
                self.killed_pids.append(p.pid)
                try:
                    p.kill()
                except OSError:
                    pass

    def run(self) -> int:
        try:
            return self._run()
        finally:
            self.cleanup_shared()

    def _run(self) -> int:
        if self.gang:
            self.spawn_gang()
        else:
            for r in range(self.n):
                self.spawn(r)
        signal.signal(signal.SIGTERM, self.request_stop)
        signal.signal(signal.SIGINT, self.request_stop)
        signal.signal(signal.SIGHUP, lambda *_: setattr(self, "roll_requested", True))
        return self._loop()

    def _loop(self) -> int:
        rc = 0
        while True:
            self.stop_signal.wait(0.2)
            if self.stopping:
                self.terminate()
                self._escalate()
            if self.roll_requested and not self.stopping:
                self.roll_requested = False
                self.rolling_update()
            alive = 0
            for r, p in list(self.procs.items()):
                code = p.poll()
                if code is None:
                    alive += 1
                    continue
                if self.stopping:
                    continue
                now = time.monotonic()
                self.restarts[r] = [t for t in self.restarts[r] if now - t < 60.0]
                if len(self.restarts[r]) >= self.max_restarts:
                    logger.error("worker %d exited with %s and hit the restart limit; shutting down", r, code)
                    rc = code or 1
                    self.terminate()
                    continue
                self.restarts[r].append(now)
                if self.gang:
                    logger.warning("rank %d exited with %s; restarting the gang", r, code)
                    self.spawn_gang()
                    alive = self.n
                    break
                logger.warning("worker %d exited with %s; restarting", r, code)
                self.spawn(r)
                alive += 1
            if self.stopping and alive == 0:
                return rc


def main(argv: Optional[List[str]] = None) -> int:
    args = parse_args(argv)
    logging.basicConfig(level=getattr(logging, str(args.log_level).upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    if args.worker:
        if os.environ.get("SCA_FABRIC_WORLD"):
            return run_fabric_worker(args)
        return run_worker(args)
    n = _n_workers(args.gpus)
    placed = _placed_world(args.spec, args.predictor)
    if placed > n:
        logger.error("the graph places nodes on %d ranks but --gpus is %d", placed, n)
        return 2
    if n == 1 and not args.supervise:
        return run_worker(args)
    raw = list(sys.argv[1:] if argv is None else argv)
    worker_argv: List[str] = []
    skip = False
    for i, a in enumerate(raw):  # drop --gpus from the workers' command line
        if skip:
            skip = False
            continue
        if a == "--gpus":
            skip = True
            continue
        if a.startswith("--gpus="):
            continue
        worker_argv.append(a)
    return Supervisor(n, worker_argv, args.max_restarts, gang=placed > 0, kill_after=args.kill_after).run()


if __name__ == "__main__":
    sys.exit(main())
