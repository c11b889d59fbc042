"""In-process deployment of a SeldonDeployment inference graph.

This replaces the reference's control plane + data plane hop chain
(operator reconcile -> engine pod -> one microservice pod per node)
with one process: the spec is validated with the operator webhook's rules,
every graph node is bound to an implementation (built-in, prepackaged server,
GPU row model behind a micro-batcher, or Python component), the native graph
is compiled once, and the native REST/gRPC front ends serve it.

Node binding order:
1. explicit ``components={"node": obj}`` argument (object, class, "module.Class"
   string, RowModel, model spec),
2. built-in implementations (SIMPLE_MODEL, SIMPLE_ROUTER, RANDOM_ABTEST,
   AVERAGE_COMBINER) -- executed natively,
3. prepackaged servers (SKLEARN_SERVER, XGBOOST_SERVER, MLFLOW_SERVER,
   TENSORFLOW_SERVER) -- loaded from ``modelUri``,
4. engine-native component implementations (EPSILON_GREEDY, THOMPSON_SAMPLING,
   MAHALANOBIS_OD, ISOLATION_FOREST_OD, VAE_OD, SEQ2SEQ_OD, ...),
5. the node's container: ``MODEL_NAME`` / ``SELDON_PYTHON_CLASS`` env var, or a
   ``python_class`` parameter, naming a Python component class.
"""
from __future__ import annotations

import importlib
import json
import logging
import pickle
import os
from typing import Any, Dict, Optional, Union

from .._native import gpu_count, native
from .adapter import PythonUnit
from .errors import EngineError
from ..parallel.device_graph import fusion_enabled
from .spec import (BUILTIN_IMPLEMENTATIONS, PREPACKAGED_SERVERS, SpecError, container_for, header_route, is_shadow,
                   iter_nodes, load_spec, predictors, select_predictor, typed_parameters, validate)

logger = logging.getLogger(__name__)

METHOD_IDS = {"TRANSFORM_INPUT": 0, "TRANSFORM_OUTPUT": 1, "ROUTE": 2, "AGGREGATE": 3, "SEND_FEEDBACK": 4,
              "PREDICT": 5}
BATCHER_KEYS = ("max_batch", "max_wait_us", "slots", "zero_copy", "zero_copy_max_bytes", "spin_wait", "cpu_batching",
                "fail_threshold", "cooldown_ms", "hang_timeout_ms")


def import_class(path: str):
    mod, _, cls = path.replace(":", ".").rpartition(".")
    if not mod:
        mod, cls = cls, cls  # reference convention: module and class share a name
    return getattr(importlib.import_module(mod), cls)


class Deployment:
    def __init__(self, spec: Union[str, Dict, None] = None, components: Optional[Dict[str, Any]] = None,
                 predictor: Optional[str] = None, deployment_name: Optional[str] = None,
                 device: Optional[int] = None, batcher: Optional[Dict[str, Any]] = None,
                 log_requests: bool = False, log_responses: bool = False, fuse: Optional[bool] = None,
                 config=None, fabric=None, _metrics_from=None):
        self.C = native()
        self.fabric = fabric
        self.sdep = load_spec(spec)
        all_preds = predictors(self.sdep)
        split = predictor is None and len(all_preds) > 1
        if split:
            # Traffic split across predictors: the first live predictor hosts the
            # front end; the others are sibling engines sharing its metrics.
            errs = [e for e in validate(self.sdep, bound=set(components or {})) if "Traffic" in e]
            if errs:
                raise SpecError(errs)
            live = [p for p in all_preds if not is_shadow(p)]
            if not live:
                raise SpecError(["SeldonDeployment has only shadow predictors"])
            predictor = live[0]["name"]
        self.predictor = select_predictor(self.sdep, predictor)
        self.components = dict(components or {})
        pname = self.predictor.get("name", "")
        for k in list(self.components):  # "predictor/node" keys target one predictor
            if "/" in k:
                p, _, n = k.partition("/")
                obj = self.components.pop(k)
                if p == pname:
                    self.components[n] = obj
        self.deployment_name = deployment_name or os.environ.get("DEPLOYMENT_NAME", "None")
        if device is None:
            device = 0 if gpu_count() > 0 else -1
        self.device = device
        self.batcher_defaults = dict(max_batch=1024, max_wait_us=0, slots=4, zero_copy=True,
                                     zero_copy_max_bytes=256 << 10, spin_wait=True)
        self.batcher_defaults.update(batcher or {})
        errs = validate({"spec": {"predictors": [self.predictor]}}, bound=set(self.components))
        errs = [e for e in errs if "Traffic" not in e]
        if errs:
            raise SpecError(errs)
        self.config = config
        ekw = config.engine_kwargs() if config is not None else dict(log_requests=log_requests,
                                                                     log_responses=log_responses)
        self.engine = self.C.Engine(json.dumps(self.predictor), self.deployment_name, "",
                                    share_metrics_with=_metrics_from, **ekw)
        self.units: Dict[str, Any] = {}
        self.python_units: Dict[str, PythonUnit] = {}
        self.batched: Dict[str, Any] = {}
        self.native_units: Dict[str, Any] = {}
        self.fused: Dict[str, Any] = {}
        self._row_models: Dict[str, Any] = {}
        self._row_nodes: Dict[str, Dict] = {}
        self.fuse = fuse if fuse is not None else fusion_enabled(self.annotations())
        self.mesh = None
        self._mesh_plan = []
        remote = set()
        from ..parallel.fabric import is_mesh

        self._mesh_entered = False
        try:
            if is_mesh(fabric):
                from ..parallel import mesh as meshmod

                self._mesh_plan = meshmod.plan(self.predictor["graph"], bound=set(self.components))
                remote = {n for p in self._mesh_plan for n in p.absorbed}
            for node, _ in iter_nodes(self.predictor["graph"]):
                if node["name"] not in remote:  # placed subtrees are built on their ranks
                    self._bind(node)
            if is_mesh(fabric):
                self._bind_mesh_programs()
        except Exception as e:
            if is_mesh(fabric) and not self._mesh_entered:
                from ..parallel import mesh as meshmod

                meshmod.abort(fabric, f"{type(e).__name__}: {e}")  # the workers wait for rank 0's setup
            raise
        self._bind_row_models()
        self.engine.finalize()
        self._servers = []
        self._span_exporter = None
        if config is not None and config.tracing:
            from ..utils.tracing import NativeSpanExporter, configure_tracing

            self._span_exporter = NativeSpanExporter(self.engine, configure_tracing("seldon-svc-orch"))
        self.peers: Dict[str, "Deployment"] = {}
        if split:
            kw = dict(components=components, deployment_name=self.deployment_name, device=device, batcher=batcher,
                      log_requests=log_requests, log_responses=log_responses, fuse=fuse, config=config,
                      _metrics_from=self.engine)
            routes, shadows = [], []
            for p in all_preds:
                if p["name"] == pname:
                    continue
                peer = Deployment(self.sdep, predictor=p["name"], **kw)
                self.peers[p["name"]] = peer
                hdr = header_route(p, self.sdep)
                if hdr is not None:
                    self.engine.add_header_route(hdr[0], hdr[1], hdr[2], peer.engine)
                if is_shadow(p):
                    shadows.append(peer.engine)
                elif int(p.get("traffic", 0) or 0) > 0 or hdr is None:
                    routes.append((peer.engine, int(p.get("traffic", 0) or 0)))
            self.engine.set_traffic(int(self.predictor.get("traffic", 0) or 0), routes, shadows)

    @classmethod
    def resolver(cls, sdep: Dict, components: Optional[Dict[str, Any]], predictor: Dict) -> "Deployment":
        """A binding-only view (no engine): resolves nodes to component objects
        / row models the same way a Deployment does (used by worker ranks)."""
        self = cls.__new__(cls)
        self.C = native()
        self.sdep = sdep
        self.predictor = predictor
        self.components = dict(components or {})
        return self

    # ----------------------------------------------------------- binding
    def _node_device(self, node: Dict) -> int:
        if self.fabric is not None and node.get("rank") is not None:
            return int(self.fabric.device)  # rank-placed: the front end's side lives on its own GPU
        d = node.get("device")
        if d is None:
            return self.device
        d = int(d)
        # Placement is a hint: a CPU deployment (device -1) runs everything on
        # the host, and GPU ordinals wrap onto the GPUs that are present.
        if self.device < 0 or d < 0:
            return -1
        n = gpu_count()
        return d % n if n > 0 else -1

    def _batcher_opts(self, node: Dict) -> Dict[str, Any]:
        opts = dict(self.batcher_defaults)
        params = typed_parameters(node)
        for k in BATCHER_KEYS + ("max_retries",):
            if k in params:
                opts[k] = params[k]
        return opts

    def bind_row_model(self, node: Dict, row_model) -> None:
        # Deferred: row models may fuse into a device graph (_bind_row_models).
        self._row_models[node["name"]] = row_model
        self._row_nodes[node["name"]] = node

    def replica_devices(self, node: Dict):
        """GPUs serving a node: ``devices: [..]`` or ``replicas: N`` (extension
        fields; N consecutive GPUs from the node's device), or every GPU with the
        ``seldon.io/gpu-replicas: all`` annotation."""
        if node.get("devices"):
            return [self._node_device({"device": int(d)}) for d in node["devices"]]
        base = self._node_device(node)
        n = int(node.get("replicas", 1) or 1)
        if str(self.annotations().get("seldon.io/gpu-replicas", "")).lower() == "all" and base >= 0:
            n = max(n, gpu_count())
        if n <= 1 or base < 0:
            return [base]
        ngpu = max(1, gpu_count())
        return [(base + i) % ngpu for i in range(n)]

    def _make_unit(self, node: Dict, row_model, whole_graph: bool = False):
        devs = self.replica_devices(node)
        opts = self._batcher_opts(node)
        retries = int(opts.pop("max_retries", 1))
        if len(devs) == 1:
            return self.C.BatchedUnit(row_model, devs[0], **opts)
        reps = []
        for i, d in enumerate(devs):
            rm = row_model.clone_on(d) if whole_graph else (row_model if i == 0 else row_model.clone())
            reps.append(self.C.BatchedUnit(rm, d, **opts))
        return self.C.ReplicaUnit(reps, max_retries=retries)

    def _bind_batched(self, node: Dict, row_model) -> None:
        unit = self._make_unit(node, row_model)
        self.engine.bind_unit(node["name"], unit)
        self.batched[node["name"]] = unit
        self.units[node["name"]] = unit

    def _bind_mesh_programs(self) -> None:
        """Rank 0 of a mesh gang: plan + connect every placed subtree (collective
        with the workers' serve_peer) and serve each as one fused unit whose
        batches run on the worker ranks (parallel/mesh.py)."""
        from ..parallel import mesh as meshmod

        mr = int(self.batcher_defaults.get("max_batch", 1024))
        self._mesh_entered = True
        st = meshmod.setup(self.fabric, self.predictor["graph"], self._no_local_stage, max_rows=mr,
                           bound=set(self.components))
        self.mesh = st
        if st.peer.get("failed_edges"):
            logger.warning("mesh peer probe: edges %s fall back to host-staged slabs (%s)", st.peer["failed_edges"],
                           "; ".join(st.peer.get("errors") or []))
        nodes = {n["name"]: n for n, _ in iter_nodes(self.predictor["graph"])}
        for p, pid, fin in zip(st.programs, st.ids, st.finals):
            pm = self.fabric.program_model(pid, list(fin.get("names") or []), bool(fin.get("flat")))
            opts = self._batcher_opts(nodes[p.root])
            opts.pop("max_retries", None)
            opts.update(cpu_batching=True, slots=int(self.fabric.slots), max_batch=st.max_rows)
            unit = self.C.BatchedUnit(pm, -1, **opts)
            self.engine.bind_fused(p.root, unit, p.absorbed)
            self.batched[p.root] = unit
            self.units[p.root] = unit
            i = st.ids.index(pid)
            logger.info("mesh program %s (%s, %d messages per batch): %s; edges %s", p.root, self.fabric.transport,
                        st.messages[i], p.describe(),
                        ", ".join(f"{e['from']}->{e['to_rank']}:{e['transport']}" for e in
                                  (st.edges[i] if i < len(st.edges) else [])))

    @staticmethod
    def _no_local_stage(node: Dict):
        raise SpecError([f"node '{node['name']}' is placed on rank 0 inside a remote program"])

    def _bind_row_models(self) -> None:
        from ..parallel import device_graph
        from ..parallel.fabric import is_mesh, peer_model_for, rank_assignments

        # Nodes placed on other ranks (``rank: r``) are served there; with the
        # star (RCCL) fabric they become peer models on this rank's GPU.
        placed = {} if is_mesh(self.fabric) else rank_assignments(self.predictor["graph"])
        for r, names in placed.items():
            if self.fabric is None:
                if r != 0:
                    raise SpecError([f"graph places nodes on rank {r}; pass fabric=init_fabric()"])
                continue
            if r == self.fabric.rank:
                continue
            for mid, name in enumerate(names):
                if name not in self._row_models:
                    raise SpecError([f"node '{name}' placed on rank {r} is not a GPU row model"])
                node = self._row_nodes[name]
                self._row_models[name] = peer_model_for(self.C, self.fabric, node, self._row_models[name], mid)
        done = set()
        if self.fuse and self._row_models:
            for fg in device_graph.plan(self.predictor["graph"], self._row_models, self.units, self._node_device):
                try:
                    gm = device_graph.build(self.C, fg, split=device_graph.split_enabled(self.annotations()))
                except Exception as e:  # stage widths disagree: the engine reports it per request
                    logger.info("device graph at %s not fused: %s", fg.root, e)
                    continue
                root = next(n for n, _ in iter_nodes(self.predictor["graph"]) if n["name"] == fg.root)
                unit = self._make_unit(root, gm, whole_graph=True)
                self.engine.bind_fused(fg.root, unit, fg.absorbed)
                self.batched[fg.root] = unit
                self.units[fg.root] = unit
                self.fused[fg.root] = fg
                logger.info("device graph %s: %s", fg.root, device_graph.describe(fg))
                done.update(fg.absorbed)
        for name, rm in self._row_models.items():
            if name not in done:
                self._bind_batched(self._row_nodes[name], rm)

    def bind_python(self, node: Dict, obj: Any) -> None:
        unit_type = node.get("type", "MODEL")
        if unit_type in (None, "UNKNOWN_TYPE"):
            unit_type = "UNKNOWN_TYPE"
        adapter = PythonUnit(obj, unit_type, node["name"])
        batch_rows, workers = self._python_options(node, obj)
        fds = []
        if workers > 0:
            try:
                fds = adapter.start_pool(workers)
            except (pickle.PicklingError, TypeError, AttributeError, RuntimeError) as e:
                logger.warning("node %s: cannot run the component in %d worker processes (%s); serving it in-process",
                               node["name"], workers, e)
        adapter.native = self.engine.bind_python(node["name"], adapter, 0, batch_rows, fds)
        self.units[node["name"]] = adapter
        self.__dict__.setdefault("python_units", {})[node["name"]] = adapter

    def _python_options(self, node: Dict, obj: Any):
        """(batch_rows, workers) of a Python node.  Precedence: node extension
        fields ``batching`` / ``workers`` > component attributes
        ``seldon_batching`` / ``seldon_workers`` > annotations
        ``seldon.io/python-batching`` / ``seldon.io/python-workers``
        (the reference's ``--workers`` / GUNICORN_WORKERS)."""
        ann = self.annotations()

        def pick(field: str, attr: str, key: str):
            if node.get(field) is not None:
                return node[field]
            if getattr(obj, attr, None) is not None:
                return getattr(obj, attr)
            return ann.get(key)

        b = pick("batching", "seldon_batching", "seldon.io/python-batching")
        if isinstance(b, str):
            b = {"true": 4096, "false": 0}.get(b.lower(), b)
        batch_rows = 4096 if b is True else int(b or 0)
        workers = int(pick("workers", "seldon_workers", "seldon.io/python-workers") or 0)
        return max(0, batch_rows), max(0, workers)

    def _instantiate(self, node: Dict, obj: Any) -> Any:
        if isinstance(obj, str):
            obj = import_class(obj)
        if isinstance(obj, type):
            obj = obj(**typed_parameters(node))
            if hasattr(obj, "load"):
                obj.load()
        return obj

    def _row_model_of(self, obj: Any):
        """The native RowModel behind a component object, or None."""
        from ..models import to_row_model

        if isinstance(obj, self.C.RowModel):
            return obj
        if isinstance(obj, self.C.Unit) or callable(getattr(obj, "native_unit", None)):
            return None
        gpu = getattr(obj, "row_model", None)
        if callable(gpu):
            rm = gpu()
            if rm is not None:
                return rm
        rm = to_row_model(obj) if not hasattr(obj, "predict_raw") else None
        if rm is not None and not any(hasattr(obj, m) for m in ("route", "aggregate", "transform_input")):
            return rm
        return None

    def shared_state_name(self, node: Dict) -> Optional[str]:
        """Name of the host-wide shared mapping of a stateful node when the
        supervisor runs several engine processes (SCA_SHARED_STATE prefix,
        SCA_WORKERS > 1), else None."""
        prefix = os.environ.get("SCA_SHARED_STATE")
        if not prefix or int(os.environ.get("SCA_WORKERS", "1") or 1) <= 1:
            return None
        import re

        tag = re.sub(r"[^A-Za-z0-9_.-]", "_", f"{self.deployment_name}_{self.predictor.get('name', '')}_{node['name']}")
        return f"{prefix}_{tag}"[:250]

    def _bind_object(self, node: Dict, obj: Any) -> None:
        obj = self._instantiate(node, obj)
        rm = self._row_model_of(obj)
        if rm is not None:
            self.bind_row_model(node, rm)
            return
        if isinstance(obj, self.C.Unit):
            self.engine.bind_unit(node["name"], obj)
            self.units[node["name"]] = obj
            return
        native_unit = getattr(obj, "native_unit", None)
        if callable(native_unit):
            share = getattr(obj, "share_state", None)
            name = self.shared_state_name(node)
            if callable(share) and name:
                share(name, int(os.environ.get("SCA_WORKER_RANK", "0") or 0))
            unit = native_unit(self._node_device(node))
            self.engine.bind_unit(node["name"], unit)
            self.units[node["name"]] = unit
            self.native_units[node["name"]] = unit
            return
        self.bind_python(node, obj)

    def _resolve(self, node: Dict):
        """What implements a node: ("builtin", None), ("object", obj) or
        ("remote", (host, port, grpc, container))."""
        name = node["name"]
        impl = node.get("implementation", "UNKNOWN_IMPLEMENTATION")
        if name in self.components:
            return "object", self.components[name]
        if impl in BUILTIN_IMPLEMENTATIONS:
            return "builtin", None
        params = typed_parameters(node)
        if impl in PREPACKAGED_SERVERS:
            from ..servers import load_prepackaged

            return "object", load_prepackaged(impl, node.get("modelUri", ""), params)
        from ..components import NATIVE_IMPLEMENTATIONS

        if impl in NATIVE_IMPLEMENTATIONS:
            return "object", NATIVE_IMPLEMENTATIONS[impl](**params)
        cls_path = params.pop("python_class", None)
        c = container_for(self.predictor, name)
        if not cls_path and c:
            for e in c.get("env", []) or []:
                if e.get("name") in ("MODEL_NAME", "SELDON_PYTHON_CLASS"):
                    cls_path = e.get("value")
        if cls_path:
            obj = import_class(cls_path)(**params)
            if hasattr(obj, "load"):
                obj.load()
            return "object", obj
        ep = node.get("endpoint") or {}
        host = ep.get("service_host") or ep.get("serviceHost")
        port = ep.get("service_port") or ep.get("servicePort")
        if host and port:
            return "remote", (host, int(port), ep.get("type", "REST") == "GRPC", c)
        raise SpecError([f"no implementation for graph node '{name}' ({impl}); pass components={{'{name}': ...}}"])

    def _bind(self, node: Dict) -> None:
        kind, what = self._resolve(node)
        if kind == "object":
            self._bind_object(node, what)
        elif kind == "remote":
            self.bind_remote(node, *what)

    def annotations(self) -> Dict[str, str]:
        ann = dict((self.sdep.get("spec") or {}).get("annotations") or {})
        ann.update(self.predictor.get("annotations") or {})
        return ann

    def bind_remote(self, node: Dict, host: str, port: int, grpc: bool, container: Optional[Dict] = None) -> None:
        """Out-of-process microservice node (reference InternalPredictionService)."""
        ann = self.annotations()
        image = (container or {}).get("image", "")
        img_name, _, img_ver = image.rpartition(":") if ":" in image else (image, "", "")
        unit = self.C.RemoteUnit(
            host, port, grpc, node.get("type", "MODEL"), node["name"], img_name, img_ver,
            int(ann.get("seldon.io/rest-connection-timeout", 200)),
            int(ann.get("seldon.io/grpc-read-timeout" if grpc else "seldon.io/rest-read-timeout", 5000)),
            int(ann.get("seldon.io/rest-connect-retries", 3)))
        self.engine.bind_unit(node["name"], unit)
        self.units[node["name"]] = unit

    # ----------------------------------------------------------- requests
    def predict(self, payload: Union[Dict, str], headers: Optional[Dict[str, str]] = None) -> Dict:
        text = payload if isinstance(payload, str) else json.dumps(payload)
        status, body = self.engine.predict_json(text, dict(headers or {}))
        out = json.loads(body)
        if status != 200:
            raise EngineError(status, out)
        return out

    def predict_raw(self, payload: Union[Dict, str]):
        text = payload if isinstance(payload, str) else json.dumps(payload)
        status, body = self.engine.predict_json(text)
        return status, json.loads(body)

    def predict_pb(self, data: bytes):
        return self.engine.predict_pb(data)

    def feedback(self, payload: Union[Dict, str]) -> Dict:
        text = payload if isinstance(payload, str) else json.dumps(payload)
        status, body = self.engine.feedback_json(text)
        out = json.loads(body)
        if status != 200:
            raise EngineError(status, out)
        return out

    def call_node(self, node: str, method: str, payload: Union[Dict, str]):
        text = payload if isinstance(payload, str) else json.dumps(payload)
        status, body = self.engine.call_node_json(node, METHOD_IDS[method], text)
        return status, json.loads(body)

    def metrics(self) -> str:
        return self.engine.metrics_text()

    def ready(self) -> bool:
        return bool(self.engine.ready())

    def batcher_stats(self) -> Dict[str, Dict]:
        out = {k: v.stats() for k, v in self.batched.items()}
        for pn, p in getattr(self, "peers", {}).items():
            out.update({f"{pn}/{k}": v for k, v in p.batcher_stats().items()})
        return out

    # -------------------------------------------------------- checkpoint
    # the reference snapshots a component's state (the pickled
    # user object) into Redis every push_frequency seconds and restores it at
    # start (python/seldon_core/persistence.py:21-85, microservice.py:227-230).
    # Here every stateful node of the graph -- native bandit routers (JSON),
    # Python components and outlier detectors (state_dict / pickle) --
    # checkpoints under persistence_<deployment>_<predictor>_<node>[_w<rank>].
    def checkpoint_key(self, node: str, worker: Optional[str] = None) -> str:
        from ..utils.persistence import state_key

        key = state_key(self.deployment_name, self.predictor.get("name", "0"), node)
        worker = os.environ.get("SCA_WORKER_RANK") if worker is None else worker
        world = int(os.environ.get("SCA_WORKERS", "1") or 1)
        return f"{key}_w{worker}" if worker and world > 1 else key

    def checkpoint(self, store=None) -> int:
        """Write every stateful node's snapshot; returns how many were written."""
        from ..utils.persistence import default_store

        store = store or default_store()
        n = 0
        for node in self.engine.node_names():
            try:
                blob = self.engine.snapshot(node)
                if blob:
                    store.set(self.checkpoint_key(node), blob)
                    n += 1
            except Exception as e:  # one unpicklable component must not stop the others
                logger.warning("checkpoint of node %s failed: %s", node, e)
        return n

    def restore_checkpoint(self, store=None) -> int:
        """Restore nodes from their snapshots; returns how many were restored."""
        from ..utils.persistence import default_store

        store = store or default_store()
        n = 0
        for node in self.engine.node_names():
            try:
                blob = store.get(self.checkpoint_key(node))
            except Exception as e:  # store unreachable: start fresh like the reference
                logger.warning("checkpoint restore of %s failed: %s", node, e)
                continue
            if blob:
                self.engine.restore(node, blob)
                n += 1
        if n:
            logger.info("restored %d node state(s) of %s", n, self.deployment_name)
        return n

    def start_checkpointing(self, push_frequency: Optional[float] = None, store=None):
        """Periodic checkpoints on a daemon thread; close() writes a last one."""
        from ..utils.persistence import Persister, default_store

        store = store or default_store()
        self._ckpt_store = store

        class _Pusher(Persister):
            def push(inner) -> None:  # noqa: N805
                self.checkpoint(store)

        self._persister = _Pusher(lambda: b"", push_frequency, store, key="-")
        self._persister.start()
        return self._persister

    # ----------------------------------------------------------- serving
    def serve(self, http_port: int = 8000, grpc_port: Optional[int] = 5001, admin_port: Optional[int] = None,
              threads: int = 4, grpc_threads: Optional[int] = None, host: str = "0.0.0.0",
              microservice_node: str = "") -> "ServerHandle":
        ports = [http_port] + ([admin_port] if admin_port else [])
        http = self.C.HttpServer(self.engine, host, ports, threads, microservice_node, True, "")
        http.start()
        grpc = None
        if grpc_port is not None:
            max_msg = (self.config.grpc_max_message_size if self.config is not None else None) or (64 << 20)
            grpc = self.C.GrpcServer(self.engine, host, grpc_port, grpc_threads or threads, microservice_node,
                                     int(max_msg))
            grpc.start()
        h = ServerHandle(self, http, grpc)
        self._servers.append(h)
        return h

    def close(self) -> None:
        for s in self._servers:
            s.stop()
        self._servers = []
        if getattr(self, "_persister", None) is not None:
            self._persister.stop()
            self.checkpoint(self._ckpt_store)  # final snapshot after the drain
            self._persister = None
        for u in list(self.batched.values()) + list(self.native_units.values()):
            u.stop()
        for a in getattr(self, "python_units", {}).values():
            if getattr(a, "native", None) is not None:
                a.native.stop()  # closes the pool sockets: workers exit on EOF
            a.stop_pool()
        for p in getattr(self, "peers", {}).values():
            p.close()
        if getattr(self, "_span_exporter", None) is not None:
            self._span_exporter.close()
            self._span_exporter = None
        if getattr(self, "fabric", None) is not None and self.fabric.rank == 0:
            self.fabric.stop_peers()  # worker ranks leave their serve loops
            self.fabric = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class ServerHandle:
    def __init__(self, dep: Deployment, http, grpc):
        self.deployment = dep
        self.http = http
        self.grpc = grpc

    @property
    def http_port(self) -> int:
        return self.http.ports[0]

    @property
    def grpc_port(self) -> Optional[int]:
        return self.grpc.port if self.grpc else None

    def drain(self, timeout_s: float = 20.0, poll_s: float = 0.01) -> bool:
        """Graceful shutdown (reference App.java:39-107 + preStop ``/pause``):
        flip readiness off so load balancers stop sending, wait up to
        ``timeout_s`` for in-flight requests to finish, then stop the servers.
        Returns True if everything in flight completed."""
        import time

        if self.http:
            self.http.paused = True
        eng = self.deployment.engine
        deadline = time.monotonic() + timeout_s
        while eng.inflight() > 0 and time.monotonic() < deadline:
            time.sleep(poll_s)
        clean = eng.inflight() == 0
        self.stop()
        return clean

    def stop(self) -> None:
        if self.http:
            self.http.stop()
            self.http = None
        if self.grpc:
            self.grpc.stop()
            self.grpc = None
