"""Rank-placed subtrees as mesh programs (``ipc`` / ``shm`` fabric transports).

The reference runs every graph node in its own pod and walks the graph from
the engine, one HTTP/gRPC round trip per node (engine/.../PredictiveUnitBean.java:
112-197 -> InternalPredictionService.java:186-453).  Here a subtree whose nodes
are placed on worker ranks (``rank: r``, one engine process per MI355X) is
planned into a PROGRAM -- a small DAG of stages with a rank each -- that every
rank of the gang derives from the same spec.  Rank 0 hands the batch to the
first stages; each stage's output goes straight to the rank that consumes it
(csrc/parallel/mesh.h); only the program's output returns to rank 0, where the
engine sees the whole subtree as one fused unit (``Engine::bind_fused``).

Stage kinds:

* ``node``: a MODEL / TRANSFORMER / OUTPUT_TRANSFORMER node on a worker rank,
  run there as a native row model (GPU kernels) or, for any other component, as
  a Python call on dense rows (``in_cols`` / ``out_cols`` node fields declare
  widths the spec cannot imply; a shape-preserving component needs neither);
* ``mean``: an AVERAGE_COMBINER over stages.  The program's final mean runs on
  rank 0's host; an inner one runs on the rank of the stage that consumes it,
  or -- when that consumer is the final mean -- on the rank of its first input
  (:func:`_place_means`).

Evaluation rules follow ``device_graph`` (the reference's
PredictiveUnitImpl.java:27-52 and AverageCombinerUnit.java:35-79): a model's
output feeds its first child; an OUTPUT_TRANSFORMER applies to its first
child's output; a combiner averages every child.

Setup is collective over the default ``torch.distributed`` group: every rank
calls :func:`setup` with the same plan (rank 0 from ``Deployment``, workers from
``serve_peer``): phase A exchanges each rank's stage widths (and rank 0's batch
size), phase B the shared-memory region names and HIP IPC handles.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..serving.spec import SpecError

FUSABLE_TYPES = {"MODEL", "TRANSFORMER", "OUTPUT_TRANSFORMER"}
KIND = {"node": 0, "mean": 1, "host": 2}


@dataclass
class StagePlan:
    node: str
    rank: Optional[int]
    kind: str                      # "node" | "mean"
    inputs: List[int]


@dataclass
class ProgramPlan:
    root: str
    stages: List[StagePlan]
    absorbed: List[str] = field(default_factory=list)

    def describe(self) -> str:
        parts = []
        for i, s in enumerate(self.stages):
            src = ",".join("in" if j < 0 else f"s{j}" for j in s.inputs)
            parts.append(f"s{i}={s.kind}:{s.node}@rank{s.rank}({src})")
        return " ".join(parts)


def _rank(node: Dict) -> Optional[int]:
    r = node.get("rank")
    return None if r is None else int(r)


def _is_combiner(node: Dict, bound: set) -> bool:
    return (node.get("implementation") == "AVERAGE_COMBINER" and node["name"] not in bound
            and bool(node.get("children")))


def _remote_node(node: Dict) -> bool:
    r = _rank(node)
    return r is not None and r > 0 and node.get("type", "MODEL") in FUSABLE_TYPES


def _fusable(node: Dict, bound: set) -> bool:
    kids = node.get("children") or []
    if _is_combiner(node, bound):
        return all(_fusable(c, bound) for c in kids)
    if not _remote_node(node):
        return False
    t = node.get("type", "MODEL")
    if t == "OUTPUT_TRANSFORMER":
        return not kids or _fusable(kids[0], bound)
    return not kids or _fusable(kids[0], bound)


def _subtree(node: Dict) -> List[Dict]:
    out = [node]
    for c in node.get("children") or []:
        out.extend(_subtree(c))
    return out


def _emit(node: Dict, in_idx: int, stages: List[StagePlan], bound: set) -> int:
    kids = node.get("children") or []
    if _is_combiner(node, bound):
        outs = [_emit(c, in_idx, stages, bound) for c in kids]
        stages.append(StagePlan(node["name"], _rank(node), "mean", outs))
        return len(stages) - 1
    if node.get("type", "MODEL") == "OUTPUT_TRANSFORMER":
        if not kids:
            return in_idx  # a leaf output transformer passes its input through
        o = _emit(kids[0], in_idx, stages, bound)
        stages.append(StagePlan(node["name"], _rank(node), "node", [o]))
        return len(stages) - 1
    stages.append(StagePlan(node["name"], _rank(node), "node", [in_idx]))
    s = len(stages) - 1
    return _emit(kids[0], s, stages, bound) if kids else s


def _place_means(stages: List[StagePlan]) -> None:
    """Ranks of a program's ``mean`` stages, consumers before producers
    (reverse topological order: a stage only reads earlier stages).  The
    program's output mean runs on rank 0's host; an inner mean runs on the
    rank of the stage that consumes it -- unless that consumer is a mean on
    rank 0 (the mesh runs only the final mean there), in which case it runs
    on the rank of its first input, as does one whose consumer has no rank."""
    last = len(stages) - 1

    def input_rank(j: int) -> Optional[int]:
        while j >= 0:
            t = stages[j]
            if t.kind != "mean" or (t.rank is not None and t.rank > 0):
                return t.rank
            j = t.inputs[0]
        return None

    for i in range(last, -1, -1):
        s = stages[i]
        if s.kind != "mean":
            continue
        if i == last:
            s.rank = 0
            continue
        consumer = next(t for t in stages[i + 1:] if i in t.inputs)
        r = consumer.rank
        if r is None or r <= 0:
            r = input_rank(s.inputs[0])
        if r is None or r <= 0:
            raise SpecError([f"combiner '{s.node}': no worker rank can run it (its inputs and consumer are on "
                             "rank 0)"])
        s.rank = r


def plan(graph: Dict, bound: Optional[set] = None) -> List[ProgramPlan]:
    """Maximal subtrees of worker-placed nodes (joined by AVERAGE_COMBINERs),
    outermost first.  Raises SpecError for a placed node that cannot run on a
    worker (routers and other rank-0 logic)."""
    bound = set(bound or ())
    found: List[ProgramPlan] = []

    def visit(node: Dict) -> None:
        if _fusable(node, bound) and (_remote_node(node) or _is_combiner(node, bound)):
            stages: List[StagePlan] = []
            out = _emit(node, -1, stages, bound)
            if out >= 0 and out == len(stages) - 1 and any(s.kind == "node" for s in stages):
                _place_means(stages)
                found.append(ProgramPlan(node["name"], stages, [n["name"] for n in _subtree(node)]))
                return
        r = _rank(node)
        if r is not None and r > 0 and not _fusable(node, bound):
            if node.get("type", "MODEL") not in FUSABLE_TYPES or _is_combiner(node, bound):
                raise SpecError([f"node '{node['name']}' ({node.get('type', 'MODEL')}) cannot be placed on rank {r}: "
                                 "only MODEL / TRANSFORMER / OUTPUT_TRANSFORMER nodes and combiners over them run "
                                 "on worker ranks"])
            # a placed node whose child must stay on rank 0 (a router, an
            # unplaced node): no program can absorb it, and silently running
            # it on rank 0 would ignore the spec's placement
            kid = (node.get("children") or [{}])[0]
            raise SpecError([f"node '{node['name']}' is placed on rank {r} but its child '{kid.get('name')}' "
                             f"({kid.get('type', 'MODEL')}, rank {kid.get('rank', 0)}) cannot run on a worker "
                             "rank: place the child on a worker too, or the node on rank 0"])
        for c in node.get("children") or []:
            visit(c)

    visit(graph)
    return found


def placed_ranks(programs: List[ProgramPlan]) -> List[int]:
    return sorted({s.rank for p in programs for s in p.stages if s.rank})


# ------------------------------------------------------------------ widths
def stage_info(res, node: Dict) -> Tuple[Dict[str, Any], Any]:
    """(info, implementation) of a stage hosted on this rank: a native row
    model, or a Python component called on dense rows."""
    kind, obj = res._resolve(node)
    if kind != "object":
        raise SpecError([f"node '{node['name']}' placed on rank {node.get('rank')} has no in-process implementation"])
    obj = res._instantiate(node, obj)
    rm = res._row_model_of(obj)
    if rm is not None:
        ic = int(rm.in_cols)
        if ic > 0:
            oc, same = int(rm.out_cols(ic)), False
        else:
            same = int(rm.out_cols(5)) == 5 and int(rm.out_cols(7)) == 7
            oc = None if same else int(rm.out_cols(1))
        info = {"kind": "node", "in": ic or None, "out": oc, "same": same,
                "names": list(rm.class_names()), "flat": bool(rm.flat_output)}
        return info, rm
    ic = node.get("in_cols")
    oc = node.get("out_cols")
    info = {"kind": "host", "in": int(ic) if ic else None, "out": int(oc) if oc else None, "same": oc is None,
            "names": [], "flat": False}
    return info, host_callable(obj, node)


def host_callable(obj: Any, node: Dict) -> Callable:
    """Dense-rows call of a Python component by node type (the reference's
    seldon_methods predict / transform_input / transform_output)."""
    import numpy as np

    from ..serving.user_model import client_predict, client_transform_input, client_transform_output

    t = node.get("type", "MODEL")
    fn = {"MODEL": client_predict, "TRANSFORMER": client_transform_input,
          "OUTPUT_TRANSFORMER": client_transform_output}[t]

    def call(X):
        out = fn(obj, X, [])
        return np.ascontiguousarray(np.asarray(out, dtype=np.float64))

    return call


def resolve_widths(p: ProgramPlan, infos: Dict[int, Dict[str, Any]]) -> Tuple[int, List[Tuple[int, int]], Dict]:
    """(program in_cols, [(in, out) per stage], final info) from the stages'
    reported widths; raises SpecError when the spec leaves a width open."""
    x = None
    for i, s in enumerate(p.stages):
        if -1 in s.inputs and s.kind == "node" and infos[i].get("in"):
            if x is not None and x != infos[i]["in"]:
                raise SpecError([f"program at '{p.root}': stages disagree on the input width ({x} vs "
                                 f"{infos[i]['in']})"])
            x = int(infos[i]["in"])
    if x is None:
        raise SpecError([f"program at '{p.root}': input width unknown; give the first placed node an 'in_cols' "
                         "field or a model with a fixed input width"])
    widths: List[Tuple[int, int]] = []
    for i, s in enumerate(p.stages):
        ins = [x if j < 0 else widths[j][1] for j in s.inputs]
        if s.kind == "mean":
            if len(set(ins)) != 1:
                raise SpecError([f"combiner '{s.node}' averages outputs of different widths {ins}"])
            widths.append((ins[0], ins[0]))
            continue
        inf = infos[i]
        w = ins[0]
        if inf.get("in") and int(inf["in"]) != w:
            raise SpecError([f"node '{s.node}' takes {inf['in']} columns but receives {w}"])
        out = w if inf.get("same") else inf.get("out")
        if not out:
            raise SpecError([f"node '{s.node}': output width unknown; give it an 'out_cols' field"])
        widths.append((w, int(out)))
    last = p.stages[-1]
    final = infos.get(len(p.stages) - 1) if last.kind == "node" else None
    if last.kind == "mean":  # a combiner's response keeps its first branch's names
        j = last.inputs[0]
        while j >= 0 and p.stages[j].kind == "mean":
            j = p.stages[j].inputs[0]
        final = infos.get(j) if j >= 0 else None
    return x, widths, (final or {"names": [], "flat": False})


# ------------------------------------------------------------------ setup
def _all_gather(obj):
    import torch.distributed as dist

    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


@dataclass
class MeshSetup:
    programs: List[ProgramPlan]
    ids: List[int]
    in_cols: List[int]
    finals: List[Dict[str, Any]]
    max_rows: int
    messages: List[int]
    peer: Dict[str, Any] = field(default_factory=dict)       # probe_peers() report
    edges: List[List[Dict[str, Any]]] = field(default_factory=list)  # per program: edge transports


def probe_peers(mesh) -> Dict[str, Any]:
    """Collective peer-readiness check before any program is laid out (VERDICT
    r5 next #3; the reference's equivalent hop is PredictiveUnitBean.java:
    170-183 -> an HTTP call that either connects or fails the request).

    Records the gang's GPUs and their ``hipDeviceCanAccessPeer`` matrix, then
    has every GPU worker open every other worker's probe buffer over HIP IPC
    and round-trip a canary through it with the copy the programs use
    (``Mesh::probe_connect``).  An edge whose probe failed becomes a
    host-staged slab ("ipc-host") in every rank's layout -- the gang serves
    instead of failing setup -- and the report says which.  A failure to run
    the probe at all on any rank aborts setup on every rank."""
    st: Dict[str, Any] = {}
    blob = b""
    try:
        blob = mesh.probe_prepare()
    except Exception as e:  # noqa: BLE001
        st["abort"] = f"rank {mesh.rank}: probe: {type(e).__name__}: {e}"[:500]
    got = _all_gather((st, blob, int(mesh.device)))
    _raise_aborts([g[0] for g in got])
    devices = [g[2] for g in got]
    row: List[int] = [-1] * len(got)
    try:
        row = list(mesh.probe_connect([g[1] for g in got]))
    except Exception as e:  # noqa: BLE001
        st["abort"] = f"rank {mesh.rank}: probe: {type(e).__name__}: {e}"[:500]
    rows = _all_gather((st, row, mesh.probe_error()))
    try:
        _raise_aborts([r[0] for r in rows])
        world = len(rows)
        ok = [[1] * world for _ in range(world)]
        failed = []
        for prod in range(world):
            for cons in range(world):
                if rows[prod][1][cons] == 0:
                    ok[prod][cons] = 0
                    failed.append(f"{prod}->{cons}")
        mesh.set_peer_ok(ok)
    finally:
        _all_gather(None)  # every worker is done with the others' probe buffers
        mesh.probe_finish()
    report: Dict[str, Any] = {"devices": devices, "probed": {str(r): rows[r][1] for r in range(len(rows))},
                              "failed_edges": failed, "errors": [r[2] for r in rows if r[2]]}
    gpus = sorted({d for d in devices if d >= 0})
    if len(gpus) > 1:
        try:
            from .._native import native

            C = native()
            report["can_access_peer"] = {f"{a}->{b}": bool(C.can_access_peer(a, b)) for a in gpus for b in gpus
                                         if a != b}
        except Exception as e:  # noqa: BLE001
            report["can_access_peer"] = {"error": str(e)[:200]}
    return report


def abort(mesh, reason: str) -> None:
    """Rank 0 could not get as far as ``setup`` (a local node failed to bind):
    take part in setup's first exchange with the reason, so the workers raise
    instead of waiting in it."""
    _all_gather({"abort": f"rank {mesh.rank}: {reason}"[:500], "max_rows": 0, "stages": {}})


def _raise_aborts(gathered) -> None:
    why = [g["abort"] for g in gathered if g.get("abort")]
    if why:
        raise SpecError([f"mesh setup failed: {w}" for w in why])


def setup(mesh, graph: Dict, resolve_stage: Callable[[Dict], Tuple[Dict, Any]], max_rows: int = 0,
          bound: Optional[set] = None) -> MeshSetup:
    """Collective: plan the graph's placed subtrees, agree on widths, build
    the shared regions and connect every rank.  `resolve_stage(node)` gives
    (info, implementation) for a node hosted on this rank.  A failure on any
    rank fails the setup on every rank (no rank is left waiting)."""
    from ..serving.spec import iter_nodes

    me = mesh.rank
    infos: Dict[str, Any] = {"max_rows": int(max_rows) if me == 0 else 0, "stages": {}}
    mine: Dict[Tuple[int, int], Any] = {}
    progs: List[ProgramPlan] = []
    try:
        progs = plan(graph, bound)
        nodes = {n["name"]: n for n, _ in iter_nodes(graph)}
        for pi, p in enumerate(progs):
            for si, s in enumerate(p.stages):
                if s.kind == "node" and s.rank == me:
                    info, impl = resolve_stage(nodes[s.node])
                    infos["stages"][f"{pi}:{si}"] = info
                    mine[(pi, si)] = (info, impl)
    except Exception as e:  # noqa: BLE001 -- reported to every rank below
        infos["abort"] = f"rank {me}: {type(e).__name__}: {e}"[:500]
    gathered = _all_gather(infos)
    _raise_aborts(gathered)
    mr = int(gathered[0]["max_rows"])
    if mr <= 0:
        raise SpecError(["mesh setup: rank 0 gave no batch size"])
    merged: Dict[str, Any] = {}
    for g in gathered:
        merged.update(g["stages"])
    peer = probe_peers(mesh) if hasattr(mesh, "probe_prepare") else {}
    ids, in_cols, finals, msgs, edges = [], [], [], [], []
    for pi, p in enumerate(progs):
        stage_infos = {si: merged[f"{pi}:{si}"] for si, s in enumerate(p.stages) if s.kind == "node"
                       and f"{pi}:{si}" in merged}
        missing = [s.node for si, s in enumerate(p.stages) if s.kind == "node" and si not in stage_infos]
        if missing:
            raise SpecError([f"mesh setup: no rank resolved {missing}"])
        x, widths, final = resolve_widths(p, stage_infos)  # same inputs everywhere: same outcome everywhere
        desc = {"max_rows": mr, "in_cols": x, "stages": []}
        for si, s in enumerate(p.stages):
            kind = "mean" if s.kind == "mean" else stage_infos[si]["kind"]
            desc["stages"].append({"rank": int(s.rank), "kind": KIND[kind], "inputs": list(s.inputs),
                                   "in_cols": widths[si][0], "out_cols": widths[si][1], "node": s.node})
        pid = mesh.add_program(desc)
        for si, s in enumerate(p.stages):
            if (pi, si) in mine:
                info, impl = mine[(pi, si)]
                if info["kind"] == "node":
                    mesh.set_model(pid, si, impl)
                else:
                    mesh.set_host_fn(pid, si, impl)
        ids.append(pid)
        in_cols.append(x)
        finals.append(final)
        msgs.append(int(mesh.messages_per_batch(pid)))
        if hasattr(mesh, "edge_transports"):
            edges.append([{"from": f"{p.stages[i].node}@{p.stages[i].rank}", "to_rank": c, "transport": t}
                          for i, c, t in mesh.edge_transports(pid)])
    status: Dict[str, Any] = {}
    blob = b""
    try:
        blob = mesh.prepare()
    except Exception as e:  # noqa: BLE001
        status["abort"] = f"rank {me}: {type(e).__name__}: {e}"[:500]
    blobs = _all_gather((status, blob))
    _raise_aborts([b[0] for b in blobs])
    try:
        try:
            mesh.connect([b[1] for b in blobs])
        except Exception as e:  # noqa: BLE001
            status["abort"] = f"rank {me}: {type(e).__name__}: {e}"[:500]
        _raise_aborts(_all_gather(status))  # doubles as the barrier before the names go
    finally:
        mesh.unlink()  # every rank has mapped every region (or failed): nothing stays in /dev/shm
    mesh.start()
    return MeshSetup(progs, ids, in_cols, finals, mr, msgs, peer, edges)
