"""Device-graph planner: fuse all-row-model subtrees into one GPU unit.

The reference runs each graph node as its own microservice and moves the
SeldonMessage between them as JSON over HTTP (engine/.../PredictiveUnitBean.java:112-197,
InternalPredictionService.java:186-453).  Here, a subtree whose nodes are all
GPU row models (TRANSFORMER / MODEL / OUTPUT_TRANSFORMER nodes bound to a
``RowModel``) joined by AVERAGE_COMBINERs is compiled into one native
``GraphModel`` (csrc/gpu/graph.h) behind one micro-batcher: the request rows go
to HBM once, every stage runs on its node's GPU, cross-GPU edges are direct
xGMI peer reads, and the combiner is the ``combine_mean_f64`` kernel.

Evaluation rules mirrored from the reference executor:

* MODEL / TRANSFORMER: transform-input (the model), children receive its
  output; with several children the default ``aggregate`` keeps the first
  child's output (PredictiveUnitImpl.java:27-52), so only child 0 is computed.
* OUTPUT_TRANSFORMER: children receive the input unchanged; the model is
  applied to the aggregated child output; a leaf is the identity
  (PredictiveUnitBean.java:128-138,188-192).
* AVERAGE_COMBINER: every child receives the input; element-wise mean of
  their 2-D outputs (AverageCombinerUnit.java:35-79).

Anything else (routers, Python components, remote nodes, built-in stubs)
stops fusion; those nodes keep their own units and the engine evaluates them.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

FUSABLE_TYPES = {"MODEL", "TRANSFORMER", "OUTPUT_TRANSFORMER"}


@dataclass
class FusedGraph:
    root: str
    stages: List[Dict[str, Any]]
    absorbed: List[str] = field(default_factory=list)   # every node of the subtree (root first)
    devices: List[int] = field(default_factory=list)

    @property
    def n_stages(self) -> int:
        return len(self.stages)


def _is_combiner(node: Dict, bound: Dict[str, Any]) -> bool:
    return (node.get("implementation") == "AVERAGE_COMBINER" and node["name"] not in bound
            and bool(node.get("children")))


def _fusable(node: Dict, row_models: Dict[str, Any], bound: Dict[str, Any]) -> bool:
    children = node.get("children") or []
    if _is_combiner(node, bound):
        ok = all(_fusable(c, row_models, bound) for c in children)
        # AverageCombinerUnit rejects 1-D (flat) outputs: keep the engine's error path.
        return ok and not any(_flat_output(c, row_models, bound) for c in children)
    if node["name"] not in row_models or node.get("type", "MODEL") not in FUSABLE_TYPES:
        return False
    return all(_fusable(c, row_models, bound) for c in children)


def _flat_output(node: Dict, row_models: Dict[str, Any], bound: Dict[str, Any]) -> bool:
    children = node.get("children") or []
    t = node.get("type", "MODEL")
    if _is_combiner(node, bound):
        return False
    if t == "OUTPUT_TRANSFORMER":
        return bool(children) and bool(row_models[node["name"]].flat_output)
    if children:
        return _flat_output(children[0], row_models, bound)
    return bool(row_models[node["name"]].flat_output)


def _subtree(node: Dict) -> List[Dict]:
    out = [node]
    for c in node.get("children") or []:
        out.extend(_subtree(c))
    return out


def _emit(node: Dict, in_idx: int, stages: List[Dict], row_models: Dict[str, Any], bound: Dict[str, Any],
          device_of: Callable[[Dict], int]) -> int:
    children = node.get("children") or []
    if _is_combiner(node, bound):
        outs = [_emit(c, in_idx, stages, row_models, bound, device_of) for c in children]
        stages.append({"kind": "mean", "inputs": outs, "device": device_of(node), "node": node["name"]})
        return len(stages) - 1
    t = node.get("type", "MODEL")
    if t == "OUTPUT_TRANSFORMER":
        if not children:
            return in_idx
        o = _emit(children[0], in_idx, stages, row_models, bound, device_of)
        stages.append({"kind": "model", "model": row_models[node["name"]], "inputs": [o],
                       "device": device_of(node), "node": node["name"]})
        return len(stages) - 1
    stages.append({"kind": "model", "model": row_models[node["name"]], "inputs": [in_idx],
                   "device": device_of(node), "node": node["name"]})
    s = len(stages) - 1
    if children:
        return _emit(children[0], s, stages, row_models, bound, device_of)
    return s


def plan(graph: Dict, row_models: Dict[str, Any], bound: Dict[str, Any],
         device_of: Callable[[Dict], int]) -> List[FusedGraph]:
    """Maximal fusable subtrees with >= 2 stages, outermost first."""
    found: List[FusedGraph] = []

    def visit(node: Dict) -> None:
        if _fusable(node, row_models, bound):
            stages: List[Dict] = []
            out = _emit(node, -1, stages, row_models, bound, device_of)
            sub = _subtree(node)
            devs = sorted({device_of(n) for n in sub})
            mixed_cpu = -1 in devs and len(devs) > 1
            if out >= 0 and out == len(stages) - 1 and len(stages) >= 2 and not mixed_cpu:
                found.append(FusedGraph(node["name"], stages, [n["name"] for n in sub], devs))
                return
        for c in node.get("children") or []:
            visit(c)

    visit(graph)
    return found


def build(C, fg: FusedGraph, in_cols: int = 0, split: int = 0):
    """Native GraphModel for a plan entry (raises if the stage widths disagree).
    ``split``: one stream per stage even on one GPU -- the multi-GPU code
    paths rehearsed on a single device: 1 = staged copies between stages (no
    peer access), 2 = direct cross-lane reads (xGMI peer access)."""
    return C.graph_model(fg.stages, in_cols, int(split))


def describe(fg: FusedGraph) -> str:
    parts = []
    for i, s in enumerate(fg.stages):
        src = ",".join("in" if j < 0 else f"s{j}" for j in s["inputs"])
        parts.append(f"s{i}={s['kind']}:{s['node']}@gpu{s['device']}({src})")
    return " ".join(parts)


def split_enabled(annotations: Optional[Dict[str, str]]) -> int:
    """``seldon.io/device-graph-split``: ``true`` builds fused graphs in split
    mode 1 (staged copies), ``peer`` in split mode 2 (direct cross-lane reads);
    see ``build``."""
    v = str((annotations or {}).get("seldon.io/device-graph-split", "")).lower()
    if v == "peer":
        return 2
    return 1 if v in ("1", "true", "yes", "on") else 0


def fusion_enabled(annotations: Optional[Dict[str, str]], default: bool = True) -> bool:
    v = (annotations or {}).get("seldon.io/device-graph")
    if v is None:
        return default
    return str(v).lower() in ("1", "true", "yes", "on")
