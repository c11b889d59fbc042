"""SeldonDeployment / PredictorSpec handling on the Python side.

* loading (JSON / YAML file, dict, or base64 ``ENGINE_PREDICTOR`` env var as the
  reference engine does: engine/.../predictors/EnginePredictor.java:58-108),
* defaulting (reference operator webhook, operator/api/v1alpha2/
  seldondeployment_webhook.go:115-338: node type/implementation defaults,
  ``version`` label, per-container service ports from 9000),
* validation with the webhook's error messages (seldondeployment_webhook.go:345-411),
* graph helpers and a Graphviz renderer (reference notebooks/visualizer.py).

MI355X extension fields (ignored by the reference): ``graph.device`` (GPU
ordinal for a node, -1 = CPU) and ``graph.replicas`` (data-parallel GPU
replicas of a node).
"""
from __future__ import annotations

import base64
import copy
import json
import os
from pathlib import Path
from typing import Any, Dict, Iterator, List, Optional, Tuple, Union

BUILTIN_IMPLEMENTATIONS = {"SIMPLE_MODEL", "SIMPLE_ROUTER", "RANDOM_ABTEST", "AVERAGE_COMBINER"}
PREPACKAGED_SERVERS = {"SKLEARN_SERVER", "XGBOOST_SERVER", "TENSORFLOW_SERVER", "MLFLOW_SERVER"}
UNIT_TYPES = ["UNKNOWN_TYPE", "ROUTER", "COMBINER", "MODEL", "TRANSFORMER", "OUTPUT_TRANSFORMER"]
METHODS = ["TRANSFORM_INPUT", "TRANSFORM_OUTPUT", "ROUTE", "AGGREGATE", "SEND_FEEDBACK"]


class SpecError(ValueError):
    def __init__(self, errors: List[str]):
        self.errors = errors
        super().__init__("; ".join(errors))


def load_spec(spec: Union[str, Path, Dict, None] = None) -> Dict:
    """Load a SeldonDeployment or PredictorSpec."""
    if spec is None:
        env = os.environ.get("ENGINE_PREDICTOR")
        if env:
            return json.loads(base64.b64decode(env).decode())
        if os.path.exists("./deploymentdef.json"):
            return json.loads(Path("./deploymentdef.json").read_text())
        return default_predictor()
    if isinstance(spec, dict):
        return copy.deepcopy(spec)
    text = str(spec)
    if os.path.exists(text):
        text = Path(text).read_text()
    text = text.strip()
    if text.startswith("{"):
        return json.loads(text)
    import yaml

    return yaml.safe_load(text)


def default_predictor() -> Dict:
    """Graph used when no spec is given (EnginePredictor.java:122-141)."""
    return {"name": "basic-predictor", "componentSpecs": [{}],
            "graph": {"name": "basic-pu", "type": "MODEL", "implementation": "SIMPLE_MODEL"}}


def is_deployment(spec: Dict) -> bool:
    return isinstance(spec.get("spec"), dict) and "predictors" in spec["spec"]


def predictors(spec: Dict) -> List[Dict]:
    return spec["spec"]["predictors"] if is_deployment(spec) else [spec]


def select_predictor(spec: Dict, name: Optional[str] = None) -> Dict:
    preds = predictors(spec)
    if not preds:
        raise SpecError(["SeldonDeployment has no predictors"])
    if name:
        for p in preds:
            if p.get("name") == name:
                return p
        raise SpecError([f"predictor {name} not found"])
    return preds[0]


def is_shadow(predictor: Dict) -> bool:
    """Shadow predictor: receives a mirrored copy of every request, its response
    is discarded (reference ``seldon.io/ambassador-shadow``, ambassador.go:119-122;
    here per predictor via ``shadow: true`` or that annotation)."""
    if predictor.get("shadow") in (True, "true", "True"):
        return True
    ann = predictor.get("annotations") or {}
    return str(ann.get("seldon.io/shadow", ann.get("seldon.io/ambassador-shadow", ""))).lower() in ("1", "true")


def header_route(predictor: Dict, sdep: Optional[Dict] = None) -> Optional[Tuple[str, str, bool]]:
    """(header, value, is_regex) routing a request to this predictor: predictor
    annotations ``seldon.io/header`` / ``seldon.io/regex-header`` (or the
    reference's ``seldon.io/ambassador-header`` / ``-regex-header`` spelling),
    value "name:value" (ambassador.go:99-118)."""
    ann = predictor.get("annotations") or {}  # per predictor: a deployment-wide header would match them all
    for key, regex in (("seldon.io/header", False), ("seldon.io/regex-header", True),
                       ("seldon.io/ambassador-header", False), ("seldon.io/ambassador-regex-header", True)):
        v = ann.get(key)
        if v and ":" in v:
            name, _, value = v.partition(":")
            return name.strip(), value.strip(), regex
    return None


def iter_nodes(graph: Dict, parent: Optional[Dict] = None) -> Iterator[Tuple[Dict, Optional[Dict]]]:
    yield graph, parent
    for c in graph.get("children", []) or []:
        yield from iter_nodes(c, graph)


def find_node(graph: Dict, name: str) -> Optional[Dict]:
    for n, _ in iter_nodes(graph):
        if n.get("name") == name:
            return n
    return None


def containers(predictor: Dict) -> List[Dict]:
    out = []
    for ps in predictor.get("componentSpecs", []) or []:
        out.extend(((ps or {}).get("spec") or {}).get("containers", []) or [])
    return out


def container_for(predictor: Dict, name: str) -> Optional[Dict]:
    for c in containers(predictor):
        if c.get("name") == name:
            return c
    return None


def typed_parameters(node: Dict) -> Dict[str, Any]:
    """PREDICTIVE_UNIT_PARAMETERS typing (python/seldon_core/microservice.py:50-87)."""
    out: Dict[str, Any] = {}
    for p in node.get("parameters", []) or []:
        v, t = p.get("value"), p.get("type", "STRING")
        if t == "INT":
            v = int(v)
        elif t in ("FLOAT", "DOUBLE"):
            v = float(v)
        elif t == "BOOL":
            v = str(v).lower() in ("1", "true")
        out[p["name"]] = v
    return out


def apply_defaults(sdep: Dict, first_port: Optional[int] = None) -> Dict:
    """Operator defaulting webhook equivalent (returns a modified deep copy)."""
    sdep = copy.deepcopy(sdep)
    first = first_port or int(os.environ.get("PREDICTIVE_UNIT_SERVICE_PORT", "9000"))
    next_port = [first]
    port_map: Dict[str, int] = {}
    if is_deployment(sdep):
        sdep.setdefault("metadata", {}).setdefault("namespace", "default")
    namespace = sdep.get("metadata", {}).get("namespace", "default")
    for p in predictors(sdep):
        p.setdefault("labels", {}).setdefault("version", p.get("name", ""))
        for node, _ in iter_nodes(p["graph"]):
            node.setdefault("type", "UNKNOWN_TYPE")
            node.setdefault("implementation", "UNKNOWN_IMPLEMENTATION")
        for j, ps in enumerate(p.get("componentSpecs", []) or []):
            for c in ((ps or {}).get("spec") or {}).get("containers", []) or []:
                name = c.get("name", "")
                if name not in port_map:
                    port_map[name] = next_port[0]
                    next_port[0] += 1
                node = find_node(p["graph"], name)
                if node is None:
                    continue
                ep = node.setdefault("endpoint", {"type": "REST"})
                ep.setdefault("type", "REST")
                ep.setdefault("service_port", port_map[name])
                host = "localhost" if j == 0 else f"{sdep.get('metadata', {}).get('name', 'sdep')}-{p.get('name')}-{name}.{namespace}.svc.cluster.local."
                ep.setdefault("service_host", host)
                env = c.setdefault("env", [])
                if not any(e.get("name") == "PREDICTIVE_UNIT_SERVICE_PORT" for e in env):
                    env.append({"name": "PREDICTIVE_UNIT_SERVICE_PORT", "value": str(ep["service_port"])})
    return sdep


def validate(sdep: Dict, bound: Optional[set] = None, schema: bool = True) -> List[str]:
    """Structural checks against ``schema/seldondeployment.schema.json`` (what
    the API server enforces from the CRD's openAPIV3Schema) followed by the
    validating-webhook rules.  ``bound``: node names with an in-process
    implementation (count as having a container)."""
    bound = bound or set()
    errors: List[str] = []
    if schema:
        from .jsonschema import validate_schema

        errors = validate_schema(sdep if "spec" in sdep else {"spec": sdep})
        if errors:
            return errors
    preds = predictors(sdep)
    seen = set()
    for i, p in enumerate(preds):
        pname = p.get("name", "")
        if pname in seen:
            errors.append(f"spec.predictors[{i}]: Invalid value: \"{pname}\": Duplicate predictor name")
        seen.add(pname)
        if "graph" not in p:
            errors.append(f"spec.predictors[{i}].graph: Required value")
            continue
        for node, _ in iter_nodes(p["graph"]):
            impl = node.get("implementation", "UNKNOWN_IMPLEMENTATION")
            ntype = node.get("type", "UNKNOWN_TYPE")
            name = node.get("name", "")
            if impl == "UNKNOWN_IMPLEMENTATION":
                if container_for(p, name) is None and name not in bound:
                    errors.append(f"spec.predictors[{i}].graph: Invalid value: \"{name}\": Can't find container for Predictive Unit")
                if ntype == "UNKNOWN_TYPE" and not node.get("methods"):
                    errors.append(f"spec.predictors[{i}].graph: Invalid value: \"{name}\": Predictive Unit has no implementation methods defined. Change to a know type or add what methods it defines")
            elif impl in PREPACKAGED_SERVERS and not node.get("modelUri"):
                errors.append(f"spec.predictors[{i}].graph: Invalid value: \"{name}\": Predictive unit modelUri required when using standalone servers")
    live = [p for p in preds if not is_shadow(p)]
    traffic = sum(int(p.get("traffic", 0) or 0) for p in live)
    name = sdep.get("metadata", {}).get("name", "")
    if traffic != 100 and len(live) > 1:
        errors.append(f"spec: Invalid value: \"{name}\": Traffic must sum to 100 for multiple predictors")
    if 0 < traffic < 100 and len(live) == 1:
        errors.append(f"spec: Invalid value: \"{name}\": Traffic must sum be 100 for a single predictor when set")
    return errors


def to_dot(graph: Dict) -> str:
    """Graphviz rendering of a predictor graph (reference notebooks/visualizer.py)."""
    lines = ["digraph predictor {", "  rankdir=LR;"]
    for node, parent in iter_nodes(graph):
        label = f"{node['name']}\\n{node.get('type', '')} {node.get('implementation', '')}".strip()
        lines.append(f"  \"{node['name']}\" [shape=box,label=\"{label}\"];")
        if parent is not None:
            lines.append(f"  \"{parent['name']}\" -> \"{node['name']}\";")
    lines.append("}")
    return "\n".join(lines)


def encode_engine_predictor(predictor: Dict) -> str:
    """base64 ENGINE_PREDICTOR value (operator/controllers/controller_utils.go:23-30)."""
    p = copy.deepcopy(predictor)
    p["traffic"] = 0
    return base64.b64encode(json.dumps(p).encode()).decode()
