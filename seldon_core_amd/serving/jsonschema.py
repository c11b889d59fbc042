"""Minimal JSON-Schema validator for the SeldonDeployment schema (SURVEY A4;
reference operator/config/crd/bases/machinelearning.seldon.io_seldondeployments.yaml,
which the API server enforces before the webhook runs).

The ``jsonschema`` package is not shipped here, so this implements the subset
the schema file uses -- ``type`` (incl. lists), ``enum``, ``properties``,
``required``, ``additionalProperties`` (bool or schema), ``items``,
``minItems``, ``minLength``, ``minimum`` / ``maximum``, ``pattern``, ``anyOf``
and local ``$ref`` (``#/$defs/...``) -- and reports errors in the Kubernetes
field-path style the API server uses (``spec.predictors[0].graph.type:
Unsupported value: "X": supported values: ...``).
"""
from __future__ import annotations

import json
import os
import re
from functools import lru_cache
from typing import Any, Dict, List

_SCHEMA_PATH = os.path.join(os.path.dirname(os.path.dirname(__file__)), "schema", "seldondeployment.schema.json")

_TYPES = {
    "object": lambda v: isinstance(v, dict),
    "array": lambda v: isinstance(v, list),
    "string": lambda v: isinstance(v, str),
    "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
    "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
    "boolean": lambda v: isinstance(v, bool),
    "null": lambda v: v is None,
}


@lru_cache(maxsize=1)
def seldon_deployment_schema() -> Dict[str, Any]:
    with open(_SCHEMA_PATH) as f:
        return json.load(f)


def _resolve(root: Dict, ref: str) -> Dict:
    if not ref.startswith("#/"):
        raise ValueError(f"only local $ref supported, got {ref}")
    node: Any = root
    for part in ref[2:].split("/"):
        node = node[part]
    return node


def _fmt(v: Any) -> str:
    return json.dumps(v) if not isinstance(v, str) else f'"{v}"'


def validate_instance(inst: Any, schema: Dict, root: Dict | None = None, path: str = "") -> List[str]:
    root = root if root is not None else schema
    errs: List[str] = []
    where = path or "<root>"
    if "$ref" in schema:
        return validate_instance(inst, _resolve(root, schema["$ref"]), root, path)
    if "anyOf" in schema:
        if not any(not validate_instance(inst, s, root, path) for s in schema["anyOf"]):
            errs.append(f"{where}: Invalid value: {_fmt(inst)}: does not match any allowed schema")
    if "enum" in schema and inst not in schema["enum"]:
        errs.append(f"{where}: Unsupported value: {_fmt(inst)}: supported values: "
                    + ", ".join(_fmt(e) for e in schema["enum"]))
        return errs
    t = schema.get("type")
    if t is not None:
        types = t if isinstance(t, list) else [t]
        if not any(_TYPES[x](inst) for x in types):
            got = type(inst).__name__
            errs.append(f"{where}: Invalid value: \"{got}\": {where} in body must be of type {' or '.join(types)}")
            return errs
    if isinstance(inst, dict):
        props = schema.get("properties", {})
        for k in schema.get("required", []):
            if k not in inst:
                errs.append(f"{path + '.' if path else ''}{k}: Required value")
        addl = schema.get("additionalProperties", True)
        for k, v in inst.items():
            sub = f"{path}.{k}" if path else k
            if k in props:
                errs.extend(validate_instance(v, props[k], root, sub))
            elif addl is False:
                errs.append(f"{sub}: Forbidden: unknown field \"{k}\"")
            elif isinstance(addl, dict):
                errs.extend(validate_instance(v, addl, root, sub))
    elif isinstance(inst, list):
        if len(inst) < schema.get("minItems", 0):
            errs.append(f"{where}: Invalid value: {len(inst)}: must have at least {schema['minItems']} items")
        if "items" in schema:
            for i, v in enumerate(inst):
                errs.extend(validate_instance(v, schema["items"], root, f"{path}[{i}]"))
    elif isinstance(inst, str):
        if len(inst) < schema.get("minLength", 0):
            errs.append(f"{where}: Invalid value: {_fmt(inst)}: must be at least {schema['minLength']} chars long")
        if "pattern" in schema and not re.search(schema["pattern"], inst):
            errs.append(f"{where}: Invalid value: {_fmt(inst)}: must match '{schema['pattern']}'")
    if _TYPES["number"](inst):
        if "minimum" in schema and inst < schema["minimum"]:
            errs.append(f"{where}: Invalid value: {inst}: must be greater than or equal to {schema['minimum']}")
        if "maximum" in schema and inst > schema["maximum"]:
            errs.append(f"{where}: Invalid value: {inst}: must be less than or equal to {schema['maximum']}")
    return errs


def validate_schema(sdep: Dict) -> List[str]:
    """Structural validation of a full SeldonDeployment document."""
    return validate_instance(sdep, seldon_deployment_schema())
