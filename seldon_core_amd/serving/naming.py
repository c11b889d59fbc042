"""Resource naming and graph helpers of the control plane (SURVEY A3/O11;
reference operator/api/v1alpha2/seldondeployment_types.go:29-190).

Kubernetes names are limited to 63 characters; long names become
``seldon-<md5>``.  Container / predictor hashes are short md5 prefixes over the
pod's (name, image) pairs, so a changed image yields a new deployment name
(rolling update).  The in-process engine uses these names for worker process
titles, status output and metric labels, so operators see the same identifiers
as with the reference operator.
"""
from __future__ import annotations

import hashlib
import re
from typing import Dict, Iterator, List, Optional

MAX_NAME = 63


def _md5(text: str) -> str:
    return hashlib.md5(text.encode()).hexdigest()


def _limit(name: str) -> str:
    return name if len(name) <= MAX_NAME else "seldon-" + _md5(name)


def container_hash(pod_spec: Dict) -> str:
    parts: List[str] = []
    for c in ((pod_spec or {}).get("spec") or {}).get("containers", []) or []:
        parts += [c.get("name", ""), c.get("image", "")]
    return _md5(":".join(parts) + ";")[:7]


def predictor_hash(predictor: Dict) -> str:
    return _md5(",".join(container_hash(ps) for ps in predictor.get("componentSpecs", []) or []) + ",")[:7]


def sdep_name(sdep: Dict) -> str:
    return _limit(sdep["spec"].get("name", "") + "-" + sdep.get("metadata", {}).get("name", ""))


def deployment_name(sdep: Dict, predictor: Dict, pod_spec: Optional[Dict] = None) -> str:
    meta_name = ((pod_spec or {}).get("metadata") or {}).get("name")
    if meta_name:
        return meta_name
    name = sdep["spec"].get("name", "") + "-" + predictor.get("name", "")
    if pod_spec is not None:
        name += "-" + container_hash(pod_spec)
    return _limit(name)


def explainer_deployment_name(sdep_name_: str, predictor: Dict) -> str:
    return _limit(f"{sdep_name_}-{predictor.get('name', '')}-explainer")


def service_orchestrator_name(sdep: Dict, predictor: Dict) -> str:
    return _limit(f"{sdep['spec'].get('name', '')}-{predictor.get('name', '')}-svc-orch-{predictor_hash(predictor)}")


def predictor_key(sdep: Dict, predictor: Dict) -> str:
    return _limit(f"{sdep.get('metadata', {}).get('name', '')}-{sdep['spec'].get('name', '')}-{predictor.get('name', '')}")


def _clean(name: str) -> str:
    return re.sub(r"[^-a-z0-9]", "-", name.lower())


def container_service_name(sdep: Dict, predictor: Dict, container: Dict) -> str:
    image = _clean(container.get("image", ""))
    name = f"{sdep['spec'].get('name', '')}-{predictor.get('name', '')}-{container.get('name', '')}"
    if image:
        name += "-" + image
    if len(name) <= MAX_NAME:
        return name
    name = f"seldon-{image}-{_md5(name)}"
    return name if len(name) <= MAX_NAME else "seldon-" + _md5(name)


def get_predictive_unit(unit: Dict, name: str) -> Optional[Dict]:
    if unit.get("name") == name:
        return unit
    for c in unit.get("children", []) or []:
        found = get_predictive_unit(c, name)
        if found is not None:
            return found
    return None


def get_engine_predictive_unit(unit: Dict) -> Optional[Dict]:
    """The node whose endpoint host is ``localhost`` (co-located with the engine)."""
    ep = unit.get("endpoint") or {}
    if (ep.get("service_host") or ep.get("serviceHost")) == "localhost":
        return unit
    for c in unit.get("children", []) or []:
        found = get_engine_predictive_unit(c)
        if found is not None:
            return found
    return None


def predictive_unit_list(unit: Dict) -> Iterator[Dict]:
    yield unit
    for c in unit.get("children", []) or []:
        yield from predictive_unit_list(c)
