"""Opt-in anonymous usage reporting (the reference deploys a
spartakus volunteer, helm-charts/seldon-core-operator/templates/
deployment_seldon-spartakus-volunteer.yaml, with extensions from
configmap_seldon-spartakus-config.yaml).

Off by default.  When enabled (operator ``--usage-database URL``, chart
``usageMetrics.enabled``) the operator posts, once per ``period``, one
spartakus-format report: a random cluster id (fresh per process, as the
reference's ``/proc/sys/kernel/random/uuid``), the API server version, each
node's OS / kernel / architecture / capacity (``cpu``, ``memory``,
``amd.com/gpu``) and the extensions ``seldon-core-amd version`` and
``seldondeployments`` (count).  No names, namespaces, specs or payloads.
"""
from __future__ import annotations

import json
import logging
import threading
import time
import urllib.request
import uuid
from typing import Dict, List, Optional

from . import __version__

logger = logging.getLogger(__name__)

CAPACITY_KEYS = ("cpu", "memory", "amd.com/gpu")


def build_report(client, cluster_id: str) -> Dict:
    try:
        master = (client.get("/version") or {}).get("gitVersion", "")
    except Exception:  # noqa: BLE001 -- best effort, like spartakus
        master = ""
    nodes: List[Dict] = []
    for n in (client.get("/api/v1/nodes") or {}).get("items", []):
        info = (n.get("status") or {}).get("nodeInfo") or {}
        cap = (n.get("status") or {}).get("capacity") or {}
        nodes.append({"id": str(uuid.uuid5(uuid.NAMESPACE_OID, cluster_id + n["metadata"].get("uid", ""))),
                      "operatingSystem": info.get("operatingSystem", ""), "osImage": info.get("osImage", ""),
                      "kernelVersion": info.get("kernelVersion", ""), "architecture": info.get("architecture", ""),
                      "kubeletVersion": info.get("kubeletVersion", ""),
                      "capacity": [{"resource": k, "value": str(cap[k])} for k in CAPACITY_KEYS if k in cap]})
    from .operator import _sdep_path

    try:
        n_sdep = len((client.get(_sdep_path(None)) or {}).get("items", []))
    except Exception:  # noqa: BLE001
        n_sdep = 0
    return {"version": "v1", "timestamp": str(int(time.time() * 1e9)), "clusterID": cluster_id,
            "masterVersion": master, "nodes": nodes,
            "extensions": [{"name": "seldon-core-amd version", "value": __version__},
                           {"name": "seldondeployments", "value": str(n_sdep)}]}


def send_report(database: str, report: Dict, timeout: float = 10.0) -> int:
    req = urllib.request.Request(database.rstrip("/") + "/", data=json.dumps(report).encode(),
                                 headers={"Content-Type": "application/json"}, method="POST")
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status


class UsageReporter:
    def __init__(self, client, database: str, period: float = 24 * 3600.0):
        self.client = client
        self.database = database
        self.period = period
        self.cluster_id = str(uuid.uuid4())
        self.sent = 0
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def report_once(self) -> bool:
        try:
            send_report(self.database, build_report(self.client, self.cluster_id))
            self.sent += 1
            return True
        except OSError as e:
            logger.info("usage report not sent: %s", e)
            return False

    def start(self) -> "UsageReporter":
        def loop():
            while not self._stop.is_set():
                self.report_once()
                self._stop.wait(self.period)

        self._th = threading.Thread(target=loop, daemon=True, name="usage-report")
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
