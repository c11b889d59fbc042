"""Engine configuration: one object built from defaults, the downward-API
annotations file, the spec's annotations, the environment and CLI flags
(later sources win).

Reference sources it replaces:

* ``engine/src/main/resources/application.properties`` -- ports, logging
  switches (``SELDON_LOG_REQUESTS``, ``SELDON_LOG_RESPONSES``,
  ``SELDON_LOG_FEEDBACK_REQUESTS``, ``SELDON_LOG_MESSAGES_EXTERNALLY``,
  ``SELDON_MESSAGE_LOGGING_SERVICE``, ``SELDON_LOG_MESSAGE_TYPE``,
  ``DEPLOYMENT_NAMESPACE``),
* ``config/CustomizationBean.java:27-49`` (``ENGINE_SERVER_PORT``),
  ``grpc/SeldonGrpcServer.java:55`` (``ENGINE_SERVER_GRPC_PORT``),
  ``config/TomcatConfig.java:45-84`` (admin port ``server.additionalPorts``),
* ``config/AnnotationsConfig.java:26-79`` (``/etc/podinfo/annotations``),
* ``predictors/EnginePredictor.java:58-108`` (``ENGINE_PREDICTOR``,
  ``DEPLOYMENT_NAME``), ``tracing/TracingProvider.java:25-40`` (``TRACING``).
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field
from typing import Dict, Mapping, Optional

ANNOTATIONS_FILE = "/etc/podinfo/annotations"


def _bool(v) -> bool:
    return str(v).strip().lower() in ("1", "true", "yes", "on")


def read_annotations(path: str = ANNOTATIONS_FILE) -> Dict[str, str]:
    """``key="value"`` lines (k8s downward API volume)."""
    out: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                line = line.strip()
                if "=" not in line:
                    continue
                k, _, v = line.partition("=")
                v = v.strip()
                if len(v) >= 2 and v[0] == v[-1] == '"':
                    v = v[1:-1].encode().decode("unicode_escape")
                out[k.strip()] = v
    except OSError:
        pass
    return out


@dataclass
class EngineConfig:
    http_port: int = 8000
    grpc_port: int = 5001
    admin_port: Optional[int] = 8082
    host: str = "0.0.0.0"
    threads: int = 4
    grpc_threads: Optional[int] = None
    deployment_name: str = "None"
    deployment_name_env: str = ""
    deployment_namespace: str = ""
    log_requests: bool = False
    log_responses: bool = False
    log_feedback: bool = False
    log_messages_externally: bool = False
    message_logging_service: str = ""
    message_type: str = "seldon.message.pair"
    tracing: bool = False
    drain_seconds: float = 20.0          # App.java:39-107 waits <= 20 s for the pool to drain
    grpc_max_message_size: Optional[int] = None
    annotations: Dict[str, str] = field(default_factory=dict)

    @classmethod
    def resolve(cls, env: Optional[Mapping[str, str]] = None, spec_annotations: Optional[Mapping[str, str]] = None,
                annotations_file: str = ANNOTATIONS_FILE, **overrides) -> "EngineConfig":
        env = os.environ if env is None else env
        c = cls()
        ann = read_annotations(annotations_file)
        ann.update(spec_annotations or {})
        c.annotations = ann
        if "seldon.io/grpc-max-message-size" in ann:
            c.grpc_max_message_size = int(ann["seldon.io/grpc-max-message-size"])
        if "seldon.io/engine-drain-seconds" in ann:
            c.drain_seconds = float(ann["seldon.io/engine-drain-seconds"])
        if "ENGINE_SERVER_PORT" in env:
            c.http_port = int(env["ENGINE_SERVER_PORT"])
        if "ENGINE_SERVER_GRPC_PORT" in env:
            c.grpc_port = int(env["ENGINE_SERVER_GRPC_PORT"])
        if "ENGINE_ADMIN_PORT" in env:
            c.admin_port = int(env["ENGINE_ADMIN_PORT"]) or None
        if env.get("DEPLOYMENT_NAME"):
            c.deployment_name = c.deployment_name_env = env["DEPLOYMENT_NAME"]
        c.deployment_namespace = env.get("DEPLOYMENT_NAMESPACE", c.deployment_namespace)
        c.log_requests = _bool(env.get("SELDON_LOG_REQUESTS", c.log_requests))
        c.log_responses = _bool(env.get("SELDON_LOG_RESPONSES", c.log_responses))
        c.log_feedback = _bool(env.get("SELDON_LOG_FEEDBACK_REQUESTS", c.log_feedback))
        c.log_messages_externally = _bool(env.get("SELDON_LOG_MESSAGES_EXTERNALLY", c.log_messages_externally))
        ns = c.deployment_namespace or "default"
        c.message_logging_service = env.get("SELDON_MESSAGE_LOGGING_SERVICE",
                                            f"http://default-broker.{ns}.svc.cluster.local")
        c.message_type = env.get("SELDON_LOG_MESSAGE_TYPE", c.message_type)
        c.tracing = _bool(env.get("TRACING", c.tracing))
        for k, v in overrides.items():
            if v is None:
                continue
            if not hasattr(c, k):
                raise TypeError(f"unknown engine config key {k}")
            setattr(c, k, v)
        return c

    def engine_kwargs(self) -> Dict:
        """Keyword arguments for the native ``Engine`` constructor."""
        return dict(log_requests=self.log_requests, log_responses=self.log_responses, log_feedback=self.log_feedback,
                    message_logging_service=self.message_logging_service,
                    log_messages_externally=self.log_messages_externally, message_type=self.message_type,
                    deployment_name_env=self.deployment_name_env, deployment_namespace=self.deployment_namespace)

    def to_dict(self) -> Dict:
        return asdict(self)
