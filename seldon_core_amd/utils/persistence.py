"""Component state persistence (reference python/seldon_core/persistence.py:12-85).

The reference pickles the whole user object into Redis under
``persistence_<deployment>_<predictor>_<unit>`` every ``push_frequency`` seconds
and restores it at start.  Here the backend is pluggable:

* ``file`` (default): ``$SELDON_PERSISTENCE_DIR/<key>.pkl`` (atomic rename),
* ``redis``: a minimal RESP client (GET/SET) against ``REDIS_SERVICE_HOST`` /
  ``REDIS_SERVICE_PORT`` -- no redis package needed.

Native units (routers, detectors) snapshot their state as JSON through
``Unit.snapshot()``; Python components are pickled like the reference.
"""
from __future__ import annotations

import logging
import os
import pickle
import socket
import threading
import time
from typing import Any, Callable, Dict, Optional

logger = logging.getLogger(__name__)

PRED_UNIT_ID = os.environ.get("PREDICTIVE_UNIT_ID", "0")
PREDICTOR_ID = os.environ.get("PREDICTOR_ID", "0")
DEPLOYMENT_ID = os.environ.get("SELDON_DEPLOYMENT_ID", "0")
DEFAULT_PUSH_FREQUENCY = 60


def state_key(deployment: str = DEPLOYMENT_ID, predictor: str = PREDICTOR_ID, unit: str = PRED_UNIT_ID) -> str:
    return f"persistence_{deployment}_{predictor}_{unit}"


def _default_dir() -> str:
    """Per-user state directory (never a shared world-writable path)."""
    base = os.environ.get("XDG_STATE_HOME") or os.path.join(os.path.expanduser("~"), ".local", "state")
    return os.path.join(base, "seldon-persistence")


class FileStore:
    """Snapshots are unpickled on restore, so only files this user owns, in a
    directory no one else can write, are ever read."""

    def __init__(self, root: Optional[str] = None):
        self.root = root or os.environ.get("SELDON_PERSISTENCE_DIR") or _default_dir()
        os.makedirs(self.root, mode=0o700, exist_ok=True)
        self._check_owned(self.root, directory=True)

    @staticmethod
    def _check_owned(path: str, directory: bool = False) -> None:
        st = os.stat(path)
        if st.st_uid != os.getuid():
            raise PermissionError(f"{path} is owned by uid {st.st_uid}, not the current user")
        if st.st_mode & 0o022:
            raise PermissionError(f"{path} is group/world-writable (mode {oct(st.st_mode & 0o777)})")

    def get(self, key: str) -> Optional[bytes]:
        p = os.path.join(self.root, key + ".pkl")
        if not os.path.exists(p):
            return None
        self._check_owned(p)
        with open(p, "rb") as f:
            return f.read()

    def set(self, key: str, value: bytes) -> None:
        p = os.path.join(self.root, key + ".pkl")
        tmp = p + ".tmp"
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "wb") as f:
            f.write(value)
        os.replace(tmp, p)


class RedisStore:
    """Tiny RESP2 client: enough for GET / SET of one blob."""

    def __init__(self, host: Optional[str] = None, port: Optional[int] = None, timeout: float = 5.0):
        self.host = host or os.environ.get("REDIS_SERVICE_HOST", "localhost")
        self.port = int(port or os.environ.get("REDIS_SERVICE_PORT", 6379))
        self.timeout = timeout

    def _cmd(self, *args: bytes) -> Any:
        payload = b"*%d\r\n" % len(args) + b"".join(b"$%d\r\n%s\r\n" % (len(a), a) for a in args)
        with socket.create_connection((self.host, self.port), timeout=self.timeout) as s:
            s.sendall(payload)
            f = s.makefile("rb")
            line = f.readline()
            kind, rest = line[:1], line[1:-2]
            if kind == b"+":
                return rest
            if kind == b"-":
                raise RuntimeError(rest.decode())
            if kind == b"$":
                n = int(rest)
                if n < 0:
                    return None
                data = f.read(n + 2)
                return data[:-2]
            if kind == b":":
                return int(rest)
            raise RuntimeError(f"unexpected redis reply {line!r}")

    def get(self, key: str) -> Optional[bytes]:
        return self._cmd(b"GET", key.encode())

    def set(self, key: str, value: bytes) -> None:
        self._cmd(b"SET", key.encode(), value)


def default_store():
    return RedisStore() if os.environ.get("SELDON_PERSISTENCE_BACKEND", "file") == "redis" else FileStore()


def restore(user_class: Callable, parameters: Dict[str, Any], store=None, key: Optional[str] = None):
    """Unpickle a previously persisted component or construct a fresh one."""
    store = store or default_store()
    key = key or state_key()
    blob = None
    try:
        blob = store.get(key)
    except Exception as e:  # store unreachable: start fresh like the reference
        logger.warning("persistence restore failed: %s", e)
    if blob:
        logger.info("Restoring saved model from %s", key)
        return pickle.loads(blob)
    return user_class(**parameters)


class Persister(threading.Thread):
    """Daemon thread snapshotting ``get_state()`` every ``push_frequency`` s."""

    def __init__(self, get_state: Callable[[], bytes], push_frequency: Optional[float] = None, store=None,
                 key: Optional[str] = None):
        super().__init__(daemon=True)
        self.get_state = get_state
        self.freq = float(push_frequency or DEFAULT_PUSH_FREQUENCY)
        self.store = store or default_store()
        self.key = key or state_key()
        self._halt = threading.Event()

    def run(self) -> None:
        while not self._halt.wait(self.freq):
            self.push()

    def push(self) -> None:
        try:
            self.store.set(self.key, self.get_state())
        except Exception as e:
            logger.warning("persistence push failed: %s", e)

    def stop(self) -> None:
        self._halt.set()


def persist(user_object: Any, push_frequency: Optional[float] = None, store=None, key: Optional[str] = None):
    t = Persister(lambda: pickle.dumps(user_object), push_frequency, store, key)
    t.start()
    return t
