"""Engine process lifecycle and ops features: config precedence, CloudEvents
request logging, graceful drain, multi-process replica supervisor.

Reference: engine/.../service/PredictionService.java:98-191 (logging),
App.java:39-107 (drain), config/AnnotationsConfig.java:26-79 (annotations file),
application.properties (env switches)."""
import http.server
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request

import pytest

import seldon_core_amd as sca
from seldon_core_amd.serving.config import EngineConfig, read_annotations

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    from portutil import free_port

    return free_port()


def test_config_precedence(tmp_path):
    ann = tmp_path / "annotations"
    ann.write_text('seldon.io/grpc-max-message-size="1000"\nseldon.io/engine-drain-seconds="3"\nother="x"\n')
    assert read_annotations(str(ann))["other"] == "x"
    env = {"ENGINE_SERVER_PORT": "9100", "SELDON_LOG_REQUESTS": "true", "DEPLOYMENT_NAME": "dep",
           "DEPLOYMENT_NAMESPACE": "ns"}
    c = EngineConfig.resolve(env=env, spec_annotations={"seldon.io/engine-drain-seconds": "5"},
                             annotations_file=str(ann), grpc_port=7000)
    assert c.http_port == 9100 and c.grpc_port == 7000
    assert c.grpc_max_message_size == 1000
    assert c.drain_seconds == 5.0  # spec annotation beats the file
    assert c.log_requests and not c.log_responses
    assert c.message_logging_service == "http://default-broker.ns.svc.cluster.local"
    assert c.deployment_name == "dep" and c.deployment_namespace == "ns"


class _Sink(http.server.BaseHTTPRequestHandler):
    got = []

    def do_POST(self):
        n = int(self.headers["Content-Length"])
        _Sink.got.append((dict(self.headers), json.loads(self.rfile.read(n))))
        self.send_response(200)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


def test_cloudevents_pair_logging():
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Sink)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    _Sink.got.clear()
    try:
        cfg = EngineConfig.resolve(env={"SELDON_LOG_MESSAGES_EXTERNALLY": "true", "DEPLOYMENT_NAME": "mydep",
                                        "DEPLOYMENT_NAMESPACE": "prod",
                                        "SELDON_MESSAGE_LOGGING_SERVICE": f"http://127.0.0.1:{srv.server_port}/"},
                                   annotations_file="/nonexistent")
        dep = sca.Deployment(None, device=-1, config=cfg)
        try:
            out = dep.predict({"meta": {"puid": "p123"}, "data": {"ndarray": [[1.0, 2.0]]}})
            assert out["meta"]["puid"] == "p123"
            dep.engine.flush_message_log()
            assert dep.engine.message_log_stats()["sent"] == 1
        finally:
            dep.close()
        headers, body = _Sink.got[0]
        h = {k.lower(): v for k, v in headers.items()}
        assert h["ce-specversion"] == "0.2" and h["ce-type"] == "seldon.message.pair"
        assert h["ce-eventid"] == "p123" and h["ce-source"] == "application/json"
        assert body["sdepName"] == "mydep" and body["namespace"] == "prod"
        assert body["request"]["data"]["ndarray"] == [[1.0, 2.0]] and "date" in body["request"]
        assert body["response"]["data"]["tensor"]["values"] == [0.1, 0.9, 0.5] and "date" in body["response"]
    finally:
        srv.shutdown()


def test_stdout_request_logging(capfd):
    cfg = EngineConfig.resolve(env={"SELDON_LOG_REQUESTS": "1", "SELDON_LOG_RESPONSES": "1",
                                    "SELDON_LOG_FEEDBACK_REQUESTS": "1"}, annotations_file="/nonexistent")
    dep = sca.Deployment(None, device=-1, config=cfg)
    try:
        req = {"meta": {"puid": "zz"}, "data": {"ndarray": [[1.0]]}}
        out = dep.predict(req)
        dep.feedback({"request": req, "response": out, "reward": 1.0})
        dep.engine.flush_message_log()
    finally:
        dep.close()
    lines = [json.loads(l) for l in capfd.readouterr().out.splitlines() if l.startswith("{")]
    assert lines[0]["meta"]["puid"] == "zz" and "ndarray" in lines[0]["data"]
    assert "tensor" in lines[1]["data"]
    assert lines[2]["reward"] == 1.0


def test_drain_waits_for_inflight():
    class Slow:
        def predict(self, X, names):
            time.sleep(0.3)
            return X

    spec = {"name": "p", "graph": {"name": "m", "type": "MODEL"}, "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, components={"m": Slow()}, device=-1)
    h = dep.serve(http_port=0, grpc_port=None, threads=2, host="127.0.0.1")
    port = h.http_port
    result = {}

    def call():
        req = urllib.request.Request(f"http://127.0.0.1:{port}/api/v0.1/predictions",
                                     data=json.dumps({"data": {"ndarray": [[1.0]]}}).encode(),
                                     headers={"Content-Type": "application/json"})
        result["body"] = json.loads(urllib.request.urlopen(req, timeout=10).read())

    t = threading.Thread(target=call)
    t.start()
    time.sleep(0.1)
    assert dep.engine.inflight() == 1
    assert h.drain(5.0) is True
    t.join()
    assert result["body"]["data"]["ndarray"] == [[1.0]]
    dep.close()


def _wait_ready(port, timeout=90):
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            if urllib.request.urlopen(f"http://127.0.0.1:{port}/ready", timeout=1).status == 200:
                return True
        except Exception:
            time.sleep(0.2)
    return False


def test_supervisor_two_workers_share_port():
    hp, gp = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--gpus", "2", "--device", "-1",
                          "--http-port", str(hp), "--grpc-port", str(gp), "--admin-port", "0", "--threads", "1",
                          "--log-level", "WARNING"], env=env, cwd=ROOT, start_new_session=True)
    try:
        assert _wait_ready(hp), "engine did not become ready"
        for _ in range(20):
            req = urllib.request.Request(f"http://127.0.0.1:{hp}/api/v0.1/predictions",
                                         data=b'{"data":{"ndarray":[[1.0]]}}',
                                         headers={"Content-Type": "application/json", "Connection": "close"})
            out = json.loads(urllib.request.urlopen(req, timeout=5).read())
            assert out["data"]["tensor"]["values"] == [0.1, 0.9, 0.5]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 0
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


def test_native_tracing_spans(tmp_path):
    trace_file = tmp_path / "spans.jsonl"
    os.environ["SELDON_TRACE_FILE"] = str(trace_file)
    try:
        cfg = EngineConfig.resolve(env={"TRACING": "1"}, annotations_file="/nonexistent")
        spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
                "graph": {"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
                          "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
                          "children": [{"name": "a", "type": "MODEL", "implementation": "SIMPLE_MODEL"},
                                       {"name": "b", "type": "MODEL", "implementation": "SIMPLE_MODEL"}]}}
        dep = sca.Deployment(spec, device=-1, config=cfg)
        out = dep.predict({"meta": {"puid": "tr1"}, "data": {"ndarray": [[1.0]]}})
        dep.close()  # flushes the exporter
    finally:
        del os.environ["SELDON_TRACE_FILE"]
    spans = [json.loads(l) for l in trace_file.read_text().splitlines()]
    root = [s for s in spans if s["name"] == "predictions"]
    assert len(root) == 1 and root[0]["tags"]["seldon.puid"] == "tr1"
    kids = [s for s in spans if s.get("parentId") == root[0]["id"]]
    names = {s["name"] for s in kids}
    branch = "a" if out["meta"]["routing"]["ab"] == 0 else "b"
    assert names == {"ab:route", f"{branch}:predict"}
    assert all(s["traceId"] == root[0]["traceId"] for s in kids)
    assert all(s["localEndpoint"]["serviceName"] == "seldon-svc-orch" for s in spans)


def test_rolling_update_swaps_model_version_without_failed_requests(tmp_path):
    """SIGHUP to the supervisor = rolling update (the reference's
    testing/scripts/test_rolling_updates.py with fixed-model images v1/v2):
    while clients keep sending, every worker is replaced by one built from the
    new spec, no request fails (beyond the reference's connect retries), every
    answer is v1 or v2, and the deployment ends on v2."""
    (tmp_path / "fixed_model.py").write_text(
        "class FixedModel:\n"
        "    def __init__(self, version='1'):\n"
        "        self.v = float(version)\n"
        "    def predict(self, X, names=None, meta=None):\n"
        "        return [[self.v] * 4 for _ in range(len(X))]\n")

    def write_spec(version):
        spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
                "graph": {"name": "m", "type": "MODEL",
                          "parameters": [{"name": "version", "value": str(version), "type": "STRING"}]}}
        (tmp_path / "spec.json").write_text(json.dumps(spec))

    write_spec(1)
    hp, gp = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{tmp_path}")
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--spec", str(tmp_path / "spec.json"),
                          "--gpus", "2", "--device", "-1", "--component", "m=fixed_model.FixedModel",
                          "--http-port", str(hp), "--grpc-port", str(gp), "--admin-port", "0", "--threads", "1",
                          "--log-level", "WARNING"], env=env, cwd=ROOT, start_new_session=True)
    seen, failed = [], []
    stop = threading.Event()

    def client():
        while not stop.is_set():
            for attempt in range(4):  # connect retries, as the reference's e2e helpers do
                try:
                    req = urllib.request.Request(f"http://127.0.0.1:{hp}/api/v0.1/predictions",
                                                 data=b'{"data":{"ndarray":[[1.0, 2.0]]}}',
                                                 headers={"Content-Type": "application/json", "Connection": "close"})
                    out = json.loads(urllib.request.urlopen(req, timeout=10).read())
                    seen.append(out["data"]["ndarray"][0][0])
                    break
                except Exception as e:  # noqa: BLE001
                    if attempt == 3:
                        failed.append(repr(e))
                    time.sleep(0.05)

    try:
        assert _wait_ready(hp), "engine did not become ready"
        th = [threading.Thread(target=client) for _ in range(3)]
        for t in th:
            t.start()
        time.sleep(1.0)
        assert seen and set(seen) == {1.0}
        write_spec(2)
        p.send_signal(signal.SIGHUP)
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline and not (len(seen) > 30 and set(seen[-30:]) == {2.0}):
            time.sleep(0.2)
        stop.set()
        for t in th:
            t.join(timeout=30)
        assert not failed, failed[:5]
        assert set(seen) <= {1.0, 2.0}
        assert set(seen[-30:]) == {2.0}, seen[-40:]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 0
    finally:
        stop.set()
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


def _pgroup_alive(pgid):
    try:
        os.killpg(pgid, 0)
        return True
    except ProcessLookupError:
        return False


def test_sigterm_during_rollout_stops_the_new_worker(tmp_path):
    """SIGTERM while a rollout waits for its new worker: the
    supervisor signals the not-yet-swapped-in worker too and exits; no
    process of the group outlives it."""
    (tmp_path / "slow_model.py").write_text(
        "import time\n"
        "class SlowModel:\n"
        "    def __init__(self, version='1'):\n"
        "        self.v = float(version)\n"
        "        if self.v > 1:\n"
        "            time.sleep(4.0)\n"
        "    def predict(self, X, names=None, meta=None):\n"
        "        return [[self.v] for _ in range(len(X))]\n")

    def write_spec(version):
        spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
                "graph": {"name": "m", "type": "MODEL",
                          "parameters": [{"name": "version", "value": str(version), "type": "STRING"}]}}
        (tmp_path / "spec.json").write_text(json.dumps(spec))

    write_spec(1)
    hp, gp = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=f"{ROOT}:{tmp_path}")
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--spec", str(tmp_path / "spec.json"),
                          "--gpus", "1", "--supervise", "--device", "-1", "--component", "m=slow_model.SlowModel",
                          "--http-port", str(hp), "--grpc-port", str(gp), "--admin-port", "0", "--threads", "1",
                          "--log-level", "WARNING"], env=env, cwd=ROOT, start_new_session=True)
    try:
        assert _wait_ready(hp), "engine did not become ready"
        write_spec(2)
        p.send_signal(signal.SIGHUP)
        time.sleep(1.5)  # the new worker is still in its 4 s __init__
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 0
        deadline = time.monotonic() + 20
        while _pgroup_alive(p.pid) and time.monotonic() < deadline:
            time.sleep(0.1)
        assert not _pgroup_alive(p.pid), "a worker outlived the supervisor"
    finally:
        if _pgroup_alive(p.pid):
            os.killpg(p.pid, signal.SIGKILL)
        if p.poll() is None:
            p.wait()


def test_single_worker_survives_sighup():
    """Without a supervisor SIGHUP is logged and ignored (its default action
    would kill the only serving process)."""
    hp, gp = _free_port(), _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("SCA_WORKER_RANK", None)
    p = subprocess.Popen([sys.executable, "-m", "seldon_core_amd.serve", "--gpus", "1", "--device", "-1",
                          "--http-port", str(hp), "--grpc-port", str(gp), "--admin-port", "0", "--threads", "1",
                          "--log-level", "WARNING"], env=env, cwd=ROOT, start_new_session=True)
    try:
        assert _wait_ready(hp), "engine did not become ready"
        p.send_signal(signal.SIGHUP)
        time.sleep(0.5)
        assert p.poll() is None
        assert _wait_ready(hp)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 0
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
