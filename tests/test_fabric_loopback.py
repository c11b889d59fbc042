"""Cross-GPU code paths on ONE GPU.

* Fabric: every rank of a rank-placed graph lives in this process on GPU 0
  over the loopback transport (csrc/parallel/fabric.h).  The front end's GPU
  path (PeerRowModel::launch on per-link streams, the fan-out gather + combine
  kernel) and the worker's (PeerServer::loop: K slots chained across X /
  compute / Y streams) run for real; only the byte mover differs from RCCL.
* Device graph: split mode gives every stage its own stream and event chain
  and forces the staged-copy branch -- what a graph spread over GPUs without
  peer access runs -- under concurrent slots and buffer growth.

Every answer is compared with a CPU oracle (scikit-learn / the host graph
walk) at 1e-12.  Reference behaviour: PredictiveUnitBean.java:159-183
(fan-out / fan-in), InternalPredictionService.java:186-453 (the hop)."""
import json
import threading
import time

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression
from seldon_core_amd.parallel.fabric import loopback_fabrics, serve_peer

pytestmark = pytest.mark.gpu


def _spec(graph, annotations=None):
    s = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}], "graph": graph}
    if annotations:
        s["annotations"] = annotations
    return s


def _rows(rng, n):
    return rng.normal(loc=4.0, scale=1.5, size=(n, 4))


class _Ranks:
    """Rank 0's Deployment + the workers' PeerServers, all on GPU 0."""

    def __init__(self, spec, comps, world, **dep_kw):
        self.fabrics = loopback_fabrics(world, 0)
        self.servers = [serve_peer(spec, f, comps) for f in self.fabrics[1:]]
        dep_kw.setdefault("fuse", False)  # one unit per node, as the rank-placed bench graphs
        self.dep = sca.Deployment(spec, components=comps, device=0, fabric=self.fabrics[0], **dep_kw)

    def close(self):
        self.dep.close()  # stops the workers' loops
        for s in self.servers:
            s.join()
        for f in self.fabrics:
            f.close()


def test_loopback_remote_model_matches_sklearn():
    lr = iris_logistic_regression()
    spec = _spec({"name": "m", "type": "MODEL", "rank": 1})
    r = _Ranks(spec, {"m": lr}, 2)
    try:
        assert r.fabrics[0].transport == "loopback" and r.fabrics[0].gpu
        assert r.dep.engine.unit_kind("m") == "gpu:rccl_peer"
        rng = np.random.default_rng(0)
        worst, rows = 0.0, 0
        for i in range(60):  # 1..300-row batches: the worker's slot buffers grow
            X = _rows(rng, 1 + (i * 37) % 300)
            got = np.asarray(r.dep.predict({"data": {"ndarray": X.tolist()}})["data"]["ndarray"])
            worst = max(worst, float(np.abs(got - lr.predict_proba(X)).max()))
            rows += len(X)
        assert worst < 1e-12, worst
    finally:
        r.close()
    srv = r.servers[0]
    assert srv.error() == "" and srv.rows == rows and srv.host_syncs >= 1


def test_loopback_concurrent_load_keeps_batches_in_flight(monkeypatch):
    """16 client threads through the batcher: the worker holds >= 2 batches
    in flight (its GPU model is slowed by a delay kernel so they pile up)."""
    monkeypatch.setenv("SCA_FABRIC_WORKER_DELAY_US", "300")
    monkeypatch.setenv("SCA_FABRIC_SLOTS", "4")
    lr = iris_logistic_regression()
    spec = _spec({"name": "m", "type": "MODEL", "rank": 1})
    r = _Ranks(spec, {"m": lr}, 2, batcher={"slots": 4, "max_batch": 64})
    errors, worst = [], [0.0]
    lock = threading.Lock()

    def client(t):
        rng = np.random.default_rng(100 + t)
        try:
            for i in range(40):
                X = _rows(rng, 1 + (i + t) % 3)
                got = np.asarray(r.dep.predict({"data": {"ndarray": X.tolist()}})["data"]["ndarray"])
                with lock:
                    worst[0] = max(worst[0], float(np.abs(got - lr.predict_proba(X)).max()))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    try:
        th = [threading.Thread(target=client, args=(t,)) for t in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        st = r.dep.batcher_stats()["m"]
    finally:
        r.close()
    srv = r.servers[0]
    assert errors == [] and worst[0] < 1e-12, (errors[:3], worst[0])
    assert srv.error() == "" and srv.slots == 4
    assert srv.max_inflight >= 2, srv.max_inflight
    assert st["batches"] < 16 * 40  # requests were batched on the way


def test_loopback_fanout_combiner_gathers_every_rank():
    """One PeerRowModel over ranks 1 and 2 (broadcast X, gather both replies,
    average on rank 0's GPU) behind a batcher, and the engine-level combiner
    over m1@rank1 + m2@rank2 + m0 local."""
    lr = iris_logistic_regression()
    C = sca.native()
    kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(3)]
    spec = _spec({"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids})
    comps = {f"m{r}": lr for r in range(3)}
    r = _Ranks(spec, comps, 3)
    try:
        rng = np.random.default_rng(1)
        for i in range(20):
            X = _rows(rng, 1 + i * 7)
            got = np.asarray(r.dep.predict({"data": {"ndarray": X.tolist()}})["data"]["ndarray"])
            np.testing.assert_allclose(got, lr.predict_proba(X), rtol=0, atol=1e-12)
        kinds = {n: r.dep.engine.unit_kind(n) for n in ("m0", "m1", "m2")}
        assert kinds == {"m0": "gpu:linear", "m1": "gpu:rccl_peer", "m2": "gpu:rccl_peer"}, kinds
    finally:
        r.close()
    for s in r.servers:
        assert s.error() == "" and s.batches > 0

    # the multi-peer model: one batch -> both workers -> combine kernel
    fabrics = loopback_fabrics(3, 0)
    spec2 = _spec({"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
                   "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]})
    servers = [serve_peer(spec2, f, {"a": lr, "b": lr}) for f in fabrics[1:]]
    unit = C.BatchedUnit(C.peer_row_model(fabrics[0], [1, 2], 0, 4, 3), 0, slots=2)
    try:
        for n in (1, 5, 64, 200):
            X = _rows(rng, n)
            np.testing.assert_allclose(unit.run(X), lr.predict_proba(X), rtol=0, atol=1e-12)
    finally:
        unit.stop()
        fabrics[0].stop_peers()
        for s in servers:
            s.join()
        for f in fabrics:
            f.close()
    for s in servers:
        assert s.error() == "" and s.rows == 1 + 5 + 64 + 200


def test_loopback_links_issue_concurrently(monkeypatch):
    """Two units, one per worker (the arms of an A/B test): each worker
    answers a batch only after D ms, so a front end that serialised its links
    would take 2 * N * D; per-link streams and mutexes take about N * D."""
    D_us, N = 20000, 12
    monkeypatch.setenv("SCA_FABRIC_WORKER_HOST_DELAY_US", str(D_us))
    lr = iris_logistic_regression()
    C = sca.native()
    fabrics = loopback_fabrics(3, 0)
    spec = _spec({"name": "ab", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
                  "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
                  "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]})
    servers = [serve_peer(spec, f, {"a": lr, "b": lr}) for f in fabrics[1:]]
    units = [C.BatchedUnit(C.peer_row_model(fabrics[0], [p], 0, 4, 3), 0, slots=1) for p in (1, 2)]
    rng = np.random.default_rng(3)
    X = _rows(rng, 2)
    ref = lr.predict_proba(X)
    outs, errs = [], []

    def drive(u):
        try:
            for _ in range(N):
                outs.append(float(np.abs(u.run(X) - ref).max()))
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    try:
        t0 = time.perf_counter()
        th = [threading.Thread(target=drive, args=(u,)) for u in units]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
    finally:
        for u in units:
            u.stop()
        fabrics[0].stop_peers()
        for s in servers:
            s.join()
        for f in fabrics:
            f.close()
    assert errs == [] and len(outs) == 2 * N and max(outs) < 1e-12
    serial = 2 * N * D_us * 1e-6
    print(json.dumps({"wall_s": round(wall, 4), "serialised_s": serial}))
    assert wall < 0.75 * serial, (wall, serial)


# ------------------------------------------------------------ device graph
def _lin(C, rng, o, i, act=0):
    return C.linear_model(rng.normal(size=(o, i)), rng.normal(size=o), act)


GRAPHS = {
    "pipeline": {"name": "tout", "type": "OUTPUT_TRANSFORMER", "children": [
        {"name": "tin", "type": "TRANSFORMER", "children": [
            {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
                {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}]}]}]},
    "combiner": {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
        {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}, {"name": "m3", "type": "MODEL"}]},
}


@pytest.mark.parametrize("mode", ["true", "peer", "peer-fault"])
@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_split_device_graph_matches_cpu_under_concurrency(name, mode, monkeypatch):
    """Split lanes on one GPU, 8 callers, 4 slots, buffer growth: "true" runs
    the staged-copy branch (GPUs without peer access), "peer" the direct
    cross-lane reads and the last lane's direct write into the caller's
    buffer (xGMI-connected GPUs, graph.cc launch_segments)."""
    C = sca.native()
    rng = np.random.default_rng(11)
    comps = {"tin": _lin(C, rng, 4, 4), "m1": _lin(C, rng, 3, 4, 1), "m2": _lin(C, rng, 3, 4, 1),
             "m3": _lin(C, rng, 3, 4, 1), "tout": _lin(C, rng, 2, 3)}
    if mode == "peer-fault":  # the start-up canary fails: the graph must fall back to staged copies
        monkeypatch.setenv("SCA_GRAPH_PEER_FAULT", "1")
    spec = _spec(GRAPHS[name], {"seldon.io/device-graph-split": mode.split("-")[0]})
    gpu = sca.Deployment(spec, components=comps, device=0, fuse=True, batcher={"slots": 4, "max_batch": 2048})
    cpu = sca.Deployment(spec, components=comps, device=-1, fuse=True)
    root = GRAPHS[name]["name"]
    try:
        info = C.graph_info(gpu.batched[root].model)
        assert info["split"] and info["stages"] >= 3, info
        assert info["peer_direct"] == (mode == "peer"), info
        assert info["split_mode"] == (1 if mode == "true" else 2), info
        # the canary runs for peer-direct graphs: the device against itself here
        assert info["peer_canary"] == ({} if mode == "true" else {"0->0": mode == "peer"}), info
        errors, worst = [], [0.0]
        lock = threading.Lock()

        def client(t):
            r = np.random.default_rng(t)
            try:
                # growth sequence per slot: 1 -> 1500 rows crosses every capacity doubling
                for n in (1, 3, 70, 129, 300, 700, 1500, 2, 65):
                    X = r.normal(size=(n, 4))
                    req = json.dumps({"data": {"tensor": {"shape": [n, 4], "values": X.ravel().tolist()}}})
                    a = np.array(gpu.predict(req)["data"]["tensor"]["values"])
                    b = np.array(cpu.predict(req)["data"]["tensor"]["values"])
                    with lock:
                        worst[0] = max(worst[0], float(np.max(np.abs(a - b) / (1e-300 + np.maximum(1.0, np.abs(b))))))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        th = [threading.Thread(target=client, args=(t,)) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert errors == [] and worst[0] < 1e-12, (errors[:3], worst[0])
        assert gpu.batcher_stats()[root]["batches"] > 0
    finally:
        gpu.close()
        cpu.close()
