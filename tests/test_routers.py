"""Bandit routers: statistics (reference components/routers/epsilon-greedy/
test_EpsilonGreedy.py:21-25), feedback learning, persistence, and the
router inside a MAB graph with feedback through the engine."""
import json

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components.routers import EpsilonGreedy, ThompsonSampling


def test_eg_route_statistics_cpu():
    r = EpsilonGreedy(n_branches=3, epsilon=0.2, best_branch=1, seed=1)
    n = 20000
    routes = [r.route(None, None) for _ in range(n)]
    p_best = sum(1 for x in routes if x == 1) / n
    assert abs(p_best - 0.8) <= 0.02


def test_eg_feedback_moves_best_branch():
    r = EpsilonGreedy(n_branches=3, epsilon=0.1, best_branch=0, seed=3)
    X = np.ones((10, 2))
    r.send_feedback(X, [], 2, 0.9, None)
    r.send_feedback(X, [], 0, 0.1, None)
    assert r.best_branch == 2
    assert r.branch_values[2] == pytest.approx(0.9)
    st = r.state()
    assert st["success"] == [1, 0, 9] and st["tries"] == [10, 0, 10]


def test_ts_learns():
    r = ThompsonSampling(n_branches=2, seed=5)
    X = np.ones((50, 1))
    for _ in range(10):
        r.send_feedback(X, [], 1, 1.0, None)
        r.send_feedback(X, [], 0, 0.0, None)
    picks = [r.route(None, None) for _ in range(500)]
    assert np.mean(picks) > 0.98


def test_router_snapshot_restore():
    r = EpsilonGreedy(n_branches=4, epsilon=0.1, best_branch=0, seed=1)
    r.send_feedback(np.ones((4, 1)), [], 3, 1.0, None)
    snap = r.model.snapshot()
    r2 = EpsilonGreedy(n_branches=4, epsilon=0.1, best_branch=0, seed=9)
    r2.model.restore(snap)
    assert r2.best_branch == 3 and r2.state()["success"] == r.state()["success"]


def _mab_deployment(device, n=4, kind="EPSILON_GREEDY", route_on=None):
    class Const:
        def __init__(self, v):
            self.v = v

        def predict(self, X, names):
            return np.full((X.shape[0], 1), float(self.v))

    children = [{"name": f"m{i}", "type": "MODEL"} for i in range(n)]
    params = [{"name": "n_branches", "value": str(n), "type": "INT"},
              {"name": "seed", "value": "7", "type": "INT"}]
    if kind == "EPSILON_GREEDY":
        params += [{"name": "epsilon", "value": "0.2", "type": "FLOAT"},
                   {"name": "best_branch", "value": "0", "type": "INT"}]
    if route_on:
        params += [{"name": "route_on", "value": route_on, "type": "STRING"}]
    spec = {"name": "mab", "graph": {"name": "router", "type": "ROUTER", "implementation": kind,
                                     "parameters": params, "children": children}}
    return sca.Deployment(spec, components={f"m{i}": Const(i) for i in range(n)}, device=device)


@pytest.mark.parametrize("kind", ["EPSILON_GREEDY", "THOMPSON_SAMPLING"])
def test_mab_graph_with_feedback_cpu(kind):
    d = _mab_deployment(-1, kind=kind)
    assert d.engine.unit_kind("router").startswith("cpu:")
    # reward only branch 3
    for _ in range(300):
        out = d.predict({"data": {"ndarray": [[1.0, 2.0]]}})
        b = out["meta"]["routing"]["router"]
        assert out["data"]["ndarray"] == [[float(b)]]
        d.feedback({"request": {"data": {"ndarray": [[1.0, 2.0]]}}, "response": out, "reward": 1.0 if b == 3 else 0.0})
    picks = [d.predict({"data": {"ndarray": [[1.0]]}})["meta"]["routing"]["router"] for _ in range(200)]
    assert np.mean(np.array(picks) == 3) > (0.7 if kind == "EPSILON_GREEDY" else 0.85)
    snap = json.loads(d.engine.snapshot("router"))
    assert sum(snap["tries"]) == 300


@pytest.mark.gpu
@pytest.mark.parametrize("route_on,kind_name", [("auto", "host:epsilon_greedy"), ("device", "gpu:epsilon_greedy")])
def test_mab_graph_gpu_router(route_on, kind_name):
    d = _mab_deployment(0, route_on=route_on)
    try:
        assert d.engine.unit_kind("router") == kind_name
        counts = np.zeros(4)
        for _ in range(2000):
            out = d.predict({"data": {"ndarray": [[1.0]]}})
            counts[out["meta"]["routing"]["router"]] += 1
        assert abs(counts[0] / 2000 - 0.8) < 0.04
    finally:
        d.close()


@pytest.mark.gpu
def test_eg_host_route_matches_bandit_kernel():
    """The host epsilon-greedy path draws from the kernel's Philox stream
    (seed, request counter): the same decision sequence as eg_route_kernel."""
    C = sca.native()
    dev = C.BanditModel(0, 5, 0.35, 11, 2)
    host = C.BanditModel(0, 5, 0.35, 11, 2)
    unit = C.BanditRouterUnit(dev, 0, device_route=True)
    try:
        picks_dev = unit.batcher.run(np.zeros((3000, 1))).ravel().astype(int)
    finally:
        unit.stop()
    picks_host = np.array([host.route_host() for _ in range(3000)])
    assert (picks_dev == picks_host).all()
    assert abs(np.mean(picks_host == 2) - 0.65) < 0.03


def test_shared_state_restore_keeps_newer_live_feedback():
    """restoring a checkpoint used to overwrite the shared bandit
    state of every worker.  Now a snapshot replaces the shared state only
    when it is newer (or the state is fresh): the first worker's restore
    installs it; a worker restarted later with the same old checkpoint pulls
    the live state and keeps the feedback applied since."""
    import os

    name = f"/sca_test_bandit_{os.getpid()}"
    try:
        src = EpsilonGreedy(n_branches=3, epsilon=0.1, best_branch=0, seed=1)
        src.send_feedback(np.ones((5, 1)), [], 1, 1.0, None)
        ckpt = src.model.snapshot()
        a = EpsilonGreedy(n_branches=3, epsilon=0.1, best_branch=0, seed=2)
        a.share_state(name, 0)
        a.model.restore(ckpt)  # fresh shared state: the checkpoint goes in
        assert a.state()["success"] == [0, 5, 0]
        a.send_feedback(np.ones((4, 1)), [], 2, 1.0, None)  # live feedback after the checkpoint
        b = EpsilonGreedy(n_branches=3, epsilon=0.1, best_branch=0, seed=3)
        b.share_state(name, 1)
        b.model.restore(ckpt)  # a restarted worker with the old checkpoint
        assert b.state()["success"] == [0, 5, 4], b.state()
        assert a.state()["success"] == [0, 5, 4], a.state()
        assert b.best_branch == a.best_branch
    finally:
        try:
            os.unlink("/dev/shm" + name)
        except OSError:
            pass
