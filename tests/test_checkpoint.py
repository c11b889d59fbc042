"""Checkpoint / resume of graph state.

Reference: python/seldon_core/persistence.py:21-85 pickles the user object to
Redis every push_frequency seconds and restores it at start; here every
stateful node of an in-engine graph (native bandit routers, Python
components, outlier detectors) checkpoints and restores through the same
store keys."""
import json
import pickle
import time

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components.outlier import OutlierMahalanobis
from seldon_core_amd.models import iris_logistic_regression
from seldon_core_amd.utils.persistence import FileStore


class Const:
    def __init__(self, v):
        self.v = v

    def predict(self, X, names):
        return np.full((X.shape[0], 1), float(self.v))


def _mab(n=3):
    params = [{"name": "n_branches", "value": str(n), "type": "INT"}, {"name": "seed", "value": "7", "type": "INT"},
              {"name": "epsilon", "value": "0.2", "type": "FLOAT"}, {"name": "best_branch", "value": "0", "type": "INT"}]
    spec = {"name": "mab", "graph": {"name": "router", "type": "ROUTER", "implementation": "EPSILON_GREEDY",
                                     "parameters": params,
                                     "children": [{"name": f"m{i}", "type": "MODEL"} for i in range(n)]}}
    return sca.Deployment(spec, components={f"m{i}": Const(i) for i in range(n)}, device=-1, deployment_name="ck")


def test_bandit_state_survives_restart(tmp_path):
    store = FileStore(str(tmp_path))
    d = _mab()
    try:
        for _ in range(60):
            out = d.predict({"data": {"ndarray": [[1.0]]}})
            b = out["meta"]["routing"]["router"]
            d.feedback({"request": {"data": {"ndarray": [[1.0]]}}, "response": out, "reward": float(b == 2)})
        assert d.checkpoint(store) >= 1
        before = json.loads(d.engine.snapshot("router"))
    finally:
        d.close()
    assert (tmp_path / "persistence_ck_mab_router.pkl").exists()
    d2 = _mab()
    try:
        assert json.loads(d2.engine.snapshot("router"))["tries"] != before["tries"]  # fresh
        assert d2.restore_checkpoint(store) >= 1
        after = json.loads(d2.engine.snapshot("router"))
        assert after["tries"] == before["tries"] and after["best"] == before["best"] == 2 and after["values"] == before["values"]
    finally:
        d2.close()


def _od_dep():
    det = OutlierMahalanobis(threshold=10, n_components=2, start_clip=20, device=-1)
    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "od", "type": "TRANSFORMER", "children": [{"name": "clf", "type": "MODEL"}]}}
    return sca.Deployment(spec, components={"od": det, "clf": iris_logistic_regression()}, device=-1,
                          deployment_name="odck"), det


def test_outlier_detector_online_state_restores(tmp_path):
    store = FileStore(str(tmp_path))
    rng = np.random.default_rng(0)
    batches = [rng.normal(size=(8, 4)).tolist() for _ in range(6)]
    a, det_a = _od_dep()
    b, det_b = _od_dep()
    try:
        for X in batches[:4]:
            a.predict({"data": {"ndarray": X}})
        a.checkpoint(store)
        b.restore_checkpoint(store)
        assert det_b is not None
        ta = a.predict({"data": {"ndarray": batches[4]}})["meta"]["tags"]["outlier-predictions"]
        tb = b.predict({"data": {"ndarray": batches[4]}})["meta"]["tags"]["outlier-predictions"]
        assert ta == tb
        _, sa = pickle.loads(a.engine.snapshot("od"))
        _, sb = pickle.loads(b.engine.snapshot("od"))
        assert set(sa) == set(sb)
        for k in sa:  # identical online state after the same traffic
            assert repr(sa[k]) == repr(sb[k]), k
    finally:
        a.close()
        b.close()


def test_state_dict_covers_online_fields():
    det = OutlierMahalanobis(n_components=2, start_clip=5, device=-1)
    det.predict(np.random.default_rng(1).normal(size=(10, 3)), [])
    st = det.state_dict()
    assert {"mean", "C", "n", "clip", "nb_outliers", "_predictions"} <= set(st)
    fresh = OutlierMahalanobis(n_components=2, start_clip=5, device=-1)
    fresh.load_state_dict(st)
    X = np.random.default_rng(2).normal(size=(4, 3))
    np.testing.assert_array_equal(fresh.predict(X, []), det.predict(X, []))
    np.testing.assert_allclose(fresh.score, det.score)


def test_periodic_and_final_checkpoint(tmp_path):
    store = FileStore(str(tmp_path))
    d = _mab()
    d.start_checkpointing(push_frequency=0.05, store=store)
    path = tmp_path / "persistence_ck_mab_router.pkl"
    t0 = time.time()
    while not path.exists() and time.time() - t0 < 5:
        time.sleep(0.02)
    assert path.exists()
    out = d.predict({"data": {"ndarray": [[1.0]]}})
    d.feedback({"request": {"data": {"ndarray": [[1.0]]}}, "response": out, "reward": 1.0})
    d.close()  # final checkpoint after the drain
    final = json.loads(path.read_bytes())
    assert sum(final["tries"]) == 1


def test_worker_keys_are_per_rank(monkeypatch):
    d = _mab()
    try:
        monkeypatch.setenv("SCA_WORKERS", "4")
        monkeypatch.setenv("SCA_WORKER_RANK", "2")
        assert d.checkpoint_key("router") == "persistence_ck_mab_router_w2"
        monkeypatch.setenv("SCA_WORKERS", "1")
        assert d.checkpoint_key("router") == "persistence_ck_mab_router"
    finally:
        d.close()


@pytest.mark.gpu
def test_gpu_bandit_router_checkpoint_roundtrip(tmp_path):
    """Device-side bandit state (pinned tries/values) survives a restart."""
    store = FileStore(str(tmp_path))

    def gpu_mab():
        params = [{"name": "n_branches", "value": "3", "type": "INT"}, {"name": "seed", "value": "7", "type": "INT"},
                  {"name": "epsilon", "value": "0.1", "type": "FLOAT"},
                  {"name": "best_branch", "value": "0", "type": "INT"},
                  {"name": "route_on", "value": "device", "type": "STRING"}]  # the batched bandit kernel
        spec = {"name": "mab", "graph": {"name": "router", "type": "ROUTER", "implementation": "EPSILON_GREEDY",
                                         "parameters": params,
                                         "children": [{"name": f"m{i}", "type": "MODEL"} for i in range(3)]}}
        return sca.Deployment(spec, components={f"m{i}": Const(i) for i in range(3)}, device=0,
                              deployment_name="gck")

    d = gpu_mab()
    try:
        assert d.engine.unit_kind("router") == "gpu:epsilon_greedy"
        for _ in range(200):
            out = d.predict({"data": {"ndarray": [[1.0]]}})
            b = out["meta"]["routing"]["router"]
            d.feedback({"request": {"data": {"ndarray": [[1.0]]}}, "response": out, "reward": float(b == 1)})
        assert d.checkpoint(store) >= 1
        before = json.loads(d.engine.snapshot("router"))
    finally:
        d.close()
    assert before["best"] == 1
    d2 = gpu_mab()
    try:
        assert d2.restore_checkpoint(store) >= 1
        after = json.loads(d2.engine.snapshot("router"))
        assert after["tries"] == before["tries"] and after["best"] == 1
        picks = [d2.predict({"data": {"ndarray": [[1.0]]}})["meta"]["routing"]["router"] for _ in range(400)]
        assert np.mean(np.array(picks) == 1) > 0.85  # exploits the restored best branch at once
    finally:
        d2.close()
