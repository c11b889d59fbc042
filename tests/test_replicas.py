"""Data-parallel node replicas (reference PredictorSpec.replicas,
seldon_deployment.proto:57): one micro-batcher per device, join-shortest-queue."""
import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression, to_row_model


def _spec(node_extra, graph=None):
    g = graph or {"name": "clf", "type": "MODEL", "children": []}
    g.update(node_extra)
    return {"name": "p", "graph": g, "componentSpecs": [{"spec": {"containers": []}}]}


def test_cpu_replicas_spread_and_agree():
    lr = iris_logistic_regression()
    dep = sca.Deployment(_spec({"devices": [-1, -1, -1]}), components={"clf": lr}, device=-1)
    try:
        assert dep.engine.unit_kind("clf").startswith("replicas3:")
        X = np.random.default_rng(0).normal(size=(4, 4))
        ref = lr.predict_proba(X)
        for _ in range(30):
            out = dep.predict({"data": {"ndarray": X.tolist()}})
            np.testing.assert_allclose(np.array(out["data"]["ndarray"]), ref, rtol=1e-12)
        per = dep.batched["clf"].stats()["per_replica"]
        assert sum(per) == 30 and min(per) >= 9  # idle replicas take turns
    finally:
        dep.close()


def test_clone_is_independent():
    C = sca.native()
    rm = to_row_model(iris_logistic_regression())
    c = rm.clone()
    X = np.random.default_rng(1).normal(size=(3, 4))
    np.testing.assert_array_equal(rm.run_cpu(X), c.run_cpu(X))
    assert c.class_names() == rm.class_names()


def test_fused_graph_replicas_cpu():
    C = sca.native()
    rng = np.random.default_rng(3)
    comps = {"t": C.linear_model(rng.normal(size=(4, 4)), rng.normal(size=4), 0),
             "m": C.linear_model(rng.normal(size=(3, 4)), rng.normal(size=3), 1)}
    graph = {"name": "t", "type": "TRANSFORMER", "children": [{"name": "m", "type": "MODEL", "children": []}]}
    dep = sca.Deployment(_spec({"devices": [-1, -1]}, graph), components=comps, device=-1)
    plain = sca.Deployment(_spec({}, {"name": "t", "type": "TRANSFORMER",
                                      "children": [{"name": "m", "type": "MODEL", "children": []}]}),
                           components=comps, device=-1, fuse=False)
    try:
        assert dep.fused and dep.engine.unit_kind("t").startswith("replicas2:gpu:graph")
        X = rng.normal(size=(5, 4))
        a = dep.predict({"data": {"ndarray": X.tolist()}})
        b = plain.predict({"data": {"ndarray": X.tolist()}})
        np.testing.assert_allclose(a["data"]["ndarray"], b["data"]["ndarray"], rtol=1e-12)
    finally:
        dep.close()
        plain.close()


@pytest.mark.gpu
def test_gpu_replica_matches_sklearn():
    lr = iris_logistic_regression()
    import torch

    n = torch.cuda.device_count()
    dep = sca.Deployment(_spec({"replicas": max(2, n)}), components={"clf": lr}, device=0)
    try:
        X = np.random.default_rng(0).normal(size=(7, 4))
        for _ in range(8):
            out = dep.predict({"data": {"ndarray": X.tolist()}})
            np.testing.assert_allclose(np.array(out["data"]["ndarray"]), lr.predict_proba(X), rtol=1e-12)
        st = dep.batched["clf"].stats()
        devs = [e["device"] for e in st["per_device"]]
        # replicas land on N consecutive GPUs: distinct devices whenever the box has them
        assert devs == [i % n for i in range(max(2, n))], devs
        assert len(set(devs)) == min(n, max(2, n))
        # sequential requests take turns over idle replicas, so every GPU served some
        assert all(e["batches"] > 0 for e in st["per_device"]), st["per_device"]
    finally:
        dep.close()
