"""Device-graph fusion: a fused all-row-model subtree must answer exactly like
the unfused per-node walk (reference PredictiveUnitBean.java:112-197 semantics),
including meta.requestPath / meta.routing and feedback traversal."""
import json

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.parallel import device_graph


def _lin(C, W, b, act=0):
    return C.linear_model(np.asarray(W, float), np.asarray(b, float), act)


def _spec(graph):
    return {"name": "p", "graph": graph, "componentSpecs": [{"spec": {"containers": []}}]}


def _components(C, rng):
    return {
        "tin": _lin(C, rng.normal(size=(4, 4)), rng.normal(size=4)),
        "m1": _lin(C, rng.normal(size=(3, 4)), rng.normal(size=3), 1),
        "m2": _lin(C, rng.normal(size=(3, 4)), rng.normal(size=3), 1),
        "m3": _lin(C, rng.normal(size=(3, 4)), rng.normal(size=3), 1),
        "tout": _lin(C, rng.normal(size=(2, 3)), rng.normal(size=2)),
    }


GRAPHS = {
    "chain": {"name": "tin", "type": "TRANSFORMER", "children": [
        {"name": "m1", "type": "MODEL", "children": []}]},
    "ensemble": {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
        {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}, {"name": "m3", "type": "MODEL"}]},
    "full": {"name": "tout", "type": "OUTPUT_TRANSFORMER", "children": [
        {"name": "tin", "type": "TRANSFORMER", "children": [
            {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
                {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}]}]}]},
    "model_two_children": {"name": "tin", "type": "MODEL", "children": [
        {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}]},
}


def _used(graph):
    out = []

    def walk(n):
        out.append(n["name"])
        for c in n.get("children", []):
            walk(c)
    walk(graph)
    return out


def _pair(name, device=-1):
    C = sca.native()
    g = GRAPHS[name]
    used = set(_used(g))
    comps = {k: v for k, v in _components(C, np.random.default_rng(7)).items() if k in used}
    fused = sca.Deployment(_spec(g), components=comps, device=device, fuse=True)
    plain = sca.Deployment(_spec(g), components=comps, device=device, fuse=False)
    return fused, plain


@pytest.mark.parametrize("name", sorted(GRAPHS))
@pytest.mark.parametrize("kind", ["tensor", "ndarray"])
def test_fused_matches_unfused(name, kind):
    fused, plain = _pair(name)
    try:
        assert fused.fused, "graph should have fused"
        assert not plain.fused
        X = np.random.default_rng(1).normal(size=(5, 4))
        data = ({"tensor": {"shape": list(X.shape), "values": X.ravel().tolist()}} if kind == "tensor"
                else {"ndarray": X.tolist()})
        req = {"meta": {"puid": "abc"}, "data": {"names": ["a", "b", "c", "d"], **data}}
        a = fused.predict(req)
        b = plain.predict(req)
        assert a["meta"]["requestPath"] == b["meta"]["requestPath"]
        assert a["meta"]["routing"] == b["meta"]["routing"]
        assert a["data"]["names"] == b["data"]["names"]
        assert kind in a["data"]
        va = np.array(a["data"]["tensor"]["values"] if kind == "tensor" else a["data"]["ndarray"])
        vb = np.array(b["data"]["tensor"]["values"] if kind == "tensor" else b["data"]["ndarray"])
        np.testing.assert_allclose(va, vb, rtol=1e-12, atol=1e-14)
        fb = fused.feedback({"request": req, "response": a, "reward": 1.0})
        assert fb is not None
        assert 'seldon_api_model_feedback_total{' in fused.metrics()
    finally:
        fused.close()
        plain.close()


def test_plan_shapes():
    C = sca.native()
    comps = _components(C, np.random.default_rng(0))
    g = GRAPHS["full"]
    plans = device_graph.plan(g, comps, {}, lambda n: int(n.get("device", 0)))
    assert len(plans) == 1
    fg = plans[0]
    assert fg.root == "tout"
    assert [s["node"] for s in fg.stages] == ["tin", "m1", "m2", "comb", "tout"]
    assert fg.stages[3]["inputs"] == [1, 2]
    assert fg.stages[4]["inputs"] == [3]
    assert set(fg.absorbed) == {"tout", "tin", "comb", "m1", "m2"}


def test_router_stops_fusion_but_children_fuse():
    C = sca.native()
    comps = _components(C, np.random.default_rng(0))
    g = {"name": "r", "type": "ROUTER", "implementation": "RANDOM_ABTEST",
         "parameters": [{"name": "ratioA", "value": "0.5", "type": "FLOAT"}],
         "children": [GRAPHS["chain"], {"name": "m2", "type": "MODEL"}]}
    dep = sca.Deployment(_spec(g), components={k: comps[k] for k in ("tin", "m1", "m2")}, device=-1)
    try:
        assert list(dep.fused) == ["tin"]
        assert dep.engine.fused_nodes("tin") == ["tin", "m1"]
        out = dep.predict({"data": {"ndarray": [[1.0, 2.0, 3.0, 4.0]]}})
        assert out["meta"]["routing"]["r"] in (0, 1)
    finally:
        dep.close()


def test_combiner_width_mismatch_falls_back_to_engine_error():
    C = sca.native()
    g = {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
        {"name": "m1", "type": "MODEL"}, {"name": "m2", "type": "MODEL"}]}
    comps = {"m1": _lin(C, np.ones((3, 2)), np.zeros(3)), "m2": _lin(C, np.ones((2, 2)), np.zeros(2))}
    dep = sca.Deployment(_spec(g), components=comps, device=-1)
    try:
        assert not dep.fused
        status, body = dep.predict_raw({"data": {"ndarray": [[1.0, 2.0]]}})
        assert status == 500 and body["code"] == 204
    finally:
        dep.close()


def test_annotation_disables_fusion():
    C = sca.native()
    spec = _spec(GRAPHS["chain"])
    spec["annotations"] = {"seldon.io/device-graph": "false"}
    comps = {k: v for k, v in _components(C, np.random.default_rng(0)).items() if k in ("tin", "m1")}
    dep = sca.Deployment(spec, components=comps, device=-1)
    try:
        assert not dep.fused
    finally:
        dep.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_fused_gpu_matches_cpu(name):
    fused, plain = _pair(name, device=0)
    cpu_f, cpu_p = _pair(name, device=-1)
    try:
        assert fused.engine.unit_kind(fused.fused and next(iter(fused.fused))).startswith("gpu:graph")
        X = np.random.default_rng(2).normal(size=(33, 4))
        req = json.dumps({"data": {"tensor": {"shape": list(X.shape), "values": X.ravel().tolist()}}})
        outs = [np.array(d.predict(req)["data"]["tensor"]["values"]) for d in (fused, plain, cpu_f, cpu_p)]
        for o in outs[1:]:
            np.testing.assert_allclose(outs[0], o, rtol=1e-12, atol=1e-14)
    finally:
        for d in (fused, plain, cpu_f, cpu_p):
            d.close()


def _linear_graph_stages(C, rng):
    comps = _components(C, rng)
    comps["bin"] = _lin(C, rng.normal(size=(1, 2)), rng.normal(size=1), 2)  # binary logistic: 2 outputs
    return [{"kind": "model", "model": comps["tin"], "inputs": [-1], "node": "tin"},
            {"kind": "model", "model": comps["m1"], "inputs": [0], "node": "m1"},
            {"kind": "model", "model": comps["m2"], "inputs": [0], "node": "m2"},
            {"kind": "model", "model": comps["m3"], "inputs": [-1], "node": "m3"},
            {"kind": "mean", "inputs": [1, 2, 3], "node": "comb"},
            {"kind": "model", "model": comps["tout"], "inputs": [4], "node": "tout"},
            {"kind": "model", "model": comps["bin"], "inputs": [5], "node": "bin"}]


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 33, 129, 1000, 5000])
def test_linear_graph_runs_as_one_kernel(rows, monkeypatch):
    """a device graph of small linear stages and means
    (transformer -> 3-way ensemble -> output transformer -> binary logistic)
    is ONE linear_graph_rows kernel per batch; it answers like the per-stage
    kernels (SCA_GRAPH_FUSE=0) and the CPU walk to 1e-12."""
    C = sca.native()
    X = np.random.default_rng(rows).normal(size=(rows, 4))
    outs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("SCA_GRAPH_FUSE", fuse)
        g = C.graph_model(_linear_graph_stages(C, np.random.default_rng(11)), 4)
        unit = C.BatchedUnit(g, 0, max_batch=8192)
        try:
            assert C.graph_info(g)["fused"] == (fuse == "1")
            outs.append(np.asarray(unit.run(X)).reshape(rows, 2))
        finally:
            unit.stop()
    ref = C.graph_model(_linear_graph_stages(C, np.random.default_rng(11)), 4).run_cpu(X)
    np.testing.assert_allclose(outs[0], ref, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(outs[1], ref, rtol=1e-12, atol=1e-13)


def test_linear_graph_fusion_rules_cpu():
    """Graphs with a non-linear stage, a wide stage or too many stages keep
    the per-stage path (the flag is decided at to_device: GPU only)."""
    C = sca.native()
    g = C.graph_model(_linear_graph_stages(C, np.random.default_rng(1)), 4)
    assert C.graph_info(g)["fused"] is False  # never placed on a GPU here


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [5, 40, 300])
def test_tree_stage_in_device_graph_writes_final_output(rows):
    """A tree ensemble launched by its own batcher folds its split-kernel part
    sums on the host (RowModel::finish_host); as a device-graph stage it must
    write its final output (the next stage reads it on the GPU)."""
    from seldon_core_amd.models import synthetic_xgboost, to_row_model

    C = sca.native()
    ens = synthetic_xgboost(200, 6, 4, seed=3)
    scaler = _lin(C, np.eye(4) * 1.5, np.zeros(4))
    tail = _lin(C, np.array([[2.0]]), np.array([-1.0]))  # reads the tree's output on the GPU
    g = C.graph_model([{"kind": "model", "model": scaler, "inputs": [-1]},
                       {"kind": "model", "model": to_row_model(ens), "inputs": [0]},
                       {"kind": "model", "model": tail, "inputs": [1]}], 4)
    unit = C.BatchedUnit(g, 0, max_batch=4096)
    direct = C.BatchedUnit(to_row_model(ens), 0, max_batch=4096)
    try:
        X = np.random.default_rng(rows).normal(size=(rows, 4))
        ref = np.asarray(ens.predict(X * 1.5)).reshape(rows, -1)
        got = np.asarray(unit.run(X)).reshape(rows, -1)
        np.testing.assert_allclose(got, 2.0 * ref - 1.0, rtol=2e-5, atol=4e-5)
        got_direct = np.asarray(direct.run(X * 1.5)).reshape(rows, -1)
        np.testing.assert_allclose(got_direct, ref, rtol=2e-5, atol=2e-5)
    finally:
        unit.stop()
        direct.stop()
