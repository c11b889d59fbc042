"""Cross-rank placement.  The mesh (csrc/parallel/mesh.h) runs here end to end
on CPU gangs (gloo rendezvous, shared-memory slabs and doorbells, device -1):
separate processes, the real native program threads on the workers and the
program units on rank 0.  tests/test_mesh_gpu.py runs the same modes with every
rank on GPU 0 over HIP IPC."""
import json
import os
import socket
import subprocess
import sys

import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression
from seldon_core_amd.parallel.fabric import rank_assignments
from seldon_core_amd.serving.deployment import Deployment
from seldon_core_amd.serving.spec import SpecError


def _spec(world):
    kids = [{"name": f"m{r}", "type": "MODEL", "rank": r} for r in range(world)]
    return {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": kids}}


def test_rank_assignments_in_graph_order():
    spec = _spec(3)
    spec["graph"]["children"].append({"name": "extra", "type": "MODEL", "rank": 1})
    assert rank_assignments(spec["graph"]) == {0: ["m0"], 1: ["m1", "extra"], 2: ["m2"]}


def test_remote_rank_without_fabric_is_rejected():
    lr = iris_logistic_regression()
    with pytest.raises(SpecError, match="fabric"):
        sca.Deployment(_spec(2), components={"m0": lr, "m1": lr}, device=-1)


def test_rank0_only_placement_runs_locally():
    lr = iris_logistic_regression()
    dep = sca.Deployment(_spec(1), components={"m0": lr}, device=-1)
    try:
        out = dep.predict({"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}})
        assert abs(sum(out["data"]["ndarray"][0]) - 1.0) < 1e-12
    finally:
        dep.close()


def test_worker_resolver_builds_row_models():
    lr = iris_logistic_regression()
    spec = _spec(2)
    res = Deployment.resolver(spec, {"m0": lr, "m1": lr}, spec)
    kind, obj = res._resolve(spec["graph"]["children"][1])
    rm = res._row_model_of(res._instantiate(spec["graph"]["children"][1], obj))
    assert kind == "object" and rm is not None and rm.in_cols == 4 and rm.out_cols(4) == 3


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    from portutil import free_port

    return free_port()


def _run_ranks(world, mode, **extra_env):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **extra_env)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "fabric_worker.py"), mode],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads([line for line in o.splitlines() if line.startswith("{")][-1]))
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_remote_model_node_cpu_fabric(world):
    outs = _run_ranks(world, "single")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    assert front["transport"] == "shm" and front["messages"] == [2], front
    last = outs[-1]
    assert last["error"] == "" and last["rows"] == front["rows"] and last["batches"] >= 1


def test_remote_model_low_cpu_batcher_cpu_fabric():
    """The batcher's low-CPU mode (blocking waits on the program's reply
    flags instead of spinning): same answers, same row counts."""
    outs = _run_ranks(2, "single", SCA_TEST_LOW_CPU="1")
    assert outs[0]["worst"] < 1e-12 and outs[0]["rows"] > 0
    assert outs[1]["error"] == "" and outs[1]["rows"] == outs[0]["rows"]


def test_combiner_gathers_from_every_rank_cpu_fabric():
    outs = _run_ranks(3, "combiner")
    assert outs[0]["errors"] == [] and outs[0]["worst"] < 1e-12
    assert outs[0]["messages"] == [2, 2], outs[0]  # m1 and m2: one program each, m0 local
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == outs[0]["rows"]


def test_remote_combiner_is_one_program_with_the_mean_on_rank0():
    outs = _run_ranks(3, "remote_combiner")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12, front
    assert front["messages"] == [4] and "mean:comb@rank0" in front["programs"][0], front
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == front["rows"]


def test_pipeline_stages_hand_off_directly():
    """scaler@1 -> scaler@2 -> iris@3: each stage sends its rows straight to
    the next rank; 4 messages per batch (0->1, 1->2, 2->3, 3->0), not the 6 of
    a round trip through rank 0 per stage."""
    outs = _run_ranks(4, "pipeline")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    assert front["messages"] == [4], front
    assert front["kinds"]["s1"].startswith("gpu:mesh_program"), front["kinds"]
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == front["rows"], w


def test_bench_pipeline_dag_fans_out_from_the_scaler_rank():
    outs = _run_ranks(4, "dag")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12, front
    assert front["messages"] == [5], front  # 0->3, 3->1, 3->2, 1->0, 2->0
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == front["rows"], w


def test_python_transformer_on_a_worker_rank():
    """Any node on any rank: a Python TRANSFORMER on rank 1 feeds the iris
    row model on rank 2."""
    outs = _run_ranks(3, "python")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    assert "node:double@rank1" in front["programs"][0] and front["messages"] == [3], front
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == front["rows"], w


def test_failing_python_stage_fails_only_its_requests():
    outs = _run_ranks(3, "python_error")
    front = outs[0]
    assert front["errors"] == [] and front["failed"] == 8 and front["worst"] < 1e-12, front
    assert outs[1]["stage_errors"] >= 1 and outs[1]["error"] == "", outs[1]


def test_native_fabric_api_present():
    C = sca.native()
    for name in ("rccl_unique_ids", "Fabric", "LoopbackHub", "PeerServer", "peer_row_model", "Mesh"):
        assert hasattr(C, name)


def test_concurrent_clients_keep_several_batches_in_flight_cpu_fabric():
    """4 client threads through an A/B router over two remote programs, the
    workers slowed down (SCA_FABRIC_WORKER_DELAY_US): every answer matches
    sklearn to 1e-12 and the workers held more than one batch at a time
    (rank 0 issues up to K = 4 batches per program ahead)."""
    outs = _run_ranks(3, "concurrent", SCA_FABRIC_SLOTS="4", SCA_FABRIC_WORKER_DELAY_US="3000")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    for w in outs[1:]:
        assert w["error"] == "" and w["slots"] == 4 and w["batches"] > 0, w
        assert 2 <= w["max_inflight"] <= 4, w


def test_large_and_wide_batches_cpu_fabric():
    """3000-row requests through 64-row slots (the request is split into
    chunks, more chunks than slots) and 784-column outputs."""
    outs = _run_ranks(2, "large")
    assert outs[0]["errors"] == [] and outs[0]["worst"] < 1e-9, outs[0]
    assert outs[1]["error"] == "" and outs[1]["rows"] == outs[0]["rows"], outs[1]


def test_worker_exits_when_front_end_dies():
    """A worker polling its rings notices rank 0's death (control socket
    EOF) and leaves with an error instead of spinning forever."""
    outs = _run_ranks(2, "orphan")
    assert "gone" in outs[1]["error"] or "closed" in outs[1]["error"], outs[1]


def test_placed_router_is_rejected():
    from seldon_core_amd.parallel.mesh import plan

    g = {"name": "r", "type": "ROUTER", "rank": 1, "children": [{"name": "m", "type": "MODEL", "rank": 2}]}
    with pytest.raises(SpecError, match="cannot be placed"):
        plan(g)


def test_plan_places_inner_means_on_their_consumer():
    from seldon_core_amd.parallel.mesh import plan

    g = {"name": "post", "type": "OUTPUT_TRANSFORMER", "rank": 3, "children": [
        {"name": "comb", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
         "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]}]}
    (p,) = plan(g)
    assert [(s.node, s.kind, s.rank, s.inputs) for s in p.stages] == [
        ("a", "node", 1, [-1]), ("b", "node", 2, [-1]), ("comb", "mean", 3, [0, 1]), ("post", "node", 3, [2])]
    assert p.absorbed == ["post", "comb", "a", "b"]


def test_plan_nested_combiners_without_ranks():
    """AVERAGE(AVERAGE(a@1, b@2), c@3) with no rank on either
    combiner: the outer mean is the program's output on rank 0; the inner one
    cannot run there, so it runs on its first input's rank."""
    from seldon_core_amd.parallel.mesh import plan

    g = {"name": "outer", "type": "COMBINER", "implementation": "AVERAGE_COMBINER", "children": [
        {"name": "inner", "type": "COMBINER", "implementation": "AVERAGE_COMBINER",
         "children": [{"name": "a", "type": "MODEL", "rank": 1}, {"name": "b", "type": "MODEL", "rank": 2}]},
        {"name": "c", "type": "MODEL", "rank": 3}]}
    (p,) = plan(g)
    assert [(s.node, s.kind, s.rank, s.inputs) for s in p.stages] == [
        ("a", "node", 1, [-1]), ("b", "node", 2, [-1]), ("inner", "mean", 1, [0, 1]), ("c", "node", 3, [-1]),
        ("outer", "mean", 0, [2, 3])]
    # explicit ranks on the combiners are not needed and do not break it
    g["rank"] = 2
    g["children"][0]["rank"] = 0
    (p,) = plan(g)
    assert [s.rank for s in p.stages] == [1, 2, 1, 3, 0]


def test_plan_deeply_nested_means_resolve_consumers_first():
    from seldon_core_amd.parallel.mesh import plan

    leaf = lambda n, r: {"name": n, "type": "MODEL", "rank": r}  # noqa: E731
    comb = lambda n, kids, **kw: {"name": n, "type": "COMBINER", "implementation": "AVERAGE_COMBINER",  # noqa: E731
                                  "children": kids, **kw}
    g = {"name": "post", "type": "OUTPUT_TRANSFORMER", "rank": 4, "children": [
        comb("o", [comb("i1", [comb("i2", [leaf("a", 1), leaf("b", 2)]), leaf("c", 3)]), leaf("d", 2)])]}
    (p,) = plan(g)
    ranks = {s.node: s.rank for s in p.stages}
    # post@4 consumes o (so o runs on 4); o consumes i1 (4); i1 consumes i2 (4)
    assert ranks == {"a": 1, "b": 2, "i2": 4, "c": 3, "i1": 4, "d": 2, "o": 4, "post": 4}


def test_placed_model_with_a_rank0_child_is_rejected():
    """a ranked MODEL that no program can absorb used to be bound
    on rank 0 silently."""
    from seldon_core_amd.parallel.mesh import plan

    g = {"name": "m", "type": "MODEL", "rank": 1, "children": [
        {"name": "r", "type": "ROUTER", "children": [{"name": "x", "type": "MODEL"}]}]}
    with pytest.raises(SpecError, match="placed on rank 1 but its child 'r'"):
        plan(g)
    g = {"name": "m", "type": "MODEL", "rank": 1, "children": [{"name": "x", "type": "MODEL"}]}
    with pytest.raises(SpecError, match="child 'x'"):
        plan(g)


def test_nested_combiner_program_runs_cpu_fabric():
    outs = _run_ranks(4, "nested_combiner")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    assert "mean:inner@rank1" in front["programs"][0] and "mean:outer@rank0" in front["programs"][0], front
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == front["rows"], w


def test_cpu_gang_edges_report_shm_and_skip_the_probe():
    outs = _run_ranks(4, "pipeline")
    front = outs[0]
    (edges,) = front["edges"]
    assert {e["transport"] for e in edges} == {"shm"}, edges
    assert front["peer"]["failed_edges"] == [] and set(front["peer"]["probed"]["1"]) == {-1}, front["peer"]
