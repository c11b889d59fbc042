"""Cross-rank placement (fabric).  The peer protocol runs here end to end on
CPU fabrics (gloo rendezvous, control + data over sockets, device -1) through
the real native PeerRowModel / PeerServer state machines; the RCCL data plane
is exercised by tools/fabric_probe.py under torchrun on GPU boxes."""
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
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
    assert front["worst"] < 1e-12 and front["rows"] > 0
    last = outs[-1]
    assert last["error"] == "" and last["rows"] == front["rows"] and last["batches"] >= 1
    assert last["host_syncs"] == 0  # CPU loop never waits on a device


def test_remote_model_low_cpu_batcher_cpu_fabric():
    """The batcher's low-CPU mode waits on the peer's link socket (ppoll)
    instead of sleeping between polls: same answers, same row counts."""
    outs = _run_ranks(2, "single", SCA_TEST_LOW_CPU="1")
    assert outs[0]["worst"] < 1e-12 and outs[0]["rows"] > 0
    assert outs[1]["error"] == "" and outs[1]["rows"] == outs[0]["rows"]


def test_combiner_gathers_from_every_rank_cpu_fabric():
    outs = _run_ranks(3, "combiner")
    assert outs[0]["worst"] < 1e-12
    for w in outs[1:]:
        assert w["error"] == "" and w["rows"] == outs[0]["rows"]


def test_native_fabric_api_present():
    C = sca.native()
    for name in ("rccl_unique_ids", "Fabric", "LoopbackHub", "PeerServer", "peer_row_model"):
        assert hasattr(C, name)


def test_concurrent_senders_keep_k_batches_in_flight_cpu_fabric():
    """4 concurrent senders x 3 ranks, K = 4 slots per worker: every answer
    (single peers and the broadcast/gather fan-out) matches sklearn to 1e-12,
    and the workers really held more than one batch in flight (headers come
    through the shared-memory ring, payloads are read ahead of compute)."""
    outs = _run_ranks(3, "concurrent", SCA_FABRIC_SLOTS="4", SCA_FABRIC_WORKER_DELAY_US="3000")
    front = outs[0]
    assert front["errors"] == [] and front["worst"] < 1e-12 and front["rows"] > 0, front
    for w in outs[1:]:
        assert w["error"] == "" and w["slots"] == 4 and w["batches"] > 0, w
        assert 2 <= w["max_inflight"] <= 4, w


def test_large_replies_arrive_in_pieces_cpu_fabric():
    outs = _run_ranks(2, "large")
    assert outs[0]["errors"] == [] and outs[0]["worst"] < 1e-12, outs[0]
    assert outs[1]["error"] == "" and outs[1]["rows"] >= 3 * 60000, outs[1]


def test_header_ring_liveness_worker_exits_when_front_end_dies():
    """A worker polling its header ring notices rank 0's death (control
    socket EOF) and leaves with an error instead of spinning forever."""
    outs = _run_ranks(2, "orphan")
    assert "gone" in outs[1]["error"] or "closed" in outs[1]["error"], outs[1]
