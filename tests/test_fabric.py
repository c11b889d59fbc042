"""Cross-rank placement (RCCL fabric) -- the parts checkable without GPUs.
The end-to-end RCCL path is exercised by tools/fabric_probe.py under torchrun
on GPU boxes (one process per GPU)."""
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


def test_native_fabric_api_present():
    C = sca.native()
    for name in ("rccl_unique_id", "Fabric", "PeerServer", "peer_row_model"):
        assert hasattr(C, name)
