"""Control-plane naming helpers (reference seldondeployment_types.go:48-190)."""
import hashlib

from seldon_core_amd.serving import naming

SDEP = {"metadata": {"name": "mydep"},
        "spec": {"name": "sdep", "predictors": [{
            "name": "main",
            "componentSpecs": [{"spec": {"containers": [{"name": "clf", "image": "seldonio/iris:0.1"}]}}],
            "graph": {"name": "clf", "endpoint": {"service_host": "localhost"},
                      "children": [{"name": "child"}]}}]}}


def test_short_names():
    p = SDEP["spec"]["predictors"][0]
    assert naming.sdep_name(SDEP) == "sdep-mydep"
    ch = hashlib.md5(b"clf:seldonio/iris:0.1;").hexdigest()[:7]
    assert naming.container_hash(p["componentSpecs"][0]) == ch
    assert naming.deployment_name(SDEP, p, p["componentSpecs"][0]) == f"sdep-main-{ch}"
    ph = hashlib.md5((ch + ",").encode()).hexdigest()[:7]
    assert naming.service_orchestrator_name(SDEP, p) == f"sdep-main-svc-orch-{ph}"
    assert naming.predictor_key(SDEP, p) == "mydep-sdep-main"
    assert naming.container_service_name(SDEP, p, p["componentSpecs"][0]["spec"]["containers"][0]) == \
        "sdep-main-clf-seldonio-iris-0-1"


def test_long_names_hash():
    long = {"metadata": {"name": "m" * 40}, "spec": {"name": "s" * 40}}
    n = naming.sdep_name(long)
    assert n.startswith("seldon-") and len(n) == 7 + 32


def test_graph_helpers():
    g = SDEP["spec"]["predictors"][0]["graph"]
    assert naming.get_predictive_unit(g, "child")["name"] == "child"
    assert naming.get_predictive_unit(g, "none") is None
    assert naming.get_engine_predictive_unit(g)["name"] == "clf"
    assert [u["name"] for u in naming.predictive_unit_list(g)] == ["clf", "child"]
