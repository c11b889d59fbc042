"""SeldonDeployment JSON schema (reference CRD
operator/config/crd/bases/machinelearning.seldon.io_seldondeployments.yaml).

The reference's own deployment documents serve as fixtures (JSON / YAML read
with safe loaders): every one must validate, except the two that are invalid
on purpose (notebooks/resources/model_invalid1.json -- integer where a string
belongs -- and the operator sample's placeholder ``foo`` field)."""
import glob
import json
import os

import pytest
import yaml

from seldon_core_amd.serving import spec
from seldon_core_amd.serving.jsonschema import validate_instance, validate_schema

REF = "/root/reference"


def _ref_docs():
    out = []
    files = glob.glob(f"{REF}/**/*.json", recursive=True) + glob.glob(f"{REF}/**/*.yaml", recursive=True)
    for f in sorted(files):
        if "/crd/" in f or "helm-charts" in f:
            continue
        try:
            with open(f) as fh:
                docs = [json.load(fh)] if f.endswith(".json") else list(yaml.safe_load_all(fh))
        except Exception:
            continue
        out += [(f, d) for d in docs if isinstance(d, dict) and d.get("kind") == "SeldonDeployment"]
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_deployments_validate():
    docs = _ref_docs()
    assert len(docs) > 50
    bad = {os.path.relpath(f, REF): validate_schema(d) for f, d in docs if validate_schema(d)}
    assert set(bad) == {"notebooks/resources/model_invalid1.json",
                        "operator/config/samples/machinelearning_v1alpha2_seldondeployment.yaml"}, bad
    errs = bad["notebooks/resources/model_invalid1.json"]
    assert any(e.startswith("spec.oauth_key: Invalid value") for e in errs)
    assert any("imagePullPolicy" in e and "must be of type string" in e for e in errs)


def test_our_examples_validate():
    for f in glob.glob(os.path.join(os.path.dirname(__file__), "..", "examples", "*.json")):
        d = json.load(open(f))
        if spec.is_deployment(d):
            assert validate_schema(d) == [], f


def test_error_messages_and_recursion():
    sdep = {"apiVersion": "machinelearning.seldon.io/v1alpha2", "kind": "SeldonDeployment",
            "metadata": {"name": "x"},
            "spec": {"predictors": [{"name": "p", "traffic": 101, "graph": {
                "name": "a", "type": "MODEL", "children": [
                    {"name": "b", "type": "SPLITTER", "parameters": [{"name": "k", "type": "LONG", "value": "1"}],
                     "endpoint": {"type": "HTTP", "service_port": 70000}}]}}]}}
    errs = validate_schema(sdep)
    assert 'spec.predictors[0].traffic: Invalid value: 101: must be less than or equal to 100' in errs
    assert any(e.startswith('spec.predictors[0].graph.children[0].type: Unsupported value: "SPLITTER"') for e in errs)
    assert any(e.startswith('spec.predictors[0].graph.children[0].parameters[0].type: Unsupported value: "LONG"')
               for e in errs)
    assert any(e.startswith('spec.predictors[0].graph.children[0].endpoint.type: Unsupported value: "HTTP"')
               for e in errs)
    assert any("service_port: Invalid value: 70000" in e for e in errs)
    # spec.validate runs the schema first and stops there
    assert spec.validate(sdep)[:len(errs)] == errs
    missing = validate_schema({"spec": {"predictors": [{"name": "p"}]}})
    assert missing == ["spec.predictors[0].graph: Required value"]


def test_validator_keywords():
    s = {"type": "object", "properties": {"a": {"anyOf": [{"type": "integer"}, {"type": "string", "pattern": "^x"}]},
                                          "b": {"type": "array", "minItems": 2, "items": {"type": "number"}}},
         "additionalProperties": {"type": "boolean"}}
    assert validate_instance({"a": 3, "b": [1, 2.5], "c": True}, s) == []
    e = validate_instance({"a": "y", "b": [1], "c": 1}, s)
    assert len(e) == 3 and e[0].startswith("a: Invalid value") and "at least 2" in e[1] and e[2].startswith("c:")
