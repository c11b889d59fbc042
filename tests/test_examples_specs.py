"""Every SeldonDeployment in examples/ loads, validates and answers a
prediction + feedback on the CPU path (GPU placement hints fold to the host)."""
import glob
import os

import numpy as np
import pytest

import seldon_core_amd as sca

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS = sorted(glob.glob(os.path.join(ROOT, "examples", "*.json")))


@pytest.mark.parametrize("path", SPECS, ids=[os.path.basename(p) for p in SPECS])
def test_example_spec_runs(path):
    dep = sca.Deployment(path, device=-1)
    try:
        req = {"data": {"names": ["a", "b", "c"], "ndarray": np.random.default_rng(0).random((2, 3)).tolist()}}
        out = dep.predict(req)
        assert "data" in out and out["meta"]["puid"]
        dep.feedback({"request": req, "response": out, "reward": 1.0})
    finally:
        dep.close()


def test_examples_present():
    assert len(SPECS) >= 7
