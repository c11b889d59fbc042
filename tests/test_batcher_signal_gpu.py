"""Batches whose kernel completes the slot event from its own dispatch
(RowModel::launch_signal -> hipExtLaunchKernelGGL, no hipEventRecord): every
answer must be visible and exact the moment the batcher reaps it."""
import concurrent.futures as cf

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import iris_logistic_regression, to_row_model


@pytest.mark.gpu
def test_signalled_linear_batches_are_exact_under_concurrency():
    clf = iris_logistic_regression()
    unit = sca.native().BatchedUnit(to_row_model(clf), 0, slots=4)
    rng = np.random.default_rng(5)
    Xs = [rng.normal(size=(1 + i % 13, 4)) * 3 for i in range(1200)]
    try:
        with cf.ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(unit.run, Xs))
        worst = max(float(np.abs(o - clf.predict_proba(X)).max()) for o, X in zip(outs, Xs))
        assert worst < 1e-12, worst
        st = unit.stats()
        assert st["requests"] >= 1200 and st["batches"] >= 1
    finally:
        unit.stop()
