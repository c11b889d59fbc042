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


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
def test_signalled_tree_batches_are_exact_under_concurrency(fused):
    """Tree ensembles: the batch's last kernel completes the event -- the
    reduce kernel of the two-pass plan (the partial kernel before it on the
    same stream), or the fused plan's partial kernel whose last workgroup
    folds the slab; both must hand back complete answers."""
    from seldon_core_amd.models import synthetic_xgboost

    ens = synthetic_xgboost(300, 6, 16, seed=9)
    d = ens.device_spec()
    d["fused_reduce"] = fused
    unit = sca.native().BatchedUnit(sca.native().tree_model(d), 0, slots=4)
    rng = np.random.default_rng(7)
    Xs = [rng.standard_normal((1 + i % 29, 16)) for i in range(600)] + [rng.standard_normal((700, 16))]
    try:
        with cf.ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(unit.run, Xs))
        for X, got in zip(Xs, outs):
            np.testing.assert_allclose(np.asarray(got).reshape(-1), ens.predict(X).reshape(-1), rtol=2e-5, atol=2e-5)
    finally:
        unit.stop()
