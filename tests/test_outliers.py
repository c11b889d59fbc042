"""Outlier detectors against independent numpy statements of
the reference algorithms (components/outlier-detection/*)."""
import os

import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components.outlier import (OutlierIsolationForest, OutlierMahalanobis, OutlierSeq2SeqLSTM,
                                                 OutlierVAE, performance)


def test_mahalanobis_online_mean_and_covariance_recursion():
    """One row per request (CoreMahalanobis.py:89-101 with nb = 1): the mean is
    the running sample mean and C_{n+1} = (n-1)/(n+1) C_n + n/(n+1)^2 d d^T,
    d = x - mean_n (the reference's normalisation, not Welford's)."""
    det = OutlierMahalanobis(n_components=3, start_clip=10 ** 9, device=-1)
    rng = np.random.default_rng(0)
    X = rng.normal(size=(60, 5)) * np.array([1, 2, 3, 0.5, 4])
    mean, C = np.zeros(5), np.zeros((5, 5))
    for i in range(len(X)):
        det.predict(X[i:i + 1], [])
        n = i
        d = X[i] - mean
        C = (n - 1.0) / (n + 1.0) * C + n / (n + 1.0) ** 2 * np.outer(d, d)
        mean = mean + d / (n + 1.0)
    np.testing.assert_allclose(det.mean, X.mean(axis=0), rtol=1e-12)
    np.testing.assert_allclose(det.mean, mean, rtol=1e-12)
    np.testing.assert_allclose(det.C, C, rtol=1e-10)


def _oracle_scores(det_before, X):
    """Scores of one batch by explicit inverses: C_i = inv(M_i),
    M_0 = V^T C V, M_i = (n+i-2)/(n+i-1) M_{i-1} + B_{i-1}."""
    from scipy.linalg import eigh

    n = det_before["n"]
    mean, C = det_before["mean"], det_before["C"]
    nb, p = X.shape
    k = det_before["k"]
    steps = np.arange(nb)
    roll = X.cumsum(axis=0) / (steps + 1)[:, None]
    new_means = mean + ((steps + 1.0) / (steps + n + 1.0))[:, None] * (roll - mean)
    means_off = np.vstack([mean[None, :], new_means[:-1]])
    d = X - means_off
    Bfull = ((n + steps) / (n + steps + 1.0))[:, None, None] * (d[:, :, None] * d[:, None, :])
    cov = (n - 1.0) / (n + max(1, nb - 1.0)) * C + Bfull.sum(axis=0) / (n + max(1, nb - 1.0))
    _, V = eigh(cov, subset_by_index=[p - k, p - 1])
    dp = X @ V - means_off @ V
    Bp = (1.0 / (n + steps + 1.0))[:, None, None] * (dp[:, :, None] * dp[:, None, :])
    M = V.T @ C @ V
    out = []
    for i in range(nb):
        if i > 0:
            M = (n + i - 2.0) / (n + i - 1.0) * M + Bp[i - 1]
        out.append(dp[i] @ np.linalg.inv(M) @ dp[i])
    return np.array(out)


def test_mahalanobis_batch_scores_match_explicit_inverse():
    det = OutlierMahalanobis(threshold=10, n_components=3, start_clip=10 ** 9, device=-1)
    rng = np.random.default_rng(1)
    for _ in range(30):
        det.predict(rng.normal(size=(2, 6)), [])
    for nb in [1, 5, 17]:
        X = rng.normal(size=(nb, 6))
        before = {"n": det.n, "mean": np.array(det.mean), "C": np.array(det.C), "k": 3}
        det.predict(X.copy(), [])
        np.testing.assert_allclose(det.score, _oracle_scores(before, X), rtol=1e-8)


def test_mahalanobis_flags_far_points_and_metrics():
    det = OutlierMahalanobis(threshold=15, n_components=2, device=-1)
    rng = np.random.default_rng(1)
    for _ in range(10):
        det.predict(rng.normal(size=(20, 4)), [])
    p = det.predict(np.vstack([rng.normal(size=(5, 4)), np.full((1, 4), 12.0)]), [])
    assert p[-1] == 1 and p[:5].sum() <= 1
    m = {x["key"] for x in det.metrics()}
    assert {"is_outlier", "outlier_score", "observation", "threshold"} <= m


def test_isolation_forest_detector_matches_sklearn():
    from sklearn.ensemble import IsolationForest

    rng = np.random.default_rng(2)
    clf = IsolationForest(n_estimators=50, random_state=0).fit(rng.normal(size=(500, 5)))
    det = OutlierIsolationForest(threshold=0.0, model=clf, device=-1)
    X = np.vstack([rng.normal(size=(30, 5)), rng.normal(size=(3, 5)) * 8])
    pred = det.predict(X, [])
    np.testing.assert_allclose(det.decision_val, clf.decision_function(X), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(pred, (clf.decision_function(X) < 0).astype(int))


def test_isolation_forest_from_npz(tmp_path):
    rng = np.random.default_rng(3)
    np.savez(tmp_path / "if.npz", X=rng.normal(size=(200, 4)))
    det = OutlierIsolationForest(load_path=str(tmp_path) + "/", device=-1)
    assert det.predict(rng.normal(size=(4, 4)), []).shape == (4,)


def test_vae_detector_random_and_feedback_metrics():
    det = OutlierVAE.random(n_features=10, hidden_layers=2, latent_dim=2, threshold=0.5, reservoir_size=50,
                            device=-1)
    rng = np.random.default_rng(4)
    X = rng.random(size=(1, 10))
    det.transform_input(X, [])
    assert det.tags()["outlier-predictions"] in ([0], [1])
    det.send_feedback(X, [], 0.0, np.array([1]))
    det.predict(rng.random(size=(1, 10)), [])
    keys = [m["key"] for m in det.metrics()]
    assert keys[:5] == ["is_outlier", "mse", "observation", "threshold", "label"]
    assert len(keys) == 23
    for _ in range(60):  # the reservoir starts refreshing the scaling stats once full
        det.predict(rng.random(size=(1, 10)), [])
    assert det.N == 62 and len(det.batch) == 50


def test_vae_weights_roundtrip(tmp_path):
    from seldon_core_amd.components.outlier import load_vae_weights, random_vae_weights, save_vae_weights

    w = random_vae_weights(8, hidden_layers=1, latent_dim=2)
    save_vae_weights(str(tmp_path / "vae.npz"), w)
    det = OutlierVAE(load_path=str(tmp_path) + "/", device=-1)
    w2 = load_vae_weights(str(tmp_path / "vae.npz"))
    assert w2["latent"] == 2 and len(w2["encoder"]) == len(w["encoder"])
    assert det.predict(np.random.default_rng(0).random(size=(3, 8)), []).shape == (3,)


def test_vae_in_graph_as_input_transformer():
    det = OutlierVAE.random(n_features=4, threshold=0.1, device=-1)
    from seldon_core_amd.models import iris_logistic_regression

    spec = {"name": "p", "componentSpecs": [{"spec": {"containers": []}}],
            "graph": {"name": "od", "type": "TRANSFORMER", "children": [{"name": "clf", "type": "MODEL"}]}}
    dep = sca.Deployment(spec, components={"od": det, "clf": iris_logistic_regression()}, device=-1)
    try:
        out = dep.predict({"data": {"ndarray": [[5.1, 3.5, 1.4, 0.2]]}})
        assert "outlier-predictions" in out["meta"]["tags"]
        assert len(out["data"]["ndarray"][0]) == 3
        assert "mse" in {m["key"] for m in out["meta"]["metrics"]}
    finally:
        dep.close()


def test_performance_helper():
    scores = performance([0, 1, 1, 0], [0, 1, 0, 0])
    assert scores[:4] == [2, 0, 1, 1] and scores[4] == 0.75


def test_seq2seq_cpu_shapes_and_threshold():
    det = OutlierSeq2SeqLSTM(threshold=0.5, timesteps=6, n_features=3, encoder_dim=(4,), decoder_dim=(8,),
                             device=-1)
    X = np.random.default_rng(5).random(size=(4, 6 * 3))
    p = det.predict(X, [])
    assert p.shape == (4,) and det.mse.shape == (4,) and (det.mse > 0).all()


def test_registered_native_implementations():
    from seldon_core_amd.components import NATIVE_IMPLEMENTATIONS

    for k in ("MAHALANOBIS_OD", "ISOLATION_FOREST_OD", "VAE_OD", "SEQ2SEQ_OD", "EPSILON_GREEDY",
              "THOMPSON_SAMPLING", "MEAN_TRANSFORMER"):
        assert k in NATIVE_IMPLEMENTATIONS


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_mahalanobis_gpu_recurrence_matches_numpy():
    rng = np.random.default_rng(6)
    cpu = OutlierMahalanobis(threshold=10, n_components=4, device=-1)
    gpu = OutlierMahalanobis(threshold=10, n_components=4, device=0)
    for nb in [1, 3, 300, 64, 1000]:
        X = rng.normal(size=(nb, 9))
        cpu.predict(X.copy(), [])
        gpu.predict(X.copy(), [])
        np.testing.assert_allclose(gpu.score, cpu.score, rtol=1e-8, atol=1e-10)


@pytest.mark.gpu
def test_mahalanobis_tracking_crosses_refresh():
    """2,100 one-row steps at p = 20 (the 256-thread kernel): every 1,024th
    tracked step re-orthogonalises the basis with a Newton-Schulz step inside
    the tracked update (no cold Jacobi re-solve on the request path any more:
    only the seed solves by Jacobi), and the scores stay on numpy's."""
    rng = np.random.default_rng(12)
    cpu = OutlierMahalanobis(n_components=3, device=-1)
    gpu = OutlierMahalanobis(n_components=3, device=0)
    for i in range(2100):
        X = rng.normal(size=(1, 20))
        cpu.predict(X.copy(), [])
        gpu.predict(X.copy(), [])
        np.testing.assert_allclose(gpu.score, cpu.score, rtol=1e-6, atol=1e-9)
    ss = gpu._dev.solver_stats()
    assert ss["jacobi_solves"] == 1 and ss["rank1_steps"] >= 2098, ss
    st = gpu.state_dict()
    np.testing.assert_allclose(st["C"], cpu.C, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [7, 40])
def test_mahalanobis_device_multirow_tracking_parity(p):
    """Requests of 1-16 rows: each row one rank-1 update of the tracked
    eigendecomposition, the residual checked after the last; requests of more
    rows (20) re-solve by Jacobi.  Scores and state match numpy over 300
    requests."""
    rng = np.random.default_rng(11)
    cpu = OutlierMahalanobis(n_components=3, device=-1)
    gpu = OutlierMahalanobis(n_components=3, device=0)
    scale = np.linspace(0.5, 2.0, p)
    for i in range(300):
        nb = [1, 2, 5, 16, 20][i % 5]
        X = rng.normal(size=(nb, p)) * scale
        cpu.predict(X.copy(), [])
        gpu.predict(X.copy(), [])
        np.testing.assert_allclose(gpu.score, cpu.score, rtol=1e-6, atol=1e-9)
    ss = gpu._dev.solver_stats()
    assert ss["rank1_steps"] > 150, ss
    st = gpu.state_dict()
    np.testing.assert_allclose(st["C"], cpu.C, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("p,k,start_clip,max_n,path", [(9, 3, 50, -1, "rank1"), (20, 4, 10, 300, "rank1"),
                                                       (5, 5, 50, -1, "rank1"), (64, 3, 100, -1, "rank1"),
                                                       (41, 2, 50, -1, "rank1"),
                                                       (9, 3, 50, -1, "jacobi"), (32, 3, 50, -1, "jacobi"),
                                                       (9, 3, 50, -1, "householder"), (64, 3, 100, -1, "householder"),
                                                       (41, 2, 50, -1, "householder")])
def test_mahalanobis_device_state_parity_over_1000_requests(p, k, start_clip, max_n, path, monkeypatch):
    """Whole _get_preds on the device for 1-row requests: state (mean, C, n,
    clip) within 1e-9 of the numpy path over a 1,000-request stream (VERDICT
    r1 next-round #6), scores to 1e-6.  "rank1" (default) tracks the
    eigendecomposition by rank-1 secular updates, Jacobi seeding it and
    re-solving every 256 steps; "jacobi" forces the warm-started Jacobi path;
    "householder" the tridiagonalisation path (p = 64 and, with the
    threshold lowered, p = 41 run its 4-wave sweep)."""
    if p == 41:
        monkeypatch.setenv("SCA_MAHA_MW_MIN_P", "32")
    if path in ("jacobi", "householder"):
        monkeypatch.setenv("SCA_MAHA_RANK1_MAX_P", "0")
    if path == "householder":
        monkeypatch.setenv("SCA_MAHA_JACOBI_MAX_P", "0")
    rng = np.random.default_rng(p)
    cpu = OutlierMahalanobis(threshold=10, n_components=k, start_clip=start_clip, max_n=max_n, device=-1)
    gpu = OutlierMahalanobis(threshold=10, n_components=k, start_clip=start_clip, max_n=max_n, device=0)
    scale = np.linspace(0.5, 3.0, p)
    scores_c, scores_g = [], []
    for i in range(1000):
        X = rng.normal(size=(1, p)) * scale + (5.0 if i % 97 == 0 else 0.0)  # a few outliers
        cpu.predict(X.copy(), [])
        gpu.predict(X.copy(), [])
        scores_c.append(cpu.score[0])
        scores_g.append(gpu.score[0])
    assert gpu._dev is not None
    ss = gpu._dev.solver_stats()
    if path == "rank1":  # most steps tracked (rank-deficient early steps and 256-step refreshes re-solve)
        assert ss["rank1_steps"] > 500, ss
    else:
        assert ss["rank1_steps"] == 0, ss
    st = gpu.state_dict()
    np.testing.assert_allclose(st["mean"], cpu.mean, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(st["C"], cpu.C, rtol=1e-9, atol=1e-12)
    assert st["n"] == cpu.n == 1000
    np.testing.assert_allclose(st["clip"][0], cpu.clip[0], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(st["clip"][1], cpu.clip[1], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(scores_g, scores_c, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_mahalanobis_device_checkpoint_roundtrip():
    rng = np.random.default_rng(1)
    a = OutlierMahalanobis(n_components=3, device=0)
    for _ in range(20):
        a.predict(rng.normal(size=(2, 7)), [])
    st = a.state_dict()
    b = OutlierMahalanobis(n_components=3, device=0)
    b.load_state_dict(st)
    X = rng.normal(size=(3, 7))
    a.predict(X.copy(), [])
    b.predict(X.copy(), [])
    np.testing.assert_allclose(a.score, b.score, rtol=1e-12)


@pytest.mark.gpu
def test_vae_and_isolation_forest_on_gpu():
    from sklearn.ensemble import IsolationForest

    rng = np.random.default_rng(7)
    clf = IsolationForest(n_estimators=100, random_state=0).fit(rng.normal(size=(400, 6)))
    det = OutlierIsolationForest(model=clf, device=0)
    X = rng.normal(size=(50, 6))
    det.predict(X, [])
    np.testing.assert_allclose(det.decision_val, clf.decision_function(X), rtol=1e-5, atol=1e-6)
    vae = OutlierVAE.random(n_features=30, hidden_layers=2, latent_dim=3, device=0)
    p = vae.predict(rng.random(size=(40, 30)), [])
    assert p.shape == (40,) and np.isfinite(vae.mse).all()


@pytest.mark.gpu
def test_seq2seq_gpu_kernel_matches_cpu():
    cpu = OutlierSeq2SeqLSTM(timesteps=8, n_features=3, encoder_dim=(5,), decoder_dim=(10,), device=-1, seed=3)
    gpu = OutlierSeq2SeqLSTM(timesteps=8, n_features=3, encoder_dim=(5,), decoder_dim=(10,), device=0, seed=3)
    X = np.random.default_rng(8).random(size=(6, 8, 3))
    a = cpu.net.mse(X)
    b = gpu.net.mse(X)  # native LSTM kernel
    c = gpu.net.mse(X)
    np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-7)
    np.testing.assert_array_equal(b, c)
    gpu.net.close()


# ------------------------------------------------- native Mahalanobis model
def _maha_stream(rng, p, sizes, scale=None):
    scale = np.linspace(0.5, 3.0, p) if scale is None else scale
    return [rng.normal(size=(nb, p)) * scale + (4.0 if i % 7 == 3 else 0.0) for i, nb in enumerate(sizes)]


@pytest.mark.parametrize("p,k,start_clip,max_n", [(9, 3, 50, -1), (6, 6, 10, 40), (1, 1, 5, -1)])
def test_mahalanobis_native_host_step_matches_numpy(p, k, start_clip, max_n):
    """The C++ host step (csrc/gpu/maha_device.cc: maha_step_host, the device
    -1 path of the segmented model) against the numpy oracle: scores and the
    final state over requests of 1-200 rows, through clipping and max_n."""
    from seldon_core_amd._native import native

    C = native()
    rng = np.random.default_rng(p + k)
    ref = OutlierMahalanobis(threshold=10, n_components=k, start_clip=start_clip, max_n=max_n, device=-1)
    rm = C.mahalanobis_model(p, k, 3.0, float(start_clip), float(max_n), 1e-8, out_mode=0)
    for X in _maha_stream(rng, p, [1, 1, 3, 60, 1, 200, 2, 1, 17]):
        ref.predict(X.copy(), [])
        got = rm.run_cpu(X).ravel()
        np.testing.assert_allclose(got, ref.score, rtol=1e-7, atol=1e-9)
    st = np.asarray(C.mahalanobis_state(rm))
    np.testing.assert_allclose(st[:p], ref.mean, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(st[p:p + p * p].reshape(p, p), ref.C, rtol=1e-10, atol=1e-12)
    assert int(st[-3]) == ref.n


def test_mahalanobis_row_model_predictions_share_state():
    """row_model(): the reference predict() output (score > threshold, 1-D)
    from the native unit; it shares the component's state, so state_dict()
    sees the requests the native node served."""
    rng = np.random.default_rng(3)
    det = OutlierMahalanobis(threshold=8, n_components=2, n_features=4, device=-1)
    ref = OutlierMahalanobis(threshold=8, n_components=2, device=-1)
    rm = det.row_model()
    assert rm is not None and rm.flat_output
    for X in _maha_stream(rng, 4, [5, 1, 30, 2]):
        want = ref.predict(X.copy(), [])
        np.testing.assert_array_equal(rm.run_cpu(X).ravel(), want)
    st = det.state_dict()
    assert st["n"] == ref.n == 38
    np.testing.assert_allclose(st["C"], ref.C, rtol=1e-10)
    assert OutlierMahalanobis(n_components=2, device=-1).row_model() is None  # p unknown


@pytest.mark.gpu
def test_mahalanobis_segmented_launch_matches_sequential_steps():
    """maha_step_segments: one launch over 6 requests = 6 sequential steps
    (host oracle), for scores and predictions."""
    import torch

    from seldon_core_amd._native import native

    C = native()
    p, k = 9, 3
    rng = np.random.default_rng(11)
    reqs = _maha_stream(rng, p, [1, 4, 1, 57, 2, 1] * 12)
    host = C.mahalanobis_model(p, k, 3.0, 50.0, -1.0, 1e-8, out_mode=0)
    want = np.concatenate([host.run_cpu(X).ravel() for X in reqs])
    X = torch.tensor(np.concatenate(reqs), dtype=torch.float64, device="cuda")
    seg = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in reqs])]), dtype=torch.int32, device="cuda")
    for mode, thr in ((0, 0.0), (1, 10.0)):
        state = torch.zeros(p * (p + 3) + 3, dtype=torch.float64, device="cuda")
        state[-2] = 1.0  # c_zero
        ws = torch.zeros(60 * (4 * p + 2 * k), dtype=torch.float64, device="cuda")
        out = torch.full((X.shape[0],), -1.0, dtype=torch.float64, device="cuda")
        eig = torch.zeros(64 * 64 + 15, dtype=torch.float64, device="cuda")  # cold start, then warm
        C.kernels.maha_step_segments(X.data_ptr(), seg.data_ptr(), len(reqs), p, k, 3.0, 50.0, -1.0, 1e-8, mode, thr,
                                     state.data_ptr(), eig.data_ptr(), ws.data_ptr(), out.data_ptr(), 0)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        if mode == 0:
            np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)
            st = state.cpu().numpy()
            np.testing.assert_allclose(st, np.asarray(C.mahalanobis_state(host)), rtol=1e-9, atol=1e-12)
        else:
            close = np.abs(want - thr) < 1e-6 * max(1.0, thr)
            np.testing.assert_array_equal(got[~close], (want[~close] > thr).astype(float))


@pytest.mark.gpu
def test_mahalanobis_device_concurrent_callers_share_launches():
    """Concurrent step() callers go through the batcher: every request is
    stepped exactly once (n = total rows) in fewer launches than requests, and
    the order-independent state (running mean / covariance before clipping)
    matches the numpy path on all rows."""
    import threading

    from seldon_core_amd._native import native

    p, k = 12, 3
    dev = native().MahalanobisDevice(p, k, 3.0, 1e12, -1.0, 1e-8, 0)
    rng = np.random.default_rng(5)
    data = [rng.normal(size=(1, p)) * np.linspace(1, 2, p) for _ in range(1600)]
    errs = []

    seqs = {}

    def worker(t):
        try:
            for i in range(t, len(data), 16):
                sc, seq = dev.step_seq(data[i])
                assert sc.shape == (1,)
                seqs[i] = seq
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs and not any(t.is_alive() for t in th)
    st = np.asarray(dev.state())
    assert int(st[-3]) == 1600
    b = dev.batches()
    assert b["requests"] == 1600 and b["batches"] < 1600
    allX = np.concatenate(data)
    np.testing.assert_allclose(st[:p], allX.mean(0), rtol=1e-9, atol=1e-12)
    # the running covariance depends on the arrival order (the reference's
    # recursion uses the running mean at each step), so the oracle replays
    # numpy in the order the device applied the requests (step_seq): every
    # request exactly once, at distinct positions 0..1599, and C equal to
    # the reference recursion in that order
    order = sorted(seqs, key=seqs.get)
    assert sorted(seqs.values()) == list(range(1600))
    ref = OutlierMahalanobis(n_components=k, start_clip=10 ** 12, device=-1)
    for i in order:
        ref.predict(data[i].copy(), [])
    Cg = st[p:p + p * p].reshape(p, p)
    np.testing.assert_allclose(Cg, Cg.T, rtol=0, atol=1e-15)
    np.testing.assert_allclose(Cg, ref.C, rtol=0, atol=1e-9)


def test_mahalanobis_python_and_native_entry_points_do_not_lose_steps():
    """the Python path pulls the shared state, steps on the host
    and pushes it back; native steps of the graph node (row_model) landing in
    between used to be overwritten.  Under the state lock every row of both
    entry points is counted (CPU placement: both paths step the host state)."""
    import threading

    rng = np.random.default_rng(21)
    det = OutlierMahalanobis(n_components=3, n_features=6, device=-1)
    rm = det.row_model()
    assert rm is not None
    X_py = [rng.normal(size=(2, 6)) for _ in range(150)]
    X_nat = [rng.normal(size=(3, 6)) for _ in range(150)]

    def python_side():
        for X in X_py:
            det.predict(X, [])

    def native_side():
        for X in X_nat:
            rm.run_cpu(X)

    th = [threading.Thread(target=python_side), threading.Thread(target=native_side)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    det._pull_state()
    assert det.n == 2 * 150 + 3 * 150, det.n
