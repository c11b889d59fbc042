"""Numerics of the hand-written gfx950 kernels vs plain PyTorch references.

Each kernel is launched directly (raw device pointers + the current torch
stream) and compared with an fp32/fp64 PyTorch implementation of the same op.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("rows,K,C,act", [(1, 4, 3, 1), (7, 4, 3, 1), (300, 4, 3, 1), (64, 30, 1, 2),
                                          (129, 64, 10, 3), (50, 200, 40, 1), (33, 5, 6, 0), (17, 8, 5, 4)])
def test_linear_f64(C_, rows, K, C, act):
    g = torch.Generator().manual_seed(rows * 31 + K)
    X = torch.randn(rows, K, dtype=torch.float64, generator=g).to(dev)
    W = torch.randn(C, K, dtype=torch.float64, generator=g).to(dev)
    b = torch.randn(C, dtype=torch.float64, generator=g).to(dev)
    out_cols = 2 if act == 2 else C
    out = torch.empty(rows, out_cols, dtype=torch.float64, device=dev)
    C_.kernels.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, act, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    z = X @ W.T + b
    if act == 0:
        ref = z
    elif act == 1:
        ref = torch.softmax(z, dim=1)
    elif act == 2:
        p = torch.sigmoid(z[:, 0])
        ref = torch.stack([1 - p, p], dim=1)
    elif act == 3:
        s = torch.sigmoid(z)
        ref = s / s.sum(dim=1, keepdim=True)
    else:
        ref = torch.sigmoid(z)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)


def _linear_ref(X, W, b, act):
    z = X @ W.T + b
    if act == 0:
        return z
    if act == 1:
        return torch.softmax(z, dim=1)
    if act == 2:
        p = torch.sigmoid(z[:, 0])
        return torch.stack([1 - p, p], dim=1)
    if act == 3:
        s = torch.sigmoid(z)
        return s / s.sum(dim=1, keepdim=True)
    return torch.sigmoid(z)


@pytest.mark.parametrize("rows,K,C,act", [(4096, 784, 10, 1), (8192, 256, 1000, 1), (64, 30, 1, 2),
                                          (1000, 37, 70, 3), (513, 100, 33, 0), (300, 17, 500, 4),
                                          (16, 4, 3, 1), (2048, 64, 1024, 1)])
@pytest.mark.parametrize("mode", ["auto", "forced"])
def test_linear_mfma_f64(C_, monkeypatch, rows, K, C, act, mode):
    """The f64 matrix-core path (v_mfma_f64_16x16x4, fused bias + activation)
    at the VERDICT r5 shapes -- (4096, 784, 10), (8192, 256, 1000), (64, 30, 1)
    -- and ragged ones (K not a multiple of 4 or 16, C not of 16, rows not of
    16), against torch fp64 at 1e-12.  'forced' runs every shape on it."""
    if mode == "forced":
        monkeypatch.setenv("SCA_LINEAR_MFMA", "2")
    expect = mode == "forced" or rows * K * C >= (1 << 20)
    assert C_.kernels.linear_uses_mfma(rows, K, C) == expect
    g = torch.Generator().manual_seed(rows * 7 + K * 3 + C)
    X = torch.randn(rows, K, dtype=torch.float64, generator=g).to(dev)
    W = (torch.randn(C, K, dtype=torch.float64, generator=g) / K ** 0.5).to(dev)
    b = torch.randn(C, dtype=torch.float64, generator=g).to(dev)
    out_cols = 2 if act == 2 else C
    out = torch.full((rows, out_cols), float("nan"), dtype=torch.float64, device=dev)
    C_.kernels.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, act, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(out, _linear_ref(X, W, b, act), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("variant", range(1, 7))
@pytest.mark.parametrize("rows,K,C,act", [(4096, 784, 10, 1), (97, 789, 20, 3), (33, 1030, 1, 2), (700, 3072, 7, 0)])
def test_linear_mfma_narrow_split_variants(C_, monkeypatch, variant, rows, K, C, act):
    """Every K-slice / chunk-group variant of the narrow MFMA tiles (1-2 class
    tiles; SCA_LINEAR_MFMA_SPLIT forces one) equals torch fp64 at 1e-12,
    including K not a multiple of 4 (scalar loads) and fewer rows than one
    16-row tile per slice."""
    monkeypatch.setenv("SCA_LINEAR_MFMA", "2")
    monkeypatch.setenv("SCA_LINEAR_MFMA_SPLIT", str(variant))
    g = torch.Generator().manual_seed(variant * 1000 + rows + K + C)
    X = torch.randn(rows, K, dtype=torch.float64, generator=g).to(dev)
    W = (torch.randn(C, K, dtype=torch.float64, generator=g) / K ** 0.5).to(dev)
    b = torch.randn(C, dtype=torch.float64, generator=g).to(dev)
    out = torch.full((rows, 2 if act == 2 else C), float("nan"), dtype=torch.float64, device=dev)
    C_.kernels.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, act, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(out, _linear_ref(X, W, b, act), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("rows,K,C", [(8192, 256, 1000), (257, 33, 257), (1000, 100, 1024), (4099, 7, 700),
                                      (300, 512, 385)])
def test_linear_wide_softmax_split_tiles(C_, monkeypatch, rows, K, C):
    """Wide softmax (C > 256) on 64-row x 128-class tiles, with the in-kernel
    last-arriver fold (SCA_LINEAR_WIDE=1) and with the rescale launch (2):
    both equal torch fp64 at 1e-12 and the one-workgroup-per-row-tile kernel
    (0), with ragged rows / classes / K."""
    monkeypatch.setenv("SCA_LINEAR_MFMA", "2")
    g = torch.Generator().manual_seed(rows + K + C)
    X = torch.randn(rows, K, dtype=torch.float64, generator=g).to(dev)
    W = (torch.randn(C, K, dtype=torch.float64, generator=g) / K ** 0.5 * 3).to(dev)
    b = torch.randn(C, dtype=torch.float64, generator=g).to(dev)
    outs = []
    for wide in ("1", "0", "2"):
        monkeypatch.setenv("SCA_LINEAR_WIDE", wide)
        out = torch.full((rows, C), float("nan"), dtype=torch.float64, device=dev)
        for _ in range(2):  # the second launch reuses nothing stale (counters / scratch are per launch)
            C_.kernels.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, 1, out.data_ptr(), _stream())
        torch.cuda.synchronize()
        outs.append(out)
    ref = _linear_ref(X, W, b, 1)
    torch.testing.assert_close(outs[0], ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-12, atol=1e-14)
    torch.testing.assert_close(outs[2], ref, rtol=1e-12, atol=1e-12)


def test_linear_wide_softmax_concurrent_streams(C_, monkeypatch):
    """Launches on different streams at once each get their own scratch."""
    monkeypatch.setenv("SCA_LINEAR_MFMA", "2")
    monkeypatch.setenv("SCA_LINEAR_WIDE", "1")
    rows, K, C = 2048, 128, 900
    g = torch.Generator().manual_seed(7)
    W = (torch.randn(C, K, dtype=torch.float64, generator=g) / K ** 0.5).to(dev)
    b = torch.randn(C, dtype=torch.float64, generator=g).to(dev)
    streams = [torch.cuda.Stream() for _ in range(4)]
    Xs = [torch.randn(rows, K, dtype=torch.float64, generator=g).to(dev) for _ in streams]
    outs = [torch.empty(rows, C, dtype=torch.float64, device=dev) for _ in streams]
    torch.cuda.synchronize()
    for _ in range(3):
        for st, X, out in zip(streams, Xs, outs):
            C_.kernels.linear_f64(X.data_ptr(), rows, K, W.data_ptr(), b.data_ptr(), C, 1, out.data_ptr(),
                                  st.cuda_stream)
    torch.cuda.synchronize()
    for X, out in zip(Xs, outs):
        torch.testing.assert_close(out, _linear_ref(X, W, b, 1), rtol=1e-12, atol=1e-12)


def test_iris_headline_shape_stays_on_the_thread_kernel(C_):
    for rows in (1, 14, 256, 4096):
        assert not C_.kernels.linear_uses_mfma(rows, 4, 3)


@pytest.fixture(scope="module")
def C_():
    from seldon_core_amd import native

    return native()


@pytest.mark.parametrize("rows", [1, 3, 64, 1000, 4096])
def test_tree_perfect_vs_cpu(C_, rows):
    from seldon_core_amd.models import synthetic_xgboost, to_row_model

    ens = synthetic_xgboost(200, 8, 16, seed=rows)
    rm = to_row_model(ens)
    unit = C_.BatchedUnit(rm, 0, max_batch=8192)
    try:
        X = np.random.default_rng(rows).standard_normal((rows, 16))
        X[0, 3] = np.nan  # exercise default direction
        got = unit.run(X)
        ref = ens.predict(X)
        np.testing.assert_allclose(np.asarray(got).reshape(ref.shape), ref, rtol=2e-5, atol=2e-5)
    finally:
        unit.stop()


@pytest.mark.parametrize("trees,depth,F,rows", [(50, 11, 10, 37), (100, 6, 300, 70), (64, 10, 20, 5),
                                               (64, 10, 20, 900), (300, 3, 8, 2000)])
def test_tree_geometries(C_, trees, depth, F, rows):
    """LDS-staged trees (depth <= 10), global-memory trees (depth 11), wide
    features without an LDS tile, fused and two-pass reduces."""
    from seldon_core_amd.models import synthetic_xgboost, to_row_model

    ens = synthetic_xgboost(trees, depth, F, seed=depth * 7 + F)
    unit = C_.BatchedUnit(to_row_model(ens), 0, max_batch=4096)
    try:
        X = np.random.default_rng(rows).standard_normal((rows, F))
        X[::7, 1] = np.nan
        np.testing.assert_allclose(np.asarray(unit.run(X)).reshape(-1), ens.predict(X).reshape(-1),
                                   rtol=2e-5, atol=2e-5)
    finally:
        unit.stop()


def test_tree_fused_reduce_many_batches(C_):
    """Fused last-workgroup reduce: many back-to-back launches of varying
    size from concurrent callers (several slots, one counter each) must all
    match, i.e. the counter is rearmed and no slab value is read stale."""
    import concurrent.futures as cf

    from seldon_core_amd.models import synthetic_xgboost, to_row_model

    ens = synthetic_xgboost(1000, 8, 32, seed=11)
    d = ens.device_spec()
    d["fused_reduce"] = True
    unit = C_.BatchedUnit(C_.tree_model(d), 0, max_batch=1024, slots=4)
    rng = np.random.default_rng(5)
    Xs = [rng.standard_normal((n, 32)) for n in list(range(1, 41)) * 3 + [64, 128, 300]]
    try:
        with cf.ThreadPoolExecutor(8) as ex:
            outs = list(ex.map(unit.run, Xs))
        for X, got in zip(Xs, outs):
            np.testing.assert_allclose(np.asarray(got).reshape(-1), ens.predict(X).reshape(-1), rtol=2e-5, atol=2e-5)
    finally:
        unit.stop()


def test_tree_lds_staging_matches_global(C_):
    """Trees staged in LDS by global_load_lds (kernel option) == traversal from
    global memory, for odd chunk starts (dword copy path) and 16-B aligned."""
    D, F, T = 6, 12, 90
    ni = (1 << D) - 1
    g = torch.Generator().manual_seed(3)
    nodes = torch.stack([torch.randn(T * ni, generator=g).view(torch.int32),
                         torch.randint(0, F, (T * ni,), generator=g, dtype=torch.int32)], 1).contiguous().to(dev)
    leaves = torch.randn(T * (ni + 1), generator=g).to(dev)
    for rows in (1, 9, 100):
        X = torch.randn(rows, F, dtype=torch.float64, generator=g).to(dev)
        rb = min(64, 1 << (rows - 1).bit_length())
        outs = []
        for begin, lds in (([0, 7, 23, 40, 41, 64, 90], 32), ([0, 16, 32, 48, 64, 80, 90], 16),
                           ([0, 7, 23, 40, 41, 64, 90], 0)):
            b = torch.tensor(begin, dtype=torch.int32, device=dev)
            nc = len(begin) - 1
            part = torch.empty(nc * rows, dtype=torch.float64, device=dev)  # fp64 slab
            C_.kernels.tree_perfect_partial(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), D, 0,
                                            b.data_ptr(), nc, rb, part.data_ptr(), _stream(), lds)
            torch.cuda.synchronize()
            outs.append(part.view(nc, rows).double().sum(0))
        torch.testing.assert_close(outs[0], outs[2], rtol=0, atol=0)
        torch.testing.assert_close(outs[1], outs[2], rtol=1e-6, atol=1e-5)


def test_tree_scores_do_not_depend_on_the_batch(C_):
    """The chunk plan follows the batch size; fp64 partial sums of the fp32
    leaves make every plan add up to the same bits, so a row scores the same
    alone or inside a 4096-row batch (the bench's sampled reply check relies
    on it)."""
    from seldon_core_amd.models import to_row_model
    from seldon_core_amd.models.trees import synthetic_xgboost

    ens = synthetic_xgboost(1000, 8, 32, seed=4)
    unit = C_.BatchedUnit(to_row_model(ens), 0, max_batch=4096)
    try:
        rng = np.random.default_rng(9)
        X = rng.normal(size=(4096, 32))
        big = np.asarray(unit.run(X)).ravel()
        for i in (0, 1, 777, 4095):
            alone = np.asarray(unit.run(X[i:i + 1])).ravel()
            assert alone[0] == big[i]
        mid = np.asarray(unit.run(X[100:164])).ravel()
        assert (mid == big[100:164]).all()
    finally:
        unit.stop()


@pytest.mark.parametrize("depth", [4, 8, 10, 12])
@pytest.mark.parametrize("transform", [0, 3])
def test_tree_whole_kernel_matches_chunked_and_cpu(C_, depth, transform):
    """Single-launch whole-ensemble kernel (batches <= whole_max_rows) vs the
    chunked two-kernel plan vs the host walker, over batch sizes that cross
    every rows-per-block choice; NaNs take the default direction."""
    from seldon_core_amd.models import synthetic_xgboost

    ens = synthetic_xgboost(700 if depth < 12 else 60, depth, 24, seed=depth + 10 * transform)
    d = ens.device_spec()
    d["transform"] = transform
    d["out_cols"] = 2 if transform == 3 else 1
    whole = C_.tree_model(dict(d, whole_max_rows=256))
    chunked = C_.tree_model(dict(d, whole_max_rows=0))
    uw, uc = C_.BatchedUnit(whole, 0, max_batch=512), C_.BatchedUnit(chunked, 0, max_batch=512)
    try:
        rng = np.random.default_rng(depth)
        for n in (1, 2, 3, 5, 16, 17, 64, 65, 200, 256):
            X = rng.standard_normal((n, 24))
            X[::5, 2] = np.nan
            a, b = np.asarray(uw.run(X)), np.asarray(uc.run(X))
            np.testing.assert_allclose(a, b, rtol=1e-13, atol=1e-13)
            np.testing.assert_allclose(a.reshape(-1), whole.run_cpu(X).reshape(-1), rtol=2e-5, atol=2e-5)
    finally:
        uw.stop()
        uc.stop()


def test_tree_wide_leaf_range_is_nearly_order_free(C_):
    """Leaves spanning ~40 binades (late trees' leaves scaled by 2^-40): the
    fp64 sums may now round differently under another chunk plan, so a row's
    score alone and inside a 4096-row batch agree to fp64 rounding rather than
    bit for bit (the claim is 'nearly order-free')."""
    from seldon_core_amd.models import synthetic_xgboost

    ens = synthetic_xgboost(1000, 8, 32, seed=21)
    d = ens.device_spec()
    leaves = np.asarray(d["leaves"], dtype=np.float32).reshape(1000, -1).copy()
    leaves[500:] *= np.float32(2.0 ** -40)
    d["leaves"] = leaves.ravel()
    unit = C_.BatchedUnit(C_.tree_model(d), 0, max_batch=4096)
    try:
        X = np.random.default_rng(2).normal(size=(4096, 32))
        big = np.asarray(unit.run(X)).ravel()
        for i in (0, 9, 4095):
            alone = np.asarray(unit.run(X[i:i + 1])).ravel()[0]
            assert abs(alone - big[i]) <= 1e-14 * max(1.0, abs(big[i])), (alone, big[i])
    finally:
        unit.stop()


def test_tree_softmax_groups(C_):
    """multi:softprob-style: 3 groups, softmax transform."""
    from seldon_core_amd.models import to_row_model
    from seldon_core_amd.models.trees import T_SOFTMAX, TreeEnsemble, synthetic_xgboost

    base = synthetic_xgboost(30, 5, 6, seed=3)
    for i, t in enumerate(base.trees):
        t.group = i % 3
    ens = TreeEnsemble(base.trees, 6, 3, 3, T_SOFTMAX, 0, 1.0, [0.1, 0.2, 0.3])
    unit = C_.BatchedUnit(to_row_model(ens), 0)
    try:
        X = np.random.default_rng(0).standard_normal((40, 6))
        np.testing.assert_allclose(unit.run(X), ens.predict(X), rtol=2e-5, atol=2e-6)
    finally:
        unit.stop()


def test_tree_sparse_random_forest(C_):
    from sklearn.datasets import make_classification
    from sklearn.ensemble import RandomForestClassifier

    from seldon_core_amd.models import to_row_model

    X, y = make_classification(n_samples=400, n_features=10, n_informative=6, n_classes=3, random_state=0)
    rf = RandomForestClassifier(n_estimators=20, random_state=0).fit(X, y)  # deep trees -> sparse layout
    rm = to_row_model(rf)
    assert rm.name == "tree_sparse"
    unit = C_.BatchedUnit(rm, 0)
    try:
        got = unit.run(X[:100])
        np.testing.assert_allclose(got, rf.predict_proba(X[:100]), rtol=1e-5, atol=1e-6)
    finally:
        unit.stop()


def test_combine_mean(C_):
    n = 1001
    ins = [torch.randn(n, dtype=torch.float64, device=dev) for _ in range(3)]
    ptrs = torch.tensor([t.data_ptr() for t in ins], dtype=torch.int64, device=dev)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    C_.kernels.combine_mean_f64(ptrs.data_ptr(), 3, n, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(out, (ins[0] + ins[1] + ins[2]) / 3, rtol=1e-14, atol=1e-14)


def test_softmax_argmax_rows(C_):
    x = torch.randn(37, 1000, dtype=torch.float64, device=dev)
    out = torch.empty_like(x)
    idx = torch.empty(37, dtype=torch.int32, device=dev)
    C_.kernels.softmax_rows_f64(x.data_ptr(), 37, 1000, out.data_ptr(), _stream())
    C_.kernels.argmax_rows_f64(x.data_ptr(), 37, 1000, idx.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(out, torch.softmax(x, dim=1), rtol=1e-12, atol=1e-14)
    assert torch.equal(idx.long(), x.argmax(dim=1))


def test_minmax_and_mean_sigmoid(C_):
    x = torch.randn(5000, dtype=torch.float64, device=dev) * 3 + 1
    out = torch.empty_like(x)
    scratch = torch.empty(2, dtype=torch.float64, device=dev)
    C_.kernels.minmax_normalize_f64(x.data_ptr(), x.numel(), out.data_ptr(), scratch.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(out, (x - x.min()) / (x.max() - x.min()), rtol=1e-13, atol=1e-13)
    m = torch.randn(70, 13, dtype=torch.float64, device=dev)
    o = torch.empty(70, dtype=torch.float64, device=dev)
    C_.kernels.mean_sigmoid_rows_f64(m.data_ptr(), 70, 13, 0.25, o.data_ptr(), _stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(o, torch.sigmoid(m.mean(dim=1) - 0.25), rtol=1e-13, atol=1e-13)


def test_eg_route_statistics(C_):
    """|p(best) - (1 - eps)| small (components/routers/epsilon-greedy/test_EpsilonGreedy.py:21-25)."""
    best = torch.tensor([1], dtype=torch.int32, device=dev)
    n = 200000
    out = torch.empty(n, dtype=torch.float64, device=dev)
    C_.kernels.eg_route(best.data_ptr(), 4, 0.1, 1234, 0, n, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    out = out.long()
    p_best = (out == 1).float().mean().item()
    assert abs(p_best - 0.9) < 0.01
    counts = torch.bincount(out.long(), minlength=4).float() / n
    for b in (0, 2, 3):
        assert abs(counts[b].item() - 0.1 / 3) < 0.01


def test_ts_route_prefers_better_arm(C_):
    alpha = torch.tensor([2.0, 50.0, 5.0], dtype=torch.float32, device=dev)
    beta = torch.tensor([50.0, 2.0, 5.0], dtype=torch.float32, device=dev)
    n = 50000
    out = torch.empty(n, dtype=torch.float64, device=dev)
    C_.kernels.ts_route(alpha.data_ptr(), beta.data_ptr(), 3, 99, 0, n, out.data_ptr(), _stream())
    torch.cuda.synchronize()
    out = out.long()
    frac = torch.bincount(out.long(), minlength=3).float() / n
    # P(Beta(50,2) > Beta(5,5)) and > Beta(2,50) is ~1
    assert frac[1].item() > 0.99
    assert out.min().item() >= 0 and out.max().item() <= 2


@pytest.mark.parametrize("trees,depth,F,rows", [(1000, 8, 32, 33), (1000, 8, 32, 100), (1000, 8, 32, 256),
                                               (300, 10, 16, 64), (97, 5, 700, 50), (64, 4, 8, 200)])
def test_tree_tile_kernel_matches_whole(C_, trees, depth, F, rows):
    """Tree-major tiles (opt-in, SCA_TREE_TILE_ROWS): trees staged in LDS per
    row tile, atomic row fold.  Launched directly against the whole-ensemble
    kernel (itself checked against the CPU ensemble above), NaN default
    directions included, twice in a row (the fold re-zeroes its
    accumulators); fp64 sums of fp32 leaves: equal to 1e-12."""
    K = C_.kernels
    g = torch.Generator().manual_seed(trees + depth + F)
    ni = (1 << depth) - 1
    thr = torch.randn(trees * ni, generator=g)
    feat = torch.randint(0, F, (trees * ni,), generator=g, dtype=torch.int32)
    feat[::3] |= torch.tensor(-2 ** 31, dtype=torch.int32)  # default-left bit on a third of the nodes
    nodes = torch.stack([thr.view(torch.int32), feat], 1).contiguous().to(dev)
    leaves = (torch.randn(trees * (ni + 1), generator=g) * 0.01).to(dev)
    s = _stream()
    for rep in range(2):
        X = torch.randn(rows, F, dtype=torch.float64, generator=g)
        X[::5, 0] = float("nan")
        X = X.to(dev)
        ref = torch.empty(rows, dtype=torch.float64, device=dev)
        K.tree_perfect_whole(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), depth, 0, trees, 1, 0, 1.0,
                             0, ref.data_ptr(), 1, s, -1)
        out = torch.full((rows,), float("nan"), dtype=torch.float64, device=dev)
        acc = torch.zeros(rows, dtype=torch.float64, device=dev)
        cnt = torch.zeros(16, dtype=torch.int32, device=dev)
        assert K.tree_perfect_tile(X.data_ptr(), rows, F, nodes.data_ptr(), leaves.data_ptr(), depth, 0, trees, 0,
                                   1.0, 0, out.data_ptr(), 1, acc.data_ptr(), cnt.data_ptr(), s)
        torch.cuda.synchronize()
        torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
        assert float(acc.abs().max()) == 0.0 and int(cnt[0]) == 0
