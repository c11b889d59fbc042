"""Fused MLP / VAE row models: CPU reference path vs sklearn / torch / numpy,
and (GPU) the MFMA kernel vs the same references."""
import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.models import to_row_model
from seldon_core_amd.models.mlp import OUT_SOFTMAX, layer, mlp_row_model, random_dense_stack


def _sk_mlp(kind="clf", n_classes=3, hidden=(37, 19), activation="relu", seed=0):
    from sklearn.neural_network import MLPClassifier, MLPRegressor

    rng = np.random.default_rng(seed)
    X = rng.normal(size=(200, 13))
    if kind == "clf":
        y = rng.integers(0, n_classes, size=200)
        est = MLPClassifier(hidden_layer_sizes=hidden, activation=activation, max_iter=50, random_state=seed)
    else:
        y = X[:, 0] * 2 + X[:, 1]
        est = MLPRegressor(hidden_layer_sizes=hidden, activation=activation, max_iter=50, random_state=seed)
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        est.fit(X, y)
    return est, X


@pytest.mark.parametrize("activation", ["relu", "tanh", "logistic"])
@pytest.mark.parametrize("n_classes", [2, 4])
def test_sklearn_mlp_classifier_cpu(activation, n_classes):
    est, X = _sk_mlp("clf", n_classes, activation=activation)
    rm = to_row_model(est)
    assert rm is not None and rm.name == "mlp"
    np.testing.assert_allclose(rm.run_cpu(X), est.predict_proba(X), rtol=2e-5, atol=2e-6)
    assert rm.class_names() == [str(c) for c in est.classes_]


def test_sklearn_mlp_regressor_cpu():
    est, X = _sk_mlp("reg")
    rm = to_row_model(est, "predict")
    assert rm.flat_output
    np.testing.assert_allclose(rm.run_cpu(X)[:, 0], est.predict(X), rtol=1e-4, atol=1e-5)


def test_torch_sequential_cpu():
    import torch

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(9, 33), torch.nn.ReLU(), torch.nn.Linear(33, 5), torch.nn.Tanh(),
                              torch.nn.Linear(5, 7), torch.nn.Softmax(dim=1))
    rm = to_row_model(net)
    X = np.random.default_rng(0).normal(size=(21, 9))
    with torch.no_grad():
        ref = net(torch.tensor(X, dtype=torch.float32)).double().numpy()
    np.testing.assert_allclose(rm.run_cpu(X), ref, rtol=1e-5, atol=1e-6)


def _vae_layers(F=12, hidden=(8, 6), latent=2, seed=0, logvar_bias=0.0):
    enc = random_dense_stack([F, *hidden], ["relu"] * len(hidden), seed)
    rng = np.random.default_rng(seed + 1)
    head_W = rng.normal(scale=0.3, size=(2 * latent, hidden[-1]))
    head_b = np.concatenate([np.zeros(latent), np.full(latent, logvar_bias)])
    enc.append(layer(head_W, head_b, "identity"))
    dec = random_dense_stack([latent, *hidden[::-1], F], ["relu"] * len(hidden) + ["sigmoid"], seed + 2)
    return enc, dec


def _np_dense(x, layers):
    for L in layers:
        z = x @ L["W"].T.astype(np.float64) + L["b"]
        x = {0: z, 1: np.maximum(z, 0), 2: 1 / (1 + np.exp(-z)), 3: np.tanh(z)}[L["act"]]
    return x


def test_vae_cpu_deterministic_limit():
    """With log_var -> -inf the sample is z_mean: score == MSE of the mean decode."""
    C = sca.native()
    enc, dec = _vae_layers(logvar_bias=-80.0)
    rm = C.vae_model(enc, 2, dec, 10, 7)
    X = np.random.default_rng(3).random(size=(9, 12))
    h = _np_dense(X, enc)
    recon = _np_dense(h[:, :2], dec)
    want = ((recon - X) ** 2).mean(axis=1)
    np.testing.assert_allclose(rm.run_cpu(X)[:, 0], want, rtol=1e-4)


def test_vae_cpu_is_stochastic_and_positive():
    C = sca.native()
    enc, dec = _vae_layers(logvar_bias=0.0)
    rm = C.vae_model(enc, 2, dec, 10, 7)
    X = np.random.default_rng(3).random(size=(5, 12))
    a, b = rm.run_cpu(X), rm.run_cpu(X)
    assert (a > 0).all() and not np.array_equal(a, b)  # fresh MC draws per call


def test_mlp_dispatch_cost_model():
    """Few 16-row tiles of a wide network -> layer-wise; many tiles of a narrow one -> fused."""
    C = sca.native()
    wide = C.mlp_model(random_dense_stack([784, 512, 256, 10], ["relu", "relu", "identity"]), 1)
    narrow = C.mlp_model(random_dense_stack([13, 37, 19, 3], ["relu", "relu", "identity"]), 1)
    assert C.mlp_layerwise(wide, 64) and not C.mlp_layerwise(narrow, 64)
    assert C.mlp_workspace_bytes(wide, 64) >= 2 * 64 * 512 * 4


def test_wide_network_falls_back_to_layerwise():
    """Activations wider than one workgroup's LDS: no fused plan, every batch
    size goes layer-wise and always gets a workspace."""
    C = sca.native()
    layers = random_dense_stack([784, 2048, 10], ["relu", "identity"])
    m = C.mlp_model(layers, 1)
    for rows in (1, 64, 4096):
        assert C.mlp_layerwise(m, rows)
        assert C.mlp_workspace_bytes(m, rows) >= rows * 2048 * 4
    X = np.random.default_rng(0).normal(size=(5, 784))
    h = np.maximum(X @ np.asarray(layers[0]["W"]).T + layers[0]["b"], 0)
    z = h @ np.asarray(layers[1]["W"]).T + layers[1]["b"]
    ref = np.exp(z - z.max(1, keepdims=True))
    ref /= ref.sum(1, keepdims=True)
    np.testing.assert_allclose(m.run_cpu(X), ref, rtol=1e-4, atol=1e-6)


def test_narrow_network_needs_no_workspace():
    C = sca.native()
    narrow = C.mlp_model(random_dense_stack([13, 37, 19, 3], ["relu", "relu", "identity"]), 1)
    assert not any(C.mlp_layerwise(narrow, r) for r in (1, 16, 256, 4096))
    assert C.mlp_workspace_bytes(narrow, 4096) == 0


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fused", "layer"])
@pytest.mark.parametrize("dims", [(13, 37, 19, 3), (784, 256, 64, 10), (5, 1, 2), (64, 128, 128, 64, 33)])
@pytest.mark.parametrize("rows", [1, 16, 37, 300])
def test_mlp_gpu_matches_torch_fp32(dims, rows, mode, monkeypatch):
    import torch

    monkeypatch.setenv("SCA_MLP_MODE", mode)  # read when the model is built
    layers = random_dense_stack(list(dims), ["relu"] * (len(dims) - 2) + ["identity"], seed=len(dims))
    rm = mlp_row_model(layers, OUT_SOFTMAX)
    X = np.random.default_rng(rows).normal(size=(rows, dims[0]))
    unit = sca.native().BatchedUnit(rm, 0)
    try:
        got = unit.run(X)
    finally:
        unit.stop()
    x = torch.tensor(X, dtype=torch.float32)
    for L in layers:
        x = x @ torch.tensor(L["W"]).T + torch.tensor(L["b"])
        if L["act"] == 1:
            x = torch.relu(x)
    ref = torch.softmax(x, 1).double().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fused", "layer"])
def test_vae_gpu_matches_cpu_reference(mode, monkeypatch):
    monkeypatch.setenv("SCA_MLP_MODE", mode)
    C = sca.native()
    enc, dec = _vae_layers(F=30, hidden=(20, 10), latent=3)
    gpu_m = C.vae_model(enc, 3, dec, 10, 11)
    cpu_m = C.vae_model(enc, 3, dec, 10, 11)
    X = np.random.default_rng(5).random(size=(40, 30))
    unit = C.BatchedUnit(gpu_m, 0)
    try:
        got = unit.run(X)  # one launch = offset 0, same Philox streams as the CPU twin
    finally:
        unit.stop()
    np.testing.assert_allclose(got[:, 0], cpu_m.run_cpu(X)[:, 0], rtol=2e-4)


# ------------------------------------------------------------------ bf16 / large-batch GEMM
def test_bf16_precision_is_an_explicit_opt_in():
    C = sca.native()
    layers = random_dense_stack([20, 32, 5], ["relu", "identity"])
    assert C.mlp_precision(C.mlp_model(layers, 1)) == "fp32"
    m = C.mlp_model(layers, 1, "bf16")
    assert C.mlp_precision(m) == "bf16" and C.mlp_layerwise(m, 4096)  # bf16 runs on the GEMM path only
    assert C.mlp_precision(m.clone()) == "bf16"
    with pytest.raises(Exception):
        C.mlp_model(layers, 1, "fp8")


def _torch_mlp(layers, X, softmax=True):
    import torch

    x = torch.tensor(X, dtype=torch.float32)
    for L in layers:
        x = x @ torch.tensor(L["W"]).T + torch.tensor(L["b"])
        if L["act"] == 1:
            x = torch.relu(x)
    return (torch.softmax(x, 1) if softmax else x).double().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 300, 1024, 8192])
@pytest.mark.parametrize("dims", [(784, 512, 256, 10), (13, 37, 19, 3)])
def test_mlp_large_batch_gemm_fp32_matches_torch(dims, rows, monkeypatch):
    """Layer-wise fp32 path (register-tiled GEMM from 512 rows) vs torch fp32."""
    monkeypatch.setenv("SCA_MLP_MODE", "layer")
    layers = random_dense_stack(list(dims), ["relu"] * (len(dims) - 2) + ["identity"], seed=3)
    X = np.random.default_rng(rows).normal(size=(rows, dims[0]))
    unit = sca.native().BatchedUnit(mlp_row_model(layers, OUT_SOFTMAX), 0, max_batch=8192)
    try:
        got = unit.run(X)
    finally:
        unit.stop()
    np.testing.assert_allclose(got, _torch_mlp(layers, X), rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 64, 1000, 8192])
@pytest.mark.parametrize("dims", [(784, 512, 256, 10), (13, 37, 19, 3), (64, 128, 128, 64, 33)])
def test_mlp_bf16_matches_torch_fp32_within_stated_tolerance(dims, rows):
    """bf16 operands / fp32 accumulation: stated tolerance 2e-2 absolute on
    softmax probabilities and 3e-2 relative on logits vs torch float32."""
    layers = random_dense_stack(list(dims), ["relu"] * (len(dims) - 2) + ["identity"], seed=4)
    X = np.random.default_rng(rows).normal(size=(rows, dims[0]))
    for out_mode, softmax in ((OUT_SOFTMAX, True), (0, False)):
        unit = sca.native().BatchedUnit(mlp_row_model(layers, out_mode, precision="bf16"), 0, max_batch=8192)
        try:
            got = unit.run(X)
        finally:
            unit.stop()
        ref = _torch_mlp(layers, X, softmax)
        if softmax:
            np.testing.assert_allclose(got, ref, atol=2e-2)
        else:
            scale = np.abs(ref).max()
            np.testing.assert_allclose(got, ref, atol=3e-2 * scale)


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rtol", [("fp32", 2e-4), ("bf16", 5e-2)])
def test_vae_large_batch_paths_match_cpu(precision, rtol, monkeypatch):
    monkeypatch.setenv("SCA_MLP_MODE", "layer")
    C = sca.native()
    enc, dec = _vae_layers(F=64, hidden=(256, 128), latent=16)
    gpu_m = C.vae_model(enc, 16, dec, 10, 11, precision)
    cpu_m = C.vae_model(enc, 16, dec, 10, 11)
    X = np.random.default_rng(5).random(size=(1000, 64))
    unit = C.BatchedUnit(gpu_m, 0, max_batch=4096)
    try:
        got = unit.run(X)[:, 0]
    finally:
        unit.stop()
    np.testing.assert_allclose(got, cpu_m.run_cpu(X)[:, 0], rtol=rtol)


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 700, 4096])
def test_mlp_bf16_binary_output_fused_epilogue(rows):
    """Binary classifier head (1 sigmoid unit -> [1 - p, p]) written by the bf16
    GEMM epilogue: stated tolerance 2e-2 absolute vs torch float32."""
    import torch

    from seldon_core_amd.models.mlp import OUT_BINARY

    layers = random_dense_stack([20, 48, 1], ["relu", "sigmoid"], seed=9)
    X = np.random.default_rng(rows).normal(size=(rows, 20))
    unit = sca.native().BatchedUnit(mlp_row_model(layers, OUT_BINARY, precision="bf16"), 0, max_batch=8192)
    try:
        got = unit.run(X)
    finally:
        unit.stop()
    x = torch.tensor(X, dtype=torch.float32)
    h = torch.relu(x @ torch.tensor(layers[0]["W"]).T + torch.tensor(layers[0]["b"]))
    p = torch.sigmoid(h @ torch.tensor(layers[1]["W"]).T + torch.tensor(layers[1]["b"])).double().numpy()[:, 0]
    assert got.shape == (rows, 2)
    np.testing.assert_allclose(got[:, 1], p, atol=2e-2)
    np.testing.assert_allclose(got[:, 0] + got[:, 1], 1.0, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("dims,out_mode", [((784, 512, 256, 10), 1), ((13, 37, 19, 3), 0), ((50, 64, 1), 2),
                                           ((31, 33), 1), ((30, 7), 0), ((37, 40, 20), 1)])
def test_mlp_lds_gemm_fp64_input_and_fused_output(dims, out_mode, monkeypatch):
    """LDS-tiled fp32 layer-wise path (>= 2048 rows): the first layer stages the
    fp64 request rows itself (odd widths take the masked scalar loads) and a
    last layer with N <= 16 writes the softmax / plain / binary output from its
    epilogue; wider heads (N = 33, 20) keep the fp32 logits + finish kernel."""
    import torch

    monkeypatch.setenv("SCA_MLP_MODE", "layer")
    acts = ["relu"] * (len(dims) - 2) + ["sigmoid" if out_mode == 2 else "identity"]
    layers = random_dense_stack(list(dims), acts, seed=len(dims) + dims[0])
    X = np.random.default_rng(dims[0]).normal(size=(4096 + 37, dims[0]))
    unit = sca.native().BatchedUnit(mlp_row_model(layers, out_mode), 0, max_batch=8192)
    try:
        got = np.asarray(unit.run(X))
    finally:
        unit.stop()
    x = torch.tensor(X, dtype=torch.float32)
    for L in layers:
        x = x @ torch.tensor(L["W"]).T + torch.tensor(L["b"])
        if L["act"] == 1:
            x = torch.relu(x)
        elif L["act"] == 2:
            x = torch.sigmoid(x)
    if out_mode == 1:
        x = torch.softmax(x, 1)
    elif out_mode == 2:
        x = torch.cat([1 - x, x], 1)
    ref = x.double().numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
