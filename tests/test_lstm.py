"""Seq2seq LSTM detector kernel (VERDICT r1 Missing #2):
BiLSTM encoder stack -> LSTM decoder stack -> Dense, greedy T-1 step decode,
per-sequence MSE, as one persistent MFMA kernel per batch.  The oracle is the
torch fp32 model (nn.LSTM bidirectional + nn.LSTMCell decode loop)."""
import numpy as np
import pytest

import seldon_core_amd as sca
from seldon_core_amd.components.outlier import OutlierSeq2SeqLSTM, Seq2SeqLSTMNet

SHAPES = [  # (F, T, encoder, decoder, act)
    (1, 140, (20,), (40,), "sigmoid"),   # the reference's ECG detector shape
    (3, 24, (8, 6), (12, 12), "linear"),  # stacked encoder (return_sequences) + stacked decoder
    (16, 10, (32,), (64,), "tanh"),
]


def _torch_mse(net, X):
    return np.mean((X - net.reconstruct(X)) ** 2, axis=(1, 2))


@pytest.mark.parametrize("F,T,enc,dec,act", SHAPES)
def test_cpu_reference_matches_torch(F, T, enc, dec, act):
    net = Seq2SeqLSTMNet(F, enc, dec, act, -1, seed=F)
    X = np.random.default_rng(F).random((4, T, F))
    got = net.native_model(T).run_cpu(X.reshape(4, -1))[:, 0]
    np.testing.assert_allclose(got, _torch_mse(net, X), rtol=1e-5, atol=1e-9)


def test_program_layout():
    C = sca.native()
    net = Seq2SeqLSTMNet(1, (20,), (40,), "sigmoid", -1)
    p = C.lstm_program(net.native_model(140))
    assert p["w_lds"] == 1 and p["lds_bytes"] <= 160 * 1024 and p["workspace_floats_per_wg"] == 0
    big = Seq2SeqLSTMNet(32, (64, 64), (128,), "sigmoid", -1)
    pb = C.lstm_program(big.native_model(8))
    assert pb["w_lds"] == 0 and pb["workspace_floats_per_wg"] == 2 * 16 * 8 * 128


def test_valu_program_layout():
    """Small-batch VALU kernel (csrc/kernels/lstm_valu.hip): the reference ECG
    shape fits with KPL = 8 (encoder 2 x 128 threads, decoder 320 + 64 for the
    Dense lanes); a model too wide for 1024 lanes falls back to MFMA."""
    C = sca.native()
    net = Seq2SeqLSTMNet(1, (20,), (40,), "sigmoid", -1)
    m = net.native_model(140)
    p = C.lstm_program(m)
    assert p["valu_ok"] == 1 and p["valu_kpl"] == 8 and p["valu_threads"] == 384
    assert p["valu_lds_bytes_r4"] <= 160 * 1024
    assert C.lstm_path(m, 1) == "valu" and C.lstm_path(m, 4 * 256) == "valu" and C.lstm_path(m, 4 * 256 + 1) == "mfma"
    big = Seq2SeqLSTMNet(32, (64, 64), (128,), "sigmoid", -1)
    assert C.lstm_program(big.native_model(8))["valu_ok"] == 0
    assert C.lstm_path(big.native_model(8), 1) == "mfma"


def test_rejects_incompatible_decoder():
    with pytest.raises(ValueError):
        Seq2SeqLSTMNet(1, (20,), (20,), "sigmoid", -1)


@pytest.mark.gpu
@pytest.mark.parametrize("F,T,enc,dec,act", SHAPES + [(32, 8, (64, 64), (128,), "sigmoid")])
@pytest.mark.parametrize("rows", [1, 16, 37])
@pytest.mark.parametrize("path", ["auto", "mfma", "valu"])
def test_gpu_kernel_matches_torch_fp32(F, T, enc, dec, act, rows, path, monkeypatch):
    if path != "auto":
        monkeypatch.setenv("SCA_LSTM_PATH", path)
    C = sca.native()
    net = Seq2SeqLSTMNet(F, enc, dec, act, -1, seed=rows)
    X = np.random.default_rng(rows).random((rows, T, F))
    unit = C.BatchedUnit(net.native_model(T), 0, max_batch=4096)
    try:
        got = np.asarray(unit.run(X.reshape(rows, -1)))[:, 0]
        assert unit.stats()["batches"] == 1  # one batch = one kernel launch
    finally:
        unit.stop()
    np.testing.assert_allclose(got, _torch_mse(net, X), rtol=1e-4, atol=1e-7)


@pytest.mark.gpu
def test_detector_scores_on_gpu():
    det = OutlierSeq2SeqLSTM(threshold=0.05, timesteps=20, n_features=2, encoder_dim=(10,), decoder_dim=(20,),
                             device=0, seed=3)
    cpu = OutlierSeq2SeqLSTM(threshold=0.05, timesteps=20, n_features=2, encoder_dim=(10,), decoder_dim=(20,),
                             device=-1, seed=3)
    X = np.random.default_rng(0).random((12, 40))
    try:
        pg = det.predict(X, [])
        pc = cpu.predict(X, [])
        np.testing.assert_array_equal(pg, pc)
        np.testing.assert_allclose(det.mse, cpu.mse, rtol=1e-4)
        assert det.net._units  # the native kernel ran
    finally:
        det.net.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [300, 700])
def test_gpu_valu_multi_row_workgroups(rows):
    """Batches past one sequence per CU: the VALU kernel packs R = 2 / 4
    sequences per workgroup."""
    C = sca.native()
    net = Seq2SeqLSTMNet(2, (10,), (20,), "sigmoid", -1, seed=5)
    X = np.random.default_rng(rows).random((rows, 30, 2))
    m = net.native_model(30)
    assert C.lstm_path(m, rows) == "valu"
    unit = C.BatchedUnit(m, 0, max_batch=4096)
    try:
        got = np.asarray(unit.run(X.reshape(rows, -1)))[:, 0]
    finally:
        unit.stop()
    np.testing.assert_allclose(got, _torch_mse(net, X), rtol=1e-4, atol=1e-7)
