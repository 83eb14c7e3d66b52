"""GPU feature path (nstl_features / nstl_autocorr) against the CPU oracle and
the reference-generated autocorrelation fixture; the drop-in
extract_audio_features on a WAV file; batched clip inference vs the reference's
per-chunk loop; a full-width C1 training run through train.main."""
import os

import numpy as np
import pytest
import torch

from oracle import data_ref
from tests.golden.make_goldens_helpers import synth_audio

pytestmark = pytest.mark.gpu


def _features(y, sr=88200):
    from neurosync_trainer_lite_amd.utils.audio.extraction.extract_features import extract_audio_features_device
    out = extract_audio_features_device(y, sr, device=torch.device("cuda:0"))
    torch.cuda.synchronize()
    return None if out is None else out.double().cpu().numpy()


def test_autocorr_matches_reference_fixture(golden):
    g = golden("features_autocorr.npz")
    cases = [(synth_audio(1.0, 3), g["ac_3"]), (synth_audio(0.73, 4), g["ac_4"])]
    y = synth_audio(0.5, 5)
    y[:3000] = 0
    y[-3000:] = 0
    cases.append((y, g["ac_silent_edges"]))
    for y, want in cases:
        got = _features(y)[:, 69:]
        # f64 lags, f32 output
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=2e-7)


@pytest.mark.parametrize("L,hop,n_lags", [(1470, 735, 187), (800, 400, 187), (1470, 735, 191), (266, 133, 40),
                                           (64, 32, 10), (1801, 900, 150)])
def test_autocorr_kernel_matches_oracle_across_frame_lengths(L, hop, n_lags):
    """nstl_autocorr (the f64 MFMA kernel: 64-sample k-steps, 13 column tiles,
    tiles past the frame skipped) at other sample rates' frame lengths, lag
    counts up to its 191 limit, frames shorter than one k-step, and a frame
    length that is not a multiple of 16, against the oracle's direct products.
    The frame mean is the exact f32-rounded mean on the GPU and numpy's f32
    pairwise sum in the reference; at 64-sample frames that DC difference alone
    moves the normalised lags by up to ~2e-6 (5e-5 relative), so that case is held
    to 3e-6 absolute; every frame length of a real sample rate (>= 266) to the
    fixture's rtol 2e-6 / atol 2e-7."""
    from neurosync_trainer_lite_amd import _hip as K
    y = synth_audio(0.4, 21)
    n = len(y)
    F = (n + 2 * (L // 2) - L) // hop + 1
    out = torch.empty(F, n_lags, dtype=torch.float64, device="cuda:0")
    K.autocorr(torch.tensor(y, device="cuda:0"), L, hop, n_lags, out, F)
    torch.cuda.synchronize()
    want = data_ref.autocorr_features_120(y, L, hop, n_lags).T
    assert want.shape == (F, n_lags)
    if L >= 266:
        np.testing.assert_allclose(out.cpu().numpy(), want, rtol=2e-6, atol=2e-7)
    else:
        np.testing.assert_allclose(out.cpu().numpy(), want, rtol=0, atol=3e-6)


@pytest.mark.parametrize("seconds,seed", [(1.0, 3), (0.73, 4), (2.5, 6), (0.09, 7)])
def test_features_match_oracle(seconds, seed):
    y = synth_audio(seconds, seed)
    want = data_ref.extract_features(y)
    got = _features(y)
    assert got.shape == want.shape == ((1 + len(y) // 735 + 1) // 2, 256)
    # MFCC branch (librosa restated; parity vs librosa itself unpinned): CMVN'd
    # coefficients and deltas are O(1); f32 DFT-GEMM/mel/DCT vs the f64 oracle
    np.testing.assert_allclose(got[:, :69], want[:, :69], rtol=0, atol=2e-3)
    np.testing.assert_allclose(got[:, 69:], want[:, 69:], rtol=2e-6, atol=2e-7)


def test_features_short_clip_rejected():
    assert _features(np.zeros(1470 + 7 * 735, np.float32) + 0.1) is None  # 8 frames
    assert _features(synth_audio(9 * 735 / 88200 + 1470 / 88200, 8)) is not None


def test_extract_audio_features_from_wav(tmp_path):
    from neurosync_trainer_lite_amd.utils.audio.extraction.extract_features import extract_audio_features
    from neurosync_trainer_lite_amd.utils.audio.load_audio import write_wav
    y = synth_audio(1.5, 9)
    p = tmp_path / "a.wav"
    write_wav(str(p), y, 88200, bits=32)
    feats, yy = extract_audio_features(str(p))
    assert feats.dtype == np.float64 and feats.shape == ((1 + len(y) // 735 + 1) // 2, 256)
    want = data_ref.extract_features(yy)
    np.testing.assert_allclose(feats[:, 69:], want[:, 69:], rtol=2e-6, atol=2e-7)
    np.testing.assert_allclose(feats[:, :69], want[:, :69], atol=2e-3)


def test_inference_matches_reference_fixture(golden):
    """The per-epoch validation inference (process_audio_features,
    audio_processing.py:50-112) of a seeded small Seq2Seq on the GPU (fp32 mode,
    chunks batched) against the reference's own run of it on the CPU
    (tests/golden/inference.npz, 300 frames: 3 chunks, overlap 16, tail)."""
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.audio.processing import audio_processing as ap
    from neurosync_trainer_lite_amd.utils.model_utils import build_model
    from oracle import model_ref
    from tests.golden.make_goldens_helpers import INFER_MODEL as mc
    g = golden("inference.npz")
    cfg = dict(training_config)
    cfg.update(hidden_dim=mc["D"], num_heads=mc["H"], n_layers=mc["L"], use_amp=False)
    dev = torch.device("cuda:0")
    model = build_model(cfg, dev)
    model.load_state_dict(model_ref.seeded_params(model_ref.param_shapes(256, mc["D"], mc["L"], 61), mc["seed"]),
                          strict=True)
    feats = np.random.default_rng(mc["seed"]).standard_normal((mc["frames"], 256)).astype(np.float32)
    assert feats.astype(np.float64).sum() == g["model_feats_sum"]
    got = ap.process_audio_features(feats, model, dev, dict(cfg, frame_size=128, overlap=16))
    want = g["model_out"]
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-5)


def test_c1_train_main_full_width(tmp_path, monkeypatch):
    """C1 shape (L4/H4/D1024) through the drop-in entry point: GPU feature
    extraction (no cache), dataset, 1 epoch, checkpoint, validation clip."""
    from neurosync_trainer_lite_amd import train as tr
    from neurosync_trainer_lite_amd.config import training_config
    from tests.test_train_plumbing import make_corpus
    monkeypatch.chdir(tmp_path)
    clip = make_corpus(str(tmp_path), cache_features=False)
    cfg = dict(training_config)
    cfg.update(n_layers=4, num_heads=4, hidden_dim=1024, n_epochs=1, batch_size=128,
               audio_path=os.path.join(clip, "audio.wav"),
               ground_truth_path=os.path.join(clip, "synth_iPhone_cal.csv"))
    steps = tr.main(cfg)
    assert steps > 0
    assert os.path.exists(os.path.join(clip, "audio_features.csv"))
    assert os.path.exists("out/model.pth") and os.path.exists(cfg["checkpoint_path"])
    stats = open("dataset/validation_plots/stats/comparison_stats_epoch_1.txt").read()
    assert "Mean Squared Error (MSE)" in stats


@pytest.mark.parametrize("key", ["reduce_in", "reduce_in_even"])
def test_cmvn_and_pair_reduce_match_reference_fixtures(golden, key):
    """The HIP frame-axis stages fed the reference-pinned fixtures directly
    (tests/golden/features_autocorr.npz, generated by the reference's own
    reduce_features / cepstral_mean_variance_normalization): the pair reduction
    of f64 rows bit for bit (f64 pair means cast to f32), CMVN then reduction
    within f32 rounding; the delta columns against the oracle's Savitzky-Golay
    restatement (librosa.feature.delta: parity unpinned)."""
    from neurosync_trainer_lite_amd import _hip as K
    g = golden("features_autocorr.npz")
    x = g[key]                                   # [C, F] f64
    out_key = "reduce_out" if key == "reduce_in" else "reduce_out_even"
    C, F = x.shape
    F60 = (F + 1) // 2
    dev = "cuda:0"
    # reduce_features on [F][cols] f64 rows (the autocorrelation-lag layout)
    red = torch.zeros(F60, C + 3, dtype=torch.float32, device=dev)
    K.reduce_frame_pairs(torch.tensor(x.T.copy(), device=dev), red, col0=3)
    torch.cuda.synchronize()
    assert np.array_equal(red[:, 3:].cpu().numpy(), g[out_key].T.astype(np.float32))
    # CMVN + deltas + reduction of coefficient rows (the MFCC layout)
    out = torch.zeros(F60, 3 * C, dtype=torch.float32, device=dev)
    K.cmvn_delta_reduce(torch.tensor(x, dtype=torch.float32, device=dev), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.float64)
    cm = g["cmvn_out"] if key == "reduce_in" else data_ref.cmvn(x)
    np.testing.assert_allclose(got[:, :C], data_ref.reduce_features(cm).T, rtol=1e-5, atol=1e-6)
    for o in (1, 2):
        want = data_ref.reduce_features(data_ref.savgol_delta(cm, o)).T
        np.testing.assert_allclose(got[:, o * C:(o + 1) * C], want, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("seconds,seed,silent", [(0.6, 11, False), (0.35, 12, True)])
def test_fused_stft_mel_matches_f64(seconds, seed, silent):
    """nstl_stft_mel (mixed-radix f32 FFT in LDS, |X|^2, Slaney bands) against the
    f64 numpy STFT power times the f64 mel basis (oracle/data_ref.mfcc_120's
    first steps).  Tolerance per frame: 2e-6 of the largest band of the frame and
    of the frame it shares a complex FFT with (frames 2j and 2j + 1 go through one
    transform as its real and imaginary parts, so each carries f32 rounding of the
    pair's energy: a silent frame beside a loud one reads ~1e-7 of it, far under
    the dB floor, top_db 80, of the MFCC that follows) plus 2e-5 relative (f32 FFT
    rounding ~ log2(n) eps)."""
    from neurosync_trainer_lite_amd import _hip as K
    sr, n_fft, hop = 88200, 1470, 735
    y = synth_audio(seconds, seed)
    if silent:  # a silent lead-in: bands near zero in the first frames
        y[:4000] = 0
    F = 1 + len(y) // hop
    yp = np.pad(y.astype(np.float64), n_fft // 2, mode="constant")
    frames = data_ref.frame_signal(yp, n_fft, hop)[:, :F]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    power = np.abs(np.fft.rfft(frames * win[:, None], axis=0)) ** 2
    ref = (data_ref.mel_basis(sr, n_fft).astype(np.float64) @ power).T  # [F, 128]
    yd = torch.tensor(y, device="cuda:0")
    mel = torch.empty(F, 128, device="cuda:0")
    K.stft_mel(yd, len(y), sr, mel, F)
    torch.cuda.synchronize()
    got = mel.double().cpu().numpy()
    fmax = ref.max(axis=1)
    pair = np.maximum(fmax, fmax[np.minimum(np.arange(F) ^ 1, F - 1)])
    bound = 2e-6 * pair[:, None] + 2e-5 * np.abs(ref)
    assert np.all(np.abs(got - ref) <= bound + 1e-30), np.max(np.abs(got - ref) / (bound + 1e-30))
    with pytest.raises(RuntimeError, match="n_frames"):
        K.stft_mel(yd, len(y), sr, mel, F + 1)
