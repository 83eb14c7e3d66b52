"""Host-side drop-in modules on CPU: data path (bit-exact vs reference goldens),
WAV ingest, chunked inference blending, CSV writer, checkpoint rotation, LR."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from neurosync_trainer_lite_amd.dataset import data_processing as dp
from neurosync_trainer_lite_amd.dataset.dataset import AudioFacialDataset, window_plan
from neurosync_trainer_lite_amd.utils.audio import load_audio as la
from neurosync_trainer_lite_amd.utils.audio.processing import audio_processing as ap
from neurosync_trainer_lite_amd.utils.csv.save_csv import save_generated_data_as_csv, timecode
from oracle import data_ref
from tests.golden.make_goldens_helpers import FakeSeq2Seq, INFER_FRAMES


def _dataset(window=128):
    ds = AudioFacialDataset.__new__(AudioFacialDataset)
    ds.micro_batch_size = window
    ds.clips, ds.index = [], []
    ds.pin = False
    return ds


def test_window_plan_matches_reference(golden):
    g = golden("data_windows.npz")
    for n in (128, 256, 300, 1848, 129):
        np.testing.assert_array_equal([s for s, _ in window_plan(n, n, 128)], g["starts_%d" % n])
    assert int(g["short_raises"]) == 1
    with pytest.raises(ValueError):
        window_plan(100, 100, 128)


def test_dataset_windows_identical_to_materialised():
    rng = np.random.default_rng(0)
    ds = _dataset()
    clips = [(rng.standard_normal((n, 256)), rng.standard_normal((n, 61))) for n in (128, 300, 257)]
    for a, f in clips:
        ds.add_clip(a, f)
    want = [w for a, f in clips for w in data_ref.windows(a, f, 128)]
    assert len(ds) == len(want)
    for i in (0, 1, 2, 100, len(ds) - 2, len(ds) - 1):
        src, trg = ds[i]
        assert src.dtype == torch.float32 and src.shape == (128, 256) and trg.shape == (128, 61)
        np.testing.assert_array_equal(src.numpy(), want[i][0])
        np.testing.assert_array_equal(trg.numpy(), want[i][1])
    # API-compatible materialised form and collate
    ex = ds.process_example(*clips[1])
    assert len(ex) == len(data_ref.window_plan(300, 300, 128))
    src, trg = AudioFacialDataset.collate_fn([ds[0], ds[5]])
    assert src.shape == (2, 128, 256) and trg.shape == (2, 128, 61)


def test_collect_features_matches_reference_bitexact(golden, tmp_path, monkeypatch):
    # pandas' CSV text round trip is not bit-exact: serve the exact arrays the
    # reference read (the fixture stores them after its own CSV read)
    g = golden("data_augment.npz")
    cols = ["Timecode", "BlendshapeCount"] + ["c%d" % i for i in range(61)]
    tables = {}
    real_read = pd.read_csv
    monkeypatch.setattr(dp.pd, "read_csv", lambda path, *a, **k: tables[str(path)] if str(path) in tables
                        else real_read(path, *a, **k))
    for tag in "abcde":
        fast, slow = (bool(v) for v in g[tag + "_flags"])
        apath = tmp_path / ("audio_features_%s.csv" % tag)
        fpath = tmp_path / ("x_iPhone_cal_%s.csv" % tag)
        apath.write_text("cached\n")
        fin = g[tag + "_facial_in"]
        tables[str(apath)] = pd.DataFrame(g[tag + "_audio_in"])
        tables[str(fpath)] = pd.DataFrame(np.hstack([np.zeros((len(fin), 1)), np.full((len(fin), 1), 61), fin]),
                                          columns=cols)
        a, f = dp.collect_features(None, str(apath), str(fpath), 88200, include_fast=fast, include_slow=slow)
        np.testing.assert_array_equal(a, g[tag + "_audio_out"])
        np.testing.assert_array_equal(f, g[tag + "_facial_out"])
    np.testing.assert_array_equal(dp.interpolate_slower(g["interp_in"]), g["interp_out"])
    np.testing.assert_array_equal(dp.smooth_facial_data(g["interp_in"]), g["smooth_out"])
    np.testing.assert_array_equal(dp.stack_with_blend([g["blend_in0"], g["blend_in1"], g["blend_in2"]], 30),
                                  g["blend_out"])


def test_wav_roundtrip(tmp_path):
    sr = 88200
    t = np.arange(sr // 10) / sr
    y = (0.5 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    p16 = tmp_path / "a16.wav"
    la.write_wav(str(p16), y, sr, bits=16)
    z, zsr = la.load_audio(str(p16), sr)
    assert zsr == sr and z.dtype == np.float32 and len(z) == len(y)
    assert np.abs(z - y).max() <= 1.0 / 32768
    pf = tmp_path / "af.wav"
    la.write_wav(str(pf), y, sr, bits=32)
    z, _ = la.load_and_preprocess_audio(str(pf), sr)
    np.testing.assert_allclose(z, y / np.abs(y).max(), rtol=1e-6)
    # resampling path (not soxr: only the length and band-limited content are checked)
    z, zsr = la.load_audio(str(p16), 44100)
    assert zsr == 44100 and abs(len(z) - len(y) // 2) <= 1
    with open(p16, "rb") as fh:
        zb, _ = la.load_audio_from_bytes(fh.read(), sr)
    assert np.abs(zb).max() == pytest.approx(1.0)


@pytest.mark.parametrize("n", INFER_FRAMES)
def test_process_audio_features_matches_reference(golden, n):
    """Chunking, reflect padding, cross-fade, tail chunk and /100 against the
    reference's own process_audio_features (tests/golden/inference.npz,
    audio_processing.py:50-112), bit for bit."""
    g = golden("inference.npz")
    feats = np.random.default_rng(n).standard_normal((n, 256))
    assert feats.sum() == g["feats_sum_%d" % n]
    got = ap.process_audio_features(feats, FakeSeq2Seq(), "cpu", {"frame_size": 128, "overlap": 16})
    assert got.shape == (n, 61)
    np.testing.assert_array_equal(got, g["fake_%d" % n])


@pytest.mark.parametrize("tag", ["f32_61", "f64_68_emotions", "f64_68_base", "zeros_long"])
def test_csv_writer_bytes_match_reference(golden, tmp_path, tag):
    """The LiveLink CSV is byte-identical to the reference writer's
    (utils/csv/save_csv.py:4-62; tests/golden/formats.npz)."""
    g = golden("formats.npz")
    out = tmp_path / "g.csv"
    save_generated_data_as_csv(g["csv_in_" + tag], str(out), include_emotion_dimensions=bool(g["csv_emo_" + tag]))
    assert out.read_bytes() == g["csv_bytes_" + tag].tobytes()


def test_feature_cache_bytes_match_reference(golden, tmp_path, monkeypatch):
    """collect_features writes the audio_features.csv cache byte-identically to
    the reference (data_processing.py:112-120) and reads it back exactly."""
    g = golden("formats.npz")
    cols = ["Timecode", "BlendshapeCount"] + ["c%d" % i for i in range(61)]
    facial = g["cache_facial"]
    fpath = tmp_path / "x_iPhone_cal.csv"
    pd.DataFrame(np.hstack([np.zeros((90, 1)), np.full((90, 1), 61), facial]), columns=cols).to_csv(fpath, index=False)
    cache = tmp_path / "audio_features.csv"
    monkeypatch.setattr(dp, "extract_audio_features", lambda path, sr: (g["cache_feats"], None))
    a1, _ = dp.collect_features("clip.wav", str(cache), str(fpath), 88200, include_fast=False)
    assert cache.read_bytes() == g["cache_bytes"].tobytes()
    monkeypatch.setattr(dp, "extract_audio_features", None)  # second read must come from the cache
    a2, _ = dp.collect_features("clip.wav", str(cache), str(fpath), 88200, include_fast=False)
    # pandas' default float parser is not round-trip exact (the reference shares this)
    np.testing.assert_allclose(a1, a2, rtol=1e-15, atol=1e-15)


def test_clip_files_naming_rule(tmp_path):
    """Folder discovery keeps the reference's rule: the facial CSV is the one
    whose name contains 'iPhone_cal' (mov_extraction.py:23); mov before mp4."""
    for name in ("a.mp4", "b.mov", "take_iPhone_cal.csv", "other.csv", "notes.txt"):
        (tmp_path / name).write_bytes(b"")
    found, cache = dp.clip_files(str(tmp_path))
    assert os.path.basename(found["facial"]) == "take_iPhone_cal.csv"
    assert {k: os.path.basename(v) for k, v in found.items() if k != "facial"} == {"mov": "b.mov", "mp4": "a.mp4"}
    assert os.path.basename(cache) == "audio_features.csv"


def test_csv_writer(tmp_path):
    assert timecode(0) == "00:00:00:00.000"
    assert timecode(61) == "00:00:01:00.016"  # the reference arithmetic truncates 0.999.. to 0
    assert timecode(3600 * 60 + 90) == "01:00:01:29.500"
    gen = np.random.default_rng(1).random((130, 61)).astype(np.float32)
    out = tmp_path / "g.csv"
    save_generated_data_as_csv(gen, str(out))
    df = pd.read_csv(out)
    assert list(df.columns[:3]) == ["Timecode", "BlendshapeCount", "EyeBlinkLeft"] and df.shape == (130, 63)
    np.testing.assert_allclose(df.iloc[:, 2:].values, gen, rtol=1e-6)
    with pytest.raises(ValueError):
        save_generated_data_as_csv(np.zeros((3, 60)), str(out))


def test_checkpoint_rotation_and_resume(tmp_path):
    from neurosync_trainer_lite_amd.utils import checkpoint_utils as cu
    model = torch.nn.Linear(4, 3)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda e: 1.0 - e / 10)
    cfg = {"checkpoint_path": str(tmp_path / "ck" / "checkpoint.pth")}
    for epoch in range(8):
        model(torch.randn(2, 4)).sum().backward()
        opt.step()
        sched.step()
        cu.save_checkpoint(model, opt, sched, epoch, epoch * 10, cfg)
    backups = [d for d in os.listdir(tmp_path / "ck") if d.startswith("backup_")]
    assert len(backups) == 5
    m2 = torch.nn.Linear(4, 3)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-3, weight_decay=1e-5)
    s2 = torch.optim.lr_scheduler.LambdaLR(o2, lambda e: 1.0 - e / 10)
    epoch, step, m2, o2, s2 = cu.load_checkpoint(cfg["checkpoint_path"], m2, o2, s2, "cpu")
    assert (epoch, step) == (7, 70)
    torch.testing.assert_close(m2.weight, model.weight)
    assert s2.last_epoch == sched.last_epoch


def test_lr_lambda_matches_reference(golden):
    from neurosync_trainer_lite_amd.utils.model_utils import lr_lambda_for
    g = golden("lr.npz")
    for key, warm in (("warm0", 0), ("warm3", 3)):
        f = lr_lambda_for({"warmup_epochs": warm, "n_epochs": 50})
        np.testing.assert_allclose([f(e) for e in range(len(g[key]))], g[key], rtol=0, atol=1e-15)


@pytest.mark.parametrize("tag", ["long_gen", "short_gen", "emotions"])
def test_comparison_stats_file_matches_reference(golden, tag, tmp_path):
    """The per-epoch statistics file (utils/validation.py:45-137) byte for byte
    against the reference's own output on the same generated / ground-truth CSVs
    (tests/golden/stats.npz, make_goldens.py gen_stats): MAE/MAPE/MSE/RMSE/r
    overall and per dimension, length alignment, NaN correlations of constant
    columns, the zero-ground-truth MAPE guard."""
    from neurosync_trainer_lite_amd.utils.validation import comparison_stats, save_comparison_stats
    g = golden("stats.npz")
    gpath, tpath, spath = tmp_path / "gen.csv", tmp_path / "gt.csv", tmp_path / "stats.txt"
    gpath.write_bytes(g["gen_" + tag].tobytes())
    tpath.write_bytes(g["gt_" + tag].tobytes())
    save_comparison_stats(str(gpath), str(tpath), str(spath))
    assert spath.read_bytes() == g["stats_" + tag].tobytes()
    overall, per_dim = comparison_stats(np.zeros((3, 61)), np.ones((4, 61)))
    assert overall['Mean Squared Error (MSE)'] == 1.0 and len(per_dim) == 61


def test_batched_fetch_equals_per_window(golden):
    """__getitems__ (the DataLoader's batched fetch into one host batch) returns
    exactly the windows __getitem__ does, tails and short streams included, and
    the DataLoader path collates it unchanged."""
    from torch.utils.data import DataLoader, random_split
    ds = _dataset()
    rng = np.random.default_rng(4)
    for na, nf in ((300, 300), (256, 260), (1000, 997), (128, 128)):
        ds.add_clip(rng.standard_normal((na, 256)), rng.standard_normal((nf, 61)))
    idx = list(rng.permutation(len(ds))[:77]) + [len(ds) - 1, 0]
    src, trg = AudioFacialDataset.collate_fn(ds.__getitems__(idx))
    for i, j in enumerate(idx):
        a, f = ds[j]
        assert torch.equal(src[i], a) and torch.equal(trg[i], f)
    train, _ = random_split(ds, [len(ds) - 10, 10], generator=torch.Generator().manual_seed(0))
    dl = DataLoader(train, batch_size=32, shuffle=False, collate_fn=AudioFacialDataset.collate_fn)
    s0, t0 = next(iter(dl))
    want = [ds[train.indices[i]] for i in range(32)]
    assert torch.equal(s0, torch.stack([w[0] for w in want])) and torch.equal(t0, torch.stack([w[1] for w in want]))
    # torch's default_collate (no collate_fn), over the Subset and the dataset itself
    for loader_ds, ids in ((train, [train.indices[i] for i in range(32)]), (ds, list(range(32)))):
        s1, t1 = next(iter(DataLoader(loader_ds, batch_size=32, shuffle=False)))
        want = [ds[i] for i in ids]
        assert torch.equal(s1, torch.stack([w[0] for w in want])) and torch.equal(t1, torch.stack([w[1] for w in want]))
