"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code.

Run here (not on the GPU box):  python tests/golden/make_goldens.py

The reference (/root/reference, Python) is imported read-only.  librosa is not
installed in this image; a stand-in module is injected into sys.modules INSIDE
THIS SCRIPT ONLY, providing ``librosa.util.frame`` as an exact numpy
equivalent (the only librosa call on the autocorrelation and data paths).  The
MFCC/delta/load calls raise if reached.  Fixtures are data only (inputs that are
regenerated from seeds, and expected outputs).
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import model_ref  # noqa: E402  (seeded parameter sets, shared with tests)
from tests.golden.make_goldens_helpers import (summary, synth_audio, full_layer_params, FakeSeq2Seq,  # noqa: E402
                                              INFER_FRAMES, INFER_MODEL)


def _install_librosa_stub():
    lib = types.ModuleType("librosa")
    util = types.ModuleType("librosa.util")
    feature = types.ModuleType("librosa.feature")

    def frame(x, frame_length, hop_length):
        return np.lib.stride_tricks.sliding_window_view(x, frame_length)[::hop_length].T

    def _absent(*a, **k):
        raise RuntimeError("librosa is not available in this image")

    util.frame = frame
    feature.mfcc = _absent
    feature.delta = _absent
    lib.util = util
    lib.feature = feature
    lib.load = _absent
    lib.resample = _absent
    sys.modules["librosa"] = lib
    sys.modules["librosa.util"] = util
    sys.modules["librosa.feature"] = feature


_install_librosa_stub()
sys.path.insert(0, REF)
from utils.model import Loss, GlobalPositionalEncoding, apply_rope_qk  # noqa: E402
from utils.model_utils import build_model, prepare_training_components  # noqa: E402
from utils.audio.extraction import extract_features_utils as efu  # noqa: E402
from dataset import data_processing as dp  # noqa: E402
from dataset.dataset import AudioFacialDataset  # noqa: E402

def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


# ---------------------------------------------------------------------------
def gen_loss():
    rng = np.random.default_rng(1)
    out = {}
    B, T, F = 3, 16, 61
    cases = {
        "random": (rng.standard_normal((B, T, F)) * 30, rng.standard_normal((B, T, F)) * 30),
        "zero_target": (rng.standard_normal((B, T, F)) * 30, np.zeros((B, T, F))),
        "zero_pred_diff": (np.repeat(rng.standard_normal((B, 1, F)), T, axis=1), rng.standard_normal((B, T, F))),
        "small": (rng.standard_normal((B, T, F)) * 0.3, rng.standard_normal((B, T, F)) * 0.3),
    }
    crit = Loss(delta=1.0, w1=1.0, w2=1.0)
    for k, (p, t) in cases.items():
        pt = torch.tensor(p, dtype=torch.float32, requires_grad=True)
        tt = torch.tensor(t, dtype=torch.float32)
        loss = crit(pt, tt)
        loss.backward()
        out[k + "_pred"] = p.astype(np.float32)
        out[k + "_trg"] = t.astype(np.float32)
        out[k + "_loss"] = np.float64(loss.item())
        out[k + "_grad"] = pt.grad.numpy()
    save("loss.npz", **out)


def gen_rope():
    rng = np.random.default_rng(2)
    x = torch.tensor(rng.standard_normal((2, 40, 128)), dtype=torch.float32)
    g = GlobalPositionalEncoding(128)(x)
    q = torch.tensor(rng.standard_normal((2, 3, 40, 64)), dtype=torch.float32)
    k = torch.tensor(rng.standard_normal((2, 3, 40, 64)), dtype=torch.float32)
    q2, k2 = apply_rope_qk(q, k)
    save("rope.npz", x=x.numpy(), global_out=g.numpy(), q=q.numpy(), k=k.numpy(),
         q_out=q2.numpy(), k_out=k2.numpy())


def _ref_model(D, H, L, seed):
    cfg = dict(input_dim=256, hidden_dim=D, n_layers=L, num_heads=H, dropout=0.0, output_dim=61,
               delta=1.0, w1=1.0, w2=1.0, learning_rate=5e-5, weight_decay=1e-5,
               warmup_epochs=0, n_epochs=50)
    torch.manual_seed(0)
    m = build_model(cfg, "cpu")
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), seed)
    assert list(params.keys()) == list(m.state_dict().keys())
    m.load_state_dict(params, strict=True)
    return cfg, m, params


def gen_model(tag, D, H, L, B, T, seed, steps=2):
    cfg, m, params = _ref_model(D, H, L, seed)
    rng = np.random.default_rng(seed + 1)
    srcs = [rng.standard_normal((B, T, 256)).astype(np.float32) for _ in range(steps)]
    trgs = [(rng.standard_normal((B, T, 61)) * 20).astype(np.float32) for _ in range(steps)]
    criterion, optimizer, scheduler = prepare_training_components(cfg, m)
    m.train()  # dropout 0.0 -> deterministic
    out = {"D": D, "H": H, "L": L, "B": B, "T": T, "seed": seed, "steps": steps}
    keys = list(params.keys())
    for s in range(steps):
        optimizer.zero_grad()
        src = torch.tensor(srcs[s])
        trg = torch.tensor(trgs[s])
        pred = m(src)
        loss = criterion(pred, trg)
        loss.backward()
        grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        total = torch.nn.utils.clip_grad_norm_(m.parameters(), 2.0)
        optimizer.step()
        out["src%d" % s] = srcs[s]
        out["trg%d" % s] = trgs[s]
        out["pred%d" % s] = pred.detach().numpy()
        out["loss%d" % s] = np.float64(loss.item())
        out["gnorm%d" % s] = np.float64(total.item())
        out["grads%d" % s] = np.stack([summary(grads[k].numpy()) for k in keys])
        out["params%d" % s] = np.stack([summary(p.detach().numpy()) for k, p in m.named_parameters()])
    save("model_%s.npz" % tag, **out)


def gen_full_layers():
    """One full-width (D=1024, H=16) encoder and decoder layer, B=1, T=128."""
    from utils.model import CustomTransformerEncoderLayer, CustomTransformerDecoderLayer
    rng = np.random.default_rng(7)
    x = rng.standard_normal((1, 128, 1024)).astype(np.float32)
    mem = rng.standard_normal((1, 128, 1024)).astype(np.float32)
    enc = CustomTransformerEncoderLayer(1024, 16, 0.0)
    dec = CustomTransformerDecoderLayer(1024, 16, 0.0)
    pe, pd_ = full_layer_params()
    assert [k[2:] for k in pe] == list(enc.state_dict().keys())
    assert [k[2:] for k in pd_] == list(dec.state_dict().keys())
    enc.load_state_dict({k[2:]: v for k, v in pe.items()})
    dec.load_state_dict({k[2:]: v for k, v in pd_.items()})
    enc.eval()
    dec.eval()
    with torch.no_grad():
        ye = enc(torch.tensor(x))
        yd = dec(torch.tensor(x), torch.tensor(mem))
    save("layers_full.npz", enc_out=summary(ye.numpy()), dec_out=summary(yd.numpy()),
         enc_rows=ye.numpy()[0, ::17], dec_rows=yd.numpy()[0, ::17])


def gen_autocorr():
    out = {}
    for seconds, seed in ((1.0, 3), (0.73, 4)):
        y = synth_audio(seconds, seed)
        ac = efu.extract_autocorrelation_features(y, 88200, 1470, 735)
        out["ac_%d" % seed] = ac
    # edge-frame fix: leading/trailing silence
    y = synth_audio(0.5, 5)
    y[:3000] = 0
    y[-3000:] = 0
    out["ac_silent_edges"] = efu.extract_autocorrelation_features(y, 88200, 1470, 735)
    rf = np.random.default_rng(6).standard_normal((5, 11))
    out["reduce_in"] = rf
    out["reduce_out"] = efu.reduce_features(rf)
    out["reduce_in_even"] = rf[:, :10]
    out["reduce_out_even"] = efu.reduce_features(rf[:, :10])
    out["cmvn_out"] = efu.cepstral_mean_variance_normalization(rf)
    save("features_autocorr.npz", **out)


class _Cfg(dict):
    pass


def gen_windows():
    out = {}
    ds = AudioFacialDataset.__new__(AudioFacialDataset)
    ds.micro_batch_size = 128
    for n in (128, 256, 300, 1848, 129):
        a = np.tile(np.arange(n, dtype=np.float64)[:, None], (1, 3))
        f = np.tile(np.arange(n, dtype=np.float64)[:, None] * 2, (1, 2))
        ex = ds.process_example(a, f)
        starts = np.array([int(e[0][0, 0].item()) for e in ex])
        # check each window is a contiguous run
        for e, s in zip(ex, starts):
            assert np.array_equal(e[0][:, 0].numpy(), np.arange(s, s + 128, dtype=np.float32))
        out["starts_%d" % n] = starts
    try:
        ds.process_example(np.zeros((100, 3)), np.zeros((100, 2)))
        out["short_raises"] = np.int64(0)
    except ValueError:
        out["short_raises"] = np.int64(1)
    save("data_windows.npz", **out)


def gen_augment():
    out = {}
    rng = np.random.default_rng(11)
    cols = ["Timecode", "BlendshapeCount"] + ["c%d" % i for i in range(61)]
    import pandas as pd
    cases = [("a", 70, 75, True, False), ("b", 80, 73, True, True), ("c", 64, 64, False, False),
             ("d", 301, 300, True, True), ("e", 45, 90, False, True)]
    with tempfile.TemporaryDirectory() as td:
        for tag, na, nf, fast, slow in cases:
            audio = rng.standard_normal((na, 7))
            facial = rng.standard_normal((nf, 61))
            apath = os.path.join(td, "audio_features_%s.csv" % tag)
            fpath = os.path.join(td, "x_iPhone_cal_%s.csv" % tag)
            pd.DataFrame(audio).to_csv(apath, index=False)
            df = pd.DataFrame(np.hstack([np.zeros((nf, 1)), np.full((nf, 1), 61), facial]), columns=cols)
            df.to_csv(fpath, index=False)
            # the reference reads the CSVs back: re-read so inputs are exactly what it saw
            audio_in = pd.read_csv(apath).values
            facial_in = pd.read_csv(fpath).drop(columns=["Timecode", "BlendshapeCount"]).values
            a_out, f_out = dp.collect_features(None, apath, fpath, 88200, include_fast=fast, include_slow=slow)
            out[tag + "_audio_in"] = audio_in
            out[tag + "_facial_in"] = facial_in
            out[tag + "_flags"] = np.array([fast, slow])
            out[tag + "_audio_out"] = a_out
            out[tag + "_facial_out"] = f_out
    x = rng.standard_normal((9, 4))
    out["interp_in"] = x
    out["interp_out"] = dp.interpolate_slower(x)
    out["smooth_out"] = dp.smooth_facial_data(x)
    seqs = [rng.standard_normal((n, 3)) for n in (40, 12, 50)]
    out["blend_in0"], out["blend_in1"], out["blend_in2"] = seqs
    out["blend_out"] = dp.stack_with_blend(seqs, 30)
    save("data_augment.npz", **out)


def gen_lr():
    from utils.model_utils import prepare_training_components as ptc
    vals = {}
    for warm in (0, 3):
        cfg = dict(delta=1.0, w1=1.0, w2=1.0, learning_rate=1.0, weight_decay=0.0,
                   warmup_epochs=warm, n_epochs=50)
        m = torch.nn.Linear(2, 2)
        _, opt, sch = ptc(cfg, m)
        lrs = []
        for e in range(52):
            lrs.append(opt.param_groups[0]["lr"])
            opt.step()
            sch.step()
        vals["warm%d" % warm] = np.array(lrs)
    save("lr.npz", **vals)


def gen_inference():
    """audio_processing.process_audio_features (the per-epoch validation
    inference) run by the reference: chunking/blend cases on an
    elementwise stand-in model, and one seeded small Seq2Seq of the reference
    (weights regenerated from the seed in the tests)."""
    from utils.audio.processing import audio_processing as ap
    out = {}
    cfg = {"frame_size": 128, "overlap": 16}
    for n in INFER_FRAMES:
        feats = np.random.default_rng(n).standard_normal((n, 256))
        out["feats_sum_%d" % n] = feats.sum()   # inputs are regenerated from the seed
        out["fake_%d" % n] = ap.process_audio_features(feats, FakeSeq2Seq(), "cpu", cfg)
    mc = INFER_MODEL
    _, m, _ = _ref_model(mc["D"], mc["H"], mc["L"], mc["seed"])
    feats = np.random.default_rng(mc["seed"]).standard_normal((mc["frames"], 256)).astype(np.float32)
    out["model_feats_sum"] = feats.astype(np.float64).sum()
    out["model_out"] = ap.process_audio_features(feats, m, "cpu", dict(cfg, overlap=16))
    save("inference.npz", **out)


def gen_formats():
    """Byte images of the files the reference writes on this path (SURVEY
    8(f)2): the LiveLink CSV (utils/csv/save_csv.py:4-62) and the
    audio_features.csv feature cache (dataset/data_processing.py:112-120)."""
    from utils.csv.save_csv import save_generated_data_as_csv
    out = {}
    rng = np.random.default_rng(41)
    cases = {"f32_61": (rng.random((130, 61)).astype(np.float32), False),
             "f64_68_emotions": (rng.standard_normal((70, 68)), True),
             "f64_68_base": (rng.standard_normal((20, 68)), False),
             "zeros_long": (np.zeros((3700, 61)), False)}   # timecodes past one minute
    with tempfile.TemporaryDirectory() as td:
        for tag, (arr, emo) in cases.items():
            path = os.path.join(td, tag + ".csv")
            save_generated_data_as_csv(arr, path, include_emotion_dimensions=emo)
            out["csv_in_" + tag] = arr
            out["csv_emo_" + tag] = np.array(emo)
            out["csv_bytes_" + tag] = np.frombuffer(open(path, "rb").read(), np.uint8)
        feats = rng.standard_normal((90, 256))
        facial = rng.standard_normal((90, 61))
        cols = ["Timecode", "BlendshapeCount"] + ["c%d" % i for i in range(61)]
        import pandas as pd
        fpath = os.path.join(td, "x_iPhone_cal.csv")
        pd.DataFrame(np.hstack([np.zeros((90, 1)), np.full((90, 1), 61), facial]), columns=cols).to_csv(
            fpath, index=False)
        cache = os.path.join(td, "audio_features.csv")
        saved = dp.extract_audio_features
        dp.extract_audio_features = lambda path, sr: (feats, None)
        try:
            dp.collect_features("clip.wav", cache, fpath, 88200, include_fast=False)
        finally:
            dp.extract_audio_features = saved
        out["cache_feats"] = feats
        out["cache_facial"] = facial
        out["cache_bytes"] = np.frombuffer(open(cache, "rb").read(), np.uint8)
    save("formats.npz", **out)


def gen_stats():
    """The per-epoch comparison statistics file (utils/validation.py:45-137,
    save_comparison_stats) written by the reference from seeded generated and
    ground-truth CSVs: generated longer and shorter than the ground truth, a
    68-column generated file (emotion columns after the 61 used ones), constant
    columns (NaN correlation) and exact zeros in the ground truth (the MAPE
    guard).  Inputs are kept as the CSV bytes the reference reads."""
    import pandas as pd
    from utils.csv.save_csv import save_generated_data_as_csv
    from utils.validation import save_comparison_stats
    out = {}
    rng = np.random.default_rng(77)
    names = ["Timecode", "BlendshapeCount"] + ["bs%d" % i for i in range(61)]
    cases = {"long_gen": (140, 120, False), "short_gen": (90, 120, False), "emotions": (100, 100, True)}
    with tempfile.TemporaryDirectory() as td:
        for tag, (ng, nt, emo) in cases.items():
            gt = rng.random((nt, 61))
            gt[:, 5] = 0.25                  # constant ground-truth column
            gt[rng.random((nt, 61)) < 0.05] = 0.0
            gen = gt[np.arange(ng) % nt] + 0.05 * rng.standard_normal((ng, 61))
            gen[:, 9] = 0.5                  # constant generated column
            if emo:
                gen = np.hstack([gen, rng.random((ng, 7))])
            gpath, tpath, spath = (os.path.join(td, tag + x) for x in ("_gen.csv", "_gt.csv", "_stats.txt"))
            save_generated_data_as_csv(gen, gpath, include_emotion_dimensions=emo)
            pd.DataFrame(np.hstack([np.arange(nt)[:, None] / 60.0, np.full((nt, 1), 61), gt]), columns=names).to_csv(
                tpath, index=False)
            save_comparison_stats(gpath, tpath, spath)
            for k, pth in (("gen", gpath), ("gt", tpath), ("stats", spath)):
                out["%s_%s" % (k, tag)] = np.frombuffer(open(pth, "rb").read(), np.uint8)
    save("stats.npz", **out)


GENERATORS = {
    "loss": gen_loss, "rope": gen_rope,
    "model_tiny": lambda: gen_model("tiny", D=128, H=2, L=2, B=2, T=32, seed=21),
    "model_mid": lambda: gen_model("mid", D=256, H=4, L=1, B=2, T=128, seed=22, steps=1),
    "layers_full": gen_full_layers, "autocorr": gen_autocorr, "windows": gen_windows, "augment": gen_augment,
    "lr": gen_lr, "inference": gen_inference, "formats": gen_formats, "stats": gen_stats,
}

if __name__ == "__main__":
    # python tests/golden/make_goldens.py [generator ...]  (default: all)
    torch.set_num_threads(8)
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name]()
