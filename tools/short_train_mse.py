"""the validation blendshape MSE (utils/validation.py:102, the
'Mean Squared Error (MSE)' line of save_comparison_stats) of the build and of the
reference step after an identical short training run -- tracked, not gated.

"Reference" here is the fp32 CPU restatement of the reference's step
(oracle/model_ref.OracleTrainer: training_utils.py:56-80 with Loss, clip 2.0 and
coupled-L2 Adam), since the reference itself cannot run without librosa; it is
pinned to the reference by tests/test_oracle.py.  Both start from the same seeded
weights, see the same batches in the same order (dropout 0, so the runs differ
only by arithmetic), and are then validated by the same drop-in pipeline:
extract_audio_features (GPU) -> process_audio_features (chunk 128 / overlap 16 /
cross-fade / /100) -> save_generated_data_as_csv -> save_comparison_stats against
the held-out clip's ground truth CSV.

The synthetic corpus is learnable (targets follow the audio): per clip an 88.2 kHz
WAV of 3 harmonics of f0 with an amplitude envelope of random rate, and 61
blendshape curves that are fixed random mixes of that envelope, its derivative and
f0 (cols 0-51 clipped to [0, 1], 52-60 0.3 tanh), plus low-pass noise.

  python tools/short_train_mse.py [--steps N] [--out FILE]   (GPU; ~1-2 min)"""
import argparse
import contextlib
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def learnable_corpus(root, clips, seconds, seed, sr=88200, fps=60):
    """Folders with audio.wav + take_iPhone_cal.csv whose targets follow the audio."""
    import pandas as pd
    from neurosync_trainer_lite_amd.utils.audio.load_audio import write_wav
    from neurosync_trainer_lite_amd.utils.csv.save_csv import BLENDSHAPE_COLUMNS
    rng = np.random.default_rng(seed)
    mix = np.random.default_rng(1000).normal(size=(3, 61))  # shared by every clip: one mapping to learn
    k = np.exp(-np.arange(-30, 31) ** 2 / (2 * 8.0 ** 2))
    k /= k.sum()
    dirs = []
    for c in range(clips):
        n, nf = int(seconds * sr), int(seconds * fps)
        t = np.arange(n) / sr
        f0 = rng.uniform(80, 300)
        rate, ph = rng.uniform(1.5, 5.0), rng.uniform(0, 6.28)
        env = lambda x: 0.5 + 0.45 * np.sin(2 * np.pi * rate * x + ph)  # noqa: E731
        y = sum((0.6 / h) * np.sin(2 * np.pi * h * f0 * t + rng.uniform(0, 6.28)) for h in (1, 2, 3))
        y = y * env(t) + 0.01 * rng.standard_normal(n)
        d = os.path.join(root, "clip%03d" % c)
        os.makedirs(d, exist_ok=True)
        write_wav(os.path.join(d, "audio.wav"), (y / np.abs(y).max()).astype(np.float32), sr)
        tf = np.arange(nf) / fps
        e = env(tf)
        de = np.gradient(e) * fps / (2 * np.pi * 5.0)
        feats = np.stack([e - 0.5, de, np.full(nf, (f0 - 190) / 110)], 1)
        z = feats @ mix * 0.6 + 0.3
        z += 0.05 * np.stack([np.convolve(rng.standard_normal(nf), k, mode="same") for _ in range(61)], 1)
        z[:, :52] = np.clip(z[:, :52], 0, 1)
        z[:, 52:] = 0.3 * np.tanh(z[:, 52:])
        df = pd.DataFrame(z, columns=BLENDSHAPE_COLUMNS)
        df.insert(0, "BlendshapeCount", 61)
        df.insert(0, "Timecode", ["%02d:%02d:%02d:%02d.000" % (i // 216000, i // 3600 % 60, i // 60 % 60, i % 60)
                                  for i in range(nf)])
        df.to_csv(os.path.join(d, "take_iPhone_cal.csv"), index=False)
        dirs.append(d)
    return dirs


class OracleModel:
    """process_audio_features' model interface (eval / encoder / decoder) over the
    oracle's parameters, on the CPU in fp32."""

    def __init__(self, params, num_heads):
        from oracle import model_ref
        self.p, self.h, self.ref = params, num_heads, model_ref

    def eval(self):
        return self

    def encoder(self, src):
        return self.ref.encoder_forward(self.p, src.cpu().float(), self.h)

    def decoder(self, mem):
        return self.ref.decoder_forward(self.p, mem, self.h)


def run(steps=300, D=256, H=4, L=2, B=16, T=128, lr=1e-4, seed=0, modes=("bf16", "fp32", "fp8"), log=print):
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.dataset.dataset import prepare_dataloader
    from neurosync_trainer_lite_amd.utils.audio.extraction.extract_features import extract_audio_features
    from neurosync_trainer_lite_amd.utils.audio.processing.audio_processing import process_audio_features
    from neurosync_trainer_lite_amd.utils.csv.save_csv import save_generated_data_as_csv
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    from neurosync_trainer_lite_amd.utils.validation import save_comparison_stats
    from oracle import model_ref

    dev = torch.device("cuda", 0)
    cfg = dict(training_config, hidden_dim=D, num_heads=H, n_layers=L, dropout=0.0, batch_size=B,
               micro_batch_size=T, frame_size=T, learning_rate=lr, warmup_epochs=0)
    out = {"config": {"hidden_dim": D, "num_heads": H, "n_layers": L, "batch": B, "seq": T, "steps": steps,
                      "lr": lr, "dropout": 0.0, "optimizer": "Adam (coupled L2 1e-5), clip 2.0, constant lr"}}
    with tempfile.TemporaryDirectory(prefix="nstl_d2_") as tmp, contextlib.redirect_stdout(sys.stderr):
        train_root, val_root = os.path.join(tmp, "train"), os.path.join(tmp, "val")
        learnable_corpus(train_root, 8, 40.0, seed)
        val_dir = learnable_corpus(val_root, 1, 20.0, seed + 77)[0]
        t0 = time.perf_counter()
        torch.manual_seed(seed)
        _, dl = prepare_dataloader(dict(cfg, root_dir=train_root, include_fast=True, include_slow=False))
        batches = []
        while len(batches) < steps:
            for src, trg in dl:
                if src.shape[0] == B:
                    batches.append((src.clone(), trg.clone()))
                if len(batches) == steps:
                    break
        feats, _ = extract_audio_features(os.path.join(val_dir, "audio.wav"))
        gt_csv = os.path.join(val_dir, "take_iPhone_cal.csv")
        out["data"] = {"train_clips": 8, "train_seconds": 40.0, "windows_per_epoch": len(dl.dataset),
                       "val_frames": int(feats.shape[0]), "build_s": round(time.perf_counter() - t0, 1)}
        params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), 5)

        def validate(model, tag):
            gen = process_audio_features(feats, model, dev, cfg)
            csv = os.path.join(tmp, "gen_%s.csv" % tag)
            save_generated_data_as_csv(gen, csv)
            stats = save_comparison_stats(csv, gt_csv, os.path.join(tmp, "stats_%s.txt" % tag))
            return gen, {k.split(" (")[0]: round(float(v), 6) for k, v in stats.items()}

        preds, losses = {}, {}
        # the reference step (fp32 CPU restatement)
        t0 = time.perf_counter()
        orc = model_ref.OracleTrainer(params, H, lr=lr, weight_decay=cfg["weight_decay"])
        ol = []
        for src, trg in batches:
            loss, _, _ = orc.step(src.float(), trg.float())
            ol.append(float(loss))
        with torch.no_grad():
            g, st = validate(OracleModel({k: v.detach() for k, v in orc.p.items()}, H), "oracle")
        preds["oracle"], losses["oracle"] = g, ol
        out["reference_fp32_cpu"] = dict(st, first_loss=round(ol[0], 4), last_loss=round(float(np.mean(ol[-10:])), 4),
                                         train_s=round(time.perf_counter() - t0, 1))
        log("reference: %s" % out["reference_fp32_cpu"])
        # untrained model: what the MSE starts from
        with torch.no_grad():
            _, st0 = validate(OracleModel(params, H), "init")
        out["untrained"] = st0
        for mode in modes:
            t0 = time.perf_counter()
            c = dict(cfg, use_amp=mode != "fp32", use_fp8=mode == "fp8")
            model = build_model(c, dev)
            model.load_state_dict(params, strict=True)
            crit, opt, _ = prepare_training_components(c, model)
            model.train()
            bl = []
            for src, trg in batches:
                opt.zero_grad()
                loss = crit(model(src.to(dev)), trg.to(dev))
                loss.backward()
                opt.step(max_norm=2.0)
                bl.append(float(loss))
            g, st = validate(model, mode)
            preds[mode] = g
            diff = g - preds["oracle"]
            out["build_" + mode] = dict(st, first_loss=round(bl[0], 4), last_loss=round(float(np.mean(bl[-10:])), 4),
                                        pred_mse_vs_reference=round(float(np.mean(diff[:, :61] ** 2)), 8),
                                        train_s=round(time.perf_counter() - t0, 1))
            log("build %s: %s" % (mode, out["build_" + mode]))
            del model, opt
            torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = run(steps=a.steps, log=lambda m: print(m, file=sys.stderr, flush=True))
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
