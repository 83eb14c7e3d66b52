"""BASELINE config C1 plumbing on CPU: a synthetic clip folder (88.2 kHz sine
.wav + zero-blendshape iPhone_cal CSV) -> load_data/collect_features ->
AudioFacialDataset -> prepare_dataloader_with_split -> train_model (epoch loop,
scheduler, checkpoint + backup rotation, final model) -> resume.

The compute model here is the CPU oracle wrapped as a Module (tests/oracle_module.py)
at reduced width, and the feature cache is written by the oracle, because the
package's own model and feature kernels run only on the GPU (they are covered by
the -m gpu tests, including a full-width C1 run)."""
import os

import numpy as np
import pandas as pd
import torch

from neurosync_trainer_lite_amd.config import training_config
from neurosync_trainer_lite_amd.utils.audio.load_audio import load_and_preprocess_audio, write_wav
from neurosync_trainer_lite_amd.utils.csv.save_csv import BLENDSHAPE_COLUMNS
from oracle import data_ref


def make_corpus(root, seconds=10.0, sr=88200, cache_features=True):
    clip = os.path.join(root, "dataset", "data", "synth")
    os.makedirs(clip, exist_ok=True)
    t = np.arange(int(seconds * sr)) / sr
    write_wav(os.path.join(clip, "audio.wav"), 0.5 * np.sin(2 * np.pi * 440 * t), sr)
    n = 601
    df = pd.DataFrame(np.zeros((n, 61)), columns=BLENDSHAPE_COLUMNS)
    df.insert(0, "BlendshapeCount", 61)
    df.insert(0, "Timecode", ["00:00:%02d:%02d.000" % (i // 60, i % 60) for i in range(n)])
    df.to_csv(os.path.join(clip, "synth_iPhone_cal.csv"), index=False)
    if cache_features:
        y, _ = load_and_preprocess_audio(os.path.join(clip, "audio.wav"))
        pd.DataFrame(data_ref.extract_features(y)).to_csv(os.path.join(clip, "audio_features.csv"), index=False)
    return clip


def test_c1_plumbing(tmp_path, monkeypatch):
    from neurosync_trainer_lite_amd import train as tr
    from neurosync_trainer_lite_amd.dataset.dataset import prepare_dataloader_with_split
    from neurosync_trainer_lite_amd.utils import checkpoint_utils, validation
    from neurosync_trainer_lite_amd.utils.model_utils import lr_lambda_for
    from tests.oracle_module import OracleLoss, OracleSeq2Seq

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    monkeypatch.chdir(tmp_path)
    make_corpus(str(tmp_path))
    calls = []
    monkeypatch.setattr(validation, "generate_and_save_facial_data", lambda *a: calls.append(a[0]))
    cfg = dict(training_config)
    cfg.update(n_epochs=2, batch_size=64, micro_batch_size=32, frame_size=32, hidden_dim=32, num_heads=2,
               n_layers=1, use_amp=False, checkpoint_path="out/checkpoints/checkpoint.pth")
    torch.manual_seed(0)
    train_ds, val_ds, train_dl, val_dl = prepare_dataloader_with_split(cfg, val_split=0.1)
    # 601 frames + fast copy (301), 30-frame blend -> 872 frames -> 841 windows of 32 (+1 tail)
    assert len(train_ds) + len(val_ds) == 872 - 32 + 1 + 1
    src, trg = next(iter(train_dl))
    assert src.shape == (64, 32, 256) and trg.shape == (64, 32, 61) and src.dtype == torch.float32
    model = OracleSeq2Seq(hidden_dim=32, num_heads=2, n_layers=1)
    opt = torch.optim.Adam(model.parameters(), lr=cfg["learning_rate"], weight_decay=cfg["weight_decay"])
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda_for(cfg))
    dev = torch.device("cpu")
    steps = tr.train_model(cfg, model, None, None, None, train_dl, val_dl, OracleLoss(), opt, sched,
                           [dev, None, None, None], use_multi_gpu=False)
    assert steps == 2 * len(train_dl)
    assert calls == [0, 1]
    assert os.path.exists("out/checkpoints/checkpoint.pth") and os.path.exists("out/model.pth")
    assert len([d for d in os.listdir("out/checkpoints") if d.startswith("backup_")]) == 1
    assert os.path.exists("dataset/validation_plots/loss/loss_epoch_2.png")
    # resume (train.py:84-93)
    m2 = OracleSeq2Seq(hidden_dim=32, num_heads=2, n_layers=1, seed=1)
    o2 = torch.optim.Adam(m2.parameters(), lr=cfg["learning_rate"], weight_decay=cfg["weight_decay"])
    s2 = torch.optim.lr_scheduler.LambdaLR(o2, lr_lambda_for(cfg))
    epoch, bstep, m2, o2, s2 = checkpoint_utils.load_checkpoint(cfg["checkpoint_path"], m2, o2, s2, dev)
    assert (epoch, bstep) == (1, steps)
    for a, b in zip(m2.parameters(), model.parameters()):
        torch.testing.assert_close(a, b)
    assert s2.get_last_lr() == sched.get_last_lr()
