"""Drop-in for the reference ``config.py`` (/root/reference/config.py:26-55): same keys,
same defaults.  Hidden keys the reference reads with defaults are listed explicitly:
``use_amp`` (train.py:25; here: bf16 compute when True, fp32 parity mode when False)
and ``overlap`` (audio_processing.py:53).  ``use_fp8`` (not a reference key, default
False) selects BASELINE config C5's fp8 q/k/v and FFN forward GEMMs.  ``num_gpus`` is no longer capped at 4: the
data-parallel path is one process per GPU (torchrun), see parallel.py."""
import os
import shutil

root_dir = os.path.dirname(os.path.abspath(__file__))
ffmpeg_path = shutil.which("ffmpeg") or "ffmpeg"

training_config = {
    'mode': 'scratch',
    'sr': 88200,
    'frame_rate': 60,
    'hidden_dim': 1024,
    'n_layers': 8,
    'num_heads': 16,
    'dropout': 0.3,
    'batch_size': 128,
    'micro_batch_size': 128,
    'learning_rate': 5e-5,
    'weight_decay': 1e-5,
    'n_epochs': 50,
    'output_dim': 61,
    'delta': 1,
    'w1': 1.0,
    'w2': 1.0,
    'w3': 1.0,
    'use_multi_gpu': False,
    'num_gpus': 1,
    'warmup_epochs': 0,
    'input_dim': 256,
    'frame_size': 128,
    'ffmpeg_path': ffmpeg_path,
    'root_dir': r"dataset/data",
    'model_path': r"out/model.pth",
    'audio_path': r"dataset/test_set/audio.wav",
    'ground_truth_path': r"dataset/test_set/testset.csv",
    'checkpoint_path': r"out/checkpoints/checkpoint.pth",
    'use_amp': True,
    'overlap': 16,
}
