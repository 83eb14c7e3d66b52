"""Drop-in for utils/audio/extraction/extract_features.py:6-46.

``extract_audio_features`` keeps the reference signature and return value
(``(f64 [F60, 256] or None, y)``); the feature math runs on the GPU in one C-ABI
call (``nstl_features``: framed STFT as an f32 MFMA GEMM, Slaney mel + dB + DCT,
CMVN, Savitzky-Golay deltas, autocorrelation lags, frame-pair reduction).
``extract_audio_features_device`` is the device-resident form used by the
training/inference paths (no host round trip).
"""
import numpy as np
import torch

from .... import _hip as K
from ..load_audio import load_and_preprocess_audio, load_audio_from_bytes

N_FEATURES = 256
MIN_FRAMES = 9


def frame_params(sr):
    frame_length = int(0.01667 * sr)  # extract_features.py:12
    return frame_length, frame_length // 2


def extract_audio_features_device(y, sr=88200, device=None, stream=None):
    """y: 1-D audio (numpy or tensor), peak-normalised -> f32 [F60, 256] tensor on
    the device, or None when the clip has fewer than 9 frames
    (extract_features.py:16-21)."""
    frame_length, hop = frame_params(sr)
    n = len(y)
    if n < frame_length or (n - frame_length) // hop + 1 < MIN_FRAMES:
        return None
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    yt = torch.as_tensor(np.ascontiguousarray(y, dtype=np.float32) if not torch.is_tensor(y) else y,
                         dtype=torch.float32).to(device).contiguous()
    f60 = K.features_frames(n, sr)
    out = torch.empty(f60, N_FEATURES, dtype=torch.float32, device=device)
    ws = torch.empty(K.features_workspace_bytes(n, sr), dtype=torch.uint8, device=device)
    K.features(yt, sr, out, ws, stream=stream)
    return out


def extract_audio_features(audio_input, sr=88200, from_bytes=False):
    """extract_features.py:6-24."""
    if from_bytes:
        y, sr = load_audio_from_bytes(audio_input, sr)
    else:
        y, sr = load_and_preprocess_audio(audio_input, sr)
    frame_length, hop = frame_params(sr)
    num_frames = (len(y) - frame_length) // hop + 1
    if num_frames < MIN_FRAMES:
        print(f"Audio file is too short: {num_frames} frames, required: {MIN_FRAMES} frames")
        return None, None
    feats = extract_audio_features_device(y, sr)
    return feats.double().cpu().numpy(), y
