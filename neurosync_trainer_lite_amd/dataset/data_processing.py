"""Drop-in for dataset/data_processing.py (clip discovery, feature cache,
length alignment and fast/slow augmentation).

Host-side, once per clip, vectorised numpy (the reference loops in Python,
data_processing.py:33-41, 100-102); every index and blend weight follows the
reference exactly (pinned by tests/golden/data_*.npz).  Features for clips
without an ``audio_features.csv`` cache are extracted on the GPU
(utils/audio/extraction/extract_features.py).
"""
import os
import subprocess

import numpy as np
import pandas as pd

from ..utils.audio.extraction.extract_features import extract_audio_features

COLUMNS_TO_DROP = ['Timecode', 'BlendshapeCount']
_NOISE_COLUMNS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60]


def load_data(root_dir, sr, processed_folders, include_fast=True, include_slow=False):
    """data_processing.py:10-26: one (audio_features, facial_data) per clip folder.
    include_fast / include_slow reach collect_features (the reference fixes them
    at its defaults, fast on and slow off; BASELINE config C4 turns slow on)."""
    examples = []
    for folder in os.listdir(root_dir):
        folder_path = os.path.join(root_dir, folder)
        if os.path.isdir(folder_path) and folder not in processed_folders:
            audio_features, facial_data = process_folder(folder_path, sr, include_fast=include_fast,
                                                         include_slow=include_slow)
            if audio_features is not None and facial_data is not None:
                examples.append((audio_features, facial_data))
                processed_folders.add(folder)
    return examples


def scale_facial_data(facial_data, scale_factor=1.1):
    """data_processing.py:28-41."""
    return np.clip(np.asarray(facial_data, dtype=np.float64) * scale_factor, -1, 1)


_CLIP_SUFFIXES = {'.mov': 'mov', '.mp4': 'mp4', '.wav': 'wav'}


def clip_files(folder_path):
    """What process_folder reads from one clip folder: {'mov', 'mp4', 'wav',
    'facial'} -> path, plus the feature-cache path.  The facial CSV is a *.csv
    whose name contains 'iPhone_cal' (the naming rule of the reference's
    find_files, utils/video/mov_extraction.py:23); where several files of one
    kind exist, the last in os.listdir order is taken, as there."""
    found = {}
    for name in os.listdir(folder_path):
        ext = os.path.splitext(name)[1]
        kind = 'facial' if (ext == '.csv' and 'iPhone_cal' in name) else _CLIP_SUFFIXES.get(ext)
        if kind is not None:
            found[kind] = os.path.join(folder_path, name)
    return found, os.path.join(folder_path, 'audio_features.csv')


def process_folder(folder_path, sr, apply_smoothing=False, apply_over_scale=False, include_fast=True,
                   include_slow=False):
    """data_processing.py:44-78.  A video clip (mov preferred over mp4, as the
    reference's ``mov_path or mp4_path``) is decoded by ffmpeg inside
    load_audio rather than first written to an audio.wav beside it; an existing
    audio.wav beside the video is used instead, as the reference's extract_audio
    does (utils/video/mov_extraction.py:44-47).  When ffmpeg fails, the clip falls
    back to its audio_features.csv cache, or is skipped without one (the
    reference's extract_audio returns None there, :60-62)."""
    found, audio_features_csv_path = clip_files(folder_path)
    facial_csv_path = found.get('facial')
    video_path = found.get('mov') or found.get('mp4')
    audio_path = video_path or found.get('wav')
    extracted = os.path.join(folder_path, 'audio.wav')
    if video_path and os.path.exists(extracted):
        print(f"Audio already exists at {extracted}")
        audio_path = extracted
    if facial_csv_path and (audio_path or os.path.exists(audio_features_csv_path)):
        try:
            audio_features, facial_data = collect_features(audio_path, audio_features_csv_path, facial_csv_path, sr,
                                                           include_fast=include_fast, include_slow=include_slow)
        except (subprocess.CalledProcessError, FileNotFoundError) as e:
            if audio_path != video_path:
                raise
            print(f"Failed to extract audio from {video_path}: {e}")
            return None, None
        if apply_over_scale:
            facial_data = scale_facial_data(facial_data)
        facial_data[:, :61] *= 100
        if apply_smoothing:
            facial_data = smooth_facial_data(facial_data)
        return audio_features, facial_data
    return None, None


def interpolate_slower(data):
    """data_processing.py:84-106: 2N-1 frames, odd frames are midpoints."""
    data = np.asarray(data)
    n = data.shape[0]
    out = np.zeros((2 * n - 1, data.shape[1]))
    out[0::2] = data
    if n > 1:
        out[1::2] = (data[:-1] + data[1:]) / 2.0
    return out


def align_lengths(audio_features, facial_data):
    """data_processing.py:125-145: centre-trim the longer stream, then truncate."""
    len_audio, len_facial = len(audio_features), len(facial_data)
    if len_audio > len_facial:
        diff = len_audio - len_facial
        audio_features = audio_features[diff // 2: len_audio - (diff - diff // 2)]
    elif len_facial > len_audio:
        diff = len_facial - len_audio
        facial_data = facial_data[diff // 2: len_facial - (diff - diff // 2)]
    n = min(len(audio_features), len(facial_data))
    return audio_features[:n], facial_data[:n]


def collect_features(audio_path, audio_features_csv_path, facial_csv_path, sr,
                     include_fast=True, include_slow=False, blend_boundaries=True, blend_frames=30):
    """data_processing.py:108-177 (same cache file format: pandas CSV, header 0..255)."""
    if os.path.exists(audio_features_csv_path):
        print(f"Loading audio features from {audio_features_csv_path}")
        audio_features = pd.read_csv(audio_features_csv_path).values
    else:
        print(f"Extracting audio features from {audio_path}")
        audio_features, _ = extract_audio_features(audio_path, sr)
        if audio_features is not None:
            pd.DataFrame(audio_features).to_csv(audio_features_csv_path, index=False)
            print(f"Audio features saved to {audio_features_csv_path}")
    facial_data = pd.read_csv(facial_csv_path).drop(columns=COLUMNS_TO_DROP).values
    audio_features, facial_data = align_lengths(audio_features, facial_data)
    audio_versions, facial_versions = [audio_features], [facial_data]
    if include_fast:
        audio_versions.append(audio_features[::2].copy())
        facial_versions.append(facial_data[::2].copy())
    if include_slow:
        audio_versions.append(interpolate_slower(audio_features))
        facial_versions.append(smooth_facial_data(interpolate_slower(facial_data)))
    if blend_boundaries:
        return stack_with_blend(audio_versions, blend_frames), stack_with_blend(facial_versions, blend_frames)
    return np.vstack(audio_versions), np.vstack(facial_versions)


def stack_with_blend(sequences, blend_frames):
    """data_processing.py:179-197: linear cross-fade of min(blend_frames, len_a,
    len_b) frames at every boundary."""
    if not sequences:
        return None
    result = sequences[0]
    for seq in sequences[1:]:
        n = min(blend_frames, result.shape[0], seq.shape[0])
        if n <= 0:
            result = np.vstack([result, seq])
            continue
        fade_out = np.linspace(1, 0, n)[:, None]
        fade_in = np.linspace(0, 1, n)[:, None]
        result = np.vstack([result[:-n], fade_out * result[-n:] + fade_in * seq[:n], seq[n:]])
    return result


def smooth_facial_data(facial_data):
    """data_processing.py:201-204: two-tap moving average, first frame kept."""
    smoothed = np.copy(facial_data)
    smoothed[1:] = (facial_data[:-1] + facial_data[1:]) / 2
    return smoothed


def remove_specified_dimensions(facial_data):
    return np.delete(facial_data, _NOISE_COLUMNS, axis=1)


def zero_specified_columns(facial_data):
    facial_data[:, _NOISE_COLUMNS] = 0
    return facial_data
