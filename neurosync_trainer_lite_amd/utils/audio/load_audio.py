"""Audio ingest (drop-in for utils/audio/load_audio.py:6-53).

The reference decodes with ``librosa.load(path, sr=88200)`` (mono mix, soxr
resampling) and peak-normalises.  librosa is not part of this framework: WAV
(RIFF PCM 8/16/24/32-bit, IEEE float 32/64, WAVE_FORMAT_EXTENSIBLE) is parsed
here, channels are averaged to mono (librosa's ``to_mono``), and other sample
rates are resampled with a windowed-sinc polyphase filter
(``scipy.signal.resample_poly``).  That resampler is not soxr: for 88.2 kHz input
(the reference's own capture rate, and every benchmark input) there is no
resampling and the samples are identical; for other rates parity is unpinned
(DESIGN.md).  Other containers (mov/mp4) are decoded by ffmpeg to mono 16-bit
PCM at 88.2 kHz on a pipe, the same samples as the audio.wav the reference
first writes with ffmpeg (utils/video/mov_extraction.py:39-62).
"""
import io
import os
import struct
import subprocess
from math import gcd

import numpy as np

TARGET_SR = 88200

_PCM, _FLOAT, _EXTENSIBLE = 1, 3, 0xFFFE


def _parse_wav(buf):
    if len(buf) < 12 or buf[0:4] != b"RIFF" or buf[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(buf):
        cid, size = buf[pos:pos + 4], struct.unpack_from("<I", buf, pos + 4)[0]
        body = buf[pos + 8: pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack_from("<HHIIHH", body, 0)
            if tag == _EXTENSIBLE and len(body) >= 26:
                tag = struct.unpack_from("<H", body, 24)[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError("WAV without fmt/data chunk")
    tag, ch, sr, bits = fmt
    if tag == _PCM:
        if bits == 8:
            x = (np.frombuffer(data, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(data, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(data[: len(data) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = (np.frombuffer(data, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
        else:
            raise ValueError("unsupported PCM width %d" % bits)
    elif tag == _FLOAT:
        x = np.frombuffer(data, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise ValueError("unsupported WAV format tag %d" % tag)
    x = x[: len(x) // ch * ch].reshape(-1, ch)
    return (x.mean(axis=1) if ch > 1 else x[:, 0]).astype(np.float32), sr


def resample(y, orig_sr, target_sr):
    if orig_sr == target_sr:
        return y
    from scipy.signal import resample_poly
    g = gcd(int(orig_sr), int(target_sr))
    return resample_poly(y, target_sr // g, orig_sr // g).astype(np.float32)


def peak_normalise(y):
    """y / max|y| when non-zero (load_audio.py:13-15)."""
    m = np.max(np.abs(y)) if y.size else 0.0
    return y / m if m > 0 else y


def _decode_container(path, sr):
    """Any container ffmpeg reads -> mono samples at ``sr`` (ffmpeg resamples).
    Decoded as 16-bit PCM and scaled by 1/32768, the samples the reference's
    audio.wav round trip gives (ffmpeg's default WAV codec is pcm_s16le,
    utils/video/mov_extraction.py:39-62, read back by librosa)."""
    from ...config import training_config
    sr = sr or TARGET_SR
    cmd = [training_config['ffmpeg_path'], '-v', 'error', '-i', path, '-vn', '-ac', '1', '-ar', str(sr),
           '-f', 's16le', '-acodec', 'pcm_s16le', '-']
    pcm = subprocess.run(cmd, check=True, stdout=subprocess.PIPE).stdout
    return np.frombuffer(pcm, '<i2').astype(np.float32) / 32768.0, sr


def load_audio(audio_path, sr=TARGET_SR):
    """load_audio.py:18-21: decode, mono, resample to ``sr``."""
    if os.path.splitext(audio_path)[1].lower() in ('.mov', '.mp4'):
        y, file_sr = _decode_container(audio_path, sr)
    else:
        with open(audio_path, "rb") as f:
            y, file_sr = _parse_wav(f.read())
    if sr is not None:
        y, file_sr = resample(y, file_sr, sr), sr
    print(f"Loaded audio file '{audio_path}' with sample rate {file_sr}")
    return y, file_sr


def load_and_preprocess_audio(audio_path, sr=TARGET_SR):
    """load_audio.py:6-16."""
    y, sr = load_audio(audio_path, sr)
    if sr != TARGET_SR:
        y, sr = resample(y, sr, TARGET_SR), TARGET_SR
    return peak_normalise(y), sr


def load_audio_from_bytes(audio_bytes, sr=TARGET_SR):
    """load_audio.py:23-33."""
    y, file_sr = _parse_wav(io.BytesIO(audio_bytes).getvalue())
    if sr is not None:
        y, file_sr = resample(y, file_sr, sr), sr
    return peak_normalise(y), file_sr


def load_audio_file_from_memory(audio_bytes, sr=TARGET_SR):
    """load_audio.py:35-45."""
    y, sr = load_audio_from_bytes(audio_bytes, sr)
    print(f"Loaded audio data with sample rate {sr}")
    return y, sr


def write_wav(path, y, sr, bits=16):
    """16-bit (or 32-bit float) mono WAV writer (test corpora, save_audio)."""
    y = np.asarray(y)
    if bits == 16:
        payload = (np.clip(y, -1.0, 32767 / 32768) * 32768.0).round().astype("<i2").tobytes()
        tag, width = _PCM, 2
    else:
        payload = y.astype("<f4").tobytes()
        tag, width = _FLOAT, 4
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(payload), b"WAVE", b"fmt ", 16, tag, 1, sr,
                      sr * width, width, 8 * width, b"data", len(payload))
    with open(path, "wb") as f:
        f.write(hdr + payload)
