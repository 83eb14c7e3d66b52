"""numpy restatement of the reference data + feature path (TEST INFRA ONLY).

Integer/index work (windowing, fast/slow augmentation, blending) follows the
reference bit-exactly; pinned by ``tests/golden/data_*.npz`` generated from the
imported reference (``tests/golden/make_goldens.py``).

Feature path:
  * autocorrelation branch (extract_features_utils.py:54-128): pinned against the
    reference run here with a ``librosa.util.frame`` stand-in (an exact numpy
    equivalent), fixture ``tests/golden/features_autocorr.npz``.
  * MFCC branch (extract_features_utils.py:17-30 -> ``librosa.feature.mfcc`` and
    ``librosa.feature.delta``): librosa is NOT installed in this image and its
    source is not on disk, so this restatement follows librosa >= 0.10's
    published algorithm (STFT center=True/pad_mode='constant', periodic Hann,
    power 2, 128 Slaney mel filters with Slaney area norm, power_to_db(ref=1,
    amin=1e-10, top_db=80), DCT-II ortho, 23 coefficients; delta = Savitzky-Golay
    width 9, mode 'interp').  PARITY UNPINNED for that branch.
"""
import numpy as np

FRAME_LENGTH = 1470  # int(0.01667 * 88200), extract_features.py:12
HOP_LENGTH = 735     # frame_length // 2, extract_features.py:13
N_MFCC = 23
N_MELS = 128
N_AUTOCORR = 187


# ----------------------------------------------------------------------------
# dataset windowing (dataset/dataset.py:58-98)
# ----------------------------------------------------------------------------
def window_plan(n_audio, n_facial, window):
    """Return the list of (start, n_valid) the reference materialises.

    Stride-1 windows start at 0..max_frames-window (dataset.py:66); one extra tail
    window starting at max_frames-window is appended when max_frames % window != 0
    (:77-96).  n_valid < window only happens for the tail of a clip shorter than
    ``window``, which the reference rejects with ValueError (shape mismatch at :91).
    """
    max_frames = max(n_audio, n_facial)
    plan = [(s, window) for s in range(0, max_frames - window + 1)]
    if max_frames % window != 0:
        start = max_frames - window
        if start < 0:
            raise ValueError("clip shorter than one window (%d < %d)" % (max_frames, window))
        plan.append((start, window))
    return plan


def windows(audio, facial, window):
    """Materialised windows as float32, exactly the reference's process_example."""
    out = []
    for start, _ in window_plan(len(audio), len(facial), window):
        a = np.zeros((window, audio.shape[1]))
        f = np.zeros((window, facial.shape[1]))
        a[:] = audio[start:start + window]
        f[:] = facial[start:start + window]
        out.append((a.astype(np.float32), f.astype(np.float32)))
    return out


# ----------------------------------------------------------------------------
# augmentation (dataset/data_processing.py)
# ----------------------------------------------------------------------------
def interpolate_slower(data):
    """data_processing.py:84-106: 2N-1 rows, odd rows are pair midpoints."""
    n = data.shape[0]
    out = np.zeros((2 * n - 1, data.shape[1]))
    out[0::2] = data
    out[1::2] = (data[:-1] + data[1:]) / 2.0
    return out


def smooth_facial_data(x):
    """data_processing.py:201-204."""
    y = np.copy(x)
    y[1:] = (x[:-1] + x[1:]) / 2
    return y


def stack_with_blend(seqs, blend_frames):
    """data_processing.py:179-197: concatenate with a linear cross-fade of
    n = min(blend_frames, len_a, len_b) rows at each boundary."""
    res = seqs[0]
    for s in seqs[1:]:
        n = min(blend_frames, res.shape[0], s.shape[0])
        if n <= 0:
            res = np.vstack([res, s])
            continue
        w1 = np.linspace(1, 0, n).reshape(n, 1)
        w2 = np.linspace(0, 1, n).reshape(n, 1)
        res = np.vstack([res[:-n], w1 * res[-n:] + w2 * s[:n], s[n:]])
    return res


def align_lengths(audio, facial):
    """data_processing.py:124-143: centre-trim the longer stream, then truncate."""
    la, lf = len(audio), len(facial)
    if la > lf:
        d = la - lf
        audio = audio[d // 2: la - (d - d // 2)]
    elif lf > la:
        d = lf - la
        facial = facial[d // 2: lf - (d - d // 2)]
    m = min(len(audio), len(facial))
    return audio[:m], facial[:m]


def augment(audio, facial, include_fast=True, include_slow=False, blend=True, blend_frames=30):
    """collect_features after the feature load, data_processing.py:124-175."""
    audio, facial = align_lengths(audio, facial)
    av, fv = [audio], [facial]
    if include_fast:
        av.append(audio[::2].copy())
        fv.append(facial.copy()[::2].copy())
    if include_slow:
        av.append(interpolate_slower(audio))
        fv.append(smooth_facial_data(interpolate_slower(facial)))
    if blend:
        return stack_with_blend(av, blend_frames), stack_with_blend(fv, blend_frames)
    return np.vstack(av), np.vstack(fv)


# ----------------------------------------------------------------------------
# features (utils/audio/extraction/*)
# ----------------------------------------------------------------------------
def reduce_features(x):
    """extract_features_utils.py:33-44: mean of frame pairs, odd tail kept. x [C, F]."""
    n = x.shape[1]
    r = x[:, : n // 2 * 2].reshape(x.shape[0], -1, 2).mean(axis=2)
    if n % 2 == 1:
        r = np.hstack((r, x[:, -1:]))
    return r


def cmvn(x):
    """extract_features_utils.py:5-8 (population std)."""
    return (x - x.mean(axis=1, keepdims=True)) / (x.std(axis=1, keepdims=True) + 1e-10)


def frame_signal(y, frame_length, hop_length):
    """librosa.util.frame equivalent: [frame_length, n_frames] view."""
    n = 1 + (len(y) - frame_length) // hop_length
    idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n)[None, :]
    return y[idx]


def autocorr_features_120(y, frame_length=FRAME_LENGTH, hop_length=HOP_LENGTH,
                          n_coeff=N_AUTOCORR):
    """extract_overlapping_autocorr + fix_edge_frames_autocorr,
    extract_features_utils.py:54-113.  Returns f64 [n_coeff, F120]."""
    pad = frame_length // 2
    yp = np.pad(y, pad_width=pad, mode="reflect")
    frames = frame_signal(yp, frame_length, hop_length)
    # float32 mean along the contiguous sample axis (numpy pairwise summation, as
    # the reference's strided librosa.util.frame view reduces it)
    mean = np.ascontiguousarray(frames.T).mean(axis=1)
    frames = frames - mean[None, :]
    w = frames * np.hanning(frame_length)[:, None]
    nf = w.shape[1]
    ac = np.empty((n_coeff + 1, nf))
    for k in range(n_coeff + 1):
        ac[k] = np.einsum("ij,ij->j", w[: frame_length - k], w[k:])
    nz = ac[0] != 0
    ac[:, nz] = ac[:, nz] / ac[0, nz]
    ac = ac[1:]
    if np.all(np.abs(ac[:, 0]) < 1e-7):
        ac[:, 0] = ac[:, 1]
    if np.all(np.abs(ac[:, -1]) < 1e-7):
        ac[:, -1] = ac[:, -2]
    return ac


def hz_to_mel_slaney(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def mel_to_hz_slaney(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_basis(sr, n_fft, n_mels=N_MELS):
    """librosa.filters.mel(htk=False, norm='slaney', fmin=0, fmax=sr/2), float32."""
    nb = 1 + n_fft // 2
    fftfreqs = np.arange(nb) * (sr / n_fft)
    mel_f = mel_to_hz_slaney(np.linspace(hz_to_mel_slaney(0.0), hz_to_mel_slaney(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, nb))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


def dct_ortho_matrix(n_in, n_out):
    """DCT-II, norm='ortho' rows 0..n_out-1: C[k, n]."""
    n = np.arange(n_in)
    k = np.arange(n_out)[:, None]
    c = np.cos(np.pi * k * (2 * n + 1) / (2.0 * n_in)) * np.sqrt(2.0 / n_in)
    c[0] /= np.sqrt(2.0)
    return c


def mfcc_120(y, sr, n_fft=FRAME_LENGTH, hop_length=HOP_LENGTH, n_mfcc=N_MFCC):
    """librosa.feature.mfcc(y, sr, n_mfcc, n_fft, hop_length) restated (see header)."""
    yp = np.pad(y.astype(np.float64), n_fft // 2, mode="constant")
    frames = frame_signal(yp, n_fft, hop_length)  # [n_fft, F]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    spec = np.fft.rfft(frames * win[:, None], axis=0)
    power = np.abs(spec) ** 2
    mel = mel_basis(sr, n_fft).astype(np.float64) @ power
    db = 10.0 * np.log10(np.maximum(1e-10, mel))
    db = np.maximum(db, db.max() - 80.0)
    return dct_ortho_matrix(N_MELS, n_mfcc) @ db


def savgol_delta(x, order, width=9):
    """librosa.feature.delta(x, width=9, order, mode='interp') = savgol_filter."""
    from scipy.signal import savgol_filter
    return savgol_filter(x, width, polyorder=order, deriv=order, axis=-1, mode="interp")


def mfcc_block(y, sr):
    """extract_overlapping_mfcc + reduce, extract_features_utils.py:11-30 -> [F60, 69]."""
    m = cmvn(mfcc_120(y, sr))
    full = np.vstack([m, savgol_delta(m, 1), savgol_delta(m, 2)])
    return reduce_features(full).T


def extract_features(y, sr=88200):
    """extract_audio_features after load (extract_features.py:6-46) -> f64 [F60, 256],
    or None if fewer than 9 frames."""
    num_frames = (len(y) - FRAME_LENGTH) // HOP_LENGTH + 1
    if num_frames < 9:
        return None
    mf = mfcc_block(y, sr)
    ac = reduce_features(autocorr_features_120(y)).T
    return np.hstack([mf, ac])


def peak_normalise(y):
    """load_audio.py:13-15."""
    m = np.max(np.abs(y))
    return y / m if m > 0 else y
