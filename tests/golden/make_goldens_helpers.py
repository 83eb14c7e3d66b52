"""Helpers shared by the fixture generator and the tests (no reference imports)."""
import numpy as np

from oracle import model_ref

SAMPLE_IDX = 32  # sampled elements per tensor in checksum-style fixtures


def summary(t):
    """Checksum of a tensor: sum, L2 norm and SAMPLE_IDX elements at fixed positions."""
    a = np.asarray(t, dtype=np.float64).ravel()
    rng = np.random.default_rng(12345)
    idx = rng.integers(0, a.size, SAMPLE_IDX)
    return np.concatenate([[a.sum(), np.sqrt((a * a).sum())], a[idx]])


def synth_audio(seconds, seed, sr=88200):
    """Seeded synthetic voice-like signal (3 harmonics, 4 Hz AM, noise), peak-normalised."""
    rng = np.random.default_rng(seed)
    t = np.arange(int(seconds * sr)) / sr
    f0 = rng.uniform(80, 300)
    y = sum((0.6 / h) * np.sin(2 * np.pi * h * f0 * t + rng.uniform(0, 6.28)) for h in (1, 2, 3))
    y = y * (0.55 + 0.45 * np.sin(2 * np.pi * 4 * t)) + 0.01 * rng.standard_normal(t.size)
    y = y.astype(np.float32)
    return y / np.max(np.abs(y))


def full_layer_params():
    """Seeded params of one full-width encoder layer ('e.' prefix, seed 8) and
    decoder layer ('d.' prefix, seed 9), in the reference's registration order."""
    shapes = model_ref.param_shapes(256, 1024, 1, 61)
    e = {"e." + k[len("encoder.transformer_encoder.0."):]: v for k, v in shapes.items()
         if k.startswith("encoder.transformer_encoder.0.")}
    d = {"d." + k[len("decoder.transformer_decoder.0."):]: v for k, v in shapes.items()
         if k.startswith("decoder.transformer_decoder.0.")}
    return model_ref.seeded_params(e, 8), model_ref.seeded_params(d, 9)


class FakeSeq2Seq:
    """A deterministic per-frame stand-in with the reference model's
    ``encoder``/``decoder`` split (what audio_processing.decode_audio_chunk calls),
    elementwise only so batching chunks cannot change a bit.  The position term
    makes every chunk boundary visible in the output."""

    def eval(self):
        return self

    def encoder(self, x):
        import torch
        return torch.tanh(x)

    def decoder(self, m):
        import torch
        pos = torch.arange(m.shape[1], dtype=m.dtype)[None, :, None]
        return m[..., :61] * 30.0 + m[..., 61:122] * 7.0 + pos * 0.25


INFER_FRAMES = (37, 128, 129, 250, 1000)   # chunking cases (short, exact, +1, ragged, long)
INFER_MODEL = dict(D=128, H=2, L=1, seed=31, frames=300)
