"""Time the GPU feature pipeline (nstl_features) on synthetic 88.2 kHz audio.
  python tools/bench_features.py [seconds]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 273.1
sr = 88200
n = int(sec * sr)
rng = np.random.default_rng(0)
t = np.arange(n) / sr
y = (0.5 * np.sin(2 * np.pi * 180 * t) * (0.6 + 0.4 * np.sin(2 * np.pi * 4 * t)) + 0.01 * rng.standard_normal(n))
y = torch.tensor((y / np.abs(y).max()).astype(np.float32), device="cuda")
f60 = K.features_frames(n, sr)
out = torch.empty(f60, 256, device="cuda")
ws = torch.empty(K.features_workspace_bytes(n, sr), dtype=torch.uint8, device="cuda")
for _ in range(2):
    K.features(y, sr, out, ws)
torch.cuda.synchronize()
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    K.features(y, sr, out, ws)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print("audio %.1f s (%d samples) -> %d frames: %.2f ms per clip, %.0f frames/s, %.1f s audio per ms"
      % (sec, n, f60, dt * 1e3, f60 / dt, sec / (dt * 1e3)))
