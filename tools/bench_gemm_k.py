"""K-scaling of the 256x256 GEMM (fixed M, N): separates the per-tile fixed cost
(prologue + epilogue) from the K-loop rate.  python tools/bench_gemm_k.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402


def t(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2] * 1e-3


M = 16384
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
PAD = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # extra output columns (ldc = N + PAD)
dev = "cuda:0"
for out_dt in (torch.bfloat16, torch.float32):
    pts = []
    for Kd in (256, 512, 1024, 2048, 4096):
        X = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
        Y = torch.empty(M, N + PAD, dtype=out_dt, device=dev)
        s = t(lambda: K.gemm(X, W, Y, M, N, Kd, ldc=N + PAD))
        pts.append((Kd, s))
        print("out %s K=%5d %8.1f us %7.1f TF/s" % (str(out_dt)[6:], Kd, s * 1e6, 2 * M * N * Kd / s / 1e12))
    # least squares s = a + b*K
    n = len(pts)
    mk = sum(k for k, _ in pts) / n
    ms = sum(s for _, s in pts) / n
    b = sum((k - mk) * (s - ms) for k, s in pts) / sum((k - mk) ** 2 for k, _ in pts)
    a = ms - b * mk
    print("  fixed %.1f us, K-loop %.1f TF/s" % (a * 1e6, 2 * M * N / b / 1e12))
