"""Time every GEMM shape of one 228M training step (B=128, T=128) through nstl_gemm.

  python tools/bench_gemm.py            (NSTL_GEMM_SMALL=1 forces the 128x128 kernel)
Prints one line per shape: TFLOP/s and microseconds (median of 20).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

M, D, F = 16384, 1024, 4096
dev = "cuda:0"
bf = torch.bfloat16


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


def r(*s, dtype=bf):
    return (torch.randn(*s, device=dev) * 0.1).to(dtype)


ws = torch.empty(64 << 20, dtype=torch.float32, device=dev)
rows = []
for name, n, k in (("qkv", 3 * D, D), ("out", D, D), ("ffn1", F, D), ("ffn2", D, F), ("kv", 2 * D, D), ("emb", D, 256)):
    X, W, b = r(M, k), r(n, k), torch.zeros(n, device=dev)
    Y = torch.empty(M, n, dtype=bf, device=dev)
    s = t(lambda: K.gemm(X, W, Y, M, n, k, epilogue=K.EPI_BIAS, bias=b))
    rows.append(("fwd " + name, 2 * M * n * k, s))
    dY, dX = r(M, n), torch.empty(M, k, dtype=torch.float32, device=dev)
    s = t(lambda: K.gemm(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, beta=1.0))
    rows.append(("dX  " + name, 2 * M * n * k, s))
    G = torch.empty(n, k, dtype=torch.float32, device=dev)
    tiles = ((n + 127) // 128) * ((k + 127) // 128)
    for split in sorted({1, max(1, min(16, 512 // tiles)), 4, 8}):
        s = t(lambda: K.gemm(dY, X, G, n, k, M, a_kmajor=False, b_kmajor=False, split_k=split, workspace=ws))
        rows.append(("dW  %s split%d" % (name, split), 2 * M * n * k, s))
for nm, fl, s in rows:
    print("%-22s %8.1f TF/s %9.1f us" % (nm, fl / s / 1e12, s * 1e6))
