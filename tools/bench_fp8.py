"""fp8 (BASELINE config C5) vs bf16 forward projections of the 228M step
(B=128, T=128 -> M=16384): median of 20 launches per (shape, epilogue), plus the
row-wise quantization passes the fp8 path adds.  One line per case:
name, TFLOP/s bf16, TFLOP/s fp8, speedup."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402
from neurosync_trainer_lite_amd.engine import rotation_tables  # noqa: E402

M, D, F, T = 16384, 1024, 4096, 128
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


def q8(x):
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=dev)
    s = torch.empty(x.shape[0], dtype=torch.float32, device=dev)
    K.fp8_quant_rows([(x, x.shape[0], x.shape[1], q, s)])
    return q, s


cs, sn = rotation_tables(T, 64, dev)
x, x4 = r(M, D), torch.relu(r(M, F))
qx, sx = q8(x)
qx4, sx4 = q8(x4)
for name, n, k, kw in (
        ("out  BIAS", D, D, dict(epilogue=K.EPI_BIAS)),
        ("ffn2 BIAS", D, F, dict(epilogue=K.EPI_BIAS)),
        ("ffn1 BIAS", F, D, dict(epilogue=K.EPI_BIAS)),
        ("ffn1 RELU_DROP", F, D, dict(epilogue=K.EPI_BIAS_RELU_DROP, p_drop=0.3, seed=5)),
        ("qkv  ROPE", 3 * D, D, dict(epilogue=K.EPI_BIAS_ROPE, rope=(cs, sn, T, 64), rope_cols=2 * D)),
        ("kvc  ROPE", 2 * D, D, dict(epilogue=K.EPI_BIAS_ROPE, rope=(cs, sn, T, 64), rope_cols=D)),
        ("ffn1 f32 none", F, D, dict(out=torch.float32))):
    out_dt = kw.pop("out", bf)
    X, QX, SX = (x, qx, sx) if k == D else (x4, qx4, sx4)
    W, b = r(n, k), torch.zeros(n, device=dev)
    QW, SW = q8(W)
    Y = torch.empty(M, n, dtype=out_dt, device=dev)
    if out_dt == torch.float32:
        kw, b = {}, None
    t16 = t(lambda: K.gemm(X, W, Y, M, n, k, bias=b, **kw))
    t8 = t(lambda: K.gemm(QX, QW, Y, M, n, k, bias=b, a_scale=SX, b_scale=SW, **kw))
    fl = 2 * M * n * k
    print("%-16s M%d N%d K%d  bf16 %7.1f us %6.0f TF/s   fp8 %7.1f us %6.0f TF/s   x%.2f" % (
        name, M, n, k, t16 * 1e6, fl / t16 / 1e12, t8 * 1e6, fl / t8 / 1e12, t16 / t8), flush=True)
for name, X in (("quant rows 16384x1024 bf16", x), ("quant rows 16384x4096 bf16", x4)):
    QX, SX = q8(X)
    tq = t(lambda: K.fp8_quant_rows([(X, X.shape[0], X.shape[1], QX, SX)]))
    by = X.numel() * 3 + X.shape[0] * 4
    print("%-28s %7.1f us  %6.2f TB/s" % (name, tq * 1e6, by / tq / 1e12), flush=True)
