"""Time the fused-epilogue GEMMs of one 228M training step (B=128, T=128), one
line per (epilogue, shape): median of 20 launches.  Compare two builds with
NSTL_LIB_PATH=<other .so> python tools/bench_gemm_epi.py"""
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


cs, sn = rotation_tables(T, 64, dev)
rows = []
x, x4 = r(M, D), r(M, F)
for name, n, k, kw in (
        ("fwd out  BIAS", D, D, dict(epilogue=K.EPI_BIAS)),
        ("fwd ffn2 BIAS", D, F, dict(epilogue=K.EPI_BIAS)),
        ("fwd ffn1 BIAS", F, D, dict(epilogue=K.EPI_BIAS)),
        ("fwd ffn1 RELU p0", F, D, dict(epilogue=K.EPI_BIAS_RELU_DROP, p_drop=0.0, seed=5)),
        ("fwd ffn1 RELU_DROP", F, D, dict(epilogue=K.EPI_BIAS_RELU_DROP, p_drop=0.3, seed=5)),
        ("fwd qkv  BIAS", 3 * D, D, dict(epilogue=K.EPI_BIAS)),
        ("fwd qkv  ROPE", 3 * D, D, dict(epilogue=K.EPI_BIAS_ROPE, rope=(cs, sn, T, 64), rope_cols=2 * D)),
        ("fwd kvc  BIAS", 2 * D, D, dict(epilogue=K.EPI_BIAS)),
        ("fwd kvc  ROPE", 2 * D, D, dict(epilogue=K.EPI_BIAS_ROPE, rope=(cs, sn, T, 64), rope_cols=D))):
    X = x if k == D else x4
    W, b = r(n, k), torch.zeros(n, device=dev)
    Y = torch.empty(M, n, dtype=bf, device=dev)
    s = t(lambda: K.gemm(X, W, Y, M, n, k, bias=b, **kw))
    rows.append((name, 2 * M * n * k, s))
    if "RELU_DROP" in name:
        nw = K.gemm_relu_mask_words(X, W, Y, M, n, k, bias=b, **kw)
        rm = torch.empty(nw, dtype=torch.int64, device=dev)
        s = t(lambda: K.gemm(X, W, Y, M, n, k, bias=b, relu_mask=rm, **kw))
        rows.append((name + "+mask", 2 * M * n * k, s))
h = torch.relu(r(M, F))
for name, n, k, out_dt, kw in (
        ("dX  out  bf16", D, D, bf, dict(beta=0.0)),
        ("dX  ffn2 bf16", D, F, bf, dict(beta=0.0)),
        ("dX  ffn2 DRELU", D, F, bf, dict(beta=0.0, epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=F, p_drop=0.3)),
        ("dX  ffn1 F32 beta1", F, D, torch.float32, dict(beta=1.0)),
        ("dX  qkv  F32 beta1", 3 * D, D, torch.float32, dict(beta=1.0)),
        ("dX  q    F32 beta1", D, D, torch.float32, dict(beta=1.0)),
        ("dX  ffn1 F32 beta0", F, D, torch.float32, dict(beta=0.0))):
    dY, W = r(M, n), r(n, k)
    dX = torch.zeros(M, k, dtype=out_dt, device=dev)
    s = t(lambda: K.gemm(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, **kw))
    rows.append((name, 2 * M * n * k, s))
    if "DRELU" in name:
        nw = K.gemm_relu_mask_words(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, **kw)
        rm = torch.zeros(nw, dtype=torch.int64, device=dev) - 1
        kw2 = dict(kw, relu_mask=rm)
        s = t(lambda: K.gemm(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, **kw2))
        rows.append((name + "+mask", 2 * M * n * k, s))
        nr = K.gemm_colsum_rows(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, **kw2)
        cp = torch.empty(nr, k, dtype=torch.float32, device=dev)
        s = t(lambda: K.gemm(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, colsum_part=cp, **kw2))
        rows.append((name + "+mask+csum", 2 * M * n * k, s))
ws = torch.empty(16 * D * D, dtype=torch.float32, device=dev)
for name, n, k, split in (("dW  out  split8", D, D, 8), ("dW  out  split16", D, D, 16),
                          ("dW  qkv  split5", 3 * D, D, 5), ("dW  ffn1 split4", F, D, 4)):
    dY, X = r(M, n), r(M, k)
    G = torch.zeros(n, k, dtype=torch.float32, device=dev)
    s = t(lambda: K.gemm(dY, X, G, n, k, M, a_kmajor=False, b_kmajor=False, split_k=split, workspace=ws))
    rows.append((name, 2 * M * n * k, s))
# one 256-tile weight-gradient GEMM without split-K (K = all 16384 tokens): the rate
# a per-layer grouped dW launch would run at; beta 0 and 1 (gradient accumulation)
dY, X = r(M, 4096), r(M, 4096)
G = torch.zeros(4096, 4096, dtype=torch.float32, device=dev)
for beta in (0.0, 1.0):
    s = t(lambda: K.gemm(dY, X, G, 4096, 4096, M, a_kmajor=False, b_kmajor=False, beta=beta))
    rows.append(("dW  4096^2 nosplit b%d" % beta, 2 * M * 4096 * 4096, s))
# the same problem with K-major operands (forward layout): isolates the cost of
# the MN-major (transpose-read) operand path
At, Bt = dY.t().contiguous(), X.t().contiguous()
s = t(lambda: K.gemm(At, Bt, G, 4096, 4096, M, a_kmajor=True, b_kmajor=True))
rows.append(("TT  4096^2 K=16384", 2 * M * 4096 * 4096, s))
s = t(lambda: K.gemm(At, X, G, 4096, 4096, M, a_kmajor=True, b_kmajor=False))
rows.append(("TN  4096^2 K=16384", 2 * M * 4096 * 4096, s))
# the step's grouped weight-gradient launches: one decoder layer (7 GEMMs, 256
# tiles) and four encoder layers (16 GEMMs, 768 tiles), K = 16384 tokens
def group(shapes):
    probs, fl = [], 0
    for n, k in shapes:
        dY, X = r(M, n), r(M, k)
        G = torch.empty(n, k, dtype=torch.float32, device=dev)
        probs.append((dY, X, G, n, k, M, dict(a_kmajor=False, b_kmajor=False)))
        fl += 2 * M * n * k
    return probs, fl


dec = [(D, F), (F, D), (D, D), (D, D), (2 * D, D), (D, D), (3 * D, D)]
enc = [(D, F), (F, D), (D, D), (3 * D, D)] * 4
for name, shapes in (("dW  group dec layer", dec), ("dW  group enc x4", enc)):
    probs, fl = group(shapes)
    s = t(lambda: K.gemm_grouped(probs))
    rows.append((name, fl, s))
    del probs
for nm, fl, s in rows:
    print("%-22s %8.1f TF/s %9.1f us" % (nm, fl / s / 1e12, s * 1e6))
