"""Forward GEMM operand layout on the step's shapes: the weight as B K-major
(TT, the forward's layout: W [N][K]) against B N-major (TN, W^T [K][N], the
dX layout), same epilogue, same data, alternated; median of 25 launches per
arm and rep.  A/B a build: NSTL_LIB_PATH=<.so>."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

M, D, F = 16384, 1024, 4096
dev = "cuda:0"
bf = torch.bfloat16


def t(fn, reps=25):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2] * 1e3


g = torch.Generator(device=dev).manual_seed(3)
x1, x4 = torch.randn(M, D, device=dev, generator=g).to(bf), torch.randn(M, F, device=dev, generator=g).to(bf)
rows = {}
for rep in range(3):
    for name, n, k, epi in (("ffn1 BIAS", F, D, "bias"), ("ffn1 RELU_DROP+mask", F, D, "relu"),
                            ("out  BIAS", D, D, "bias"), ("qkv  BIAS", 3 * D, D, "bias"),
                            ("ffn2 BIAS", D, F, "bias")):
        X = x1 if k == D else x4
        W = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(bf)
        Wt = W.t().contiguous()
        b = torch.randn(n, device=dev, generator=g) * 0.02
        kw = dict(epilogue=K.EPI_BIAS, bias=b)
        if epi == "relu":
            kw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=5)
        Y1, Y2 = torch.empty(M, n, dtype=bf, device=dev), torch.empty(M, n, dtype=bf, device=dev)
        kw1, kw2 = dict(kw), dict(kw, b_kmajor=False)
        if epi == "relu":
            nw = K.gemm_relu_mask_words(X, W, Y1, M, n, k, **kw1)
            kw1["relu_mask"] = torch.empty(nw, dtype=torch.int64, device=dev)
            kw2["relu_mask"] = torch.empty(nw, dtype=torch.int64, device=dev)
        K.gemm(X, W, Y1, M, n, k, **kw1)
        K.gemm(X, Wt, Y2, M, n, k, **kw2)
        torch.cuda.synchronize()
        same = torch.equal(Y1, Y2) and (epi != "relu" or torch.equal(kw1["relu_mask"], kw2["relu_mask"]))
        tt = t(lambda: K.gemm(X, W, Y1, M, n, k, **kw1))
        tn = t(lambda: K.gemm(X, Wt, Y2, M, n, k, **kw2))
        rows.setdefault(name, []).append((tt, tn, same))
for name, v in rows.items():
    print("%-22s TT %s  TN %s  outputs identical %s" % (
        name, " ".join("%6.1f" % a for a, _, _ in v), " ".join("%6.1f" % b for _, b, _ in v), all(s for _, _, s in v)))
