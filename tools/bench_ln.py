"""LayerNorm(+dropout+residual) fwd/bwd at the 228M step's shape (M=16384, D=1024,
bf16, two dropout masks, f32 residual gradient).  python tools/bench_ln.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

M, D = 16384, 1024
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


x, y = torch.randn(M, D, device=dev).to(bf), torch.randn(M, D, device=dev).to(bf)
gamma, beta = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev) * 0.1
s, out = torch.empty(M, D, dtype=bf, device=dev), torch.empty(M, D, dtype=bf, device=dev)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
dres = torch.randn(M, D, device=dev)
ds = torch.empty(M, D, device=dev)
dbr = torch.empty(M, D, dtype=bf, device=dev)
n_part = 256
part = torch.empty(3, n_part, D, device=dev)


def mk():
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.BF16, M, D
    a.x, a.y = x.data_ptr(), y.data_ptr()
    a.n_masks, a.p_drop, a.seed1, a.seed2 = 2, 0.3, 11, 12
    a.gamma, a.beta, a.eps = gamma.data_ptr(), beta.data_ptr(), 1e-5
    a.s_out, a.out, a.mean, a.rstd = s.data_ptr(), out.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    a.s_in, a.dout, a.ds, a.dbranch = s.data_ptr(), dres.data_ptr(), ds.data_ptr(), dbr.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part, a.dbranch_part = (part[0].data_ptr(), part[1].data_ptr(), n_part,
                                                              part[2].data_ptr())
    return a


a = mk()
tf = t(lambda: K.ln_fwd(a))
tb = t(lambda: K.ln_bwd(a))
fb = M * D * (2 + 2 + 2 + 2)
bb = M * D * (2 + 4 + 4 + 2)
print("ln fwd %6.1f us (%4.2f TB/s)   ln bwd %6.1f us (%4.2f TB/s)" % (tf * 1e6, fb / tf / 1e12, tb * 1e6, bb / tb / 1e12))
