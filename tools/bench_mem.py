"""The step's memory-bound kernels at the 228M shape (16,384 rows x D = 1024,
bf16, dropout 0.3), as the engine calls them, against a torch copy of the same
byte count: LayerNorm forward (x + dropout(y) -> s, out, stats), LayerNorm
backward (s, f32 residual gradient in place, bf16 hand-off, two masks, dbranch
and its column-sum partials) and the Adam update of 235 M parameters.
  python tools/bench_mem.py [n_part ...]     (LayerNorm backward partial blocks)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

R, D = 16384, 1024
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


def line(name, s, nbytes):
    print("%-34s %8.1f us  %6.2f TB/s  (%.0f MB)" % (name, s * 1e6, nbytes / s * 1e-12, nbytes / 1e6), flush=True)


x = torch.randn(R, D, device=dev).to(bf)
y = torch.randn(R, D, device=dev).to(bf)
s_out = torch.empty(R, D, dtype=bf, device=dev)
out = torch.empty(R, D, dtype=bf, device=dev)
mean = torch.empty(R, device=dev)
rstd = torch.empty(R, device=dev)
gamma = torch.ones(D, device=dev)
beta = torch.zeros(D, device=dev)


def ln_fwd(n_masks=1):
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.dtype_code(bf), R, D
    a.x, a.y = x.data_ptr(), y.data_ptr()
    a.n_masks, a.p_drop, a.seed1, a.seed2 = n_masks, 0.3 if n_masks else 0.0, 11, 12
    a.gamma, a.beta, a.eps = gamma.data_ptr(), beta.data_ptr(), 1e-5
    a.s_out, a.out, a.mean, a.rstd = s_out.data_ptr(), out.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    K.ln_fwd(a)


dres = torch.randn(R, D, device=dev) * 1e-3
dadd = (torch.randn(R, D, device=dev) * 1e-3).to(bf)
dbranch = torch.empty(R, D, dtype=bf, device=dev)
ln_fwd()
torch.cuda.synchronize()


def ln_bwd(n_part, part, n_masks=2):
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.dtype_code(bf), R, D
    a.n_masks, a.p_drop, a.seed1, a.seed2 = n_masks, 0.3 if n_masks else 0.0, 11, 12
    a.gamma, a.beta, a.eps = gamma.data_ptr(), beta.data_ptr(), 1e-5
    a.mean, a.rstd = mean.data_ptr(), rstd.data_ptr()
    a.s_in, a.dout, a.ds, a.dbranch = s_out.data_ptr(), dres.data_ptr(), dres.data_ptr(), dbranch.data_ptr()
    a.dout2 = dadd.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part = part[0].data_ptr(), part[1].data_ptr(), n_part
    a.dbranch_part = part[2].data_ptr()
    K.ln_bwd(a)


parts = [int(v) for v in sys.argv[1:]] or [int(os.environ.get("NSTL_LN_PARTS", "256"))]
for nm in (1, 2, 0):
    line("LayerNorm fwd (%d masks)" % nm, t(lambda: ln_fwd(nm)), R * D * 2 * 4)
for n_part in parts:
    part = torch.empty(3, n_part, D, device=dev)
    for nm in (2, 1, 0):
        line("LayerNorm bwd (%d masks) n_part %d" % (nm, n_part), t(lambda: ln_bwd(n_part, part, nm)),
             R * D * (2 + 4 + 2 + 4 + 2))
if os.environ.get("NSTL_BENCH_LN_ONLY"):
    sys.exit(0)

N = 235_000_000
p = torch.randn(N, device=dev) * 0.02
g = torch.randn(N, device=dev) * 1e-3
m = torch.zeros(N, device=dev)
v = torch.zeros(N, device=dev)
lowp = torch.empty(N, dtype=bf, device=dev)
coef = torch.ones(1, device=dev)


def adam():
    a = K.AdamArgs()
    a.p, a.g, a.m, a.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
    a.p_lowp, a.lowp_dtype, a.n = lowp.data_ptr(), K.dtype_code(bf), N
    a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.step = 1e-4, 0.9, 0.999, 1e-8, 1e-5, 3
    a.coef = coef.data_ptr()
    K.adam_step(a)


line("Adam (235 M params)", t(adam, reps=10), N * 30)
src = torch.empty(R * D * 4 // 4, device=dev)
dst = torch.empty_like(src)
line("torch copy 64 MB f32", t(lambda: dst.copy_(src)), src.numel() * 8)
big = torch.empty(N, device=dev)
line("torch copy 940 MB f32", t(lambda: big.copy_(p), reps=10), N * 8)
