"""Fused clip + Adam over a 228M-parameter arena (f32 p/g/m/v + bf16 shadow):
time of nstl_sumsq + nstl_adam_step and the HBM rate (30 B/param).
NSTL_LIB_PATH=<other .so> compares builds."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

n = 235_380_736
dev = "cuda:0"
p, g = torch.randn(n, device=dev), torch.randn(n, device=dev) * 1e-3
m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
low = torch.empty(n, dtype=torch.bfloat16, device=dev)
part = torch.empty(1024, device=dev)
norm = torch.empty(1, device=dev)
a = K.AdamArgs()
a.p, a.g, a.m, a.v, a.p_lowp, a.lowp_dtype, a.n = (p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                                    low.data_ptr(), K.BF16, n)
a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.step = 1e-4, 0.9, 0.999, 1e-8, 1e-5, 1
a.sumsq_partial, a.n_partial, a.max_norm, a.norm_out = part.data_ptr(), 1024, 2.0, norm.data_ptr()
ts = {"sumsq": [], "adam": []}
for it in range(25):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    K.sumsq(g, n, part, 1024)
    e[1].record()
    K.adam_step(a)
    e[2].record()
    torch.cuda.synchronize()
    if it >= 5:
        ts["sumsq"].append(e[0].elapsed_time(e[1]))
        ts["adam"].append(e[1].elapsed_time(e[2]))
med = {k: sorted(x)[len(x) // 2] for k, x in ts.items()}
print("sumsq %.1f us (%.2f TB/s)   adam %.1f us (%.2f TB/s)" % (
    med["sumsq"] * 1e3, 4 * n / med["sumsq"] / 1e9, med["adam"] * 1e3, 30 * n / med["adam"] / 1e9))
