"""Where does the persistent GEMM differ from its one-shot halves?  Prints, per
256x256 tile that differs, its coordinates and max diff (bf16 forward, bias)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

dev = "cuda:0"
cus = torch.cuda.get_device_properties(0).multi_processor_count
N, Kd = 2048, 1024
M = 2 * cus // (N // 256) * 256
g = torch.Generator().manual_seed(1)
X = torch.randn(M, Kd, generator=g).to(torch.bfloat16).to(dev)
W = (torch.randn(N, Kd, generator=g) * 0.05).to(torch.bfloat16).to(dev)
b = torch.randn(N, generator=g).to(dev)
full = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
K.gemm(X, W, full, M, N, Kd, epilogue=K.EPI_BIAS, bias=b)
halves = []
for i0 in (0, M // 2):
    h = torch.empty(M // 2, N, dtype=torch.bfloat16, device=dev)
    K.gemm(X[i0:], W, h, M // 2, N, Kd, epilogue=K.EPI_BIAS, bias=b)
    halves.append(h)
ref = torch.cat(halves)
ex = (X.double() @ W.double().T) + b.double()
torch.cuda.synchronize()
d = (full.float() - ref.float()).abs()
print("M", M, "max diff", d.max().item(), "frac differ", (d > 0).double().mean().item())
bad = 0
for tm in range(M // 256):
    for tn in range(N // 256):
        t = d[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256]
        if t.max().item() > 0:
            e_full = (full[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256].double() - ex[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256]).abs().max().item()
            e_ref = (ref[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256].double() - ex[tm * 256:(tm + 1) * 256, tn * 256:(tn + 1) * 256]).abs().max().item()
            nz = (t > 0).nonzero()
            if bad < 40:
                print("tile", tm, tn, "max", t.max().item(), "n", len(nz), "rows", nz[:, 0].min().item(), nz[:, 0].max().item(),
                      "cols", nz[:, 1].min().item(), nz[:, 1].max().item(), "err vs f64: full %.3e one-shot %.3e" % (e_full, e_ref))
            bad += 1
print("tiles differing", bad, "of", (M // 256) * (N // 256))
rel = d / torch.maximum(full.float().abs(), ref.float().abs()).clamp_min(1e-30)
top = torch.topk(rel.flatten(), 8)
for v, ix in zip(top.values.tolist(), top.indices.tolist()):
    i, j = divmod(ix, N)
    print("rel %.3e at (%d,%d): persistent %.6f one-shot %.6f f64 %.6f" % (v, i, j, full[i, j].item(), ref[i, j].item(), ex[i, j].item()))
