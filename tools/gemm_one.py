"""Run one GEMM shape repeatedly (for rocprofv3 --pmc passes).
  python tools/gemm_one.py {fwd|dx|dw} N K [reps] [split]   (M = 16384 tokens)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

kind, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
split = int(sys.argv[5]) if len(sys.argv) > 5 else 1
M, dev, bf = 16384, "cuda:0", torch.bfloat16
X = (torch.randn(M, k, device=dev) * 0.1).to(bf)
W = (torch.randn(n, k, device=dev) * 0.1).to(bf)
b = torch.zeros(n, device=dev)
dY = (torch.randn(M, n, device=dev) * 0.1).to(bf)
Y = torch.empty(M, n, dtype=bf, device=dev)
dX = torch.zeros(M, k, dtype=torch.float32, device=dev)
G = torch.empty(n, k, dtype=torch.float32, device=dev)
ws = torch.empty(max(1, split * n * k), dtype=torch.float32, device=dev)
for _ in range(reps):
    if kind == "fwd":
        K.gemm(X, W, Y, M, n, k, epilogue=K.EPI_BIAS, bias=b)
    elif kind == "dx":
        K.gemm(dY, W, dX, M, k, n, a_kmajor=True, b_kmajor=False, beta=1.0)
    else:
        K.gemm(dY, X, G, n, k, M, a_kmajor=False, b_kmajor=False, split_k=split, workspace=ws)
torch.cuda.synchronize()
