"""GEMM time against the persistent grid size (NSTL_PERSIST_CUS caps it; read
per call): whole-tile rounds at 256 workgroups, the stream-K tail below.
The step's shapes (M = 16,384 tokens).  python tools/bench_sk.py [cus ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

dev = "cuda:0"
bf = torch.bfloat16
M = 16384


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
    return ts[len(ts) // 2] * 1e3


cases = []
for name, n, k in [("fwd ffn2", 1024, 4096), ("fwd ffn1", 4096, 1024), ("fwd qkv", 3072, 1024), ("fwd out", 1024, 1024)]:
    X = torch.randn(M, k, device=dev).to(bf)
    W = (torch.randn(n, k, device=dev) * 0.05).to(bf)
    C = torch.empty(M, n, dtype=bf, device=dev)
    cases.append((name, 2.0 * M * n * k, lambda X=X, W=W, C=C, n=n, k=k: K.gemm(X, W, C, M, n, k)))
dY = torch.randn(M, 4096, device=dev).to(bf)
Xa = torch.randn(M, 4096, device=dev).to(bf)
G = torch.empty(4096, 4096, device=dev)
cases.append(("dW 4096^2", 2.0 * M * 4096 * 4096,
              lambda: K.gemm(dY, Xa, G, 4096, 4096, M, a_kmajor=False, b_kmajor=False)))
cus = [int(x) for x in sys.argv[1:]] or [256, 248, 240, 224]
print("%-10s" % "" + "".join("%14s" % ("%d WGs" % c) for c in cus))
for name, fl, fn in cases:
    row = []
    for c in cus:
        os.environ["NSTL_PERSIST_CUS"] = str(c)
        row.append(t(fn))
    os.environ.pop("NSTL_PERSIST_CUS", None)
    print("%-10s" % name + "".join("%8.1f us %+4.0f%%" % (x, 100 * (x / row[0] - 1)) for x in row))
