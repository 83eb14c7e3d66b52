"""Library reference point: torch.matmul (hipBLASLt) on the 228M step's GEMM shapes,
bf16 in / bf16 out, median of 20.  Context for tools/bench_gemm*.py only."""
import torch

M, D, F = 16384, 1024, 4096
dev = "cuda:0"


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


for name, m, n, k in (("fwd out", M, D, D), ("fwd ffn2", M, D, F), ("fwd ffn1", M, F, D), ("fwd qkv", M, 3 * D, D),
                      ("dX ffn1", M, D, F), ("dX qkv", M, D, 3 * D), ("dX ffn2", M, F, D),
                      ("dW ffn1", F, D, M), ("dW out", D, D, M), ("big 8192^3", 8192, 8192, 8192)):
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
    bt = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    s1 = t(lambda: torch.matmul(a, b))
    s2 = t(lambda: torch.nn.functional.linear(a, bt))
    print("%-12s %5dx%5dx%5d  NN %7.1f TF/s %8.1f us   NT %7.1f TF/s %8.1f us" % (
        name, m, n, k, 2 * m * n * k / s1 / 1e12, s1 * 1e6, 2 * m * n * k / s2 / 1e12, s2 * 1e6))
