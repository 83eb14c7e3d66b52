"""GEMM time against the persistent grid size: the step's shapes (M = 16,384
tokens) on 256 workgroups, on fewer (NSTL_PERSIST_CUS caps the grid; read per
call) with the stream-K tail (NSTL_GEMM4_SK=1) or whole-tile rounds
(NSTL_GEMM4_SK=0), and on a CU-masked stream ceding 8 CUs (one per XCD).
  python tools/bench_sk.py [cus ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402

dev = "cuda:0"
bf = torch.bfloat16
M = 16384


def masked_stream(k):
    fn = ctypes.CDLL(K.LIB_PATH).hipExtStreamCreateWithCUMask
    fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    n = torch.cuda.get_device_properties(0).multi_processor_count
    mask = (ctypes.c_uint32 * ((n + 31) // 32))()
    for c in range(k, n):
        mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    assert fn(ctypes.byref(st), (n + 31) // 32, mask) == 0
    return torch.cuda.ExternalStream(st.value, device=dev)


def t(fn, stream, reps=20):
    with torch.cuda.stream(stream):
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
    cases.append((name, lambda X=X, W=W, C=C, n=n, k=k: K.gemm(X, W, C, M, n, k)))
dY = torch.randn(M, 4096, device=dev).to(bf)
Xa = torch.randn(M, 4096, device=dev).to(bf)
G = torch.empty(4096, 4096, device=dev)
cases.append(("dW 4096^2", lambda: K.gemm(dY, Xa, G, 4096, 4096, M, a_kmajor=False, b_kmajor=False)))
main = torch.cuda.current_stream()
m8 = masked_stream(8)
arms = [("256", main, {}), ("256 SK inst", main, {"NSTL_GEMM4_SK": "2"}), ("248 SK", main, {"NSTL_PERSIST_CUS": "248", "NSTL_GEMM4_SK": "1"}),
        ("248 whole", main, {"NSTL_PERSIST_CUS": "248", "NSTL_GEMM4_SK": "0"}),
        ("mask8 SK", m8, {"NSTL_GEMM4_SK": "1"}), ("mask8 whole", m8, {"NSTL_GEMM4_SK": "0"}),
        ("mask8 G240", m8, {"NSTL_PERSIST_CUS": "240"}), ("mask8 G224", m8, {"NSTL_PERSIST_CUS": "224"}),
        ("mask8 G256", m8, {"NSTL_PERSIST_CUS": "256"})]
print("stream_cus: main %d, mask8 %d" % (K.stream_cus(main.cuda_stream), K.stream_cus(m8.cuda_stream)))
print("%-10s" % "" + "".join("%16s" % a[0] for a in arms))
for name, fn in cases:
    row = []
    for _, st, env in arms:
        for kk in ("NSTL_PERSIST_CUS", "NSTL_GEMM4_SK"):
            os.environ.pop(kk, None)
        os.environ.update(env)
        row.append(t(fn, st))
    for kk in ("NSTL_PERSIST_CUS", "NSTL_GEMM4_SK"):
        os.environ.pop(kk, None)
    print("%-10s" % name + "".join("%9.1f %+5.0f%%" % (x, 100 * (x / row[0] - 1)) for x in row))
