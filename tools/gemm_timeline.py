"""Per-workgroup timeline of the 256x256 ring GEMM from the diagnostic stamp build
(make -C neurosync_trainer_lite_amd/csrc stamps -> libnstl_hip_stamps.so).

Wave 0 of each workgroup stamps the global 100 MHz clock at tile entry, after
the prologue, after the K loop and after its epilogue stores retired.  Tiles are
grouped per CU in entry order ("round" r = the r-th tile a CU ran); for each
round the medians of entry offset, prologue, K loop, epilogue and the gap since
the same CU's previous tile are printed, in microseconds.  Read the SHARES: the
stamps' own waits make the build slower than the product.

    NSTL_LIB_PATH=neurosync_trainer_lite_amd/libnstl_hip_stamps.so python tools/gemm_timeline.py
"""
import ctypes
import os
import statistics as stt
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402
from neurosync_trainer_lite_amd.engine import rotation_tables  # noqa: E402

M, D, F, T = 16384, 1024, 4096, 128
dev = "cuda:0"
bf = torch.bfloat16
W = 8


def r(*s, dtype=bf):
    return (torch.randn(*s, device=dev) * 0.1).to(dtype)


def read_stamps(n):
    buf = (ctypes.c_ulonglong * (n * W))()
    K.check(K.lib().nstl_debug_gemm_stamps(buf, n * W), "stamps")
    return [list(buf[i * W:(i + 1) * W]) for i in range(n)]


def med(xs):
    return stt.median(xs) if xs else float("nan")


def timeline(name, fn, nblocks, flops):
    for _ in range(30):  # clocks settle
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K.check(K.lib().nstl_debug_gemm_stamps_clear(), "clear")
    torch.cuda.synchronize()
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    ev_us = a.elapsed_time(b) * 1e3
    st = [s for s in read_stamps(nblocks) if s[0] != 0]
    t0 = min(s[0] for s in st)
    tend = max(s[3] for s in st)
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    per_cu = {}
    for s in st:
        per_cu.setdefault((s[5] & 0xF, (s[4] >> 8) & 0xFF), []).append(s)
    rounds = {}
    for lst in per_cu.values():
        lst.sort(key=lambda s: s[0])
        prev = None
        for i, s in enumerate(lst):
            rounds.setdefault(i, []).append((s, prev))
            prev = s
    print("%s: %d tiles on %d CUs, event %.1f us, stamped span %.1f us (%.0f TF/s by event)"
          % (name, len(st), len(per_cu), ev_us, us(tend - t0), flops / ev_us / 1e6))
    print("  round  tiles   entry[min/med/max]      prologue  kloop   epi    gap_since_prev_end")
    for i in sorted(rounds):
        rr = rounds[i]
        ent = [us(s[0] - t0) for s, _ in rr]
        pro = [us(s[1] - s[0]) for s, _ in rr]
        kl = [us(s[2] - s[1]) for s, _ in rr]
        ep = [us(s[3] - s[2]) for s, _ in rr]
        gap = [us(s[0] - p[3]) for s, p in rr if p is not None]
        print("  %5d %6d  %6.1f/%6.1f/%6.1f   %7.2f %7.2f %6.2f   %6.2f"
              % (i, len(rr), min(ent), med(ent), max(ent), med(pro), med(kl), med(ep), med(gap)))
    ends = sorted(us(s[3] - t0) for s in st)
    print("  tile end times: p10 %.1f  p50 %.1f  p90 %.1f  max %.1f" % (
        ends[len(ends) // 10], ends[len(ends) // 2], ends[9 * len(ends) // 10], ends[-1]))


def main():
    cs, sn = rotation_tables(T, 64, dev)
    x, x4 = r(M, D), r(M, F)
    for name, n, k, kw in (
            ("fwd out  BIAS", D, D, dict(epilogue=K.EPI_BIAS)),
            ("fwd ffn2 BIAS", D, F, dict(epilogue=K.EPI_BIAS)),
            ("fwd ffn1 RELU_DROP", F, D, dict(epilogue=K.EPI_BIAS_RELU_DROP, p_drop=0.3, seed=5)),
            ("fwd qkv  ROPE", 3 * D, D, dict(epilogue=K.EPI_BIAS_ROPE, rope=(cs, sn, T, 64), rope_cols=2 * D))):
        X = x if k == D else x4
        Wt, b = r(n, k), torch.zeros(n, device=dev)
        Y = torch.empty(M, n, dtype=bf, device=dev)
        timeline(name, lambda: K.gemm(X, Wt, Y, M, n, k, bias=b, **kw), (M // 256) * (n // 256), 2 * M * n * k)
    # dX: dY [M][N_out] K-major, W [N_out][N_in] read MN-major
    for name, n, k in (("dX  ffn2 (N=4096,K=1024)", F, D), ("dX  qkv (N=1024,K=3072)", D, 3 * D)):
        dy, Wt = r(M, k), r(k, n)
        Y = torch.empty(M, n, dtype=bf, device=dev)
        timeline(name, lambda: K.gemm(dy, Wt, Y, M, n, k, a_kmajor=True, b_kmajor=False), (M // 256) * (n // 256),
                 2 * M * n * k)
    # dW: dY^T X, both read MN-major, f32 out
    for name, n, k in (("dW  ffn1 (4096x1024, K=16384)", F, D),):
        dy, xx = r(M, n), r(M, k)
        G = torch.empty(n, k, dtype=torch.float32, device=dev)
        timeline(name, lambda: K.gemm(dy, xx, G, n, k, M, a_kmajor=False, b_kmajor=False), (n // 256) * (k // 256),
                 2 * M * n * k)


if __name__ == "__main__":
    main()
