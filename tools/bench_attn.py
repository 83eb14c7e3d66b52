"""Attention kernels at the 228M step's shape (B=128, T=128, H=16, dh=64, bf16,
q|k|v as slices of one [M, 3D] buffer): fwd and bwd time with dropout 0.3 vs 0
(the difference is the counter-hash mask cost).  python tools/bench_attn.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neurosync_trainer_lite_amd import _hip as K  # noqa: E402
from neurosync_trainer_lite_amd.engine import rotation_tables  # noqa: E402

T = int(os.environ.get("NSTL_BENCH_T", "128"))     # 256: BASELINE C5's long clips (B halved)
B, H, DH = 128 * 128 // T, 16, 64
D, M = H * DH, B * T
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


qkv = (torch.randn(M, 3 * D, device=dev) * 0.5).to(bf)
o = torch.empty(M, D, dtype=bf, device=dev)
lse = torch.empty(B * H * T, device=dev)
do = (torch.randn(M, D, device=dev) * 0.1).to(bf)
dqkv = torch.empty(M, 3 * D, dtype=bf, device=dev)
dsum = torch.empty(B * H * T, device=dev)
cs, sn = rotation_tables(T, DH, dev)
extra = {}
mask = None
if os.environ.get("NSTL_ATTN_MASK", "1") == "1":   # stored keep bits (0: re-hash in backward)
    mask = torch.empty(B * H * T * T // 8, dtype=torch.uint8, device=dev)
for p in [float(x) for x in os.environ.get("NSTL_BENCH_P", "0.3,0.0").split(",")]:
    def args():
        a = K.attn_args(K.BF16, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                        qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 77)
        a.dout, a.dout_ld = do.data_ptr(), D
        a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                        dqkv[:, 2 * D:].data_ptr(), 3 * D)
        rope = 0 if os.environ.get("NSTL_BENCH_NOROPE") == "1" else 1   # RoPE^T off: its cost in the epilogue
        a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), rope, rope
        a.dsum = dsum.data_ptr()
        if mask is not None:
            a.mask_bits = mask.data_ptr()
        if os.environ.get("NSTL_BENCH_BIAS", "1") == "1":   # fused q|k|v bias column sums, as the step
            rows = K.attn_bias_rows(a)
            if rows:
                extra["part"] = torch.empty(rows, 3 * D, device=dev)
                a.dbias_part = extra["part"].data_ptr()
        return a
    a = args()
    tf = t(lambda: K.attn_fwd(a))
    tb = t(lambda: K.attn_bwd(a))
    fl_f, fl_b = 4 * B * H * T * T * DH, 10 * B * H * T * T * DH
    print("p=%.1f  fwd %7.1f us (%5.1f TF/s)   bwd %7.1f us (%5.1f TF/s)" % (
        p, tf * 1e6, fl_f / tf / 1e12, tb * 1e6, fl_b / tb / 1e12))
