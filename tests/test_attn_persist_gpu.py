"""The persistent fused attention backward (csrc/attention.hip
attn_bwd_persist_kernel: 2 workgroups per CU walk the heads, the next head's
Q / dO / K images and LSE loaded by LDS-DMA under the current head's epilogue)
against the one-workgroup-per-head fused kernel (NSTL_ATTN_BWD=oneshot): the
same per-head arithmetic in the same order, so dQ, dK, dV and the bias partials
agree bit for bit.  B*H = 6 (fewer heads than workgroups), 1040 (uneven heads
per workgroup) and 2048 (the 228M step); stored keep bits, re-hashed dropout,
no dropout; with and without RoPE^T.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.engine import rotation_tables

DEV = "cuda:0"
bf = torch.bfloat16


def rnd(*shape, dtype=bf, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV, dtype=torch.float32) * scale).to(dtype)


@pytest.mark.parametrize("B,H,p,mode,rope", [(2, 3, 0.3, "stored", True), (65, 16, 0.3, "stored", True),
                                              (128, 16, 0.3, "stored", True), (65, 16, 0.3, "rehash", True),
                                              (65, 16, 0.0, "none", True), (65, 16, 0.3, "stored", False)])
def test_persistent_bwd_matches_oneshot(monkeypatch, B, H, p, mode, rope):
    T, dh = 128, 64
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, scale=0.5, seed=1)
    do = rnd(M, D, seed=2)
    cs, sn = rotation_tables(T, dh, DEV)
    o = torch.empty(M, D, dtype=bf, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    mask = torch.zeros(B * H * T * T // 64, dtype=torch.int64, device=DEV)

    def args():
        a = K.attn_args(K.BF16, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                        qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 321, dh=dh)
        if mode == "stored":
            a.mask_bits = mask.data_ptr()
        return a

    K.attn_fwd(args())
    outs = []
    for arm in ("oneshot", "persist"):
        monkeypatch.setenv("NSTL_ATTN_BWD", arm)
        a = args()
        dqkv = torch.full((M, 3 * D), float("nan"), dtype=bf, device=DEV)
        a.dout, a.dout_ld = do.data_ptr(), D
        a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                        dqkv[:, 2 * D:].data_ptr(), 3 * D)
        if rope:
            a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
        dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
        a.dsum = dsum.data_ptr()
        rows = K.attn_bias_rows(a)
        part = torch.full((rows, 3 * D), float("nan"), device=DEV)
        a.dbias_part = part.data_ptr()
        K.kernel_counts_reset()
        K.attn_bwd(a)
        torch.cuda.synchronize()
        assert K.kernel_counts()["attn_bwd_fused"] == 1
        outs.append((dqkv, part))
    monkeypatch.delenv("NSTL_ATTN_BWD")
    assert not torch.isnan(outs[1][0].float()).any() and not torch.isnan(outs[1][1]).any()
    assert torch.equal(outs[0][0], outs[1][0]), "dq|dk|dv"
    assert torch.equal(outs[0][1], outs[1][1]), "bias partials"
