"""Per-kernel parity of the production kernels at the 228M step's shapes
(B=128, T=128, D=1024, H=16: M = 16,384 rows), held to float64 of the same
bf16-rounded operands (reference: utils/model.py:110-158, the Linear layers and
MultiHeadAttention the step runs).

GEMMs: f32 outputs, every element within 1e-5 of sum_k |a_ik b_kj| (the
magnitude the f32 accumulation rounds against), on the kernels the bench runs:
the 4-wave persistent kernel (forward TT, dX TN, the grouped weight gradients
NN with K = 16,384 tokens) and the ring kernel (the f32 beta-1 dX that
accumulates the residual gradient).

Attention: the persistent forward and the fused backward over all 2,048 (b, h)
blocks at p = 0 against a float64 restatement (softmax(QK^T/8) V; dQ, dK with
the RoPE rotation transposed, dV).  Their outputs are bf16, so the bound is the
bf16 output rounding plus the kernels' bf16 P / dS operands: the RMS error
relative to the RMS of the reference and the max error relative to the max.
Each test prints its worst errors.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.engine import rotation_tables

DEV = "cuda:0"
bf = torch.bfloat16
M, D, F, H, T, B = 16384, 1024, 4096, 16, 128, 128


def rnd(*shape, dtype=bf, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV, dtype=torch.float32) * scale).to(dtype)


def bound_check(got, A, Bm, ref, tag, eps=1e-5):
    """|got - ref| <= eps * (|A| @ |B|) elementwise (A [m, k], Bm [k, n], float64)."""
    mag = A.abs() @ Bm.abs()
    err = (got.double() - ref).abs()
    ratio = (err / mag.clamp_min(1e-300)).max().item()
    print("%s: max |err| / sum|a b| = %.3e (bound %.0e), max |err| = %.3e" % (tag, ratio, eps, err.max().item()))
    assert ratio <= eps, (tag, ratio)


@pytest.mark.parametrize("case", ["fwd_ffn1", "fwd_qkv", "dx_ffn2", "dx_out"])
def test_gemm4_production_f32_vs_f64(case):
    n, k, bkm = {"fwd_ffn1": (F, D, True), "fwd_qkv": (3 * D, D, True), "dx_ffn2": (D, F, False),
                 "dx_out": (D, D, False)}[case]
    A = rnd(M, k, seed=1)
    W = rnd(n, k, scale=0.03, seed=2) if bkm else rnd(k, n, scale=0.03, seed=2)
    C = torch.empty(M, n, dtype=torch.float32, device=DEV)
    K.kernel_counts_reset()
    K.gemm(A, W, C, M, n, k, a_kmajor=True, b_kmajor=bkm)
    torch.cuda.synchronize()
    assert K.kernel_counts()["gemm4"] == 1
    A64 = A.double()
    B64 = W.double().T if bkm else W.double()
    bound_check(C, A64, B64, A64 @ B64, "gemm4 " + case)


def test_ring_f32_beta1_dx_vs_f64():
    """The residual-gradient accumulation dX += dY W (f32, beta 1) on the ring kernel."""
    n, k = D, F
    dY, W = rnd(M, k, seed=3), rnd(k, n, scale=0.03, seed=4)
    C0 = rnd(M, n, dtype=torch.float32, seed=5)
    C = C0.clone()
    K.kernel_counts_reset()
    K.gemm(dY, W, C, M, n, k, a_kmajor=True, b_kmajor=False, beta=1.0)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["gemm_ring"] == 1 and c["gemm4"] == 0, c
    A64, B64 = dY.double(), W.double()
    ref = C0.double() + A64 @ B64
    # the f32 addition of C0 rounds against |C0| as well
    mag = A64.abs() @ B64.abs() + C0.double().abs()
    ratio = ((C.double() - ref).abs() / mag).max().item()
    print("ring f32 beta-1 dX: max |err| / (sum|a b| + |c0|) = %.3e" % ratio)
    assert ratio <= 1e-5


def test_grouped_dw_decoder_layer_vs_f64():
    """One decoder layer's weight gradients as the step launches them (7 problems,
    K = 16,384 tokens, f32 out, beta 0, sum-of-squares partials)."""
    shapes = [(D, F), (F, D), (D, D), (D, D), (2 * D, D), (D, D), (3 * D, D)]
    probs, outs, ins = [], [], []
    nt = sum((n // 256) * (k // 256) for n, k in shapes)
    sq = torch.zeros(nt * 8, dtype=torch.float32, device=DEV)
    used = 0
    for i, (n, k) in enumerate(shapes):
        dY, X = rnd(M, n, scale=0.1, seed=10 + i), rnd(M, k, seed=20 + i)
        G = torch.empty(n, k, dtype=torch.float32, device=DEV)
        t = (n // 256) * (k // 256) * 8
        probs.append((dY, X, G, n, k, M, dict(a_kmajor=False, b_kmajor=False, sq_part=sq[used:used + t])))
        used += t
        outs.append(G)
        ins.append((dY, X))
    K.kernel_counts_reset()
    K.gemm_grouped(probs)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["gemm4"] == 1 and c["gemm4_tiles"] == nt, c
    tot = 0.0
    for (n, k), G, (dY, X) in zip(shapes, outs, ins):
        A64, B64 = dY.double().T, X.double()
        bound_check(G, A64, B64, A64 @ B64, "grouped dW %dx%d" % (n, k))
        tot += float((G.double() ** 2).sum())
    rs = abs(float(sq.double().sum()) - tot) / tot
    print("grouped dW sum-of-squares partials vs the stored gradients: rel %.2e" % rs)
    assert rs < 1e-6


def _rms_max(got, ref):
    got, ref = got.double(), ref.double()
    e = got - ref
    return (e.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()).item(), (e.abs().max() / ref.abs().max()).item()


def test_attention_production_fwd_bwd_vs_f64():
    """All 2,048 (b, h) blocks of the 228M step's self-attention, p = 0."""
    dh = D // H
    qkv = rnd(M, 3 * D, scale=0.5, seed=30)
    o = torch.empty(M, D, dtype=bf, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a = K.attn_args(K.dtype_code(bf), B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                    qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), 0.0, 0, dh=dh)
    K.kernel_counts_reset()
    K.attn_fwd(a)
    do = rnd(M, D, seed=31)
    dqkv = torch.zeros(M, 3 * D, dtype=bf, device=DEV)
    cs, sn = rotation_tables(T, dh, DEV)
    a.dout, a.dout_ld = do.data_ptr(), D
    a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                    dqkv[:, 2 * D:].data_ptr(), 3 * D)
    a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
    dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a.dsum = dsum.data_ptr()
    K.attn_bwd(a)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["attn_fwd"] == 1 and c["attn_bwd_fused"] == 1 and c["attn_bwd_split"] == 0, c

    def heads(x):
        return x.double().view(B, T, H, dh).transpose(1, 2)

    q = heads(qkv[:, :D]).requires_grad_(True)
    k = heads(qkv[:, D:2 * D]).requires_grad_(True)
    v = heads(qkv[:, 2 * D:]).requires_grad_(True)
    s = (q @ k.transpose(-1, -2)) * dh ** -0.5
    rl = torch.logsumexp(s, -1)
    ro = torch.softmax(s, -1) @ v
    r_o, m_o = _rms_max(o, ro.transpose(1, 2).reshape(M, D))
    lse_err = ((lse.double() - rl.reshape(-1)).abs().max()).item()
    ro.backward(heads(do))
    c64, s64 = cs.double(), sn.double()

    def rope_back(g):
        e, od = g[..., 0::2], g[..., 1::2]
        r = torch.empty_like(g)
        r[..., 0::2] = e * c64 + od * s64
        r[..., 1::2] = -e * s64 + od * c64
        return r.transpose(1, 2).reshape(M, D)

    r_dq, m_dq = _rms_max(dqkv[:, :D], rope_back(q.grad))
    r_dk, m_dk = _rms_max(dqkv[:, D:2 * D], rope_back(k.grad))
    r_dv, m_dv = _rms_max(dqkv[:, 2 * D:], v.grad.transpose(1, 2).reshape(M, D))
    print("attention fwd: O rms %.2e max %.2e, lse max abs %.2e" % (r_o, m_o, lse_err))
    print("attention bwd (fused, 2048 blocks): dQ rms %.2e max %.2e | dK rms %.2e max %.2e | dV rms %.2e max %.2e"
          % (r_dq, m_dq, r_dk, m_dk, r_dv, m_dv))
    # bf16 outputs: rounding alone is ~1.1e-3 rms relative; P and dS enter the
    # products as bf16 as well
    assert r_o < 4e-3 and m_o < 1e-2, (r_o, m_o)
    assert lse_err < 1e-4, lse_err
    for r, m in ((r_dq, m_dq), (r_dk, m_dk), (r_dv, m_dv)):
        assert r < 8e-3 and m < 2e-2, (r, m)
