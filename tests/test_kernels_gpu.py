"""Per-kernel parity on the MI355X: HIP kernel vs a float64 torch reference.

Tolerances: f32 kernels use the f32-input MFMA (an exact f32 fma chain), so
they sit at ~1e-6 relative to sum|a*b|; bf16 kernels take bf16-rounded inputs
(the reference uses the same rounded inputs) and differ by accumulation order
plus output rounding (2^-8 relative when the output is bf16).
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.engine import rotation_tables

DEV = "cuda:0"


def rnd(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).to(dtype).to(DEV)


def f64(t):
    return t.detach().double().cpu()


def check(got, ref, rel, what):
    got, ref = f64(got), f64(ref)
    scale = ref.abs().max().item() + 1e-30
    err = (got - ref).abs().max().item()
    assert err <= rel * scale, "%s: max err %.3e vs scale %.3e (rel %.1e)" % (what, err, scale, rel)


DTS = [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)]


@pytest.mark.parametrize("dt,tol", DTS)
@pytest.mark.parametrize("M,N,Kd", [(300, 200, 136), (128, 128, 64), (17, 61, 1024), (512, 384, 256)])
def test_gemm_forward_bias(dt, tol, M, N, Kd):
    A, W = rnd(M, Kd, dtype=dt, seed=1), rnd(N, Kd, dtype=dt, scale=0.05, seed=2)
    bias = rnd(N, seed=3)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K.gemm(A, W, C, M, N, Kd, epilogue=K.EPI_BIAS, bias=bias)
    torch.cuda.synchronize()
    check(C, f64(A) @ f64(W).T + f64(bias), 1e-5, "gemm NT f32-out")
    C2 = torch.empty(M, N, dtype=dt, device=DEV)
    K.gemm(A, W, C2, M, N, Kd, epilogue=K.EPI_BIAS, bias=bias)
    check(C2, f64(A) @ f64(W).T + f64(bias), 1e-5 if dt == torch.float32 else 8e-3, "gemm NT")


@pytest.mark.parametrize("dt,tol", DTS)
@pytest.mark.parametrize("M,N,Kd", [(256, 192, 320), (100, 61, 1024), (384, 1024, 4096 // 4)])
def test_gemm_dx_layout(dt, tol, M, N, Kd):
    """C[M,Kd] (+)= dY[M,N] W[N,Kd]: A K-major, B read MN-major (transpose read)."""
    dY, W = rnd(M, N, dtype=dt, seed=4), rnd(N, Kd, dtype=dt, seed=5)
    C0 = rnd(M, Kd, seed=6)
    C = C0.clone()
    # reduction dim N need not be a multiple of 8 if the row stride is and padding is zero
    ldy = (N + 7) // 8 * 8
    dYp = torch.zeros(M, ldy, dtype=dt, device=DEV)
    dYp[:, :N] = dY
    K.gemm(dYp, W, C, M, Kd, N, a_kmajor=True, b_kmajor=False, lda=ldy, beta=1.0)
    check(C, f64(C0) + f64(dY) @ f64(W), 1e-5, "gemm dX")


@pytest.mark.parametrize("dt,tol", DTS)
@pytest.mark.parametrize("Mt,N,Kd,split", [(512, 192, 136, 1), (2048, 256, 128, 4), (1000, 61, 256, 3), (4096, 128, 384, 8)])
def test_gemm_dw_layout(dt, tol, Mt, N, Kd, split):
    """C[N,Kd] = beta*C + dY^T X: both operands read MN-major; split-K reduce."""
    ldy = (N + 7) // 8 * 8
    dY = torch.zeros(Mt, ldy, dtype=dt, device=DEV)
    dY[:, :N] = rnd(Mt, N, dtype=dt, seed=7)
    X = rnd(Mt, Kd, dtype=dt, seed=8)
    C0 = rnd(N, Kd, seed=9)
    C = C0.clone()
    ws = torch.empty(max(1, split * N * Kd), dtype=torch.float32, device=DEV)
    K.gemm(dY, X, C, N, Kd, Mt, a_kmajor=False, b_kmajor=False, lda=ldy, beta=0.5, split_k=split, workspace=ws)
    check(C, 0.5 * f64(C0) + f64(dY[:, :N]).T @ f64(X), 1e-5, "gemm dW")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_rope_epilogue(dt):
    B, T, D = 3, 32, 256
    M = B * T
    X, W, b = rnd(M, 128, dtype=dt, seed=10), rnd(3 * D, 128, dtype=dt, scale=0.1, seed=11), rnd(3 * D, seed=12)
    cs, sn = rotation_tables(T, 64, DEV)
    C = torch.empty(M, 3 * D, dtype=torch.float32, device=DEV)
    K.gemm(X, W, C, M, 3 * D, 128, epilogue=K.EPI_BIAS_ROPE, bias=b, rope=(cs, sn, T, 64), rope_cols=2 * D)
    y = f64(X) @ f64(W).T + f64(b)
    ref = y.clone()
    c, s = f64(cs), f64(sn)
    for blk in range(2 * D // 64):
        z = y[:, blk * 64:(blk + 1) * 64].reshape(B, T, 64)
        e, o = z[..., 0::2], z[..., 1::2]
        r = torch.empty_like(z)
        r[..., 0::2] = e * c - o * s
        r[..., 1::2] = e * s + o * c
        ref[:, blk * 64:(blk + 1) * 64] = r.reshape(M, 64)
    check(C, ref, 1e-5, "gemm rope")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_relu_dropout_and_backward(dt):
    M, N, Kd = 256, 512, 128
    X, W, b = rnd(M, Kd, dtype=dt, seed=13), rnd(N, Kd, dtype=dt, scale=0.1, seed=14), rnd(N, seed=15)
    H0 = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K.gemm(X, W, H0, M, N, Kd, epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.0)
    ref = torch.relu(f64(X) @ f64(W).T + f64(b))
    check(H0, ref, 1e-5, "relu p=0")
    H = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K.gemm(X, W, H, M, N, Kd, epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=1234)
    h, r = f64(H), ref
    pos = r > 1e-3
    kept = (h[pos] != 0)
    frac = kept.double().mean().item()
    assert abs(frac - 0.7) < 0.02, frac
    torch.testing.assert_close(h[pos][kept], r[pos][kept] / 0.7, rtol=1e-4, atol=1e-5)
    # deterministic in the seed
    H2 = torch.empty_like(H)
    K.gemm(X, W, H2, M, N, Kd, epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=1234)
    assert torch.equal(H, H2)
    # backward epilogue: dH = (dA W2) * (a > 0) / (1-p)
    a = H.to(dt)
    dA, W2 = rnd(M, 64, dtype=dt, seed=16), rnd(64, N, dtype=dt, seed=17)
    dH = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K.gemm(dA, W2, dH, M, N, 64, a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=a, ld_aux=N,
           p_drop=0.3)
    refd = (f64(dA) @ f64(W2)) * (f64(a) > 0).double() / 0.7
    check(dH, refd, 1e-5, "drelu")


@pytest.mark.parametrize("case", ["fwd_bias", "dx_bf16", "dx_f32_beta1", "fwd_f32"])
def test_gemm4_plain(case):
    """Plain GEMMs on full 256^2 tiles run on the 4-wave persistent kernel
    (csrc/gemm4.h) through nstl_gemm: the launch counter sees them, and the results
    match the f64 product for K-major and MN-major B, bf16 (with bias) and f32
    output.  f32 output with beta != 0 stays on the ring kernel."""
    if os.environ.get("NSTL_GEMM4") == "0":
        pytest.skip("4-wave kernel off")
    dt, M, N, Kd = torch.bfloat16, 4096, 1024 + 256, 1024 + 128
    b = rnd(N, seed=503)
    K.kernel_counts_reset()
    if case in ("fwd_bias", "fwd_f32"):
        X, W = rnd(M, Kd, dtype=dt, seed=501), rnd(N, Kd, dtype=dt, scale=0.05, seed=502)
        C = torch.empty(M, N, dtype=dt if case == "fwd_bias" else torch.float32, device=DEV)
        kw = dict(epilogue=K.EPI_BIAS, bias=b) if case == "fwd_bias" else {}
        K.gemm(X, W, C, M, N, Kd, **kw)
        ref = f64(X) @ f64(W).T + (f64(b) if case == "fwd_bias" else 0)
    else:
        dY, W = rnd(M, Kd, dtype=dt, seed=504), rnd(Kd, N, dtype=dt, scale=0.05, seed=505)
        if case == "dx_bf16":
            C = torch.empty(M, N, dtype=dt, device=DEV)
            K.gemm(dY, W, C, M, N, Kd, a_kmajor=True, b_kmajor=False)
            ref = f64(dY) @ f64(W)
        else:
            C0 = rnd(M, N, seed=506)
            C = C0.clone()
            K.gemm(dY, W, C, M, N, Kd, a_kmajor=True, b_kmajor=False, beta=1.0)
            ref = f64(C0) + f64(dY) @ f64(W)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    if case != "dx_f32_beta1":
        assert c["gemm4"] == 1 and c["gemm4_tiles"] == (M // 256) * (N // 256) and c["gemm_ring"] == 0, c
    else:
        assert c["gemm4"] == 0 and c["gemm_ring"] == 1, c
    check(C, ref, 1e-2 if C.dtype == dt else 1e-4, "gemm4 " + case)


@pytest.mark.parametrize("case", ["k_not_64", "partial_tile", "misaligned_c", "few_tiles"])
def test_gemm_outside_gemm4(case):
    """A GEMM the 4-wave kernel turns away (K not a multiple of 64, a partial 256^2
    tile, a C pointer off 16-byte alignment) runs on the ring / 128 kernels with the
    same result; a small full-tile problem (16 tiles) runs on the 4-wave kernel."""
    dt = torch.bfloat16
    M, N, Kd = {"k_not_64": (4096, 2048, 1000), "partial_tile": (4096 + 128, 2048, 1024),
                "misaligned_c": (4096, 2048, 1024), "few_tiles": (1024, 1024, 1024)}[case]
    X, W = rnd(M, Kd, dtype=dt, seed=511), rnd(N, Kd, dtype=dt, scale=0.05, seed=512)
    if case == "misaligned_c":
        buf = torch.empty(M * N + 8, dtype=dt, device=DEV)
        C = buf[4:4 + M * N].view(M, N)  # 8-byte offset: not 16-byte aligned
    else:
        C = torch.empty(M, N, dtype=dt, device=DEV)
    K.kernel_counts_reset()
    K.gemm(X, W, C, M, N, Kd)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    if case == "few_tiles":
        assert c["gemm4"] == 1 and c["gemm_ring"] + c["gemm128"] == 0, c
    else:
        assert c["gemm4"] == 0 and c["gemm_ring"] + c["gemm128"] == 1, c
    check(C, f64(X) @ f64(W).T, 1e-2, "outside gemm4 " + case)


def test_gemm_rejects_bad_args():
    A = torch.zeros(16, 12, device=DEV)
    C = torch.zeros(16, 16, device=DEV)
    with pytest.raises(RuntimeError, match="lda"):
        K.gemm(A, A, C, 16, 16, 12, lda=10)


@pytest.mark.parametrize("M,N", [(16384 // 8, 4096), (1000, 2048)])
def test_gemm_drelu_colsum_partials(M, N):
    """colsum_part: the dReLU epilogue's per-128-row column sums of the stored dh
    (FFN1 bias gradient) against torch on the stored output; ragged M."""
    Kd = 512
    dY, W = rnd(M, Kd, dtype=torch.bfloat16, seed=120), rnd(Kd, N, dtype=torch.bfloat16, seed=121)
    h = torch.relu(rnd(M, N, dtype=torch.bfloat16, seed=122))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kw = dict(a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=0.25)
    rows = K.gemm_colsum_rows(dY, W, out, M, N, Kd, **kw)
    assert rows == (M + 127) // 128
    part = torch.full((rows, N), float("nan"), device=DEV)
    K.gemm(dY, W, out, M, N, Kd, colsum_part=part, **kw)
    bgrad = torch.zeros(N, device=DEV)
    K.reduce_rows(part, rows, N, bgrad, 0.0)
    torch.cuda.synchronize()
    check(bgrad, f64(out).sum(0), 1e-5, "dReLU colsum")
    ref = (f64(dY) @ f64(W)) * (f64(h) > 0) / 0.75
    check(out, ref, 1e-2, "dReLU out")
    # other epilogues / the 128 kernel cannot produce the sums
    assert K.gemm_colsum_rows(dY, W, out, M, N, Kd, a_kmajor=True, b_kmajor=False) == 0
    with pytest.raises(RuntimeError, match="colsum_part"):
        K.gemm(dY, W, out, M, N, Kd, a_kmajor=True, b_kmajor=False, colsum_part=part)


def _keep_pattern_np(seed, M, N, p):
    """Keep decision of element (i, j) under common.h's dropout hash:
    nstl_fmix32(pair ^ seed_term), low / high 16 bits against the threshold."""
    import numpy as np
    seed_term = (seed & 0xFFFFFFFF) ^ (((seed >> 32) * 0x27D4EB2F) & 0xFFFFFFFF)
    thresh = int(p * 65536.0 + 0.5)
    pair = (np.arange(M, dtype=np.uint64)[:, None] * (N // 2) + np.arange(N // 2, dtype=np.uint64)[None, :])
    h = (pair.astype(np.uint32) ^ np.uint32(seed_term)).astype(np.uint64)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    keep = np.empty((M, N), dtype=bool)
    keep[:, 0::2] = (h & 0xFFFF) >= thresh
    keep[:, 1::2] = (h >> 16) >= thresh
    return keep


@pytest.mark.parametrize("Kd", [256, 1024, 2048])
def test_gemm_relu_dropout_keep_pattern_matches_hash(Kd):
    """The ring kernel's ReLU-dropout epilogue keeps element (i, j) by the dropout
    hash of its pair index (common.h): with every pre-activation positive, the
    zero pattern is exactly the hash's, at short, medium and long K."""
    M, N = 2048, 1024
    X = rnd(M, Kd, dtype=torch.bfloat16, seed=150)
    W = rnd(N, Kd, dtype=torch.bfloat16, seed=151, scale=0.01)
    bias = torch.full((N,), 50.0, device=DEV)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=bias, p_drop=0.3, seed=(7 << 32) + 1234)
    words = K.gemm_relu_mask_words(X, W, h, M, N, Kd, **kw)
    assert words > 0  # the ring kernel (the path with a relu_mask layout) runs this shape
    mask = torch.zeros(words, dtype=torch.int64, device=DEV)
    K.gemm(X, W, h, M, N, Kd, relu_mask=mask, **kw)
    torch.cuda.synchronize()
    assert torch.equal((h != 0).cpu(), torch.from_numpy(_keep_pattern_np((7 << 32) + 1234, M, N, 0.3)))


@pytest.mark.parametrize("M,N", [(1024, 2048), (1000, 4096)])
def test_gemm_relu_mask_roundtrip(M, N):
    """relu_mask: the ReLU-dropout forward epilogue's keep&positive bits drive the
    dReLU backward epilogue to exactly the result of reading the saved hidden."""
    Kd = 512
    X, W1 = rnd(M, Kd, dtype=torch.bfloat16, seed=140), rnd(N, Kd, dtype=torch.bfloat16, seed=141)
    b1 = 0.1 * rnd(N, seed=142)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    fw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b1, p_drop=0.3, seed=31)
    words = K.gemm_relu_mask_words(X, W1, h, M, N, Kd, **fw)
    assert words == ((M + 63) // 64) * 8 * ((N + 7) // 8)
    mask = torch.zeros(words, dtype=torch.int64, device=DEV)
    K.gemm(X, W1, h, M, N, Kd, relu_mask=mask, **fw)
    h2 = torch.empty_like(h)
    K.gemm(X, W1, h2, M, N, Kd, **fw)
    dY, W2 = rnd(M, Kd, dtype=torch.bfloat16, seed=143), rnd(Kd, N, dtype=torch.bfloat16, seed=144)
    bw = dict(a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=0.3)
    assert K.gemm_relu_mask_words(dY, W2, h, M, N, Kd, **bw) == words
    d1, d2 = torch.empty_like(h), torch.empty_like(h)
    K.gemm(dY, W2, d1, M, N, Kd, relu_mask=mask, **bw)
    K.gemm(dY, W2, d2, M, N, Kd, **bw)
    torch.cuda.synchronize()
    assert torch.equal(h, h2)
    assert torch.equal(d1, d2)
    kept = (h.float() > 0).float().mean().item()
    assert 0.2 < kept < 0.5, kept   # ~0.7 keep x ~0.5 positive
    # the 128 kernel / other epilogues cannot use the mask
    assert K.gemm_relu_mask_words(X, W1, h, M, N, Kd, epilogue=K.EPI_BIAS, bias=b1) == 0


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_grouped_weight_gradients(beta):
    """nstl_gemm_grouped: independent dW = dY^T X problems of different shapes in one
    launch equal the same problems done one by one (and torch)."""
    m = 1024
    shapes = [(512, 256), (256, 768), (768, 512), (256, 256)]
    probs, refs, outs = [], [], []
    for i, (n, k) in enumerate(shapes):
        dY, X = rnd(m, n, dtype=torch.bfloat16, seed=80 + i), rnd(m, k, dtype=torch.bfloat16, seed=90 + i)
        G = rnd(n, k, seed=100 + i)
        ref = f64(dY).t() @ f64(X) + beta * f64(G)
        probs.append((dY, X, G, n, k, m, dict(a_kmajor=False, b_kmajor=False, beta=beta)))
        refs.append(ref)
        outs.append(G)
    K.gemm_grouped(probs)
    torch.cuda.synchronize()
    for (n, k), G, ref in zip(shapes, outs, refs):
        check(G, ref, 1e-5, "grouped dW %dx%d" % (n, k))


def test_gemm_grouped_rejects_mixed_layouts():
    A = torch.zeros(256, 256, dtype=torch.bfloat16, device=DEV)
    C = torch.zeros(256, 256, device=DEV)
    with pytest.raises(RuntimeError, match="differs"):
        K.gemm_grouped([(A, A, C, 256, 256, 256, dict(a_kmajor=False, b_kmajor=False)),
                        (A, A, C, 256, 256, 256, dict(a_kmajor=True, b_kmajor=False))])
    with pytest.raises(RuntimeError, match="256-kernel"):
        K.gemm_grouped([(A, A, C, 256, 128, 256, dict(a_kmajor=False, b_kmajor=False))])


# ---------------------------------------------------------------------------
def attn_ref(q, k, v, scale, mask=None, p=0.0):
    s = (q @ k.transpose(-1, -2)) * scale
    lse = torch.logsumexp(s, -1)
    P = torch.softmax(s, -1)
    Pd = P * mask / (1 - p) if mask is not None else P
    return Pd @ v, lse


def rope_back_ref(g, cs, sn):
    e, o = g[..., 0::2], g[..., 1::2]
    r = torch.empty_like(g)
    r[..., 0::2] = e * cs + o * sn
    r[..., 1::2] = -e * sn + o * cs
    return r


@pytest.mark.parametrize("dt,T,dh", [(torch.float32, 32, 64), (torch.float32, 128, 64), (torch.bfloat16, 64, 64),
                                     (torch.bfloat16, 128, 64), (torch.bfloat16, 256, 64),
                                     # generic kernels: ragged T, head_dim != 64 (BASELINE C1: 4 x 256)
                                     (torch.float32, 48, 64), (torch.bfloat16, 100, 128),
                                     (torch.float32, 128, 256), (torch.bfloat16, 128, 256), (torch.float32, 7, 24)])
def test_attention_fwd_bwd(dt, T, dh):
    B, H = 2, 3
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=dt, seed=20)
    o = torch.empty(M, D, dtype=dt, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    code = K.dtype_code(dt)
    a = K.attn_args(code, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D, qkv[:, 2 * D:].data_ptr(),
                    3 * D, o.data_ptr(), D, lse.data_ptr(), 0.0, 0, dh=dh)
    K.attn_fwd(a)
    torch.cuda.synchronize()
    q = f64(qkv[:, :D]).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    k = f64(qkv[:, D:2 * D]).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    v = f64(qkv[:, 2 * D:]).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    ro, rl = attn_ref(q, k, v, dh ** -0.5)
    tol = 5e-6 if dt == torch.float32 else 1e-2
    check(o, ro.transpose(1, 2).reshape(M, D), tol, "attn out")
    check(lse, rl.reshape(-1), 1e-5 if dt == torch.float32 else 1e-2, "attn lse")
    do = rnd(M, D, dtype=dt, seed=21)
    dqkv = torch.zeros(M, 3 * D, dtype=dt, device=DEV)
    cs, sn = rotation_tables(T, dh, DEV)
    a.dout, a.dout_ld = do.data_ptr(), D
    a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                    dqkv[:, 2 * D:].data_ptr(), 3 * D)
    a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
    dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a.dsum = dsum.data_ptr()
    K.attn_bwd(a)
    torch.cuda.synchronize()
    # reference uses the kernel's own (rounded) output o for D = rowsum(dO*O) consistency
    ro.backward(f64(do).view(B, T, H, dh).transpose(1, 2))
    c64, s64 = f64(cs), f64(sn)
    rdq = rope_back_ref(q.grad, c64, s64).transpose(1, 2).reshape(M, D)
    rdk = rope_back_ref(k.grad, c64, s64).transpose(1, 2).reshape(M, D)
    rdv = v.grad.transpose(1, 2).reshape(M, D)
    tolb = 2e-5 if dt == torch.float32 else 3e-2
    check(dqkv[:, :D], rdq, tolb, "dq")
    check(dqkv[:, D:2 * D], rdk, tolb, "dk")
    check(dqkv[:, 2 * D:], rdv, tolb, "dv")


@pytest.mark.parametrize("dt,T", [(torch.float32, 64), (torch.bfloat16, 64), (torch.float32, 40),
                                  (torch.bfloat16, 40)])
def test_attention_dropout_consistency(dt, T):
    """dh = T with V = I reveals the keep-mask through the output; check the rate, then
    check fwd and bwd against a reference that uses exactly that mask (T=40: generic kernels)."""
    B, H, dh, p = 2, 2, T, 0.3
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=dt, scale=0.5, seed=30)
    eye = torch.eye(T, dtype=dt, device=DEV)
    vI = eye.repeat(B, H)  # [B*T, H*dh], V[b,t,h,:] = e_t
    o = torch.empty(M, D, dtype=torch.float32 if dt == torch.float32 else dt, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    code = K.dtype_code(dt)
    a = K.attn_args(code, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D, vI.data_ptr(), D,
                    o.data_ptr(), D, lse.data_ptr(), p, 777, dh=dh)
    K.attn_fwd(a)
    torch.cuda.synchronize()
    Pd = f64(o).view(B, T, H, dh).transpose(1, 2)  # = P * mask / (1-p)
    mask = (Pd != 0).double()
    frac = mask.mean().item()
    assert abs(frac - 0.7) < 0.03, frac
    q = f64(qkv[:, :D]).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    k = f64(qkv[:, D:2 * D]).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    v = rnd(M, D, dtype=dt, seed=31)
    vv = f64(v).view(B, T, H, dh).transpose(1, 2).requires_grad_(True)
    ro, _ = attn_ref(q, k, vv, dh ** -0.5, mask, p)
    o2 = torch.empty(M, D, dtype=dt, device=DEV)
    a2 = K.attn_args(code, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D, v.data_ptr(), D,
                     o2.data_ptr(), D, lse.data_ptr(), p, 777, dh=dh)
    K.attn_fwd(a2)
    tol = 5e-6 if dt == torch.float32 else 1e-2
    check(o2, ro.transpose(1, 2).reshape(M, D), tol, "attn dropout out")
    do = rnd(M, D, dtype=dt, seed=32)
    dq, dk, dv = (torch.zeros(M, D, dtype=dt, device=DEV) for _ in range(3))
    a2.dout, a2.dout_ld = do.data_ptr(), D
    a2.dq, a2.dq_ld, a2.dk, a2.dk_ld, a2.dv, a2.dv_ld = dq.data_ptr(), D, dk.data_ptr(), D, dv.data_ptr(), D
    dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a2.dsum = dsum.data_ptr()
    K.attn_bwd(a2)
    torch.cuda.synchronize()
    ro.backward(f64(do).view(B, T, H, dh).transpose(1, 2))
    tolb = 2e-5 if dt == torch.float32 else 3e-2
    check(dq, q.grad.transpose(1, 2).reshape(M, D), tolb, "dq (dropout)")
    check(dk, k.grad.transpose(1, 2).reshape(M, D), tolb, "dk (dropout)")
    check(dv, vv.grad.transpose(1, 2).reshape(M, D), tolb, "dv (dropout)")


@pytest.mark.parametrize("dt,T", [(torch.bfloat16, 64), (torch.bfloat16, 128), (torch.bfloat16, 256),
                                  (torch.float32, 128)])
def test_attention_stored_mask_bits(dt, T):
    """The forward's stored keep bits (nstl_attn_args.mask_bits) drive the backward
    to the same bits as re-hashing (seed, element): identical outputs, keep rate 1-p."""
    B, H, dh, p = 2, 3, 64, 0.3
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=dt, scale=0.5, seed=70)
    do = rnd(M, D, dtype=dt, seed=71)
    cs, sn = rotation_tables(T, dh, DEV)
    code = K.dtype_code(dt)
    outs = []
    for stored in (False, True):
        o = torch.empty(M, D, dtype=dt, device=DEV)
        lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
        dqkv = torch.zeros(M, 3 * D, dtype=dt, device=DEV)
        dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
        mask = torch.full((B * H * T * T // 64,), -1, dtype=torch.int64, device=DEV)
        a = K.attn_args(code, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                        qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 4242, dh=dh)
        if stored:
            a.mask_bits = mask.data_ptr()
        K.attn_fwd(a)
        a.dout, a.dout_ld = do.data_ptr(), D
        a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                        dqkv[:, 2 * D:].data_ptr(), 3 * D)
        a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
        a.dsum = dsum.data_ptr()
        K.attn_bwd(a)
        torch.cuda.synchronize()
        outs.append((o.clone(), dqkv.clone(), mask.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    bits = outs[1][2].cpu().numpy().view(np.uint8)
    frac = np.unpackbits(bits).mean()
    assert abs(frac - (1 - p)) < 0.01, frac


@pytest.mark.parametrize("B,H,p,stored", [(2, 3, 0.3, True), (65, 16, 0.3, True), (128, 16, 0.3, True),
                                          (65, 16, 0.0, False), (65, 16, 0.3, False)])
def test_attention_fwd_persistent_matches_oneshot(B, H, p, stored, monkeypatch):
    """The persistent forward (bf16, T=128: heads walked by 2 workgroups per CU with
    the next head's K / V / Q prefetched by LDS-DMA) against the one-workgroup-per-head
    kernel: O, LSE and the stored keep bits bit-identical.  B*H = 6 (fewer heads than
    workgroups), 1040 (some workgroups take 3 heads, others 2) and 2048 (the 228M step)."""
    T, dh = 128, 64
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=torch.bfloat16, scale=0.5, seed=95)
    outs = []
    for mode in ("oneshot", "persist"):
        monkeypatch.setenv("NSTL_ATTN_FWD", mode)
        o = torch.full((M, D), float("nan"), dtype=torch.bfloat16, device=DEV)
        lse = torch.full((B * H * T,), float("nan"), dtype=torch.float32, device=DEV)
        mask = torch.full((B * H * T * T // 64,), -1, dtype=torch.int64, device=DEV)
        a = K.attn_args(K.BF16, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                        qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 1234, dh=dh)
        if stored:
            a.mask_bits = mask.data_ptr()
        K.attn_fwd(a)
        torch.cuda.synchronize()
        outs.append((o, lse, mask))
    assert not torch.isnan(outs[1][0].float()).any() and not torch.isnan(outs[1][1]).any()
    assert torch.equal(outs[0][0], outs[1][0]), "O"
    assert torch.equal(outs[0][1], outs[1][1]), "LSE"
    assert torch.equal(outs[0][2], outs[1][2]), "keep bits"


@pytest.mark.parametrize("dt,T", [(torch.bfloat16, 128), (torch.bfloat16, 64), (torch.bfloat16, 256),
                                  (torch.float32, 96)])
def test_attention_bias_partials(dt, T):
    """dbias_part: the backward's fused column sums of dq | dk | dv (as stored) give
    the q/k/v projection bias gradients after a row reduction."""
    B, H, dh = 3, 2, 64
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=dt, scale=0.5, seed=110)
    o = torch.empty(M, D, dtype=dt, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a = K.attn_args(K.dtype_code(dt), B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                    qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), 0.2, 99, dh=dh)
    K.attn_fwd(a)
    do = rnd(M, D, dtype=dt, seed=111)
    dqkv = torch.zeros(M, 3 * D, dtype=dt, device=DEV)
    cs, sn = rotation_tables(T, dh, DEV)
    a.dout, a.dout_ld = do.data_ptr(), D
    a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                    dqkv[:, 2 * D:].data_ptr(), 3 * D)
    a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
    dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a.dsum = dsum.data_ptr()
    rows = K.attn_bias_rows(a)
    assert rows == B * ((T + 127) // 128)
    part = torch.full((rows, 3 * D), float("nan"), device=DEV)
    a.dbias_part = part.data_ptr()
    K.attn_bwd(a)
    out = torch.full((3 * D,), 5.0, device=DEV)
    K.reduce_rows_strided(part, 3 * D, rows, 3 * D, out, 1.0)
    qpart = torch.zeros(D, device=DEV)
    K.reduce_rows_strided(part[:, D:], 3 * D, rows, D, qpart, 0.0)   # the k window alone
    torch.cuda.synchronize()
    ref = f64(dqkv).sum(0)
    check(out - 5.0, ref, 1e-5, "fused q|k|v bias grads")
    check(qpart, ref[D:2 * D], 1e-5, "k window")
    # the generic kernels do not produce the sums
    a.dh = 32
    assert K.attn_bias_rows(a) == 0


def test_dropout_hash_statistics():
    """The counter hash behind every dropout mask (common.h nstl_pair_hash), read
    back through the attention forward's stored keep bits (1M elements, p=0.3):
    keep rate 1-p, and independent decisions for the two halves of one hash
    (keys k, k+1), neighbouring hashes (k, k+2), neighbouring queries and
    different heads."""
    B, H, T, dh, p = 4, 16, 128, 64, 0.3
    M, D = B * T, H * dh
    qkv = rnd(M, 3 * D, dtype=torch.bfloat16, scale=0.5, seed=90)
    o = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    mask = torch.zeros(B * H * T * T // 64, dtype=torch.int64, device=DEV)
    a = K.attn_args(K.BF16, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                    qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 20240917, dh=dh)
    a.mask_bits = mask.data_ptr()
    K.attn_fwd(a)
    torch.cuda.synchronize()
    nt = T // 16
    w = mask.cpu().numpy().view(np.uint64).reshape(B * H, nt, nt, 4)  # [bh][qt][kt][key % 4]
    bits = ((w[..., None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8)
    # bit 16 * ((key % 16) / 4) + query % 16  ->  keep[bh][query][key]
    keep = bits.reshape(B * H, nt, nt, 4, 4, 16).transpose(0, 1, 5, 2, 4, 3).reshape(B * H, T, T).astype(np.float64)
    q = 1.0 - p
    assert abs(keep.mean() - q) < 0.003, keep.mean()
    pairs = {
        "halves of one hash (k, k+1)": (keep[:, :, 0::2], keep[:, :, 1::2]),
        "neighbouring hashes (k, k+2)": (keep[:, :, 0:-2:2], keep[:, :, 2::2]),
        "neighbouring queries": (keep[:, :-1, :], keep[:, 1:, :]),
    }
    for what, (x, y) in pairs.items():
        joint = (x * y).mean()
        assert abs(joint - q * q) < 0.004, (what, joint)
    agree = (keep[0::2] == keep[1::2]).mean()  # head 2i vs head 2i+1
    assert abs(agree - (q * q + p * p)) < 0.006, agree


@pytest.mark.parametrize("T", [32, 96, 128])
def test_attention_bwd_fused_matches_split(T, monkeypatch):
    """The fused one-workgroup-per-(b, h) backward (bf16, T <= 128) against the split
    dQ / dK+dV kernels on the same forward: dropout from stored keep bits, RoPE^T,
    bias partials.  T=96 leaves two waves of the workgroup without keys."""
    B, H, dh, p = 3, 2, 64, 0.3
    M, D = B * T, H * dh
    dt = torch.bfloat16
    qkv = rnd(M, 3 * D, dtype=dt, scale=0.5, seed=120)
    do = rnd(M, D, dtype=dt, seed=121)
    o = torch.empty(M, D, dtype=dt, device=DEV)
    lse = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    mask = torch.zeros(B * H * T * T // 64, dtype=torch.int64, device=DEV)
    cs, sn = rotation_tables(T, dh, DEV)
    a = K.attn_args(K.BF16, B, T, H, qkv.data_ptr(), 3 * D, qkv[:, D:].data_ptr(), 3 * D,
                    qkv[:, 2 * D:].data_ptr(), 3 * D, o.data_ptr(), D, lse.data_ptr(), p, 7, dh=dh)
    a.mask_bits = mask.data_ptr()
    K.attn_fwd(a)
    dsum = torch.empty(B * H * T, dtype=torch.float32, device=DEV)
    a.dout, a.dout_ld = do.data_ptr(), D
    a.rope_cos, a.rope_sin, a.rope_q, a.rope_k = cs.data_ptr(), sn.data_ptr(), 1, 1
    a.dsum = dsum.data_ptr()
    rows = K.attn_bias_rows(a)
    res = []
    # fused: RoPE^T angles recomputed in the kernel (default); fused_table: from the tables
    modes = ("split", "fused", "fused_table")
    for mode in modes:
        monkeypatch.setenv("NSTL_ATTN_BWD", mode)
        monkeypatch.setenv("NSTL_ROPE_BWD", "table" if mode == "fused_table" else "fast")
        dqkv = torch.full((M, 3 * D), float("nan"), dtype=dt, device=DEV)
        part = torch.full((rows, 3 * D), float("nan"), device=DEV)
        a.dq, a.dq_ld, a.dk, a.dk_ld, a.dv, a.dv_ld = (dqkv.data_ptr(), 3 * D, dqkv[:, D:].data_ptr(), 3 * D,
                                                        dqkv[:, 2 * D:].data_ptr(), 3 * D)
        a.dbias_part = part.data_ptr()
        K.attn_bwd(a)
        torch.cuda.synchronize()
        res.append((dqkv, part))
    ds, ps = res[0]
    for (df, pf), mode in zip(res[1:], modes[1:]):
        assert torch.isfinite(f64(df)).all() and torch.isfinite(f64(pf)).all(), mode
        for i, nm in enumerate(("dq", "dk", "dv")):
            check(df[:, i * D:(i + 1) * D], ds[:, i * D:(i + 1) * D], 1e-2, mode + " " + nm)
        check(pf, f64(df).view(B, T, 3 * D).sum(1), 1e-5, mode + " bias partials = column sums of the stored grads")
        check(pf, ps, 1e-2, mode + " vs split bias partials")
    # recomputed angles vs the tables: the same rotation to well inside bf16 rounding
    for i in range(2):
        check(res[1][0][:, i * D:(i + 1) * D], res[2][0][:, i * D:(i + 1) * D], 8e-3, "fast vs table RoPE^T")


def test_attention_rejects_bad_shapes():
    t = torch.zeros(64, 3 * 64, device=DEV)
    lse = torch.zeros(64, device=DEV)
    a = K.attn_args(K.F32, 1, 48, 1, t.data_ptr(), 192, t.data_ptr(), 192, t.data_ptr(), 192, t.data_ptr(), 64,
                    lse.data_ptr(), 0.0, 0, dh=60)
    with pytest.raises(RuntimeError, match="head_dim"):
        K.attn_fwd(a)
    a.dh, a.T = 64, 5000
    with pytest.raises(RuntimeError, match="T must be"):
        K.attn_fwd(a)


# ---------------------------------------------------------------------------
def ln_args(dt, rows, D, x, y, g, b, s, out, stats, n_masks=0, p=0.0, seeds=(0, 0)):
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.dtype_code(dt), rows, D
    a.x, a.y = K.ptr(x), y.data_ptr()
    a.n_masks, a.p_drop, a.seed1, a.seed2 = n_masks, p, seeds[0], seeds[1]
    a.gamma, a.beta, a.eps = g.data_ptr(), b.data_ptr(), 1e-5
    a.s_out, a.out, a.mean, a.rstd = K.ptr(s), out.data_ptr(), stats[0].data_ptr(), stats[1].data_ptr()
    return a


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [128, 256, 1024])
def test_layernorm_fwd_bwd(dt, D):
    rows = 96
    x, y = rnd(rows, D, dtype=dt, seed=40), rnd(rows, D, dtype=dt, seed=41)
    g, b = 1 + 0.1 * rnd(D, seed=42), 0.1 * rnd(D, seed=43)
    s = torch.empty(rows, D, dtype=dt, device=DEV)
    out = torch.empty(rows, D, dtype=dt, device=DEV)
    stats = torch.empty(2, rows, device=DEV)
    K.ln_fwd(ln_args(dt, rows, D, x, y, g, b, s, out, stats))
    torch.cuda.synchronize()
    xs = (f64(x) + f64(y)).requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xs, (D,), f64(g), f64(b), 1e-5)
    tol = 2e-6 if dt == torch.float32 else 1e-2
    check(out, ref, tol, "ln out")
    check(s, f64(x) + f64(y), 1e-7 if dt == torch.float32 else 4e-3, "ln s")
    dout = rnd(rows, D, seed=44)
    ds = torch.empty(rows, D, device=DEV)
    dbr = torch.empty(rows, D, dtype=dt, device=DEV)
    npart = 8
    gp, bp = torch.empty(npart, D, device=DEV), torch.empty(npart, D, device=DEV)
    a = ln_args(dt, rows, D, x, y, g, b, None, out, stats)
    a.s_in, a.dout, a.ds, a.dbranch = s.data_ptr(), dout.data_ptr(), ds.data_ptr(), dbr.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part = gp.data_ptr(), bp.data_ptr(), npart
    K.ln_bwd(a)
    torch.cuda.synchronize()
    # reference from the kernel's saved s (what backward actually consumes)
    ss = f64(s).requires_grad_(True)
    gg, bb = f64(g).requires_grad_(True), f64(b).requires_grad_(True)
    r2 = torch.nn.functional.layer_norm(ss, (D,), gg, bb, 1e-5)
    r2.backward(f64(dout))
    tolb = 1e-5 if dt == torch.float32 else 1e-2
    check(ds, ss.grad, tolb, "ln ds")
    check(dbr, ss.grad, tolb, "ln dbranch")
    # bf16: the kernel's xhat uses the forward (f32) statistics of s, the reference
    # recomputes them from the bf16-rounded s -> differences at bf16 rounding level
    check(f64(gp).sum(0), gg.grad, 1e-5 if dt == torch.float32 else 2e-3, "ln dgamma")
    check(f64(bp).sum(0), bb.grad, 1e-5, "ln dbeta")


@pytest.mark.parametrize("D", [128, 256, 512, 1024])
@pytest.mark.parametrize("with_x", [True, False])
def test_layernorm_fwd_global_pe(D, with_x):
    """rot_out = GlobalPositionalEncoding(out) (model.py:29-48, :246) fused into
    the final encoder LayerNorm; x = None is the plain LN of y."""
    from neurosync_trainer_lite_amd.engine import rotation_tables
    dt, T, rows = torch.float32, 50, 100
    x, y = rnd(rows, D, seed=60), rnd(rows, D, seed=61)
    g, b = 1 + 0.1 * rnd(D, seed=62), 0.1 * rnd(D, seed=63)
    out = torch.empty(rows, D, device=DEV)
    rot = torch.empty(rows, D, device=DEV)
    stats = torch.empty(2, rows, device=DEV)
    cs, sn = rotation_tables(T, D, DEV)
    a = ln_args(dt, rows, D, x if with_x else None, y, g, b, None, out, stats)
    a.rot_out, a.rope_cos, a.rope_sin, a.rope_T = rot.data_ptr(), cs.data_ptr(), sn.data_ptr(), T
    K.ln_fwd(a)
    torch.cuda.synchronize()
    inp = f64(x) + f64(y) if with_x else f64(y)
    ref = torch.nn.functional.layer_norm(inp, (D,), f64(g), f64(b), 1e-5)
    check(out, ref, 2e-6, "ln out")
    t = torch.arange(rows) % T
    c, s_ = f64(cs)[t], f64(sn)[t]
    e, o = ref[:, 0::2], ref[:, 1::2]
    rr = torch.stack([e * c - o * s_, e * s_ + o * c], dim=-1).reshape(rows, D)
    check(rot, rr, 2e-6, "ln rot_out")
    check(stats[0], inp.mean(1), 1e-6, "ln mean")


@pytest.mark.parametrize("dt,D", [(torch.bfloat16, 1024), (torch.float32, 128), (torch.bfloat16, 256)])
def test_layernorm_bwd_dout2_addend(dt, D):
    """dout2 (a Linear's input gradient in the compute dtype) is added to dout:
    same result as one f32 gradient dout + dout2."""
    rows = 64
    x, y = rnd(rows, D, dtype=dt, seed=130), rnd(rows, D, dtype=dt, seed=131)
    g, b = 1 + 0.1 * rnd(D, seed=132), 0.1 * rnd(D, seed=133)
    s = torch.empty(rows, D, dtype=dt, device=DEV)
    out = torch.empty(rows, D, dtype=dt, device=DEV)
    stats = torch.empty(2, rows, device=DEV)
    K.ln_fwd(ln_args(dt, rows, D, x, y, g, b, s, out, stats))
    g1, g2 = rnd(rows, D, seed=134), rnd(rows, D, dtype=dt, seed=135)
    res = []
    for split in (True, False):
        ds = torch.empty(rows, D, device=DEV)
        part = torch.empty(2, 4, D, device=DEV)
        a = ln_args(dt, rows, D, x, y, g, b, None, out, stats)
        dout = g1 if split else g1 + g2.float()
        a.s_in, a.dout, a.ds, a.dbranch = s.data_ptr(), dout.data_ptr(), ds.data_ptr(), None
        a.dgamma_part, a.dbeta_part, a.n_part = part[0].data_ptr(), part[1].data_ptr(), 4
        if split:
            a.dout2 = g2.data_ptr()
        K.ln_bwd(a)
        torch.cuda.synchronize()
        res.append((ds, part))
    check(res[0][0], res[1][0], 1e-6, "ds with dout2")
    check(res[0][1], res[1][1], 1e-6, "dgamma/dbeta with dout2")


@pytest.mark.parametrize("n_masks", [1, 2])
def test_layernorm_dropout_masks(n_masks):
    dt, rows, D, p = torch.float32, 64, 256, 0.3
    x = torch.zeros(rows, D, device=DEV)
    y = torch.ones(rows, D, device=DEV)
    g, b = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
    s = torch.empty(rows, D, device=DEV)
    out = torch.empty(rows, D, device=DEV)
    stats = torch.empty(2, rows, device=DEV)
    K.ln_fwd(ln_args(dt, rows, D, x, y, g, b, s, out, stats, n_masks, p, (11, 22)))
    torch.cuda.synchronize()
    m = f64(s) * (1 - p) ** n_masks  # = m1*m2 in {0,1}
    assert set(np.unique(m.numpy().round(6))) <= {0.0, 1.0}
    assert abs(m.mean().item() - 0.7 ** n_masks) < 0.02
    # backward: dbranch = ds * mask / (1-p)^n
    dout = rnd(rows, D, seed=45)
    ds = torch.empty(rows, D, device=DEV)
    dbr = torch.empty(rows, D, device=DEV)
    gp, bp = torch.empty(4, D, device=DEV), torch.empty(4, D, device=DEV)
    a = ln_args(dt, rows, D, x, y, g, b, None, out, stats, n_masks, p, (11, 22))
    a.s_in, a.dout, a.ds, a.dbranch = s.data_ptr(), dout.data_ptr(), ds.data_ptr(), dbr.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part = gp.data_ptr(), bp.data_ptr(), 4
    K.ln_bwd(a)
    torch.cuda.synchronize()
    check(dbr, f64(ds) * m / (1 - p) ** n_masks, 1e-6, "dbranch masks")


@pytest.mark.parametrize("rows,npart", [(37, 4), (1000, 125)])
def test_layernorm_bwd_ragged_partials(rows, npart):
    """Row counts that do not fill the last block's waves; the fused bias-gradient
    partials (dbranch_part) against torch on the same masked dbranch."""
    dt, D, p = torch.bfloat16, 1024, 0.3
    x, y = rnd(rows, D, dtype=dt, seed=50), rnd(rows, D, dtype=dt, seed=51)
    g, b = 1 + 0.1 * rnd(D, seed=52), 0.1 * rnd(D, seed=53)
    s = torch.empty(rows, D, dtype=dt, device=DEV)
    out = torch.empty(rows, D, dtype=dt, device=DEV)
    stats = torch.empty(2, rows, device=DEV)
    K.ln_fwd(ln_args(dt, rows, D, x, y, g, b, s, out, stats, 2, p, (5, 6)))
    dout = rnd(rows, D, seed=54)
    ds = torch.empty(rows, D, device=DEV)
    dbr = torch.empty(rows, D, dtype=dt, device=DEV)
    part = torch.empty(3, npart, D, device=DEV)
    a = ln_args(dt, rows, D, x, y, g, b, None, out, stats, 2, p, (5, 6))
    a.s_in, a.dout, a.ds, a.dbranch = s.data_ptr(), dout.data_ptr(), ds.data_ptr(), dbr.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part = part[0].data_ptr(), part[1].data_ptr(), npart
    a.dbranch_part = part[2].data_ptr()
    K.ln_bwd(a)
    torch.cuda.synchronize()
    ss = f64(s).requires_grad_(True)
    gg, bb = f64(g).requires_grad_(True), f64(b).requires_grad_(True)
    torch.nn.functional.layer_norm(ss, (D,), gg, bb, 1e-5).backward(f64(dout))
    check(ds, ss.grad, 1e-2, "ln ds")
    # the same masks as the forward: dbranch / ds is 0 or 1/(1-p)^2
    ratio = f64(dbr)[f64(ds).abs() > 1e-3] / f64(ds)[f64(ds).abs() > 1e-3]
    assert ((ratio.abs() < 1e-6) | ((ratio - 1 / 0.49).abs() < 0.02)).all()
    check(f64(part[0]).sum(0), gg.grad, 2e-3, "ln dgamma")
    check(f64(part[1]).sum(0), bb.grad, 1e-5, "ln dbeta")
    check(f64(part[2]).sum(0), f64(dbr).sum(0), 1e-5, "ln dbranch colsum")


# ---------------------------------------------------------------------------
def test_loss_matches_reference_golden(golden):
    from neurosync_trainer_lite_amd.utils.model import Loss
    g = golden("loss.npz")
    crit = Loss(delta=1.0, w1=1.0, w2=1.0)
    for case in ("random", "zero_target", "zero_pred_diff", "small"):
        p = torch.tensor(g[case + "_pred"], device=DEV, requires_grad=True)
        t = torch.tensor(g[case + "_trg"], device=DEV)
        loss = crit(p, t)
        loss.backward()
        ref = float(g[case + "_loss"])
        assert abs(loss.item() - ref) <= 2e-6 * max(1.0, abs(ref)), (case, loss.item(), ref)
        gr = g[case + "_grad"]
        np.testing.assert_allclose(p.grad.cpu().numpy(), gr, rtol=1e-4, atol=1e-5 * np.abs(gr).max())


def test_loss_full_batch_shape_and_scale():
    from neurosync_trainer_lite_amd.utils.model import Loss
    from oracle import model_ref
    B, T, F = 128, 128, 61
    p = rnd(B, T, F, scale=30, seed=50).requires_grad_(True)
    t = rnd(B, T, F, scale=30, seed=51)
    loss = Loss()(p, t)
    (loss * 3.0).backward()
    pc = f64(p).requires_grad_(True)
    lr = model_ref.loss_fn(pc, f64(t))
    (lr * 3.0).backward()
    assert abs(loss.item() - lr.item()) < 1e-5 * abs(lr.item())
    check(p.grad, pc.grad, 1e-4, "loss grad (scaled)")


# ---------------------------------------------------------------------------
def test_adam_clip_matches_oracle():
    from oracle import model_ref
    n = 1_000_003
    p = rnd(n, seed=60)
    g = rnd(n, scale=0.01, seed=61)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    p16 = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    part = torch.empty(1024, device=DEV)
    norm = torch.empty(1, device=DEV)
    pr, mr, vr = f64(p).float(), torch.zeros(n), torch.zeros(n)
    for step in range(1, 4):
        gs = g * step
        K.sumsq(gs, n, part, 1024)
        a = K.AdamArgs()
        a.p, a.g, a.m, a.v = p.data_ptr(), gs.data_ptr(), m.data_ptr(), v.data_ptr()
        a.p_lowp, a.lowp_dtype, a.n = p16.data_ptr(), K.BF16, n
        a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = 1e-3, 0.9, 0.999, 1e-8, 1e-2
        a.step, a.sumsq_partial, a.n_partial, a.max_norm, a.norm_out = step, part.data_ptr(), 1024, 2.0, norm.data_ptr()
        K.adam_step(a)
        torch.cuda.synchronize()
        gr = f64(gs).float()
        truth = f64(gs).norm().item()  # the kernel accumulates in f64; torch-CPU f32 norm is ~1e-5 off
        assert abs(norm.item() - truth) < 1e-6 * truth
        assert abs(norm.item() - model_ref.clip_grad_norm([gr.clone()], 2.0).item()) < 3e-5 * truth
        # clip with the kernel's norm (where g*coef and wd*p cancel, a 1e-5 change of
        # coef moves the Adam direction a lot), then compare the update math exactly
        coef = min(1.0, 2.0 / (norm.item() + 1e-6))
        model_ref.adam_l2_step([pr], [gr * torch.tensor(coef, dtype=torch.float32)], [mr], [vr], step, 1e-3,
                               weight_decay=1e-2)
        torch.testing.assert_close(p.cpu(), pr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p16.cpu(), p.cpu().to(torch.bfloat16))


def test_adam_coef_path_matches_sumsq_path():
    """The engine's path (nstl_clip_coef, then nstl_adam_step reading `coef`:
    adam_gcoef_kernel, whichever NSTL_ADAM_NT / NSTL_ADAM_U variant the process
    runs) is bit-identical to the one-launch sumsq path (adam_kernel)."""
    n = 1_000_003
    g = rnd(n, scale=0.01, seed=63)
    part = torch.empty(1024, device=DEV)
    K.sumsq(g, n, part, 1024)
    coef, norm = torch.empty(1, device=DEV), torch.empty(1, device=DEV)
    K.clip_coef(part, 1024, 2.0, coef, norm)
    outs = []
    for use_coef in (False, True):
        p = rnd(n, seed=62)
        m, v = rnd(n, scale=0.01, seed=64), rnd(n, scale=1e-4, seed=65).abs()
        p16 = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        a = K.AdamArgs()
        a.p, a.g, a.m, a.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        a.p_lowp, a.lowp_dtype, a.n = p16.data_ptr(), K.BF16, n
        a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = 1e-3, 0.9, 0.999, 1e-8, 1e-2
        a.step, a.max_norm = 3, 2.0
        if use_coef:
            a.coef = coef.data_ptr()
        else:
            a.sumsq_partial, a.n_partial = part.data_ptr(), 1024
        K.adam_step(a)
        outs.append((p, m, v, p16))
    torch.cuda.synchronize()
    for name, x, y in zip(("p", "m", "v", "p16"), *outs):
        assert torch.equal(x, y), (name, (x.float() - y.float()).abs().max().item(), (x != y).sum().item())


def test_small_kernels():
    rows, cols = 600, 200
    x = rnd(rows, cols, dtype=torch.bfloat16, seed=70)
    part = torch.empty((rows + 255) // 256, cols, device=DEV)
    out = torch.ones(cols, device=DEV)
    K.colsum(x, cols, rows, cols, part, out, 1.0)
    check(out, 1 + f64(x).sum(0), 1e-6, "colsum")
    src = rnd(rows, 61, seed=71)
    dst = torch.full((rows, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    sc = torch.tensor([0.5], device=DEV)
    K.copy2d(src, 61, dst, 64, rows, 61, 64, scale=sc)
    check(dst[:, :61], 0.5 * f64(src), 5e-3, "copy2d")
    assert (dst[:, 61:] == 0).all()
    T, D = 16, 128
    y = rnd(2 * T, D, seed=72)
    cs, sn = rotation_tables(T, D, DEV)
    r = torch.empty_like(y)
    K.rope(y, D, r, D, 2 * T, D, cs, sn, T, D)
    back = torch.zeros_like(y)
    K.rope(r, D, back, D, 2 * T, D, cs, sn, T, D, inverse=True, accumulate=True)
    check(back, y, 1e-6, "rope inverse")


# ---------------------------------------------------------------------------
# 256x256 LDS-DMA kernel (selected for bf16 problems with >= 64 of its tiles)
@pytest.mark.parametrize("M,N,Kd", [(2048, 2048, 512), (2000, 2304, 256), (4096, 1024, 1024)])
def test_gemm256_forward(M, N, Kd):
    dt = torch.bfloat16
    A, W, b = rnd(M, Kd, dtype=dt, seed=80), rnd(N, Kd, dtype=dt, scale=0.05, seed=81), rnd(N, seed=82)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    K.gemm(A, W, C, M, N, Kd, epilogue=K.EPI_BIAS, bias=b)
    torch.cuda.synchronize()
    check(C, f64(A) @ f64(W).T + f64(b), 1e-5, "gemm256 NT")


@pytest.mark.parametrize("M,N,Kd", [(2048, 2048, 512), (4096, 1024, 2048)])
def test_gemm256_dx(M, N, Kd):
    dt = torch.bfloat16
    dY, W = rnd(M, N, dtype=dt, seed=83), rnd(N, Kd, dtype=dt, seed=84)
    C0 = rnd(M, Kd, seed=85)
    C = C0.clone()
    K.gemm(dY, W, C, M, Kd, N, a_kmajor=True, b_kmajor=False, beta=1.0)
    torch.cuda.synchronize()
    check(C, f64(C0) + f64(dY) @ f64(W), 1e-5, "gemm256 dX")


@pytest.mark.parametrize("Mt,N,Kd,split", [(4096, 512, 512, 16), (2048, 2048, 512, 1), (8192, 768, 512, 8)])
def test_gemm256_dw(Mt, N, Kd, split):
    dt = torch.bfloat16
    dY, X = rnd(Mt, N, dtype=dt, seed=86), rnd(Mt, Kd, dtype=dt, seed=87)
    C0 = rnd(N, Kd, seed=88)
    C = C0.clone()
    ws = torch.empty(split * N * Kd, dtype=torch.float32, device=DEV)
    K.gemm(dY, X, C, N, Kd, Mt, a_kmajor=False, b_kmajor=False, beta=1.0, split_k=split, workspace=ws)
    torch.cuda.synchronize()
    check(C, f64(C0) + f64(dY).T @ f64(X), 1e-5, "gemm256 dW")


def test_gemm256_epilogues():
    """RoPE / ReLU-dropout / dReLU epilogues through the 256 kernel (bf16 out)."""
    dt, B, T, D = torch.bfloat16, 16, 128, 1024
    M = B * T
    X, W, b = rnd(M, 256, dtype=dt, seed=89), rnd(3 * D, 256, dtype=dt, scale=0.05, seed=90), rnd(3 * D, seed=91)
    cs, sn = rotation_tables(T, 64, DEV)
    C = torch.empty(M, 3 * D, dtype=dt, device=DEV)
    K.gemm(X, W, C, M, 3 * D, 256, epilogue=K.EPI_BIAS_ROPE, bias=b, rope=(cs, sn, T, 64), rope_cols=2 * D)
    y = f64(X) @ f64(W).T + f64(b)
    ref = y.clone()
    c, s = f64(cs), f64(sn)
    z = y[:, :2 * D].reshape(B, T, 2 * D // 64, 64).permute(0, 2, 1, 3)
    e, o = z[..., 0::2], z[..., 1::2]
    r = torch.empty_like(z)
    r[..., 0::2] = e * c - o * s
    r[..., 1::2] = e * s + o * c
    ref[:, :2 * D] = r.permute(0, 2, 1, 3).reshape(M, 2 * D)
    check(C, ref, 8e-3, "gemm256 rope")
    H = torch.empty(M, 3 * D, dtype=dt, device=DEV)
    K.gemm(X, W, H, M, 3 * D, 256, epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=5)
    h = f64(H)
    pos = torch.relu(y) > 1e-2
    kept = h[pos] != 0
    assert abs(kept.double().mean().item() - 0.7) < 0.01
    torch.testing.assert_close(h[pos][kept], (torch.relu(y)[pos][kept] / 0.7), rtol=1e-2, atol=1e-3)


def test_reduce_rows_batch():
    """nstl_reduce_rows_batch: jobs of different shapes, strides and betas in one
    launch give exactly the per-job column sums (reduce_rows3's order)."""
    jobs, refs = [], []
    for k, (n_part, cols, ld, beta) in enumerate([(256, 1024, 1024, 0.0), (128, 3072, 3072, 1.0),
                                                  (17, 61, 64, 0.5), (128, 1024, 3072, 0.0)]):
        part = rnd(n_part, ld, seed=200 + k)
        out = rnd(cols, seed=300 + k)
        refs.append(beta * f64(out) + f64(part[:, :cols]).sum(0))
        jobs.append((part, ld, n_part, cols, out, beta))
    K.reduce_rows_batch(jobs)
    torch.cuda.synchronize()
    for k, (job, ref) in enumerate(zip(jobs, refs)):
        check(job[4], ref, 1e-6, "batched reduce job %d" % k)
    with pytest.raises(RuntimeError, match="jobs"):
        K.reduce_rows_batch(jobs * 5)


def test_transpose_bf16_batched_bit_exact():
    """nstl_transpose_bf16: several jobs of different shapes in one launch, padded
    leading dimensions on both sides, every element moved exactly."""
    shapes = [(64, 64), (1024, 3072), (4096, 1024), (192, 640)]
    xs, ys = [], []
    for i, (r, c) in enumerate(shapes):
        full = rnd(r, c + 8 * (i % 2), dtype=torch.bfloat16, seed=40 + i).to(DEV)
        x = full[:, :c]
        ybuf = torch.full((c, r + 16 * (i % 2)), 7.0, dtype=torch.bfloat16, device=DEV)
        xs.append(x)
        ys.append(ybuf)
    K.transpose_bf16([(x, y[:, :x.shape[0]]) for x, y in zip(xs, ys)])
    torch.cuda.synchronize()
    for x, y in zip(xs, ys):
        r = x.shape[0]
        assert torch.equal(y[:, :r].cpu(), x.cpu().t()), x.shape
        assert (y[:, r:] == 7.0).all(), "wrote past rows"


def test_transpose_bf16_rejects_bad_shapes():
    x = torch.zeros(100, 128, dtype=torch.bfloat16, device=DEV)
    y = torch.empty(128, 100, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="multiples of 64"):
        K.transpose_bf16([(x, y)])
