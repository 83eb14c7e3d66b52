"""CU-tolerant grids: the 4-wave GEMM on fewer workgroups than tiles per round.

A compute stream that cedes CUs (to RCCL's channels during backward) gets a
persistent grid of nstl_stream_cus() workgroups, 8 x the fewest CUs its mask
leaves on one XCD.  When that grid does not divide the tile count, the last
G + T % G tiles are dealt stream-K (csrc/gemm4.h StreamK): every workgroup a
contiguous, equal range of 256-deep K units, a split tile's two partials summed
by its second contributor.  NSTL_PERSIST_CUS caps the grid so the tail runs on
an unmasked stream too (NSTL_GEMM4_SK=1 turns the tail on: it is off by
default, measured slower than a partial round of whole tiles on most shapes,
DESIGN.md section 5).  Split tiles add two f32 partials (x + y, the same
whichever arrives last), so f32 outputs agree with the whole-tile run to f32
rounding and bf16 outputs to one rounding step in rare elements; both are held
to float64.
"""
import ctypes
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.engine import rotation_tables

DEV = "cuda:0"
bf = torch.bfloat16


def rnd(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).to(dtype).to(DEV)


def f64(t):
    return t.detach().double().cpu()


def rel_err(got, ref):
    got, ref = f64(got), f64(ref)
    return (got - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)


def sk_and_whole(monkeypatch, fn, cus):
    """fn() on a grid capped to `cus` workgroups (stream-K tail), then on the full grid."""
    monkeypatch.setenv("NSTL_GEMM4_SK", "1")
    monkeypatch.setenv("NSTL_PERSIST_CUS", str(cus))
    K.kernel_counts_reset()
    a = fn()
    torch.cuda.synchronize()
    c = K.kernel_counts()
    monkeypatch.delenv("NSTL_PERSIST_CUS")
    K.kernel_counts_reset()
    b = fn()
    torch.cuda.synchronize()
    c2 = K.kernel_counts()
    assert c2["gemm4"] == 1 and c2["gemm4_sk"] == 0, c2
    return a, b, c


def bf16_close(a, b):
    """bf16 outputs of f32 sums that differ only in the association of two partials."""
    d = (a.float() - b.float()).abs()
    frac = (d > 0).float().mean().item()
    assert frac < 1e-3, frac
    assert d.max().item() <= 2 ** -7 * b.float().abs().max().item()


# (M, N, K, grid): T = 128 tiles on 100 (one stream-K round), 1024 on 250 (three
# whole rounds, then 274 tiles over 250), 256 on 200 with the minimum K of 4 units
@pytest.mark.parametrize("M,N,Kd,cus", [(4096, 2048, 1024, 100), (16384, 4096, 1024, 250), (4096, 4096, 1024, 200)])
def test_stream_k_f32_out_vs_f64(monkeypatch, M, N, Kd, cus):
    dY, W = rnd(M, Kd, dtype=bf, seed=1), rnd(Kd, N, dtype=bf, scale=0.05, seed=2)

    def run():
        C = torch.full((M, N), float("nan"), dtype=torch.float32, device=DEV)
        K.gemm(dY, W, C, M, N, Kd, a_kmajor=True, b_kmajor=False, alpha=0.5)
        return C

    cs, cw, cnt = sk_and_whole(monkeypatch, run, cus)
    assert cnt["gemm4"] == 1 and cnt["gemm4_sk"] == 1, cnt
    assert not torch.isnan(cs).any()
    A64, B64 = f64(dY), f64(W)
    mag = A64.abs() @ B64.abs()
    ratio = ((f64(cs) - 0.5 * (A64 @ B64)).abs() / (0.5 * mag).clamp_min(1e-300)).max().item()
    print("stream-K f32 %dx%dx%d on %d: max |err| / sum|a b| = %.2e" % (M, N, Kd, cus, ratio))
    assert ratio <= 1e-5
    assert rel_err(cs, cw) < 1e-5


def test_stream_k_bias_bf16(monkeypatch):
    M, N, Kd = 4096, 4096, 2048
    X, W, b = rnd(M, Kd, dtype=bf, seed=3), rnd(N, Kd, dtype=bf, scale=0.05, seed=4), rnd(N, seed=5)

    def run():
        C = torch.empty(M, N, dtype=bf, device=DEV)
        K.gemm(X, W, C, M, N, Kd, epilogue=K.EPI_BIAS, bias=b)
        return C

    cs, cw, cnt = sk_and_whole(monkeypatch, run, 200)
    assert cnt["gemm4_sk"] == 1, cnt
    bf16_close(cs, cw)
    assert rel_err(cs, f64(X) @ f64(W).T + f64(b)) < 1e-2


def test_stream_k_relu_dropout_then_drelu(monkeypatch):
    """FFN1 forward (ReLU + dropout keep bits) and the FFN2 dX with dReLU + column sums."""
    M, N, Kd = 4096, 4096, 1024
    X, W1, b1 = rnd(M, Kd, dtype=bf, seed=6), rnd(N, Kd, dtype=bf, scale=0.05, seed=7), rnd(N, seed=8)
    fw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b1, p_drop=0.3, seed=9)
    words = K.gemm_relu_mask_words(X, W1, torch.empty(M, N, dtype=bf, device=DEV), M, N, Kd, **fw)

    def fwd():
        h = torch.empty(M, N, dtype=bf, device=DEV)
        m = torch.full((words,), -1, dtype=torch.int64, device=DEV)
        K.gemm(X, W1, h, M, N, Kd, relu_mask=m, **fw)
        return h, m

    (hs, ms), (hw, mw), cnt = sk_and_whole(monkeypatch, fwd, 200)
    assert cnt["gemm4_sk"] == 1, cnt
    bf16_close(hs, hw)
    # keep & positive bits: only where a stored value crossed zero by one rounding step
    diff_bits = sum(bin(int(x)).count("1") for x in (ms ^ mw).cpu().tolist() if x)
    assert diff_bits <= (hs != hw).sum().item(), diff_bits
    dY, W2 = rnd(M, 1024, dtype=bf, seed=10), rnd(1024, N, dtype=bf, scale=0.05, seed=11)
    bw = dict(a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=hw, ld_aux=N, p_drop=0.3, relu_mask=mw)
    rows = K.gemm_colsum_rows(dY, W2, hw, M, N, 1024, **bw)

    def bwd():
        d = torch.empty(M, N, dtype=bf, device=DEV)
        part = torch.empty(rows, N, dtype=torch.float32, device=DEV)
        K.gemm(dY, W2, d, M, N, 1024, colsum_part=part, **bw)
        return d, part

    (ds, ps), (dw, pw), cnt = sk_and_whole(monkeypatch, bwd, 200)
    assert cnt["gemm4_sk"] == 1, cnt
    bf16_close(ds, dw)
    assert rel_err(ps.sum(0), f64(ds).sum(0)) < 1e-5
    ref = (f64(dY) @ f64(W2)) * (f64(hw) > 0).double() / 0.7
    assert rel_err(ds, ref) < 1e-2


def test_stream_k_rope(monkeypatch):
    M, N, Kd, T = 4096, 3072, 1024, 128
    X, W, b = rnd(M, Kd, dtype=bf, seed=12), rnd(N, Kd, dtype=bf, scale=0.05, seed=13), rnd(N, seed=14)
    cs_, sn_ = rotation_tables(T, 64, DEV)

    def run():
        C = torch.empty(M, N, dtype=bf, device=DEV)
        K.gemm(X, W, C, M, N, Kd, epilogue=K.EPI_BIAS_ROPE, bias=b, rope=(cs_, sn_, T, 64), rope_cols=2048)
        return C

    cs, cw, cnt = sk_and_whole(monkeypatch, run, 150)
    assert cnt["gemm4_sk"] == 1, cnt
    bf16_close(cs, cw)


def test_stream_k_grouped_dw(monkeypatch):
    """One decoder layer's weight gradients (256 tiles, K = 4096 tokens) on 240
    workgroups: f64 bound per problem, sum-of-squares partials in total."""
    D, F, Mt = 1024, 4096, 4096
    shapes = [(D, F), (F, D), (D, D), (D, D), (2 * D, D), (D, D), (3 * D, D)]
    ins = [(rnd(Mt, n, dtype=bf, scale=0.1, seed=20 + i), rnd(Mt, k, dtype=bf, seed=40 + i))
           for i, (n, k) in enumerate(shapes)]
    nt = sum((n // 256) * (k // 256) for n, k in shapes)

    def run():
        probs, outs = [], []
        sq = torch.full((nt * 8,), float("nan"), dtype=torch.float32, device=DEV)
        used = 0
        for (dY, X), (n, k) in zip(ins, shapes):
            G = torch.full((n, k), float("nan"), dtype=torch.float32, device=DEV)
            t = (n // 256) * (k // 256) * 8
            probs.append((dY, X, G, n, k, Mt, dict(a_kmajor=False, b_kmajor=False, beta=0.0,
                                                    sq_part=sq[used:used + t])))
            used += t
            outs.append(G)
        K.gemm_grouped(probs)
        return outs, sq

    (os_, ss), (ow, sw), cnt = sk_and_whole(monkeypatch, run, 240)
    assert cnt["gemm4"] == 1 and cnt["gemm4_sk"] == 1 and cnt["gemm4_tiles"] == nt, cnt
    for G, Gw, (n, k), (dY, X) in zip(os_, ow, shapes, ins):
        A64, B64 = f64(dY).T, f64(X)
        ratio = ((f64(G) - A64 @ B64).abs() / (A64.abs() @ B64.abs()).clamp_min(1e-300)).max().item()
        print("stream-K grouped dW %dx%d: max |err| / sum|a b| = %.2e" % (n, k, ratio))
        assert ratio <= 1e-5
        assert rel_err(G, Gw) < 1e-5
    assert not torch.isnan(ss).any()
    tot = sum(float((g.double() ** 2).sum()) for g in os_)
    assert abs(float(ss.double().sum()) - tot) < 1e-5 * tot


def masked_stream(excluded):
    """A HIP stream of torch's runtime restricted to the CUs not in `excluded`."""
    hip = ctypes.CDLL(K.LIB_PATH)
    fn = hip.hipExtStreamCreateWithCUMask
    fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(n):
        if c not in excluded:
            mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    assert fn(ctypes.byref(st), words, mask) == 0
    return torch.cuda.ExternalStream(st.value, device=DEV), n


def test_masked_stream_grid_and_gemm(monkeypatch):
    """Mask bit i is a CU of XCD i % 8, shader engine (i / 8) % 4: a stream ceding
    one CU of every (XCD, SE) pair (bits 0..31) runs 32 fewer persistent
    workgroups, and so does one ceding a single CU (bit 0: that SE's share
    sets the grid); the GEMM on it takes the stream-K tail."""
    monkeypatch.setenv("NSTL_GEMM4_SK", "1")  # read per call; undone even when an assertion fails
    s1, n = masked_stream(set(range(32)))
    s2, _ = masked_stream({0})
    assert K.stream_cus(torch.cuda.current_stream().cuda_stream) == n
    assert K.stream_cus(s1.cuda_stream) == n - 32
    assert K.stream_cus(s2.cuda_stream) == n - 32
    M, N, Kd = 4096, 4096, 1024
    X, W = rnd(M, Kd, dtype=bf, seed=50), rnd(N, Kd, dtype=bf, scale=0.05, seed=51)
    C = torch.empty(M, N, dtype=torch.float32, device=DEV)
    torch.cuda.synchronize()
    K.kernel_counts_reset()
    with torch.cuda.stream(s1):
        K.gemm(X, W, C, M, N, Kd)
    s1.synchronize()
    c = K.kernel_counts()
    assert c["gemm4"] == 1 and c["gemm4_sk"] == 1, c
    assert rel_err(C, f64(X) @ f64(W).T) < 1e-5
