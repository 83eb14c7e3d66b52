"""The 4-wave persistent GEMM (csrc/gemm4.h) against the 8-wave ring kernel and
float64, through nstl_gemm / nstl_gemm_grouped.

Both kernels accumulate k in the same order (one 16x16x32 MFMA per 32-deep k
slice, slices in order), so their f32 accumulators agree bit for bit and every
epilogue that does the same elementwise math gives bit-identical bf16 outputs.
The ReLU keep bits must match word for word: the forward writes them in the
ring kernel's layout and the dReLU epilogue of either kernel (or the fp8 one)
reads them.  Column sums and sums of squares are formed in a different order
and are held to f32 rounding.  NSTL_GEMM4=0 (read per call) selects the ring
kernel for the reference run.
"""
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


def both(monkeypatch, fn):
    """fn() under the 4-wave kernel and under the ring kernel; the launch counts of
    the first run prove which kernel ran."""
    monkeypatch.setenv("NSTL_GEMM4", "1")
    K.kernel_counts_reset()
    a = fn()
    torch.cuda.synchronize()
    c = K.kernel_counts()
    monkeypatch.setenv("NSTL_GEMM4", "0")
    b = fn()
    torch.cuda.synchronize()
    monkeypatch.delenv("NSTL_GEMM4")
    return a, b, c


# shapes: one round of 256^2 tiles and several (the persistent tile loop and the
# cross-tile prefetch), K-major and MN-major B
SHAPES = [(1024, 1024, 256), (2048, 3072, 512), (8192, 2048, 384)]


@pytest.mark.parametrize("M,N,Kd", SHAPES)
@pytest.mark.parametrize("bkm", [True, False])
def test_gemm4_bias_matches_ring_bitwise(monkeypatch, M, N, Kd, bkm):
    X = rnd(M, Kd, dtype=bf, seed=1)
    W = rnd(N, Kd, dtype=bf, scale=0.05, seed=2) if bkm else rnd(Kd, N, dtype=bf, scale=0.05, seed=2)
    b = rnd(N, seed=3)

    def run():
        C = torch.empty(M, N, dtype=bf, device=DEV)
        K.gemm(X, W, C, M, N, Kd, a_kmajor=True, b_kmajor=bkm, epilogue=K.EPI_BIAS, bias=b)
        return C

    c4, cr, cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1 and cnt["gemm4_tiles"] == (M // 256) * (N // 256), cnt
    assert torch.equal(c4, cr)
    ref = (f64(X) @ (f64(W).T if bkm else f64(W))) + f64(b)
    assert rel_err(c4, ref) < 1e-2


@pytest.mark.parametrize("M,N,Kd", [(2048, 4096, 256), (8192, 1024, 512)])
def test_gemm4_relu_dropout_mask_matches_ring(monkeypatch, M, N, Kd):
    """ReLU + dropout: identical outputs and identical keep&positive words."""
    X, W, b = rnd(M, Kd, dtype=bf, seed=11), rnd(N, Kd, dtype=bf, scale=0.05, seed=12), rnd(N, seed=13)
    kw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=77)
    words = K.gemm_relu_mask_words(X, W, torch.empty(M, N, dtype=bf, device=DEV), M, N, Kd, **kw)
    assert words == (M // 64) * 8 * (N // 8)

    def run():
        C = torch.empty(M, N, dtype=bf, device=DEV)
        mask = torch.full((words,), -1, dtype=torch.int64, device=DEV)
        K.gemm(X, W, C, M, N, Kd, relu_mask=mask, **kw)
        return C, mask

    (c4, m4), (cr, mr), cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1, cnt
    assert torch.equal(c4, cr)
    assert torch.equal(m4, mr)


@pytest.mark.parametrize("M,N,Kd", [(2048, 1024, 512), (4096, 4096, 256)])
def test_gemm4_drelu_mask_colsum_matches_ring(monkeypatch, M, N, Kd):
    """dReLU from the keep bits (+ column sums of the stored dh): outputs bitwise,
    column sums to f32 rounding, both against each other and float64."""
    # keep bits from a forward of the same shape (written by the ring kernel)
    X, W1, b1 = rnd(M, 128, dtype=bf, seed=21), rnd(N, 128, dtype=bf, seed=22), rnd(N, seed=23)
    fw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b1, p_drop=0.3, seed=5)
    h = torch.empty(M, N, dtype=bf, device=DEV)
    words = K.gemm_relu_mask_words(X, W1, h, M, N, 128, **fw)
    mask = torch.zeros(words, dtype=torch.int64, device=DEV)
    K.gemm(X, W1, h, M, N, 128, relu_mask=mask, **fw)
    dY, W2 = rnd(M, Kd, dtype=bf, seed=24), rnd(Kd, N, dtype=bf, scale=0.05, seed=25)
    bw = dict(a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=0.3, relu_mask=mask)
    rows = K.gemm_colsum_rows(dY, W2, h, M, N, Kd, **bw)
    assert rows == M // 128

    def run():
        d = torch.empty(M, N, dtype=bf, device=DEV)
        part = torch.empty(rows, N, dtype=torch.float32, device=DEV)
        K.gemm(dY, W2, d, M, N, Kd, colsum_part=part, **bw)
        return d, part

    (d4, p4), (dr, pr), cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1, cnt
    assert torch.equal(d4, dr)
    assert rel_err(p4.sum(0), f64(d4).sum(0)) < 1e-5
    assert rel_err(p4, pr) < 1e-5
    ref = (f64(dY) @ f64(W2)) * (f64(h) > 0).double() / 0.7
    assert rel_err(d4, ref) < 1e-2


@pytest.mark.parametrize("T,rope_cols,dim", [(128, 2048, 64), (64, 1024, 64), (256, 1024, 32), (64, 960, 96),
                                               (128, 1024, 16)])
def test_gemm4_rope_matches_ring(monkeypatch, T, rope_cols, dim):
    """q|k|v + RoPE (the tables staged in LDS) against the ring kernel (which reads
    them from global memory) and float64.  Head dims below 64 and not a power of
    two (rows of fewer than 16 or of 24 table chunks) check that the LDS table's
    swizzle stays inside each row (with chunk ^ (t & 15) a 32-wide row
    wrote into the next row's slots)."""
    M, N, Kd = 4096, 3072, 256
    X, W, b = rnd(M, Kd, dtype=bf, seed=31), rnd(N, Kd, dtype=bf, scale=0.05, seed=32), rnd(N, seed=33)
    cs, sn = rotation_tables(T, dim, DEV)

    def run():
        C = torch.empty(M, N, dtype=bf, device=DEV)
        K.gemm(X, W, C, M, N, Kd, epilogue=K.EPI_BIAS_ROPE, bias=b, rope=(cs, sn, T, dim), rope_cols=rope_cols)
        return C

    c4, cr, cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1, cnt
    # the rotation's products are rounded separately here (no FMA contraction, as
    # the reference's f32 elementwise ops); the ring kernel contracts them: a few
    # outputs differ by one bf16 rounding step
    diff = (c4.float() - cr.float()).abs()
    assert (diff > 0).float().mean().item() < 2e-3
    assert diff.max().item() <= 2 ** -7 * cr.float().abs().max().item()
    # and the rotation itself against float64 (positions t = row % T, pairs of the head dim)
    z = f64(X) @ f64(W).T + f64(b)
    c64, s64 = f64(cs), f64(sn)
    t = torch.arange(M) % T
    zr = z.clone()
    for h0 in range(0, rope_cols, dim):
        e, o = z[:, h0:h0 + dim:2], z[:, h0 + 1:h0 + dim:2]
        zr[:, h0:h0 + dim:2] = e * c64[t] - o * s64[t]
        zr[:, h0 + 1:h0 + dim:2] = e * s64[t] + o * c64[t]
    assert rel_err(c4, zr) < 1e-2


@pytest.mark.parametrize("L,M", [(8, 2048), (3, 4096)])
def test_gemm4_grouped_rope_bit_identical_to_single(L, M):
    """The decoder's cross-attention k|v projections of all L layers as ONE grouped
    launch (gemm4_kernel<..., EM_ROPE, GROUPED>: shared A, per-problem B / C /
    bias, one RoPE table) give exactly the outputs of L single launches: the same
    tiles, the same k order and the same epilogue per element.  Also the engine's
    switch (NSTL_KV_GROUPED) and the argument check that the table is shared."""
    D, T, dim = 1024, 128, 64
    X = rnd(M, D, dtype=bf, seed=41)
    Ws = [rnd(2 * D, D, dtype=bf, scale=0.05, seed=42 + l) for l in range(L)]
    bs = [rnd(2 * D, seed=60 + l) for l in range(L)]
    cs, sn = rotation_tables(T, dim, DEV)
    kw = lambda l: dict(epilogue=K.EPI_BIAS_ROPE, bias=bs[l], rope=(cs, sn, T, dim), rope_cols=D)
    single = []
    for l in range(L):
        C = torch.empty(M, 2 * D, dtype=bf, device=DEV)
        K.gemm(X, Ws[l], C, M, 2 * D, D, **kw(l))
        single.append(C)
    grouped = [torch.full((M, 2 * D), float("nan"), dtype=bf, device=DEV) for _ in range(L)]
    K.kernel_counts_reset()
    K.gemm_grouped([(X, Ws[l], grouped[l], M, 2 * D, D, kw(l)) for l in range(L)])
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["gemm4"] == 1 and c["gemm4_tiles"] == L * (M // 256) * (2 * D // 256), c
    for l in range(L):
        assert torch.equal(grouped[l], single[l]), l
    cs2, sn2 = rotation_tables(T, dim, DEV)
    with pytest.raises(RuntimeError, match="share one table"):
        K.gemm_grouped([(X, Ws[0], grouped[0], M, 2 * D, D, kw(0)),
                        (X, Ws[1], grouped[1], M, 2 * D, D, dict(kw(1), rope=(cs2, sn2, T, dim)))])


def test_gemm4_odd_stage_count_stays_on_ring():
    """K % 128 != 0 (an odd number of 64-deep stages): the ring kernel runs it."""
    M, N, Kd = 2048, 1024, 320
    X, W = rnd(M, Kd, dtype=bf, seed=37), rnd(N, Kd, dtype=bf, scale=0.05, seed=38)
    C = torch.empty(M, N, dtype=bf, device=DEV)
    K.kernel_counts_reset()
    K.gemm(X, W, C, M, N, Kd)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["gemm4"] == 0 and c["gemm_ring"] == 1, c
    assert rel_err(C, f64(X) @ f64(W).T) < 1e-2


def test_gemm4_rope_table_past_lds_stays_on_ring(monkeypatch):
    """T * rope_dim * 4 > 32 KB (C5's T = 256): the ring kernel runs it."""
    M, N, Kd, T = 2048, 1024, 256, 256
    X, W, b = rnd(M, Kd, dtype=bf, seed=34), rnd(N, Kd, dtype=bf, scale=0.05, seed=35), rnd(N, seed=36)
    cs, sn = rotation_tables(T, 64, DEV)
    C = torch.empty(M, N, dtype=bf, device=DEV)
    K.kernel_counts_reset()
    K.gemm(X, W, C, M, N, Kd, epilogue=K.EPI_BIAS_ROPE, bias=b, rope=(cs, sn, T, 64), rope_cols=N)
    torch.cuda.synchronize()
    c = K.kernel_counts()
    assert c["gemm4"] == 0 and c["gemm_ring"] == 1, c


@pytest.mark.parametrize("Mt", [1024, 4096])
def test_gemm4_grouped_dw_sq_partials(monkeypatch, Mt):
    """Grouped weight gradients (NN, f32 out, beta 0): every problem bitwise against
    the ring kernel's grouped launch; the sum-of-squares partials (4 per tile here,
    8 there) agree in total."""
    shapes = [(1024, 512), (256, 1024), (512, 768), (768, 256)]
    ins = [(rnd(Mt, n, dtype=bf, seed=40 + i), rnd(Mt, k, dtype=bf, seed=50 + i)) for i, (n, k) in enumerate(shapes)]
    nt = sum((n // 256) * (k // 256) for n, k in shapes)

    def run():
        probs, outs = [], []
        sq = torch.full((nt * 8,), float("nan"), dtype=torch.float32, device=DEV)
        used = 0
        for (dY, X), (n, k) in zip(ins, shapes):
            G = torch.empty(n, k, dtype=torch.float32, device=DEV)
            t = (n // 256) * (k // 256) * 8
            probs.append((dY, X, G, n, k, Mt, dict(a_kmajor=False, b_kmajor=False, beta=0.0, sq_part=sq[used:used + t])))
            used += t
            outs.append(G)
        K.gemm_grouped(probs)
        return outs, sq

    (o4, s4), (orr, sr), cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1 and cnt["gemm_group"] == 0, cnt
    for a, b_, (n, k), (dY, X) in zip(o4, orr, shapes, ins):
        ref = f64(dY).T @ f64(X)
        e4, er = rel_err(a, ref), rel_err(b_, ref)
        print("grouped dW %dx%d: gemm4 %.2e ring %.2e vs f64, bitwise equal %s" % (n, k, e4, er, torch.equal(a, b_)))
        assert e4 < 1e-5 and er < 1e-5
    assert not torch.isnan(s4).any()
    tot = sum(float((g.double() ** 2).sum()) for g in o4)
    assert abs(float(s4.double().sum()) - tot) < 1e-5 * tot
    assert abs(float(s4.double().sum()) - float(sr.double().sum())) < 1e-5 * tot


def test_gemm4_f32_out_and_alpha(monkeypatch):
    """f32 output, alpha != 1, MN-major B (a dX into a fresh f32 buffer)."""
    M, N, Kd = 4096, 2048, 768
    dY, W = rnd(M, Kd, dtype=bf, seed=61), rnd(Kd, N, dtype=bf, scale=0.05, seed=62)

    def run():
        C = torch.empty(M, N, dtype=torch.float32, device=DEV)
        K.gemm(dY, W, C, M, N, Kd, a_kmajor=True, b_kmajor=False, alpha=0.5)
        return C

    c4, cr, cnt = both(monkeypatch, run)
    assert cnt["gemm4"] == 1, cnt
    assert torch.equal(c4, cr)
    assert rel_err(c4, 0.5 * f64(dY) @ f64(W)) < 2e-6


def test_gemm4_stress_many_rounds():
    """16 rounds of tiles per workgroup at the smallest K the kernel takes (nk = 4:
    the next tile's stages are staged from the tile's third step on), checked
    against float64 on every row."""
    M, N, Kd = 16384, 4096, 256
    X, W = rnd(M, Kd, dtype=bf, seed=71), rnd(N, Kd, dtype=bf, scale=0.05, seed=72)
    C = torch.empty(M, N, dtype=bf, device=DEV)
    K.kernel_counts_reset()
    K.gemm(X, W, C, M, N, Kd)
    torch.cuda.synchronize()
    assert K.kernel_counts()["gemm4"] == 1
    ref = (X.double() @ W.double().T)
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.parametrize("layout,M,N,Kd", [("tt", 4096, 2048, 2048), ("tn", 8192, 1024, 4096), ("nn", 1024, 2048, 8192),
                                           ("tt_drelu", 2048, 4096, 2048), ("tt_relu", 2048, 4096, 2048)])
def test_gemm4_r3_ring_bit_identical(monkeypatch, layout, M, N, Kd):
    """The 3 + 2 slot ring (R3, taken for K >= 2048: the stage DMA spread over both
    half-steps) accumulates in the same order as the two-stage ring: outputs,
    keep bits and column sums bit for bit (NSTL_GEMM4_R3=0 selects the two-stage
    ring, read per call)."""
    ak, bk = layout != "nn", layout in ("tt", "tt_relu")
    if layout == "nn":
        X, W = rnd(Kd, M, dtype=bf, seed=61), rnd(Kd, N, dtype=bf, scale=0.05, seed=62)
    else:
        X = rnd(M, Kd, dtype=bf, seed=61)
        W = rnd(N, Kd, dtype=bf, scale=0.05, seed=62) if bk else rnd(Kd, N, dtype=bf, scale=0.05, seed=62)
    b = rnd(N, seed=63)
    kw = dict(a_kmajor=ak, b_kmajor=bk)
    f32 = layout == "nn"
    if layout == "tt":
        kw.update(epilogue=K.EPI_BIAS, bias=b)
    if layout == "tt_relu":
        kw.update(epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=9)
    mask = None
    if layout == "tt_drelu":
        # keep bits from a forward of the same output shape
        X1, W1 = rnd(M, 256, dtype=bf, seed=64), rnd(N, 256, dtype=bf, seed=65)
        fw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=b, p_drop=0.3, seed=5)
        h = torch.empty(M, N, dtype=bf, device=DEV)
        mask = torch.zeros(K.gemm_relu_mask_words(X1, W1, h, M, N, 256, **fw), dtype=torch.int64, device=DEV)
        K.gemm(X1, W1, h, M, N, 256, relu_mask=mask, **fw)
        kw.update(a_kmajor=True, b_kmajor=False, epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=0.3,
                  relu_mask=mask)

    def run(r3):
        monkeypatch.setenv("NSTL_GEMM4_R3", r3)
        C = torch.full((M, N), float("nan"), dtype=torch.float32 if f32 else bf, device=DEV)
        extra = {}
        if layout == "tt_relu":
            extra["relu_mask"] = torch.full((K.gemm_relu_mask_words(X, W, C, M, N, Kd, **kw),), -1, dtype=torch.int64,
                                            device=DEV)
        if layout == "tt_drelu":
            extra["colsum_part"] = torch.full((K.gemm_colsum_rows(X, W, C, M, N, Kd, **kw), N), float("nan"),
                                              device=DEV)
        K.kernel_counts_reset()
        K.gemm(X, W, C, M, N, Kd, **kw, **extra)
        torch.cuda.synchronize()
        assert K.kernel_counts()["gemm4"] == 1
        return C, extra

    (c1, e1), (c0, e0) = run("1"), run("0")
    monkeypatch.delenv("NSTL_GEMM4_R3")
    assert torch.equal(c1, c0)
    for k in e1:
        assert torch.equal(e1[k], e0[k]), k
    ref = (f64(X).T if layout == "nn" else f64(X)) @ (f64(W).T if bk else f64(W))
    if layout == "nn":
        assert rel_err(c1, ref) < 1e-5
