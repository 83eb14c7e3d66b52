"""fp8 operand path of BASELINE config C5 on the MI355X: row-wise e4m3
quantization (bit-exact against oracle/fp8_ref.py) and the fp8 GEMM
(v_mfma_scale_f32_32x32x64_f8f6f4 ring kernel) against the float64 product of
the same quantized operands, with each fused epilogue.

Tolerance of the GEMM: the e4m3 products are exact, but the scaled f8f6f4
MFMA does not accumulate its 64-product blocks as an exact f32 fma chain
(measured 1.9e-5 of max|C| at K = 1024), so 1e-4 relative to max|C| for f32
output and 1e-2 for bf16 output (8 mantissa bits); a layout or scaling error
is O(1)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from neurosync_trainer_lite_amd import _hip as K
    from neurosync_trainer_lite_amd.engine import rotation_tables

from oracle import fp8_ref

DEV = "cuda:0"


def rnd(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).to(dtype)


def quant_gpu(x):
    rows, cols = x.shape
    q = torch.empty(rows, cols, dtype=torch.float8_e4m3fn, device=DEV)
    s = torch.empty(rows, dtype=torch.float32, device=DEV)
    K.fp8_quant_rows([(x, rows, cols, q, s)])
    return q, s


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(300, 1024), (64, 4096), (5, 16)])
def test_quant_rows_bit_exact(dtype, rows, cols):
    x = rnd(rows, cols, dtype=dtype, seed=rows + cols)
    x[0] = 0                                   # all-zero row: scale 1, q 0
    if rows > 2:
        x[1] *= 1e-6                           # tiny row (subnormal e4m3 codes)
        x[2, : cols // 2] *= 1e4               # wide dynamic range inside one row
    q, s = quant_gpu(x.to(DEV))
    torch.cuda.synchronize()
    q_ref, s_ref = fp8_ref.quant_rows(x)
    assert torch.equal(s.cpu(), s_ref), "row scales differ"
    qb, qrb = q.cpu().view(torch.uint8), q_ref.view(torch.uint8)
    bad = (qb != qrb).nonzero()
    assert bad.numel() == 0, "%d codes differ, first at %s: %d vs %d" % (
        bad.shape[0], bad[0].tolist(), qb[tuple(bad[0])], qrb[tuple(bad[0])])


def test_quant_rows_batch_and_strides():
    xs = [rnd(256, 1088, dtype=torch.bfloat16, seed=s).to(DEV) for s in range(3)]
    jobs, outs = [], []
    for x in xs:
        q = torch.zeros(256, 1104, dtype=torch.float8_e4m3fn, device=DEV)  # ldq > cols
        s = torch.empty(256, dtype=torch.float32, device=DEV)
        jobs.append((x[:, :1024], 256, 1024, q, s))
        outs.append((q, s))
    K.fp8_quant_rows(jobs)
    torch.cuda.synchronize()
    for x, (q, s) in zip(xs, outs):
        q_ref, s_ref = fp8_ref.quant_rows(x[:, :1024].cpu())
        assert torch.equal(s.cpu(), s_ref)
        assert torch.equal(q[:, :1024].cpu().view(torch.uint8), q_ref.view(torch.uint8))
        assert (q[:, 1024:].cpu().view(torch.uint8) == 0).all(), "wrote past cols"


def fp8_operands(M, N, K_, seed):
    a = rnd(M, K_, dtype=torch.bfloat16, seed=seed).to(DEV)
    b = rnd(N, K_, dtype=torch.bfloat16, seed=seed + 1, scale=0.05).to(DEV)
    qa, sa = quant_gpu(a)
    qb, sb = quant_gpu(b)
    return qa, sa, qb, sb


def close(got, ref, rel, what):
    got, ref = got.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (got - ref).abs().max().item()
    assert err <= rel * scale, "%s: max err %.3e vs scale %.3e (rel %.1e)" % (what, err, scale, rel)


@pytest.mark.parametrize("M,N,K_", [(512, 768, 1024), (300, 256, 64), (512, 512, 128), (256, 512, 192),
                                    (1024, 1024, 4096), (257, 300, 256)])
def test_fp8_gemm_f32(M, N, K_):
    qa, sa, qb, sb = fp8_operands(M, N, K_, M + N + K_)
    c = torch.full((M, N), float("nan"), dtype=torch.float32, device=DEV)
    K.gemm(qa, qb, c, M, N, K_, a_scale=sa, b_scale=sb)
    torch.cuda.synchronize()
    close(c, fp8_ref.gemm(qa.cpu(), sa.cpu(), qb.cpu(), sb.cpu()), 1e-4, "fp8 gemm %dx%dx%d" % (M, N, K_))


@pytest.mark.parametrize("T", [128, 256])
def test_fp8_gemm_bias_relu_rope(T):
    """Bias, ReLU and RoPE epilogues of the fp8 GEMM against float64 of the same
    quantized operands; T = 256 is C5's long-clip position table (its RoPE GEMMs
    run on the fp8 kernel with the 256-position tables)."""
    M, N, K_ = 512, 1024, 1024
    qa, sa, qb, sb = fp8_operands(M, N, K_, 7)
    ref = fp8_ref.gemm(qa.cpu(), sa.cpu(), qb.cpu(), sb.cpu())
    bias = rnd(N, seed=3, scale=0.1).to(DEV)
    ref_b = ref + bias.double().cpu()
    c = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    K.gemm(qa, qb, c, M, N, K_, a_scale=sa, b_scale=sb, epilogue=K.EPI_BIAS, bias=bias)
    torch.cuda.synchronize()
    close(c, ref_b, 1e-2, "bias")
    K.gemm(qa, qb, c, M, N, K_, a_scale=sa, b_scale=sb, epilogue=K.EPI_BIAS_RELU_DROP, bias=bias, p_drop=0.0)
    torch.cuda.synchronize()
    close(c, ref_b.clamp_min(0), 1e-2, "bias+relu")
    # RoPE over the first 512 columns (dh 64), T positions
    dh = 64
    K.kernel_counts_reset()
    cos_t, sin_t = rotation_tables(T, dh, DEV)
    K.gemm(qa, qb, c, M, N, K_, a_scale=sa, b_scale=sb, epilogue=K.EPI_BIAS_ROPE, bias=bias,
           rope=(cos_t, sin_t, T, dh), rope_cols=512)
    torch.cuda.synchronize()
    c_ = K.kernel_counts()
    assert c_["gemm_fp8"] == 1 and c_["gemm_fp8_rope"] == 1, c_
    r = ref_b.clone()
    t = torch.arange(M) % T
    cs, sn = cos_t.double().cpu()[t], sin_t.double().cpu()[t]          # [M, dh/2]
    x = r[:, :512].view(M, 8, dh // 2, 2)
    x0, x1 = x[..., 0].clone(), x[..., 1].clone()
    x[..., 0] = x0 * cs[:, None, :] - x1 * sn[:, None, :]
    x[..., 1] = x0 * sn[:, None, :] + x1 * cs[:, None, :]
    close(c, r, 1e-2, "bias+rope")


def test_fp8_relu_dropout_keep_bits_match_bf16_kernel():
    """The fp8 ReLU-dropout epilogue draws the same keep pattern (seed, element)
    as the bf16 kernel: with every pre-activation positive, the keep&positive bit
    words of both kernels are identical (M = 2048: the bf16 ring kernel needs
    >= 32 tiles)."""
    M, N, K_ = 2048, 1024, 1024
    a = rnd(M, K_, dtype=torch.bfloat16, seed=11).to(DEV)
    b = rnd(N, K_, dtype=torch.bfloat16, seed=12, scale=0.01).to(DEV)
    bias = torch.full((N,), 50.0, device=DEV)
    qa, sa = quant_gpu(a)
    qb, sb = quant_gpu(b)
    c8 = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    c16 = torch.empty_like(c8)
    kw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=bias, p_drop=0.3, seed=1234)
    words = K.gemm_relu_mask_words(a, b, c16, M, N, K_, **kw)
    assert words > 0 and K.gemm_relu_mask_words(qa, qb, c8, M, N, K_, a_scale=sa, b_scale=sb, **kw) == words
    m8 = torch.zeros(words, dtype=torch.int64, device=DEV)
    m16 = torch.zeros_like(m8)
    K.gemm(qa, qb, c8, M, N, K_, a_scale=sa, b_scale=sb, relu_mask=m8, **kw)
    K.gemm(a, b, c16, M, N, K_, relu_mask=m16, **kw)
    torch.cuda.synchronize()
    assert torch.equal(m8, m16)
    assert torch.equal(c8 == 0, c16 == 0)
    keep = (c16 != 0).float().mean().item()
    assert 0.65 < keep < 0.75


def test_fp8_gemm_rejects_bad_layouts():
    qa, sa, qb, sb = fp8_operands(256, 256, 128, 1)
    c = torch.empty(256, 256, dtype=torch.float32, device=DEV)
    with pytest.raises(RuntimeError, match="K-major"):
        K.gemm(qa, qb, c, 256, 256, 128, a_scale=sa, b_scale=sb, a_kmajor=False, lda=256)
    with pytest.raises(RuntimeError, match="row scales"):
        K.gemm(qa, qb, c, 256, 256, 128, a_scale=sa)
    with pytest.raises(RuntimeError, match="K % 64"):
        K.gemm(qa[:, :96], qb[:, :96], c, 256, 256, 96, a_scale=sa, b_scale=sb, lda=128, ldb=128)


def test_fp8_228m_forward_within_metric_gate():
    """C5 at the 228M configuration (D=1024, H=16, L=8): the fp8 forward (default
    scope: attention projections + encoder FFN linear1) against the fp32 oracle
    on bench.py's parity batch (2 windows x 128 frames, seeded weights): MSE
    within the metric's 1e-3 gate, and the HIP path runs exactly the scope the
    oracle simulation (tests/test_fp8_cpu.py) decided; the relative RMS error
    stays under 5 % whatever the output scale."""
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model
    from oracle import model_ref
    D, H, L = 1024, 16, 8
    cfg = dict(training_config, hidden_dim=D, num_heads=H, n_layers=L, dropout=0.0, use_amp=True, use_fp8=True)
    model = build_model(cfg, DEV)
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), 11)
    model.load_state_dict(params, strict=True)
    src = torch.randn(2, 128, 256, generator=torch.Generator().manual_seed(12))
    model.eval()
    K.kernel_counts_reset()
    with torch.no_grad():
        p8 = model(src.to(DEV)).double().cpu()
    torch.cuda.synchronize()
    c = K.kernel_counts()
    eng = model.engine()
    got = set()
    for n, rows in eng.fp8_groups():  # fused q|k|v (rows 3) / cross k|v (rows 2): one GEMM, first name
        base = n.rsplit(".", 2)[0] + "."
        got |= {base + x for x in (("q_linear", "k_linear", "v_linear")[:rows] if rows == 3 else
                                   ("k_linear", "v_linear") if rows == 2 else (n.rsplit(".", 2)[1],))}
    assert got == set(fp8_ref.scope_linears("attn+enc_ffn1", L)), got ^ set(fp8_ref.scope_linears("attn+enc_ffn1", L))
    assert c["gemm_fp8"] == 5 * L, c  # per layer: enc q|k|v, ffn1; dec q|k|v, cross q, cross k|v
    ref = model_ref.seq2seq_forward(params, src, H).double()
    mse = ((p8 - ref) ** 2).mean().item()
    # the metric's gate is absolute; the relative RMS error keeps the check
    # independent of the output scale at this init (measured ~3.5 %)
    rel = (mse / (ref ** 2).mean().item()) ** 0.5
    print("C5 fp8 forward: mse %.3e, relative RMS error %.4f" % (mse, rel))
    assert mse < 1e-3, mse
    assert rel < 0.05, rel


def test_fp8_model_forward_and_step():
    """Whole small model in fp8 mode (C5, scope "all" to cover every fp8
    epilogue): the forward stays within a few percent of the fp32 oracle
    (relative L2 < 5e-2, a functional bound at this width; the metric gate is
    test_fp8_228m_forward_within_metric_gate), differs from bf16 mode (the fp8
    GEMMs ran), and a training step runs and re-quantizes the updated weights on
    the next forward."""
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    from oracle import model_ref
    D, H, L, B, T = 256, 4, 2, 4, 64
    cfg = dict(training_config, hidden_dim=D, num_heads=H, n_layers=L, dropout=0.0, use_amp=True, use_fp8=True,
               fp8_scope="all")
    model = build_model(cfg, DEV)
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), 21)
    model.load_state_dict(params, strict=True)
    g = torch.Generator().manual_seed(5)
    src = torch.randn(B, T, 256, generator=g)
    trg = torch.randn(B, T, 61, generator=g) * 20
    with torch.no_grad():
        ref = model_ref.seq2seq_forward(params, src, H).double()
        model.eval()
        p8 = model(src.to(DEV)).double().cpu()
        model.set_fp8(False)
        p16 = model(src.to(DEV)).double().cpu()
        model.set_fp8(True)
    rel8 = ((p8 - ref).norm() / ref.norm()).item()
    rel16 = ((p16 - ref).norm() / ref.norm()).item()
    assert rel8 < 5e-2, (rel8, rel16)
    assert not torch.equal(p8, p16)
    model.train()
    crit, opt, _ = prepare_training_components(cfg, model)
    losses = []
    for _ in range(2):
        opt.zero_grad()
        loss = crit(model(src.to(DEV)), trg.to(DEV))
        loss.backward()
        opt.step(max_norm=2.0)
        losses.append(loss.item())
    assert all(l == l for l in losses)
    eng = model.engine()
    q, sc = eng._fp8_w[("encoder.transformer_encoder.0.ffn.linear1.weight", 1)]
    w = eng.w("encoder.transformer_encoder.0.ffn.linear1.weight")
    q_ref, s_ref = fp8_ref.quant_rows(w.cpu())
    with torch.no_grad():
        model.eval()
        model(src.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(sc.cpu(), s_ref) and torch.equal(q.cpu().view(torch.uint8), q_ref.view(torch.uint8))


def test_ln_fwd_fused_fp8_copy_matches_standalone():
    """nstl_ln_fwd's optional q8 output is exactly nstl_fp8_quant_rows of its
    bf16 output (LayerNorm -> fp8 projection hand-off of config C5)."""
    rows, D = 300, 1024
    x = rnd(rows, D, dtype=torch.bfloat16, seed=1).to(DEV)
    y = rnd(rows, D, dtype=torch.bfloat16, seed=2).to(DEV)
    gamma = (1 + 0.1 * rnd(D, seed=3)).to(DEV)
    beta = (0.1 * rnd(D, seed=4)).to(DEV)
    out = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    q8 = torch.zeros(rows, D + 64, dtype=torch.float8_e4m3fn, device=DEV)
    s8 = torch.empty(rows, device=DEV)
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.BF16, rows, D
    a.x, a.y = x.data_ptr(), y.data_ptr()
    a.n_masks, a.p_drop, a.seed1, a.seed2 = 2, 0.3, 11, 12
    a.gamma, a.beta, a.eps = gamma.data_ptr(), beta.data_ptr(), 1e-5
    a.out, a.mean, a.rstd = out.data_ptr(), mean.data_ptr(), rstd.data_ptr()
    a.q8, a.ldq8, a.q8_scale = q8.data_ptr(), q8.stride(0), s8.data_ptr()
    K.ln_fwd(a)
    torch.cuda.synchronize()
    q_ref, s_ref = fp8_ref.quant_rows(out.cpu())
    assert torch.equal(s8.cpu(), s_ref)
    assert torch.equal(q8[:, :D].cpu().view(torch.uint8), q_ref.view(torch.uint8))


# ---------------------------------------------------------------- fp8 backward
# (C5: every FFN linear2 input-gradient GEMM dh = dReLU(dy W2) on e4m3 operands)

@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(1024, 4096), (4096, 1024), (64, 128)])
def test_quant_cols_bit_exact(dtype, rows, cols):
    """nstl_fp8_quant_cols(W) is exactly quant_rows(W^T): the e4m3 W^T operand and
    its per-input-channel scales, with an all-zero column and a tiny one."""
    x = rnd(rows, cols, dtype=dtype, seed=rows + 3 * cols, scale=0.05)
    x[:, 0] = 0
    x[:, 1] *= 1e-6
    x[: rows // 2, 2] *= 1e3
    xd = x.to(DEV)
    q = torch.zeros(cols, rows + 16, dtype=torch.float8_e4m3fn, device=DEV)  # ldq > rows
    s = torch.empty(cols, dtype=torch.float32, device=DEV)
    K.fp8_quant_cols([(xd, rows, cols, q, s)])
    torch.cuda.synchronize()
    q_ref, s_ref = fp8_ref.quant_rows(x.t().contiguous())
    assert torch.equal(s.cpu(), s_ref), "column scales differ"
    assert torch.equal(q[:, :rows].cpu().view(torch.uint8), q_ref.view(torch.uint8))
    assert (q[:, rows:].cpu().view(torch.uint8) == 0).all(), "wrote past rows"


def test_quant_cols_rejects_bad_shapes():
    x = torch.zeros(100, 128, dtype=torch.bfloat16, device=DEV)
    q = torch.empty(128, 112, dtype=torch.float8_e4m3fn, device=DEV)
    s = torch.empty(128, dtype=torch.float32, device=DEV)
    with pytest.raises(RuntimeError, match="multiples of 64"):
        K.fp8_quant_cols([(x, 100, 128, q, s)])


def test_ln_bwd_fused_fp8_copy_matches_standalone():
    """nstl_ln_bwd's optional q8 output is exactly nstl_fp8_quant_rows of the
    dbranch it stores (dropout applied, bf16-rounded): the LayerNorm backward ->
    fp8 FFN linear2 input-gradient hand-off."""
    rows, D = 512, 1024
    s_in = rnd(rows, D, dtype=torch.bfloat16, seed=21).to(DEV)
    dout = rnd(rows, D, seed=22).to(DEV)
    gamma = (1 + 0.1 * rnd(D, seed=23)).to(DEV)
    beta = (0.1 * rnd(D, seed=24)).to(DEV)
    mean = s_in.float().mean(1)
    rstd = torch.rsqrt(s_in.float().var(1, unbiased=False) + 1e-5)
    ds = torch.empty(rows, D, device=DEV)
    db = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
    n_part = 8
    parts = torch.empty(3, n_part, D, device=DEV)
    q8 = torch.zeros(rows, D, dtype=torch.float8_e4m3fn, device=DEV)
    s8 = torch.empty(rows, device=DEV)
    a = K.LnArgs()
    a.dtype, a.rows, a.D = K.BF16, rows, D
    a.n_masks, a.p_drop, a.seed1 = 1, 0.3, 77
    a.gamma, a.beta, a.eps = gamma.data_ptr(), beta.data_ptr(), 1e-5
    a.mean, a.rstd = mean.data_ptr(), rstd.data_ptr()
    a.s_in, a.dout, a.ds, a.dbranch = s_in.data_ptr(), dout.data_ptr(), ds.data_ptr(), db.data_ptr()
    a.dgamma_part, a.dbeta_part, a.n_part = parts[0].data_ptr(), parts[1].data_ptr(), n_part
    a.q8, a.ldq8, a.q8_scale = q8.data_ptr(), q8.stride(0), s8.data_ptr()
    K.ln_bwd(a)
    torch.cuda.synchronize()
    q_ref, s_ref = fp8_ref.quant_rows(db.cpu())
    assert torch.equal(s8.cpu(), s_ref)
    assert torch.equal(q8.cpu().view(torch.uint8), q_ref.view(torch.uint8))
    assert (db == 0).float().mean().item() > 0.25  # the dropout mask reached dbranch (and its copy)


def test_fp8_gemm_drelu_mask_and_colsum():
    """The fp8 dReLU epilogue (FFN linear2 input gradient, C5 backward): dh =
    keep&positive(h) * (s_dy[i] s_w[j] sum_r qdy[i][r] qwt[j][r]) / (1 - p), read from
    the forward's keep bits, plus the bias-gradient column-sum partials of the bf16
    values stored, against the float64 product of the same quantized operands."""
    M, N, K_ = 2048, 1024, 512       # dh [M, N] = dy [M, K_] W2 [K_, N]
    p = 0.3
    dy = rnd(M, K_, dtype=torch.bfloat16, seed=31).to(DEV)
    w2 = rnd(K_, N, dtype=torch.bfloat16, seed=32, scale=0.05).to(DEV)
    qdy, sdy = quant_gpu(dy)
    qwt = torch.empty(N, K_, dtype=torch.float8_e4m3fn, device=DEV)
    swt = torch.empty(N, dtype=torch.float32, device=DEV)
    K.fp8_quant_cols([(w2, K_, N, qwt, swt)])
    # the forward's keep&positive bits: an FFN1 forward (ReLU-dropout epilogue) of a random h
    x = rnd(M, 256, dtype=torch.bfloat16, seed=33).to(DEV)
    w1 = rnd(N, 256, dtype=torch.bfloat16, seed=34, scale=0.1).to(DEV)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    fkw = dict(epilogue=K.EPI_BIAS_RELU_DROP, bias=torch.zeros(N, device=DEV), p_drop=p, seed=99)
    words = K.gemm_relu_mask_words(x, w1, h, M, N, 256, **fkw)
    mask = torch.zeros(words, dtype=torch.int64, device=DEV)
    K.gemm(x, w1, h, M, N, 256, relu_mask=mask, **fkw)
    dh = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kw = dict(epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=p, a_scale=sdy, b_scale=swt)
    assert K.gemm_relu_mask_words(qdy, qwt, dh, M, N, K_, **kw) == words
    rows = K.gemm_colsum_rows(qdy, qwt, dh, M, N, K_, **kw)
    assert rows == M // 128
    part = torch.full((rows, N), float("nan"), device=DEV)
    K.gemm(qdy, qwt, dh, M, N, K_, relu_mask=mask, colsum_part=part, **kw)
    torch.cuda.synchronize()
    ref = fp8_ref.gemm(qdy.cpu(), sdy.cpu(), qwt.cpu(), swt.cpu())
    keep = (h.cpu() > 0).double()
    ref = ref * keep / (1 - p)
    close(dh, ref, 1e-2, "fp8 dReLU")
    assert torch.equal(dh.cpu() == 0, keep == 0) or ((dh.cpu() == 0) & (keep != 0)).float().mean() < 1e-4
    close(part.sum(0), dh.double().sum(0), 1e-5, "column sums of the stored dh")


def _grads(model, crit, src, trg):
    model.train()
    for p_ in model.parameters():
        p_.grad = None
    crit(model(src), trg).backward()
    torch.cuda.synchronize()
    return {n: p_.grad.detach().double().cpu().clone() for n, p_ in model.named_parameters()}


def test_fp8_backward_gradients_near_bf16_step():
    """fp8 backward (C5) at the 228M width (D=1024, H=16, L=2, B=16, T=128,
    dropout 0.3, same seed): every FFN linear2 input-gradient GEMM runs in fp8 (the
    launch counter sees them), and each parameter's gradient stays within 0.12
    relative (L2) of the same step with the bf16 backward -- the bf16 step's own
    distance from the fp32 oracle is ~0.1 at this width
    (tests/test_production_gpu.py), so e4m3 dh adds error of that order and no
    more; the global gradient norm agrees to 2 %."""
    from neurosync_trainer_lite_amd.config import training_config
    from neurosync_trainer_lite_amd.utils.model_utils import build_model, prepare_training_components
    from oracle import model_ref
    D, H, L, B, T = 1024, 16, 2, 16, 128
    cfg = dict(training_config, hidden_dim=D, num_heads=H, n_layers=L, dropout=0.3, use_amp=True, use_fp8=True)
    model = build_model(cfg, DEV)
    params = model_ref.seeded_params(model_ref.param_shapes(256, D, L, 61), 41)
    model.load_state_dict(params, strict=True)
    crit, _, _ = prepare_training_components(cfg, model)
    g = torch.Generator().manual_seed(42)
    src = torch.randn(B, T, 256, generator=g).to(DEV)
    trg = (torch.randn(B, T, 61, generator=g) * 20).to(DEV)
    torch.manual_seed(7)
    g16 = _grads(model, crit, src, trg)
    model.set_fp8(True, backward=True)
    torch.manual_seed(7)
    K.kernel_counts_reset()
    g8 = _grads(model, crit, src, trg)
    c = K.kernel_counts()
    assert c["gemm_fp8"] == 5 * L + 2 * L, c  # forward scope + one FFN linear2 dX per layer
    worst = []
    for n in g16:
        a, b = g8[n], g16[n]
        rel = ((a - b).norm() / (b.norm() + 1e-30)).item()
        worst.append((rel, n))
    worst.sort(reverse=True)
    print("fp8-backward vs bf16-backward, worst relative gradient differences:", worst[:6])
    assert worst[0][0] < 0.12, worst[:6]
    n8 = torch.sqrt(sum((v ** 2).sum() for v in g8.values())).item()
    n16 = torch.sqrt(sum((v ** 2).sum() for v in g16.values())).item()
    assert abs(n8 - n16) < 0.02 * n16, (n8, n16)


# ---------------------------------------------------------------------------
# the 4-wave persistent fp8 kernel (csrc/gemm4.h gemm4f8_kernel:
# v_mfma_scale_f32_16x16x128_f8f6f4, the bf16 kernel's 16 x 16 accumulator
# layout and epilogues with the row / column scales applied first) on full
# 256^2 tiles, K a multiple of 256 (>= 512); NSTL_GEMM4_F8=0 (read per call)
# selects the 8-wave fp8 ring kernel for comparison.
def _rope_ref(z, M, T, dh, cols, cs, sn):
    t = torch.arange(M) % T
    c64, s64 = cs.double().cpu()[t], sn.double().cpu()[t]
    r = z.clone()
    x = r[:, :cols].view(M, cols // dh, dh // 2, 2)
    x0, x1 = x[..., 0].clone(), x[..., 1].clone()
    x[..., 0] = x0 * c64[:, None, :] - x1 * s64[:, None, :]
    x[..., 1] = x0 * s64[:, None, :] + x1 * c64[:, None, :]
    return r


@pytest.mark.parametrize("epi,M,N,K_", [("bias", 2048, 1024, 1024), ("bias", 4096, 3072, 512),
                                         ("relu", 2048, 4096, 1024), ("rope128", 4096, 3072, 1024),
                                         ("rope256", 4096, 2048, 1024), ("drelu", 2048, 4096, 1024)])
def test_fp8_gemm4_epilogues_vs_f64_and_ring(monkeypatch, epi, M, N, K_):
    """Each epilogue of the fp8 4-wave kernel against float64 of the same e4m3
    operands and scales (bf16 output: 1e-2 of max|C|), and against the fp8 ring
    kernel (outputs within a bf16 step in rare elements: the two accumulate the
    128-byte blocks in different MFMA shapes).  rope256 is C5's T = 256 table,
    held in LDS as bf16 (f32 does not fit): rotation within 1e-2.  The keep bits
    of the ReLU-dropout epilogue and the dReLU column sums are compared with the
    ring kernel's."""
    qa, sa, qb, sb = fp8_operands(M, N, K_, M + N + K_)
    ref = fp8_ref.gemm(qa.cpu(), sa.cpu(), qb.cpu(), sb.cpu())
    bias = rnd(N, seed=3, scale=0.1).to(DEV)
    kw = dict(a_scale=sa, b_scale=sb)
    extra_ref = None
    if epi == "bias":
        kw.update(epilogue=K.EPI_BIAS, bias=bias)
        want = ref + bias.double().cpu()
    elif epi == "relu":
        kw.update(epilogue=K.EPI_BIAS_RELU_DROP, bias=bias, p_drop=0.0)
        want = (ref + bias.double().cpu()).clamp_min(0)
    elif epi.startswith("rope"):
        T = int(epi[4:])
        cs, sn = rotation_tables(T, 64, DEV)
        kw.update(epilogue=K.EPI_BIAS_ROPE, bias=bias, rope=(cs, sn, T, 64), rope_cols=N // 2)
        want = _rope_ref(ref + bias.double().cpu(), M, T, 64, N // 2, cs, sn)
    else:  # drelu: keep bits from an fp8 forward of the same output shape
        X1, W1 = rnd(M, 512, dtype=torch.bfloat16, seed=5).to(DEV), rnd(N, 512, dtype=torch.bfloat16, seed=6).to(DEV)
        qx, sx = quant_gpu(X1)
        qw, sw = quant_gpu(W1)
        h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        fw = dict(a_scale=sx, b_scale=sw, epilogue=K.EPI_BIAS_RELU_DROP, bias=bias, p_drop=0.3, seed=11)
        mask = torch.zeros(K.gemm_relu_mask_words(qx, qw, h, M, N, 512, **fw), dtype=torch.int64, device=DEV)
        K.gemm(qx, qw, h, M, N, 512, relu_mask=mask, **fw)
        kw.update(epilogue=K.EPI_DRELU_DROP, aux=h, ld_aux=N, p_drop=0.3, relu_mask=mask)
        want = ref * (h.double().cpu() > 0) / 0.7
        extra_ref = h

    def run(arm):
        monkeypatch.setenv("NSTL_GEMM4_F8", arm)
        c = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        extra = {}
        if epi == "relu":
            extra["relu_mask"] = torch.full((K.gemm_relu_mask_words(qa, qb, c, M, N, K_, **kw),), -1,
                                            dtype=torch.int64, device=DEV)
        if epi == "drelu":
            extra["colsum_part"] = torch.full((K.gemm_colsum_rows(qa, qb, c, M, N, K_, **kw), N), float("nan"),
                                              device=DEV)
        K.kernel_counts_reset()
        K.gemm(qa, qb, c, M, N, K_, **kw, **extra)
        torch.cuda.synchronize()
        return c, extra, K.kernel_counts()

    (c4, e4, n4), (cr, er, nr) = run("1"), run("0")
    monkeypatch.delenv("NSTL_GEMM4_F8")
    assert n4["gemm4_fp8"] == 1 and n4["gemm_fp8"] == 1, n4
    assert nr["gemm4_fp8"] == 0 and nr["gemm_fp8"] == 1, nr
    close(c4, want, 1e-2, "fp8 gemm4 " + epi)
    d = (c4.float() - cr.float()).abs()
    assert d.max().item() <= 2 ** -6 * cr.float().abs().max().item(), epi
    if epi == "relu":
        flips = torch.bitwise_xor(e4["relu_mask"], er["relu_mask"])
        nbits = sum(bin(int(x) & (2 ** 64 - 1)).count("1") for x in flips[flips != 0].tolist())
        assert nbits <= 1e-4 * 64 * flips.numel(), nbits
    if epi == "drelu":
        close(e4["colsum_part"].sum(0), c4.double().sum(0), 1e-4, "fp8 gemm4 dReLU column sums")
        assert extra_ref is not None
