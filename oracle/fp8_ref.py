"""CPU restatement of the fp8 operand path of BASELINE config C5 (fp8 QKV/FFN
projections) -- TEST INFRASTRUCTURE: only tests/, smoke() and bench.py's
checks import this module; the product path never does.

This is not in the reference: it computes every Linear under fp16 autocast
(utils/training_utils.py:64, torch.amp.autocast).  C5 asks for fp8 QKV/FFN
GEMMs, so this file pins the build's own scheme (include/nstl.h,
nstl_fp8_quant_rows and dtype NSTL_FP8 of nstl_gemm); how far an fp8 model's
output sits from the reference's is a tolerance (MSE) statement, measured by
tests/test_fp8_gpu.py and bench.py, not bit-exactness.

Scheme (row-wise scaling): row i of X gets amax_i = max_j |x_ij|,
s_i = amax_i / 448 (1 for an all-zero row), q_ij = e4m3fn(clamp(x_ij * (448 /
amax_i), -448, 448)) rounded to nearest even; an fp8 GEMM returns
s_a[i] s_b[j] sum_r qa[i][r] qb[j][r] (f32 accumulation).
"""
import torch

E4M3_MAX = 448.0


def quant_rows(x):
    """x: float tensor [rows, cols] (f32 or bf16) -> (q float8_e4m3fn, scale f32 [rows])."""
    x = x.float()
    amax = x.abs().amax(dim=1)
    pos = amax > 0
    one = torch.ones_like(amax)
    inv = torch.where(pos, torch.full_like(amax, E4M3_MAX) / torch.where(pos, amax, one), one)
    scale = torch.where(pos, amax / E4M3_MAX, one)
    q = (x * inv[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q, scale


def dequant(q, scale):
    return q.float() * scale[:, None]


def gemm(qa, sa, qb, sb):
    """s_a[i] s_b[j] sum_r qa[i][r] qb[j][r] in float64 (the products are exact)."""
    acc = qa.double() @ qb.double().T
    return acc * sa.double()[:, None] * sb.double()[None, :]


# ----------------------------------------------------------------------------
# C5 scope: which Linears run on fp8 operands (engine.Seq2SeqEngine.fp8_groups)
# ----------------------------------------------------------------------------
def scope_linears(scope, n_layers):
    """Module names (reference state_dict prefixes) of the Linears whose forward
    is fp8 under `scope` ("attn+enc_ffn1" or "all")."""
    out = []
    for l in range(n_layers):
        e = "encoder.transformer_encoder.%d." % l
        out += [e + "self_attn.q_linear", e + "self_attn.k_linear", e + "self_attn.v_linear", e + "ffn.linear1"]
        if scope == "all":
            out += [e + "ffn.linear2"]
        d = "decoder.transformer_decoder.%d." % l
        out += [d + "self_attn.q_linear", d + "self_attn.k_linear", d + "self_attn.v_linear",
                d + "multihead_attn.q_linear", d + "multihead_attn.k_linear", d + "multihead_attn.v_linear"]
        if scope == "all":
            out += [d + "ffn.linear1", d + "ffn.linear2"]
    return out


def simulated_forward(params, src, num_heads, scope):
    """The oracle forward (model_ref.seq2seq_forward, fp32) with the scope's
    Linears taking row-quantized e4m3 operands (quant_rows of the input rows and
    of the weight rows, products in f32): the fp8 model's error budget without
    its bf16 rounding elsewhere."""
    import torch.nn.functional as F
    from oracle import model_ref
    names = set(scope_linears(scope, model_ref.n_layers_of(params)))
    orig = model_ref.linear

    def q(x):
        qx, sx = quant_rows(x.reshape(-1, x.shape[-1]))
        return dequant(qx, sx).reshape(x.shape)

    def lin(p, name, x):
        if name in names:
            return F.linear(q(x), q(p[name + ".weight"]), p[name + ".bias"])
        return orig(p, name, x)

    model_ref.linear = lin
    try:
        return model_ref.seq2seq_forward(params, src, num_heads)
    finally:
        model_ref.linear = orig
