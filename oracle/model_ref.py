"""Functional torch-CPU restatement of the reference Seq2Seq step (TEST INFRA ONLY).

Parameters are a plain ``{state_dict_key: tensor}`` mapping with the reference's
key names (``/root/reference/utils/model.py`` module tree), so the same dict
loads into the HIP model with ``load_state_dict(strict=True)``.

Pinned against the imported reference by ``tests/golden/make_goldens.py``
(fixtures ``tests/golden/*.npz``) and ``tests/test_oracle.py``.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

LN_EPS = 1e-5


# ----------------------------------------------------------------------------
# positional rotations
# ----------------------------------------------------------------------------
def rotation_tables(seq_len, dim):
    """cos/sin tables, float32, as reference model.py:36-42 / :67-73 build them.

    angle[t, i] = t * exp(-ln(10000) * (2i) / dim), computed in float32.
    """
    position = torch.arange(seq_len, dtype=torch.float32).unsqueeze(1)
    two_i = torch.arange(0, dim, 2, dtype=torch.float32)
    inv_freq = torch.exp(-torch.log(torch.tensor(10000.0)) * two_i / dim)
    angle = position * inv_freq
    return torch.cos(angle), torch.sin(angle)


def rotate_pairs(x, cos, sin):
    """Rotate interleaved pairs (2i, 2i+1) of the last dim (model.py:44-48, :75-79)."""
    xe = x[..., 0::2]
    xo = x[..., 1::2]
    cos = cos.to(x.device, x.dtype)
    sin = sin.to(x.device, x.dtype)
    out = torch.empty_like(x)
    out[..., 0::2] = xe * cos - xo * sin
    out[..., 1::2] = xe * sin + xo * cos
    return out


def global_pe(x):
    """GlobalPositionalEncoding(use_rope=True).forward, model.py:29-53. x [B,T,D]."""
    cos, sin = rotation_tables(x.shape[1], x.shape[2])
    return rotate_pairs(x, cos, sin)


def head_rope(q):
    """apply_rope_qk per tensor, model.py:60-83. q [B,H,T,dh]."""
    cos, sin = rotation_tables(q.shape[2], q.shape[3])
    return rotate_pairs(q, cos, sin)


# ----------------------------------------------------------------------------
# blocks
# ----------------------------------------------------------------------------
def linear(p, name, x):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def layer_norm(p, name, x):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], LN_EPS)


def attention(p, name, xq, xkv, num_heads, attn_dropout=0.0, training=False):
    """MultiHeadAttention.forward, model.py:110-141 (SDPA path, no mask)."""
    B, Tq, D = xq.shape
    Tk = xkv.shape[1]
    dh = D // num_heads
    q = linear(p, name + ".q_linear", xq).view(B, Tq, num_heads, dh).transpose(1, 2)
    k = linear(p, name + ".k_linear", xkv).view(B, Tk, num_heads, dh).transpose(1, 2)
    v = linear(p, name + ".v_linear", xkv).view(B, Tk, num_heads, dh).transpose(1, 2)
    q = head_rope(q)
    k = head_rope(k)
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(dh)
    a = torch.softmax(s, dim=-1)
    if training and attn_dropout > 0:
        a = F.dropout(a, attn_dropout, True)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, Tq, D)
    return linear(p, name + ".out_linear", o)


def ffn(p, name, x, dropout=0.0, training=False):
    """FeedForwardNetwork.forward, model.py:153-158."""
    h = F.relu(linear(p, name + ".linear1", x))
    h = F.dropout(h, dropout, training)
    return linear(p, name + ".linear2", h)


def encoder_layer(p, name, x, num_heads, dropout=0.0, training=False):
    """CustomTransformerEncoderLayer.forward (post-LN), model.py:173-181."""
    d = lambda t: F.dropout(t, dropout, training)
    a = d(attention(p, name + ".self_attn", x, x, num_heads, dropout, training))
    x = layer_norm(p, name + ".norm1", x + d(a))
    f = ffn(p, name + ".ffn", x, dropout, training)
    return layer_norm(p, name + ".norm2", x + d(f))


def decoder_layer(p, name, x, mem, num_heads, dropout=0.0, training=False):
    """CustomTransformerDecoderLayer.forward (post-LN), model.py:196-208."""
    d = lambda t: F.dropout(t, dropout, training)
    a = d(attention(p, name + ".self_attn", x, x, num_heads, dropout, training))
    x = layer_norm(p, name + ".norm1", x + d(a))
    c = d(attention(p, name + ".multihead_attn", x, mem, num_heads, dropout, training))
    x = layer_norm(p, name + ".norm2", x + d(c))
    f = ffn(p, name + ".ffn", x, dropout, training)
    return layer_norm(p, name + ".norm3", x + d(f))


def n_layers_of(p):
    n = 0
    while ("encoder.transformer_encoder.%d.norm1.weight" % n) in p:
        n += 1
    return n


def encoder_forward(p, src, num_heads, dropout=0.0, training=False):
    """Encoder.forward, model.py:223-230."""
    x = global_pe(linear(p, "encoder.embedding", src))
    for i in range(n_layers_of(p)):
        x = encoder_layer(p, "encoder.transformer_encoder.%d" % i, x, num_heads, dropout, training)
    return layer_norm(p, "encoder.layer_norm", x)


def decoder_forward(p, mem, num_heads, dropout=0.0, training=False):
    """Decoder.forward, model.py:245-251 (memory = un-rotated encoder output)."""
    x = global_pe(mem)
    for i in range(n_layers_of(p)):
        x = decoder_layer(p, "decoder.transformer_decoder.%d" % i, x, mem, num_heads, dropout, training)
    x = layer_norm(p, "decoder.layer_norm", x)
    return linear(p, "decoder.fc_output", x)


def seq2seq_forward(p, src, num_heads, dropout=0.0, training=False):
    """Seq2Seq.forward, model.py:263-266."""
    return decoder_forward(p, encoder_forward(p, src, num_heads, dropout, training),
                           num_heads, dropout, training)


# ----------------------------------------------------------------------------
# loss, clip, optimizer
# ----------------------------------------------------------------------------
def loss_fn(pred, trg, delta=1.0, w1=1.0, w2=1.0, w3=1.0):
    """Loss.forward, model.py:278-291: Huber(beta=delta) + L1 of first differences
    + (1 - mean directional cosine of first differences), eps 1e-8 on the norm."""
    rec = F.smooth_l1_loss(pred, trg, beta=delta)
    dp = pred[:, 1:] - pred[:, :-1]
    dt = trg[:, 1:] - trg[:, :-1]
    temp = F.l1_loss(dp, dt)
    pn = dp / (dp.norm(dim=-1, keepdim=True) + 1e-8)
    tn = dt / (dt.norm(dim=-1, keepdim=True) + 1e-8)
    cos = (pn * tn).sum(-1)
    return w1 * rec + w2 * temp + w3 * (1 - cos.mean())


def clip_grad_norm(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ semantics as used at training_utils.py:73:
    total = ||(||g_i||)_i||_2; coef = max_norm / (total + 1e-6) clamped to 1; g *= coef."""
    norms = torch.stack([g.norm(2) for g in grads])
    total = norms.norm(2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return total


def adam_l2_step(params, grads, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999,
                 eps=1e-8, weight_decay=0.0):
    """torch.optim.Adam (amsgrad=False) as built at model_utils.py:11: coupled L2
    (grad += wd * p), bias-corrected moments.  ``step`` is the post-increment count."""
    bc1 = 1 - beta1 ** step
    bc2_sqrt = math.sqrt(1 - beta2 ** step)
    step_size = lr / bc1
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        if weight_decay != 0:
            g = g.add(p, alpha=weight_decay)
        m.lerp_(g, 1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = (v.sqrt() / bc2_sqrt).add_(eps)
        p.addcdiv_(m, denom, value=-step_size)


def lr_lambda(epoch, warmup_epochs, n_epochs):
    """LambdaLR factor, model_utils.py:13-16."""
    if epoch < warmup_epochs:
        return float(epoch) / float(max(1, warmup_epochs))
    return max(0.0, float(n_epochs - epoch) / float(max(1, n_epochs - warmup_epochs)))


class OracleTrainer:
    """One reference training step (training_utils.py:56-80, use_amp=False path):
    zero_grad -> fwd -> Loss -> backward -> clip_grad_norm_(2.0) -> Adam.step."""

    def __init__(self, params, num_heads, lr=5e-5, weight_decay=1e-5, clip=2.0,
                 delta=1.0, w1=1.0, w2=1.0, w3=1.0, dropout=0.0, dtype=torch.float32):
        self.keys = list(params.keys())
        self.p = {k: v.detach().clone().to(dtype).requires_grad_(True) for k, v in params.items()}
        self.num_heads = num_heads
        self.lr, self.wd, self.clip = lr, weight_decay, clip
        self.loss_args = (delta, w1, w2, w3)
        self.dropout = dropout
        self.m = [torch.zeros_like(self.p[k]) for k in self.keys]
        self.v = [torch.zeros_like(self.p[k]) for k in self.keys]
        self.step_count = 0

    def step(self, src, trg):
        for k in self.keys:
            self.p[k].grad = None
        pred = seq2seq_forward(self.p, src, self.num_heads, self.dropout, self.dropout > 0)
        loss = loss_fn(pred, trg, *self.loss_args)
        loss.backward()
        grads = [self.p[k].grad for k in self.keys]
        self.last_grads = {k: self.p[k].grad.detach().clone() for k in self.keys}
        with torch.no_grad():
            total = clip_grad_norm(grads, self.clip)
            self.step_count += 1
            adam_l2_step([self.p[k] for k in self.keys], grads, self.m, self.v,
                         self.step_count, self.lr, weight_decay=self.wd)
        return loss.detach(), total, pred.detach()


# ----------------------------------------------------------------------------
# deterministic parameter sets (numpy Generator: version-stable across boxes)
# ----------------------------------------------------------------------------
def param_shapes(input_dim, hidden_dim, n_layers, output_dim, ffn_mult=4):
    """Ordered {key: shape} of the reference module tree (model.py:213-266),
    in registration order (= state_dict / parameters() order)."""
    D, Fd = hidden_dim, ffn_mult * hidden_dim
    shapes = {}

    def lin(name, o, i):
        shapes[name + ".weight"] = (o, i)
        shapes[name + ".bias"] = (o,)

    def ln(name):
        shapes[name + ".weight"] = (D,)
        shapes[name + ".bias"] = (D,)

    def mha(name):
        for s in ("q_linear", "k_linear", "v_linear", "out_linear"):
            lin(name + "." + s, D, D)

    lin("encoder.embedding", D, input_dim)
    for i in range(n_layers):
        b = "encoder.transformer_encoder.%d" % i
        mha(b + ".self_attn")
        lin(b + ".ffn.linear1", Fd, D)
        lin(b + ".ffn.linear2", D, Fd)
        ln(b + ".norm1")
        ln(b + ".norm2")
    ln("encoder.layer_norm")
    for i in range(n_layers):
        b = "decoder.transformer_decoder.%d" % i
        mha(b + ".self_attn")
        mha(b + ".multihead_attn")
        lin(b + ".ffn.linear1", Fd, D)
        lin(b + ".ffn.linear2", D, Fd)
        ln(b + ".norm1")
        ln(b + ".norm2")
        ln(b + ".norm3")
    lin("decoder.fc_output", output_dim, D)
    ln("decoder.layer_norm")
    return shapes


def seeded_params(shapes, seed, w_std=0.02, b_std=0.02, ln_std=0.1):
    """Linear weights N(0, w_std) (init_weights, training_utils.py:336-341) but with
    non-zero biases and perturbed LayerNorm affine so every parameter path is exercised."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in shapes.items():
        is_ln = ("norm" in k.split(".")[-2]) or k.split(".")[-2] == "layer_norm"
        if is_ln and k.endswith(".weight"):
            a = 1.0 + ln_std * rng.standard_normal(shp)
        elif is_ln:
            a = ln_std * rng.standard_normal(shp)
        elif k.endswith(".weight"):
            a = w_std * rng.standard_normal(shp)
        else:
            a = b_std * rng.standard_normal(shp)
        out[k] = torch.from_numpy(a.astype(np.float32))
    return out
