"""Drop-in for the reference's ``utils/model.py`` (/root/reference/utils/model.py).

Same classes, constructor signatures, module tree and therefore the same
``state_dict`` keys/shapes (344 tensors at the 228M config).  The compute does
NOT run module-by-module: ``Seq2Seq.forward`` / ``Encoder.forward`` /
``Decoder.forward`` dispatch the whole graph to the MI355X engine
(``neurosync_trainer_lite_amd/engine.py``) over libnstl_hip.so, and ``Loss`` to
the fused loss kernel.  There is no CPU path: on a non-CUDA tensor these raise.
"""
import weakref

import torch
import torch.nn as nn

from .. import _hip as K
from ..engine import Seq2SeqEngine, Seq2SeqFunction, rotation_tables


def _require_gpu(t, what):
    if not t.is_cuda:
        raise RuntimeError("%s runs only on the MI355X HIP path (got a %s tensor; there is no CPU fallback)"
                           % (what, t.device.type))


def _rope_apply(x, dim):
    """Rotate interleaved pairs of the last dim of x [..., T, dim] (position = dim -2)."""
    T = x.shape[-2]
    cs, sn = rotation_tables(T, dim, x.device)
    xc = x.contiguous()
    out = torch.empty_like(xc)
    rows = xc.numel() // dim
    K.rope(xc, dim, out, dim, rows, dim, cs, sn, T, dim)
    return out


def _owner_engine(module, device):
    ref = getattr(module, "_owner_ref", None)
    owner = ref() if ref is not None else None
    return owner.engine(device) if owner is not None else None


# -------------------------------------------------------------------------------------------
class GlobalPositionalEncoding(nn.Module):
    """model.py:13-53.  use_rope=True rotates pairs (2i, 2i+1) by t*10000^(-2i/d)."""

    def __init__(self, d_model, max_len=10000, use_global_positional_encoding=True, use_rope=True):
        super().__init__()
        self.use_global_positional_encoding = use_global_positional_encoding
        self.use_rope = use_rope
        self.d_model = d_model
        if use_global_positional_encoding and not use_rope:
            raise NotImplementedError("only the RoPE global encoding (the reference default) is implemented")

    def forward(self, x):
        if not self.use_global_positional_encoding:
            return x
        _require_gpu(x, "GlobalPositionalEncoding")
        if x.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("float32/bfloat16 expected")
        return _rope_apply(x, self.d_model)


def apply_rope_qk(q, k, use_local_positional_encoding=True):
    """model.py:60-83: per-head RoPE on q, k [B, H, T, dh]."""
    if not use_local_positional_encoding:
        return q, k
    _require_gpu(q, "apply_rope_qk")
    assert q.size(-1) % 2 == 0, "head_dim must be even for RoPE"
    return _rope_apply(q, q.size(-1)), _rope_apply(k, k.size(-1))


class MultiHeadAttention(nn.Module):
    """model.py:89-141 parameter container (q/k/v/out_linear).  Its math runs fused
    inside the engine (QKV GEMM + RoPE epilogue, nstl_attn_*, out GEMM)."""

    def __init__(self, hidden_dim, num_heads, dropout=0.0):
        super().__init__()
        assert hidden_dim % num_heads == 0, "Hidden dimension must be divisible by the number of heads"
        self.num_heads = num_heads
        self.head_dim = hidden_dim // num_heads
        self.scaling = self.head_dim ** -0.5
        self.q_linear = nn.Linear(hidden_dim, hidden_dim)
        self.k_linear = nn.Linear(hidden_dim, hidden_dim)
        self.v_linear = nn.Linear(hidden_dim, hidden_dim)
        self.out_linear = nn.Linear(hidden_dim, hidden_dim)
        self.attn_dropout = nn.Dropout(dropout)
        self.resid_dropout = nn.Dropout(dropout)
        self.dropout = dropout
        self.flash = True

    def forward(self, *a, **k):
        raise RuntimeError("MultiHeadAttention runs fused inside Seq2Seq/Encoder/Decoder on MI355X")


class FeedForwardNetwork(nn.Module):
    """model.py:146-158 parameter container (linear1 -> ReLU -> dropout -> linear2)."""

    def __init__(self, hidden_dim, dim_feedforward=2048, dropout=0.0):
        super().__init__()
        self.linear1 = nn.Linear(hidden_dim, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, hidden_dim)

    def forward(self, x):
        raise RuntimeError("FeedForwardNetwork runs fused inside Seq2Seq/Encoder/Decoder on MI355X")


class CustomTransformerEncoderLayer(nn.Module):
    """model.py:163-181 (post-LN encoder layer) parameter container."""

    def __init__(self, hidden_dim, num_heads, dropout=0.0):
        super().__init__()
        self.self_attn = MultiHeadAttention(hidden_dim, num_heads, dropout)
        self.ffn = FeedForwardNetwork(hidden_dim, 4 * hidden_dim, dropout)
        self.norm1 = nn.LayerNorm(hidden_dim)
        self.norm2 = nn.LayerNorm(hidden_dim)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)

    def forward(self, src, mask=None):
        raise RuntimeError("encoder layers run fused inside Encoder on MI355X")


class CustomTransformerDecoderLayer(nn.Module):
    """model.py:183-208 (post-LN decoder layer: self-attn, cross-attn, FFN)."""

    def __init__(self, hidden_dim, num_heads, dropout=0.0):
        super().__init__()
        self.self_attn = MultiHeadAttention(hidden_dim, num_heads, dropout)
        self.multihead_attn = MultiHeadAttention(hidden_dim, num_heads, dropout)
        self.ffn = FeedForwardNetwork(hidden_dim, 4 * hidden_dim, dropout)
        self.norm1 = nn.LayerNorm(hidden_dim)
        self.norm2 = nn.LayerNorm(hidden_dim)
        self.norm3 = nn.LayerNorm(hidden_dim)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.dropout3 = nn.Dropout(dropout)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None):
        raise RuntimeError("decoder layers run fused inside Decoder on MI355X")


class Encoder(nn.Module):
    """model.py:213-230."""

    def __init__(self, input_dim, hidden_dim, n_layers, num_heads, dropout=0.0, use_norm=True):
        super().__init__()
        if not use_norm:
            raise NotImplementedError("use_norm=False is not part of the reference configuration")
        self.embedding = nn.Linear(input_dim, hidden_dim)
        self.global_pos_encoder = GlobalPositionalEncoding(hidden_dim)
        self.transformer_encoder = nn.ModuleList(
            [CustomTransformerEncoderLayer(hidden_dim, num_heads, dropout) for _ in range(n_layers)])
        self.layer_norm = nn.LayerNorm(hidden_dim)

    def forward(self, x):
        """Inference-path encoder (audio_processing.py:28): returns f32 [B, T, D]."""
        _require_gpu(x, "Encoder")
        eng = _owner_engine(self, x.device)
        if eng is None:
            raise RuntimeError("Encoder must belong to a Seq2Seq to run")
        with torch.no_grad():
            eng._prologue(self.training)
            eng.base_seed = eng.draw_seed()
            B, T, _ = x.shape
            bb = eng.bufs(B, T, False)
            mem = eng.encode(bb, x, T)
            out = torch.empty(B * T, eng.D, dtype=torch.float32, device=x.device)
            K.cast(mem, out)
            return out.view(B, T, eng.D)


class Decoder(nn.Module):
    """model.py:235-251."""

    def __init__(self, output_dim, hidden_dim, n_layers, num_heads, dropout=0.0, use_norm=True):
        super().__init__()
        if not use_norm:
            raise NotImplementedError("use_norm=False is not part of the reference configuration")
        self.global_pos_encoder = GlobalPositionalEncoding(hidden_dim)
        self.transformer_decoder = nn.ModuleList(
            [CustomTransformerDecoderLayer(hidden_dim, num_heads, dropout) for _ in range(n_layers)])
        self.fc_output = nn.Linear(hidden_dim, output_dim)
        self.layer_norm = nn.LayerNorm(hidden_dim)

    def forward(self, encoder_outputs):
        """Inference-path decoder (audio_processing.py:29): f32 [B, T, out]."""
        _require_gpu(encoder_outputs, "Decoder")
        eng = _owner_engine(self, encoder_outputs.device)
        if eng is None:
            raise RuntimeError("Decoder must belong to a Seq2Seq to run")
        with torch.no_grad():
            eng._prologue(self.training)
            eng.base_seed = eng.draw_seed()
            B, T, D = encoder_outputs.shape
            bb = eng.bufs(B, T, False)
            mem = bb.mem
            e = encoder_outputs.reshape(B * T, D)
            K.copy2d(e, e.stride(0), mem, D, B * T, D, D)
            pred = eng.decode(bb, mem, T)
            return pred[:, :eng.out_dim].reshape(B, T, eng.out_dim)


class Seq2Seq(nn.Module):
    """model.py:256-266.  forward(src f32 [B,T,input_dim]) -> f32 [B,T,output_dim]."""

    def __init__(self, encoder, decoder, device):
        super().__init__()
        self.encoder = encoder
        self.decoder = decoder
        self.device = device
        # back-references as weakrefs (a Module attribute would register a submodule)
        object.__setattr__(encoder, "_owner_ref", weakref.ref(self))
        object.__setattr__(decoder, "_owner_ref", weakref.ref(self))
        self.compute_dtype = torch.bfloat16
        self.fp8 = False
        self.fp8_scope = "attn+enc_ffn1"
        self.dropout_p = encoder.transformer_encoder[0].ffn.dropout.p if len(encoder.transformer_encoder) else 0.0
        self._engine = None
        self._anchor = torch.zeros((), requires_grad=True)
        self._register_state_dict_hook(_compact_state_dict)

    def state_dict(self, *args, **kwargs):
        eng = self.__dict__.get("_engine")
        if eng is not None and eng.master_stale:
            raise RuntimeError("parameters are sharded across ranks (FusedAdam.shard): call "
                               "optimizer.consolidate() on every rank before state_dict()")
        return super().state_dict(*args, **kwargs)

    def engine(self, device=None):
        """The MI355X engine owning this model's parameter arena (built on first use)."""
        if self._engine is None:
            dev = torch.device(device) if device is not None else next(self.parameters()).device
            if dev.type != "cuda":
                raise RuntimeError("Seq2Seq runs only on the MI355X HIP path (device %s)" % dev)
            self._engine = Seq2SeqEngine(self, dev, self.compute_dtype)
            self._engine.set_fp8(self.fp8, self.fp8_scope)
        return self._engine

    def set_compute_dtype(self, dtype):
        """bf16 (default, mixed precision) or float32 (parity mode)."""
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("compute dtype must be bfloat16 or float32")
        if self._engine is not None and self._engine.dt != dtype:
            raise RuntimeError("set the compute dtype before the first forward")
        self.compute_dtype = dtype

    def set_fp8(self, on=True, scope=None):
        """BASELINE config C5: run projections' forward GEMMs on e4m3 operands
        with row-wise scales (bf16 compute dtype only).  scope: "attn+enc_ffn1"
        (default: every attention q/k/v projection and the encoder FFN linear1,
        within the 1e-3 forward-MSE gate) or "all" (every q/k/v and FFN GEMM)."""
        if on and self.compute_dtype != torch.bfloat16:
            raise ValueError("fp8 projections need the bf16 compute dtype (use_amp=True)")
        self.fp8 = bool(on)
        if scope is not None:
            self.fp8_scope = scope
        if self._engine is not None:
            self._engine.set_fp8(self.fp8, self.fp8_scope)

    def forward(self, src):
        _require_gpu(src, "Seq2Seq")
        if src.dtype != torch.float32:
            src = src.float()
        eng = self.engine(src.device)
        if torch.is_grad_enabled():
            return Seq2SeqFunction.apply(src, self._anchor, eng, self.training)
        return eng.forward(src, self.training, save=False).clone()


def _compact_state_dict(module, state_dict, prefix, local_metadata):
    # parameters are views into the flat arena; hand out compact copies so a saved
    # state_dict has the reference's per-tensor storage (and no arena padding)
    for k in list(state_dict.keys()):
        state_dict[k] = state_dict[k].clone()
    return state_dict


class _LossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, trg, delta, w1, w2, w3):
        B, T, F = pred.shape
        if pred.stride(2) != 1 or pred.stride(0) != T * pred.stride(1):
            pred = pred.contiguous()
        trg = trg.to(device=pred.device, dtype=torch.float32)
        if trg.stride(2) != 1 or trg.stride(0) != T * trg.stride(1):
            trg = trg.contiguous()
        dpred = torch.empty(B, T, F, dtype=torch.float32, device=pred.device)
        out = torch.empty(4, dtype=torch.float32, device=pred.device)
        partial = torch.empty(B, 4, dtype=torch.float32, device=pred.device)
        a = K.LossArgs()
        a.B, a.T, a.F = B, T, F
        a.pred, a.pred_ld = pred.data_ptr(), pred.stride(1)
        a.trg, a.trg_ld = trg.data_ptr(), trg.stride(1)
        a.delta, a.w1, a.w2, a.w3, a.grad_scale = delta, w1, w2, w3, 1.0
        a.dpred, a.dpred_dtype, a.dpred_ld = dpred.data_ptr(), K.F32, F
        a.partial, a.loss_out = partial.data_ptr(), out.data_ptr()
        K.loss_fwd_bwd(a)
        ctx.save_for_backward(dpred)
        ctx.parts = out
        return out[0]

    @staticmethod
    def backward(ctx, grad_out):
        (dpred,) = ctx.saved_tensors
        B, T, F = dpred.shape
        g = torch.empty_like(dpred)
        go = grad_out.reshape(1).to(torch.float32).contiguous()
        K.copy2d(dpred.view(B * T, F), F, g.view(B * T, F), F, B * T, F, F, scale=go)
        return g, None, None, None, None, None


class Loss(nn.Module):
    """model.py:268-291: w1*SmoothL1(beta=delta) + w2*L1(first differences)
    + w3*(1 - mean directional cosine of first differences), fused fwd+bwd."""

    def __init__(self, delta=1.0, w1=1.0, w2=1.0, w3=1.0):
        super().__init__()
        self.delta = delta
        self.w1 = w1
        self.w2 = w2
        self.w3 = w3

    def forward(self, predictions, targets, current_step=None, total_steps=None):
        _require_gpu(predictions, "Loss")
        if predictions.dtype != torch.float32:
            predictions = predictions.float()
        return _LossFunction.apply(predictions, targets, float(self.delta), float(self.w1), float(self.w2),
                                   float(self.w3))
