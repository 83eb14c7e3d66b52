"""Seq2Seq training executor on MI355X: the reference forward/backward graph of
``utils/model.py`` (Seq2Seq, :256-266) scheduled explicitly over libnstl_hip.so.

Design (MI355X-first):
  * Parameter arena.  All 344 parameters live in ONE flat f32 buffer (plus a
    same-layout f32 gradient arena and, in bf16 mode, a bf16 shadow the GEMMs
    read).  nn.Parameters are views into it, so ``state_dict`` keys/shapes are
    the reference's, while q/k/v (and cross k/v) weights are contiguous and feed
    one fused projection GEMM.  Layout order = reverse backward order, so
    gradient buckets complete front-to-back (all-reduce overlap, parallel.py).
  * Activations are saved in preallocated per-(B, T) workspaces (288 GB HBM:
    ~8 GB at the 228M / 128x128 config); no allocator traffic in the step.
  * Fusions: bias+RoPE in the q/k projection epilogue, bias+ReLU+dropout in
    FFN1, dropout(s)+residual+LayerNorm in one kernel, ReLU/dropout backward in
    the FFN2 dX epilogue, RoPE backward in the attention-backward store.
  * Dropout masks are counter hashes (seed, element) regenerated in backward.
"""
import os
import weakref

import torch

from . import _hip as K

# per-layer dropout sites (distinct hash streams)
_SITE = {"attn": 1, "resid": 2, "drop1": 3, "ffn": 4, "drop2": 5,
         "xattn": 6, "xresid": 7, "drop2x": 8, "drop3": 9}


def _seed(base, enc, layer, site):
    return (base * 0x9E3779B1 + (0 if enc else 1 << 20) + layer * 64 + _SITE[site]) & 0xFFFFFFFFFFFFFFFF


def rotation_tables(seq_len, dim, device):
    """cos/sin [T, dim/2] f32, computed exactly as the reference does (model.py:36-42,
    :67-73: float32 position * exp(-ln(10000) * 2i / dim)) then moved to the device."""
    position = torch.arange(seq_len, dtype=torch.float32).unsqueeze(1)
    two_i = torch.arange(0, dim, 2, dtype=torch.float32)
    inv_freq = torch.exp(-torch.log(torch.tensor(10000.0)) * two_i / dim)
    angle = position * inv_freq
    return torch.cos(angle).contiguous().to(device), torch.sin(angle).contiguous().to(device)


def _span(t):
    """Byte range [lo, hi) a (possibly strided 2-D) view covers."""
    lo = t.data_ptr()
    n = 1 + sum((d - 1) * st for d, st in zip(t.shape, t.stride())) if t.numel() else 0
    return lo, lo + n * t.element_size()


ARENA_ALIGN = 64 * 840
# encoder layers whose weight gradients share one grouped GEMM: 4 x 192 tiles of
# 256^2 = 768 = three full rounds on 256 CUs (one layer alone: 0.75 of a round)
ENC_GROUP = 4
# the 4-wave GEMM's RoPE table budget in LDS (csrc/gemm4.h ROPE_LDS): T * rope_dim * 4 bytes
ROPE_LDS_BYTES = 32768


def _pad64(n):
    return (n + 63) // 64 * 64


_UNBOUND = object()  # Seq2SeqEngine.ensure_bound: no p.grad seen yet

class _Buffers:
    """Activation workspace for one (B, T, save) shape."""

    def __init__(self, eng, B, T, save):
        dev, dt = eng.device, eng.dt
        D, Fd, L = eng.D, eng.Fd, eng.L
        M = B * T
        nl = L if save else 1
        e = lambda *s, dtype=dt: torch.empty(*s, dtype=dtype, device=dev)
        self.B, self.T, self.M = B, T, M
        self.src = e(M, eng.in_dim)
        self.x0 = e(M, D)
        # encoder
        self.e_qkv = [e(M, 3 * D) for _ in range(nl)]
        self.e_o = [e(M, D) for _ in range(nl)]
        self.e_lse = [e(B * eng.H * T, dtype=torch.float32) for _ in range(nl)]
        self.e_s1 = [e(M, D) for _ in range(nl)]
        self.e_x1 = [e(M, D) for _ in range(nl)]
        self.e_h = [e(M, Fd) for _ in range(nl)]
        self.e_s2 = [e(M, D) for _ in range(nl)]
        self.e_x2 = [e(M, D) for _ in range(nl)]
        self.e_stats = [e(4, M, dtype=torch.float32) for _ in range(nl)]  # mean1 rstd1 mean2 rstd2
        self.mem = e(M, D)
        self.xdec0 = e(M, D)
        self.encf_stats = e(2, M, dtype=torch.float32)
        # decoder
        self.d_qkv = [e(M, 3 * D) for _ in range(nl)]
        self.d_o = [e(M, D) for _ in range(nl)]
        self.d_lse = [e(B * eng.H * T, dtype=torch.float32) for _ in range(nl)]
        self.d_s1 = [e(M, D) for _ in range(nl)]
        self.d_x1 = [e(M, D) for _ in range(nl)]
        self.d_qc = [e(M, D) for _ in range(nl)]
        self.d_kvc = [e(M, 2 * D) for _ in range(nl)]
        self.d_oc = [e(M, D) for _ in range(nl)]
        self.d_lsec = [e(B * eng.H * T, dtype=torch.float32) for _ in range(nl)]
        self.d_s2 = [e(M, D) for _ in range(nl)]
        self.d_x2 = [e(M, D) for _ in range(nl)]
        self.d_h = [e(M, Fd) for _ in range(nl)]
        self.d_s3 = [e(M, D) for _ in range(nl)]
        self.d_x3 = [e(M, D) for _ in range(nl)]
        self.d_stats = [e(6, M, dtype=torch.float32) for _ in range(nl)]
        self.xf = e(M, D)
        self.decf_stats = e(2, M, dtype=torch.float32)
        self.y = e(M, D)  # branch scratch (out_linear / FFN2 outputs)
        self.save = save
        if save:
            f32 = torch.float32
            self.dres = e(M, D, dtype=f32)
            self.dmem = e(M, D, dtype=f32)
            self.dy = e(M, D)
            self.dy_f, self.dy_x = e(M, D), e(M, D)  # decoder: dy of FFN2 / cross out_linear (grouped dW)
            # encoder: per-layer dy / dh / dqkv for ENC_GROUP layers whose weight
            # gradients are one grouped launch (slot = layer % ENC_GROUP)
            G = min(ENC_GROUP, L)
            self.g_dyf = [e(M, D) for _ in range(G)]
            self.g_dyo = [e(M, D) for _ in range(G)]
            self.g_dh = [e(M, Fd) for _ in range(G)]
            self.g_dqkv = [e(M, 3 * D) for _ in range(G)]
            self.dadd = e(M, D)  # a Linear's input gradient (dtype), added by the next LN backward
            self.dattn = e(M, D)
            self.dqkv = e(M, 3 * D)
            self.dq = e(M, D)
            # cross-attention k|v gradients: with Engine.dmem_concat every decoder
            # layer's side by side (the memory gradient is then ONE GEMM over
            # K = L * 2D), else one layer's.  Only the active mode's buffer exists
            # (dkv_all is 512 MB at the 228M shape); kv_grad() allocates on a switch.
            self.dkv = None if eng.dmem_concat else e(M, 2 * D)
            self.dkv_all = e(M, nl * 2 * D) if eng.dmem_concat else None
            self.dh = e(M, Fd)
            self.demb = e(M, D)
            self.dpred = torch.zeros(M, 64, dtype=dt, device=dev)
            self.dsum = e(B * eng.H * T, dtype=f32)  # attention backward rowsum(dO * O)
            # attention backward: per-(batch, 128 rows) column sums of dq | dk | dv (bias grads)
            # (two: a decoder layer's cross and self attention reduce in one batch)
            self.abias_slots = [e(B * ((T + 127) // 128), 3 * D, dtype=f32) for _ in range(2)]
            self.abias = self.abias_slots[0]
            # FFN2 dX (dReLU epilogue): per-128-row column sums of dh (FFN1 bias grad)
            self.hpart = e((M + 127) // 128, Fd, dtype=f32)
            # FFN hidden keep&positive bits (FFN1 epilogue -> FFN2 dX epilogue), 1 bit/element
            nmw = ((M + 63) // 64) * 8 * ((Fd + 7) // 8)
            self.e_rmask = [e(nmw, dtype=torch.int64) for _ in range(L)]
            self.d_rmask = [e(nmw, dtype=torch.int64) for _ in range(L)]
            self.e_rmask_ok = [False] * L
            self.d_rmask_ok = [False] * L
            # attention dropout keep bits, written by the forward, read by the backward
            nw = max(1, B * eng.H * T * T // 64)
            self.e_mask = [e(nw, dtype=torch.int64) for _ in range(L)]
            self.d_mask = [e(nw, dtype=torch.int64) for _ in range(L)]
            self.d_maskc = [e(nw, dtype=torch.int64) for _ in range(L)]
            # LN backward blocks (8 waves each, >= 1 row per wave); NSTL_LN_PARTS: A/B only
            self.n_part = max(1, min(int(os.environ.get("NSTL_LN_PARTS", "256")), M // 8))
            # one per LayerNorm of a layer (3 in a decoder layer): batched reduction
            self.ln_parts = [e(3, self.n_part, D, dtype=f32) for _ in range(3)]
            self.ln_part = self.ln_parts[0]
            self.col_part = e((M + 255) // 256, max(Fd, 3 * D, 64), dtype=f32)
            self.ws = e(eng.splitk_ws_elems(M), dtype=f32)

    def layer(self, lst, l):
        return lst[l if self.save else 0]

    def kv_grad(self, eng, l):
        """Decoder layer l's cross-attention k|v gradient buffer [M, 2D]."""
        D = eng.D
        if eng.dmem_concat:
            if self.dkv_all is None:
                self.dkv_all = torch.empty(self.M, eng.L * 2 * D, dtype=eng.dt, device=eng.device)
            return self.dkv_all[:, 2 * D * l:2 * D * (l + 1)]
        if self.dkv is None:
            self.dkv = torch.empty(self.M, 2 * D, dtype=eng.dt, device=eng.device)
        return self.dkv


class Seq2SeqEngine:
    """Owns the parameter/gradient arenas of one Seq2Seq module and runs it."""

    def __init__(self, model, device, compute_dtype):
        self.model = model
        self.device = torch.device(device)
        self.dt = compute_dtype
        enc, dec = model.encoder, model.decoder
        self.D = enc.embedding.out_features
        self.in_dim = enc.embedding.in_features
        self.out_dim = dec.fc_output.out_features
        self.L = len(enc.transformer_encoder)
        self.H = enc.transformer_encoder[0].self_attn.num_heads
        self.dh = self.D // self.H
        self.Fd = enc.transformer_encoder[0].ffn.linear1.out_features
        self.dropout = model.dropout_p
        self._wpending = []        # (lo, hi, event): queued optimizer updates of arena ranges (queue_update)
        self._upd_ranges = None    # [(stage key, (lo, hi))]: the update order of queue_update
        self._check_shapes()
        self._build_arena()
        self._bufs = {}
        self._rope = {}
        self.generation = 0
        self.grads_fresh = True
        self.grad_reducer = None   # parallel.GradAllReducer when data-parallel
        self.grad_scale_t = None   # device f32 [1]: loss-gradient pre-scale (1/world)
        self.seed_salt = 0         # data-parallel rank: distinct dropout streams per replica
        # NSTL_DW_STREAM=1: weight-gradient GEMMs run on a second HIP stream beside
        # the dX chain.  Off by default: +0.5 % step rate at the 228M config (424.3k
        # vs 422.3k frames/s), while the per-launch GEMM timing then overlaps.
        self.dw_stream_on = os.environ.get("NSTL_DW_STREAM", "0") == "1"
        self._side = None          # torch.cuda.Stream for dW (+ bias colsum)
        self._side_reads = []      # (lo, hi, event): bytes a queued dW still reads
        # NSTL_DW_GROUP=0: one GEMM per weight gradient (split-K) instead of one
        # grouped launch per decoder layer (its 7 weight gradients are 256 tiles)
        # and per ENC_GROUP encoder layers (4 x 4 weight gradients, 768 tiles)
        self.dw_group_on = os.environ.get("NSTL_DW_GROUP", "1") != "0"
        self._defer = None         # weight-gradient jobs of the current decoder layer
        # NSTL_FUSED_BIAS=0: q/k/v and FFN1 bias gradients by colsum() instead of
        # the attention-backward / dReLU-epilogue column sums
        self.fused_bias_on = os.environ.get("NSTL_FUSED_BIAS", "1") != "0"
        # NSTL_RES_HANDOFF=0: input gradients of the Linears fed by a LayerNorm are
        # accumulated into the f32 residual gradient by the GEMM (read-modify-write)
        # instead of being written in the compute dtype and added by the next LN backward
        self.res_handoff_on = os.environ.get("NSTL_RES_HANDOFF", "1") != "0"
        self._dadd_pending = False
        # NSTL_DMEM_CONCAT=0: the memory gradient accumulated into the f32 dmem by one
        # K = 2D GEMM per decoder layer instead of one K = L * 2D GEMM after the decoder
        self.dmem_concat = os.environ.get("NSTL_DMEM_CONCAT", "1") != "0"
        self._wkv = None           # [W_kv_0; ...; W_kv_{L-1}] slab (_kv_weights)
        self._kv_all_done = False  # decode(): every layer's cross k|v projected in one launch
        # NSTL_RELU_MASK=0: the FFN2 dX epilogue reads the saved hidden h for its
        # dReLU instead of the 1-bit keep&positive mask the FFN1 epilogue writes
        self.relu_mask_on = os.environ.get("NSTL_RELU_MASK", "1") != "0"
        # NSTL_REDUCE_BATCH=0: each LayerNorm / bias-gradient partial reduction is
        # its own launch instead of one batched launch per backward layer
        self.reduce_batch_on = os.environ.get("NSTL_REDUCE_BATCH", "1") != "0"
        # BASELINE config C5: the q/k/v and FFN projections' forward GEMMs take e4m3
        # operands with row-wise scales (oracle/fp8_ref.py; Seq2Seq.set_fp8 or the
        # config key 'use_fp8').  Backward keeps the bf16 weights and activations.
        self.fp8 = False
        self.fp8_scope = "attn+enc_ffn1"
        self._fp8_w = None         # (weight name, rows) -> (e4m3 [rows*N, K], f32 scales [rows*N])
        self._fp8_act = {}         # M -> (e4m3 scratch [M, max(D, Fd)], scales [M], e4m3 mem, mem scales)
        self._xq = {}              # data_ptr of an activation -> its live e4m3 copy (q, scales)
        # fp8 backward (C5, set_fp8(..., backward=True) / config key 'fp8_backward'):
        # the FFN linear2 input gradient dh = dy W2 (dReLU epilogue) on e4m3 operands
        # -- dy row-quantized by the LayerNorm backward that writes it, W2^T
        # column-quantized once per forward.  Every other backward GEMM stays bf16.
        self.fp8_bwd = False
        self._fp8_wt = None        # weight name -> (e4m3 W^T [in, out], f32 scales [in])
        self._fp8_wt_fresh = False  # did the current forward quantize _fp8_wt
        self._fp8_dy = {}          # M -> (e4m3 [M, D], scales [M])
        # NSTL_WT=1: the input-gradient GEMMs (dX = dY W) read a transposed bf16 copy
        # W^T [in, out] (K-major, the layout both the ring kernel and hipBLASLt run
        # fastest), refreshed by one batched transpose at the start of every backward,
        # instead of W in place as an MN-major operand.  Off: the GEMMs gain what the
        # transpose costs (587.3k vs 587.4k frames/s same-box, profiles/r3_wt_ab.txt)
        self.wt_on = os.environ.get("NSTL_WT", "0") == "1"
        self._wt = None            # (weight name, rows) -> bf16 W^T [in, rows * out]
        self._wt_ok = False        # _wt holds this backward's weights
        # NSTL_FUSED_NORM=0: the clip norm re-reads the whole gradient arena
        # (nstl_sumsq) instead of taking the grouped weight-gradient GEMMs' per-tile
        # sums of squares (their epilogue, nstl_gemm_args.sq_part) plus nstl_sumsq
        # over the rest of the arena (head, embedding, vectors: ~0.3 % of it)
        self.fused_norm_on = os.environ.get("NSTL_FUSED_NORM", "1") != "0"
        self._sq_buf = None        # f32 [tiles * 8] partials of the grouped dW launches
        self._sq_used = 0
        self._sq_ok = False
        self.sq_state = None       # (g32._version, partial count) after a backward that produced them
        self.sq_rest_partials = 64  # nstl_sumsq partials per norm_rest range (FusedAdam.step)
        self._red = None           # pending (part, ld, n_part, cols, out, beta) jobs
        self._ln_slot = 0          # next LayerNorm partial buffer of the layer
        self._ab_slot = 0          # next attention bias partial buffer of the layer

    # ------------------------------------------------------------------ setup
    def _check_shapes(self):
        D, H = self.D, self.H
        if D % H or (D // H) % 8 or D // H > 512:
            raise ValueError("head_dim must be a multiple of 8 up to 512 (hidden_dim=%d, num_heads=%d)" % (D, H))
        if D % 128 or D > 1024:
            raise ValueError("hidden_dim must be a multiple of 128 and <= 1024 (got %d)" % D)
        if self.out_dim > 64:
            raise ValueError("output_dim must be <= 64 (got %d)" % self.out_dim)
        if self.in_dim % 8:
            raise ValueError("input_dim must be a multiple of 8 (got %d)" % self.in_dim)

    def _arena_order(self):
        """Parameter names in arena order (reverse of backward completion)."""
        L = self.L
        order = ["decoder.fc_output.weight", "decoder.fc_output.bias",
                 "decoder.layer_norm.weight", "decoder.layer_norm.bias"]
        for l in reversed(range(L)):
            b = "decoder.transformer_decoder.%d." % l
            for n in ("norm3", "norm2", "norm1"):
                order += [b + n + ".weight", b + n + ".bias"]
            order += [b + "ffn.linear2.weight", b + "ffn.linear2.bias", b + "ffn.linear1.weight", b + "ffn.linear1.bias"]
            m = b + "multihead_attn."
            order += [m + "out_linear.weight", m + "out_linear.bias", m + "q_linear.weight", m + "q_linear.bias",
                      m + "k_linear.bias", m + "v_linear.bias"]
            s = b + "self_attn."
            order += [s + "out_linear.weight", s + "out_linear.bias",
                      s + "q_linear.weight", s + "k_linear.weight", s + "v_linear.weight",
                      s + "q_linear.bias", s + "k_linear.bias", s + "v_linear.bias"]
        # the cross-attention k|v weights of all decoder layers, in layer order: the
        # B operand [W_kv_0; ...; W_kv_{L-1}] of the memory-gradient GEMM is then a
        # view of the arena (_kv_weights).  After the decoder layers, so the prefix
        # a decoder layer's backward completes still holds only final gradients.
        for l in range(L):
            m = "decoder.transformer_decoder.%d.multihead_attn." % l
            order += [m + "k_linear.weight", m + "v_linear.weight"]
        order += ["encoder.layer_norm.weight", "encoder.layer_norm.bias"]
        for l in reversed(range(L)):
            b = "encoder.transformer_encoder.%d." % l
            for n in ("norm2", "norm1"):
                order += [b + n + ".weight", b + n + ".bias"]
            order += [b + "ffn.linear2.weight", b + "ffn.linear2.bias", b + "ffn.linear1.weight", b + "ffn.linear1.bias"]
            s = b + "self_attn."
            order += [s + "out_linear.weight", s + "out_linear.bias",
                      s + "q_linear.weight", s + "k_linear.weight", s + "v_linear.weight",
                      s + "q_linear.bias", s + "k_linear.bias", s + "v_linear.bias"]
        order += ["encoder.embedding.weight", "encoder.embedding.bias"]
        return order

    def _build_arena(self):
        """Two regions: the matrices (reverse backward order), padded to a multiple
        of ARENA_ALIGN so they split into equal 64-aligned shards for 1..8 ranks
        (sharded optimizer), then the vectors (biases, LayerNorm gamma/beta, ~0.1 %
        of the parameters) that the kernels read in f32: the sharded optimizer
        keeps those replicated (parallel.zero1_step)."""
        named = dict(self.model.named_parameters())
        order = self._arena_order()
        if sorted(order) != sorted(named):
            raise RuntimeError("unexpected parameter set: %s" % sorted(set(order) ^ set(named)))
        mats = [n for n in order if named[n].dim() > 1]
        vecs = [n for n in order if named[n].dim() <= 1]
        self.offsets = {}
        off = 0
        for n in mats:
            k = named[n].numel()
            self.offsets[n] = (off, k, tuple(named[n].shape))
            off += _pad64(k)
        self.n_shardable = off = (off + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN
        for n in vecs:
            k = named[n].numel()
            self.offsets[n] = (off, k, tuple(named[n].shape))
            off += _pad64(k)
        self.numel = off
        # gradient-bucket readiness (GradAllReducer): after the backward of the
        # parameter `name` the matrices' prefix up to here is final
        self.end_of, hi = {}, 0
        for n in order:
            o, k, _ = self.offsets[n]
            if named[n].dim() > 1:
                hi = o + _pad64(k)
            self.end_of[n] = hi
        # arena ranges whose gradients the grouped dW launches do NOT produce (the
        # head and embedding weights take the split-K path; the vectors come from
        # reductions): the fused clip norm runs nstl_sumsq over these only
        lo = _pad64(named["decoder.fc_output.weight"].numel())
        hi = self.offsets["encoder.embedding.weight"][0]
        for n in mats:
            o = self.offsets[n][0]
            assert (lo <= o < hi) == (".transformer_" in n), n
        self.norm_rest = [(0, lo), (hi, off)]
        self.sq_tiles = sum(((named[n].shape[0] + 255) // 256) * ((named[n].shape[1] + 255) // 256)
                            for n in mats if ".transformer_" in n)
        self.master_stale = False  # sharded optimizer: p32 matrices outside this rank's shard are old
        dev = self.device
        self.p32 = torch.zeros(off, dtype=torch.float32, device=dev)
        self.g32 = torch.zeros(off, dtype=torch.float32, device=dev)
        self.p16 = torch.zeros(off, dtype=self.dt, device=dev) if self.dt != torch.float32 else self.p32
        with torch.no_grad():
            for n in order:
                o, k, shp = self.offsets[n]
                self.p32[o:o + k].view(shp).copy_(named[n].detach().to(dev))
        self._params = [(n, named[n]) for n in order]
        self._rebind()
        self.refresh_shadow()

    def _rebind(self):
        me = weakref.ref(self)
        for n, p in self._params:
            o, k, shp = self.offsets[n]
            p.data = self.p32[o:o + k].view(shp)
            p.grad = self.g32[o:o + k].view(shp)
            p._nstl_engine = me
        self.name_of = {id(p): n for n, p in self._params}
        self._first_ptr = self._params[0][1].data_ptr()
        self._grad_views = None

    def ensure_bound(self, versions=True):
        """Re-pack if someone replaced parameter storage (e.g. model.to()); keep
        every p.grad on its arena slice; refresh the compute-dtype shadow after an
        in-place change of a parameter (versions=False skips that check: the
        backward uses the weights its forward used).  Runs on the host in front of
        the backward's first launch, where the GPU waits for it: the common case is
        one identity test per parameter (~340 in the 228M model)."""
        p0 = self._params[0][1]
        if p0.data_ptr() != self._first_ptr or p0.device != self.device:
            self.sync_pending()
            with torch.no_grad():
                for n, p in self._params:
                    o, k, shp = self.offsets[n]
                    self.p32[o:o + k].view(shp).copy_(p.detach().to(self.device))
            self._rebind()
            self.refresh_shadow()
        gv = getattr(self, "_grad_views", None)
        if gv is None:  # a sentinel, not None: a p.grad of None must fail the identity test
            gv = self._grad_views = [_UNBOUND] * len(self._params)
        gbase = None
        for i, (n, p) in enumerate(self._params):
            gp = p.grad
            if gp is not gv[i]:
                if gbase is None:
                    gbase = self.g32.data_ptr()
                o, k, shp = self.offsets[n]
                if gp is None or gp.data_ptr() != gbase + 4 * o:
                    gp = p.grad = self.g32[o:o + k].view(shp)
                    self.grads_fresh = True
                gv[i] = gp
        if versions and any(p._version != v for (n, p), v in zip(self._params, self._version_list)):
            self.refresh_shadow()

    def refresh_shadow(self):
        self.sync_pending()
        if self.p16 is not self.p32:
            K.cast(self.p32, self.p16, stream=K.stream_of(self.device))
        self._versions = {n: p._version for n, p in self._params}
        self._version_list = [p._version for n, p in self._params]

    def zero_grad(self):
        """Next backward overwrites the gradient arena instead of accumulating."""
        self.grads_fresh = True

    # ------------------------------------------------ deferred weight updates
    # FusedAdam.overlap_next_forward: the optimizer's update is queued on a side
    # stream in arena ranges -- the f32 vectors (biases, LayerNorm) first, then
    # the matrices of each forward stage in forward order (embedding, encoder
    # layers, decoder layers, head) -- and the next forward makes its stream wait
    # for a stage's range just before that stage reads its weights, so the update
    # of later layers runs under the forward of earlier ones.  Every other entry
    # that reads or writes the arenas waits for all of it first (sync_pending).
    def update_ranges(self):
        if self._upd_ranges is None:
            def rng(names):
                return (min(self.offsets[n][0] for n in names),
                        max(self.offsets[n][0] + _pad64(self.offsets[n][1]) for n in names))

            def is_kv(n):  # the cross-attention k|v block (after the decoder layers)
                return ".multihead_attn.k_linear.weight" in n or ".multihead_attn.v_linear.weight" in n

            def mats(prefix):
                return [n for n in self.offsets
                        if n.startswith(prefix) and len(self.offsets[n][2]) > 1 and not is_kv(n)]
            st = [("vec", (self.n_shardable, self.numel)), ("emb", rng(["encoder.embedding.weight"]))]
            st += [(("enc", l), rng(mats("encoder.transformer_encoder.%d." % l))) for l in range(self.L)]
            st += [("dec_kv", rng([n for n in self.offsets if is_kv(n)]))]
            st += [(("dec", l), rng(mats("decoder.transformer_decoder.%d." % l))) for l in range(self.L)]
            st += [("head", rng(["decoder.fc_output.weight"]))]
            # the stages partition the arena: an update range never covers a parameter twice
            cuts = sorted(r for _, r in st)
            assert all(a[1] <= b[0] for a, b in zip(cuts, cuts[1:])), cuts
            self._upd_ranges = st
            self._stage_rng = dict(st)
        return self._upd_ranges

    def queue_update(self, fn, stream):
        """fn(lo, hi) enqueues the optimizer update of arena range [lo, hi) on
        `stream` (a torch.cuda.Stream); ranges in update_ranges() order."""
        self.sync_pending()
        for _, (lo, hi) in self.update_ranges():
            fn(lo, hi)
            ev = torch.cuda.Event()
            ev.record(stream)
            self._wpending.append((lo, hi, ev))

    def _await(self, lo, hi):
        main = torch.cuda.current_stream(self.device)
        keep = []
        for l, h, ev in self._wpending:
            if l < hi and lo < h:
                main.wait_event(ev)
            else:
                keep.append((l, h, ev))
        self._wpending = keep

    def await_stage(self, key):
        """The current stream waits for the queued update of stage `key`'s weights
        (a decoder layer's include its cross-attention k|v, kept in their own block)."""
        if self._wpending:
            self._await(*self._stage_rng[key])
            if isinstance(key, tuple) and key[0] == "dec":
                self._await(*self._stage_rng["dec_kv"])

    def sync_pending(self):
        """The current stream waits for every queued update."""
        if self._wpending:
            self._await(0, self.numel)

    # views ----------------------------------------------------------------
    def w(self, name, rows=1):
        """Compute-dtype view of `rows` consecutive weight matrices starting at `name`."""
        o, k, shp = self.offsets[name]
        return self.p16[o:o + k * rows].view(shp[0] * rows, *shp[1:])

    def b(self, name, rows=1):
        o, k, _ = self.offsets[name]
        return self.p32[o:o + k * rows]

    def _kv_weights(self):
        """The decoder cross-attention k|v weights (compute dtype) stacked in one
        contiguous [L * 2D, D] slab, the B operand of the concatenated memory-gradient
        GEMM: a view of the arena (_arena_order keeps them side by side in layer
        order); otherwise copied every backward (the optimizer has moved the
        weights) on the current stream, which backward() makes the engine's stream."""
        D, L = self.D, self.L
        k0 = self.offsets["decoder.transformer_decoder.0.multihead_attn.k_linear.weight"][0]
        if all(self.offsets["decoder.transformer_decoder.%d.multihead_attn.%s_linear.weight" % (l, kv)][0]
               == k0 + (2 * l + (kv == "v")) * D * D for l in range(L) for kv in ("k", "v")):
            return self.p16[k0:k0 + L * 2 * D * D].view(L * 2 * D, D)
        if self._wkv is None:
            self._wkv = torch.empty(L * 2 * D, D, dtype=self.dt, device=self.device)
        for l in range(L):
            self._wkv[2 * D * l:2 * D * (l + 1)].copy_(
                self.w("decoder.transformer_decoder.%d.multihead_attn.k_linear.weight" % l, 2))
        return self._wkv

    def gw(self, name, rows=1):
        o, k, shp = self.offsets[name]
        return self.g32[o:o + k * rows].view(shp[0] * rows, *shp[1:])

    def gb(self, name, rows=1):
        o, k, _ = self.offsets[name]
        return self.g32[o:o + k * rows]

    def rope(self, T, dim):
        key = (T, dim)
        if key not in self._rope:
            self._rope[key] = rotation_tables(T, dim, self.device)
        return self._rope[key]

    def bufs(self, B, T, save):
        key = (B, T, save)
        if key not in self._bufs:
            if save:  # keep at most one training workspace alive
                for k2 in [k for k in self._bufs if k[2]]:
                    del self._bufs[k2]
            self._bufs[key] = _Buffers(self, B, T, save)
        return self._bufs[key]

    def splitk_ws_elems(self, M):
        best = 0
        for n, k in ((self.D, self.D), (3 * self.D, self.D), (self.Fd, self.D), (self.D, self.Fd),
                     (2 * self.D, self.D), (self.D, self.in_dim), (self.out_dim, self.D)):
            best = max(best, self.splits(n, k, M) * n * k)
        return max(best, 1)

    @staticmethod
    def splits(n, k, m):
        """split-K for a weight-gradient GEMM C[n,k] = sum over m tokens.  Mirrors the
        kernel choice in nstl_gemm: >= 32 tiles of 256^2 -> the 256 kernel, aim for
        ~256 blocks; else the 128 kernel, aim for ~512 blocks (tools/bench_gemm.py)."""
        t256 = ((n + 255) // 256) * ((k + 255) // 256)
        if t256 >= 32 and n >= 256 and k >= 256:
            target, tiles = 256, t256
        else:
            target, tiles = 512, ((n + 127) // 128) * ((k + 127) // 128)
        s = max(1, min(16, target // tiles))
        while s > 1 and m // s < 1024:
            s -= 1
        return s

    # ------------------------------------------------------------------ fp8
    FP8_SCOPES = ("attn+enc_ffn1", "all")

    def fp8_groups(self):
        """(weight name, rows) of the projections whose forward runs in fp8 (C5:
        q/k/v and FFN).  Scope "attn+enc_ffn1" (default): every attention input
        projection -- self-attention q|k|v (3 matrices, one GEMM), the decoder's
        cross-attention q and k|v -- and the encoder's FFN linear1.  Scope "all"
        adds the encoder FFN linear2 and the decoder FFN: its forward misses the
        metric's 1e-3 MSE gate (1.8-2.5e-3 at the 228M config, e4m3's 3 mantissa
        bits; per-32 E8M0 block scales do not change it), while this scope
        measures 6.4-7.8e-4 over four seeded models (tests/test_fp8_cpu.py)."""
        out = []
        for l in range(self.L):
            pre = "encoder.transformer_encoder.%d." % l
            out += [(pre + "self_attn.q_linear.weight", 3), (pre + "ffn.linear1.weight", 1)]
            if self.fp8_scope == "all":
                out += [(pre + "ffn.linear2.weight", 1)]
        for l in range(self.L):
            pre = "decoder.transformer_decoder.%d." % l
            out += [(pre + "self_attn.q_linear.weight", 3), (pre + "multihead_attn.q_linear.weight", 1),
                    (pre + "multihead_attn.k_linear.weight", 2)]
            if self.fp8_scope == "all":
                out += [(pre + "ffn.linear1.weight", 1), (pre + "ffn.linear2.weight", 1)]
        return out

    def fp8_scope_desc(self):
        """What runs in fp8 (bench.py reports it with the C5 line, so lines of
        different scopes are not compared as if they were one configuration)."""
        fwd = {"attn+enc_ffn1": "attention q/k/v (self and cross) + encoder FFN linear1 forward GEMMs",
               "all": "attention q/k/v + every FFN linear1/linear2 forward GEMM"}[self.fp8_scope]
        groups = sorted({n.split(".", 3)[-1] if n.startswith(("encoder", "decoder")) else n
                         for n, _ in self.fp8_groups()})
        enc = sorted({n.split(".", 3)[-1] for n, _ in self.fp8_groups() if n.startswith("encoder")})
        dec = sorted({n.split(".", 3)[-1] for n, _ in self.fp8_groups() if n.startswith("decoder")})
        bwd = self.fp8_bwd
        return {"scope": self.fp8_scope, "forward": fwd,
                "backward": ("FFN linear2 input-gradient GEMMs (every layer) on e4m3 dy (row scales, from the "
                             "LayerNorm backward) and e4m3 W2^T (input-channel scales); other backward GEMMs bf16")
                if bwd else "bf16",
                "backward_launches": len(self.fp8_bwd_groups()) if bwd else 0,
                "encoder_groups": enc, "decoder_groups": dec, "launches_per_forward": len(self.fp8_groups()),
                "summary": fwd + ("; fp8 backward" if bwd else "; bf16 backward")} if groups else None

    def fp8_bwd_groups(self):
        """Weights whose input-gradient GEMM runs in fp8 when fp8_bwd is on: every
        FFN linear2 (encoder and decoder).  The forward's MSE gate does not apply to
        the backward; the gradient bound is tests/test_fp8_gpu.py's."""
        return ["%s.%d.ffn.linear2.weight" % (st, l) for st in ("encoder.transformer_encoder",
                                                               "decoder.transformer_decoder") for l in range(self.L)]

    def wt_groups(self):
        """(weight name, rows) of the input-gradient GEMMs that read the transposed
        bf16 copy (every layer projection; the FFN linear2 not when its dX runs in
        fp8), plus ("kv", 0): the stacked cross-attention k|v slab of the
        concatenated memory-gradient GEMM."""
        out = []
        fp8_w2 = self.fp8 and self.fp8_bwd
        for l in range(self.L):
            for pre, names in (("encoder.transformer_encoder.%d." % l, ("self_attn",)),
                               ("decoder.transformer_decoder.%d." % l, ("self_attn", "multihead_attn"))):
                for a in names:
                    if a == "self_attn":
                        out.append((pre + a + ".q_linear.weight", 3))
                    else:
                        out.append((pre + a + ".q_linear.weight", 1))
                        if not self.dmem_concat:
                            out.append((pre + a + ".k_linear.weight", 2))
                    out.append((pre + a + ".out_linear.weight", 1))
                out.append((pre + "ffn.linear1.weight", 1))
                if not fp8_w2:
                    out.append((pre + "ffn.linear2.weight", 1))
        if self.dmem_concat:
            out.append(("kv", 0))
        return out

    def _refresh_wt(self):
        """W^T copies of this backward's weights (one batched transpose launch)."""
        self._wt_ok = False
        if not (self.wt_on and self.dt == torch.bfloat16):
            return
        groups = self.wt_groups()
        if self._wt is None or set(self._wt) != set(groups):
            src = {g: (self._kv_weights() if g[0] == "kv" else self.w(*g)) for g in groups}
            if any(x.shape[0] % 64 or x.shape[1] % 64 for x in src.values()):
                self.wt_on = False
                return
            self._wt = {g: torch.empty(x.shape[1], x.shape[0], dtype=self.dt, device=self.device)
                        for g, x in src.items()}
        K.transpose_bf16([(self._kv_weights() if g[0] == "kv" else self.w(*g), y) for g, y in self._wt.items()],
                         stream=self.st)
        self._wt_ok = True

    def set_fp8(self, on, scope=None, backward=None):
        if on and self.dt != torch.bfloat16:
            raise ValueError("fp8 projections need the bf16 compute dtype (use_amp=True)")
        if scope is not None:
            if scope not in self.FP8_SCOPES:
                raise ValueError("fp8 scope must be one of %s" % (self.FP8_SCOPES,))
            if scope != self.fp8_scope:
                self._fp8_w = None  # re-quantize the new set
            self.fp8_scope = scope
        if backward is not None:
            self.fp8_bwd = bool(backward)
        self.fp8 = bool(on)

    def _fp8_on(self, name, rows=1):
        """Does the projection `name` run in fp8 in this forward?"""
        return self.fp8 and self._fp8_w is not None and (name, rows) in self._fp8_w

    def _fp8_weights(self):
        """Quantize the fp8 projections' weights from the bf16 shadow (one batched
        launch; every forward, so an optimizer step or a load is always seen)."""
        if self._fp8_w is None:
            self._fp8_w = {}
            for name, rows in self.fp8_groups():
                n, k = self.w(name, rows).shape
                self._fp8_w[(name, rows)] = (torch.empty(n, k, dtype=torch.float8_e4m3fn, device=self.device),
                                             torch.empty(n, dtype=torch.float32, device=self.device))
        jobs = []
        for (name, rows), (q, sc) in self._fp8_w.items():
            W = self.w(name, rows)
            jobs.append((W, W.shape[0], W.shape[1], q, sc))
        K.fp8_quant_rows(jobs, stream=self.st)
        if self.fp8_bwd:
            if self._fp8_wt is None:
                self._fp8_wt = {}
                for name in self.fp8_bwd_groups():
                    n, k = self.w(name).shape
                    self._fp8_wt[name] = (torch.empty(k, n, dtype=torch.float8_e4m3fn, device=self.device),
                                          torch.empty(k, dtype=torch.float32, device=self.device))
            K.fp8_quant_cols([(self.w(name), self.w(name).shape[0], self.w(name).shape[1], q, sc)
                              for name, (q, sc) in self._fp8_wt.items()], stream=self.st)

    def _fp8_dy_bufs(self, M):
        """e4m3 copy of the LayerNorm backward's dbranch [M, D] and its row scales."""
        if M not in self._fp8_dy:
            self._fp8_dy = {M: (torch.empty(M, self.D, dtype=torch.float8_e4m3fn, device=self.device),
                                torch.empty(M, dtype=torch.float32, device=self.device))}
        return self._fp8_dy[M]

    def _fp8_bufs(self, M):
        if M not in self._fp8_act:
            e8 = lambda *s: torch.empty(*s, dtype=torch.float8_e4m3fn, device=self.device)
            f = lambda n: torch.empty(n, dtype=torch.float32, device=self.device)
            self._fp8_act = {M: (e8(M, max(self.D, self.Fd)), f(M), e8(M, self.D), f(M))}
        return self._fp8_act[M]

    def _fp8_target(self, x, mem):
        """Where the e4m3 copy of x goes: the scratch (valid until the next copy
        into it) or the decoder memory's own buffer (all cross-attention k|v
        projections of a forward share it)."""
        M, cols = x.shape
        q, sc, qm, sm = self._fp8_bufs(M)
        if mem:
            return qm, sm
        self._xq = {p: v for p, v in self._xq.items() if v[0].data_ptr() != q.data_ptr()}
        return q[:, :cols], sc

    def _fp8_quant(self, x, mem=False):
        """Row-wise e4m3 copy of activation x [M, cols] by the standalone kernel."""
        q, sc = self._fp8_target(x, mem)
        K.fp8_quant_rows([(x, x.shape[0], x.shape[1], q, sc)], stream=self.st)
        self._xq[x.data_ptr()] = (q, sc)
        return q, sc

    # ------------------------------------------------------------ primitives
    def _gemm_fwd(self, x, wname, out, epi, rows=1, rope=None, rope_cols=0, p_drop=0.0, seed=0, relu_mask=None,
                  xq=None):
        """Projection forward; `relu_mask` (FFN1): also write the keep&positive bits of
        the hidden for the backward's dReLU when the kernel can (returns whether).
        In fp8 mode the C5 projections take e4m3 operands (`xq`: x already quantized)."""
        W = self.w(wname, rows)
        bias = self.b(wname.replace(".weight", ".bias"), rows)
        kw = dict(epilogue=epi, bias=bias, rope=rope, rope_cols=rope_cols, p_drop=p_drop, seed=seed)
        m, n, k = x.shape[0], W.shape[0], W.shape[1]
        if self.fp8 and (wname, rows) in self._fp8_w:
            qw, sw = self._fp8_w[(wname, rows)]
            if xq is None:
                xq = self._xq.get(x.data_ptr()) or self._fp8_quant(x)
            x, sx = xq
            W = qw
            kw.update(a_scale=sx, b_scale=sw)
        use = relu_mask is not None and self.relu_mask_on and \
            0 < K.gemm_relu_mask_words(x, W, out, m, n, k, **kw) <= relu_mask.numel()
        K.gemm(x, W, out, m, n, k, relu_mask=relu_mask if use else None, stream=self.st, **kw)
        return use

    def _dw(self, dy, x, wname, rows, bf, ws, bias=True):
        """grad(W) (+)= dy^T x ; grad(b) (+)= colsum(dy) (unless the bias gradient
        was already produced by the LayerNorm backward that wrote dy).  Inside a
        decoder layer the GEMM is queued for that layer's grouped launch."""
        G = self.gw(wname, rows)
        n, k = G.shape
        m = dy.shape[0]
        if self._defer is not None:
            self._defer.append((dy, x, G, bf))
            if bias:
                bname = wname.replace(".weight", ".bias")
                K.colsum(dy, dy.stride(0), m, n, self.cur.col_part, self.gb(bname, rows), bf, stream=self.st)
            return
        if ".transformer_" in wname:
            self._sq_ok = False  # a layer weight gradient without the grouped epilogue's partials
        s = self.splits(n, k, m)
        st = self._side_begin()
        K.gemm(dy, x, G, n, k, m, a_kmajor=False, b_kmajor=False, beta=bf, split_k=s, workspace=ws, stream=st)
        if bias:
            bname = wname.replace(".weight", ".bias")
            K.colsum(dy, dy.stride(0), m, n, self.cur.col_part, self.gb(bname, rows), bf, stream=st)
        self._side_end(dy)

    def _dw_flush(self, ws):
        """Launch the queued weight gradients: one grouped GEMM (no split-K) when
        every problem suits the 256 kernel, else one split-K GEMM each."""
        jobs, self._defer = self._defer, None
        ok = all(self.dt == torch.bfloat16 and G.shape[0] >= 256 and G.shape[1] >= 256 and dy.shape[0] >= 256
                 and dy.shape[0] % 64 == 0 for dy, x, G, bf in jobs) and len(jobs) <= K.GEMM_GROUP_MAX
        if ok:
            probs = []
            for dy, x, G, bf in jobs:
                kw = dict(a_kmajor=False, b_kmajor=False, beta=bf)
                if self._sq_ok:
                    nt = ((G.shape[0] + 255) // 256) * ((G.shape[1] + 255) // 256) * 8
                    kw["sq_part"] = self._sq_buf[self._sq_used:self._sq_used + nt]
                    self._sq_used += nt
                probs.append((dy, x, G, G.shape[0], G.shape[1], dy.shape[0], kw))
            K.gemm_grouped(probs, stream=self.st)
            return
        self._sq_ok = False
        for dy, x, G, bf in jobs:
            n, k = G.shape
            m = dy.shape[0]
            K.gemm(dy, x, G, n, k, m, a_kmajor=False, b_kmajor=False, beta=bf, split_k=self.splits(n, k, m),
                   workspace=ws, stream=self.st)

    # ---------------------------------------------------- side (dW) stream
    # A dW GEMM only reads dy (a backward scratch buffer) and a saved activation
    # and only writes its own gradient slice, the split-K workspace and the
    # colsum partials (all private to the side stream).  So it may run beside
    # the dX chain: it waits for the main stream at launch (dy is ready), and
    # the main stream waits for it only before overwriting that dy buffer.
    def _side_begin(self):
        if self._side is None:
            return self.st
        ev = torch.cuda.Event()
        ev.record(self._main)
        self._side.wait_event(ev)
        return self._side.cuda_stream

    def _side_end(self, dy):
        if self._side is None:
            return
        ev = torch.cuda.Event()
        ev.record(self._side)
        lo, hi = _span(dy)
        self._side_reads.append((lo, hi, ev))

    def _guard(self, *outs):
        """The main stream is about to write `outs`: wait for dW reads of them."""
        if not self._side_reads:
            return
        spans = [_span(t) for t in outs if t is not None]
        keep = []
        for lo, hi, ev in self._side_reads:
            if any(lo < h and l < hi for l, h in spans):
                self._main.wait_event(ev)
            else:
                keep.append((lo, hi, ev))
        self._side_reads = keep

    def _side_join(self):
        if self._side is not None:
            self._main.wait_stream(self._side)
            self._side_reads = []

    def _dx(self, dy, wname, rows, out, beta, epi=K.EPI_NONE, aux=None, p_drop=0.0, colsum=None, relu_mask=None,
            dyq=None):
        """out (+)= dy W  (W: [N][K] read as [r][j]).  colsum = (partials, grad(b), beta):
        the bias gradient of the Linear whose input gradient `out` is, from the
        epilogue's column sums; returns False when the kernel cannot produce them.
        `dyq` = (e4m3 dy, row scales): the fp8 form, on W^T's e4m3 copy."""
        W = self.w(wname, rows)
        n, k = W.shape
        self._guard(out)
        kw = dict(a_kmajor=True, b_kmajor=False, beta=beta, epilogue=epi, aux=aux,
                  ld_aux=aux.stride(0) if aux is not None else 0, p_drop=p_drop)
        if dyq is not None:
            qt, st = self._fp8_wt[wname]
            dy, W = dyq[0], qt
            kw.update(b_kmajor=True, a_scale=dyq[1], b_scale=st)
        elif self._wt_ok and (wname, rows) in self._wt:
            W = self._wt[(wname, rows)]
            kw["b_kmajor"] = True
        if relu_mask is not None and 0 < K.gemm_relu_mask_words(dy, W, out, dy.shape[0], k, n, **kw) \
                <= relu_mask.numel():
            kw["relu_mask"] = relu_mask
        m = dy.shape[0]
        nrows = K.gemm_colsum_rows(dy, W, out, m, k, n, **kw) if colsum is not None and self.fused_bias_on else 0
        fused = 0 < nrows <= (colsum[0].shape[0] if colsum is not None else 0)
        K.gemm(dy, W, out, m, k, n, colsum_part=colsum[0] if fused else None, stream=self.st, **kw)
        if fused:
            self._reduce(colsum[0], k, nrows, k, colsum[1], colsum[2])
        return fused

    def _dx_res(self, dy, wname, rows, last=False):
        """Input gradient of a Linear whose input is a LayerNorm output: accumulate
        it into the f32 residual gradient.  Handoff mode writes it in the compute
        dtype (as the reference's autocast rounds it) for the next LN backward to
        add; `last` (the consumer is not an LN backward) keeps the f32 accumulate."""
        bb = self.cur
        if self.res_handoff_on and not last:
            assert not self._dadd_pending
            self._dx(dy, wname, rows, bb.dadd, 0.0)
            self._dadd_pending = True
        else:
            self._dx(dy, wname, rows, bb.dres, 1.0)

    def _ln(self, x, y, out, stats, prefix, n_masks, seeds, s_out, rot=None, T=None, q8=None):
        """LayerNorm tail; in fp8 mode (q8 = 'scratch' / 'mem') it also writes the
        row-wise e4m3 copy of `out` that the next fp8 projection reads."""
        a = K.LnArgs()
        a.dtype = K.dtype_code(self.dt)
        a.rows, a.D = out.shape[0], self.D
        a.x, a.y = K.ptr(x), K.ptr(y)
        a.n_masks, a.p_drop = n_masks, self.p
        a.seed1, a.seed2 = seeds
        a.gamma, a.beta, a.eps = self.b(prefix + ".weight").data_ptr(), self.b(prefix + ".bias").data_ptr(), 1e-5
        a.s_out, a.out, a.mean, a.rstd = K.ptr(s_out), out.data_ptr(), stats[0].data_ptr(), stats[1].data_ptr()
        if rot is not None:
            cs, sn = self.rope(T, self.D)
            a.rot_out, a.rope_cos, a.rope_sin, a.rope_T = rot.data_ptr(), cs.data_ptr(), sn.data_ptr(), T
        if self.fp8 and q8 is not None:
            q, sc = self._fp8_target(out, q8 == "mem")
            a.q8, a.ldq8, a.q8_scale = q.data_ptr(), q.stride(0), sc.data_ptr()
        K.ln_fwd(a, stream=self.st)
        if self.fp8 and q8 is not None:
            self._xq[out.data_ptr()] = (q, sc)

    def _ln_bwd(self, s_in, stats, prefix, dres_in, dres_out, dbranch, n_masks, seeds, bf, bias_of=None, q8=None):
        """LayerNorm(+dropout+residual) backward; with `bias_of`, the column sums of
        dbranch become grad(bias) of that Linear (its output was the LN branch);
        `q8` = (e4m3 [rows, D], scales [rows]): also the row-wise e4m3 copy of dbranch."""
        bb = self.cur
        a = K.LnArgs()
        a.dtype = K.dtype_code(self.dt)
        a.rows, a.D = s_in.shape[0], self.D
        a.n_masks, a.p_drop = n_masks, self.p
        a.seed1, a.seed2 = seeds
        a.gamma, a.beta, a.eps = self.b(prefix + ".weight").data_ptr(), self.b(prefix + ".bias").data_ptr(), 1e-5
        a.mean, a.rstd = stats[0].data_ptr(), stats[1].data_ptr()
        self._guard(dbranch)
        a.s_in, a.dout, a.ds, a.dbranch = s_in.data_ptr(), dres_in.data_ptr(), dres_out.data_ptr(), K.ptr(dbranch)
        if self._dadd_pending:
            a.dout2 = bb.dadd.data_ptr()
            self._dadd_pending = False
        part = bb.ln_part
        if self._red is not None:
            part = bb.ln_parts[self._ln_slot]
            self._ln_slot += 1
        a.dgamma_part, a.dbeta_part, a.n_part = part[0].data_ptr(), part[1].data_ptr(), bb.n_part
        if bias_of is not None:
            a.dbranch_part = part[2].data_ptr()
        if q8 is not None:
            a.q8, a.ldq8, a.q8_scale = q8[0].data_ptr(), q8[0].stride(0), q8[1].data_ptr()
        K.ln_bwd(a, stream=self.st)
        outs = [self.gb(prefix + ".weight"), self.gb(prefix + ".bias")]
        if bias_of is not None:
            outs.append(self.gb(bias_of))
        if self._red is not None:
            for m, out in enumerate(outs):
                self._reduce(part[m], self.D, bb.n_part, self.D, out, bf)
        else:
            K.reduce_rows3(part, bb.n_part, self.D, outs, bf, stream=self.st)

    def _attn(self, q, k, v, o, lse, seed, T, B, mask=None):
        a = K.attn_args(K.dtype_code(self.dt), B, T, self.H, 0, 0, 0, 0, 0, 0, 0, 0, 0, self.p, seed, dh=self.dh)
        K.attn_set(a, q=q, k=k, v=v, o=o, lse=lse, mask_bits=mask)
        K.attn_fwd(a, stream=self.st)

    def _attn_bwd(self, q, k, v, o, lse, do, dq, dk, dv, seed, T, B, mask=None, bias=(), bf=0.0):
        """Attention backward.  `bias`: (column offset in q|k|v, columns, grad(bias)
        view) -- the projection bias gradients, reduced from the kernel's fused
        column sums.  Returns False when the call took the generic kernels (no
        sums: the caller's colsum provides them)."""
        a = K.attn_args(K.dtype_code(self.dt), B, T, self.H, 0, 0, 0, 0, 0, 0, 0, 0, 0, self.p, seed, dh=self.dh)
        cs, sn = self.rope(T, self.dh)
        a.rope_q, a.rope_k = 1, 1
        K.attn_set(a, q=q, k=k, v=v, o=o, lse=lse, dout=do, dq=dq, dk=dk, dv=dv, rope_cos=cs, rope_sin=sn,
                   dsum=self.cur.dsum, mask_bits=mask)
        part = self.cur.abias
        if self._red is not None:
            part = self.cur.abias_slots[self._ab_slot]
            self._ab_slot += 1
        rows = K.attn_bias_rows(a) if bias and self.fused_bias_on else 0
        fused = 0 < rows <= part.shape[0]
        if fused:
            K.attn_set(a, dbias_part=part)
        self._guard(dq, dk, dv)
        K.attn_bwd(a, stream=self.st)
        for off, n, out in (bias if fused else ()):
            self._reduce(part[:, off:], part.stride(0), rows, n, out, bf)
        return fused

    # ---------------------------------------------- batched row reductions
    def _reduce(self, part, ld, n_part, cols, out, beta):
        """out = beta*out + rowsum(part): queued for the layer's batched launch, or now."""
        if self._red is None:
            K.reduce_rows_strided(part, ld, n_part, cols, out, beta, stream=self.st)
            return
        if len(self._red) == K.REDUCE_BATCH_MAX:
            self._red_flush(reopen=True)
        self._red.append((part, ld, n_part, cols, out, beta))

    def _red_open(self):
        if self.reduce_batch_on:
            self._red, self._ln_slot, self._ab_slot = [], 0, 0

    def _red_flush(self, reopen=False):
        """Launch the queued reductions (their partial buffers are free afterwards)."""
        jobs, self._red = self._red, None
        if jobs:
            K.reduce_rows_batch(jobs, stream=self.st)
        if reopen:
            self._red = []

    # --------------------------------------------------------------- forward
    def _enc_layer(self, bb, l, x, T):
        self.await_stage(("enc", l))
        D, B = self.D, bb.B
        pre = "encoder.transformer_encoder.%d." % l
        sd = lambda s: _seed(self.base_seed, True, l, s)
        qkv, o, lse = bb.layer(bb.e_qkv, l), bb.layer(bb.e_o, l), bb.layer(bb.e_lse, l)
        self._gemm_fwd(x, pre + "self_attn.q_linear.weight", qkv, K.EPI_BIAS_ROPE, rows=3,
                       rope=(*self.rope(T, self.dh), T, self.dh), rope_cols=2 * D)
        self._attn(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, sd("attn"), T, B,
                   mask=bb.e_mask[l] if bb.save else None)
        self._gemm_fwd(o, pre + "self_attn.out_linear.weight", bb.y, K.EPI_BIAS)
        st = bb.layer(bb.e_stats, l)
        x1 = bb.layer(bb.e_x1, l)
        self._ln(x, bb.y, x1, st[0:2], pre + "norm1", 2, (sd("resid"), sd("drop1")), bb.layer(bb.e_s1, l),
                 q8="scratch")
        h = bb.layer(bb.e_h, l)
        ok = self._gemm_fwd(x1, pre + "ffn.linear1.weight", h, K.EPI_BIAS_RELU_DROP, p_drop=self.p, seed=sd("ffn"),
                            relu_mask=bb.e_rmask[l] if bb.save else None)
        if bb.save:
            bb.e_rmask_ok[l] = ok
        self._gemm_fwd(h, pre + "ffn.linear2.weight", bb.y, K.EPI_BIAS)
        x2 = bb.layer(bb.e_x2, l)
        self._ln(x1, bb.y, x2, st[2:4], pre + "norm2", 1, (sd("drop2"), 0), bb.layer(bb.e_s2, l),
                 q8="scratch" if l + 1 < self.L else None)
        return x2

    def _dec_layer(self, bb, l, x, mem, T):
        self.await_stage(("dec", l))
        D, B = self.D, bb.B
        pre = "decoder.transformer_decoder.%d." % l
        sd = lambda s: _seed(self.base_seed, False, l, s)
        L_ = lambda lst: bb.layer(lst, l)
        st = L_(bb.d_stats)
        qkv = L_(bb.d_qkv)
        self._gemm_fwd(x, pre + "self_attn.q_linear.weight", qkv, K.EPI_BIAS_ROPE, rows=3,
                       rope=(*self.rope(T, self.dh), T, self.dh), rope_cols=2 * D)
        self._attn(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], L_(bb.d_o), L_(bb.d_lse), sd("attn"), T, B,
                   mask=bb.d_mask[l] if bb.save else None)
        self._gemm_fwd(L_(bb.d_o), pre + "self_attn.out_linear.weight", bb.y, K.EPI_BIAS)
        x1 = L_(bb.d_x1)
        self._ln(x, bb.y, x1, st[0:2], pre + "norm1", 2, (sd("resid"), sd("drop1")), L_(bb.d_s1), q8="scratch")
        qc, kvc = L_(bb.d_qc), L_(bb.d_kvc)
        self._gemm_fwd(x1, pre + "multihead_attn.q_linear.weight", qc, K.EPI_BIAS_ROPE,
                       rope=(*self.rope(T, self.dh), T, self.dh), rope_cols=D)
        if not self._kv_all_done:
            self._gemm_fwd(mem, pre + "multihead_attn.k_linear.weight", kvc, K.EPI_BIAS_ROPE, rows=2,
                           rope=(*self.rope(T, self.dh), T, self.dh), rope_cols=D, xq=self._mem_q)
        self._attn(qc, kvc[:, :D], kvc[:, D:], L_(bb.d_oc), L_(bb.d_lsec), sd("xattn"), T, B,
                   mask=bb.d_maskc[l] if bb.save else None)
        self._gemm_fwd(L_(bb.d_oc), pre + "multihead_attn.out_linear.weight", bb.y, K.EPI_BIAS)
        x2 = L_(bb.d_x2)
        self._ln(x1, bb.y, x2, st[2:4], pre + "norm2", 2, (sd("xresid"), sd("drop2x")), L_(bb.d_s2),
                 q8="scratch" if self._fp8_on(pre + "ffn.linear1.weight") else None)
        h = L_(bb.d_h)
        ok = self._gemm_fwd(x2, pre + "ffn.linear1.weight", h, K.EPI_BIAS_RELU_DROP, p_drop=self.p, seed=sd("ffn"),
                            relu_mask=bb.d_rmask[l] if bb.save else None)
        if bb.save:
            bb.d_rmask_ok[l] = ok
        self._gemm_fwd(h, pre + "ffn.linear2.weight", bb.y, K.EPI_BIAS)
        x3 = L_(bb.d_x3)
        self._ln(x2, bb.y, x3, st[4:6], pre + "norm3", 1, (sd("drop3"), 0), L_(bb.d_s3),
                 q8="scratch" if l + 1 < self.L else None)
        return x3

    def _cross_kv_all(self, bb, mem, T):
        """The cross-attention k|v projections of every decoder layer (their A is
        the same encoder output) as ONE grouped launch before the decoder layers:
        on the 4-wave kernel one launch of L x 512 tiles instead of L launches of
        two rounds each, so the per-launch fill, drain and boundary are paid once
        (gemm4_kernel<..., EM_ROPE, GROUPED>).  Only when every layer keeps its own
        k|v buffer (a training forward), the projections are bf16 (not in the fp8
        scope), the shapes are whole 256 x 256 tiles and the RoPE table fits beside
        the 4-wave kernel's stages (T = 128 at head dim 64); otherwise each layer
        projects its own (returns False).
        NSTL_KV_GROUPED=0: per layer (A/B)."""
        D, L = self.D, self.L
        name = "decoder.transformer_decoder.%d.multihead_attn.k_linear.weight"
        # the 4-wave kernel's whole-tile shapes (M, N multiples of 256; K of 128, >= 256)
        tiles_ok = bb.M % 256 == 0 and (2 * D) % 256 == 0 and D % 128 == 0 and D >= 256
        if (not bb.save or L < 2 or not tiles_ok or os.environ.get("NSTL_KV_GROUPED", "1") == "0" or self.dt != torch.bfloat16
                or T * self.dh * 4 > ROPE_LDS_BYTES or any(self.fp8 and (name % l, 2) in self._fp8_w for l in range(L))):
            return False
        if self._wpending:
            self._await(*self._stage_rng["dec_kv"])
        rope = (*self.rope(T, self.dh), T, self.dh)
        probs = [(mem, self.w(name % l, 2), bb.d_kvc[l], bb.M, 2 * D, D,
                  dict(epilogue=K.EPI_BIAS_ROPE, bias=self.b((name % l).replace(".weight", ".bias"), 2), rope=rope,
                       rope_cols=D)) for l in range(L)]
        for i in range(0, L, K.GEMM_GROUP_MAX):
            K.gemm_grouped(probs[i:i + K.GEMM_GROUP_MAX], stream=self.st)
        return True

    def _prologue(self, training):
        self.ensure_bound()
        self.st = K.stream_of(self.device)
        self.p = float(self.dropout) if training else 0.0
        self._xq = {}  # e4m3 activation copies never outlive a forward
        self.await_stage("vec")  # biases and LayerNorm parameters of every stage
        # e4m3 W2^T is quantized only by forwards run with the fp8 backward on; the
        # backward of a forward that did not refresh it must not use an older copy
        self._fp8_wt_fresh = bool(self.fp8 and self.fp8_bwd)
        if self.fp8:
            self.sync_pending()  # every fp8 weight is quantized up front
            self._fp8_weights()

    def encode(self, bb, src, T):
        """Encoder forward; returns the encoder output `mem` (compute dtype)."""
        M = bb.M
        if self.dt == torch.float32 and src.is_contiguous():
            x_src = src.view(M, self.in_dim)
        else:
            K.copy2d(src.reshape(M, self.in_dim), self.in_dim, bb.src, self.in_dim, M, self.in_dim, self.in_dim,
                     stream=self.st)
            x_src = bb.src
        self.await_stage("emb")
        self._gemm_fwd(x_src, "encoder.embedding.weight", bb.x0, K.EPI_BIAS_ROPE,
                       rope=(*self.rope(T, self.D), T, self.D), rope_cols=self.D)
        self.x_src = x_src
        x = bb.x0
        for l in range(self.L):
            x = self._enc_layer(bb, l, x, T)
        self._ln(None, x, bb.mem, bb.encf_stats, "encoder.layer_norm", 0, (0, 0), None, rot=bb.xdec0, T=T, q8="mem")
        return bb.mem

    def decode(self, bb, mem, T, xdec0=None):
        """Decoder forward from `mem`; returns pred f32 [M, 64] (first out_dim valid)."""
        if xdec0 is None:
            K.rope(mem, self.D, bb.xdec0, self.D, bb.M, self.D, *self.rope(T, self.D), T, self.D, stream=self.st)
            xdec0 = bb.xdec0
        x = xdec0
        self._mem_q = (self._xq.get(mem.data_ptr()) or self._fp8_quant(mem, mem=True)) if self.fp8 else None
        self._kv_all_done = self._cross_kv_all(bb, mem, T)
        for l in range(self.L):
            x = self._dec_layer(bb, l, x, mem, T)
        self._ln(None, x, bb.xf, bb.decf_stats, "decoder.layer_norm", 0, (0, 0), None)
        pred = torch.empty(bb.M, 64, dtype=torch.float32, device=self.device)
        self.await_stage("head")
        self._gemm_fwd(bb.xf, "decoder.fc_output.weight", pred, K.EPI_BIAS)
        return pred

    def draw_seed(self):
        """Dropout seed of one forward: torch's RNG (so torch.manual_seed reproduces
        a run) mixed with the replica's rank."""
        if self.p <= 0:
            return 0
        return (int(torch.randint(0, 2 ** 62, (1,)).item()) + self.seed_salt * 0x9E3779B97F4A7C15) % (1 << 62)

    def forward(self, src, training, save):
        B, T, _ = src.shape
        self._prologue(training)
        self.base_seed = self.draw_seed()
        bb = self.bufs(B, T, save)
        mem = self.encode(bb, src, T)
        pred = self.decode(bb, mem, T, xdec0=bb.xdec0)
        if save:
            self.generation += 1
            self.saved = dict(bb=bb, T=T, p=self.p, seed=self.base_seed, gen=self.generation, x_src=self.x_src,
                              fp8_wt=self._fp8_wt_fresh)
        return pred[:, :self.out_dim].view(B, T, self.out_dim)

    # -------------------------------------------------------------- backward
    def backward(self, grad_pred, gen):
        sv = self.saved
        if gen != sv["gen"]:
            raise RuntimeError("Seq2Seq forward was run again before backward of an earlier forward")
        bb, T = sv["bb"], sv["T"]
        self.ensure_bound(versions=False)
        self.sync_pending()
        self.cur = bb
        self._main = torch.cuda.current_stream(self.device)
        self.st = self._main.cuda_stream
        if self.dw_stream_on and self._side is None:
            from .parallel import side_stream
            self._side = side_stream(self.device)
        self._side_reads = []
        self.p, self.base_seed = sv["p"], sv["seed"]
        self._dadd_pending = False
        self._red = None
        self._refresh_wt()
        bf = 0.0 if self.grads_fresh else 1.0
        self.sq_state = None
        self._sq_ok = self.fused_norm_on and self.dt == torch.bfloat16 and self.grad_reducer is None
        self._sq_used = 0
        if self._sq_ok and self._sq_buf is None:
            # + the rest-of-arena nstl_sumsq partials FusedAdam appends (sq_rest_partials per range)
            self._sq_buf = torch.empty(self.sq_tiles * 8 + self.sq_rest_partials * len(self.norm_rest),
                                       dtype=torch.float32, device=self.device)
        M, D, L = bb.M, self.D, self.L
        ws = bb.ws
        dres = bb.dres
        # head: pred = xf W^T + b
        g = grad_pred.reshape(M, self.out_dim)
        K.copy2d(g, g.stride(0), bb.dpred, 64, M, self.out_dim, 64, scale=self.grad_scale_t, stream=self.st)
        red = self.grad_reducer
        if red is not None:
            red.begin(self.grads_fresh)
        ready = (lambda name: self._ready(red, self.end_of[name])) if red is not None else (lambda name: None)
        dpred = bb.dpred[:, :self.out_dim]
        self._dw(dpred, bb.xf, "decoder.fc_output.weight", 1, bf, ws)
        K.gemm(bb.dpred, self.w("decoder.fc_output.weight"), dres, M, D, self.out_dim, a_kmajor=True,
               b_kmajor=False, lda=64, beta=0.0, stream=self.st)
        x_last = bb.layer(bb.d_x3, L - 1)
        self._ln_bwd(x_last, bb.decf_stats, "decoder.layer_norm", dres, dres, None, 0, (0, 0), bf)
        ready("decoder.layer_norm.bias")
        for l in reversed(range(L)):
            self._red_open()
            self._dec_layer_bwd(bb, l, T, bf, first=(l == L - 1))
            self._red_flush()
            ready("decoder.transformer_decoder.%d.self_attn.v_linear.bias" % l)
        if self.dmem_concat:
            # dmem = sum_l dkv_l W_kv_l = [dkv_0 | ... | dkv_{L-1}] [W_kv_0; ...; W_kv_{L-1}]:
            # one single-round GEMM with K = L * 2D (L accumulating K = 2D GEMMs each
            # read and wrote the f32 dmem, 128 MB per launch at the 228M shape)
            if self._wt_ok and ("kv", 0) in self._wt:
                Wt = self._wt[("kv", 0)]
                K.gemm(bb.dkv_all, Wt, bb.dmem, M, D, Wt.shape[1], a_kmajor=True, b_kmajor=True, beta=0.0,
                       stream=self.st)
            else:
                W = self._kv_weights()
                K.gemm(bb.dkv_all, W, bb.dmem, M, D, W.shape[0], a_kmajor=True, b_kmajor=False, beta=0.0,
                       stream=self.st)
        # decoder input x = GPE(mem): dmem += GPE^T(dres)
        cs, sn = self.rope(T, D)
        K.rope(dres, D, bb.dmem, D, M, D, cs, sn, T, D, inverse=True, accumulate=True, stream=self.st)
        x_last = bb.layer(bb.e_x2, L - 1)
        self._ln_bwd(x_last, bb.encf_stats, "encoder.layer_norm", bb.dmem, dres, None, 0, (0, 0), bf)
        ready("encoder.layer_norm.bias")
        # encoder weight gradients: one grouped launch per ENC_GROUP layers
        enc_group = self.dw_group_on and self._side is None
        for l in reversed(range(L)):
            if enc_group and self._defer is None:
                self._defer = []
            self._red_open()
            self._enc_layer_bwd(bb, l, T, bf, slot=(l % ENC_GROUP) if enc_group else None)
            self._red_flush()
            if enc_group and l % ENC_GROUP == 0:
                self._dw_flush(ws)
            if not enc_group or l % ENC_GROUP == 0:
                ready("encoder.transformer_encoder.%d.self_attn.v_linear.bias" % l)
        # embedding + global PE: x0 = GPE(src W^T + b)
        self._guard(bb.demb)
        K.rope(dres, D, bb.demb, D, M, D, cs, sn, T, D, inverse=True, stream=self.st)
        self._dw(bb.demb, sv["x_src"], "encoder.embedding.weight", 1, bf, ws)
        self._side_join()
        if red is not None:
            red.finish()
        self.grads_fresh = False
        if self._sq_ok and self._sq_used == self.sq_tiles * 8:
            self.sq_state = (self.g32._version, self._sq_used)

    def take_sq_partials(self):
        """The grouped dW launches' sums of squares of the last backward; consumed
        once.  Only valid when nothing wrote the gradient arena since that
        backward.  The version check catches in-place writes through a p.grad
        view, but NOT writers outside autograd's version counter (c10d
        collectives, ``.data`` aliases, kernels given g32 pointers): callers use
        this only when their own loop guarantees that (FusedAdam.
        trust_backward_norm), and every writer in this package calls
        invalidate_sq()."""
        st, self.sq_state = self.sq_state, None
        if st is None or st[0] != self.g32._version:
            return None
        return self._sq_buf[:st[1]]

    def invalidate_sq(self):
        """The gradient arena was written after backward: the epilogue partials no
        longer describe it (the next clip norm re-reads the arena)."""
        self.sq_state = None

    def _ready(self, red, upto):
        """Gradient arena prefix final: its all-reduce is ordered after both streams
        (the side stream waits for the main one and the collective follows it)."""
        if self._side is None:
            red.ready(upto)
            return
        self._side_begin()
        with torch.cuda.stream(self._side):
            red.ready(upto)

    def _attn_block_bwd(self, bb, pre, x_in, qkv, o, lse, st, s1, norm, seeds, T, bf, mask, last=False,
                        dy=None, dqkv=None):
        """Backward through x1 = LN(x_in + drop(drop(out_linear(attn(x_in))))) (self-attention)."""
        D, ws = self.D, bb.ws
        dy = bb.dy if dy is None else dy
        dqkv = bb.dqkv if dqkv is None else dqkv
        self._ln_bwd(s1, st, pre + norm, bb.dres, bb.dres, dy, 2, seeds[0:2], bf,
                     bias_of=pre + "self_attn.out_linear.bias")
        self._dw(dy, o, pre + "self_attn.out_linear.weight", 1, bf, ws, bias=False)
        self._dx(dy, pre + "self_attn.out_linear.weight", 1, bb.dattn, 0.0)
        fused = self._attn_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], o, lse, bb.dattn,
                               dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:], seeds[2], T, bb.B, mask=mask,
                               bias=[(0, 3 * D, self.gb(pre + "self_attn.q_linear.bias", 3))], bf=bf)
        self._dw(dqkv, x_in, pre + "self_attn.q_linear.weight", 3, bf, ws, bias=not fused)
        self._dx_res(dqkv, pre + "self_attn.q_linear.weight", 3, last=last)

    def _ffn_bwd(self, bb, pre, x_in, h, s_out, st, norm, seed_drop, bf, dy=None, rmask=None, dh=None):
        """Backward through x_out = LN(x_in + drop(FFN(x_in)))."""
        ws = self.cur.ws
        dy = bb.dy if dy is None else dy
        dh = bb.dh if dh is None else dh
        w2 = pre + "ffn.linear2.weight"
        dyq = self._fp8_dy_bufs(dy.shape[0]) if self.fp8 and self.fp8_bwd and self._fp8_wt \
            and w2 in self._fp8_wt and self.saved.get("fp8_wt", False) else None
        self._ln_bwd(s_out, st, pre + norm, bb.dres, bb.dres, dy, 1, (seed_drop, 0), bf,
                     bias_of=pre + "ffn.linear2.bias", q8=dyq)
        self._dw(dy, h, w2, 1, bf, ws, bias=False)
        fused = self._dx(dy, w2, 1, dh, 0.0, epi=K.EPI_DRELU_DROP, aux=h, p_drop=self.p,
                         colsum=(bb.hpart, self.gb(pre + "ffn.linear1.bias"), bf), relu_mask=rmask, dyq=dyq)
        self._dw(dh, x_in, pre + "ffn.linear1.weight", 1, bf, ws, bias=not fused)
        self._dx_res(dh, pre + "ffn.linear1.weight", 1)

    def _enc_layer_bwd(self, bb, l, T, bf, slot=None):
        """`slot`: this layer's weight gradients are queued for a grouped launch,
        so its dy / dh / dqkv live in per-slot buffers until then."""
        pre = "encoder.transformer_encoder.%d." % l
        sd = lambda s: _seed(self.base_seed, True, l, s)
        st = bb.e_stats[l]
        x_in = bb.x0 if l == 0 else bb.e_x2[l - 1]
        sl = (lambda lst: lst[slot]) if slot is not None else (lambda lst: None)
        self._ffn_bwd(bb, pre, bb.e_x1[l], bb.e_h[l], bb.e_s2[l], st[2:4], "norm2", sd("drop2"), bf,
                      rmask=bb.e_rmask[l] if bb.e_rmask_ok[l] else None, dy=sl(bb.g_dyf), dh=sl(bb.g_dh))
        self._attn_block_bwd(bb, pre, x_in, bb.e_qkv[l], bb.e_o[l], bb.e_lse[l], st[0:2], bb.e_s1[l], "norm1",
                             (sd("resid"), sd("drop1"), sd("attn")), T, bf, bb.e_mask[l], last=(l == 0),
                             dy=sl(bb.g_dyo), dqkv=sl(bb.g_dqkv))

    def _dec_layer_bwd(self, bb, l, T, bf, first):
        D, ws = self.D, bb.ws
        pre = "decoder.transformer_decoder.%d." % l
        sd = lambda s: _seed(self.base_seed, False, l, s)
        st = bb.d_stats[l]
        x_in = bb.xdec0 if l == 0 else bb.d_x3[l - 1]
        grouped = self.dw_group_on and self._side is None
        if grouped:
            self._defer = []
        self._ffn_bwd(bb, pre, bb.d_x2[l], bb.d_h[l], bb.d_s3[l], st[4:6], "norm3", sd("drop3"), bf,
                      dy=bb.dy_f if grouped else None, rmask=bb.d_rmask[l] if bb.d_rmask_ok[l] else None)
        # cross attention block: x2 = LN(x1 + drop(drop(out(attn(q(x1), kv(mem))))))
        m = pre + "multihead_attn."
        dyx = bb.dy_x if grouped else bb.dy
        self._ln_bwd(bb.d_s2[l], st[2:4], pre + "norm2", bb.dres, bb.dres, dyx, 2, (sd("xresid"), sd("drop2x")), bf,
                     bias_of=m + "out_linear.bias")
        self._dw(dyx, bb.d_oc[l], m + "out_linear.weight", 1, bf, ws, bias=False)
        self._dx(dyx, m + "out_linear.weight", 1, bb.dattn, 0.0)
        kvc = bb.d_kvc[l]
        dkv = bb.kv_grad(self, l)
        fused = self._attn_bwd(bb.d_qc[l], kvc[:, :D], kvc[:, D:], bb.d_oc[l], bb.d_lsec[l], bb.dattn,
                               bb.dq, dkv[:, :D], dkv[:, D:], sd("xattn"), T, bb.B, mask=bb.d_maskc[l],
                               bias=[(0, D, self.gb(m + "q_linear.bias")), (D, 2 * D, self.gb(m + "k_linear.bias", 2))],
                               bf=bf)
        self._dw(bb.dq, bb.d_x1[l], m + "q_linear.weight", 1, bf, ws, bias=not fused)
        self._dx_res(bb.dq, m + "q_linear.weight", 1)
        self._dw(dkv, bb.mem, m + "k_linear.weight", 2, bf, ws, bias=not fused)
        if not self.dmem_concat:
            self._dx(dkv, m + "k_linear.weight", 2, bb.dmem, 0.0 if first else 1.0)
        self._attn_block_bwd(bb, pre, x_in, bb.d_qkv[l], bb.d_o[l], bb.d_lse[l], st[0:2], bb.d_s1[l], "norm1",
                             (sd("resid"), sd("drop1"), sd("attn")), T, bf, bb.d_mask[l], last=(l == 0))
        if grouped:
            self._dw_flush(ws)


class Seq2SeqFunction(torch.autograd.Function):
    """Autograd node for the whole Seq2Seq: forward saves activations in the
    engine workspace; backward writes parameter gradients into the arena."""

    @staticmethod
    def forward(ctx, src, anchor, engine, training):
        pred = engine.forward(src, training, save=True)
        ctx.engine = engine
        ctx.gen = engine.generation
        return pred

    @staticmethod
    def backward(ctx, grad_pred):
        ctx.engine.backward(grad_pred, ctx.gen)
        return None, None, None, None
