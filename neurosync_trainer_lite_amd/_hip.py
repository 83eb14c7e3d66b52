"""ctypes bindings to libnstl_hip.so (C ABI declared in include/nstl.h).

The shared library is built in-tree (``python __graft_entry__.py`` / ``make -C
neurosync_trainer_lite_amd/csrc``).  There is no fallback: if the library is
missing or a call fails, a RuntimeError is raised.

torch must be imported before the library is loaded, so that the HIP runtime
torch already mapped (SONAME libamdhip64.so.7) is the one the library binds to.
"""
import ctypes
import os

import torch  # noqa: F401  (load order: torch's HIP runtime first)

# NSTL_LIB_PATH: A/B timing of another build of the same sources (tools/ only)
LIB_PATH = os.environ.get("NSTL_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                            "libnstl_hip.so")

F32, BF16, FP8 = 0, 1, 2
EPI_NONE, EPI_BIAS, EPI_BIAS_RELU_DROP, EPI_BIAS_ROPE, EPI_DRELU_DROP = 0, 1, 2, 3, 4

_vp = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_u64 = ctypes.c_uint64
_fp = ctypes.POINTER(ctypes.c_float)


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", _i32), ("c_dtype", _i32), ("a_kmajor", _i32), ("b_kmajor", _i32),
        ("A", _vp), ("lda", _i64), ("B", _vp), ("ldb", _i64), ("C", _vp), ("ldc", _i64),
        ("M", _i32), ("N", _i32), ("K", _i32),
        ("alpha", _f32), ("beta", _f32), ("epilogue", _i32),
        ("bias", _vp), ("aux", _vp), ("ld_aux", _i64),
        ("p_drop", _f32), ("seed", _u64),
        ("rope_cos", _vp), ("rope_sin", _vp), ("rope_T", _i32), ("rope_dim", _i32), ("rope_cols", _i32),
        ("split_k", _i32), ("workspace", _vp), ("workspace_bytes", _i64), ("colsum_part", _vp),
        ("relu_mask", _vp), ("a_scale", _vp), ("b_scale", _vp), ("sq_part", _vp),
    ]


class Fp8Job(ctypes.Structure):
    _fields_ = [("x", _vp), ("ldx", _i64), ("q", _vp), ("ldq", _i64), ("scale", _vp), ("rows", _i32), ("cols", _i32)]


FP8_BATCH_MAX = 64


class TransposeJob(ctypes.Structure):
    _fields_ = [("x", _vp), ("ldx", _i64), ("y", _vp), ("ldy", _i64), ("rows", _i32), ("cols", _i32)]


TRANSPOSE_BATCH_MAX = 64


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", _i32), ("B", _i32), ("T", _i32), ("H", _i32), ("dh", _i32),
        ("q", _vp), ("q_ld", _i64), ("k", _vp), ("k_ld", _i64), ("v", _vp), ("v_ld", _i64),
        ("o", _vp), ("o_ld", _i64), ("lse", _vp),
        ("p_drop", _f32), ("seed", _u64),
        ("dout", _vp), ("dout_ld", _i64), ("dq", _vp), ("dq_ld", _i64), ("dk", _vp), ("dk_ld", _i64),
        ("dv", _vp), ("dv_ld", _i64),
        ("rope_cos", _vp), ("rope_sin", _vp), ("rope_q", _i32), ("rope_k", _i32),
        ("dsum", _vp), ("mask_bits", _vp), ("dbias_part", _vp),
    ]


class LnArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", _i32), ("rows", _i32), ("D", _i32),
        ("x", _vp), ("y", _vp),
        ("n_masks", _i32), ("p_drop", _f32), ("seed1", _u64), ("seed2", _u64),
        ("gamma", _vp), ("beta", _vp), ("eps", _f32),
        ("s_out", _vp), ("out", _vp), ("mean", _vp), ("rstd", _vp),
        ("rot_out", _vp), ("rope_cos", _vp), ("rope_sin", _vp), ("rope_T", _i32),
        ("s_in", _vp), ("dout", _vp), ("ds", _vp), ("dbranch", _vp),
        ("dgamma_part", _vp), ("dbeta_part", _vp), ("n_part", _i32), ("dbranch_part", _vp), ("dout2", _vp),
        ("q8", _vp), ("ldq8", _i64), ("q8_scale", _vp),
    ]


class LossArgs(ctypes.Structure):
    _fields_ = [
        ("B", _i32), ("T", _i32), ("F", _i32),
        ("pred", _vp), ("pred_ld", _i64), ("trg", _vp), ("trg_ld", _i64),
        ("delta", _f32), ("w1", _f32), ("w2", _f32), ("w3", _f32), ("grad_scale", _f32),
        ("dpred", _vp), ("dpred_dtype", _i32), ("dpred_ld", _i64),
        ("partial", _vp), ("loss_out", _vp),
    ]


class AdamArgs(ctypes.Structure):
    _fields_ = [
        ("p", _vp), ("g", _vp), ("m", _vp), ("v", _vp),
        ("p_lowp", _vp), ("lowp_dtype", _i32), ("n", _i64),
        ("lr", _f32), ("beta1", _f32), ("beta2", _f32), ("eps", _f32), ("weight_decay", _f32),
        ("step", _i32), ("sumsq_partial", _vp), ("n_partial", _i32), ("max_norm", _f32), ("norm_out", _vp),
        ("coef", _vp),
    ]


class ReduceJob(ctypes.Structure):
    _fields_ = [("part", _vp), ("ld", _i64), ("n_part", _i32), ("cols", _i32), ("out", _vp), ("beta", _f32)]


REDUCE_BATCH_MAX = 16

# every symbol include/nstl.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "nstl_gemm", "nstl_gemm_grouped", "nstl_gemm_colsum_rows", "nstl_gemm_relu_mask_words",
    "nstl_gemm_workspace_bytes",
    "nstl_attn_fwd", "nstl_attn_bwd", "nstl_attn_bias_rows", "nstl_ln_fwd", "nstl_ln_bwd",
    "nstl_reduce_rows", "nstl_reduce_rows_strided", "nstl_reduce_rows3", "nstl_reduce_rows_batch",
    "nstl_colsum", "nstl_rope",
    "nstl_loss_fwd_bwd", "nstl_sumsq", "nstl_adam_step", "nstl_clip_coef", "nstl_cast", "nstl_copy2d", "nstl_autocorr",
    "nstl_features", "nstl_stft_mel", "nstl_features_workspace_bytes", "nstl_features_frames", "nstl_last_error_string",
    "nstl_version", "nstl_fp8_quant_rows", "nstl_fp8_quant_cols", "nstl_kernel_counts", "nstl_kernel_counts_reset",
    "nstl_cmvn_delta_reduce", "nstl_reduce_frame_pairs", "nstl_transpose_bf16", "nstl_stream_cus", "nstl_mask_grid",
    "nstl_ipc_handle", "nstl_ipc_open", "nstl_ipc_close", "nstl_copy_engine", "nstl_shard_sum",
]
IPC_HANDLE_BYTES = 64

# nstl_kernel_counts order (NSTL_K_* in include/nstl.h)
KERNEL_COUNT_NAMES = ["gemm128", "gemm_ring", "gemm_ring_tiles", "gemm_group", "gemm_group_tiles",
                      "gemm_splitk_reduce", "gemm_fp8", "attn_fwd", "attn_fwd_generic", "attn_bwd_fused",
                      "attn_bwd_split", "attn_bwd_generic", "gemm4", "gemm4_tiles", "gemm4_sk", "gemm_fp8_rope", "gemm4_fp8"]

_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the library is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libnstl_hip.so not found at %s: build it with `python __graft_entry__.py` "
                "(make -C neurosync_trainer_lite_amd/csrc). There is no CPU fallback." % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        P = ctypes.POINTER
        L.nstl_gemm.argtypes = [P(GemmArgs), _vp]
        L.nstl_gemm_grouped.argtypes = [P(GemmArgs), _i32, _vp]
        L.nstl_fp8_quant_rows.argtypes = [_i32, P(Fp8Job), _i32, _vp]
        L.nstl_fp8_quant_cols.argtypes = [_i32, P(Fp8Job), _i32, _vp]
        L.nstl_transpose_bf16.argtypes = [P(TransposeJob), _i32, _vp]
        L.nstl_gemm_colsum_rows.argtypes = [P(GemmArgs)]
        L.nstl_gemm_colsum_rows.restype = _i32
        L.nstl_gemm_relu_mask_words.argtypes = [P(GemmArgs)]
        L.nstl_gemm_relu_mask_words.restype = _i64
        L.nstl_gemm_workspace_bytes.argtypes = [_i32, _i32, _i32]
        L.nstl_gemm_workspace_bytes.restype = _i64
        L.nstl_attn_fwd.argtypes = [P(AttnArgs), _vp]
        L.nstl_attn_bwd.argtypes = [P(AttnArgs), _vp]
        L.nstl_attn_bias_rows.argtypes = [P(AttnArgs)]
        L.nstl_attn_bias_rows.restype = _i32
        L.nstl_ln_fwd.argtypes = [P(LnArgs), _vp]
        L.nstl_ln_bwd.argtypes = [P(LnArgs), _vp]
        L.nstl_reduce_rows.argtypes = [_vp, _i32, _i32, _vp, _f32, _vp]
        L.nstl_reduce_rows_strided.argtypes = [_vp, _i64, _i32, _i32, _vp, _f32, _vp]
        L.nstl_reduce_rows3.argtypes = [_vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _f32, _vp]
        L.nstl_reduce_rows_batch.argtypes = [P(ReduceJob), _i32, _vp]
        L.nstl_colsum.argtypes = [_i32, _vp, _i64, _i32, _i32, _vp, _vp, _f32, _vp]
        L.nstl_rope.argtypes = [_i32, _vp, _i64, _i32, _vp, _i64, _i32, _i32, _vp, _vp, _i32, _i32, _i32, _i32, _vp]
        L.nstl_loss_fwd_bwd.argtypes = [P(LossArgs), _vp]
        L.nstl_sumsq.argtypes = [_vp, _i64, _vp, _i32, _vp]
        L.nstl_adam_step.argtypes = [P(AdamArgs), _vp]
        L.nstl_clip_coef.argtypes = [_vp, _i32, _f32, _vp, _vp, _vp]
        L.nstl_cast.argtypes = [_i32, _vp, _i32, _vp, _i64, _vp]
        L.nstl_copy2d.argtypes = [_i32, _vp, _i64, _i32, _vp, _i64, _i32, _i32, _i32, _vp, _vp]
        L.nstl_autocorr.argtypes = [_vp, _i64, _i32, _i32, _i32, _vp, _i32, _vp]
        L.nstl_features.argtypes = [_vp, _i64, _i32, _vp, _i64, _i32, _vp, _i64, _vp]
        L.nstl_stft_mel.argtypes = [_vp, _i64, _i32, _vp, _i32, _vp]
        L.nstl_features_workspace_bytes.argtypes = [_i64, _i32]
        L.nstl_features_workspace_bytes.restype = _i64
        L.nstl_features_frames.argtypes = [_i64, _i32]
        L.nstl_features_frames.restype = _i32
        L.nstl_last_error_string.restype = ctypes.c_char_p
        L.nstl_version.restype = _i32
        L.nstl_cmvn_delta_reduce.argtypes = [_vp, _i32, _i32, _vp, _i64, _vp]
        L.nstl_reduce_frame_pairs.argtypes = [_vp, _i32, _i32, _vp, _i64, _i32, _vp]
        L.nstl_kernel_counts.argtypes = [_vp, _i32]
        L.nstl_kernel_counts.restype = _i32
        L.nstl_kernel_counts_reset.restype = None
        L.nstl_stream_cus.argtypes = [_vp]
        L.nstl_stream_cus.restype = _i32
        L.nstl_mask_grid.argtypes = [_vp, _i32]
        L.nstl_mask_grid.restype = _i32
        L.nstl_ipc_handle.argtypes = [_vp, _vp, ctypes.POINTER(_i64)]
        L.nstl_ipc_open.argtypes = [_vp, ctypes.POINTER(_vp)]
        L.nstl_ipc_close.argtypes = [_vp]
        L.nstl_copy_engine.argtypes = [_vp, _vp, _i64, _vp]
        L.nstl_shard_sum.argtypes = [_vp, _vp, _i64, _i32, _i64, _vp, _vp, _i32, _vp]
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().nstl_last_error_string().decode(errors="replace")
        raise RuntimeError("%s failed (code %d): %s" % (what, rc, msg))


def cmvn_delta_reduce(x, out, stream=None):
    """x f32 [ncoef, F] (device) -> out f32 [(F+1)/2, >= 3 ncoef] (nstl_cmvn_delta_reduce)."""
    ncoef, F = x.shape
    check(lib().nstl_cmvn_delta_reduce(x.data_ptr(), ncoef, F, out.data_ptr(), out.stride(0),
                                       stream if stream is not None else stream_of()), "nstl_cmvn_delta_reduce")


def reduce_frame_pairs(x, out, col0=0, stream=None):
    """x f64 [F, cols] (device) -> out f32 [(F+1)/2, >= col0 + cols] (nstl_reduce_frame_pairs)."""
    F, cols = x.shape
    check(lib().nstl_reduce_frame_pairs(x.data_ptr(), F, cols, out.data_ptr(), out.stride(0), col0,
                                        stream if stream is not None else stream_of()), "nstl_reduce_frame_pairs")


def kernel_counts():
    """{family: launches} since the last kernel_counts_reset() (nstl_kernel_counts)."""
    n = len(KERNEL_COUNT_NAMES)
    buf = (ctypes.c_int64 * n)()
    total = lib().nstl_kernel_counts(ctypes.cast(buf, _vp), n)
    if total != n and not os.environ.get("NSTL_LIB_PATH"):
        raise RuntimeError("nstl_kernel_counts: library has %d counters, bindings %d" % (total, n))
    # an older build loaded for an A/B (NSTL_LIB_PATH) may have fewer: the rest read 0
    return dict(zip(KERNEL_COUNT_NAMES, buf))


def kernel_counts_reset():
    lib().nstl_kernel_counts_reset()


def mask_grid(excluded, ncu=256):
    """nstl_mask_grid: the persistent grid a CU mask clearing `excluded` bits allows."""
    words = (ncu + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for c in range(ncu):
        if c not in excluded:
            m[c // 32] |= 1 << (c % 32)
    return lib().nstl_mask_grid(m, ncu)


def stream_cus(stream=None):
    """Persistent-grid workgroups for `stream` (nstl_stream_cus: its CU mask, balanced over the XCDs)."""
    return lib().nstl_stream_cus(stream if stream is not None else stream_of())


def ptr(t):
    """Device pointer of a tensor (or None)."""
    return None if t is None else t.data_ptr()


def stream_of(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float8_e4m3fn:
        return FP8
    raise TypeError("unsupported dtype %s (float32 / bfloat16 / float8_e4m3fn)" % dt)


# ---------------------------------------------------------------------------
# thin call wrappers
# ---------------------------------------------------------------------------
def gemm(A, B, C, M, N, K, *, stream=None, **kw):
    """C[i,j] = alpha sum_r A(i,r) B(j,r) (+beta C) + epilogue.  See include/nstl.h."""
    a = gemm_args(A, B, C, M, N, K, **kw)
    check(lib().nstl_gemm(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_gemm")


def gemm_relu_mask_words(A, B, C, M, N, K, **kw):
    """64-bit words nstl_gemm would read/write as relu_mask for these arguments (0: unsupported)."""
    return lib().nstl_gemm_relu_mask_words(ctypes.byref(gemm_args(A, B, C, M, N, K, **kw)))


def gemm_colsum_rows(A, B, C, M, N, K, **kw):
    """Partial rows nstl_gemm would write to colsum_part for these arguments (0: unsupported)."""
    return lib().nstl_gemm_colsum_rows(ctypes.byref(gemm_args(A, B, C, M, N, K, **kw)))


GEMM_GROUP_MAX = 16


def gemm_grouped(problems, stream=None):
    """Independent GEMMs in one launch (nstl_gemm_grouped): `problems` is a list of
    (A, B, C, M, N, K, kwargs) with the gemm() keyword arguments."""
    arr = (GemmArgs * len(problems))()
    for i, (A, B, C, M, N, K, kw) in enumerate(problems):
        arr[i] = gemm_args(A, B, C, M, N, K, **kw)
    check(lib().nstl_gemm_grouped(arr, len(problems), stream if stream is not None else stream_of()),
          "nstl_gemm_grouped")


# ---------------------------------------------------------------------------
# operand extents: every tensor handed to a kernel must hold the last element
# the call addresses (the kernels take plain pointers and strides and do not
# know the allocation: an oversize M, K or ld would read or write past it)
# ---------------------------------------------------------------------------
def _room(t):
    """Bytes from t.data_ptr() to the end of its storage."""
    st = t.untyped_storage()
    return st.data_ptr() + st.nbytes() - t.data_ptr()


def _need(t, last, what):
    """t must hold element index `last` (in t's element size) past its first."""
    if t is None or last < 0:
        return
    if (last + 1) * t.element_size() > _room(t):
        raise ValueError("%s: the call addresses element %d but the tensor's storage holds %d from its start"
                         % (what, last, _room(t) // t.element_size()))


def _need_mat(t, rows, cols, ld, what):
    """A row-major [rows][cols] operand with row stride ld (elements): its last
    addressed element lies inside the storage.  (Stride rules -- ld >= cols, the
    alignments -- are the library's own argument checks.)"""
    if rows > 0 and cols > 0:
        _need(t, (rows - 1) * ld + cols - 1, what)


def _ceil(x, m):
    return (x + m - 1) // m * m


def gemm_check(A, B, C, M, N, K, a):
    """Extents of every operand of one nstl_gemm call (a: the filled GemmArgs)."""
    if M <= 0 or N <= 0 or K <= 0:
        raise ValueError("nstl_gemm: empty problem %dx%dx%d" % (M, N, K))
    vec = 16 // A.element_size()  # K-major rows are read in 16-byte chunks
    if a.a_kmajor:
        _need_mat(A, M, _ceil(K, vec), a.lda, "nstl_gemm A [M][K]")
    else:
        _need_mat(A, K, _ceil(M, vec), a.lda, "nstl_gemm A [K][M]")
    if a.b_kmajor:
        _need_mat(B, N, _ceil(K, vec), a.ldb, "nstl_gemm B [N][K]")
    else:
        _need_mat(B, K, _ceil(N, vec), a.ldb, "nstl_gemm B [K][N]")
    _need_mat(C, M, N, a.ldc, "nstl_gemm C [M][N]")


def _check_side(t, n, what):
    if t is not None:
        _need(t, n - 1, what)


def gemm_args(A, B, C, M, N, K, *, a_kmajor=True, b_kmajor=True, lda=None, ldb=None, ldc=None,
              alpha=1.0, beta=0.0, epilogue=EPI_NONE, bias=None, aux=None, ld_aux=0, p_drop=0.0, seed=0,
              rope=None, rope_cols=0, split_k=1, workspace=None, colsum_part=None, relu_mask=None,
              a_scale=None, b_scale=None, sq_part=None):
    """The GemmArgs of one call, with every operand's extent checked against the
    tensor's storage (ValueError before anything is launched)."""
    a = GemmArgs()
    a.dtype = dtype_code(A.dtype)
    a.c_dtype = dtype_code(C.dtype)
    a.a_kmajor, a.b_kmajor = int(a_kmajor), int(b_kmajor)
    a.A, a.B, a.C = A.data_ptr(), B.data_ptr(), C.data_ptr()
    a.lda = lda if lda is not None else A.stride(-2) if A.dim() > 1 else K
    a.ldb = ldb if ldb is not None else B.stride(-2) if B.dim() > 1 else K
    a.ldc = ldc if ldc is not None else C.stride(-2)
    a.M, a.N, a.K = M, N, K
    a.alpha, a.beta = alpha, beta
    a.epilogue = epilogue
    a.bias = ptr(bias)
    a.aux = ptr(aux)
    a.ld_aux = ld_aux
    a.p_drop = p_drop
    a.seed = seed & 0xFFFFFFFFFFFFFFFF
    if rope is not None:
        cos_t, sin_t, rT, rdim = rope
        a.rope_cos, a.rope_sin, a.rope_T, a.rope_dim = cos_t.data_ptr(), sin_t.data_ptr(), rT, rdim
        a.rope_cols = rope_cols
    a.split_k = split_k
    if workspace is not None:
        a.workspace = workspace.data_ptr()
        a.workspace_bytes = workspace.numel() * workspace.element_size()
    a.colsum_part = ptr(colsum_part)
    a.relu_mask = ptr(relu_mask)
    a.a_scale, a.b_scale = ptr(a_scale), ptr(b_scale)
    a.sq_part = ptr(sq_part)
    gemm_check(A, B, C, M, N, K, a)
    _check_side(bias, N, "nstl_gemm bias [N]")
    if aux is not None:
        _need_mat(aux, M, N, ld_aux, "nstl_gemm aux [M][ld_aux]")
    if rope is not None:
        _check_side(rope[0], rT * (rdim // 2), "nstl_gemm rope_cos [T][dim/2]")
        _check_side(rope[1], rT * (rdim // 2), "nstl_gemm rope_sin [T][dim/2]")
    _check_side(relu_mask, ((M + 63) // 64) * 8 * ((N + 7) // 8), "nstl_gemm relu_mask words")
    _check_side(colsum_part, ((M + 127) // 128) * N, "nstl_gemm colsum_part [M/128][N]")
    _check_side(sq_part, ((M + 255) // 256) * ((N + 255) // 256) * 8, "nstl_gemm sq_part [tiles][8]")
    _check_side(a_scale, M, "nstl_gemm a_scale [M]")
    _check_side(b_scale, N, "nstl_gemm b_scale [N]")
    return a


def _fp8_jobs(fn, jobs, stream, what):
    if not jobs:
        return
    dt = jobs[0][0].dtype
    for lo in range(0, len(jobs), FP8_BATCH_MAX):
        chunk = jobs[lo:lo + FP8_BATCH_MAX]
        arr = (Fp8Job * len(chunk))()
        for i, (x, rows, cols, q, scale) in enumerate(chunk):
            if x.dtype != dt or q.dtype != torch.float8_e4m3fn or scale.dtype != torch.float32:
                raise TypeError("%s: x of one dtype, q float8_e4m3fn, scale float32" % what)
            arr[i] = Fp8Job(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0), scale.data_ptr(), rows, cols)
        check(fn(dtype_code(dt), arr, len(chunk), stream if stream is not None else stream_of()), what)


def fp8_quant_rows(jobs, stream=None):
    """Row-wise e4m3 quantization (nstl_fp8_quant_rows): `jobs` is a list of
    (x, rows, cols, q, scale) with x f32/bf16 [rows, >= cols], q float8_e4m3fn
    [rows, >= cols] and scale f32 [rows]; all jobs share x's dtype."""
    _fp8_jobs(lib().nstl_fp8_quant_rows, jobs, stream, "nstl_fp8_quant_rows")


def fp8_quant_cols(jobs, stream=None):
    """Column-wise (transposed) e4m3 quantization (nstl_fp8_quant_cols): jobs
    (x, rows, cols, q, scale) with x [rows, >= cols], q float8_e4m3fn [cols, >= rows]
    = quant_rows(x^T), scale f32 [cols]."""
    _fp8_jobs(lib().nstl_fp8_quant_cols, jobs, stream, "nstl_fp8_quant_cols")


def transpose_bf16(jobs, stream=None):
    """Batched bf16 transpose (nstl_transpose_bf16): jobs (x, y) with x bf16
    [rows, cols] (row stride >= cols) and y bf16 [cols, rows] (row stride >= rows)."""
    for lo in range(0, len(jobs), TRANSPOSE_BATCH_MAX):
        chunk = jobs[lo:lo + TRANSPOSE_BATCH_MAX]
        arr = (TransposeJob * len(chunk))()
        for i, (x, y) in enumerate(chunk):
            if x.dtype != torch.bfloat16 or y.dtype != torch.bfloat16 or y.shape != (x.shape[1], x.shape[0]):
                raise TypeError("nstl_transpose_bf16: x bf16 [r, c] and y bf16 [c, r]")
            arr[i] = TransposeJob(x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), x.shape[0], x.shape[1])
        check(lib().nstl_transpose_bf16(arr, len(chunk), stream if stream is not None else stream_of()),
              "nstl_transpose_bf16")


def attn_args(dtype, B, T, H, q, q_ld, k, k_ld, v, v_ld, o, o_ld, lse, p_drop, seed, dh=64):
    a = AttnArgs()
    a.dtype = dtype
    a.B, a.T, a.H, a.dh = B, T, H, dh
    a.q, a.q_ld, a.k, a.k_ld, a.v, a.v_ld = q, q_ld, k, k_ld, v, v_ld
    a.o, a.o_ld, a.lse = o, o_ld, lse
    a.p_drop, a.seed = p_drop, seed & 0xFFFFFFFFFFFFFFFF
    return a


def attn_set(a, **ops):
    """Point the AttnArgs `a` (attn_args) at tensors, each checked against the
    extent the call addresses: q, k, v, o, dout, dq, dk, dv (row stride from the
    tensor, B*T rows of H*dh), lse / dsum ([B*H*T] f32), mask_bits ([B*H*T*T/64]
    words), rope_cos / rope_sin ([T][dh/2] f32), dbias_part ([rows][3*H*dh] f32,
    rows = attn_bias_rows)."""
    rows, cols = a.B * a.T, a.H * a.dh
    for name, t in ops.items():
        if t is None:
            setattr(a, name, None)
            continue
        if name in ("q", "k", "v", "o", "dout", "dq", "dk", "dv"):
            ld = t.stride(0)
            _need_mat(t, rows, cols, ld, "nstl_attn %s [B*T][H*dh]" % name)
            setattr(a, name + "_ld", ld)
        elif name in ("lse", "dsum"):
            _check_side(t, a.B * a.H * a.T, "nstl_attn %s [B*H*T]" % name)
        elif name == "mask_bits":
            _check_side(t, a.B * a.H * a.T * a.T // 64, "nstl_attn mask_bits [B*H*T*T/64]")
        elif name in ("rope_cos", "rope_sin"):
            _check_side(t, a.T * (a.dh // 2), "nstl_attn %s [T][dh/2]" % name)
        elif name == "dbias_part":
            _check_side(t, attn_bias_rows(a) * 3 * cols, "nstl_attn dbias_part [rows][3*H*dh]")
        else:
            raise TypeError("attn_set: unknown operand %r" % name)
        setattr(a, name, t.data_ptr())
    return a


def attn_bias_rows(a):
    return lib().nstl_attn_bias_rows(ctypes.byref(a))


def attn_fwd(a, stream=None):
    check(lib().nstl_attn_fwd(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_attn_fwd")


def attn_bwd(a, stream=None):
    check(lib().nstl_attn_bwd(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_attn_bwd")


def ln_fwd(a, stream=None):
    check(lib().nstl_ln_fwd(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_ln_fwd")


def ln_bwd(a, stream=None):
    check(lib().nstl_ln_bwd(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_ln_bwd")


def reduce_rows3(part, n_part, cols, outs, beta, stream=None):
    """part: [n_mat][rows >= n_part][cols] f32; outs: n_mat f32 vectors."""
    ptrs = [o.data_ptr() for o in outs] + [None] * (3 - len(outs))
    check(lib().nstl_reduce_rows3(part.data_ptr(), part.stride(0), len(outs), n_part, cols, ptrs[0], ptrs[1], ptrs[2],
                                  beta, stream if stream is not None else stream_of()), "nstl_reduce_rows3")


def reduce_rows_batch(jobs, stream=None):
    """jobs: (part, ld, n_part, cols, out, beta) with part a tensor (its first
    element is row 0, column 0 of the job) and out an f32 tensor; one launch."""
    if not jobs:
        return
    if len(jobs) > REDUCE_BATCH_MAX:
        raise RuntimeError("nstl_reduce_rows_batch: at most %d jobs (got %d)" % (REDUCE_BATCH_MAX, len(jobs)))
    arr = (ReduceJob * len(jobs))(*[ReduceJob(ptr(part), ld, n_part, cols, out.data_ptr(), beta)
                                    for part, ld, n_part, cols, out, beta in jobs])
    check(lib().nstl_reduce_rows_batch(arr, len(jobs), stream if stream is not None else stream_of()),
          "nstl_reduce_rows_batch")


def reduce_rows(part, n_part, cols, out, beta, stream=None):
    check(lib().nstl_reduce_rows(part.data_ptr(), n_part, cols, out.data_ptr(), beta,
                                 stream if stream is not None else stream_of()), "nstl_reduce_rows")


def reduce_rows_strided(part, ld, n_part, cols, out, beta, stream=None):
    """out (+)= column sums of part[:n_part, :cols] (f32, rows ld floats apart; part
    may be a column-offset view)."""
    check(lib().nstl_reduce_rows_strided(part.data_ptr(), ld, n_part, cols, out.data_ptr(), beta,
                                         stream if stream is not None else stream_of()), "nstl_reduce_rows_strided")


def colsum(x, ld, rows, cols, partial, out, beta, stream=None):
    check(lib().nstl_colsum(dtype_code(x.dtype), x.data_ptr(), ld, rows, cols, partial.data_ptr(), out.data_ptr(),
                            beta, stream if stream is not None else stream_of()), "nstl_colsum")


def rope(inp, in_ld, out, out_ld, rows, cols, cos_t, sin_t, T, rope_dim, inverse=False, accumulate=False,
         stream=None):
    check(lib().nstl_rope(dtype_code(inp.dtype), inp.data_ptr(), in_ld, dtype_code(out.dtype), out.data_ptr(), out_ld,
                          rows, cols, cos_t.data_ptr(), sin_t.data_ptr(), T, rope_dim, int(inverse), int(accumulate),
                          stream if stream is not None else stream_of()), "nstl_rope")


def loss_fwd_bwd(a, stream=None):
    check(lib().nstl_loss_fwd_bwd(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_loss_fwd_bwd")


def sumsq(g, n, partial, n_partial, stream=None):
    check(lib().nstl_sumsq(g.data_ptr(), n, partial.data_ptr(), n_partial,
                           stream if stream is not None else stream_of()), "nstl_sumsq")


def clip_coef(partial, n_partial, max_norm, coef, norm_out=None, stream=None):
    check(lib().nstl_clip_coef(partial.data_ptr(), n_partial, float(max_norm), coef.data_ptr(),
                               norm_out.data_ptr() if norm_out is not None else None,
                               stream if stream is not None else stream_of()), "nstl_clip_coef")


def ipc_handle(t):
    """The 64-byte IPC handle of the allocation holding device tensor t
    (nstl_ipc_handle) and t's byte offset in it."""
    h = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    off = _i64()
    check(lib().nstl_ipc_handle(t.data_ptr(), h, ctypes.byref(off)), "nstl_ipc_handle")
    return h.raw, off.value


def ipc_open(handle):
    """Map another process's allocation (nstl_ipc_open); returns its base pointer."""
    p = _vp()
    check(lib().nstl_ipc_open(ctypes.create_string_buffer(handle, IPC_HANDLE_BYTES), ctypes.byref(p)), "nstl_ipc_open")
    return p.value


def ipc_close(ptr):
    check(lib().nstl_ipc_close(ptr), "nstl_ipc_close")


def copy_engine(dst_ptr, src, nbytes, stream=None):
    """nbytes from device tensor src to the device address dst_ptr on the copy
    engines (nstl_copy_engine: no kernel)."""
    if not src.is_contiguous() or nbytes > src.numel() * src.element_size():
        raise ValueError("copy_engine: %d bytes past the (contiguous) source tensor" % nbytes)
    check(lib().nstl_copy_engine(dst_ptr, src.data_ptr(), nbytes, stream if stream is not None else stream_of()),
          "nstl_copy_engine")


def shard_sum(own, slots, n_slots, out, partial, n_partial, stream=None):
    """out = own + slots[0] + ... (slot order) and the sum-of-squares partials of
    out (nstl_shard_sum).  own / out f32 [n]; slots f32 [n_slots][ld >= n]."""
    n = own.numel()
    ld = slots.stride(0) if n_slots else n
    if out.numel() < n or (n_slots and (slots.shape[0] < n_slots or slots.shape[1] < n)):
        raise ValueError("shard_sum: operand sizes")
    _check_side(partial, n_partial, "nstl_shard_sum partial")
    check(lib().nstl_shard_sum(own.data_ptr(), slots.data_ptr() if n_slots else None, ld, n_slots, n, out.data_ptr(),
                               partial.data_ptr(), n_partial, stream if stream is not None else stream_of()),
          "nstl_shard_sum")


def stft_mel(y, n_samples, sr, mel, n_frames, stream=None):
    """Fused STFT -> power -> mel power [n_frames][128] (nstl_stft_mel)."""
    check(lib().nstl_stft_mel(y.data_ptr(), n_samples, sr, mel.data_ptr(), n_frames,
                              stream if stream is not None else stream_of()), "nstl_stft_mel")


def adam_step(a, stream=None):
    check(lib().nstl_adam_step(ctypes.byref(a), stream if stream is not None else stream_of()), "nstl_adam_step")


def cast(src, dst, n=None, stream=None):
    n = src.numel() if n is None else n
    check(lib().nstl_cast(dtype_code(src.dtype), src.data_ptr(), dtype_code(dst.dtype), dst.data_ptr(), n,
                          stream if stream is not None else stream_of()), "nstl_cast")


def copy2d(src, src_ld, dst, dst_ld, rows, cols, dst_cols, scale=None, stream=None):
    check(lib().nstl_copy2d(dtype_code(src.dtype), src.data_ptr(), src_ld, dtype_code(dst.dtype), dst.data_ptr(),
                            dst_ld, rows, cols, dst_cols, ptr(scale), stream if stream is not None else stream_of()),
          "nstl_copy2d")


def autocorr(y, frame_length, hop_length, n_lags, out, n_frames, stream=None):
    check(lib().nstl_autocorr(y.data_ptr(), y.numel(), frame_length, hop_length, n_lags, out.data_ptr(), n_frames,
                              stream if stream is not None else stream_of()), "nstl_autocorr")


def features_frames(n_samples, sr):
    return lib().nstl_features_frames(n_samples, sr)


def features_workspace_bytes(n_samples, sr):
    return lib().nstl_features_workspace_bytes(n_samples, sr)


def features(y, sr, out, workspace, stream=None):
    """y: f32 [S] on the device -> out f32 [F60, >=256] (see include/nstl.h)."""
    check(lib().nstl_features(y.data_ptr(), y.numel(), sr, out.data_ptr(), out.stride(0), out.shape[0],
                              workspace.data_ptr(), workspace.numel() * workspace.element_size(),
                              stream if stream is not None else stream_of()), "nstl_features")
