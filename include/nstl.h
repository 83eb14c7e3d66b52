/*
 * nstl.h — C ABI of libnstl_hip.so, the MI355X (gfx950) kernels behind the
 * NeuroSync Trainer Lite training hot path.
 *
 * The reference (wolfi/NeuroSync_Trainer_Lite) has no native code and no FFI:
 * its hot path is PyTorch eager.  Each entry point below replaces the PyTorch
 * op(s) the reference dispatches to at the cited file:line; the Python host
 * layer (neurosync_trainer_lite_amd/, loaded with ctypes) keeps the reference's
 * module/function surface on top of it.
 *
 * Conventions
 *   - plain pointers + sizes; every buffer is caller-owned (device memory);
 *     no allocation inside any call; scratch comes in via *workspace.
 *   - `stream` is a hipStream_t passed as void*; every launch goes on it.
 *   - return 0 on success, a hipError_t value otherwise (1 = invalid value);
 *     nstl_last_error_string() describes the last failure on this thread.
 *   - dtype codes: NSTL_F32 = 0, NSTL_BF16 = 1, NSTL_FP8 = 2 (GEMM operands
 *     only: OCP e4m3 bytes + f32 row scales, see nstl_fp8_quant_rows).
 *     Row-major everywhere.
 */
#ifndef NSTL_H
#define NSTL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { NSTL_F32 = 0, NSTL_BF16 = 1, NSTL_FP8 = 2 };

enum {
  NSTL_EPI_NONE = 0,           /* C = alpha*acc + beta*C                        */
  NSTL_EPI_BIAS = 1,           /* + bias[j]                                     */
  NSTL_EPI_BIAS_RELU_DROP = 2, /* dropout(relu(acc + bias))                     */
  NSTL_EPI_BIAS_ROPE = 3,      /* rotate pairs of (acc + bias), cols < rope_cols */
  NSTL_EPI_DRELU_DROP = 4      /* acc * (aux[i,j] > 0) / (1-p)  (backward)       */
};

/* C[i,j] = alpha * sum_r A(i,r) B(j,r)  (+ beta*C, + epilogue).
 *   a_kmajor: A stored [M][K] (r contiguous) else [K][M];
 *   b_kmajor: B stored [N][K] else [K][N].
 * Replaces nn.Linear forward/backward GEMMs: utils/model.py:113-115,138
 * (MultiHeadAttention q/k/v/out_linear), :154,:157 (FeedForwardNetwork),
 * :216/:224 (Encoder.embedding), :242/:251 (Decoder.fc_output); the bias+ReLU+
 * dropout epilogue replaces F.relu + nn.Dropout at :155-156, the RoPE epilogue
 * replaces apply_rope_qk (:60-83) and GlobalPositionalEncoding (:29-53). */
typedef struct nstl_gemm_args {
  int dtype;      /* element type of A and B */
  int c_dtype;    /* element type of C */
  int a_kmajor, b_kmajor;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  int M, N, K;
  float alpha, beta;
  int epilogue;
  const float* bias;                   /* [N] f32 */
  const void* aux; int64_t ld_aux;     /* DRELU_DROP: saved post-dropout activation (dtype) */
  float p_drop; uint64_t seed;         /* BIAS_RELU_DROP / DRELU_DROP */
  const float* rope_cos; const float* rope_sin; /* [rope_T][rope_dim/2] f32 */
  int rope_T, rope_dim, rope_cols;
  int split_k;                         /* >1: f32 partials in workspace, then reduce */
  void* workspace; int64_t workspace_bytes;
  float* colsum_part;                  /* optional [nstl_gemm_colsum_rows()][N] f32: per-128-row
                                          column sums of C as stored (DRELU_DROP on the 256
                                          kernel: the FFN1 bias gradient before nstl_reduce_rows) */
  uint64_t* relu_mask;                 /* optional [nstl_gemm_relu_mask_words()]: BIAS_RELU_DROP
                                          writes, DRELU_DROP reads (instead of aux) the bits
                                          "kept and positive" of the FFN hidden, 1 bit/element */
  const float* a_scale;                /* dtype NSTL_FP8: f32 row scales of A [M] and of B [N]   */
  const float* b_scale;                /* (nstl_fp8_quant_rows); C = a_scale[i] b_scale[j] acc   */
  float* sq_part;                      /* optional, nstl_gemm_grouped with f32 C only: [tiles][8] f32,
                                          tile t = its 256x256 tile index in the problem (row-major over
                                          ceil(M/256) x ceil(N/256)): the sums of squares of C as stored,
                                          one per wave -- the weight gradients' share of clip_grad_norm_
                                          (utils/training_utils.py:73) without re-reading them */
} nstl_gemm_args;
int nstl_gemm(const nstl_gemm_args* args, void* stream);
/* Rows of colsum_part for these arguments, or 0 when the call cannot produce it. */
int nstl_gemm_colsum_rows(const nstl_gemm_args* args);
/* 64-bit words of relu_mask for these arguments (the 256 kernel's ReLU-dropout or
   dReLU epilogue, bf16), or 0 when the call cannot use it. */
int64_t nstl_gemm_relu_mask_words(const nstl_gemm_args* args);

/* Up to NSTL_GEMM_GROUP_MAX independent problems in ONE launch (grouped GEMM):
   each a bf16 problem for the 256x256 kernel (M, N >= 256, K % 64 == 0), no
   epilogue, no split-K, all with the same a_kmajor / b_kmajor / c_dtype and
   beta use (0 / nonzero); alpha, beta, pointers and shapes per problem.  The
   weight gradients of one decoder layer (utils/model.py:193-216 Linears,
   backward) are 256 tiles: one full round with no split-K partials; those of
   four encoder layers are 768 tiles: three. */
#define NSTL_GEMM_GROUP_MAX 16
int nstl_gemm_grouped(const nstl_gemm_args* args, int n, void* stream);
int64_t nstl_gemm_workspace_bytes(int M, int N, int split_k);

/* Row-wise fp8 quantization (BASELINE config C5: fp8 QKV/FFN projections; the
 * reference computes these Linears under fp16 autocast, utils/training_utils.py
 * :64, so fp8 is a precision choice of C5, not a restatement).
 * Row i of X[rows][cols] gets amax_i = max_j |x_ij|, the f32 scale
 * s_i = amax_i / 448 (448 = the largest e4m3 value; 1 for an all-zero row) and
 * q_ij = e4m3(x_ij * (448 / amax_i)) (OCP e4m3fn, round to nearest even), so
 * x_ij ~ s_i q_ij.  An fp8 GEMM (dtype NSTL_FP8) takes A's scales as a_scale and
 * B's as b_scale.  Constraints: cols % 16 == 0, ldx % 8 == 0, ldq % 16 == 0,
 * 16-byte aligned rows.  Up to NSTL_FP8_BATCH_MAX independent jobs of one
 * source dtype per launch (all the projection weights after an optimizer step). */
#define NSTL_FP8_BATCH_MAX 64
typedef struct nstl_fp8_job {
  const void* x; int64_t ldx;   /* source (x_dtype) */
  void* q; int64_t ldq;         /* e4m3 out [rows][ldq] */
  float* scale;                 /* f32 out [rows] */
  int rows, cols;
} nstl_fp8_job;
int nstl_fp8_quant_rows(int x_dtype, const nstl_fp8_job* jobs, int n, void* stream);
/* The transposed form: job (x [rows][ldx], cols) writes Q [cols][ldq] and scale
 * [cols] = nstl_fp8_quant_rows of X^T, i.e. per-column scales.  The weight operand
 * of the fp8 input-gradient GEMM (dX = dY W, contraction over W's rows): the
 * transposed weights, K-major over the output channels, one scale per input
 * channel.  rows % 64 == 0, cols % 64 == 0, ldq % 16 == 0 and ldq >= rows.
 * Replaces nothing in the reference (fp8 is BASELINE config C5's precision
 * choice; the reference's backward of utils/model.py:153-158 runs under autocast). */
int nstl_fp8_quant_cols(int x_dtype, const nstl_fp8_job* jobs, int n, void* stream);

/* Non-causal multi-head attention with per-head RoPE already applied to q,k
 * (by the projection epilogue), softmax scale 1/sqrt(dh), attention-probability
 * dropout.  Replaces F.scaled_dot_product_attention at utils/model.py:126-127.
 * Element (b,t,h,d) of X lives at X[(b*T + t)*X_ld + h*dh + d].
 * Constraints: dh == 64; T % 16 == 0; T <= 256 (bf16) / 128 (f32). */
typedef struct nstl_attn_args {
  int dtype;
  int B, T, H, dh;
  const void* q; int64_t q_ld;
  const void* k; int64_t k_ld;
  const void* v; int64_t v_ld;
  void* o; int64_t o_ld;
  float* lse;                 /* [B*H*T] f32: log-sum-exp of scaled scores */
  float p_drop; uint64_t seed;
  const void* dout; int64_t dout_ld;   /* backward only */
  void* dq; int64_t dq_ld;
  void* dk; int64_t dk_ld;
  void* dv; int64_t dv_ld;
  const float* rope_cos; const float* rope_sin;  /* [T][dh/2]; non-null: dq,dk rotated back */
  int rope_q, rope_k;
  float* dsum;                /* backward scratch [B*H*T] f32: rowsum(dO * O) */
  uint64_t* mask_bits;        /* optional [B*H*T*T/64]: the dropout keep bits.  Forward
                                 writes them, backward reads them instead of re-hashing
                                 (MFMA path: head_dim 64; ignored elsewhere).  NULL:
                                 both directions hash (seed, element). */
  float* dbias_part;          /* optional backward output [nstl_attn_bias_rows()][3*H*dh] f32:
                                 per-(batch, 128-row block) column sums of dq | dk | dv as
                                 stored = the q/k/v projection bias gradients before the
                                 final row reduction (nstl_reduce_rows). MFMA path only. */
} nstl_attn_args;
int nstl_attn_fwd(const nstl_attn_args* args, void* stream);
int nstl_attn_bwd(const nstl_attn_args* args, void* stream);
/* Rows of dbias_part for these arguments, or 0 when the call takes the generic
   kernels (which do not produce it). */
int nstl_attn_bias_rows(const nstl_attn_args* args);

/* Post-LN residual block tail: s = x + dropout(dropout(y)); out = LN(s).
 * Replaces `src = src + self.dropoutN(src2); src = self.normN(src)` at
 * utils/model.py:175-180, :198-207, the final LayerNorms :228-229, :249-250, and
 * (rot_out) the decoder-input GlobalPositionalEncoding at :246. */
typedef struct nstl_ln_args {
  int dtype; int rows, D;
  const void* x;           /* residual (dtype), may be NULL */
  const void* y;           /* branch (dtype) */
  int n_masks; float p_drop; uint64_t seed1, seed2;
  const float* gamma; const float* beta; float eps;
  void* s_out;             /* saved pre-norm sum (dtype) */
  void* out;               /* LN output (dtype) */
  float* mean; float* rstd;
  void* rot_out; const float* rope_cos; const float* rope_sin; int rope_T;
  /* backward */
  const void* s_in;        /* saved pre-norm sum */
  const float* dout;       /* f32 [rows][D] */
  float* ds;               /* f32 [rows][D] (may alias dout) */
  void* dbranch;           /* dtype: ds * masks / (1-p)^n_masks, may be NULL */
  float* dgamma_part; float* dbeta_part; int n_part;   /* [n_part][D]; n_part <= rows/8
                                                          (rows/4 when D % 256 != 0) */
  float* dbranch_part;     /* optional [n_part][D]: column sums of dbranch (the bias
                              gradient of the Linear that produced y) */
  const void* dout2;       /* optional dtype [rows][D], added to dout: the input gradient
                              of a Linear fed by this LN's output, kept in dtype as the
                              reference's autocast casts it (utils/model.py Linears) */
  /* optional (bf16 only): the row-wise e4m3 copy [rows][ldq8] and its row scales,
     exactly nstl_fp8_quant_rows of the stored values (BASELINE config C5): in the
     forward of `out` (the fp8 q/k/v / FFN GEMM operand), in the backward of
     `dbranch` (the A operand of the fp8 FFN linear2 input-gradient GEMM) */
  void* q8; int64_t ldq8; float* q8_scale;
} nstl_ln_args;
int nstl_ln_fwd(const nstl_ln_args* args, void* stream);
int nstl_ln_bwd(const nstl_ln_args* args, void* stream);

/* out[j] = beta*out[j] + sum_p part[p][j]  (f32) */
int nstl_reduce_rows(const float* part, int n_part, int cols, float* out, float beta, void* stream);
/* the same over a column window of a wider matrix: rows ld floats apart */
int nstl_reduce_rows_strided(const float* part, int64_t ld, int n_part, int cols, float* out, float beta,
                             void* stream);
/* Several independent row reductions in ONE launch (a backward layer's LayerNorm
 * and bias-gradient partials): out[j] = beta*out[j] + sum_p part[p*ld + j]. */
#define NSTL_REDUCE_BATCH_MAX 16
typedef struct nstl_reduce_job {
  const float* part; int64_t ld; int n_part; int cols; float* out; float beta;
} nstl_reduce_job;
int nstl_reduce_rows_batch(const nstl_reduce_job* jobs, int n, void* stream);
/* Three such reductions in one launch: matrix m at part + m*mat_stride -> out_m
 * (LayerNorm backward's dgamma / dbeta / fused bias-grad partials). */
int nstl_reduce_rows3(const float* part, int64_t mat_stride, int n_mat, int n_part, int cols, float* out0,
                      float* out1, float* out2, float beta, void* stream);
/* Column sums of X[rows][cols] (bias gradients): out[j] = beta*out[j] + sum_i X[i][j].
 * partial: [ceil(rows/256)][cols] f32 scratch. */
int nstl_colsum(int dtype, const void* x, int64_t ld, int rows, int cols, float* partial,
                float* out, float beta, void* stream);

/* Interleaved-pair rotation of rows (RoPE / global PE).  inverse: rotate by -theta.
 * accumulate: out += result (out must be f32). Position t = row % T. */
int nstl_rope(int in_dtype, const void* in, int64_t in_ld, int out_dtype, void* out, int64_t out_ld,
              int rows, int cols, const float* cos_t, const float* sin_t, int T, int rope_dim,
              int inverse, int accumulate, void* stream);

/* Fused Loss forward + backward.  Replaces Loss.forward (utils/model.py:278-291)
 * and its autograd backward.  loss_out[0..3] = total, rec, temp, dir. */
typedef struct nstl_loss_args {
  int B, T, F;
  const float* pred; int64_t pred_ld;
  const float* trg; int64_t trg_ld;
  float delta, w1, w2, w3;
  float grad_scale;
  void* dpred; int dpred_dtype; int64_t dpred_ld;   /* columns F..dpred_ld-1 zeroed */
  float* partial;          /* [B][4] scratch */
  float* loss_out;         /* [4] */
} nstl_loss_args;
int nstl_loss_fwd_bwd(const nstl_loss_args* args, void* stream);

/* Global gradient L2 norm, stage 1: partial[i] = sum of squares of a slice.
 * n_partial <= 1024. Replaces clip_grad_norm_'s norm (utils/training_utils.py:73). */
int nstl_sumsq(const float* g, int64_t n, float* partial, int n_partial, void* stream);

/* Clip + Adam(coupled L2) over one flat f32 arena: replaces
 * torch.nn.utils.clip_grad_norm_(params, max_norm) + torch.optim.Adam.step
 * (utils/training_utils.py:73-74, utils/model_utils.py:11). */
typedef struct nstl_adam_args {
  float* p; const float* g; float* m; float* v;
  void* p_lowp; int lowp_dtype;        /* optional low-precision shadow copy of p */
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay;
  int step;                            /* post-increment step count (>= 1) */
  const float* sumsq_partial; int n_partial;   /* NULL: no clipping */
  float max_norm;
  float* norm_out;                     /* [1] pre-clip total norm, may be NULL */
  const float* coef;                   /* device [1] clip coefficient from nstl_clip_coef, or NULL;
                                          exclusive with sumsq_partial.  The kernel then uses no LDS,
                                          so a range update can share CUs with a ring GEMM */
} nstl_adam_args;
int nstl_adam_step(const nstl_adam_args* args, void* stream);

/* clip_grad_norm_'s coefficient min(1, max_norm / (norm + 1e-6)) from nstl_sumsq
 * partials (and/or nstl_gemm_args.sq_part partials), n_partial <= 2^20, into
 * coef_out[0] (and the pre-clip norm into norm_out[0] when non-NULL): the form
 * nstl_adam_step's coef reads (utils/training_utils.py:73-74). */
int nstl_clip_coef(const float* partial, int n_partial, float max_norm, float* coef_out, float* norm_out,
                   void* stream);

/* 2-D strided copy with conversion: dst[i][j] = scale * src[i][j] for j < cols,
 * 0 for cols <= j < dst_cols (zero padding).  scale: device f32 scalar or NULL (1). */
int nstl_copy2d(int src_dtype, const void* src, int64_t src_ld, int dst_dtype, void* dst, int64_t dst_ld,
                int rows, int cols, int dst_cols, const float* scale, void* stream);

/* Batched bf16 transpose: job k writes y[j][i] = x[i][j] for x [rows][ldx] ->
 * y [cols][ldy].  The input-gradient GEMMs' weight operand (dX = dY W contracts
 * over W's rows): the transposed bf16 copy W^T [in][out] is K-major, the layout
 * the GEMM kernels read fastest, refreshed once per backward from the bf16
 * shadow.  rows % 64 == 0, cols % 64 == 0, ldx / ldy multiples of 8, 16-byte
 * aligned; up to NSTL_TRANSPOSE_BATCH_MAX jobs per launch.  Replaces nothing in
 * the reference (a layout choice; autograd's mm backward of utils/model.py's
 * Linears reads W in place). */
#define NSTL_TRANSPOSE_BATCH_MAX 64
typedef struct nstl_transpose_job {
  const void* x; int64_t ldx;
  void* y; int64_t ldy;
  int rows, cols;
} nstl_transpose_job;
int nstl_transpose_bf16(const nstl_transpose_job* jobs, int n, void* stream);

/* dtype conversion (f32 <-> bf16), n elements. */
int nstl_cast(int src_dtype, const void* src, int dst_dtype, void* dst, int64_t n, void* stream);

/* Feature extraction (utils/audio/extraction/extract_features_utils.py:54-113):
 * per 120 Hz frame of the reflect-padded clip: DC removal, symmetric Hann,
 * autocorrelation lags 1..n_lags normalised by lag 0, edge-frame fix.
 * y: f32 [n_samples]; out: f64 [n_frames][n_lags]. */
int nstl_autocorr(const float* y, int64_t n_samples, int frame_length, int hop_length, int n_lags,
                  double* out, int n_frames, void* stream);

/* Fused STFT -> power -> mel (BASELINE config C5's fused STFT/mel kernel;
 * utils/audio/extraction/extract_features_utils.py:17-30 up to the dB step):
 * centre-padded periodic-Hann frames of n_fft = int(0.01667 sr) every n_fft/2
 * samples, mixed-radix FFT (n_fft over radices 2, 3, 4, 5, 7), |X|^2 of bins
 * 0..n_fft/2, 128 Slaney mel filters.  mel_out: f32 [n_frames][128] power,
 * n_frames = 1 + n_samples / (n_fft/2).  nstl_features runs the same kernel. */
int nstl_stft_mel(const float* y, int64_t n_samples, int sr, float* mel_out, int n_frames, void* stream);

/* Combined per-clip audio features: extract_and_combine_features after the
 * load (utils/audio/extraction/extract_features.py:6-46 with
 * extract_features_utils.py:5-44,54-128): MFCC(23, CMVN) + delta + delta2
 * (Savitzky-Golay width 9, mode 'interp') and autocorrelation lags 1..187,
 * STFT frames (n_fft = int(0.01667 sr), hop n_fft/2) reduced by frame pairs.
 * y: f32 [n_samples] peak-normalised audio at sr; out: f32 [n_out_frames][ld_out],
 * columns 0..255 = [mfcc | d | dd | autocorr].  n_out_frames must equal
 * nstl_features_frames(); the caller rejects clips with fewer than 9 frames
 * (extract_features.py:19-21), the library returns hipErrorInvalidValue.
 * Workspace (caller-owned): nstl_features_workspace_bytes(). */
int nstl_features(const float* y, int64_t n_samples, int sr, float* out, int64_t ld_out, int n_out_frames,
                  void* workspace, int64_t workspace_bytes, void* stream);
int64_t nstl_features_workspace_bytes(int64_t n_samples, int sr);
int nstl_features_frames(int64_t n_samples, int sr);

/* The frame-axis stages of nstl_features on their own.
 * nstl_cmvn_delta_reduce: x f32 [ncoef][F] (coefficient-major, F >= 9) ->
 *   out f32 [(F+1)/2][ld_out], columns [0, ncoef) = reduce(cmvn(x)),
 *   [ncoef, 2 ncoef) = reduce(delta1(cmvn(x))), [2 ncoef, 3 ncoef) = reduce(delta2(...)).
 *   Replaces cepstral_mean_variance_normalization + librosa.feature.delta +
 *   reduce_features (extract_features_utils.py:5-8, :25-27, :33-44).
 * nstl_reduce_frame_pairs: x f64 [F][cols] -> out f32 [(F+1)/2] rows, columns
 *   [col0, col0 + cols) = means of frame pairs (2k, 2k+1), an odd last frame kept
 *   (reduce_features, extract_features_utils.py:33-44, on the autocorrelation lags). */
int nstl_cmvn_delta_reduce(const float* x, int ncoef, int F, float* out, int64_t ld_out, void* stream);
int nstl_reduce_frame_pairs(const double* x, int F, int cols, float* out, int64_t ld_out, int col0, void* stream);

const char* nstl_last_error_string(void);
int nstl_version(void);

/* Launch counters by kernel family, process-wide (host side, counted at each
 * launch): lets a test assert which kernels a call path took, e.g. that a
 * production-shape step ran the 256x256 ring GEMM and the fused attention
 * backward.  No reference counterpart (verification aid). */
enum {
  NSTL_K_GEMM128 = 0,        /* 128x128 GEMM launches (small / f32 problems) */
  NSTL_K_GEMM_RING,          /* 256x256 LDS-DMA ring GEMM launches */
  NSTL_K_GEMM_RING_TILES,    /*   ... their 256x256 output tiles */
  NSTL_K_GEMM_GROUP,         /* grouped ring GEMM launches (weight gradients) */
  NSTL_K_GEMM_GROUP_TILES,   /*   ... their tiles */
  NSTL_K_GEMM_SPLITK_REDUCE, /* split-K combine launches */
  NSTL_K_GEMM_FP8,           /* fp8 GEMM launches (either kernel) */
  NSTL_K_ATTN_FWD,           /* MFMA attention forward */
  NSTL_K_ATTN_FWD_GENERIC,
  NSTL_K_ATTN_BWD_FUSED,     /* one-kernel attention backward */
  NSTL_K_ATTN_BWD_SPLIT,     /* dQ + dK/dV kernel pairs */
  NSTL_K_ATTN_BWD_GENERIC,
  NSTL_K_GEMM4,              /* 4-wave persistent 256x256 GEMM launches (csrc/gemm4.h) */
  NSTL_K_GEMM4_TILES,        /*   ... their 256x256 output tiles */
  NSTL_K_GEMM4_SK,           /*   ... launches with a stream-K tail (grid not dividing the tiles) */
  NSTL_K_GEMM_FP8_ROPE,      /* fp8 GEMM launches with the RoPE epilogue (C5 q|k|v, cross q, cross k|v) */
  NSTL_K_GEMM4F8,            /* fp8 GEMM launches on the 4-wave persistent kernel (the rest: NSTL_K_GEMM_FP8) */
  NSTL_K_COUNT
};
/* Copy-engine ZeRO-1 (parallel.ShardPusher; replaces the reference's gather of
 * every gradient to cuda:0 and broadcast back, utils/training_utils.py:228-257).
 * Each rank exports its receive buffer with nstl_ipc_handle; every other rank
 * maps it with nstl_ipc_open and, during backward, pushes the slices of its
 * gradient arena that the owner's shard holds with nstl_copy_engine: a device-
 * to-device copy on the copy engines (no kernel, no CU taken from the step).
 * After a collective orders every push before it, the owner forms its shard's
 * gradient with nstl_shard_sum. */
#define NSTL_IPC_HANDLE_BYTES 64
/* handle_out: NSTL_IPC_HANDLE_BYTES naming the allocation that holds ptr;
   offset_out: ptr's byte offset in it.  nstl_ipc_open returns that allocation's
   base in the calling process (add the offset). */
int nstl_ipc_handle(const void* ptr, void* handle_out, int64_t* offset_out);
int nstl_ipc_open(const void* handle, void** ptr_out);
int nstl_ipc_close(void* ptr);
int nstl_copy_engine(void* dst, const void* src, int64_t bytes, void* stream);
/* out[i] = own[i] + slots[0][i] + ... + slots[n_slots-1][i] (f32, slot order;
 * slot k at slots + k * ld), and partial[b] = the sum of squares of block b of
 * out exactly as nstl_sumsq(out, n, partial, n_partial) computes it -- the
 * reduce-scatter and the clip norm's first stage (utils/training_utils.py:73)
 * in one pass over the shard.  Starts with a system-scope acquire: the slots
 * are written by other devices' copy engines. */
int nstl_shard_sum(const float* own, const float* slots, int64_t ld, int n_slots, int64_t n, float* out,
                   float* partial, int n_partial, void* stream);

/* Workgroups a persistent one-per-CU grid launches on `stream` (the GEMM and
 * attention-forward grids): 32 x the fewest CUs the stream's CU mask leaves on
 * one (XCD, shader engine) pair (mask bit i = a CU of XCD i % 8, SE (i / 8) % 4).
 * A compute stream that cedes CUs to the gradient collectives should cede them
 * evenly over the 32 pairs (multiples of 32 mask bits from bit 0). */
int nstl_stream_cus(void* stream);
/* The rule nstl_stream_cus applies to a CU mask of `ncu` bits (host only, no
 * device needed): 32 x the fewest set bits of any (XCD, SE) pair; 0 when ncu is
 * not a multiple of 32. */
int nstl_mask_grid(const uint32_t* mask, int ncu);
/* Copies min(n, NSTL_K_COUNT) counters to out; returns NSTL_K_COUNT. */
int nstl_kernel_counts(int64_t* out, int n);
void nstl_kernel_counts_reset(void);

#ifdef __cplusplus
}
#endif
#endif
