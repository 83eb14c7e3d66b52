#include <stdlib.h>
// Optimizer + small memory-bound kernels over flat f32 arenas.
//   nstl_sumsq      : stage 1 of the global grad norm (clip_grad_norm_, utils/training_utils.py:73)
//   nstl_adam_step  : clip coefficient + Adam with coupled L2 (torch.optim.Adam(weight_decay),
//                     utils/model_utils.py:11) + bf16 shadow copy, one pass over the arena
//   nstl_cast, nstl_colsum (bias grads), nstl_reduce_rows, nstl_rope
#include <algorithm>
#include <cmath>

#include "../../include/nstl.h"
#include "common.h"
#include "status.h"

namespace {
constexpr int NT = 256;

// Sum of squares of one slice per block (grid = the partial count).  SUM: the
// slice is first formed as own + slots[0] + slots[1] + ... (in slot order, f32)
// and written to `out` (nstl_shard_sum: the copy-engine ZeRO-1 reduction);
// the squares are then accumulated exactly as for a plain read of `out`, so the
// partials are bit-identical to nstl_sumsq of the summed shard.
struct SumSrc {
  const float* own;
  const float* slots;  // [n_slots][ld]
  int64_t ld;
  int n_slots;
  float* out;
};

template <bool SUM>
NSTL_DEV float sum_one(const float* g, const SumSrc& s, int64_t i) {
  if constexpr (!SUM) {
    return g[i];
  } else {
    float x = s.own[i];
    for (int k = 0; k < s.n_slots; ++k) x += s.slots[k * s.ld + i];
    s.out[i] = x;
    return x;
  }
}
template <bool SUM>
NSTL_DEV f32x4 sum_four(const float* g, const SumSrc& s, int64_t i4) {
  if constexpr (!SUM) {
    return ((const f32x4*)g)[i4];
  } else {
    f32x4 x = ((const f32x4*)s.own)[i4];
    for (int k = 0; k < s.n_slots; ++k) x += ((const f32x4*)(s.slots + k * s.ld))[i4];
    ((f32x4*)s.out)[i4] = x;
    return x;
  }
}

template <bool SUM>
__global__ __launch_bounds__(NT) void sumsq_kernel(const float* g, int64_t n, float* partial, SumSrc src) {
  if constexpr (SUM) {
    // the slots were written by other GPUs' copy engines (peer writes into this
    // device's memory, ordered before this launch by a collective): a
    // system-scope acquire drops any line of them this device's caches kept
    // from an earlier step
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(n, lo + per);
  double acc = 0.0;
  // vector body (16-byte aligned part)
  int64_t v0 = (lo + 3) & ~(int64_t)3, v1 = hi & ~(int64_t)3;
  if (v0 > hi) v0 = hi;
  if (v1 < v0) v1 = v0;
  for (int64_t i = lo + threadIdx.x; i < v0; i += NT) {
    const float x = sum_one<SUM>(g, src, i);
    acc += (double)x * x;
  }
  // four 16-byte loads in flight per thread before their squares are summed
  int64_t i = v0 / 4 + threadIdx.x;
  for (; i + 3 * NT < v1 / 4; i += 4 * NT) {
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = sum_four<SUM>(g, src, i + u * NT);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      acc += (double)(x[u][0] * x[u][0] + x[u][1] * x[u][1]) + (double)(x[u][2] * x[u][2] + x[u][3] * x[u][3]);
  }
  for (; i < v1 / 4; i += NT) {
    const f32x4 x = sum_four<SUM>(g, src, i);
    acc += (double)(x[0] * x[0] + x[1] * x[1]) + (double)(x[2] * x[2] + x[3] * x[3]);
  }
  for (int64_t i = v1 + threadIdx.x; i < hi; i += NT) {
    const float x = sum_one<SUM>(g, src, i);
    acc += (double)x * x;
  }
  __shared__ double red[NT / 64];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int k = 0; k < NT / 64; ++k) s += red[k];
    partial[blockIdx.x] = (float)s;
  }
}

struct AdamParams {
  float* p; const float* g; float* m; float* v; char* lowp; int lowp_bf16;
  int64_t n;
  float lr, b1, b2, eps, wd, step_size, bc2_sqrt;
  const float* part; int n_part; float max_norm; float* norm_out;
  const float* coef;  // precomputed clip coefficient (adam_gcoef_kernel)
};

// NT: the f32 master, gradient and moments stream through once per step with
// nontemporal loads / stores (their next use is a whole step later), leaving the
// caches to the bf16 shadow the next forward's GEMMs read
// The update of one element (m, v in place; returns the new parameter), shared
// by every Adam kernel.  Contraction is off and the FMAs are explicit, so the
// rounding is fixed by the source: an element rounds the same whether a kernel
// reaches it in an unrolled pass or a tail loop (left to the compiler, the
// unrolled form differed by 1 ulp on 12 of 10^6 elements).
NSTL_DEV float adam_math(const AdamParams& a, float coef, float pv, float g, float& m, float& v) {
#pragma clang fp contract(off)
  const float gc = fmaf(a.wd, pv, g * coef);               // clip, then L2 (coupled)
  m = fmaf(1.f - a.b1, gc - m, m);                         // torch lerp form
  v = fmaf(v, a.b2, ((1.f - a.b2) * gc) * gc);
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  return fmaf(-a.step_size, m / denom, pv);
}

template <bool NT_ = false>
NSTL_DEV void adam_elem(const AdamParams& a, float coef, int64_t i) {
  auto ld = [](const float* q) { return NT_ ? __builtin_nontemporal_load(q) : *q; };
  auto st = [](float* q, float x) {
    if (NT_) __builtin_nontemporal_store(x, q);
    else *q = x;
  };
  const float pv = ld(a.p + i);
  const float g = ld(a.g + i);
  float m = ld(a.m + i);
  float v = ld(a.v + i);
  const float np = adam_math(a, coef, pv, g, m, v);
  st(a.p + i, np);
  st(a.m + i, m);
  st(a.v + i, v);
  if (a.lowp) {
    if (a.lowp_bf16) ((bf16*)a.lowp)[i] = (bf16)np;
    else ((float*)a.lowp)[i] = np;
  }
}

// clip_grad_norm_'s coefficient from the sumsq partials, by wave 0 of a block
// (the reduction order every caller of clip_coef_wave shares)
NSTL_DEV float clip_coef_wave(const float* part, int n_part, float max_norm, float* total_out) {
  double s = 0;
  for (int k = threadIdx.x; k < n_part; k += 64) s += part[k];
  s = wave_sum_d(s);
  const float total = (float)sqrt(s);
  const float c = max_norm / (total + 1e-6f);
  *total_out = total;
  return c < 1.f ? c : 1.f;
}

__global__ __launch_bounds__(NT) void adam_kernel(AdamParams a) {
  __shared__ float coef_s;
  if (threadIdx.x < 64) {
    float coef = 1.f, total = 0.f;
    if (a.part) coef = clip_coef_wave(a.part, a.n_part, a.max_norm, &total);
    if (threadIdx.x == 0) {
      if (a.part && blockIdx.x == 0 && a.norm_out) a.norm_out[0] = total;
      coef_s = coef;
    }
  }
  __syncthreads();
  const float coef = coef_s;
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < a.n; i += stride) adam_elem(a, coef, i);
}

// nstl_clip_coef: the coefficient (and the pre-clip norm) once, into device memory
__global__ __launch_bounds__(64) void clip_coef_kernel(const float* part, int n_part, float max_norm, float* coef,
                                                       float* norm_out) {
  float total = 0.f;
  const float c = clip_coef_wave(part, n_part, max_norm, &total);
  if (threadIdx.x == 0) {
    coef[0] = c;
    if (norm_out) norm_out[0] = total;
  }
}

// the same over many partials (the ring GEMM's per-(tile, wave) sums of squares
// of the weight gradients + the rest of the arena's nstl_sumsq partials): one
// 1024-thread block, double sums in a fixed order
__global__ __launch_bounds__(1024) void clip_coef_many_kernel(const float* part, int n_part, float max_norm,
                                                             float* coef, float* norm_out) {
  __shared__ double red[16];
  double s = 0;
  // ~28k partials at the 228M shape: 8 loads in flight per lane, summed in the
  // same order as one at a time (which waited a memory latency per partial)
  int k = threadIdx.x;
  for (; k + 7 * 1024 < n_part; k += 8 * 1024) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = part[k + u * 1024];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; k < n_part; k += 1024) s += part[k];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int w = 0; w < 16; ++w) t += red[w];
    const float total = (float)sqrt(t);
    const float c = max_norm / (total + 1e-6f);
    coef[0] = c < 1.f ? c : 1.f;
    if (norm_out) norm_out[0] = total;
  }
}

// Adam with the coefficient read from device memory: no LDS, so its workgroups
// fit on a CU beside a 160 KB ring-GEMM workgroup (the range updates that run
// under the next forward, FusedAdam.overlap_next_forward)
template <bool NT_, int U = 1>
__global__ __launch_bounds__(NT) void adam_gcoef_kernel(AdamParams a) {
  const float coef = *a.coef;
  const int64_t stride = (int64_t)gridDim.x * NT;
  int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if constexpr (U > 1) {
    // U elements per pass, every load issued before the first store (the
    // compiler cannot hoist loads above stores to possibly aliasing arrays):
    // U x 4 loads in flight per lane
    auto ld = [](const float* q) { return NT_ ? __builtin_nontemporal_load(q) : *q; };
    auto st = [](float* q, float x) {
      if (NT_) __builtin_nontemporal_store(x, q);
      else *q = x;
    };
    for (; i + (U - 1) * stride < a.n; i += U * stride) {
      float pv[U], g[U], m[U], v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pv[u] = ld(a.p + i + u * stride);
        g[u] = ld(a.g + i + u * stride);
        m[u] = ld(a.m + i + u * stride);
        v[u] = ld(a.v + i + u * stride);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float np = adam_math(a, coef, pv[u], g[u], m[u], v[u]);
        const int64_t k = i + u * stride;
        st(a.p + k, np);
        st(a.m + k, m[u]);
        st(a.v + k, v[u]);
        if (a.lowp) {
          if (a.lowp_bf16) ((bf16*)a.lowp)[k] = (bf16)np;
          else ((float*)a.lowp)[k] = np;
        }
      }
    }
  }
  for (; i < a.n; i += stride) adam_elem<NT_>(a, coef, i);
}

__global__ void cast_kernel(int src_bf16, const void* src, int dst_bf16, void* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = src_bf16 ? (float)((const bf16*)src)[i] : ((const float*)src)[i];
    if (dst_bf16) ((bf16*)dst)[i] = (bf16)v;
    else ((float*)dst)[i] = v;
  }
}

__global__ void copy2d_kernel(int src_bf16, const void* src, int64_t src_ld, int dst_bf16, void* dst, int64_t dst_ld,
                              int rows, int cols, int dst_cols, const float* scale) {
  const float sc = scale ? scale[0] : 1.f;
  const int64_t total = (int64_t)rows * dst_cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / dst_cols), j = (int)(e % dst_cols);
    float v = 0.f;
    if (j < cols) {
      const int64_t s = (int64_t)i * src_ld + j;
      v = sc * (src_bf16 ? (float)((const bf16*)src)[s] : ((const float*)src)[s]);
    }
    const int64_t d = (int64_t)i * dst_ld + j;
    if (dst_bf16) ((bf16*)dst)[d] = (bf16)v;
    else ((float*)dst)[d] = v;
  }
}

constexpr int COLSUM_ROWS = 256;
// Column sums, stage 1: block = 256-row chunk x 256 columns; each thread owns
// 8 contiguous columns (one 16-byte load per row) of one of 8 row groups.
template <typename T>
__global__ __launch_bounds__(NT) void colsum_vec_kernel(const T* x, int64_t ld, int rows, int cols, float* partial) {
  constexpr int EPV = 16 / sizeof(T);     // elements per 16-byte load
  constexpr int CT = 256 / EPV;           // column threads per block row
  constexpr int RG = NT / CT;             // row groups
  const int ct = threadIdx.x % CT, rg = threadIdx.x / CT;
  const int c0 = blockIdx.x * 256 + ct * EPV;
  const int r0 = blockIdx.y * COLSUM_ROWS, r1 = min(rows, r0 + COLSUM_ROWS);
  float acc[EPV];
#pragma unroll
  for (int j = 0; j < EPV; ++j) acc[j] = 0.f;
  if (c0 < cols) {
    // 4 rows' loads in flight, then their adds in row order (the sums of the
    // one-row-at-a-time loop, which waited a memory latency per row)
    int r = r0 + rg;
    for (; r + 3 * RG < r1; r += 4 * RG) {
      uint4 u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) u[q] = *(const uint4*)(x + (int64_t)(r + q * RG) * ld + c0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const T* e = (const T*)&u[q];
#pragma unroll
        for (int j = 0; j < EPV; ++j) acc[j] += to_f32(e[j]);
      }
    }
    for (; r < r1; r += RG) {
      const uint4 u = *(const uint4*)(x + (int64_t)r * ld + c0);
      const T* e = (const T*)&u;
#pragma unroll
      for (int j = 0; j < EPV; ++j) acc[j] += to_f32(e[j]);
    }
  }
  __shared__ float red[RG][256];
#pragma unroll
  for (int j = 0; j < EPV; ++j) red[rg][ct * EPV + j] = acc[j];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (threadIdx.x < 256 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) s += red[g][threadIdx.x];
    partial[(int64_t)blockIdx.y * cols + c] = s;
  }
}

// any cols / ld (e.g. the 61-column head gradient): block = 64 columns x 4 row
// groups over a 256-row chunk, loads unrolled so several rows are in flight
template <typename T>
__global__ __launch_bounds__(NT) void colsum_kernel(const T* x, int64_t ld, int rows, int cols, float* partial) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * COLSUM_ROWS, r1 = min(rows, r0 + COLSUM_ROWS);
  float s = 0.f;
  if (j < cols) {
#pragma unroll 8
    for (int r = r0 + rg; r < r1; r += NT / 64) s += to_f32(x[(int64_t)r * ld + j]);
  }
  __shared__ float red[NT / 64][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < cols) partial[(int64_t)blockIdx.y * cols + j] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// out[j] = beta*out[j] + sum_k part[k][j]: block = 64 columns x 4 row groups
__global__ __launch_bounds__(NT) void reduce_rows_kernel(const float* part, int n_part, int cols, float* out,
                                                         float beta, int64_t ld) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (j < cols) {
    int k = rg;
    for (; k + 12 < n_part; k += 16)
      s += (part[(int64_t)k * ld + j] + part[(int64_t)(k + 4) * ld + j]) +
           (part[(int64_t)(k + 8) * ld + j] + part[(int64_t)(k + 12) * ld + j]);
    for (; k < n_part; k += 4) s += part[(int64_t)k * ld + j];
  }
  __shared__ float red[4][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < cols) {
    const float t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    out[j] = beta != 0.f ? beta * out[j] + t : t;
  }
}

template <typename TI, typename TO>
__global__ void rope_kernel(const TI* in, int64_t in_ld, TO* out, int64_t out_ld, int rows, int cols,
                            const float* cs, const float* sn, int T, int rope_dim, int inverse, int acc) {
  const int half = cols >> 1;
  const int64_t total = (int64_t)rows * half;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / half), pj = (int)(e % half);
    const int j = 2 * pj;
    const int t = i % T, pr = (j % rope_dim) >> 1;
    const float c = cs[t * (rope_dim / 2) + pr], s = inverse ? -sn[t * (rope_dim / 2) + pr] : sn[t * (rope_dim / 2) + pr];
    const float a = to_f32(in[(int64_t)i * in_ld + j]), b = to_f32(in[(int64_t)i * in_ld + j + 1]);
    float ra = a * c - b * s, rb = a * s + b * c;
    TO* o = out + (int64_t)i * out_ld + j;
    if (acc) {
      ra += to_f32(o[0]);
      rb += to_f32(o[1]);
    }
    o[0] = from_f32<TO>(ra);
    o[1] = from_f32<TO>(rb);
  }
}

// Batched bf16 transpose, one 64 x 64 tile per workgroup: 16-byte row loads into
// a padded LDS tile, 16-byte row stores of the transposed tile (both sides
// coalesced; HBM-bound at 4 B per element).
struct TpBatch {
  nstl_transpose_job j[NSTL_TRANSPOSE_BATCH_MAX];
};
__global__ __launch_bounds__(NT) void transpose_bf16_kernel(TpBatch b) {
  const nstl_transpose_job& J = b.j[blockIdx.z];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  if (c0 >= J.cols || r0 >= J.rows) return;
  __shared__ uint32_t tile[64][33];  // 64 source rows of 64 bf16 (pairs), one dword of padding
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = h * 32 + (t >> 3), c = (t & 7) * 8;
    const uint4 v = *(const uint4*)((const bf16*)J.x + (int64_t)(r0 + r) * J.ldx + c0 + c);
    tile[r][c / 2] = v.x;
    tile[r][c / 2 + 1] = v.y;
    tile[r][c / 2 + 2] = v.z;
    tile[r][c / 2 + 3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // output row c0 + oc (a source column), 8 source rows ob .. ob + 7
    const int q = h * NT + t, oc = q >> 3, ob = (q & 7) * 8;
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = tile[ob + 2 * e][oc >> 1], hi = tile[ob + 2 * e + 1][oc >> 1];
      o[e] = (oc & 1) ? ((lo >> 16) | (hi & 0xFFFF0000u)) : ((lo & 0xFFFFu) | (hi << 16));
    }
    *(uint4*)((bf16*)J.y + (int64_t)(c0 + oc) * J.ldy + r0 + ob) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

int grid_for(int64_t n, int per_thread = 1) {
  int64_t g = (n + (int64_t)NT * per_thread - 1) / ((int64_t)NT * per_thread);
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}
}  // namespace

extern "C" int nstl_sumsq(const float* g, int64_t n, float* partial, int n_partial, void* stream) {
  NSTL_CHECK_ARG(g && partial && n > 0 && n_partial > 0 && n_partial <= 1024, "nstl_sumsq: bad args");
  NSTL_CHECK_ARG(((uintptr_t)g % 16) == 0, "nstl_sumsq: g must be 16-byte aligned");
  hipLaunchKernelGGL(sumsq_kernel<false>, dim3(n_partial), dim3(NT), 0, (hipStream_t)stream, g, n, partial, SumSrc{});
  NSTL_LAUNCH_CHECK("nstl_sumsq");
  return 0;
}

extern "C" int nstl_shard_sum(const float* own, const float* slots, int64_t ld, int n_slots, int64_t n, float* out,
                              float* partial, int n_partial, void* stream) {
  NSTL_CHECK_ARG(own && out && partial && n > 0 && n_partial > 0 && n_partial <= 1024 && n_slots >= 0 &&
                     (n_slots == 0 || (slots && ld >= n)),
                 "nstl_shard_sum: bad args");
  NSTL_CHECK_ARG((((uintptr_t)own | (uintptr_t)out | (uintptr_t)slots) % 16) == 0 && ld % 4 == 0,
                 "nstl_shard_sum: 16-byte aligned arrays and slot stride");
  hipLaunchKernelGGL(sumsq_kernel<true>, dim3(n_partial), dim3(NT), 0, (hipStream_t)stream, out, n, partial,
                     SumSrc{own, slots, ld, n_slots, out});
  NSTL_LAUNCH_CHECK("nstl_shard_sum");
  return 0;
}

extern "C" int nstl_adam_step(const nstl_adam_args* a, void* stream) {
  NSTL_CHECK_ARG(a && a->p && a->g && a->m && a->v && a->n > 0, "nstl_adam_step: bad args");
  NSTL_CHECK_ARG(a->step >= 1, "nstl_adam_step: step must be >= 1");
  NSTL_CHECK_ARG(!a->sumsq_partial || (a->n_partial > 0 && a->n_partial <= 1024), "nstl_adam_step: partials");
  AdamParams p;
  p.p = a->p; p.g = a->g; p.m = a->m; p.v = a->v;
  p.lowp = (char*)a->p_lowp; p.lowp_bf16 = a->lowp_dtype == NSTL_BF16;
  p.n = a->n;
  p.lr = a->lr; p.b1 = a->beta1; p.b2 = a->beta2; p.eps = a->eps; p.wd = a->weight_decay;
  // bias corrections in double on the host, handed to the kernel as f32 scalars
  // (torch's foreach Adam casts its python-float scalars the same way)
  const double bc1 = 1.0 - std::pow((double)a->beta1, a->step);
  const double bc2 = 1.0 - std::pow((double)a->beta2, a->step);
  p.step_size = (float)(a->lr / bc1);
  p.bc2_sqrt = (float)std::sqrt(bc2);
  p.part = a->sumsq_partial; p.n_part = a->n_partial; p.max_norm = a->max_norm; p.norm_out = a->norm_out;
  p.coef = a->coef;
  // scalar elements (16-byte vectorised forms measured slower: x1 +4 %, x2
  // unrolled +4-8 %, tools/bench_adam.py), strided by the grid
  if (a->coef) {
    NSTL_CHECK_ARG(!a->sumsq_partial, "nstl_adam_step: coef and sumsq_partial are exclusive");
    // NSTL_ADAM_GRID: cap on its workgroups (how many CUs a range update shares)
    static const int cap = [] {
      const char* e = getenv("NSTL_ADAM_GRID");
      return e ? std::max(1, atoi(e)) : 8192;
    }();
    // NSTL_ADAM_NT=0: plain loads / stores (A/B; read per call).  Nontemporal is the
    // default: +0.4 % step rate same-box (586.7k vs 584.3k frames/s, 3 reps)
    const char* ne = getenv("NSTL_ADAM_NT");
    // two elements per lane and pass with all 8 loads in flight (default: +0.35 %
    // step same-box, 586.6-587.6k vs 584.7-585.9k); NSTL_ADAM_U=1 | 4 for A/B
    static const int unroll = [] {
      const char* e = getenv("NSTL_ADAM_U");
      return e ? atoi(e) : 2;
    }();
    if (!(ne && ne[0] == '0') && unroll == 2)
      hipLaunchKernelGGL((adam_gcoef_kernel<true, 2>), dim3(std::min(grid_for(a->n, 4), cap)), dim3(NT), 0,
                         (hipStream_t)stream, p);
    else if (!(ne && ne[0] == '0') && unroll == 4)
      hipLaunchKernelGGL((adam_gcoef_kernel<true, 4>), dim3(std::min(grid_for(a->n, 4), cap)), dim3(NT), 0,
                         (hipStream_t)stream, p);
    else if (!(ne && ne[0] == '0'))
      hipLaunchKernelGGL(adam_gcoef_kernel<true>, dim3(std::min(grid_for(a->n, 4), cap)), dim3(NT), 0,
                         (hipStream_t)stream, p);
    else
      hipLaunchKernelGGL(adam_gcoef_kernel<false>, dim3(std::min(grid_for(a->n, 4), cap)), dim3(NT), 0,
                         (hipStream_t)stream, p);
  } else {
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(a->n, 4)), dim3(NT), 0, (hipStream_t)stream, p);
  }
  NSTL_LAUNCH_CHECK("nstl_adam_step");
  return 0;
}

extern "C" int nstl_clip_coef(const float* partial, int n_partial, float max_norm, float* coef_out, float* norm_out,
                              void* stream) {
  NSTL_CHECK_ARG(partial && coef_out && n_partial > 0 && n_partial <= (1 << 20), "nstl_clip_coef: bad args");
  if (n_partial <= 1024)
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, partial, n_partial, max_norm,
                       coef_out, norm_out);
  else
    hipLaunchKernelGGL(clip_coef_many_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, partial, n_partial,
                       max_norm, coef_out, norm_out);
  NSTL_LAUNCH_CHECK("nstl_clip_coef");
  return 0;
}

extern "C" int nstl_cast(int src_dtype, const void* src, int dst_dtype, void* dst, int64_t n, void* stream) {
  NSTL_CHECK_ARG(src && dst && n >= 0, "nstl_cast: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n, 4)), dim3(NT), 0, (hipStream_t)stream,
                     src_dtype == NSTL_BF16, src, dst_dtype == NSTL_BF16, dst, n);
  NSTL_LAUNCH_CHECK("nstl_cast");
  return 0;
}

extern "C" int nstl_transpose_bf16(const nstl_transpose_job* jobs, int n, void* stream) {
  NSTL_CHECK_ARG(jobs != nullptr && n >= 1 && n <= NSTL_TRANSPOSE_BATCH_MAX, "nstl_transpose_bf16: 1..%d jobs (got %d)",
                 NSTL_TRANSPOSE_BATCH_MAX, n);
  TpBatch b;
  int wide = 0, tall = 0;
  for (int k = 0; k < n; ++k) {
    const nstl_transpose_job& J = jobs[k];
    NSTL_CHECK_ARG(J.x && J.y, "nstl_transpose_bf16: job %d: null pointer", k);
    NSTL_CHECK_ARG(J.rows > 0 && J.cols > 0 && J.rows % 64 == 0 && J.cols % 64 == 0,
                   "nstl_transpose_bf16: job %d: rows and cols must be positive multiples of 64 (got %d x %d)", k,
                   J.rows, J.cols);
    NSTL_CHECK_ARG(J.ldx >= J.cols && J.ldy >= J.rows && J.ldx % 8 == 0 && J.ldy % 8 == 0 &&
                       ((uintptr_t)J.x | (uintptr_t)J.y) % 16 == 0,
                   "nstl_transpose_bf16: job %d: leading dimensions (multiples of 8, >= the row length) and "
                   "16-byte aligned pointers", k);
    b.j[k] = J;
    wide = std::max(wide, J.cols);
    tall = std::max(tall, J.rows);
  }
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(wide / 64, tall / 64, n), dim3(NT), 0, (hipStream_t)stream, b);
  NSTL_LAUNCH_CHECK("nstl_transpose_bf16");
  return 0;
}

extern "C" int nstl_copy2d(int src_dtype, const void* src, int64_t src_ld, int dst_dtype, void* dst, int64_t dst_ld,
                           int rows, int cols, int dst_cols, const float* scale, void* stream) {
  NSTL_CHECK_ARG(src && dst && rows >= 0 && cols >= 0 && dst_cols >= cols && src_ld >= cols && dst_ld >= dst_cols,
                 "nstl_copy2d: bad args");
  if (rows == 0 || dst_cols == 0) return 0;
  hipLaunchKernelGGL(copy2d_kernel, dim3(grid_for((int64_t)rows * dst_cols)), dim3(NT), 0, (hipStream_t)stream,
                     src_dtype == NSTL_BF16, src, src_ld, dst_dtype == NSTL_BF16, dst, dst_ld, rows, cols, dst_cols,
                     scale);
  NSTL_LAUNCH_CHECK("nstl_copy2d");
  return 0;
}

extern "C" int nstl_colsum(int dtype, const void* x, int64_t ld, int rows, int cols, float* partial, float* out,
                           float beta, void* stream) {
  NSTL_CHECK_ARG(x && partial && out && rows > 0 && cols > 0 && ld >= cols, "nstl_colsum: bad args");
  const int nchunk = (rows + COLSUM_ROWS - 1) / COLSUM_ROWS;
  hipStream_t st = (hipStream_t)stream;
  const int epv = dtype == NSTL_BF16 ? 8 : 4;
  const bool vec = cols % epv == 0 && ld % epv == 0 && ((uintptr_t)x % 16) == 0;
  if (vec) {
    dim3 grid((cols + 255) / 256, nchunk);
    if (dtype == NSTL_BF16)
      hipLaunchKernelGGL(colsum_vec_kernel<bf16>, grid, dim3(NT), 0, st, (const bf16*)x, ld, rows, cols, partial);
    else
      hipLaunchKernelGGL(colsum_vec_kernel<float>, grid, dim3(NT), 0, st, (const float*)x, ld, rows, cols, partial);
  } else {
    dim3 grid((cols + 63) / 64, nchunk);
    if (dtype == NSTL_BF16)
      hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(NT), 0, st, (const bf16*)x, ld, rows, cols, partial);
    else
      hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(NT), 0, st, (const float*)x, ld, rows, cols, partial);
  }
  NSTL_LAUNCH_CHECK("nstl_colsum");
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((cols + 63) / 64), dim3(NT), 0, st, partial, nchunk, cols, out, beta,
                     (int64_t)cols);
  NSTL_LAUNCH_CHECK("nstl_colsum reduce");
  return 0;
}

// Column j of rows rg, rg + 16, rg + 32, ... of a [n_part][ld] f32 matrix, summed in
// that order (the order reduce_rows3 / reduce_batch have always used, so results
// are unchanged), with the loads of 8 rows issued before their adds: the plain
// loop waited one memory latency per row (latency-bound: ~11 us for a decoder
// layer's 12 MB of partials).
NSTL_DEV float strided_col_sum(const float* pm, int64_t ld, int n_part, int rg, int j) {
  float s = 0.f;
  int k = rg;
  for (; k + 7 * 16 < n_part; k += 8 * 16) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = pm[(int64_t)(k + 16 * u) * ld + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < n_part; k += 16) s += pm[(int64_t)k * ld + j];
  return s;
}

// Up to three [n_part][cols] partial-sum matrices (stride mat_stride floats)
// reduced over rows into three outputs in one launch: 64 columns x 16 row
// groups per block, blockIdx.y = matrix.
__global__ __launch_bounds__(1024) void reduce_rows3_kernel(const float* part, int64_t mat_stride, int n_part,
                                                            int cols, float* o0, float* o1, float* o2, float beta) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float* out = blockIdx.y == 0 ? o0 : blockIdx.y == 1 ? o1 : o2;
  const float* pm = part + blockIdx.y * mat_stride;
  const float s = j < cols ? strided_col_sum(pm, cols, n_part, rg, j) : 0.f;
  __shared__ float red[16][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < cols && out != nullptr) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][cl];
    out[j] = beta != 0.f ? beta * out[j] + t : t;
  }
}

extern "C" int nstl_reduce_rows3(const float* part, int64_t mat_stride, int n_mat, int n_part, int cols, float* out0,
                                 float* out1, float* out2, float beta, void* stream) {
  NSTL_CHECK_ARG(part && out0 && n_mat >= 1 && n_mat <= 3 && n_part > 0 && cols > 0, "nstl_reduce_rows3: bad args");
  NSTL_CHECK_ARG(n_mat < 2 || out1, "nstl_reduce_rows3: out1 missing");
  NSTL_CHECK_ARG(n_mat < 3 || out2, "nstl_reduce_rows3: out2 missing");
  hipLaunchKernelGGL(reduce_rows3_kernel, dim3((cols + 63) / 64, n_mat), dim3(1024), 0, (hipStream_t)stream, part,
                     mat_stride, n_part, cols, out0, out1, out2, beta);
  NSTL_LAUNCH_CHECK("nstl_reduce_rows3");
  return 0;
}

// Up to NSTL_REDUCE_BATCH_MAX such reductions (any part / ld / rows / cols)
// in one launch: block b -> job j with block_end[j-1] <= b < block_end[j]; each
// block reduces 64 columns of its job with reduce_rows3's order (16 row groups,
// then the groups in order), so results do not depend on the batching.
struct ReduceBatch {
  const float* part[NSTL_REDUCE_BATCH_MAX];
  int64_t ld[NSTL_REDUCE_BATCH_MAX];
  float* out[NSTL_REDUCE_BATCH_MAX];
  int n_part[NSTL_REDUCE_BATCH_MAX];
  int cols[NSTL_REDUCE_BATCH_MAX];
  float beta[NSTL_REDUCE_BATCH_MAX];
  int block_end[NSTL_REDUCE_BATCH_MAX];
  int n;
};

__global__ __launch_bounds__(1024) void reduce_batch_kernel(ReduceBatch rb) {
  int jb = 0;
  while (jb + 1 < rb.n && (int)blockIdx.x >= rb.block_end[jb]) ++jb;
  const int blk = blockIdx.x - (jb > 0 ? rb.block_end[jb - 1] : 0);
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blk * 64 + cl, cols = rb.cols[jb], n_part = rb.n_part[jb];
  const float* pm = rb.part[jb];
  const int64_t ld = rb.ld[jb];
  const float s = j < cols ? strided_col_sum(pm, ld, n_part, rg, j) : 0.f;
  __shared__ float red[16][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && j < cols) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][cl];
    float* out = rb.out[jb];
    const float beta = rb.beta[jb];
    out[j] = beta != 0.f ? beta * out[j] + t : t;
  }
}

extern "C" int nstl_reduce_rows_batch(const nstl_reduce_job* jobs, int n, void* stream) {
  NSTL_CHECK_ARG(jobs && n >= 1 && n <= NSTL_REDUCE_BATCH_MAX, "nstl_reduce_rows_batch: 1..%d jobs (got %d)",
                 NSTL_REDUCE_BATCH_MAX, n);
  ReduceBatch rb;
  rb.n = n;
  int blocks = 0;
  for (int k = 0; k < n; ++k) {
    const nstl_reduce_job& jb = jobs[k];
    NSTL_CHECK_ARG(jb.part && jb.out && jb.n_part > 0 && jb.cols > 0 && jb.ld >= jb.cols,
                   "nstl_reduce_rows_batch: bad job %d", k);
    rb.part[k] = jb.part; rb.ld[k] = jb.ld; rb.out[k] = jb.out;
    rb.n_part[k] = jb.n_part; rb.cols[k] = jb.cols; rb.beta[k] = jb.beta;
    blocks += (jb.cols + 63) / 64;
    rb.block_end[k] = blocks;
  }
  hipLaunchKernelGGL(reduce_batch_kernel, dim3(blocks), dim3(1024), 0, (hipStream_t)stream, rb);
  NSTL_LAUNCH_CHECK("nstl_reduce_rows_batch");
  return 0;
}

extern "C" int nstl_reduce_rows(const float* part, int n_part, int cols, float* out, float beta, void* stream) {
  return nstl_reduce_rows_strided(part, cols, n_part, cols, out, beta, stream);
}

extern "C" int nstl_reduce_rows_strided(const float* part, int64_t ld, int n_part, int cols, float* out, float beta,
                                        void* stream) {
  NSTL_CHECK_ARG(part && out && n_part > 0 && cols > 0 && ld >= cols, "nstl_reduce_rows: bad args");
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((cols + 63) / 64), dim3(NT), 0, (hipStream_t)stream, part, n_part,
                     cols, out, beta, ld);
  NSTL_LAUNCH_CHECK("nstl_reduce_rows");
  return 0;
}

extern "C" int nstl_rope(int in_dtype, const void* in, int64_t in_ld, int out_dtype, void* out, int64_t out_ld,
                         int rows, int cols, const float* cos_t, const float* sin_t, int T, int rope_dim, int inverse,
                         int accumulate, void* stream) {
  NSTL_CHECK_ARG(in && out && cos_t && sin_t && rows > 0 && cols > 0 && cols % 2 == 0 && rope_dim % 2 == 0 &&
                     T > 0, "nstl_rope: bad args");
  NSTL_CHECK_ARG(!accumulate || out_dtype == NSTL_F32, "nstl_rope: accumulate needs f32 output");
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_for((int64_t)rows * cols / 2);
#define NSTL_ROPE(TI, TO)                                                                                 \
  hipLaunchKernelGGL((rope_kernel<TI, TO>), dim3(grid), dim3(NT), 0, st, (const TI*)in, in_ld, (TO*)out, \
                     out_ld, rows, cols, cos_t, sin_t, T, rope_dim, inverse, accumulate)
  if (in_dtype == NSTL_BF16 && out_dtype == NSTL_BF16) NSTL_ROPE(bf16, bf16);
  else if (in_dtype == NSTL_BF16) NSTL_ROPE(bf16, float);
  else if (out_dtype == NSTL_BF16) NSTL_ROPE(float, bf16);
  else NSTL_ROPE(float, float);
#undef NSTL_ROPE
  NSTL_LAUNCH_CHECK("nstl_rope");
  return 0;
}
