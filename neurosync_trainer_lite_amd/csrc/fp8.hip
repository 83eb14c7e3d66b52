// Row-wise fp8 quantization of GEMM operands (BASELINE config C5: fp8 QKV/FFN
// projections; nstl.h nstl_fp8_quant_rows).  One wave per row.  Rows of 4096
// bf16 (the FFN hidden) are held in registers: loads, wave max, cast, 8-byte
// stores of e4m3.  Other widths: pass 1 takes max |x| over the row,
// pass 2 re-reads it (an L2 hit) and casts.  HBM-bound: (2 or 4) + 1 bytes per
// element.
#include <algorithm>

#include "../../include/nstl.h"

#include "common.h"
#include "status.h"

namespace {

struct Fp8Batch {
  nstl_fp8_job j[NSTL_FP8_BATCH_MAX];
  int n;
};

// two f32 -> two e4m3 bytes (OCP e4m3fn on gfx950, round to nearest even)
NSTL_DEV uint32_t pk_fp8(float a, float b) {
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xffffu;
}

template <bool XF32>
NSTL_DEV void load8(const nstl_fp8_job& J, int i, int c0, float (&v)[8]) {
  if (XF32) {
    const float* src = (const float*)J.x + (int64_t)i * J.ldx + c0;
    const f32x4 a = *(const f32x4*)src, b = *(const f32x4*)(src + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
  } else {
    const bf16x8 a = *(const bf16x8*)((const bf16*)J.x + (int64_t)i * J.ldx + c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)a[e];
  }
}

template <bool XF32>
__global__ __launch_bounds__(256) void fp8_quant_rows_kernel(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int nchunk = J.cols >> 3;  // 8-element chunks per row
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < J.rows; i += gridDim.x * 4) {
    float am = 0.f;
    for (int c = lane; c < nchunk; c += 64) {
      float v[8];
      load8<XF32>(J, i, c * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
    }
    am = wave_max(am);
    const float inv = am > 0.f ? 448.f / am : 1.f;
    if (lane == 0) J.scale[i] = am > 0.f ? am / 448.f : 1.f;
    for (int c = lane; c < nchunk; c += 64) {
      float v[8];
      load8<XF32>(J, i, c * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e] * inv, -448.f), 448.f);
      const uint32_t lo = pk_fp8(v[0], v[1]) | (pk_fp8(v[2], v[3]) << 16);
      const uint32_t hi = pk_fp8(v[4], v[5]) | (pk_fp8(v[6], v[7]) << 16);
      *(uint2*)((uint8_t*)J.q + (int64_t)i * J.ldq + c * 8) = make_uint2(lo, hi);
    }
  }
}

// Single pass for rows of exactly NCH * 512 elements: the row stays in
// registers between the max and the cast.
template <bool XF32, int NCH>
__global__ __launch_bounds__(256) void fp8_quant_rows_reg_kernel(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.y];
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < J.rows; i += gridDim.x * 4) {
    float v[NCH][8];
#pragma unroll
    for (int c = 0; c < NCH; ++c) load8<XF32>(J, i, (lane + 64 * c) * 8, v[c]);
    float am = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[c][e]));
    am = wave_max(am);
    const float inv = am > 0.f ? 448.f / am : 1.f;
    if (lane == 0) J.scale[i] = am > 0.f ? am / 448.f : 1.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = fminf(fmaxf(v[c][e] * inv, -448.f), 448.f);
      const uint32_t lo = pk_fp8(v[c][0], v[c][1]) | (pk_fp8(v[c][2], v[c][3]) << 16);
      const uint32_t hi = pk_fp8(v[c][4], v[c][5]) | (pk_fp8(v[c][6], v[c][7]) << 16);
      *(uint2*)((uint8_t*)J.q + (int64_t)i * J.ldq + (lane + 64 * c) * 8) = make_uint2(lo, hi);
    }
  }
}


// Column-wise (transposed) form: Q[c][r] = e4m3(x[r][c] * 448 / amax_c), scale[c] =
// amax_c / 448 over column c -- exactly nstl_fp8_quant_rows applied to X^T.  The
// fp8 input-gradient GEMM's weight operand: dX = dY W needs W^T's rows (input
// channels) K-major over the output channels.  Four launches over a grid of 64 x 64
// tiles (every job of the batch at once): zero the scales, per-tile column maxima
// combined by an unsigned atomic max on the bits of |x| (non-negative floats order
// as their bits) held in the scale array itself, the quantized transpose of each
// tile through LDS (64 contiguous bytes per output row), and the scales from the
// maxima.  (r3: one workgroup per 64-column strip walking all rows took 191 us for
// the 16 W2 matrices of the 228M model: latency-bound.)
constexpr int QC_T = 64;

template <bool XF32>
NSTL_DEV float load1(const nstl_fp8_job& J, int r, int c) {
  if (XF32) return ((const float*)J.x)[(int64_t)r * J.ldx + c];
  return (float)((const bf16*)J.x)[(int64_t)r * J.ldx + c];
}

// tile (bx -> column tile, by -> row tile) of job blockIdx.z, if inside it
NSTL_DEV bool qc_tile(const nstl_fp8_job& J, int& c0, int& r0) {
  c0 = blockIdx.x * QC_T;
  r0 = blockIdx.y * QC_T;
  return c0 < J.cols && r0 < J.rows;
}

__global__ __launch_bounds__(256) void fp8_qc_zero(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.y];
  for (int c = blockIdx.x * 256 + threadIdx.x; c < J.cols; c += gridDim.x * 256) J.scale[c] = 0.f;
}

template <bool XF32>
__global__ __launch_bounds__(256) void fp8_qc_amax(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.z];
  int c0, r0;
  if (!qc_tile(J, c0, r0)) return;
  __shared__ float amx[4][QC_T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float am = 0.f;
#pragma unroll 4
  for (int r = w; r < QC_T; r += 4) am = fmaxf(am, fabsf(load1<XF32>(J, r0 + r, c0 + lane)));
  amx[w][lane] = am;
  __syncthreads();
  if (tid < QC_T) {
    const float a = fmaxf(fmaxf(amx[0][tid], amx[1][tid]), fmaxf(amx[2][tid], amx[3][tid]));
    atomicMax((unsigned*)J.scale + c0 + tid, __float_as_uint(a));
  }
}

template <bool XF32>
__global__ __launch_bounds__(256) void fp8_qc_quant(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.z];
  int c0, r0;
  if (!qc_tile(J, c0, r0)) return;
  __shared__ float tile[QC_T][QC_T + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll 4
  for (int rr = w; rr < QC_T; rr += 4) tile[rr][lane] = load1<XF32>(J, r0 + rr, c0 + lane);
  // thread t writes output row c0 + t / 4, bytes 16 (t % 4) .. + 15 of the tile's 64
  const int oc = tid >> 2, ob = (tid & 3) * 16;
  const float oam = J.scale[c0 + oc];  // still the maximum (fp8_qc_scale runs after)
  const float oinv = oam > 0.f ? 448.f / oam : 1.f;
  __syncthreads();
  uint32_t o[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fminf(fmaxf(tile[ob + 4 * h + e][oc] * oinv, -448.f), 448.f);
    o[h] = pk_fp8(v[0], v[1]) | (pk_fp8(v[2], v[3]) << 16);
  }
  *(uint4*)((uint8_t*)J.q + (int64_t)(c0 + oc) * J.ldq + r0 + ob) = make_uint4(o[0], o[1], o[2], o[3]);
}

__global__ __launch_bounds__(256) void fp8_qc_scale(Fp8Batch b) {
  const nstl_fp8_job& J = b.j[blockIdx.y];
  for (int c = blockIdx.x * 256 + threadIdx.x; c < J.cols; c += gridDim.x * 256) {
    const float a = J.scale[c];
    J.scale[c] = a > 0.f ? a / 448.f : 1.f;
  }
}
}  // namespace

extern "C" int nstl_fp8_quant_rows(int x_dtype, const nstl_fp8_job* jobs, int n, void* stream) {
  NSTL_CHECK_ARG(jobs != nullptr && n >= 1 && n <= NSTL_FP8_BATCH_MAX, "nstl_fp8_quant_rows: 1..%d jobs (got %d)",
                 NSTL_FP8_BATCH_MAX, n);
  NSTL_CHECK_ARG(x_dtype == NSTL_F32 || x_dtype == NSTL_BF16, "nstl_fp8_quant_rows: bad source dtype %d", x_dtype);
  Fp8Batch b;
  b.n = n;
  int most = 0, cols = jobs[0].cols;
  for (int k = 0; k < n; ++k) {
    const nstl_fp8_job& J = jobs[k];
    NSTL_CHECK_ARG(J.x && J.q && J.scale, "nstl_fp8_quant_rows: job %d: null pointer", k);
    NSTL_CHECK_ARG(J.rows > 0 && J.cols > 0 && J.cols % 16 == 0,
                   "nstl_fp8_quant_rows: job %d: cols must be a positive multiple of 16 (got %d x %d)", k, J.rows,
                   J.cols);
    NSTL_CHECK_ARG(J.ldx >= J.cols && J.ldx % 8 == 0 && ((uintptr_t)J.x % 16) == 0,
                   "nstl_fp8_quant_rows: job %d: source rows must be 16-byte aligned (ldx %% 8 == 0)", k);
    NSTL_CHECK_ARG(J.ldq >= J.cols && J.ldq % 16 == 0 && ((uintptr_t)J.q % 16) == 0,
                   "nstl_fp8_quant_rows: job %d: ldq must be a multiple of 16 >= cols", k);
    b.j[k] = J;
    most = std::max(most, J.rows);
    if (J.cols != cols) cols = 0;
  }
  const int blocks = std::min((most + 3) / 4, 4096);
  dim3 grid(blocks, n), block(256);
  hipStream_t st = (hipStream_t)stream;
  // every job 4096 wide (bf16, the FFN hidden): the register-resident single pass
  // (31.7 vs 51 us at 16384 rows; at 1024 wide two passes are faster: 12.8 vs 14.7 us)
  if (x_dtype == NSTL_BF16 && cols == 4096) hipLaunchKernelGGL((fp8_quant_rows_reg_kernel<false, 8>), grid, block, 0, st, b);
  else if (x_dtype == NSTL_F32) hipLaunchKernelGGL((fp8_quant_rows_kernel<true>), grid, block, 0, st, b);
  else hipLaunchKernelGGL((fp8_quant_rows_kernel<false>), grid, block, 0, st, b);
  NSTL_LAUNCH_CHECK("nstl_fp8_quant_rows");
  return 0;
}

extern "C" int nstl_fp8_quant_cols(int x_dtype, const nstl_fp8_job* jobs, int n, void* stream) {
  NSTL_CHECK_ARG(jobs != nullptr && n >= 1 && n <= NSTL_FP8_BATCH_MAX, "nstl_fp8_quant_cols: 1..%d jobs (got %d)",
                 NSTL_FP8_BATCH_MAX, n);
  NSTL_CHECK_ARG(x_dtype == NSTL_F32 || x_dtype == NSTL_BF16, "nstl_fp8_quant_cols: bad source dtype %d", x_dtype);
  Fp8Batch b;
  b.n = n;
  int widest = 0, tallest = 0;
  for (int k = 0; k < n; ++k) {
    const nstl_fp8_job& J = jobs[k];
    NSTL_CHECK_ARG(J.x && J.q && J.scale, "nstl_fp8_quant_cols: job %d: null pointer", k);
    NSTL_CHECK_ARG(J.rows > 0 && J.cols > 0 && J.rows % QC_T == 0 && J.cols % QC_T == 0,
                   "nstl_fp8_quant_cols: job %d: rows and cols must be positive multiples of 64 (got %d x %d)", k,
                   J.rows, J.cols);
    NSTL_CHECK_ARG(J.ldx >= J.cols, "nstl_fp8_quant_cols: job %d: ldx < cols", k);
    NSTL_CHECK_ARG(J.ldq >= J.rows && J.ldq % 16 == 0 && ((uintptr_t)J.q % 16) == 0,
                   "nstl_fp8_quant_cols: job %d: ldq must be a multiple of 16 >= rows (Q is [cols][ldq])", k);
    b.j[k] = J;
    widest = std::max(widest, J.cols);
    tallest = std::max(tallest, J.rows);
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 g1((widest + 255) / 256, n), g2(widest / QC_T, tallest / QC_T, n), block(256);
  hipLaunchKernelGGL(fp8_qc_zero, g1, block, 0, st, b);
  if (x_dtype == NSTL_F32) hipLaunchKernelGGL((fp8_qc_amax<true>), g2, block, 0, st, b);
  else hipLaunchKernelGGL((fp8_qc_amax<false>), g2, block, 0, st, b);
  if (x_dtype == NSTL_F32) hipLaunchKernelGGL((fp8_qc_quant<true>), g2, block, 0, st, b);
  else hipLaunchKernelGGL((fp8_qc_quant<false>), g2, block, 0, st, b);
  hipLaunchKernelGGL(fp8_qc_scale, g1, block, 0, st, b);
  NSTL_LAUNCH_CHECK("nstl_fp8_quant_cols");
  return 0;
}
