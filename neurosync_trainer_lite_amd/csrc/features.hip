// Audio feature kernels (utils/audio/extraction/extract_features_utils.py).
//
// nstl_autocorr restates extract_overlapping_autocorr + fix_edge_frames_autocorr
// (:54-113): reflect-pad frame_length/2, frames of frame_length every
// hop_length, per-frame DC removal, symmetric Hann (np.hanning), lags
// 0..n_lags by direct products (the reference computes a full 2N-1-lag
// np.correlate and keeps n_lags+1 of them), normalise by lag 0 when non-zero,
// drop lag 0, replicate near-silent edge frames.  The windowed frame lives in LDS
// as f64 (the reference is f64 from the window on); the default kernel
// (autocorr3_kernel) runs the lag products as a per-frame f64 GEMM on the matrix
// cores, one wave per frame; the VALU forms below it stay behind switches.
#include <algorithm>
#include <cmath>
#include <deque>
#include <mutex>
#include <vector>

#include "../../include/nstl.h"
#include "common.h"
#include "status.h"

namespace {
constexpr int NT = 256;
constexpr int MAX_FRAME = 4096;

// One workgroup per frame.  Lags 0..n_lags are computed by 24 groups of 8
// consecutive lags x 10 chunks of the sample index: a thread slides an 8-wide
// register window along w (two LDS reads per 8 f64 FMAs), chunk partials are
// summed in LDS.  w is zero-padded past the frame, so sum_{k<L} w[k] w[k+lag]
// needs no per-lag bound.
constexpr int AC_LG = 8;      // lags per thread
constexpr int AC_GROUPS = 24; // lag groups: up to 192 lags (0..n_lags <= 191)
constexpr int AC_CHUNKS = 10; // sample-index chunks

__global__ __launch_bounds__(NT) void autocorr_kernel(const float* y, int64_t n, int L, int hop, int n_lags,
                                                       const double* __restrict__ hann, double* out) {
  __shared__ double w[MAX_FRAME + AC_LG * AC_GROUPS];
  __shared__ double part[AC_CHUNKS][AC_LG * AC_GROUPS];
  __shared__ double red[NT / 64];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int64_t start = (int64_t)f * hop - L / 2;
  double s = 0.0;
  for (int k = tid; k < L; k += NT) {
    int64_t i = start + k;
    if (i < 0) i = -i;                       // numpy 'reflect' (edge not repeated)
    if (i >= n) i = 2 * (n - 1) - i;
    const double v = (double)y[i];
    w[k] = v;
    s += v;
  }
  for (int k = L + tid; k < L + AC_LG * AC_GROUPS; k += NT) w[k] = 0.0;
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / L;
  // the reference subtracts the mean in float32 (frames are float32 until the
  // float64 window multiplies them)
  const float mean_f = (float)mean;
  for (int k = tid; k < L; k += NT) {
    const float c = (float)w[k] - mean_f;
    w[k] = (double)c * hann[k];
  }
  __syncthreads();
  if (tid < AC_GROUPS * AC_CHUNKS) {
    const int g = tid % AC_GROUPS, c = tid / AC_GROUPS;
    const int l0 = g * AC_LG;
    const int chunk = (L + AC_CHUNKS - 1) / AC_CHUNKS;
    const int k0 = c * chunk, k1 = min(L, k0 + chunk);
    double acc[AC_LG], win[AC_LG];
#pragma unroll
    for (int r = 0; r < AC_LG; ++r) {
      acc[r] = 0.0;
      win[r] = w[k0 + l0 + r];
    }
    for (int k = k0; k < k1; ++k) {
      const double a = w[k];
#pragma unroll
      for (int r = 0; r < AC_LG; ++r) acc[r] = fma(a, win[r], acc[r]);
#pragma unroll
      for (int r = 0; r < AC_LG - 1; ++r) win[r] = win[r + 1];
      win[AC_LG - 1] = w[k + l0 + AC_LG];
    }
#pragma unroll
    for (int r = 0; r < AC_LG; ++r) part[c][l0 + r] = acc[r];
  }
  __syncthreads();
  __shared__ double ac0;
  for (int lag = tid; lag <= n_lags; lag += NT) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < AC_CHUNKS; ++c) acc += part[c][lag];
    if (lag == 0) ac0 = acc;
    if (lag > 0) out[(int64_t)f * n_lags + (lag - 1)] = acc;
  }
  __syncthreads();
  if (ac0 != 0.0)
    for (int lag = tid; lag < n_lags; lag += NT) out[(int64_t)f * n_lags + lag] /= ac0;
}

// Register-tiled form (default; NSTL_AUTOCORR_V1=1 keeps the kernel above):
// a thread owns 16 consecutive lags over one 16-aligned chunk of the sample
// index and, per block of 16 samples, reads a[16] = w[k..k+15] and b[31] =
// w[k+l0..k+l0+30] from LDS (16-byte reads) for 256 f64 FMAs -- no register
// shifting (the sliding window above moves 7 registers per 8 FMAs).  12 lag
// groups x 20 chunks = 240 threads; chunk partials summed in LDS in chunk order.
// r3: the partials overwrite the frame image once every thread is done with it
// (one barrier), so a workgroup holds max(frame, partials) = 31 KB of LDS instead
// of 46 KB (5 workgroups per CU instead of 3), and every thread forms lag 0 from
// the same partials in the same order, so the normalisation is one pass over
// registers instead of a second read-modify-write of the output.
constexpr int AC2_LG = 16, AC2_GROUPS = 12, AC2_CHUNKS = 20;
constexpr int AC2_NT = 256;

size_t ac2_chunk(int L) { return ((size_t)(L + AC2_CHUNKS - 1) / AC2_CHUNKS + AC2_LG - 1) / AC2_LG * AC2_LG; }
size_t ac2_wlen(int L) { return ac2_chunk(L) * AC2_CHUNKS + AC2_LG * AC2_GROUPS + 2 * AC2_LG; }
size_t ac2_lds(int L) {
  return (std::max(ac2_wlen(L), (size_t)AC2_CHUNKS * AC2_LG * AC2_GROUPS) + 8) * sizeof(double);
}

__global__ __launch_bounds__(AC2_NT) void autocorr2_kernel(const float* y, int64_t n, int L, int hop, int n_lags,
                                                            const double* __restrict__ hann, double* out, int chunk,
                                                            int wlen) {
  extern __shared__ __attribute__((aligned(16))) double ac2_smem[];
  double* w = ac2_smem;                  // [wlen]: the windowed frame, zero tail
  double* part = ac2_smem;               // [AC2_CHUNKS][AC2_LG * AC2_GROUPS], over w after the products
  const int wpart = std::max(wlen, AC2_CHUNKS * AC2_LG * AC2_GROUPS);
  double* red = ac2_smem + wpart;        // [4] wave sums
  const int f = blockIdx.x, tid = threadIdx.x;
  const int64_t start = (int64_t)f * hop - L / 2;
  double s = 0.0;
  for (int k = tid; k < L; k += AC2_NT) {
    int64_t i = start + k;
    if (i < 0) i = -i;                   // numpy 'reflect' (edge not repeated)
    if (i >= n) i = 2 * (n - 1) - i;
    const double v = (double)y[i];
    w[k] = v;
    s += v;
  }
  for (int k = L + tid; k < wlen; k += AC2_NT) w[k] = 0.0;
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / L;
  // the reference subtracts the mean in float32 (frames are float32 until the
  // float64 window multiplies them)
  const float mean_f = (float)mean;
  for (int k = tid; k < L; k += AC2_NT) {
    const float c = (float)w[k] - mean_f;
    w[k] = (double)c * hann[k];
  }
  __syncthreads();
  const bool worker = tid < AC2_GROUPS * AC2_CHUNKS;
  const int g = tid % AC2_GROUPS, c = tid / AC2_GROUPS;
  const int l0 = g * AC2_LG;
  double acc[AC2_LG];
#pragma unroll
  for (int r = 0; r < AC2_LG; ++r) acc[r] = 0.0;
  if (worker) {
    // Block kb needs b = w[kb + l0 .. kb + l0 + 31]; its upper half is the next
    // block's lower half, so the window slides by 16 values per block: two blocks per
    // iteration with the halves in named registers (lo | mid | hi), 16 new b values
    // per block instead of 32 (LDS reads per 256 FMAs: 16 instead of 24).  Same
    // products in the same order per accumulator as the one-block form.
    const int k0 = c * chunk, k1 = min(L, k0 + chunk);
    auto ld16 = [&](double (&v)[AC2_LG], int at) {  // at % 16 == 0
#pragma unroll
      for (int j = 0; j < AC2_LG; j += 2) {
        const double2 t = *(const double2*)(w + at + j);
        v[j] = t.x;
        v[j + 1] = t.y;
      }
    };
    auto block = [&](const double (&a)[AC2_LG], const double (&lo)[AC2_LG], const double (&hi)[AC2_LG]) {
#pragma unroll
      for (int j = 0; j < AC2_LG; ++j)
#pragma unroll
        for (int r = 0; r < AC2_LG; ++r) acc[r] = fma(a[j], j + r < AC2_LG ? lo[j + r] : hi[j + r - AC2_LG], acc[r]);
    };
    double lo[AC2_LG];
    ld16(lo, k0 + l0);
    int kb = k0;
    for (; kb + AC2_LG < k1; kb += 2 * AC2_LG) {
      double a[AC2_LG], mid[AC2_LG], hi[AC2_LG];
      ld16(a, kb);
      ld16(mid, kb + l0 + AC2_LG);
      block(a, lo, mid);
      ld16(a, kb + AC2_LG);
      ld16(hi, kb + l0 + 2 * AC2_LG);
      block(a, mid, hi);
#pragma unroll
      for (int j = 0; j < AC2_LG; ++j) lo[j] = hi[j];
    }
    if (kb < k1) {
      double a[AC2_LG], mid[AC2_LG];
      ld16(a, kb);
      ld16(mid, kb + l0 + AC2_LG);
      block(a, lo, mid);
    }
  }
  __syncthreads();  // every thread is done with w: the partials take its place
  if (worker) {
#pragma unroll
    for (int r = 0; r < AC2_LG; r += 2)
      *(double2*)(part + c * AC2_LG * AC2_GROUPS + l0 + r) = make_double2(acc[r], acc[r + 1]);
  }
  __syncthreads();
  // lag 0, summed by every thread in chunk order (the value the lag loop forms for lag 0)
  double ac0 = 0.0;
#pragma unroll
  for (int cc = 0; cc < AC2_CHUNKS; ++cc) ac0 += part[cc * AC2_LG * AC2_GROUPS];
  for (int lag = 1 + tid; lag <= n_lags; lag += AC2_NT) {
    double v = 0.0;
#pragma unroll
    for (int cc = 0; cc < AC2_CHUNKS; ++cc) v += part[cc * AC2_LG * AC2_GROUPS + lag];
    out[(int64_t)f * n_lags + (lag - 1)] = ac0 != 0.0 ? v / ac0 : v;
  }
}

// MFMA form (r3, default): the lag products of one frame as a small f64 GEMM.
// With n = 16 b + a, r[k] = sum_a P[a][a + k] where P[a][m] = sum_b x[16b + a]
// x[16b + m] (a < 16, m < 16 AC3_TILES), i.e. P = U^T V over the 16-sample blocks
// b with U[b][a] = x[16b + a] and V[b][m] = x[16b + m].  On
// v_mfma_f64_16x16x4_f64 (one f64 of A and of B per lane: A[i = lane & 15][kk =
// lane >> 4], B[kk][j = lane & 15]; D col = lane & 15, row = (lane >> 4) + 4 v)
// k-step s covers blocks 4s..4s+3 and both operands are one contiguous LDS read:
// A = x[64 s + lane], B(tile t) = x[64 s + 16 t + lane].  A tile whose B lies
// past the frame (64 s + 16 t >= L, ~5 % of them) is skipped by a scalar branch;
// with the accumulators in VGPRs (Makefile: -amdgpu-mfma-vgpr-form) that costs
// no copies (in the default AGPR form the compiler routes every branched MFMA
// through a copy in and out of the AGPRs).  The matrix cores run the f64 FMAs the
// register-tiled kernel above issues on the VALU (same peak rate on gfx950), so the
// operand reads, loop and address work move off the issue port that bounds it.
// One wave per frame, four frames per workgroup, no workgroup barrier; P leaves
// the accumulators one 16 x 16 tile at a time through LDS (over the dead frame
// image) and its diagonals complete 16 lags per tile.
constexpr int AC3_TILES = 13;  // P columns 0..207: lags up to 192
constexpr int AC3_WAVES = 4;
constexpr int AC3_TW = 48;
constexpr int AC3_LD = 24;     // loads per lane in the one-batch frame load: frames up to 1536 samples     // padded tile row (doubles): 16 zeros | 16 values | 16 zeros
__host__ __device__ inline int ac3_steps(int L) { return (L + 63) / 64; }
int ac3_xlen(int L) {  // largest B index 64 (S - 1) + 16 (TILES - 1) + 63, and room for the padded tile
  return std::max(64 * ac3_steps(L) + 16 * (AC3_TILES - 1), 16 * AC3_TW);
}
size_t ac3_lds(int L) { return (size_t)AC3_WAVES * ac3_xlen(L) * sizeof(double); }

// orders this wave's LDS accesses across lanes (LDS executes one wave's
// instructions in order; this keeps the compiler from moving them)
NSTL_DEV void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64 * AC3_WAVES) void autocorr3_kernel(const float* __restrict__ y, int64_t n, int L,
                                                                   int hop, int n_lags, int n_frames,
                                                                   const double* __restrict__ hann,
                                                                   double* __restrict__ out, int xlen) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) double ac3_smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = blockIdx.x * AC3_WAVES + wv;
  if (f >= n_frames) return;  // whole waves only; nothing below synchronises the workgroup
  double* x = ac3_smem + (size_t)wv * xlen;
  const int64_t start = (int64_t)f * hop - L / 2;
  double s = 0.0;
  float mean_f;
  if (L <= 64 * AC3_LD && n < ((int64_t)1 << 29)) {
    // every sample and window load of the lane in flight at once (one memory
    // latency per frame), 32-bit buffer offsets; mean and window from registers
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, (int)(n * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc((void*)hann, 0, L * 8, 0x00020000);
    const int st0 = (int)start, nn = (int)n;
    float v[AC3_LD];
    double h[AC3_LD];
#pragma unroll
    for (int u = 0; u < AC3_LD; ++u) {
      const int k = 64 * u + lane, kk = k < L ? k : L - 1;
      int i = st0 + kk;
      i = i < 0 ? -i : i;  // numpy 'reflect' (edge not repeated)
      i = i >= nn ? 2 * (nn - 1) - i : i;
      v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, i * 4, 0, 0));
      h[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(hr, kk * 8, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < AC3_LD; ++u)
      if (64 * u + lane < L) s += (double)v[u];
    s = wave_sum_d(s);
    // the reference subtracts the mean in float32 (frames are float32 until the
    // float64 window multiplies them)
    mean_f = (float)(s / L);
#pragma unroll
    for (int u = 0; u < AC3_LD; ++u) {
      const int k = 64 * u + lane;
      if (k < L) x[k] = (double)(v[u] - mean_f) * h[u];
    }
    for (int k = L + lane; k < xlen; k += 64) x[k] = 0.0;
  } else {
    // the frame, 8 loads in flight per lane
    for (int k0 = 0; k0 < L; k0 += 8 * 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 64 * u + lane;
        int64_t i = start + (k < L ? k : L - 1);
        if (i < 0) i = -i;  // numpy 'reflect' (edge not repeated)
        if (i >= n) i = 2 * (n - 1) - i;
        v[u] = y[i];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 64 * u + lane;
        if (k < L) {
          x[k] = (double)v[u];
          s += (double)v[u];
        }
      }
    }
    for (int k = L + lane; k < xlen; k += 64) x[k] = 0.0;
    s = wave_sum_d(s);
    // the reference subtracts the mean in float32 (frames are float32 until the
    // float64 window multiplies them)
    mean_f = (float)(s / L);
    for (int k0 = 0; k0 < L; k0 += 8 * 64) {
      double h[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 64 * u + lane;
        h[u] = hann[k < L ? k : L - 1];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 64 * u + lane;
        if (k < L) {
          const float c = (float)x[k] - mean_f;
          x[k] = (double)c * h[u];
        }
      }
    }
  }
  wave_lds_order();
  d4 acc[AC3_TILES];
#pragma unroll
  for (int t = 0; t < AC3_TILES; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  const int S = ac3_steps(L);
  for (int st = 0; st < S; ++st) {
    const double* xs = x + 64 * st + lane;
    double b[AC3_TILES];
#pragma unroll
    for (int t = 0; t < AC3_TILES; ++t) b[t] = xs[16 * t];
#pragma unroll
    for (int t = 0; t < AC3_TILES; ++t)
      if (64 * st + 16 * t < L) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(b[0], b[t], acc[t], 0, 0, 0);
  }
  // Diagonal sums.  The frame image is dead: a zero-padded tile T[16][AC3_TW] with
  // the accumulator tile in columns 16..31 takes its place.  r[16 t + c] =
  // D_t(c) + D_{t+1}(c - 16) (D_t(o) = sum_a P_t[a][a + o]): lanes (c, part) read
  // 8 rows of the upper diagonal c (parts 0, 1) or the lower diagonal c - 16 (parts
  // 2, 3), branch-free through the padding; lane c carries D_t(c) into the next tile.
  wave_lds_order();
  double* T = x;
  for (int k = lane; k < 16 * AC3_TW; k += 64) T[k] = 0.0;
  const int c = lane & 15, part = lane >> 4;
  const int rb = 8 * (part & 1), col0 = part < 2 ? 16 + c : c;
  double* orow = out + (int64_t)f * n_lags;
  double carry = 0.0, r0 = 0.0;
#pragma unroll
  for (int t = 0; t < AC3_TILES; ++t) {
    wave_lds_order();
#pragma unroll
    for (int v = 0; v < 4; ++v) T[(part + 4 * v) * AC3_TW + 16 + c] = acc[t][v];
    wave_lds_order();
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d += T[(rb + i) * AC3_TW + col0 + rb + i];
    d += __shfl_xor(d, 16);                  // lanes 0..15: D_t(c); lanes 32..47: D_t(c - 16)
    const double low = __shfl(d, c + 32);
    if (t == 0) {
      r0 = __shfl(d, 0);                     // lag 0 (D_1(-16) is empty)
    } else {
      const int k = 16 * (t - 1) + c;
      if (lane < 16 && k >= 1 && k <= n_lags) {
        const double v = carry + low;
        orow[k - 1] = r0 != 0.0 ? v / r0 : v;
      }
    }
    carry = d;
  }
}

// np.hanning(L) (symmetric), computed on the host in f64 once per (device, L)
int get_hann(int L, const double** out) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<int, int>, double*>> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nstl::fail((int)hipErrorNoDevice, "autocorr: no device");
  std::lock_guard<std::mutex> lock(mu);
  for (auto& e : cache)
    if (e.first.first == dev && e.first.second == L) {
      *out = e.second;
      return 0;
    }
  std::vector<double> h(L);
  for (int k = 0; k < L; ++k) h[k] = L > 1 ? 0.5 - 0.5 * std::cos(2.0 * M_PI * k / (L - 1)) : 1.0;
  double* d = nullptr;
  if (hipMalloc((void**)&d, L * sizeof(double)) != hipSuccess) return nstl::fail((int)hipErrorOutOfMemory, "autocorr: alloc");
  if (hipMemcpy(d, h.data(), L * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    return nstl::fail((int)hipErrorUnknown, "autocorr: upload");
  cache.push_back({{dev, L}, d});
  *out = d;
  return 0;
}

__global__ void autocorr_edges(double* out, int n_frames, int n_lags) {
  // fix_edge_frames_autocorr: replicate a near-all-zero first/last frame
  __shared__ int zero_first, zero_last;
  if (threadIdx.x == 0) {
    zero_first = 1;
    zero_last = 1;
  }
  __syncthreads();
  for (int l = threadIdx.x; l < n_lags; l += blockDim.x) {
    if (fabs(out[l]) >= 1e-7) zero_first = 0;
    if (fabs(out[(int64_t)(n_frames - 1) * n_lags + l]) >= 1e-7) zero_last = 0;
  }
  __syncthreads();
  if (zero_first && n_frames > 1)
    for (int l = threadIdx.x; l < n_lags; l += blockDim.x) out[l] = out[n_lags + l];
  __syncthreads();
  if (zero_last && n_frames > 1)
    for (int l = threadIdx.x; l < n_lags; l += blockDim.x)
      out[(int64_t)(n_frames - 1) * n_lags + l] = out[(int64_t)(n_frames - 2) * n_lags + l];
}
}  // namespace

extern "C" int nstl_autocorr(const float* y, int64_t n_samples, int frame_length, int hop_length, int n_lags,
                             double* out, int n_frames, void* stream) {
  NSTL_CHECK_ARG(y && out && n_samples > frame_length / 2 && frame_length > 1 && frame_length <= MAX_FRAME,
                 "nstl_autocorr: bad sizes");
  NSTL_CHECK_ARG(hop_length > 0 && n_lags > 0 && n_lags < frame_length && n_lags < AC_LG * AC_GROUPS,
                 "nstl_autocorr: bad lags");
  const int64_t padded = n_samples + 2 * (frame_length / 2);
  const int expect = (int)((padded - frame_length) / hop_length + 1);
  NSTL_CHECK_ARG(n_frames == expect, "nstl_autocorr: n_frames %d != %d", n_frames, expect);
  hipStream_t st = (hipStream_t)stream;
  const double* hann = nullptr;
  if (int rc = get_hann(frame_length, &hann)) return rc;
  static const bool v1 = [] {
    const char* e = getenv("NSTL_AUTOCORR_V1");
    return e && e[0] == '1';
  }();
  static const bool v2 = [] {
    const char* e = getenv("NSTL_AUTOCORR_V2");
    return e && e[0] == '1';
  }();
  if (!v1 && !v2 && n_lags < 16 * (AC3_TILES - 1) && ac3_lds(frame_length) <= 65536) {
    hipLaunchKernelGGL(autocorr3_kernel, dim3((n_frames + AC3_WAVES - 1) / AC3_WAVES), dim3(64 * AC3_WAVES),
                       ac3_lds(frame_length), st, y, n_samples, frame_length, hop_length, n_lags, n_frames, hann, out,
                       ac3_xlen(frame_length));
  } else if (!v1 && n_lags < AC2_LG * AC2_GROUPS && ac2_lds(frame_length) <= 65536) {
    hipLaunchKernelGGL(autocorr2_kernel, dim3(n_frames), dim3(AC2_NT), ac2_lds(frame_length), st, y, n_samples,
                       frame_length, hop_length, n_lags, hann, out, (int)ac2_chunk(frame_length),
                       (int)ac2_wlen(frame_length));
  } else {
    hipLaunchKernelGGL(autocorr_kernel, dim3(n_frames), dim3(NT), 0, st, y, n_samples, frame_length, hop_length,
                       n_lags, hann, out);
  }
  NSTL_LAUNCH_CHECK("nstl_autocorr");
  hipLaunchKernelGGL(autocorr_edges, dim3(1), dim3(256), 0, st, out, n_frames, n_lags);
  NSTL_LAUNCH_CHECK("nstl_autocorr edges");
  return 0;
}

// ============================================================================
// MFCC branch + combined features (extract_features.py:6-46,
// extract_features_utils.py:5-44 -> librosa.feature.mfcc / delta).
//
//   frames  : centre-padded (zeros, n_fft/2 each side) frames of n_fft samples
//             every hop, times the periodic Hann window           [F][kp] f32
//   X       : frames @ DFT basis (cos | sin rows), nstl_gemm f32 MFMA [F][2nb]
//   mel dB  : |X|^2 -> 128 Slaney filters -> 10 log10(max(1e-10, .)) [F][128],
//             running clip-wide max (ordered-int atomicMax)
//   mfcc    : max(dB, max-80) -> DCT-II ortho rows 0..22 (coefficient-major) [23][F]
//   final   : per coefficient CMVN (population std, +1e-10), Savitzky-Golay
//             width-9 deltas (orders 1, 2; mode 'interp' edge fits), mean of
//             frame pairs (odd tail kept) -> out[:, 0:69]; autocorr lags reduced
//             the same way -> out[:, 69:256].
// The librosa algorithm is restated from its published definition (librosa is
// absent from this image): parity for this branch is unpinned, see DESIGN.md.
// ============================================================================
namespace {
constexpr int FFT_MAX = 4096;  // largest n_fft of the fused STFT/mel path
constexpr int N_MELS = 128;
constexpr int N_MFCC = 23;
constexpr int N_AC = 187;
constexpr int SG_W = 9;  // delta width

struct FeatTables {
  int dev = -1, sr = 0, n_fft = 0, nb = 0, kp = 0;
  float* basis = nullptr;   // [2nb][kp]: rows 0..nb-1 cos, nb..2nb-1 sin (window in frames)
  float* window = nullptr;  // [n_fft] periodic Hann
  float* melK = nullptr;    // [N_MELS][nbp] zero-padded GEMM operand (K-major)
  int nbp = 0;
  float* dct = nullptr;     // [N_MFCC][N_MELS]
  float* sg = nullptr;      // [2 orders][SG_W fit positions][SG_W taps]
  // fused STFT/mel (stft_mel_kernel): radices of n_fft (nf = 0: n_fft has a prime
  // factor > 7, the DFT-GEMM path serves it), twiddles, mel filters as bands
  int nf = 0, radix[16] = {};
  float2* tw = nullptr;     // [n_fft] exp(-2 pi i k / n_fft), built in f64
  int* band = nullptr;      // [N_MELS][3]: first bin, bin count, offset in bw of each filter
  float* bw = nullptr;      // [nnz] filter weights, band after band
  int nnz = 0;
};

// n over {4, 2, 3, 5, 7} (fours first); 0 when another prime factor remains
int fft_radices(int n, int* f) {
  int k = 0;
  for (int r : {4, 2, 3, 5, 7})
    while (n % r == 0 && k < 16) {
      f[k++] = r;
      n /= r;
    }
  return n == 1 ? k : 0;
}

double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

// E[t0][j]: the order-th derivative at position t0 of the least-squares
// polynomial (degree `order`) through samples j = 0..SG_W-1.  Interior outputs
// use t0 = SG_W/2; scipy's mode='interp' edges use the first/last window.
void savgol_table(int order, float* E) {
  const int P = order + 1;
  double G[3][3] = {}, Ginv[3][3] = {};
  for (int a = 0; a < P; ++a)
    for (int b = 0; b < P; ++b)
      for (int t = 0; t < SG_W; ++t) G[a][b] += std::pow((double)t, a + b);
  // invert the (P x P) normal matrix (Gauss-Jordan, P <= 3)
  double M[3][6] = {};
  for (int a = 0; a < P; ++a) {
    for (int b = 0; b < P; ++b) M[a][b] = G[a][b];
    M[a][P + a] = 1.0;
  }
  for (int c = 0; c < P; ++c) {
    int piv = c;
    for (int r = c + 1; r < P; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
    for (int k = 0; k < 2 * P; ++k) std::swap(M[c][k], M[piv][k]);
    const double d = M[c][c];
    for (int k = 0; k < 2 * P; ++k) M[c][k] /= d;
    for (int r = 0; r < P; ++r)
      if (r != c) {
        const double f = M[r][c];
        for (int k = 0; k < 2 * P; ++k) M[r][k] -= f * M[c][k];
      }
  }
  for (int a = 0; a < P; ++a)
    for (int b = 0; b < P; ++b) Ginv[a][b] = M[a][P + b];
  for (int t0 = 0; t0 < SG_W; ++t0)
    for (int j = 0; j < SG_W; ++j) {
      // coefficient q of the fit = sum_b Ginv[q][b] * j^b * x_j
      double e = 0.0;
      for (int q = order; q < P; ++q) {
        double cq = 0.0;
        for (int b = 0; b < P; ++b) cq += Ginv[q][b] * std::pow((double)j, b);
        double fall = 1.0;  // q! / (q-order)!
        for (int i = 0; i < order; ++i) fall *= (q - i);
        e += cq * fall * std::pow((double)t0, q - order);
      }
      E[t0 * SG_W + j] = (float)e;
    }
}

int upload(void** dst, const void* src, size_t bytes) {
  if (hipMalloc(dst, bytes) != hipSuccess) return nstl::fail((int)hipErrorOutOfMemory, "features: table alloc");
  if (hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
    return nstl::fail((int)hipErrorUnknown, "features: table upload");
  return 0;
}

// constant tables per (device, sr), built once and kept for the process
int get_tables(int sr, const FeatTables** out) {
  static std::mutex mu;
  static std::vector<FeatTables*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nstl::fail((int)hipErrorNoDevice, "features: no device");
  std::lock_guard<std::mutex> lock(mu);
  for (auto* t : cache)
    if (t->dev == dev && t->sr == sr) {
      *out = t;
      return 0;
    }
  auto* t = new FeatTables();
  t->dev = dev;
  t->sr = sr;
  t->n_fft = (int)(0.01667 * sr);
  t->nb = t->n_fft / 2 + 1;
  t->kp = (t->n_fft + 3) / 4 * 4;
  const int n_fft = t->n_fft, nb = t->nb, kp = t->kp;
  t->nbp = (nb + 63) / 64 * 64;
  std::vector<float> basis((size_t)2 * nb * kp, 0.f), win(n_fft), dct(N_MFCC * N_MELS);
  std::vector<float> melK((size_t)N_MELS * t->nbp, 0.f);
  for (int k = 0; k < nb; ++k)
    for (int n = 0; n < n_fft; ++n) {
      // exact integer phase reduction keeps the f64 argument small
      const double ph = 2.0 * M_PI * (double)(((int64_t)k * n) % n_fft) / n_fft;
      basis[(size_t)k * kp + n] = (float)std::cos(ph);
      basis[(size_t)(nb + k) * kp + n] = (float)std::sin(ph);
    }
  for (int n = 0; n < n_fft; ++n) win[n] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * n / n_fft));
  // librosa.filters.mel(sr, n_fft, n_mels=128, fmin=0, fmax=sr/2, htk=False, norm='slaney')
  std::vector<double> mel_f(N_MELS + 2);
  const double m_lo = hz_to_mel(0.0), m_hi = hz_to_mel(sr / 2.0);
  for (int i = 0; i < N_MELS + 2; ++i) mel_f[i] = mel_to_hz(m_lo + (m_hi - m_lo) * i / (N_MELS + 1));
  for (int i = 0; i < N_MELS; ++i) {
    const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
    for (int b = 0; b < nb; ++b) {
      const double fb = b * ((double)sr / n_fft);
      const double lower = -(mel_f[i] - fb) / (mel_f[i + 1] - mel_f[i]);
      const double upper = (mel_f[i + 2] - fb) / (mel_f[i + 2] - mel_f[i + 1]);
      const double w = std::max(0.0, std::min(lower, upper)) * enorm;
      melK[(size_t)i * t->nbp + b] = (float)w;
    }
  }
  for (int k = 0; k < N_MFCC; ++k)
    for (int m = 0; m < N_MELS; ++m)
      dct[k * N_MELS + m] = (float)(std::cos(M_PI * k * (2 * m + 1) / (2.0 * N_MELS)) *
                                    std::sqrt((k == 0 ? 1.0 : 2.0) / N_MELS));
  float sg[2 * SG_W * SG_W];
  savgol_table(1, sg);
  savgol_table(2, sg + SG_W * SG_W);
  // fused STFT/mel tables
  t->nf = n_fft <= FFT_MAX ? fft_radices(n_fft, t->radix) : 0;
  std::vector<float2> tw(n_fft);
  for (int k = 0; k < n_fft; ++k) {
    const double ph = 2.0 * M_PI * k / n_fft;
    tw[k] = make_float2((float)std::cos(ph), (float)-std::sin(ph));
  }
  std::vector<int> band(3 * N_MELS, 0);
  std::vector<float> bw;
  for (int i = 0; i < N_MELS; ++i) {
    int lo = -1, hi = -1;
    for (int b = 0; b < nb; ++b)
      if (melK[(size_t)i * t->nbp + b] != 0.f) {
        if (lo < 0) lo = b;
        hi = b;
      }
    band[3 * i] = lo < 0 ? 0 : lo;
    band[3 * i + 1] = lo < 0 ? 0 : hi - lo + 1;
    band[3 * i + 2] = (int)bw.size();
    for (int b = lo; lo >= 0 && b <= hi; ++b) bw.push_back(melK[(size_t)i * t->nbp + b]);
  }
  t->nnz = (int)bw.size();
  // stft_mel_kernel's LDS (stft_mel_lds): within the 64 KB a launch gets without opt-in
  if (t->nf > 0 && (size_t)3 * n_fft * 8 + (size_t)n_fft * 4 + 3 * N_MELS * 4 + (size_t)t->nnz * 4 > 65536) t->nf = 0;
  int rc = upload((void**)&t->basis, basis.data(), basis.size() * 4);
  if (!rc) rc = upload((void**)&t->tw, tw.data(), tw.size() * sizeof(float2));
  if (!rc) rc = upload((void**)&t->band, band.data(), band.size() * sizeof(int));
  if (!rc) rc = upload((void**)&t->bw, bw.data(), std::max<size_t>(1, bw.size()) * 4);
  if (!rc) rc = upload((void**)&t->window, win.data(), win.size() * 4);
  if (!rc) rc = upload((void**)&t->melK, melK.data(), melK.size() * 4);
  if (!rc) rc = upload((void**)&t->dct, dct.data(), dct.size() * 4);
  if (!rc) rc = upload((void**)&t->sg, sg, sizeof(sg));
  if (rc) return rc;
  cache.push_back(t);
  *out = t;
  return 0;
}

__global__ __launch_bounds__(256) void stft_frames_kernel(const float* __restrict__ y, int64_t n, int n_fft, int hop,
                                                          int kp, const float* __restrict__ win,
                                                          float* __restrict__ frames) {
  const int f = blockIdx.x;
  const int64_t start = (int64_t)f * hop - n_fft / 2;  // center=True, zero padding
  float* row = frames + (int64_t)f * kp;
  for (int k = threadIdx.x; k < kp; k += 256) {
    const int64_t i = start + k;
    row[k] = (k < n_fft && i >= 0 && i < n) ? y[i] * win[k] : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Fused STFT -> power -> mel (BASELINE C5's fused STFT/mel kernel;
// extract_features_utils.py:17-30 up to the dB step, librosa.feature.melspectrogram
// restated): per frame the centre-padded (zeros), periodic-Hann-windowed frame
// goes through a mixed-radix (4, 2, 3, 5, 7) Stockham FFT in LDS -- f32, twiddles
// rounded from an f64 table -- then |X|^2 of bins 0..n_fft/2 and the 128 Slaney
// filters as contiguous bands of weights.  Writes mel power [F][128] and the
// clip-wide max (the dB floor's reference).  Replaces frames -> DFT GEMM
// (4.3 MFLOP per frame on the f32 MFMA) -> |X|^2 -> mel GEMM -> max: one launch,
// ~0.1 MFLOP per frame, the audio read once per frame (L2) and 512 B written.
constexpr int FFT_NT = 256, FFT_FPB = 8;  // threads, frames per workgroup (tables loaded once)

NSTL_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// One Stockham pass of radix R: n/R butterflies, each combining R interleaved
// sub-transforms of length ns into one of length ns*R (natural order after the
// last pass).  Twiddles tw[k] = exp(-2 pi i k / n); W_R^m = tw[m n / R].
template <int R>
NSTL_DEV void fft_pass(const float2* src, float2* dst, int n, int ns, const float2* tw) {
  const int m = n / R, ts = n / (ns * R);
  float2 W[R];
#pragma unroll
  for (int k = 0; k < R; ++k) W[k] = tw[k * m];
  for (int j = threadIdx.x; j < m; j += FFT_NT) {
    const int jn = j % ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = src[j + r * m];
#pragma unroll
    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * jn * ts]);  // r jn ts < n
    const int base = (j - jn) * R + jn;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      float2 acc = v[0];
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const float2 w = W[(r * q) % R];
        acc.x = fmaf(v[r].x, w.x, fmaf(-v[r].y, w.y, acc.x));
        acc.y = fmaf(v[r].x, w.y, fmaf(v[r].y, w.x, acc.y));
      }
      dst[base + q * ns] = acc;
    }
  }
}

struct FftPlanArg { int n, nf, radix[16]; };

// dynamic LDS: twiddles [n] float2 | buffers 2 x [n] float2 | window [n] | band [3*128] int | weights [nnz]
__global__ __launch_bounds__(FFT_NT) void stft_mel_kernel(const float* __restrict__ y, int64_t n_samples, int hop,
                                                          FftPlanArg plan, const float2* __restrict__ tw_g,
                                                          const float* __restrict__ win_g,
                                                          const int* __restrict__ band_g,
                                                          const float* __restrict__ bw_g, int nnz, int F,
                                                          float* __restrict__ mel, int* __restrict__ key) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = plan.n, tid = threadIdx.x;
  float2* tw = (float2*)smem;
  float2* buf0 = tw + n;
  float2* buf1 = buf0 + n;
  float* win = (float*)(buf1 + n);
  int* band = (int*)(win + n);
  float* bw = (float*)(band + 3 * N_MELS);
  for (int k = tid; k < n; k += FFT_NT) {
    tw[k] = tw_g[k];
    win[k] = win_g[k];
  }
  for (int k = tid; k < 3 * N_MELS; k += FFT_NT) band[k] = band_g[k];
  for (int k = tid; k < nnz; k += FFT_NT) bw[k] = bw_g[k];
  float vmax = 0.f;
  const int nb = n / 2 + 1;
  // Two real frames per complex FFT (r3): frame f0 in the real part, f0 + 1 in the
  // imaginary part, Z = X0 + i X1; X0[k] = (Z[k] + conj Z[n-k]) / 2 and
  // X1[k] = (Z[k] - conj Z[n-k]) / 2i, so |X0|^2 = ((zr + zr')^2 + (zi - zi')^2) / 4
  // and |X1|^2 = ((zr - zr')^2 + (zi + zi')^2) / 4 with z' = Z[(n - k) % n]: half the
  // FFT passes (and barriers) per frame.
  for (int fi = 0; fi < FFT_FPB; fi += 2) {
    const int f0 = blockIdx.x * FFT_FPB + fi;
    if (f0 >= F) break;  // uniform over the workgroup
    const bool two = f0 + 1 < F;
    __syncthreads();    // tables loaded / the previous pair's mel reads are done
    const int64_t start = (int64_t)f0 * hop - n / 2;  // center=True, zero padding
    for (int k = tid; k < n; k += FFT_NT) {
      const int64_t i0 = start + k, i1 = i0 + hop;
      const float a = i0 >= 0 && i0 < n_samples ? y[i0] * win[k] : 0.f;
      const float b = two && i1 >= 0 && i1 < n_samples ? y[i1] * win[k] : 0.f;
      buf0[k] = make_float2(a, b);
    }
    __syncthreads();
    float2* src = buf0;
    float2* dst = buf1;
    int ns = 1;
    for (int p = 0; p < plan.nf; ++p) {
      const int r = plan.radix[p];
      switch (r) {
        case 2: fft_pass<2>(src, dst, n, ns, tw); break;
        case 3: fft_pass<3>(src, dst, n, ns, tw); break;
        case 4: fft_pass<4>(src, dst, n, ns, tw); break;
        case 5: fft_pass<5>(src, dst, n, ns, tw); break;
        default: fft_pass<7>(src, dst, n, ns, tw); break;
      }
      ns *= r;
      float2* t = src;
      src = dst;
      dst = t;
      __syncthreads();
    }
    float* pw = (float*)dst;  // |X0|^2 of bins 0..nb-1, then |X1|^2, into the free buffer
    for (int b = tid; b < nb; b += FFT_NT) {
      const float2 z = src[b], zc = src[b == 0 ? 0 : n - b];
      const float ar = z.x + zc.x, ai = z.y - zc.y, br = z.x - zc.x, bi = z.y + zc.y;
      pw[b] = 0.25f * (ar * ar + ai * ai);
      pw[nb + b] = 0.25f * (br * br + bi * bi);
    }
    __syncthreads();
    const int which = tid / N_MELS, m = tid % N_MELS;  // 2 x 128 threads: frame f0 + which, filter m
    if (which < 2 && (which == 0 || two)) {
      const int lo = band[3 * m], cnt = band[3 * m + 1], off = band[3 * m + 2];
      const float* pwf = pw + which * nb;
      float acc = 0.f;
      for (int t = 0; t < cnt; ++t) acc = fmaf(bw[off + t], pwf[lo + t], acc);
      mel[(int64_t)(f0 + which) * N_MELS + m] = acc;
      vmax = fmaxf(vmax, acc);
    }
  }
  if (key != nullptr) {
    vmax = wave_max(vmax);
    if ((tid & 63) == 0) atomicMax(key, __float_as_int(vmax));
  }
}

// Wave-per-pair form (r3, default for n_fft <= SW_MAXN): the workgroup shares the
// tables and nothing else; each wave owns one pair of frames at a time in its own
// LDS buffer and runs the whole transform with no workgroup barrier.  A pass is
// in place: every lane reads the R inputs of its n/(R 64) butterflies into
// registers, the wave's LDS accesses are ordered (in order within a wave), and the
// outputs go to the same buffer.  The power spectrum is written over the buffer
// the same way, then the 2 x 128 mel bands come from it.  Same arithmetic per
// element and same order as stft_mel_kernel.
constexpr int SW_WAVES = 4, SW_MAXN = 1536, SW_NBIN = (SW_MAXN / 2 + 1 + 63) / 64;

template <int R, int NBL>
NSTL_DEV void fft_pass_wave(float2* buf, int n, int ns, const float2* tw, int lane) {
  static_assert(NBL * 64 * R >= SW_MAXN, "butterflies per lane");
  const int m = n / R, ts = n / (ns * R);
  float2 W[R];
#pragma unroll
  for (int k = 0; k < R; ++k) W[k] = tw[k * m];
  float2 v[NBL][R];
#pragma unroll
  for (int i = 0; i < NBL; ++i) {
    const int j = lane + 64 * i;
    if (j < m) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[i][r] = buf[j + r * m];
    }
  }
  wave_lds_order();  // every input is in registers before any output lands
#pragma unroll
  for (int i = 0; i < NBL; ++i) {
    const int j = lane + 64 * i;
    if (j < m) {
      const int jn = j % ns;
#pragma unroll
      for (int r = 1; r < R; ++r) v[i][r] = cmul(v[i][r], tw[r * jn * ts]);  // r jn ts < n
      const int base = (j - jn) * R + jn;
#pragma unroll
      for (int q = 0; q < R; ++q) {
        float2 acc = v[i][0];
#pragma unroll
        for (int r = 1; r < R; ++r) {
          const float2 w = W[(r * q) % R];
          acc.x = fmaf(v[i][r].x, w.x, fmaf(-v[i][r].y, w.y, acc.x));
          acc.y = fmaf(v[i][r].x, w.y, fmaf(v[i][r].y, w.x, acc.y));
        }
        buf[base + q * ns] = acc;
      }
    }
  }
  wave_lds_order();
}

__host__ __device__ inline size_t stft_wave_tables(int n, int nnz) {
  return ((size_t)n * 8 + (size_t)n * 4 + 3 * N_MELS * 4 + (size_t)nnz * 4 + 15) / 16 * 16;
}
size_t stft_wave_lds(int n, int nnz) { return stft_wave_tables(n, nnz) + (size_t)SW_WAVES * n * 8; }

// pairs of frames: wave w of workgroup b takes pairs (b SW_WAVES + w) ppw .. + ppw - 1
__global__ __launch_bounds__(64 * SW_WAVES) void stft_mel_wave_kernel(
    const float* __restrict__ y, int64_t n_samples, int hop, FftPlanArg plan, const float2* __restrict__ tw_g,
    const float* __restrict__ win_g, const int* __restrict__ band_g, const float* __restrict__ bw_g, int nnz, int F,
    float* __restrict__ mel, int* __restrict__ key, int ppw) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = plan.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float2* tw = (float2*)smem;
  float* win = (float*)(tw + n);
  int* band = (int*)(win + n);
  float* bw = (float*)(band + 3 * N_MELS);
  float2* buf = (float2*)(smem + stft_wave_tables(n, nnz)) + (size_t)wv * n;
  for (int k = tid; k < n; k += 64 * SW_WAVES) {
    tw[k] = tw_g[k];
    win[k] = win_g[k];
  }
  for (int k = tid; k < 3 * N_MELS; k += 64 * SW_WAVES) band[k] = band_g[k];
  for (int k = tid; k < nnz; k += 64 * SW_WAVES) bw[k] = bw_g[k];
  __syncthreads();  // the tables: the only workgroup barrier
  // the clip as a buffer resource (the launcher keeps 4 n_samples < 2^31)
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, (int)(n_samples * 4), 0x00020000);
  const int nb = n / 2 + 1, npairs = (F + 1) / 2;
  float vmax = 0.f;
  for (int pi = 0; pi < ppw; ++pi) {
    const int pr = (blockIdx.x * SW_WAVES + wv) * ppw + pi;
    if (pr >= npairs) break;  // uniform over the wave
    const int f0 = 2 * pr;
    const bool two = f0 + 1 < F;
    const int64_t start = (int64_t)f0 * hop - n / 2;  // center=True, zero padding
    // both frames' samples: every load of the lane in flight at once (one memory
    // latency per pair; a load-use loop pays ~n/64 of them).  Buffer loads with
    // 32-bit offsets: a sample outside the clip (the centre padding, a negative
    // offset wraps past the range) reads as 0 from the range check.
    float a[SW_MAXN / 64], b[SW_MAXN / 64];
    const int o0 = (int)start * 4;
#pragma unroll
    for (int u = 0; u < SW_MAXN / 64; ++u) {
      const int off = o0 + (lane + 64 * u) * 4;
      a[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, off, 0, 0));
      b[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, off + hop * 4, 0, 0));
    }
    wave_lds_order();  // the previous pair's mel reads are done
#pragma unroll
    for (int u = 0; u < SW_MAXN / 64; ++u) {
      const int k = lane + 64 * u;
      if (k < n) buf[k] = make_float2(a[u] * win[k], two ? b[u] * win[k] : 0.f);
    }
    wave_lds_order();
    int ns = 1;
    for (int p = 0; p < plan.nf; ++p) {
      const int r = plan.radix[p];
      switch (r) {
        case 2: fft_pass_wave<2, 12>(buf, n, ns, tw, lane); break;
        case 3: fft_pass_wave<3, 8>(buf, n, ns, tw, lane); break;
        case 4: fft_pass_wave<4, 6>(buf, n, ns, tw, lane); break;
        case 5: fft_pass_wave<5, 5>(buf, n, ns, tw, lane); break;
        default: fft_pass_wave<7, 4>(buf, n, ns, tw, lane); break;
      }
      ns *= r;
    }
    // |X0|^2, |X1|^2 of bins 0..nb-1 (see stft_mel_kernel) over the buffer
    float2 z[SW_NBIN], zc[SW_NBIN];
#pragma unroll
    for (int i = 0; i < SW_NBIN; ++i) {
      const int b = lane + 64 * i;
      if (b < nb) {
        z[i] = buf[b];
        zc[i] = buf[b == 0 ? 0 : n - b];
      }
    }
    wave_lds_order();
    float* pw = (float*)buf;
#pragma unroll
    for (int i = 0; i < SW_NBIN; ++i) {
      const int b = lane + 64 * i;
      if (b < nb) {
        const float ar = z[i].x + zc[i].x, ai = z[i].y - zc[i].y, br = z[i].x - zc[i].x, bi = z[i].y + zc[i].y;
        pw[b] = 0.25f * (ar * ar + ai * ai);
        pw[nb + b] = 0.25f * (br * br + bi * bi);
      }
    }
    wave_lds_order();
#pragma unroll
    for (int i = 0; i < 2 * N_MELS / 64; ++i) {
      const int e = lane + 64 * i, which = e / N_MELS, m = e % N_MELS;
      if (which == 0 || two) {
        const int lo = band[3 * m], cnt = band[3 * m + 1], off = band[3 * m + 2];
        const float* pwf = pw + which * nb;
        float acc = 0.f;
        for (int t = 0; t < cnt; ++t) acc = fmaf(bw[off + t], pwf[lo + t], acc);
        mel[(int64_t)(f0 + which) * N_MELS + m] = acc;
        vmax = fmaxf(vmax, acc);
      }
    }
  }
  if (key != nullptr) {
    vmax = wave_max(vmax);
    if (lane == 0) atomicMax(key, __float_as_int(vmax));
  }
}

size_t stft_mel_lds(int n, int nnz) { return (size_t)3 * n * 8 + (size_t)n * 4 + 3 * N_MELS * 4 + (size_t)nnz * 4; }

// |X|^2 for bins 0..nb-1 into rows of nbp (zero tail): the mel GEMM's A operand
__global__ __launch_bounds__(256) void power_kernel(const float* __restrict__ X, int F, int nb, int nbp,
                                                   float* __restrict__ P) {
  const int64_t total = (int64_t)F * nbp;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int f = (int)(e / nbp), b = (int)(e % nbp);
    float v = 0.f;
    if (b < nb) {
      const float c = X[(int64_t)f * 2 * nb + b], s = X[(int64_t)f * 2 * nb + nb + b];
      v = c * c + s * s;
    }
    P[e] = v;
  }
}

// clip-wide max of the mel power (non-negative floats order as their bits)
__global__ __launch_bounds__(256) void melmax_kernel(const float* __restrict__ mel, int64_t n, int* __restrict__ key) {
  float m = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) m = fmaxf(m, mel[e]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(key, __float_as_int(m));
}

// mfcc[k][f] = sum_m dct[k][m] * max(db[f][m], max_db - 80), db = 10 log10(max(1e-10, mel))
__global__ __launch_bounds__(256) void dct_kernel(const float* __restrict__ mel, int F, const float* __restrict__ dct,
                                                  const int* __restrict__ max_key, float* __restrict__ mfcc) {
  __shared__ float tile[64][N_MELS + 1];
  const int f0 = blockIdx.x * 64;
  const float floor_db = 10.f * log10f(fmaxf(1e-10f, __int_as_float(*max_key))) - 80.f;
  for (int i = threadIdx.x; i < 64 * N_MELS; i += 256) {
    const int r = i / N_MELS, m = i % N_MELS;
    tile[r][m] = f0 + r < F ? fmaxf(10.f * log10f(fmaxf(1e-10f, mel[(int64_t)(f0 + r) * N_MELS + m])), floor_db) : 0.f;
  }
  __syncthreads();
  const int r = threadIdx.x & 63;
  for (int k = threadIdx.x >> 6; k < N_MFCC; k += 4) {
    float acc = 0.f;
    for (int m = 0; m < N_MELS; ++m) acc = fmaf(dct[k * N_MELS + m], tile[r][m], acc);
    if (f0 + r < F) mfcc[(int64_t)k * F + f0 + r] = acc;
  }
}

// CMVN, Savitzky-Golay deltas and the pair reduction of the MFCC rows -> out
// columns [c | ncoef + c | 2 ncoef + c] (ncoef = 23 in the feature pipeline), over
// the whole chip (r3; one workgroup per coefficient ran on 23 CUs: 78 -> 18 us per
// 16k output frames).  Stage 1: f64 sums of
// x and x^2 per (coefficient, chunk of frames); stage 2: one thread per output
// row, every block re-deriving mean and deviation from the partials.  The
// deviation is sum (x - mean_f)^2 = sum x^2 - 2 mean_f sum x + F mean_f^2 in f64,
// the two-pass value up to f64 rounding.
constexpr int CMVN_CH = 32;
__global__ __launch_bounds__(256) void cmvn_stats_kernel(const float* __restrict__ mfcc, int F,
                                                         double* __restrict__ part) {
  __shared__ double red[2][4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int chunk = (F + CMVN_CH - 1) / CMVN_CH, i0 = ch * chunk, i1 = min(F, i0 + chunk);
  const float* x = mfcc + (int64_t)c * F;
  double s = 0.0, q = 0.0;
  for (int i = i0 + threadIdx.x; i < i1; i += 256) {
    const double v = x[i];
    s += v;
    q += v * v;
  }
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[(c * CMVN_CH + ch) * 2] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[(c * CMVN_CH + ch) * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ __launch_bounds__(256) void cmvn_delta_out_kernel(const float* __restrict__ mfcc, int F, int ncoef,
                                                             const float* __restrict__ sg,
                                                             const double* __restrict__ part, float* __restrict__ out,
                                                             int64_t ldo, int F60) {
  const int c = blockIdx.x;
  double S = 0.0, Q = 0.0;
  for (int k = 0; k < CMVN_CH; ++k) {
    S += part[(c * CMVN_CH + k) * 2];
    Q += part[(c * CMVN_CH + k) * 2 + 1];
  }
  const float mean = (float)(S / (double)F);
  const double dev = Q - 2.0 * (double)mean * S + (double)F * (double)mean * (double)mean;
  const float sd = sqrtf((float)dev / (float)F);
  const float inv = 1.f / (sd + 1e-10f);
  const float* x = mfcc + (int64_t)c * F;
  const int r = blockIdx.y * 256 + threadIdx.x;
  if (r >= F60) return;
  float v[3] = {0.f, 0.f, 0.f};
  const int j_end = min(2 * r + 2, F);
  for (int j = 2 * r; j < j_end; ++j) {
    const int w0 = min(max(j - SG_W / 2, 0), F - SG_W), t0 = j - w0;
    float d1 = 0.f, d2 = 0.f;
#pragma unroll
    for (int t = 0; t < SG_W; ++t) {
      const float nv = (x[w0 + t] - mean) * inv;
      d1 = fmaf(sg[t0 * SG_W + t], nv, d1);
      d2 = fmaf(sg[SG_W * SG_W + t0 * SG_W + t], nv, d2);
    }
    v[0] += (x[j] - mean) * inv;
    v[1] += d1;
    v[2] += d2;
  }
  const float scale = j_end - 2 * r == 2 ? 0.5f : 1.f;
  float* o = out + (int64_t)r * ldo;
  o[c] = v[0] * scale;
  o[ncoef + c] = v[1] * scale;
  o[2 * ncoef + c] = v[2] * scale;
}

int launch_cmvn(const float* mfcc, int F, int ncoef, const float* sg, double* part, float* out, int64_t ldo, int F60,
                hipStream_t st) {
  hipLaunchKernelGGL(cmvn_stats_kernel, dim3(ncoef, CMVN_CH), dim3(256), 0, st, mfcc, F, part);
  hipLaunchKernelGGL(cmvn_delta_out_kernel, dim3(ncoef, (F60 + 255) / 256), dim3(256), 0, st, mfcc, F, ncoef, sg,
                     part, out, ldo, F60);
  NSTL_LAUNCH_CHECK("cmvn");
  return 0;
}
__device__ double g_cmvn_part[64 * CMVN_CH * 2];  // nstl_cmvn_delta_reduce's partials (ncoef <= 64)

// autocorr lags [F][n_lags] f64 -> pair means -> out[:, col0 + lag] f32
__global__ __launch_bounds__(256) void reduce_ac_kernel(const double* __restrict__ ac, int F, int n_lags,
                                                        float* __restrict__ out, int64_t ldo, int col0, int F60) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)F60 * n_lags) return;
  const int r = (int)(i / n_lags), l = (int)(i % n_lags);
  const int j = 2 * r;
  const double v = j + 1 < F ? (ac[(int64_t)j * n_lags + l] + ac[(int64_t)(j + 1) * n_lags + l]) / 2.0
                             : ac[(int64_t)j * n_lags + l];
  out[(int64_t)r * ldo + col0 + l] = (float)v;
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct FeatLayout {
  int n_fft, hop, nb, kp, F, F60;
  size_t frames, X, db, mfcc, ac, key, cmvn, total;
};

FeatLayout feat_layout(int64_t n_samples, int sr) {
  FeatLayout L;
  L.n_fft = (int)(0.01667 * sr);
  L.hop = L.n_fft / 2;
  L.nb = L.n_fft / 2 + 1;
  L.kp = (L.n_fft + 3) / 4 * 4;
  L.F = L.hop > 0 ? (int)(1 + n_samples / L.hop) : 0;
  L.F60 = (L.F + 1) / 2;
  size_t off = 0;
  L.frames = off; off += align256((size_t)L.F * L.kp * 4);
  L.X = off;      off += align256((size_t)L.F * 2 * L.nb * 4);
  L.db = off;     off += align256((size_t)L.F * N_MELS * 4);
  L.mfcc = off;   off += align256((size_t)L.F * N_MFCC * 4);
  L.ac = off;     off += align256((size_t)L.F * N_AC * 8);
  L.key = off;    off += 256;
  L.cmvn = off;   off += align256((size_t)N_MFCC * CMVN_CH * 2 * 8);
  L.total = off;
  return L;
}

__global__ void init_key(int* k) { *k = 0; }  // mel power >= 0: bits of 0.f

// The autocorrelation depends on the audio only, so nstl_features forks it onto a
// side stream (one per device, created once) and joins before the lag reduction:
// the f64-MFMA-bound autocorrelation runs beside the latency-bound STFT/mel, DCT
// and CMVN chain instead of after it.  NSTL_FEATURES_FORK=0 keeps one stream.
struct FeatFork {
  int dev = -1;
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
std::mutex g_fork_mu;  // held from the fork record to the join wait of one call

bool fork_on() {
  static const bool on = [] {
    const char* e = getenv("NSTL_FEATURES_FORK");
    return !(e && e[0] == '0');
  }();
  return on;
}

// caller holds g_fork_mu
FeatFork* get_fork() {
  static std::deque<FeatFork> forks;  // stable addresses as devices are added
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  for (auto& f : forks)
    if (f.dev == dev) return &f;
  FeatFork f;
  f.dev = dev;
  if (hipStreamCreateWithFlags(&f.side, hipStreamNonBlocking) != hipSuccess) return nullptr;
  if (hipEventCreateWithFlags(&f.fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&f.join, hipEventDisableTiming) != hipSuccess)
    return nullptr;
  forks.push_back(f);
  return &forks.back();
}

// NSTL_FEATURES_FFT=0: the frames -> DFT GEMM -> power -> mel GEMM path instead
// of the fused STFT/mel kernel (A/B comparisons; also any n_fft with a prime
// factor > 7)
bool use_fft(const FeatTables* T) {
  static const int on = [] {
    const char* e = getenv("NSTL_FEATURES_FFT");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on && T->nf > 0;
}

int launch_stft_mel(const FeatTables* T, const float* y, int64_t n_samples, int hop, int F, float* mel, int* key,
                    hipStream_t st) {
  FftPlanArg plan;
  plan.n = T->n_fft;
  plan.nf = T->nf;
  for (int i = 0; i < 16; ++i) plan.radix[i] = T->radix[i];
  static const bool wg_form = [] {
    const char* e = getenv("NSTL_STFT_WG");
    return e && e[0] == '1';
  }();
  if (!wg_form && T->n_fft <= SW_MAXN && n_samples < (int64_t)1 << 29) {
    const size_t lw = stft_wave_lds(T->n_fft, T->nnz);
    int dev = 0, cus = 0, per_cu = 0;
    if (hipFuncSetAttribute((const void*)stft_mel_wave_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lw) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stft_mel_wave_kernel, 64 * SW_WAVES, lw) != hipSuccess)
      return nstl::fail((int)hipErrorInvalidValue, "nstl_features: stft_mel wave kernel setup failed");
    const int npairs = (F + 1) / 2, waves = cus * std::max(per_cu, 1) * SW_WAVES;
    const int ppw = std::max(1, (npairs + waves - 1) / waves);
    const int grid = (npairs + ppw * SW_WAVES - 1) / (ppw * SW_WAVES);
    hipLaunchKernelGGL(stft_mel_wave_kernel, dim3(grid), dim3(64 * SW_WAVES), lw, st, y, n_samples, hop, plan, T->tw,
                       T->window, T->band, T->bw, T->nnz, F, mel, key, ppw);
    NSTL_LAUNCH_CHECK("nstl_features stft_mel (wave)");
    return 0;
  }
  const size_t lds = stft_mel_lds(T->n_fft, T->nnz);
  NSTL_CHECK_ARG(lds <= 160 * 1024, "nstl_features: n_fft %d too large for the fused STFT/mel kernel", T->n_fft);
  hipLaunchKernelGGL(stft_mel_kernel, dim3((F + FFT_FPB - 1) / FFT_FPB), dim3(FFT_NT), lds, st, y, n_samples, hop,
                     plan, T->tw, T->window, T->band, T->bw, T->nnz, F, mel, key);
  NSTL_LAUNCH_CHECK("nstl_features stft_mel");
  return 0;
}
}  // namespace

extern "C" int nstl_stft_mel(const float* y, int64_t n_samples, int sr, float* mel_out, int n_frames, void* stream) {
  NSTL_CHECK_ARG(y && mel_out, "nstl_stft_mel: null pointer");
  NSTL_CHECK_ARG(sr >= 8000 && sr <= 192000, "nstl_stft_mel: sr %d out of range", sr);
  const FeatLayout L = feat_layout(n_samples, sr);
  NSTL_CHECK_ARG(n_samples >= L.n_fft, "nstl_stft_mel: %lld samples < one frame", (long long)n_samples);
  NSTL_CHECK_ARG(n_frames == L.F, "nstl_stft_mel: n_frames %d != %d", n_frames, L.F);
  const FeatTables* T = nullptr;
  if (int rc = get_tables(sr, &T)) return rc;
  NSTL_CHECK_ARG(T->nf > 0, "nstl_stft_mel: n_fft %d has a prime factor > 7", T->n_fft);
  return launch_stft_mel(T, y, n_samples, L.hop, L.F, mel_out, nullptr, (hipStream_t)stream);
}

extern "C" int64_t nstl_features_workspace_bytes(int64_t n_samples, int sr) {
  return (int64_t)feat_layout(n_samples, sr).total;
}

extern "C" int nstl_features_frames(int64_t n_samples, int sr) { return feat_layout(n_samples, sr).F60; }

extern "C" int nstl_features(const float* y, int64_t n_samples, int sr, float* out, int64_t ld_out, int n_out_frames,
                             void* workspace, int64_t workspace_bytes, void* stream) {
  NSTL_CHECK_ARG(y && out && workspace, "nstl_features: null pointer");
  NSTL_CHECK_ARG(sr >= 8000 && sr <= 192000, "nstl_features: sr %d out of range", sr);
  const FeatLayout L = feat_layout(n_samples, sr);
  NSTL_CHECK_ARG(L.n_fft <= MAX_FRAME && n_samples >= L.n_fft, "nstl_features: %lld samples < one frame",
                 (long long)n_samples);
  // extract_features.py:16-21: fewer than 9 frames is rejected by the caller;
  // the Savitzky-Golay fit needs them as well
  NSTL_CHECK_ARG((n_samples - L.n_fft) / L.hop + 1 >= 9, "nstl_features: fewer than 9 frames");
  NSTL_CHECK_ARG(n_out_frames == L.F60, "nstl_features: n_out_frames %d != %d", n_out_frames, L.F60);
  NSTL_CHECK_ARG(ld_out >= 2 * N_MFCC + N_MFCC + N_AC, "nstl_features: ld_out < 256");
  NSTL_CHECK_ARG(workspace_bytes >= (int64_t)L.total, "nstl_features: workspace too small");
  const FeatTables* T = nullptr;
  if (int rc = get_tables(sr, &T)) return rc;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* frames = (float*)(ws + L.frames);
  float* X = (float*)(ws + L.X);
  float* db = (float*)(ws + L.db);
  float* mf = (float*)(ws + L.mfcc);
  double* ac = (double*)(ws + L.ac);
  int* key = (int*)(ws + L.key);
  std::unique_lock<std::mutex> fork_lk(g_fork_mu, std::defer_lock);
  FeatFork* fk = nullptr;
  if (fork_on()) {
    fork_lk.lock();
    fk = get_fork();
  }
  // Once the side stream is forked, every return joins it first: the side stream
  // reads y and writes the workspace, and the caller's allocator may hand those
  // blocks out again on st as soon as st has passed its last use of them.
  struct ForkJoin {
    FeatFork* fk = nullptr;
    hipStream_t st = nullptr;
    bool joined = false;
    ~ForkJoin() {
      if (fk != nullptr && !joined) {
        (void)hipEventRecord(fk->join, fk->side);
        (void)hipStreamWaitEvent(st, fk->join, 0);
      }
    }
  } fj;
  if (fk != nullptr) {
    if (hipEventRecord(fk->fork, st) != hipSuccess || hipStreamWaitEvent(fk->side, fk->fork, 0) != hipSuccess)
      return nstl::fail((int)hipErrorLaunchFailure, "nstl_features: side-stream fork failed");
    fj.fk = fk;
    fj.st = st;
    if (int rc = nstl_autocorr(y, n_samples, L.n_fft, L.hop, N_AC, ac, L.F, fk->side)) return rc;
    if (hipEventRecord(fk->join, fk->side) != hipSuccess)
      return nstl::fail((int)hipErrorLaunchFailure, "nstl_features: side-stream join failed");
  }

  if (use_fft(T)) {
    // fused STFT/mel: mel power -> db buffer, clip-wide max -> key
    hipLaunchKernelGGL(init_key, dim3(1), dim3(1), 0, st, key);
    if (int rc = launch_stft_mel(T, y, n_samples, L.hop, L.F, db, key, st)) return rc;
  } else {
  hipLaunchKernelGGL(stft_frames_kernel, dim3(L.F), dim3(256), 0, st, y, n_samples, L.n_fft, L.hop, L.kp, T->window,
                     frames);
  NSTL_LAUNCH_CHECK("nstl_features frames");
  nstl_gemm_args g = {};
  g.dtype = NSTL_F32; g.c_dtype = NSTL_F32; g.a_kmajor = 1; g.b_kmajor = 1;
  g.A = frames; g.lda = L.kp; g.B = T->basis; g.ldb = L.kp; g.C = X; g.ldc = 2 * L.nb;
  g.M = L.F; g.N = 2 * L.nb; g.K = L.kp; g.alpha = 1.f; g.beta = 0.f; g.epilogue = NSTL_EPI_NONE; g.split_k = 1;
  if (int rc = nstl_gemm(&g, stream)) return rc;
  // mel power = |X|^2 (frames buffer reused) @ mel^T, f32 MFMA GEMM
  float* P = frames;
  const int64_t np = (int64_t)L.F * T->nbp;
  hipLaunchKernelGGL(power_kernel, dim3((unsigned)std::min<int64_t>((np + 255) / 256, 65536)), dim3(256), 0, st, X,
                     L.F, L.nb, T->nbp, P);
  NSTL_LAUNCH_CHECK("nstl_features power");
  nstl_gemm_args gm = {};
  gm.dtype = NSTL_F32; gm.c_dtype = NSTL_F32; gm.a_kmajor = 1; gm.b_kmajor = 1;
  gm.A = P; gm.lda = T->nbp; gm.B = T->melK; gm.ldb = T->nbp; gm.C = db; gm.ldc = N_MELS;
  gm.M = L.F; gm.N = N_MELS; gm.K = T->nbp; gm.alpha = 1.f; gm.beta = 0.f; gm.epilogue = NSTL_EPI_NONE; gm.split_k = 1;
  if (int rc = nstl_gemm(&gm, stream)) return rc;
  hipLaunchKernelGGL(init_key, dim3(1), dim3(1), 0, st, key);
  const int64_t nm = (int64_t)L.F * N_MELS;
  hipLaunchKernelGGL(melmax_kernel, dim3((unsigned)std::min<int64_t>((nm + 255) / 256, 1024)), dim3(256), 0, st, db,
                     nm, key);
  NSTL_LAUNCH_CHECK("nstl_features mel");
  }
  hipLaunchKernelGGL(dct_kernel, dim3((L.F + 63) / 64), dim3(256), 0, st, db, L.F, T->dct, key, mf);
  NSTL_LAUNCH_CHECK("nstl_features dct");
  if (int rc = launch_cmvn(mf, L.F, N_MFCC, T->sg, (double*)(ws + L.cmvn), out, ld_out, L.F60, st)) return rc;
  if (fk != nullptr) {
    fj.joined = true;
    if (hipStreamWaitEvent(st, fk->join, 0) != hipSuccess)
      return nstl::fail((int)hipErrorLaunchFailure, "nstl_features: side-stream join failed");
  } else if (int rc = nstl_autocorr(y, n_samples, L.n_fft, L.hop, N_AC, ac, L.F, stream)) {
    return rc;
  }
  const int64_t n_red = (int64_t)L.F60 * N_AC;
  hipLaunchKernelGGL(reduce_ac_kernel, dim3((unsigned)((n_red + 255) / 256)), dim3(256), 0, st, ac, L.F, N_AC, out,
                     ld_out, 3 * N_MFCC, L.F60);
  NSTL_LAUNCH_CHECK("nstl_features reduce");
  return 0;
}

// The two frame-axis stages of the feature pipeline on their own (their
// reference counterparts are pinned by tests/golden/features_autocorr.npz):
// cepstral_mean_variance_normalization + librosa.feature.delta (width 9, orders
// 1 and 2) + reduce_features of [ncoef][F] coefficient rows, and reduce_features
// of [F][cols] f64 rows (the autocorrelation lags).
extern "C" int nstl_cmvn_delta_reduce(const float* x, int ncoef, int F, float* out, int64_t ld_out, void* stream) {
  NSTL_CHECK_ARG(x && out && ncoef > 0 && F >= SG_W, "nstl_cmvn_delta_reduce: bad sizes (F >= %d)", SG_W);
  NSTL_CHECK_ARG(ld_out >= 3 * ncoef, "nstl_cmvn_delta_reduce: ld_out < 3 ncoef");
  const FeatTables* T = nullptr;
  if (int rc = get_tables(88200, &T)) return rc;  // the Savitzky-Golay table does not depend on sr
  NSTL_CHECK_ARG(ncoef <= 64, "nstl_cmvn_delta_reduce: ncoef <= 64");
  double* part = nullptr;
  if (hipGetSymbolAddress((void**)&part, HIP_SYMBOL(g_cmvn_part)) != hipSuccess)
    return nstl::fail((int)hipErrorUnknown, "nstl_cmvn_delta_reduce: partials buffer");
  return launch_cmvn(x, F, ncoef, T->sg, part, out, ld_out, (F + 1) / 2, (hipStream_t)stream);
}

extern "C" int nstl_reduce_frame_pairs(const double* x, int F, int cols, float* out, int64_t ld_out, int col0,
                                       void* stream) {
  NSTL_CHECK_ARG(x && out && F > 0 && cols > 0 && col0 >= 0 && ld_out >= col0 + cols,
                 "nstl_reduce_frame_pairs: bad sizes");
  const int F60 = (F + 1) / 2;
  const int64_t n = (int64_t)F60 * cols;
  hipLaunchKernelGGL(reduce_ac_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, F, cols,
                     out, ld_out, col0, F60);
  NSTL_LAUNCH_CHECK("nstl_reduce_frame_pairs");
  return 0;
}
