#include <stdlib.h>
// Post-LN residual tails of the NeuroSync Seq2Seq layers (utils/model.py:175-180,
// :198-207, final norms :228-229/:249-250):
//   forward : s = x + y * m1 * m2 / (1-p)^n ; out = (s - mean) * rstd * gamma + beta
//             (+ optional global-PE rotation of `out`, model.py:246)
//   backward: ds = rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat));
//             dbranch = ds * masks / (1-p)^n ; per-block dgamma/dbeta partials.
// One wave per row; each lane owns VPL = D/64 columns: contiguous (D = 128), or
// when D % 256 == 0 four-column groups 256 apart (every wave instruction then
// covers one contiguous span).
#include <algorithm>

#include "../../include/nstl.h"
#include "common.h"
#include "status.h"

namespace {

constexpr int NT = 256;

template <typename T, int VPL>
NSTL_DEV void load_row(const T* p, float (&v)[VPL]) {
  if constexpr ((VPL * sizeof(T)) % 16 == 0) {
    constexpr int NV = VPL * sizeof(T) / 16;
    constexpr int EPV = 16 / sizeof(T);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const uint4 u = ((const uint4*)p)[k];
      const T* e = (const T*)&u;
#pragma unroll
      for (int j = 0; j < EPV; ++j) v[k * EPV + j] = to_f32(e[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < VPL; ++j) v[j] = to_f32(p[j]);
  }
}

template <typename T, int VPL>
NSTL_DEV void store_row(T* p, const float (&v)[VPL]) {
  if constexpr ((VPL * sizeof(T)) % 16 == 0) {
    constexpr int NV = VPL * sizeof(T) / 16;
    constexpr int EPV = 16 / sizeof(T);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      uint4 u;
      T* e = (T*)&u;
#pragma unroll
      for (int j = 0; j < EPV; ++j) e[j] = from_f32<T>(v[k * EPV + j]);
      ((uint4*)p)[k] = u;
    }
  } else {
#pragma unroll
    for (int j = 0; j < VPL; ++j) p[j] = from_f32<T>(v[j]);
  }
}

struct LnParams {
  const char* x; const char* y;
  int rows, D;
  int n_masks; uint32_t thresh; float inv_keep; uint64_t seed1, seed2;
  const float* gamma; const float* beta; float eps;
  char* s_out; char* out; float* mean; float* rstd;
  char* rot_out; const float* rope_cos; const float* rope_sin; int rope_T;
  const char* s_in; const float* dout; float* ds; char* dbranch;
  const char* dout2;  // optional dtype addend of dout
  float* dgp; float* dbp; float* dyp;
  uint8_t* q8; int64_t ldq8; float* q8_scale;  // forward: row-wise e4m3 copy of out (fp8.hip rule)
};

// dropout scale of the element pair (idx, idx+1), idx even: 1 or 2 stacked masks
// (32-bit pair index idx / 2: the launcher checks rows * D <= 2^33)
NSTL_DEV void branch_scale2(const LnParams& p, uint64_t idx, float& m0, float& m1) {
  bool a0, a1, b0 = true, b1 = true;
  const uint32_t pair = (uint32_t)(idx >> 1);
  nstl_keep2_32(nstl_seed_term(p.seed1), pair, p.thresh, a0, a1);
  if (p.n_masks >= 2) nstl_keep2_32(nstl_seed_term(p.seed2), pair, p.thresh, b0, b1);
  const float s = p.n_masks >= 2 ? p.inv_keep * p.inv_keep : p.inv_keep;
  m0 = (a0 && b0) ? s : 0.f;
  m1 = (a1 && b1) ? s : 0.f;
}

template <typename T, int VPL>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(LnParams p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int c0 = lane * VPL;
  const int64_t base = (int64_t)row * p.D + c0;
  float s[VPL];
  load_row<T, VPL>((const T*)p.y + base, s);
  if (p.thresh && p.n_masks > 0) {
#pragma unroll
    for (int j = 0; j < VPL; j += 2) {
      float m0, m1;
      branch_scale2(p, (uint64_t)base + j, m0, m1);
      s[j] *= m0;
      s[j + 1] *= m1;
    }
  }
  if (p.x) {
    float xv[VPL];
    load_row<T, VPL>((const T*)p.x + base, xv);
#pragma unroll
    for (int j = 0; j < VPL; ++j) s[j] += xv[j];
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) sum += s[j];
  const float mean = wave_sum(sum) / p.D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const float d = s[j] - mean;
    sq += d * d;
  }
  const float rstd = rsqrtf(wave_sum(sq) / p.D + p.eps);
  if (p.s_out) store_row<T, VPL>((T*)p.s_out + base, s);
  float o[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) o[j] = (s[j] - mean) * rstd * p.gamma[c0 + j] + p.beta[c0 + j];
  // round to the storage type first so `rot_out` rotates exactly what `out` holds
#pragma unroll
  for (int j = 0; j < VPL; ++j) o[j] = to_f32(from_f32<T>(o[j]));
  store_row<T, VPL>((T*)p.out + base, o);
  if (lane == 0) {
    p.mean[row] = mean;
    p.rstd[row] = rstd;
  }
  if (p.rot_out) {
    const int t = row % p.rope_T, half = p.D >> 1;
    float r[VPL];
#pragma unroll
    for (int j = 0; j < VPL; j += 2) {
      const int pr = (c0 + j) >> 1;
      const float c = p.rope_cos[t * half + pr], sn = p.rope_sin[t * half + pr];
      r[j] = o[j] * c - o[j + 1] * sn;
      r[j + 1] = o[j] * sn + o[j + 1] * c;
    }
    store_row<T, VPL>((T*)p.rot_out + base, r);
  }
}

template <typename T, int VPL>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(LnParams p) {
  const int lane = threadIdx.x & 63;
  const int c0 = lane * VPL;
  float gam[VPL], dg[VPL], db[VPL], dyb[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    gam[j] = p.gamma[c0 + j];
    dg[j] = 0.f;
    db[j] = 0.f;
    dyb[j] = 0.f;
  }
  for (int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6); row < p.rows; row += gridDim.x * (NT / 64)) {
    const int64_t base = (int64_t)row * p.D + c0;
    const float mean = p.mean[row], rstd = p.rstd[row];
    float xh[VPL], gy[VPL];
    load_row<T, VPL>((const T*)p.s_in + base, xh);
    load_row<float, VPL>(p.dout + base, gy);
    if (p.dout2) {
      float g2[VPL];
      load_row<T, VPL>((const T*)p.dout2 + base, g2);
#pragma unroll
      for (int j = 0; j < VPL; ++j) gy[j] += g2[j];
    }
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xh[j] = (xh[j] - mean) * rstd;
      dg[j] += gy[j] * xh[j];
      db[j] += gy[j];
      const float gg = gy[j] * gam[j];
      a1 += gg;
      a2 += gg * xh[j];
    }
    const float m1 = wave_sum(a1) / p.D, m2 = wave_sum(a2) / p.D;
    float d[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) d[j] = rstd * (gy[j] * gam[j] - m1 - xh[j] * m2);
    store_row<float, VPL>(p.ds + base, d);
    if (p.dbranch) {
      if (p.thresh && p.n_masks > 0) {
#pragma unroll
        for (int j = 0; j < VPL; j += 2) {
          float m0, m1;
          branch_scale2(p, (uint64_t)base + j, m0, m1);
          d[j] *= m0;
          d[j + 1] *= m1;
        }
      }
#pragma unroll
      for (int j = 0; j < VPL; ++j) d[j] = to_f32(from_f32<T>(d[j]));  // sum what is stored
      store_row<T, VPL>((T*)p.dbranch + base, d);
#pragma unroll
      for (int j = 0; j < VPL; ++j) dyb[j] += d[j];
    }
  }
  // per-block partials: reduce the 4 waves through LDS
  __shared__ float red[3][NT / 64][1024];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    red[0][w][c0 + j] = dg[j];
    red[1][w][c0 + j] = db[j];
    red[2][w][c0 + j] = dyb[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.D; c += NT) {
    float a = 0.f, b = 0.f, y = 0.f;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
      a += red[0][k][c];
      b += red[1][k][c];
      y += red[2][k][c];
    }
    p.dgp[(int64_t)blockIdx.x * p.D + c] = a;
    p.dbp[(int64_t)blockIdx.x * p.D + c] = b;
    if (p.dyp) p.dyp[(int64_t)blockIdx.x * p.D + c] = y;
  }
}

// Backward for D % 256 == 0 (the step's D = 1024): 8 waves per block, lane l
// owns columns k*256 + 4l .. +3 (k < D/256), so every load/store instruction of
// a wave covers one contiguous 512 B (bf16) / 1 KB (f32) span, and the next
// row's inputs are loaded before the current row is reduced (two rows in flight
// per wave: ~100 KB per CU, what HBM latency needs).
constexpr int NTB = 512;

template <typename T>
NSTL_DEV void load4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 2) {
    const uint2 u = *(const uint2*)p;
    const T* e = (const T*)&u;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = to_f32(e[j]);
  } else {
    const float4 u = *(const float4*)p;
    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
  }
}
// G consecutive columns of a row (G = 8: one 16-byte bf16 access, two for f32)
template <typename T, int G>
NSTL_DEV void loadG(const T* p, float (&v)[G]) {
  if constexpr (G == 4) {
    load4<T>(p, v);
  } else if constexpr (sizeof(T) == 2) {
    const uint4 u = *(const uint4*)p;
    const T* e = (const T*)&u;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = to_f32(e[j]);
  } else {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
NSTL_DEV void store4(T* p, const float* v);
template <typename T, int G>
NSTL_DEV void storeG(T* p, const float* v) {
  if constexpr (G == 4) {
    store4<T>(p, v);
  } else if constexpr (sizeof(T) == 2) {
    uint4 u;
    T* e = (T*)&u;
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = from_f32<T>(v[j]);
    *(uint4*)p = u;
  } else {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename T>
NSTL_DEV void store4(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    uint2 u;
    T* e = (T*)&u;
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = from_f32<T>(v[j]);
    *(uint2*)p = u;
  } else {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// The row-wise e4m3 copy of a stored row v (already rounded to the storage type),
// the same arithmetic as nstl_fp8_quant_rows: the forward's LN output (the next fp8
// projection's operand) or, in the backward, dbranch (the fp8 input-gradient GEMM's
// A operand).  Interleaved column map: lane l owns columns k*64G + G*l .. +G-1.
template <int VPL, int G>
NSTL_DEV void q8_row(const LnParams& p, int row, int lane, const float (&v)[VPL]) {
  constexpr int NK = VPL / G, SPAN = 64 * G;
  float am = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) am = fmaxf(am, fabsf(v[j]));
  am = wave_max(am);
  const float inv = am > 0.f ? 448.f / am : 1.f;
  if (lane == 0) p.q8_scale[row] = am > 0.f ? am / 448.f : 1.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    float x[G];
#pragma unroll
    for (int e = 0; e < G; ++e) x[e] = fminf(fmaxf(v[G * k + e] * inv, -448.f), 448.f);
    uint32_t b[G / 4];
#pragma unroll
    for (int h = 0; h < G / 4; ++h)
      b[h] = ((uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h], x[4 * h + 1], 0, false) & 0xffffu) |
             (((uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h + 2], x[4 * h + 3], 0, false) & 0xffffu) << 16);
    uint8_t* q = p.q8 + (int64_t)row * p.ldq8 + k * SPAN + G * lane;
    if constexpr (G == 8) *(uint2*)q = make_uint2(b[0], b[1]);
    else *(uint32_t*)q = b[0];
  }
}

template <typename T, int VPL, int G>
__global__ __launch_bounds__(NTB) void ln_bwd_kernel_il(LnParams p) {
  constexpr int NK = VPL / G;  // G-column groups per lane
  constexpr int SPAN = 64 * G;
  constexpr int NWB = NTB / 64;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float gam[VPL], dg[VPL], db[VPL], dyb[VPL];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < G; ++e) {
      gam[G * k + e] = p.gamma[k * SPAN + G * lane + e];
      dg[G * k + e] = db[G * k + e] = dyb[G * k + e] = 0.f;
    }
  const int stride = gridDim.x * NWB;
  int row = blockIdx.x * NWB + w;
  float xh[VPL], gy[VPL], mean = 0.f, rstd = 0.f;
  auto load = [&](int r, float (&x)[VPL], float (&g)[VPL], float& mu, float& rs) {
    const int64_t base = (int64_t)r * p.D + G * lane;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float t4[G], g4[G], a4[G];
#pragma unroll
      for (int e = 0; e < G; ++e) a4[e] = 0.f;
      loadG<T, G>((const T*)p.s_in + base + k * SPAN, t4);
      loadG<float, G>(p.dout + base + k * SPAN, g4);
      if (p.dout2) loadG<T, G>((const T*)p.dout2 + base + k * SPAN, a4);
#pragma unroll
      for (int e = 0; e < G; ++e) {
        x[G * k + e] = t4[e];
        g[G * k + e] = g4[e] + a4[e];
      }
    }
    mu = p.mean[r];
    rs = p.rstd[r];
  };
  if (row < p.rows) load(row, xh, gy, mean, rstd);
  for (; row < p.rows; row += stride) {
    const int nxt = row + stride;
    float xn[VPL], gn[VPL], mn = 0.f, rn = 0.f;
    if (nxt < p.rows) load(nxt, xn, gn, mn, rn);
    const int64_t base = (int64_t)row * p.D + G * lane;
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xh[j] = (xh[j] - mean) * rstd;
      dg[j] += gy[j] * xh[j];
      db[j] += gy[j];
      const float gg = gy[j] * gam[j];
      a1 += gg;
      a2 += gg * xh[j];
    }
    const float m1 = wave_sum(a1) / p.D, m2 = wave_sum(a2) / p.D;
    float d[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) d[j] = rstd * (gy[j] * gam[j] - m1 - xh[j] * m2);
#pragma unroll
    for (int k = 0; k < NK; ++k) storeG<float, G>(p.ds + base + k * SPAN, d + G * k);
    if (p.dbranch) {
      if (p.thresh && p.n_masks > 0) {
#pragma unroll
        for (int k = 0; k < NK; ++k)
#pragma unroll
          for (int e = 0; e < G; e += 2) {
            float s0, s1;
            branch_scale2(p, (uint64_t)base + k * SPAN + e, s0, s1);
            d[G * k + e] *= s0;
            d[G * k + e + 1] *= s1;
          }
      }
#pragma unroll
      for (int j = 0; j < VPL; ++j) d[j] = to_f32(from_f32<T>(d[j]));  // sum what is stored
#pragma unroll
      for (int k = 0; k < NK; ++k) storeG<T, G>((T*)p.dbranch + base + k * SPAN, d + G * k);
#pragma unroll
      for (int j = 0; j < VPL; ++j) dyb[j] += d[j];
      if (p.q8) q8_row<VPL, G>(p, row, lane, d);  // fp8 backward: the e4m3 copy of dbranch
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      xh[j] = xn[j];
      gy[j] = gn[j];
    }
    mean = mn;
    rstd = rn;
  }
  // per-block partials: reduce the waves through LDS, column order
  __shared__ float red[3][NWB][1024];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < G; ++e) {
      const int c = k * SPAN + G * lane + e;
      red[0][w][c] = dg[G * k + e];
      red[1][w][c] = db[G * k + e];
      red[2][w][c] = dyb[G * k + e];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < p.D; c += NTB) {
    float a = 0.f, b = 0.f, y = 0.f;
#pragma unroll
    for (int k = 0; k < NWB; ++k) {
      a += red[0][k][c];
      b += red[1][k][c];
      y += red[2][k][c];
    }
    p.dgp[(int64_t)blockIdx.x * p.D + c] = a;
    p.dbp[(int64_t)blockIdx.x * p.D + c] = b;
    if (p.dyp) p.dyp[(int64_t)blockIdx.x * p.D + c] = y;
  }
}

// Forward with the interleaved column map of ln_bwd_kernel_il (D % 256 == 0):
// lane l owns columns k*256 + 4l .. +3, one row per wave.
template <typename T, int VPL, int G>
__global__ __launch_bounds__(NT) void ln_fwd_kernel_il(LnParams p) {
  constexpr int NK = VPL / G;
  constexpr int SPAN = 64 * G;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (row >= p.rows) return;
  const int64_t base = (int64_t)row * p.D + G * lane;
  float s[VPL], xv[VPL];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    float y4[G], x4[G];
#pragma unroll
    for (int e = 0; e < G; ++e) x4[e] = 0.f;
    loadG<T, G>((const T*)p.y + base + k * SPAN, y4);
    if (p.x) loadG<T, G>((const T*)p.x + base + k * SPAN, x4);
#pragma unroll
    for (int e = 0; e < G; ++e) {
      s[G * k + e] = y4[e];
      xv[G * k + e] = x4[e];
    }
  }
  if (p.thresh && p.n_masks > 0) {
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int e = 0; e < G; e += 2) {
        float m0, m1;
        branch_scale2(p, (uint64_t)base + k * SPAN + e, m0, m1);
        s[G * k + e] *= m0;
        s[G * k + e + 1] *= m1;
      }
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    s[j] += xv[j];
    sum += s[j];
  }
  const float mean = wave_sum(sum) / p.D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const float d = s[j] - mean;
    sq += d * d;
  }
  const float rstd = rsqrtf(wave_sum(sq) / p.D + p.eps);
  float o[VPL];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    if (p.s_out) storeG<T, G>((T*)p.s_out + base + k * SPAN, s + G * k);
#pragma unroll
    for (int e = 0; e < G; ++e) {
      const int c = k * SPAN + G * lane + e;
      // round to the storage type first so `rot_out` rotates exactly what `out` holds
      o[G * k + e] = to_f32(from_f32<T>((s[G * k + e] - mean) * rstd * p.gamma[c] + p.beta[c]));
    }
    storeG<T, G>((T*)p.out + base + k * SPAN, o + G * k);
  }
  if (lane == 0) {
    p.mean[row] = mean;
    p.rstd[row] = rstd;
  }
  if (p.q8) q8_row<VPL, G>(p, row, lane, o);
  if (p.rot_out) {
    const int t = row % p.rope_T, half = p.D >> 1;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      float r[G];
#pragma unroll
      for (int e = 0; e < G; e += 2) {
        const int pr = (k * SPAN + G * lane + e) >> 1;
        const float c = p.rope_cos[t * half + pr], sn = p.rope_sin[t * half + pr];
        r[e] = o[G * k + e] * c - o[G * k + e + 1] * sn;
        r[e + 1] = o[G * k + e] * sn + o[G * k + e + 1] * c;
      }
      storeG<T, G>((T*)p.rot_out + base + k * SPAN, r);
    }
  }
}

// NSTL_LN_G8=0: four-column lane groups (8-byte bf16 accesses) when D % 512 == 0
bool ln_g8() {
  static const int v = [] {
    const char* e = getenv("NSTL_LN_G8");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return v != 0;
}

template <typename T, bool BWD>
int dispatch(const LnParams& p, int grid, hipStream_t st) {
#define NSTL_LN_CASE(V)                                                                     \
  case V:                                                                                   \
    if (BWD && V % 8 == 0 && ln_g8())                                                       \
      hipLaunchKernelGGL((ln_bwd_kernel_il<T, (V % 8 == 0 ? V : 8), 8>), dim3(grid), dim3(NTB), 0, st, p); \
    else if (BWD && V % 4 == 0)                                                             \
      hipLaunchKernelGGL((ln_bwd_kernel_il<T, (V % 4 == 0 ? V : 4), 4>), dim3(grid), dim3(NTB), 0, st, p); \
    else if (BWD) hipLaunchKernelGGL((ln_bwd_kernel<T, V>), dim3(grid), dim3(NT), 0, st, p); \
    else if (V % 8 == 0 && ln_g8())                                                         \
      hipLaunchKernelGGL((ln_fwd_kernel_il<T, (V % 8 == 0 ? V : 8), 8>), dim3(grid), dim3(NT), 0, st, p); \
    else if (V % 4 == 0)                                                                    \
      hipLaunchKernelGGL((ln_fwd_kernel_il<T, (V % 4 == 0 ? V : 4), 4>), dim3(grid), dim3(NT), 0, st, p); \
    else hipLaunchKernelGGL((ln_fwd_kernel<T, V>), dim3(grid), dim3(NT), 0, st, p);        \
    break;
  switch (p.D / 64) {
    NSTL_LN_CASE(2)
    NSTL_LN_CASE(4)
    NSTL_LN_CASE(8)
    NSTL_LN_CASE(16)
    default:
      return nstl::fail((int)hipErrorInvalidValue, "nstl_ln: D=%d unsupported (128/256/512/1024)", p.D);
  }
#undef NSTL_LN_CASE
  NSTL_LAUNCH_CHECK(BWD ? "nstl_ln_bwd" : "nstl_ln_fwd");
  return 0;
}

int fill(LnParams& p, const nstl_ln_args* a) {
  NSTL_CHECK_ARG(a != nullptr, "nstl_ln: null args");
  NSTL_CHECK_ARG(a->dtype == NSTL_F32 || a->dtype == NSTL_BF16, "nstl_ln: bad dtype");
  NSTL_CHECK_ARG(a->rows > 0 && a->D > 0 && a->D % 64 == 0 && a->D <= 1024, "nstl_ln: bad shape");
  NSTL_CHECK_ARG(a->gamma && a->beta, "nstl_ln: gamma/beta missing");
  NSTL_CHECK_ARG(a->n_masks >= 0 && a->n_masks <= 2 && a->p_drop >= 0.f && a->p_drop < 1.f, "nstl_ln: dropout");
  NSTL_CHECK_ARG(a->p_drop == 0.f || nstl_pair_index32_ok((uint64_t)a->rows * a->D),
                 "nstl_ln: rows*D past 2^33 dropout elements (32-bit pair index)");
  p.x = (const char*)a->x; p.y = (const char*)a->y;
  p.rows = a->rows; p.D = a->D;
  p.n_masks = a->n_masks;
  p.thresh = nstl_drop_thresh(a->p_drop);
  p.inv_keep = 1.0f / (1.0f - a->p_drop);
  p.seed1 = a->seed1; p.seed2 = a->seed2;
  p.gamma = a->gamma; p.beta = a->beta; p.eps = a->eps;
  p.s_out = (char*)a->s_out; p.out = (char*)a->out; p.mean = a->mean; p.rstd = a->rstd;
  p.rot_out = (char*)a->rot_out; p.rope_cos = a->rope_cos; p.rope_sin = a->rope_sin; p.rope_T = a->rope_T;
  p.s_in = (const char*)a->s_in; p.dout = a->dout; p.ds = a->ds; p.dbranch = (char*)a->dbranch;
  p.dgp = a->dgamma_part; p.dbp = a->dbeta_part; p.dyp = a->dbranch_part;
  p.dout2 = (const char*)a->dout2;
  p.q8 = (uint8_t*)a->q8; p.ldq8 = a->ldq8; p.q8_scale = a->q8_scale;
  return 0;
}

}  // namespace

extern "C" int nstl_ln_fwd(const nstl_ln_args* a, void* stream) {
  LnParams p;
  int rc = fill(p, a);
  if (rc) return rc;
  NSTL_CHECK_ARG(a->y && a->out && a->mean && a->rstd, "nstl_ln_fwd: null tensor");
  NSTL_CHECK_ARG(!a->rot_out || (a->rope_cos && a->rope_sin && a->rope_T > 0), "nstl_ln_fwd: rope tables");
  NSTL_CHECK_ARG(!a->q8 || (a->dtype == NSTL_BF16 && a->q8_scale && a->D % 256 == 0 && a->ldq8 >= a->D &&
                            a->ldq8 % 16 == 0 && ((uintptr_t)a->q8 % 16) == 0),
                 "nstl_ln_fwd: q8 needs bf16, D %% 256 == 0, q8_scale and a 16-byte aligned ldq8 >= D");
  const int grid = (a->rows + NT / 64 - 1) / (NT / 64);
  return a->dtype == NSTL_BF16 ? dispatch<bf16, false>(p, grid, (hipStream_t)stream)
                               : dispatch<float, false>(p, grid, (hipStream_t)stream);
}

extern "C" int nstl_ln_bwd(const nstl_ln_args* a, void* stream) {
  LnParams p;
  int rc = fill(p, a);
  if (rc) return rc;
  NSTL_CHECK_ARG(a->s_in && a->dout && a->ds && a->mean && a->rstd, "nstl_ln_bwd: null tensor");
  NSTL_CHECK_ARG(a->dgamma_part && a->dbeta_part && a->n_part > 0, "nstl_ln_bwd: partials");
  NSTL_CHECK_ARG(!a->q8 || (a->dbranch && a->dtype == NSTL_BF16 && a->q8_scale && a->D % 256 == 0 &&
                            a->ldq8 >= a->D && a->ldq8 % 16 == 0 && ((uintptr_t)a->q8 % 16) == 0),
                 "nstl_ln_bwd: q8 needs dbranch, bf16, D %% 256 == 0, q8_scale and a 16-byte aligned ldq8 >= D");
  // n_part blocks; each needs at least one row per wave (4 waves; 8 when D % 256 == 0)
  const int nw = (a->D % 256 == 0) ? NTB / 64 : NT / 64;
  const int grid = std::min(a->n_part, (a->rows + nw - 1) / nw);
  NSTL_CHECK_ARG(grid == a->n_part, "nstl_ln_bwd: n_part (%d) must be <= rows/%d", a->n_part, nw);
  return a->dtype == NSTL_BF16 ? dispatch<bf16, true>(p, grid, (hipStream_t)stream)
                               : dispatch<float, true>(p, grid, (hipStream_t)stream);
}
