// Multi-head attention forward/backward for the NeuroSync Seq2Seq
// (replaces F.scaled_dot_product_attention, utils/model.py:126-127, and its
// autograd backward; RoPE (apply_rope_qk, :60-83) is applied to q/k by the
// projection epilogue, and rotated back here on dq/dk).
//
// Shapes are short: T <= 256 frames, dh = 64.  A whole (batch, head) key/value
// sequence fits in LDS, so there is no online softmax and no cross-workgroup
// reduction:
//   forward : workgroup = (b, h, 64 query rows); each wave 16 rows; scores for
//             all keys live in MFMA accumulators; exact softmax; P^T is staged
//             through a per-wave LDS image (one 8-byte write per lane and key
//             tile) and read back with transpose reads as the A operand of P.V.
//   backward: workgroup = (b, h); phase 1 waves own 16-key tiles and accumulate
//             dK, dV over all queries; phase 2 waves own 16-query tiles and
//             accumulate dQ (scores/probabilities recomputed from the saved LSE).
// Q/K/V/dO tiles arrive by LDS-DMA (global_load_lds_dwordx4, all in flight
// together; bank swizzle applied on the source address).  Dropout keep-mask is a
// counter hash of (b, h, key, query): regenerated in backward, never stored.
#include <algorithm>

#include "../../include/nstl.h"
#include "common.h"
#include "status.h"

namespace {

constexpr int DH = 64;
constexpr int NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnParams {
  const char* q; int64_t q_ld;
  const char* k; int64_t k_ld;
  const char* v; int64_t v_ld;
  char* o; int64_t o_ld;
  float* lse;
  float* dsum;
  uint64_t* mask;  // dropout keep bits (fast path), see mask_word()
  float* dbias;    // optional [B * nblk][3 * H * DH] column sums of dq | dk | dv (fast path)
  const char* dout; int64_t dout_ld;
  char* dq; int64_t dq_ld;
  char* dk; int64_t dk_ld;
  char* dv; int64_t dv_ld;
  const float* rope_cos; const float* rope_sin; int rope_q, rope_k;
  int B, T, H, dh;
  float scale;
  uint32_t thresh; float inv_keep; uint64_t seed;
};

// LDS-DMA rows [0, nrows) of a (b, h) slice (64 elements per row) into an
// ImgK<RB> image.  One wave instruction moves 1 KB = 1024/RB rows; the image
// swizzle is applied to the per-lane source chunk.
template <int RB, int NW = NT / 64>
NSTL_DEV void dma_rows(char* img, const char* g, int64_t ld_bytes, int nrows, int wave, int lane) {
  constexpr int RPK = 1024 / RB, CPR = RB / 16;
  const int ninst = nrows / RPK;
  for (int q = wave; q < ninst; q += NW) {
    const int row = q * RPK + lane / CPR, pc = lane % CPR;
    const int x = RB == 128 ? ((row >> 1) & 7) : (row & 15);
    const int lc = pc ^ x;
    const char* src = g + row * ld_bytes + lc * 16;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)(img + q * 1024), 16, 0, 0);
  }
}

template <typename T>
NSTL_DEV void store_elem(char* base, int64_t e, float v) {
  ((T*)base)[e] = from_f32<T>(v);
}

// dropout element index: key-major so that (q, q+1) form a hash pair
NSTL_DEV uint64_t drop_idx(int bh, int T, int q, int k) { return ((uint64_t)bh * T + k) * T + q; }

// Stored keep bits (MFMA path): one 64-bit word per (query tile qt, key tile kt,
// query % 4) of a head, bit 16 * ((q % 16) / 4) + key % 16 -- exactly the
// ballot of the keep decisions of one accumulator register r over a wave in
// the forward / dQ layout (lane 16g + c: query 4g + r, key c).  A head's words
// are [qt][kt][4] (T*T/64 of them).
NSTL_DEV int64_t mask_word(int bh, int nt, int qt, int kt, int r) {
  return (((int64_t)bh * nt + qt) * nt + kt) * 4 + r;
}
NSTL_DEV uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src), hi = __shfl((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
NSTL_DEV uint64_t readlane64(uint64_t v, int src) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, src);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

// four consecutive values of one lane as an 8-byte (bf16) / 16-byte (f32) LDS write
NSTL_DEV void put4(char* dst, float a, float b, float c, float d, bf16) {
  *(bf16x4*)dst = (bf16x4){(bf16)a, (bf16)b, (bf16)c, (bf16)d};
}
NSTL_DEV void put4(char* dst, float a, float b, float c, float d, float) {
  *(f32x4*)dst = (f32x4){a, b, c, d};
}

// ----------------------------------------------------------------------------
// Forward: one workgroup of FWD_NT/64 waves per (b, h) and 16*FWD_NT/64 queries
// (all of T=128), so K and V are staged once per (b, h); each wave owns 16
// query rows.
constexpr int FWD_NT = 512, FWD_QB = 16 * FWD_NT / 64;

template <typename T>
__global__ __launch_bounds__(FWD_NT) void attn_fwd_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;   // 128 (bf16) / 256 (f32)
  constexpr int RBP = 16 * ESZ;   // P^T image rows: 16 queries
  typedef ImgK<RBK> Img;
  typedef ImgPlain<RBP> ImgP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Kimg = smem;
  char* Vimg = Kimg + T_ * RBK;
  char* Qimg = Vimg + T_ * RBK;
  char* Pimg = Qimg + FWD_QB * RBK;

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int qb0 = blockIdx.x * FWD_QB;
  const int nq = min(FWD_QB, T_ - qb0);
  const int64_t tok0 = (int64_t)b * T_;
  constexpr int NW = FWD_NT / 64;

  dma_rows<RBK, NW>(Kimg, p.k + (tok0 * p.k_ld + h * DH) * ESZ, p.k_ld * ESZ, T_, w, lane);
  dma_rows<RBK, NW>(Vimg, p.v + (tok0 * p.v_ld + h * DH) * ESZ, p.v_ld * ESZ, T_, w, lane);
  dma_rows<RBK, NW>(Qimg, p.q + ((tok0 + qb0) * p.q_ld + h * DH) * ESZ, p.q_ld * ESZ, nq, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int q0 = w * 16;  // local row base of this wave
  if (q0 < nq) {
    Frag fq[2];
    frag_row<Img>(fq[0], Qimg, q0 + (lane & 15), 8 * g);
    frag_row<Img>(fq[1], Qimg, q0 + (lane & 15), 32 + 8 * g);
    f32x4 s[16];
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) {
      s[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (kt < nkt) {
        Frag fk0, fk1;
        frag_row<Img>(fk0, Kimg, kt * 16 + (lane & 15), 8 * g);
        frag_row<Img>(fk1, Kimg, kt * 16 + (lane & 15), 32 + 8 * g);
        mma16(s[kt], fq[0], fk0);
        mma16(s[kt], fq[1], fk1);
      }
    }
    const float c2 = p.scale * LOG2E;
    float mx[4], sum[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 16; ++kt)
        if (kt < nkt) m = fmaxf(m, s[kt][r]);
      m = fmaxf(m, __shfl_xor(m, 1));
      m = fmaxf(m, __shfl_xor(m, 2));
      m = fmaxf(m, __shfl_xor(m, 4));
      m = fmaxf(m, __shfl_xor(m, 8));
      mx[r] = m;
      float sm = 0.f;
#pragma unroll
      for (int kt = 0; kt < 16; ++kt)
        if (kt < nkt) {
          const float e = exp2f((s[kt][r] - m) * c2);
          s[kt][r] = e;
          sm += e;
        }
      sm += __shfl_xor(sm, 1);
      sm += __shfl_xor(sm, 2);
      sm += __shfl_xor(sm, 4);
      sm += __shfl_xor(sm, 8);
      sum[r] = sm;
    }
    // dropout + P^T (unnormalised) into this wave's image [T keys][16 rows]
    char* Pw = Pimg + w * max(T_, 64) * RBP;  // also holds the 16 x 64 O tile
    const int qrow = qb0 + q0 + 4 * g;  // this lane's first query (even)
    uint32_t mlo = 0, mhi = 0;          // lane kt*4 + r: keep bits of (kt, r)
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) {
      if (kt < nkt) {
        const int key = kt * 16 + (lane & 15);
        float v0 = s[kt][0], v1 = s[kt][1], v2 = s[kt][2], v3 = s[kt][3];
        if (p.thresh) {
          bool k0, k1, k2, k3;
          const uint64_t idx = drop_idx(bh, T_, qrow, key);
          nstl_keep2(p.seed, idx, p.thresh, k0, k1);
          nstl_keep2(p.seed, idx + 2, p.thresh, k2, k3);
          v0 = k0 ? v0 * p.inv_keep : 0.f;
          v1 = k1 ? v1 * p.inv_keep : 0.f;
          v2 = k2 ? v2 * p.inv_keep : 0.f;
          v3 = k3 ? v3 * p.inv_keep : 0.f;
          if (p.mask) {  // the 4 ballots (wave-uniform) into lanes kt*4 .. +3
            const uint64_t b[4] = {__ballot(k0), __ballot(k1), __ballot(k2), __ballot(k3)};
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (lane == kt * 4 + r) {
                mlo = (uint32_t)b[r];
                mhi = (uint32_t)(b[r] >> 32);
              }
          }
        }
        put4(Pw + key * RBP + 4 * g * ESZ, v0, v1, v2, v3, T());
      }
    }
    if (p.thresh && p.mask && lane < nkt * 4)
      p.mask[mask_word(bh, nkt, (qb0 + q0) >> 4, 0, 0) + lane] = ((uint64_t)mhi << 32) | mlo;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nkt / 2; ++ks) {
      Frag fp;
      frag_col<ImgP>(fp, Pw, 0, ks * 32, lane);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        Frag fv;
        frag_col<Img>(fv, Vimg, dt * 16, ks * 32, lane);
        mma16(o[dt], fp, fv);
      }
    }
    // O: stage 16 x 64 through the (now free) P^T image, store 16-byte rows
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    char* Ow = Pw;  // [16 rows][64 d] of T = 64 * RBP bytes
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float inv = 1.f / sum[r];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *(T*)(Ow + (4 * g + r) * RBK + (dt * 16 + (lane & 15)) * ESZ) = from_f32<T>(o[dt][r] * inv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int CPR = RBK / 16;
#pragma unroll
    for (int c = lane; c < 16 * CPR; c += 64) {
      const int row = c / CPR, ch = c % CPR;
      const uint4 val = *(const uint4*)(Ow + row * RBK + ch * 16);
      *(uint4*)(p.o + ((tok0 + qb0 + q0 + row) * p.o_ld + h * DH) * ESZ + ch * 16) = val;
    }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        p.lse[(int64_t)bh * T_ + qb0 + q0 + 4 * g + r] = mx[r] * p.scale + logf(sum[r]);
    }
  }
}

// rotate a (row t, col d) accumulator element back by -theta (RoPE^T)
NSTL_DEV float rope_back(float v, int t, int d, const float* cs, const float* sn) {
  const float partner = __shfl_xor(v, 1);
  const float c = cs[t * (DH / 2) + (d >> 1)], s = sn[t * (DH / 2) + (d >> 1)];
  return (d & 1) ? (v * c - partner * s) : (v * c + partner * s);
}

// A wave's 16 x 64 result tile (lane: rows 4g+r, column dt*16 + (lane&15)) to
// global memory through the wave's LDS scratch: element writes into a dense
// [16][64] image, then 16-byte row chunks (2-byte scattered stores write
// 32-byte pieces of 4 rows per instruction).
template <typename T>
NSTL_DEV void store_tile16x64(const float (&v)[4][4], char* scr, char* gbase, int64_t ld_elems, int lane) {
  constexpr int ESZ = (int)sizeof(T), RB = DH * ESZ, CPR = RB / 16;
  const int g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *(T*)(scr + (4 * g + r) * RB + (dt * 16 + (lane & 15)) * ESZ) = from_f32<T>(v[dt][r]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int row = c / CPR, ch = c % CPR;
    *(uint4*)(gbase + (int64_t)row * ld_elems * ESZ + ch * 16) = *(const uint4*)(scr + row * RB + ch * 16);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Bias gradients fused into the backward stores: column sums of a wave's stored
// 16 x 64 tile (rounded to T, as colsum() of the stored tensor would see it) go
// to red[w][64]; the LAST wave to finish (an LDS arrival counter, no barrier,
// so early waves leave at once) adds the block's waves in fixed order and
// writes one partial row: deterministic, no float atomics.
template <typename T>
NSTL_DEV void wave_colsum16x64(const float (&v)[4][4], float* red, int w, int lane) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float c = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) c += to_f32(from_f32<T>(v[dt][r]));
    c += __shfl_xor(c, 16);
    c += __shfl_xor(c, 32);
    if (lane < 16) red[w * 64 + dt * 16 + lane] = c;
  }
}
NSTL_DEV bool last_to_arrive(unsigned* cnt, int nw, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's red[] writes are done
  unsigned old = 0;
  if (lane == 0) old = atomicAdd(cnt, 1u);
  return __shfl(old, 0) == (unsigned)(nw - 1);
}
NSTL_DEV void wave_sum_out(const float* red, int nw, float* out, int lane) {
  float c = 0.f;
  for (int k = 0; k < nw; ++k) c += red[k * 64 + lane];
  out[lane] = c;
}

// ---------------------------------------------------------------------------
// Backward, as two kernels (8 waves, 128 rows: all of T=128, so each (b, h)
// operand is staged once) with ~48 KB LDS, 3 resident per CU:
//   attn_bwd_dq : workgroup = (b, h, 128 queries); K, V of (b, h) in LDS; a wave
//                 owns 16 queries: D = rowsum(dO * O) (also written to p.dsum
//                 for the second kernel), dS over all keys, dQ = dS K (RoPE^T).
//   attn_bwd_dkv: workgroup = (b, h, 128 keys); Q, dO of (b, h) in LDS; a wave
//                 owns 16 keys: dV = P_drop^T dO, dK = dS^T Q (RoPE^T).
// A wave's own rows come straight from global memory into MFMA fragments.
constexpr int BWD_NT = 512, BWD_ROWS = 16 * BWD_NT / 64;  // 8 waves, 128 rows

template <typename T>
NSTL_DEV void gload_frag(typename FragT<T>::type& f, const T* row, int k0);
template <>
NSTL_DEV void gload_frag<bf16>(bf16x8& f, const bf16* row, int k0) {
  f = *(const bf16x8*)(row + k0);
}
template <>
NSTL_DEV void gload_frag<float>(f32x8& f, const float* row, int k0) {
  const f32x4 lo = *(const f32x4*)(row + k0), hi = *(const f32x4*)(row + k0 + 4);
  f = (f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <typename T>
__global__ __launch_bounds__(BWD_NT) void attn_bwd_dq_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;
  typedef ImgK<RBK> Img;
  constexpr int RBS = 16 * ESZ;
  typedef ImgPlain<RBS> ImgS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Kimg = smem;
  char* Vimg = Kimg + T_ * RBK;
  char* scratch = Vimg + T_ * RBK;

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;
  const int q0 = blockIdx.x * BWD_ROWS + w * 16;
  dma_rows<RBK, BWD_NT / 64>(Kimg, p.k + (tok0 * p.k_ld + h * DH) * ESZ, p.k_ld * ESZ, T_, w, lane);
  dma_rows<RBK, BWD_NT / 64>(Vimg, p.v + (tok0 * p.v_ld + h * DH) * ESZ, p.v_ld * ESZ, T_, w, lane);
  const bool act = q0 < T_;
  Frag fq[2], fo[2];
  float lq[4], dqv[4];
  if (act) {
    const int qr = q0 + (lane & 15);
    const T* qrow = (const T*)p.q + (tok0 + qr) * p.q_ld + h * DH;
    const T* drow = (const T*)p.dout + (tok0 + qr) * p.dout_ld + h * DH;
    const T* orow = (const T*)p.o + (tok0 + qr) * p.o_ld + h * DH;
    Frag oo[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gload_frag<T>(fq[u], qrow, 32 * u + 8 * g);
      gload_frag<T>(fo[u], drow, 32 * u + 8 * g);
      gload_frag<T>(oo[u], orow, 32 * u + 8 * g);
    }
    // D for row (lane & 15): 16 of its products per lane, then across the 4 groups
    float dpart = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) dpart += to_f32(fo[u][e]) * to_f32(oo[u][e]);
    dpart += __shfl_xor(dpart, 16);
    dpart += __shfl_xor(dpart, 32);
    if (g == 0) p.dsum[(int64_t)bh * T_ + qr] = dpart;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dqv[r] = __shfl(dpart, 4 * g + r);
      lq[r] = p.lse[(int64_t)bh * T_ + q0 + 4 * g + r] * LOG2E;
    }
  }
  float* red = (float*)(scratch + (BWD_NT / 64) * 2 * 32 * RBS);  // [8 waves][64] bias partials
  unsigned* arrived = (unsigned*)(red + 2 * (BWD_NT / 64) * 64);
  if (tid == 0) *arrived = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* bias_row = p.dbias ? p.dbias + (int64_t)(b * gridDim.x + blockIdx.x) * 3 * p.H * DH : nullptr;
  if (!act) {
    if (bias_row) {
      red[w * 64 + lane] = 0.f;
      if (last_to_arrive(arrived, BWD_NT / 64, lane)) wave_sum_out(red, BWD_NT / 64, bias_row + h * DH, lane);
    }
    return;
  }

  const float c2 = p.scale * LOG2E;
  char* S2 = scratch + w * 2 * 32 * RBS;
  // stored keep bits of this wave's 16 queries: lane kt*4 + r holds word (kt, r)
  const bool use_mask = p.thresh && p.mask;
  uint64_t mword = 0;
  if (use_mask && lane < nkt * 4) mword = p.mask[mask_word(bh, nkt, q0 >> 4, 0, 0) + lane];
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < nkt / 2; ++kc) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kt = kc * 2 + u;
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      Frag fb;
      frag_row<Img>(fb, Kimg, kt * 16 + (lane & 15), 8 * g);
      mma16(s, fq[0], fb);
      frag_row<Img>(fb, Kimg, kt * 16 + (lane & 15), 32 + 8 * g);
      mma16(s, fq[1], fb);
      frag_row<Img>(fb, Vimg, kt * 16 + (lane & 15), 8 * g);
      mma16(dp, fo[0], fb);
      frag_row<Img>(fb, Vimg, kt * 16 + (lane & 15), 32 + 8 * g);
      mma16(dp, fo[1], fb);
      // accumulator: row = query (4g + r), col = key
      const int key = kt * 16 + (lane & 15);
      bool keep[4] = {true, true, true, true};
      if (use_mask) {
#pragma unroll
        for (int r = 0; r < 4; ++r) keep[r] = (readlane64(mword, kt * 4 + r) >> lane) & 1;
      } else if (p.thresh) {
        const uint64_t idx = drop_idx(bh, T_, q0 + 4 * g, key);
        nstl_keep2(p.seed, idx, p.thresh, keep[0], keep[1]);
        nstl_keep2(p.seed, idx + 2, p.thresh, keep[2], keep[3]);
      }
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = exp2f(s[r] * c2 - lq[r]);
        float dpd = dp[r];
        if (p.thresh) dpd = keep[r] ? dpd * p.inv_keep : 0.f;
        ds[r] = pv * (dpd - dqv[r]);
      }
      // transposed image [key][query]
      put4(S2 + (u * 16 + (lane & 15)) * RBS + 4 * g * ESZ, ds[0], ds[1], ds[2], ds[3], T());
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    Frag fa;
    frag_col<ImgS>(fa, S2, 0, 0, lane);  // A(i = query, r = key)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      Frag fb;
      frag_col<Img>(fb, Kimg, dt * 16, kc * 32, lane);
      mma16(dq[dt], fa, fb);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  float vq[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + 4 * g + r;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = dt * 16 + (lane & 15);
      float x = dq[dt][r] * p.scale;
      if (p.rope_q) x = rope_back(x, q, d, p.rope_cos, p.rope_sin);
      vq[dt][r] = x;
    }
  }
  store_tile16x64<T>(vq, S2, p.dq + ((tok0 + q0) * p.dq_ld + h * DH) * ESZ, p.dq_ld, lane);
  if (bias_row) {
    wave_colsum16x64<T>(vq, red, w, lane);
    if (last_to_arrive(arrived, BWD_NT / 64, lane)) wave_sum_out(red, BWD_NT / 64, bias_row + h * DH, lane);
  }
}

template <typename T>
__global__ __launch_bounds__(BWD_NT) void attn_bwd_dkv_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;
  typedef ImgK<RBK> Img;
  constexpr int RBS = 16 * ESZ;
  typedef ImgPlain<RBS> ImgS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Qimg = smem;
  char* Dimg = Qimg + T_ * RBK;
  float* lse_s = (float*)(Dimg + T_ * RBK);
  float* dq_s = lse_s + T_;
  char* scratch = (char*)(dq_s + T_);

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;
  const int k0 = blockIdx.x * BWD_ROWS + w * 16;
  dma_rows<RBK, BWD_NT / 64>(Qimg, p.q + (tok0 * p.q_ld + h * DH) * ESZ, p.q_ld * ESZ, T_, w, lane);
  dma_rows<RBK, BWD_NT / 64>(Dimg, p.dout + (tok0 * p.dout_ld + h * DH) * ESZ, p.dout_ld * ESZ, T_, w, lane);
  for (int i = tid; i < T_; i += BWD_NT) {
    lse_s[i] = p.lse[(int64_t)bh * T_ + i] * LOG2E;
    dq_s[i] = p.dsum[(int64_t)bh * T_ + i];
  }
  const bool act = k0 < T_;
  Frag fk[2], fv[2];
  if (act) {
    const int kr = k0 + (lane & 15);
    const T* krow = (const T*)p.k + (tok0 + kr) * p.k_ld + h * DH;
    const T* vrow = (const T*)p.v + (tok0 + kr) * p.v_ld + h * DH;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gload_frag<T>(fk[u], krow, 32 * u + 8 * g);
      gload_frag<T>(fv[u], vrow, 32 * u + 8 * g);
    }
  }
  float* red = (float*)(scratch + (BWD_NT / 64) * 2 * 32 * RBS);  // [2][8 waves][64] bias partials
  unsigned* arrived = (unsigned*)(red + 2 * (BWD_NT / 64) * 64);
  if (tid == 0) *arrived = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int NWB = BWD_NT / 64;
  float* bias_row = p.dbias ? p.dbias + (int64_t)(b * gridDim.x + blockIdx.x) * 3 * p.H * DH : nullptr;
  if (!act) {
    if (bias_row) {
      red[w * 64 + lane] = 0.f;
      red[NWB * 64 + w * 64 + lane] = 0.f;
      if (last_to_arrive(arrived, NWB, lane)) {
        wave_sum_out(red, NWB, bias_row + p.H * DH + h * DH, lane);
        wave_sum_out(red + NWB * 64, NWB, bias_row + 2 * p.H * DH + h * DH, lane);
      }
    }
    return;
  }

  const float c2 = p.scale * LOG2E;
  char* S1 = scratch + w * 2 * 32 * RBS;  // [32 rows][16] images
  // stored keep bits for this wave's 16 keys: lane 4*qt + r holds word (qt, k0/16, r)
  const bool use_mask = p.thresh && p.mask;
  uint64_t mword = 0;
  if (use_mask && (lane >> 2) < nkt) mword = p.mask[mask_word(bh, nkt, lane >> 2, k0 >> 4, lane & 3)];
  char* S2 = S1 + 32 * RBS;
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int qc = 0; qc < nkt / 2; ++qc) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qt = qc * 2 + u;
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
      Frag fb;
      frag_row<Img>(fb, Qimg, qt * 16 + (lane & 15), 8 * g);
      mma16(st, fk[0], fb);
      frag_row<Img>(fb, Qimg, qt * 16 + (lane & 15), 32 + 8 * g);
      mma16(st, fk[1], fb);
      frag_row<Img>(fb, Dimg, qt * 16 + (lane & 15), 8 * g);
      mma16(dpt, fv[0], fb);
      frag_row<Img>(fb, Dimg, qt * 16 + (lane & 15), 32 + 8 * g);
      mma16(dpt, fv[1], fb);
      // accumulator: row = key (4g + r), col = query
      const int q = qt * 16 + (lane & 15);
      const float lq = lse_s[q], dqv = dq_s[q];
      // query q's bits for keys k0 + 4g .. +3: 4 consecutive bits of word (qt, q % 4)
      uint32_t nib = 0;
      if (use_mask) nib = (uint32_t)(shfl64(mword, 4 * qt + (lane & 3)) >> (16 * ((lane & 15) >> 2) + 4 * g));
      float pd[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 4 * g + r;
        const float pv = exp2f(st[r] * c2 - lq);
        float pdr = pv, dpd = dpt[r];
        if (p.thresh) {
          const bool keep = use_mask ? ((nib >> r) & 1) : nstl_keep(p.seed, drop_idx(bh, T_, q, key), p.thresh);
          pdr = keep ? pv * p.inv_keep : 0.f;
          dpd = keep ? dpd * p.inv_keep : 0.f;
        }
        pd[r] = pdr;
        ds[r] = pv * (dpd - dqv);
      }
      // transposed images [query][key]: this lane's 4 keys are contiguous
      const int qr = u * 16 + (lane & 15);
      put4(S1 + qr * RBS + 4 * g * ESZ, pd[0], pd[1], pd[2], pd[3], T());
      put4(S2 + qr * RBS + 4 * g * ESZ, ds[0], ds[1], ds[2], ds[3], T());
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    Frag fa1, fa2;
    frag_col<ImgS>(fa1, S1, 0, 0, lane);  // A(i = key, r = query)
    frag_col<ImgS>(fa2, S2, 0, 0, lane);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      Frag fb;
      frag_col<Img>(fb, Dimg, dt * 16, qc * 32, lane);
      mma16(dv[dt], fa1, fb);
      frag_col<Img>(fb, Qimg, dt * 16, qc * 32, lane);
      mma16(dk[dt], fa2, fb);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  float vk[4][4], vv[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + 4 * g + r;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = dt * 16 + (lane & 15);
      float x = dk[dt][r] * p.scale;
      if (p.rope_k) x = rope_back(x, key, d, p.rope_cos, p.rope_sin);
      vk[dt][r] = x;
      vv[dt][r] = dv[dt][r];
    }
  }
  store_tile16x64<T>(vk, S1, p.dk + ((tok0 + k0) * p.dk_ld + h * DH) * ESZ, p.dk_ld, lane);
  store_tile16x64<T>(vv, S1, p.dv + ((tok0 + k0) * p.dv_ld + h * DH) * ESZ, p.dv_ld, lane);
  if (bias_row) {
    wave_colsum16x64<T>(vk, red, w, lane);
    wave_colsum16x64<T>(vv, red + NWB * 64, w, lane);
    if (last_to_arrive(arrived, NWB, lane)) {
      wave_sum_out(red, NWB, bias_row + p.H * DH + h * DH, lane);
      wave_sum_out(red + NWB * 64, NWB, bias_row + 2 * p.H * DH + h * DH, lane);
    }
  }
}

size_t fwd_lds_bytes(int T, int esz) {
  return (size_t)(2 * T + FWD_QB) * DH * esz + (FWD_NT / 64) * (size_t)std::max(T, 64) * 16 * esz;
}
size_t bwd_lds_bytes(int T, int esz) {  // either backward kernel (+ 2 x [8][64] f32 bias partials + counter)
  return (size_t)2 * T * DH * esz + 2 * T * 4 + (BWD_NT / 64) * 2 * 32 * 16 * (size_t)esz +
         2 * (BWD_NT / 64) * 64 * 4 + 16;
}

// ---------------------------------------------------------------------------
// Generic path: any even head_dim that is a multiple of 8 (<= 512) and any T
// (<= 4096).  One wave per query row (forward, dq) or per key row (dk, dv);
// the wave's own row is staged in LDS as f32, the other operand's rows stream
// from global memory (L2-resident per (b, h)), softmax rows live in LDS.  It
// serves the shapes the MFMA kernels above do not (e.g. BASELINE C1: 4 heads
// of 256) with the same dropout stream (drop_idx / nstl_keep), scale, LSE and
// RoPE^T conventions, so the two paths are interchangeable.
// ---------------------------------------------------------------------------
constexpr int G_MAX_DH = 512, G_MAX_T = 4096;

NSTL_DEV void load8(const bf16* g, float* v) {
  const bf16x8 x = *(const bf16x8*)g;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = (float)x[k];
}
NSTL_DEV void load8(const float* g, float* v) {
  const f32x4 a = *(const f32x4*)g, b = *(const f32x4*)(g + 4);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = a[k];
    v[4 + k] = b[k];
  }
}

// dot(global row g[0..dh), LDS f32 row s[0..dh))
template <typename T>
NSTL_DEV float dot_gs(const T* g, const float* s, int dh) {
  float acc = 0.f;
  for (int d = 0; d < dh; d += 8) {
    float v[8];
    load8(g + d, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = fmaf(v[k], s[d + k], acc);
  }
  return acc;
}

template <typename T>
NSTL_DEV float dot_gg(const T* a, const T* b, int dh) {
  float acc = 0.f;
  for (int d = 0; d < dh; d += 8) {
    float x[8], y[8];
    load8(a + d, x);
    load8(b + d, y);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = fmaf(x[k], y[k], acc);
  }
  return acc;
}

template <typename T>
NSTL_DEV const T* row_ptr(const char* base, int64_t ld, int64_t tok, int h, int dh) {
  return (const T*)base + tok * ld + (int64_t)h * dh;
}

// RoPE^T on a row held as (d = i*64 + lane): the pair partner is lane ^ 1
NSTL_DEV float rope_back_g(float v, int t, int d, int dh, const float* cs, const float* sn) {
  const float partner = __shfl_xor(v, 1);
  if (d >= dh) return v;
  const float c = cs[t * (dh / 2) + (d >> 1)], s = sn[t * (dh / 2) + (d >> 1)];
  return (d & 1) ? (v * c - partner * s) : (v * c + partner * s);
}

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_generic(AttnParams p) {
  extern __shared__ float gsm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int T_ = p.T, dh = p.dh, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int q = blockIdx.x * 4 + w;
  const bool act = q < T_;
  float* qs = gsm + w * (dh + T_);
  float* sc = qs + dh;
  const int64_t tok0 = (int64_t)b * T_;
  if (act) {
    const T* qr = row_ptr<T>(p.q, p.q_ld, tok0 + q, h, dh);
    for (int d = lane; d < dh; d += 64) qs[d] = to_f32(qr[d]);
  }
  __syncthreads();
  if (act) {
    float mx = -INFINITY;
    for (int j = lane; j < T_; j += 64) {
      const float sv = dot_gs(row_ptr<T>(p.k, p.k_ld, tok0 + j, h, dh), qs, dh) * p.scale;
      sc[j] = sv;
      mx = fmaxf(mx, sv);
    }
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < T_; j += 64) sum += expf(sc[j] - mx);
    sum = wave_sum(sum);
    const float lse = mx + logf(sum);
    for (int j = lane; j < T_; j += 64) {
      float pv = expf(sc[j] - lse);
      if (p.thresh) pv = nstl_keep(p.seed, drop_idx(bh, T_, q, j), p.thresh) ? pv * p.inv_keep : 0.f;
      sc[j] = pv;
    }
    if (lane == 0) p.lse[(int64_t)bh * T_ + q] = lse;
  }
  __syncthreads();
  if (act) {
    for (int d = lane; d < dh; d += 64) {
      float acc = 0.f;
      for (int j = 0; j < T_; ++j) acc = fmaf(sc[j], to_f32(row_ptr<T>(p.v, p.v_ld, tok0 + j, h, dh)[d]), acc);
      store_elem<T>(p.o, (tok0 + q) * p.o_ld + (int64_t)h * dh + d, acc);
    }
  }
}

// dq (one wave per query row)
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_dq_generic(AttnParams p) {
  extern __shared__ float gsm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int T_ = p.T, dh = p.dh, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int q = blockIdx.x * 4 + w;
  const bool act = q < T_;
  float* qs = gsm + w * (2 * dh + T_);
  float* dos = qs + dh;
  float* sc = dos + dh;
  const int64_t tok0 = (int64_t)b * T_;
  float Dq = 0.f;
  if (act) {
    const T* qr = row_ptr<T>(p.q, p.q_ld, tok0 + q, h, dh);
    const T* dr = row_ptr<T>(p.dout, p.dout_ld, tok0 + q, h, dh);
    const T* orow = row_ptr<T>(p.o, p.o_ld, tok0 + q, h, dh);
    for (int d = lane; d < dh; d += 64) {
      qs[d] = to_f32(qr[d]);
      const float g = to_f32(dr[d]);
      dos[d] = g;
      Dq = fmaf(g, to_f32(orow[d]), Dq);
    }
    Dq = wave_sum(Dq);
  }
  __syncthreads();
  if (act) {
    const float lse = p.lse[(int64_t)bh * T_ + q];
    for (int j = lane; j < T_; j += 64) {
      const float pv = expf(dot_gs(row_ptr<T>(p.k, p.k_ld, tok0 + j, h, dh), qs, dh) * p.scale - lse);
      float dp = dot_gs(row_ptr<T>(p.v, p.v_ld, tok0 + j, h, dh), dos, dh);
      if (p.thresh) dp = nstl_keep(p.seed, drop_idx(bh, T_, q, j), p.thresh) ? dp * p.inv_keep : 0.f;
      sc[j] = pv * (dp - Dq);
    }
  }
  __syncthreads();
  if (act) {
    for (int d0 = 0; d0 < dh; d0 += 64) {
      const int d = d0 + lane;
      float acc = 0.f;
      if (d < dh)
        for (int j = 0; j < T_; ++j) acc = fmaf(sc[j], to_f32(row_ptr<T>(p.k, p.k_ld, tok0 + j, h, dh)[d]), acc);
      float v = acc * p.scale;
      if (p.rope_q) v = rope_back_g(v, q, d, dh, p.rope_cos, p.rope_sin);
      if (d < dh) store_elem<T>(p.dq, (tok0 + q) * p.dq_ld + (int64_t)h * dh + d, v);
    }
  }
}

// dk, dv (one wave per key row)
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_dkv_generic(AttnParams p) {
  extern __shared__ float gsm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int T_ = p.T, dh = p.dh, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int j = blockIdx.x * 4 + w;
  const bool act = j < T_;
  float* ks = gsm + w * (2 * dh + 2 * T_);
  float* vs = ks + dh;
  float* pd = vs + dh;
  float* ds = pd + T_;
  const int64_t tok0 = (int64_t)b * T_;
  if (act) {
    const T* kr = row_ptr<T>(p.k, p.k_ld, tok0 + j, h, dh);
    const T* vr = row_ptr<T>(p.v, p.v_ld, tok0 + j, h, dh);
    for (int d = lane; d < dh; d += 64) {
      ks[d] = to_f32(kr[d]);
      vs[d] = to_f32(vr[d]);
    }
  }
  __syncthreads();
  if (act) {
    for (int i = lane; i < T_; i += 64) {
      const T* dr = row_ptr<T>(p.dout, p.dout_ld, tok0 + i, h, dh);
      const float pv = expf(dot_gs(row_ptr<T>(p.q, p.q_ld, tok0 + i, h, dh), ks, dh) * p.scale -
                            p.lse[(int64_t)bh * T_ + i]);
      float dp = dot_gs(dr, vs, dh);
      const float Di = dot_gg(dr, row_ptr<T>(p.o, p.o_ld, tok0 + i, h, dh), dh);
      float pdv = pv;
      if (p.thresh) {
        const bool keep = nstl_keep(p.seed, drop_idx(bh, T_, i, j), p.thresh);
        pdv = keep ? pv * p.inv_keep : 0.f;
        dp = keep ? dp * p.inv_keep : 0.f;
      }
      pd[i] = pdv;
      ds[i] = pv * (dp - Di);
    }
  }
  __syncthreads();
  if (act) {
    for (int d0 = 0; d0 < dh; d0 += 64) {
      const int d = d0 + lane;
      float av = 0.f, ak = 0.f;
      if (d < dh)
        for (int i = 0; i < T_; ++i) {
          av = fmaf(pd[i], to_f32(row_ptr<T>(p.dout, p.dout_ld, tok0 + i, h, dh)[d]), av);
          ak = fmaf(ds[i], to_f32(row_ptr<T>(p.q, p.q_ld, tok0 + i, h, dh)[d]), ak);
        }
      float vk = ak * p.scale;
      if (p.rope_k) vk = rope_back_g(vk, j, d, dh, p.rope_cos, p.rope_sin);
      if (d < dh) {
        store_elem<T>(p.dk, (tok0 + j) * p.dk_ld + (int64_t)h * dh + d, vk);
        store_elem<T>(p.dv, (tok0 + j) * p.dv_ld + (int64_t)h * dh + d, av);
      }
    }
  }
}

bool use_fast(const nstl_attn_args* a) {
  return a->dh == DH && a->T % 32 == 0 && a->T <= (a->dtype == NSTL_BF16 ? 256 : 128);
}

int fill(AttnParams& p, const nstl_attn_args* a, bool bwd) {
  NSTL_CHECK_ARG(a != nullptr, "nstl_attn: null args");
  NSTL_CHECK_ARG(a->dtype == NSTL_F32 || a->dtype == NSTL_BF16, "nstl_attn: bad dtype");
  NSTL_CHECK_ARG(a->dh > 0 && a->dh % 8 == 0 && a->dh <= G_MAX_DH,
                 "nstl_attn: head_dim must be a multiple of 8 up to %d (got %d)", G_MAX_DH, a->dh);
  NSTL_CHECK_ARG(a->T > 0 && a->T <= G_MAX_T, "nstl_attn: T must be in [1, %d] (got %d)", G_MAX_T, a->T);
  NSTL_CHECK_ARG(a->B > 0 && a->H > 0, "nstl_attn: empty batch");
  NSTL_CHECK_ARG(a->q && a->k && a->v && a->o && a->lse, "nstl_attn: null tensor");
  const int vec = a->dtype == NSTL_F32 ? 4 : 8;
  NSTL_CHECK_ARG(a->q_ld % vec == 0 && a->k_ld % vec == 0 && a->v_ld % vec == 0 && a->o_ld % vec == 0,
                 "nstl_attn: ld alignment");
  NSTL_CHECK_ARG(((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v | (uintptr_t)a->o) % 16 == 0,
                 "nstl_attn: tensors must be 16-byte aligned");
  NSTL_CHECK_ARG(a->p_drop >= 0.f && a->p_drop < 1.f, "nstl_attn: p_drop out of range");
  if (bwd) {
    NSTL_CHECK_ARG(a->dout && a->dq && a->dk && a->dv, "nstl_attn_bwd: null gradient tensor");
    NSTL_CHECK_ARG(a->dout_ld % vec == 0 && (uintptr_t)a->dout % 16 == 0, "nstl_attn_bwd: dout alignment");
    NSTL_CHECK_ARG(a->dq_ld % vec == 0 && a->dk_ld % vec == 0 && a->dv_ld % vec == 0 &&
                       ((uintptr_t)a->dq | (uintptr_t)a->dk | (uintptr_t)a->dv) % 16 == 0,
                   "nstl_attn_bwd: dq/dk/dv must be 16-byte aligned");
    NSTL_CHECK_ARG(!(a->rope_q || a->rope_k) || (a->rope_cos && a->rope_sin), "nstl_attn_bwd: rope tables");
    NSTL_CHECK_ARG(!use_fast(a) || a->dsum, "nstl_attn_bwd: dsum scratch [B*H*T] f32 missing");
    NSTL_CHECK_ARG(!a->dbias_part || use_fast(a), "nstl_attn_bwd: dbias_part needs the MFMA path (head_dim 64)");
  }
  p.q = (const char*)a->q; p.q_ld = a->q_ld;
  p.k = (const char*)a->k; p.k_ld = a->k_ld;
  p.v = (const char*)a->v; p.v_ld = a->v_ld;
  p.o = (char*)a->o; p.o_ld = a->o_ld;
  p.lse = a->lse;
  p.dsum = a->dsum;
  p.mask = a->mask_bits;
  p.dbias = a->dbias_part;
  p.dout = (const char*)a->dout; p.dout_ld = a->dout_ld;
  p.dq = (char*)a->dq; p.dq_ld = a->dq_ld;
  p.dk = (char*)a->dk; p.dk_ld = a->dk_ld;
  p.dv = (char*)a->dv; p.dv_ld = a->dv_ld;
  p.rope_cos = a->rope_cos; p.rope_sin = a->rope_sin;
  p.rope_q = a->rope_q; p.rope_k = a->rope_k;
  p.B = a->B; p.T = a->T; p.H = a->H; p.dh = a->dh;
  p.scale = 1.0f / sqrtf((float)a->dh);
  p.thresh = nstl_drop_thresh(a->p_drop);
  p.inv_keep = 1.0f / (1.0f - a->p_drop);
  p.seed = a->seed;
  return 0;
}

template <typename K>
int launch(K kern, dim3 grid, size_t lds, hipStream_t st, const AttnParams& p, const char* what, int nt = NT) {
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return nstl::fail((int)e, "%s: LDS request %zu: %s", what, lds, hipGetErrorString(e));
  hipLaunchKernelGGL(kern, grid, dim3(nt), lds, st, p);
  NSTL_LAUNCH_CHECK(what);
  return 0;
}

}  // namespace

extern "C" int nstl_attn_fwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, false);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  hipStream_t st = (hipStream_t)stream;
  if (!use_fast(a)) {
    dim3 grid((a->T + 3) / 4, a->B * a->H);
    const size_t lds = 4 * (size_t)(a->dh + a->T) * 4;
    if (a->dtype == NSTL_BF16) return launch(attn_fwd_generic<bf16>, grid, lds, st, p, "nstl_attn_fwd generic");
    return launch(attn_fwd_generic<float>, grid, lds, st, p, "nstl_attn_fwd generic");
  }
  dim3 grid((a->T + FWD_QB - 1) / FWD_QB, a->B * a->H);
  const size_t lds = fwd_lds_bytes(a->T, esz);
  if (a->dtype == NSTL_BF16) return launch(attn_fwd_kernel<bf16>, grid, lds, st, p, "nstl_attn_fwd", FWD_NT);
  return launch(attn_fwd_kernel<float>, grid, lds, st, p, "nstl_attn_fwd", FWD_NT);
}

extern "C" int nstl_attn_bwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, true);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  hipStream_t st = (hipStream_t)stream;
  if (!use_fast(a)) {
    dim3 grid((a->T + 3) / 4, a->B * a->H);
    const size_t lq = 4 * (size_t)(2 * a->dh + a->T) * 4, lkv = 4 * (size_t)(2 * a->dh + 2 * a->T) * 4;
    if (a->dtype == NSTL_BF16) {
      if ((rc = launch(attn_bwd_dq_generic<bf16>, grid, lq, st, p, "nstl_attn_bwd generic dq"))) return rc;
      return launch(attn_bwd_dkv_generic<bf16>, grid, lkv, st, p, "nstl_attn_bwd generic dkv");
    }
    if ((rc = launch(attn_bwd_dq_generic<float>, grid, lq, st, p, "nstl_attn_bwd generic dq"))) return rc;
    return launch(attn_bwd_dkv_generic<float>, grid, lkv, st, p, "nstl_attn_bwd generic dkv");
  }
  dim3 grid((a->T + BWD_ROWS - 1) / BWD_ROWS, a->B * a->H);
  const size_t lds = bwd_lds_bytes(a->T, esz);
  if (a->dtype == NSTL_BF16) {
    if ((rc = launch(attn_bwd_dq_kernel<bf16>, grid, lds, st, p, "nstl_attn_bwd dq", BWD_NT))) return rc;
    return launch(attn_bwd_dkv_kernel<bf16>, grid, lds, st, p, "nstl_attn_bwd dkv", BWD_NT);
  }
  if ((rc = launch(attn_bwd_dq_kernel<float>, grid, lds, st, p, "nstl_attn_bwd dq", BWD_NT))) return rc;
  return launch(attn_bwd_dkv_kernel<float>, grid, lds, st, p, "nstl_attn_bwd dkv", BWD_NT);
}

extern "C" int nstl_attn_bias_rows(const nstl_attn_args* a) {
  if (a == nullptr || !use_fast(a)) return 0;
  return a->B * ((a->T + BWD_ROWS - 1) / BWD_ROWS);
}
