// MFMA GEMM for gfx950: C[i,j] = alpha * sum_r A(i,r) B(j,r) (+beta*C) + epilogue.
//
// One kernel template covers the three products of nn.Linear training
// (utils/model.py Linear layers):
//   forward  Y  = X W^T   A=X [M][K] (K-major), B=W [N][K] (K-major)
//   backward dX = dY W    A=dY [M][N] (K-major), B=W [N][K] read as [r][j] (MN-major)
//   backward dW = dY^T X  A=dY [M][N] read as [r][i], B=X [M][K] read as [r][j]
// K-major tiles are staged into 128-byte-row LDS images and read with
// ds_read_b128; MN-major tiles keep the global layout in LDS and are read with
// the gfx950 transpose read ds_read_b64_tr_b16 (bf16), so no transpose pass.
//
// Tile 128x128, BK = 128 bytes of reduction index (64 bf16 / 32 f32), 4 waves
// (2x2) each owning 64x64 = 4x4 MFMA 16x16 tiles, register-staged double-
// buffered LDS (one barrier per K tile), XCD-aware tile order.
#include <stdlib.h>
#include <string.h>

#include "../../include/nstl.h"
#include <map>
#include <mutex>
#include <type_traits>
#include <string>

#include "common.h"
#include "status.h"

namespace {

constexpr int BM = 128, BN = 128, NTHREADS = 256;
constexpr int TILE_BYTES = 16384;

struct GemmParams {
  const char* A; int64_t lda;
  const char* B; int64_t ldb;
  char* C; int64_t ldc;
  int M, N, K;
  int c_f32;
  float alpha, beta;
  int epi;
  const float* bias;
  const char* aux; int64_t ld_aux; int aux_f32;
  float inv_keep; uint32_t thresh; uint64_t seed;
  const float* rope_cos; const float* rope_sin; int rope_T, rope_dim, rope_cols;
  int rope_fast;  // ring epilogue: cos/sin recomputed from t * inv_freq instead of read from the tables
  float* ws;
  int debug_skip_epilogue; int k_chunk;  // split-K: partial slabs [z][M][N]
  float* colsum_part;  // [ceil(M/128)][N]: column sums of C as stored (dReLU ring epilogue)
  uint64_t* relu_mask;  // ReLU-dropout keep&positive bits, ring epilogue layout (relu_mask_index)
  const float* a_scale; const float* b_scale;  // fp8: row scales of A [M] and of B [N]
  float* sq_part;  // grouped f32 ring epilogue: sum of squares of C as stored, per (tile, wave) [tiles][8]
  int direct_epi;  // EM_BF16 ring epilogue from registers (permlane swaps) on full tiles; 0: LDS staging
};

// Epilogue over a wave's MT x 4 grid of 16x16 accumulators whose origin is
// (row0, col0).  Each 16 x 64 slab goes through the wave's own LDS scratch
// (16 x 68 f32) and comes back as 4 consecutive columns per lane: 16-byte
// (f32) / 8-byte (bf16) stores, RoPE pairs lane-local.  Ops: alpha, split-K
// slab, bias / ReLU+dropout / RoPE / dReLU+dropout, beta*C.
constexpr int EPI_LD = 68;  // floats per scratch row (64 + 4 pad)

// bias / ReLU+dropout / RoPE / dReLU+dropout on four consecutive columns
// j..j+3 of row i (no alpha, beta or store)
NSTL_DEV f32x4 epi_math4(const GemmParams& p, int i, int j, f32x4 v) {
  const int epi = p.epi;
  if (p.bias != nullptr && epi != NSTL_EPI_NONE && epi != NSTL_EPI_DRELU_DROP) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += j + e < p.N ? p.bias[j + e] : 0.f;
  }
  if (epi == NSTL_EPI_BIAS_RELU_DROP) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    if (p.thresh) {
      // (i*N + j) is even when N is even (j is a multiple of 4): two pair hashes
      const uint64_t idx = (uint64_t)i * p.N + j;
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        bool k0, k1;
        if ((idx & 1) == 0) {
          nstl_keep2(p.seed, idx + e, p.thresh, k0, k1);
        } else {
          k0 = nstl_keep(p.seed, idx + e, p.thresh);
          k1 = nstl_keep(p.seed, idx + e + 1, p.thresh);
        }
        v[e] = k0 ? v[e] * p.inv_keep : 0.f;
        v[e + 1] = k1 ? v[e + 1] * p.inv_keep : 0.f;
      }
    }
  } else if (epi == NSTL_EPI_BIAS_ROPE) {
    if (j < p.rope_cols) {
      const int t = i % p.rope_T, half = p.rope_dim >> 1;
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const int pair = ((j + e) % p.rope_dim) >> 1;
        const float c = p.rope_cos[t * half + pair], sn = p.rope_sin[t * half + pair];
        const float x0 = v[e], x1 = v[e + 1];
        v[e] = x0 * c - x1 * sn;
        v[e + 1] = x0 * sn + x1 * c;
      }
    }
  } else if (epi == NSTL_EPI_DRELU_DROP) {
    const int64_t x = (int64_t)i * p.ld_aux + j;
    float av[4];
    if (!p.aux_f32 && j + 3 < p.N && (p.ld_aux & 3) == 0) {
      const bf16x4 a4 = *(const bf16x4*)((const bf16*)p.aux + x);
#pragma unroll
      for (int e = 0; e < 4; ++e) av[e] = (float)a4[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        av[e] = j + e < p.N ? (p.aux_f32 ? ((const float*)p.aux)[x + e] : (float)((const bf16*)p.aux)[x + e]) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = av[e] > 0.f ? v[e] * p.inv_keep : 0.f;
  }
  return v;
}

NSTL_DEV void epi_store4(const GemmParams& p, int i, int j, f32x4 v) {
  if (p.ws != nullptr) {
    float* w = p.ws + ((int64_t)blockIdx.y * p.M + i) * p.N + j;
    if (j + 3 < p.N && (p.N & 3) == 0) {
      *(f32x4*)w = (f32x4){v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (j + e < p.N) w[e] = v[e];
    }
    return;
  }
  v = epi_math4(p, i, j, v);
  const int64_t o = (int64_t)i * p.ldc + j;
  const bool vec = j + 3 < p.N && (p.ldc & 3) == 0 && ((uintptr_t)p.C % (p.c_f32 ? 16 : 8)) == 0;
  if (p.c_f32) {
    float* c = (float*)p.C + o;
    if (vec) {
      if (p.beta != 0.f) {
        const f32x4 old = *(const f32x4*)c;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += p.beta * old[e];
      }
      *(f32x4*)c = (f32x4){v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (j + e < p.N) c[e] = p.beta != 0.f ? v[e] + p.beta * c[e] : v[e];
    }
  } else {
    bf16* c = (bf16*)p.C + o;
    if (vec) {
      if (p.beta != 0.f) {
        const bf16x4 old = *(const bf16x4*)c;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += p.beta * (float)old[e];
      }
      *(bf16x4*)c = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (j + e < p.N) c[e] = (bf16)(p.beta != 0.f ? v[e] + p.beta * (float)c[e] : v[e]);
    }
  }
}

// HALF slabs at a time: an unrolled (statically indexed) copy of the
// accumulators into the wave's scratch, then a runtime loop that never touches
// `acc` (so the big epilogue body is not replicated and acc stays in registers).
template <int MT, int HALF>
NSTL_DEV void gemm_epilogue(const GemmParams& p, f32x4 (&acc)[MT][4], int row0, int col0, int lane, float* scr) {
#pragma unroll
  for (int ph = 0; ph < MT / HALF; ++ph) {
#pragma unroll
    for (int a = 0; a < HALF; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          scr[(a * 16 + 4 * (lane >> 4) + r) * EPI_LD + 16 * b + (lane & 15)] = acc[ph * HALF + a][b][r] * p.alpha;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 1
    for (int pass = 0; pass < HALF * 4; ++pass) {
      const int rr = pass * 4 + (lane >> 4), cc = (lane & 15) * 4;
      const f32x4 x = *(const f32x4*)(scr + rr * EPI_LD + cc);
      const int i = row0 + ph * HALF * 16 + rr;
      if (i < p.M && col0 + cc < p.N) epi_store4(p, i, col0 + cc, x);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <typename T, bool KMAJ, int RB>
struct Stager {
  // 16 KB tile = 1024 chunks of 16 B, 4 per thread.
  static constexpr int EPC = 16 / (int)sizeof(T);  // elements per chunk
  uint4 reg[4];
  int lds_off[4];

  // rows_total: extent of the non-reduction dim (M or N); row0: tile origin in it.
  NSTL_DEV void load(const char* base, int64_t ld, int row0, int rows_total, int k0, int K, int tid) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = s * NTHREADS + tid;
      int gi, gk;
      if (KMAJ) {
        const int row = c >> 3, chunk = c & 7;
        gi = row0 + row;
        gk = k0 + chunk * EPC;
        lds_off[s] = ImgK<128>::off(row, chunk * 16);
      } else {
        constexpr int CPR = RB / 16;
        const int row = c / CPR, chunk = c % CPR;
        gk = k0 + row;
        gi = row0 + chunk * EPC;
        lds_off[s] = ImgMN<RB>::off(row, chunk * 16);
      }
      const bool ok = gi < rows_total && gk < K;
      const int64_t e = KMAJ ? ((int64_t)gi * ld + gk) : ((int64_t)gk * ld + gi);
      if (ok)
        reg[s] = *(const uint4*)(base + e * (int64_t)sizeof(T));
      else
        reg[s] = make_uint4(0, 0, 0, 0);
    }
  }
  NSTL_DEV void store(char* img) {
#pragma unroll
    for (int s = 0; s < 4; ++s) *(uint4*)(img + lds_off[s]) = reg[s];
  }
};

template <typename T, bool AK, bool BKM>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_kernel(GemmParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int BK = 128 / (int)sizeof(T);
  constexpr int MN_RB = 128 * (int)sizeof(T);
  constexpr int A_RB = AK ? 128 : MN_RB;
  constexpr int B_RB = BKM ? 128 : MN_RB;
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nt_m = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int id = xcd_remap(blockIdx.x, nt_m * nt_n);
  const int tm = id / nt_n, tn = id % nt_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = blockIdx.y * p.k_chunk;
  const int kz1 = min(p.K, kz0 + p.k_chunk);
  const int nk = (kz1 - kz0 + BK - 1) / BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  Stager<T, AK, A_RB> sa;
  Stager<T, BKM, B_RB> sb;
  if (nk > 0) {
    sa.load(p.A, p.lda, m0, p.M, kz0, kz1, tid);
    sb.load(p.B, p.ldb, n0, p.N, kz0, kz1, tid);
    sa.store(smem[0][0]);
    sb.store(smem[0][1]);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k1 = kz0 + (kt + 1) * BK;
      sa.load(p.A, p.lda, m0, p.M, k1, kz1, tid);
      sb.load(p.B, p.ldb, n0, p.N, k1, kz1, tid);
    }
    const char* Ai = smem[cur][0];
    const char* Bi = smem[cur][1];
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      Frag fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (AK)
          frag_row<ImgK<128>>(fa[t], Ai, wm * 64 + t * 16 + (lane & 15), kk * 32 + 8 * (lane >> 4));
        else
          frag_col<ImgMN<A_RB>>(fa[t], Ai, wm * 64 + t * 16, kk * 32, lane);
        if (BKM)
          frag_row<ImgK<128>>(fb[t], Bi, wn * 64 + t * 16 + (lane & 15), kk * 32 + 8 * (lane >> 4));
        else
          frag_col<ImgMN<B_RB>>(fb[t], Bi, wn * 64 + t * 16, kk * 32, lane);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) mma16(acc[a][b], fa[a], fb[b]);
    }
    if (more) {
      sa.store(smem[cur ^ 1][0]);
      sb.store(smem[cur ^ 1][1]);
    }
    __syncthreads();
  }

  // the K loop ended on a barrier: the staging buffers are free for the epilogue
  gemm_epilogue<4, 2>(p, acc, m0 + wm * 64, n0 + wn * 64, lane, (float*)&smem[0][0][0] + wave * 32 * EPI_LD);
}


// 256x256 tiles (the ring kernels below).  A 128^2 tile moves (128+128)*2 B per
// 2*128^2 FLOP = 64 FLOP/B through L2, which at the MFMA rate needs ~39 TB/s (>
// the ~34.5 TB/s aggregate L2); 256^2 halves that.  The LDS-DMA writes LDS
// lane-linearly (1 KB per wave instruction), so the bank swizzle is applied to
// the per-lane SOURCE address and undone by the same read mapping.
constexpr int BIG = 256, BIG_NT = 512;

// ===========================================================================
// 256x256 tile, 8 waves (2 x 4, each 128 x 64), BK = 32, a ring of FIVE 32 KB
// LDS-DMA stages (160 KB), two wave groups staggered by one barrier.
//
// Step s of a wave = R(s) | barrier | M(s) | barrier, where
//   R(s): ds_read its 12 fragments of tile s, stage tile s+3 (LDS-DMA);
//   M(s): s_waitcnt lgkmcnt(0), 32 MFMAs.
// Waves 4-7 (wm = 1) take one extra barrier up front, so on every SIMD one wave
// runs M while its partner (wm = 0 <-> 1, same SIMD) runs R: the matrix pipe
// alternates between the two waves instead of draining at every barrier.
// With barriers numbered B(k): group 0 runs R0(s) B(2s) M0(s) B(2s+1), group 1
// runs R1(s) B(2s+1) M1(s) B(2s+2).
//   RAW: tile T is read after B(2T-1) (group 0) / B(2T) (group 1); every wave
//        retires its share of tile T before it reaches B(2T-1): group 0 at the
//        end of M0(T-1), group 1 at the end of R1(T-1) -> vmcnt(8) (tiles T+1,
//        T+2 may still fly).
//   WAR: tile T overwrites the slot of tile T-5, whose last reads retire before
//        B(2T-8); tile T is staged in R(T-3), after B(2T-7) / B(2T-6).
constexpr int R_BK = 32, R_SLOT = 32768, R_STAGES = 5;

// Bank swizzle of the K-major 64-byte-row images.  A fragment read
// (ds_read_b128, lane l: row l & 15, chunk l >> 4) is served in lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} (+ the same at chunk + 2 for lanes
// 32-63, MI355X_MICROARCH.md "LDS"); the identity image puts rows r and r + 12 /
// r + 4 and r + 8 of a group on one 16-byte bank slot (2-way, measured:
// SQ_LDS_BANK_CONFLICT ~3.7 extra cycles per LDS instruction).  XOR-ing the
// chunk with 2 ((r >> 2) & 1) gives all 16 lanes of a group distinct slots.
NSTL_DEV int kswz(int row) { return ((row >> 2) & 1) << 1; }

// Per-lane LDS-DMA sources of one operand's 16 KB stage (2 wave-instructions
// per wave), computed once per tile: a K-step then only adds a wave-uniform
// byte offset (k0 * 2 for K-major rows, k0 * ld * 2 for MN-major rows), so the
// staging issue in the R phase is one 64-bit add per instruction instead of the
// index arithmetic (and, in the grouped kernel, the reload of the problem's
// parameters from the kernel-argument memory) it used to redo every K-step.
template <bool KMAJ>
NSTL_DEV void glds_src32(const char* (&src)[2], const char* base, int64_t ld, int row0, int rows_total, int wave,
                         int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int q = wave * 2 + s;
    if (KMAJ) {  // 64-byte rows (32 k), 16 rows per KB, chunk c of row r at c ^ kswz(r)
      const int row = 16 * q + (lane >> 2), ch = (lane & 3) ^ kswz(row);
      const int gi = min(row0 + row, rows_total - 1);
      src[s] = base + ((int64_t)gi * ld + ch * 8) * 2;
    } else {     // 512-byte rows (256 m/n), 2 rows per KB, ImgMN<512>
      const int row = 2 * q + (lane >> 5), pc = lane & 31;
      const int x = (row & 3) | (((row >> 3) & 1) << 2);
      const int lc = pc ^ (x << 1);
      const int gi = min(row0 + lc * 8, ((rows_total - 1) / 8) * 8);
      src[s] = base + ((int64_t)row * ld + gi) * 2;
    }
  }
}

NSTL_DEV void glds_issue32(char* img, const char* const (&src)[2], int64_t off, int wave) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src[s] + off),
                                     (void __attribute__((address_space(3)))*)(img + (wave * 2 + s) * 1024), 16, 0, 0);
}

// one tile's staging state: the sources of A and B and their per-k byte strides
struct RingSrc {
  const char* a[2];
  const char* b[2];
  int64_t a_kb, b_kb;  // bytes per unit of k
};

template <bool AK, bool BKM>
NSTL_DEV RingSrc ring_src(const GemmParams& p, int m0, int n0, int wave, int lane) {
  RingSrc r;
  glds_src32<AK>(r.a, p.A, p.lda, m0, p.M, wave, lane);
  glds_src32<BKM>(r.b, p.B, p.ldb, n0, p.N, wave, lane);
  r.a_kb = AK ? 2 : 2 * p.lda;
  r.b_kb = BKM ? 2 : 2 * p.ldb;
  return r;
}

NSTL_DEV void ring_stage(char* slot, const RingSrc& r, int k0, int wave) {
  glds_issue32(slot, r.a, (int64_t)k0 * r.a_kb, wave);
  glds_issue32(slot + R_SLOT / 2, r.b, (int64_t)k0 * r.b_kb, wave);
}

#define NSTL_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// LDS fragment reads as inline asm: the compiler cannot prove a ds_read does
// not alias an in-flight LDS-DMA write to another ring slot and would put an
// s_waitcnt vmcnt(0) in front of every K-step's first read, draining the
// prefetch.  Ordering is by the explicit vmcnt/barrier protocol above, and
// the consumer waits with an explicit lgkmcnt(0) + sched_barrier.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x2_t __attribute__((ext_vector_type(2)));
NSTL_DEV uint32_t lds_u32(const char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
NSTL_DEV void asm_frag_k64(bf16x8& f, uint32_t img, int row, int r) {
  // 64-byte rows, 16-byte chunk c of row `row` at c ^ kswz(row) (r: a multiple of 8)
  i32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(img + row * 64 + ((((r >> 3) ^ kswz(row)) & 3) << 4)));
  f = __builtin_bit_cast(bf16x8, v);
}
NSTL_DEV void asm_frag_mn512(bf16x8& f, uint32_t img, int col16, int lane) {
  // ImgMN<512> transpose reads (see frag_col), r0 = 0
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int rb = 8 * g;
  const int byte = (col16 + 4 * pp) * 2;
  i32x2_t v0, v1;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v0) : "v"(img + ImgMN<512>::off(rb + q, byte)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v1) : "v"(img + ImgMN<512>::off(rb + 4 + q, byte)));
  const bf16x4 b0 = __builtin_bit_cast(bf16x4, v0), b1 = __builtin_bit_cast(bf16x4, v1);
  f = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
}

// this wave's share of tile t+1 has landed; later tiles (issued up to t+3) fly on
NSTL_DEV void retire_next(int t, int nk) {
  const int ahead = min(nk, t + 4) - (t + 2);
  if (ahead >= 2) NSTL_VMCNT(8);
  else if (ahead == 1) NSTL_VMCNT(4);
  else NSTL_VMCNT(0);
}

// ---------------------------------------------------------------------------
// Epilogues of the ring kernel.  acc[a][b] holds, in lane l, row 16a + (l&15)
// and columns 16b + 4(l>>4) + 0..3 of the wave's 128 x 64 block, so the raw
// accumulators go to the wave's LDS scratch with one 16-byte write per group
// (f32, two passes of 64 rows).  A compact loop reads row-major chunks back
// and stores 16 bytes per lane: a wave instruction writes 8 rows x 128 B
// (bf16) / 4 rows x 256 B (f32), whole cache lines.  (Storing the 4-column
// groups straight from the accumulators writes 32-byte pieces: ~2x slower.)
//
// The epilogue kind is a template parameter (EM_*), so each instantiation
// carries only its own elementwise code: the generic, branchy form measured
// ~800 VALU + 600 SALU instructions per wave per tile (≈5 µs per 256^2 tile,
// VALU-issue bound).  vmcnt counts loads and stores together, so the input
// loads of a 64-row pass (RoPE cos/sin, the dReLU operand, old C) are all
// issued before the pass's first store: one memory latency per pass (loading
// one iteration ahead paid ~1 µs per iteration).  The bias (fixed per lane)
// is loaded once per tile.
enum { EM_GENERIC = 0, EM_BF16 = 1, EM_RELU_DROP = 2, EM_ROPE = 3, EM_DRELU = 4, EM_F32 = 5, EM_WS = 6 };

constexpr int RING_EPI_RB = 64 * 4 + 16;          // padded f32 scratch row
constexpr int RING_EPI_WAVE = 64 * RING_EPI_RB;   // 17 KB per wave (8 waves: 136 KB)

NSTL_DEV void stage_half(const f32x4 (&acc)[8][4], int half, const GemmParams& p, int row0, int lane, char* scr) {
  const float alpha = p.alpha;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      *(f32x4*)(scr + (16 * a + (lane & 15)) * RING_EPI_RB + (16 * b + 4 * (lane >> 4)) * 4) =
          acc[half * 4 + a][b] * alpha;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ReLU mask word of (64-row block, lane row r0 in 0..7, 8-column group): byte k
// = rows r0 + 8k of the block, bit e = column 8g + e -- one word per lane and
// 64-row pass of the ring epilogue (bf16 output, 8 columns per lane).
NSTL_DEV int64_t relu_mask_index(int N, int row_block64, int r0, int j) {
  return ((int64_t)row_block64 * 8 + r0) * ((N + 7) >> 3) + (j >> 3);
}

// the same for the fp8 kernel's 32x32 accumulators (v_mfma_scale_f32_32x32x64,
// operands swapped): acc[a][b] register r of lane l is row 32a + (l & 31),
// column 32b + 8(r >> 2) + 4(l >> 5) + (r & 3) of the wave's 128 x 64 block
// (fp8 operands: the row scale a_scale[row] is applied here, per lane and row)
NSTL_DEV void stage_half(const f32x16 (&acc)[4][2], int half, const GemmParams& p, int row0, int lane, char* scr) {
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2) {
    const int r = 32 * a2 + (lane & 31);
    const int i = row0 + 64 * half + r;
    const float sc = (i < p.M ? p.a_scale[i] : 0.f) * p.alpha;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& x = acc[half * 2 + a2][b];
        *(f32x4*)(scr + r * RING_EPI_RB + (32 * b + 8 * g + 4 * (lane >> 5)) * 4) =
            (f32x4){x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]} * sc;
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// SC: fp8 operands -- values come scaled by a_scale[row] (stage_half); times b_scale[col] here
template <int EM, bool SC, typename ACC>
NSTL_DEV void ring_epi(const GemmParams& p, const ACC& acc, int row0, int col0, int lane, char* scr,
                       int sq_slot = 0) {
  constexpr bool F32OUT = EM == EM_F32 || EM == EM_WS;
  constexpr int ESZ = F32OUT ? 4 : 2;
  constexpr int CW = 16 / ESZ;   // columns per lane per store (8 bf16 / 4 f32)
  constexpr int LPR = 64 / CW;   // lanes per 64-column row (8 / 16)
  constexpr int RPI = 64 / LPR;  // rows per wave instruction (8 / 4)
  constexpr int NIT = 64 / RPI;  // iterations per 64-row pass
  // per-iteration input registers, all issued before a pass starts
  // old C (f32 out) in two sub-passes of NI iterations (64 VGPRs for a whole pass
  // would push the kernel past 256); the other inputs one sub-pass per pass
  constexpr int SUBS = EM == EM_F32 ? 2 : 1;
  constexpr int NI = NIT / SUBS;
  constexpr int ND = EM == EM_DRELU ? NI : 1;                         // dReLU operand (bf16 x 8)
  constexpr int NF = EM == EM_F32 ? NI : (EM == EM_ROPE ? 2 * NI : 1);  // old C / cos|sin (f32 x 4)
  char* const C = EM == EM_WS ? (char*)(p.ws + (int64_t)blockIdx.y * p.M * p.N) : p.C;
  const int64_t ldc = EM == EM_WS ? p.N : p.ldc;
  const int c = (lane % LPR) * CW, j = col0 + c;
  const bool colok = j < p.N;
  const bool vec = j + CW <= p.N && (ldc % CW) == 0 && ((uintptr_t)C % 16) == 0;
  const bool use_beta = EM == EM_F32 && p.beta != 0.f;
  float bias[CW], csc[CW];
#pragma unroll
  for (int e = 0; e < CW; ++e) bias[e] = 0.f;
  if (SC) {
#pragma unroll
    for (int e = 0; e < CW; ++e) csc[e] = j + e < p.N ? p.b_scale[j + e] : 0.f;
  }
  if ((EM == EM_BF16 || EM == EM_RELU_DROP || EM == EM_ROPE) && p.bias != nullptr) {
#pragma unroll
    for (int e = 0; e < CW; ++e) bias[e] = j + e < p.N ? p.bias[j + e] : 0.f;
  }
  const bool rope_col = EM == EM_ROPE && j < p.rope_cols;
  const uint32_t seed_term = nstl_seed_term(p.seed);
  const int rhalf = p.rope_dim >> 1;
  // cos/sin of 8 columns = 4 consecutive table entries (16 B) when rope_dim % 8 == 0
  const bool rope_vec = (p.rope_dim & 7) == 0;
  const int rope_pr = EM == EM_ROPE && rope_col ? (j % p.rope_dim) >> 1 : 0;  // fixed per lane
  // a pass's rows ib + it * RPI span < 64 rows: with rope_T >= 64 their positions
  // follow from the pass's first by one conditional wrap (no integer modulo per row)
  const bool rope_tinc = EM == EM_ROPE && p.rope_T >= 64;
  float rope_if[4];  // inv_freq of this lane's 4 rotation pairs (NSTL_GEMM_ROPE=fast)
#pragma unroll
  for (int e = 0; e < 4; ++e)
    rope_if[e] = EM == EM_ROPE ? expf(-9.21034049987793f * (float)(2 * (rope_pr + e)) / (float)p.rope_dim) : 0.f;
  const int r0 = lane / LPR;
  // dReLU epilogue: column sums of the stored dh (the FFN1 bias gradient)
  const bool csum_on = EM == EM_DRELU && p.colsum_part != nullptr;
  float csum[CW];
#pragma unroll
  for (int e = 0; e < CW; ++e) csum[e] = 0.f;
  const bool rmask = (EM == EM_RELU_DROP || EM == EM_DRELU) && p.relu_mask != nullptr;
  // f32 out (the weight gradients): sum of squares of the stored values, the
  // clip norm's partial (clip_grad_norm_, utils/training_utils.py:73) without
  // re-reading the gradient arena
  const bool sq_on = EM == EM_F32 && p.sq_part != nullptr;
  float ssq = 0.f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
   const int ib = row0 + half * 64 + r0;
   const int tb = EM == EM_ROPE && rope_col ? ib % p.rope_T : 0;
   const int64_t midx = relu_mask_index(p.N, (row0 + half * 64) >> 6, r0, j);
   // dReLU from the forward's mask word (8 B per lane and pass instead of 8 x 16 B of h)
   uint64_t mword = 0;
   if (EM == EM_DRELU && rmask && colok && ib < p.M) mword = p.relu_mask[midx];
#pragma unroll
   for (int sub = 0; sub < SUBS; ++sub) {
    // Issue every input load of this (sub-)pass first: one memory latency per
    // pass instead of one per iteration (and no load queued behind the stores).
    bf16x8 ind[ND];
    f32x4 inf[NF];
#pragma unroll
    for (int iu = 0; iu < NI; ++iu) {
      const int it = sub * NI + iu;
      const int i = ib + it * RPI;
      const bool ok = i < p.M && colok;
      if (EM == EM_ROPE) {
        f32x4 cs = {1.f, 1.f, 1.f, 1.f}, sn = {0.f, 0.f, 0.f, 0.f};
        if (ok && rope_col) {
          int t;
          if (rope_tinc) {
            t = tb + it * RPI;
            t = t >= p.rope_T ? t - p.rope_T : t;
          } else {
            t = i % p.rope_T;
          }
          if (rope_vec && p.rope_fast) {
            // angle = f32(t) * inv_freq with inv_freq = expf(-ln(1e4) * 2i / d), which is
            // NOT the tables' pow form, then the hardware sin / cos, which lose accuracy as
            // the angle grows: only a kernel-level tolerance covers this (off by default;
            // it needs a parity test against the tables at the largest production T first)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = (float)t * rope_if[e];
              sn[e] = __sinf(a);
              cs[e] = __cosf(a);
            }
          } else if (rope_vec) {
            cs = *(const f32x4*)(p.rope_cos + t * rhalf + rope_pr);
            sn = *(const f32x4*)(p.rope_sin + t * rhalf + rope_pr);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int pr = ((j + 2 * e) % p.rope_dim) >> 1;
              cs[e] = p.rope_cos[t * rhalf + pr];
              sn[e] = p.rope_sin[t * rhalf + pr];
            }
          }
        }
        inf[2 * iu] = cs;
        inf[2 * iu + 1] = sn;
      } else if (EM == EM_DRELU) {
        bf16x8 a8 = {};
        if (ok && !rmask) {
          const bf16* ap = (const bf16*)p.aux + (int64_t)i * p.ld_aux + j;
          if (vec && (p.ld_aux % CW) == 0) {
            a8 = *(const bf16x8*)ap;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] = j + e < p.N ? ap[e] : (bf16)0.f;
          }
        }
        ind[iu % ND] = a8;
      } else if (EM == EM_F32) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        if (ok && use_beta) {
          const float* cp = (const float*)C + (int64_t)i * ldc + j;
          if (vec) {
            o = *(const f32x4*)cp;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = j + e < p.N ? cp[e] : 0.f;
          }
        }
        inf[iu % NF] = o;
      }
    }
    if (sub == 0) stage_half(acc, half, p, row0, lane, scr);
    auto body = [&](int iu) {
      const int it = sub * NI + iu;
      const int i = ib + it * RPI;
      const char* src = scr + (it * RPI + r0) * RING_EPI_RB + c * 4;
      float v[CW];
      {
        // the wave's own scratch, read by asm: as plain loads the compiler put
        // vmcnt(0) in front of each (the ring's stage DMA may alias), i.e. a wait
        // for every store of the iterations before
        f32x4 v0, v1;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v0) : "v"(lds_u32(src)) : "memory");
        if (CW == 8) asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(v1) : "v"(lds_u32(src)) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v0[e];
        if (CW == 8) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[(4 + e) % CW] = v1[e];
        }
      }
      if (i < p.M && colok) {
        if (SC) {
#pragma unroll
          for (int e = 0; e < CW; ++e) v[e] *= csc[e];
        }
#pragma unroll
        for (int e = 0; e < CW; ++e) v[e] += bias[e];
        if (EM == EM_RELU_DROP) {
#pragma unroll
          for (int e = 0; e < CW; ++e) v[e] = fmaxf(v[e], 0.f);
          if (p.thresh) {
            // pair index of element (i, j): N even, j % 8 == 0; 32-bit (launcher check)
            const uint32_t pair = (uint32_t)i * (uint32_t)(p.N >> 1) + (uint32_t)(j >> 1);
#pragma unroll
            for (int e = 0; e < CW; e += 2) {
              bool k0, k1;
              nstl_keep2_32(seed_term, pair + (e >> 1), p.thresh, k0, k1);
              v[e] = k0 ? v[e] * p.inv_keep : 0.f;
              v[e + 1] = k1 ? v[e + 1] * p.inv_keep : 0.f;
            }
          }
          if (rmask) {
            uint32_t bits = 0;
#pragma unroll
            for (int e = 0; e < CW; ++e) bits |= ((bf16)v[e] > (bf16)0.f ? 1u : 0u) << e;  // as stored
            mword |= (uint64_t)bits << (8 * it);
          }
        } else if (EM == EM_ROPE) {
          if (rope_col) {
            const f32x4 cs = inf[(2 * iu) % NF], sn = inf[(2 * iu + 1) % NF];
#pragma unroll
            for (int e = 0; e < CW; e += 2) {
              const float x0 = v[e], x1 = v[e + 1];
              v[e] = x0 * cs[(e / 2) % 4] - x1 * sn[(e / 2) % 4];
              v[e + 1] = x0 * sn[(e / 2) % 4] + x1 * cs[(e / 2) % 4];
            }
          }
        } else if (EM == EM_DRELU) {
          if (rmask) {
            const uint32_t bits = (uint32_t)(mword >> (8 * it));
#pragma unroll
            for (int e = 0; e < CW; ++e) v[e] = ((bits >> e) & 1) ? v[e] * p.inv_keep : 0.f;
          } else {
            const bf16x8 a8 = ind[iu % ND];
#pragma unroll
            for (int e = 0; e < CW; ++e) v[e] = (float)a8[e % 8] > 0.f ? v[e] * p.inv_keep : 0.f;
          }
          if (csum_on) {
#pragma unroll
            for (int e = 0; e < CW; ++e) csum[e] += (float)(bf16)v[e];  // sum what is stored
          }
        } else if (EM == EM_F32) {
          if (use_beta) {
            const f32x4 o = inf[iu % NF];
#pragma unroll
            for (int e = 0; e < CW; ++e) v[e] += p.beta * o[e % 4];
          }
          if (sq_on) {
#pragma unroll
            for (int e = 0; e < CW; ++e)
              if (vec || j + e < p.N) ssq += v[e] * v[e];
          }
        }
        char* dst = C + ((int64_t)i * ldc + j) * ESZ;
        if (p.debug_skip_epilogue == 2) {  // NSTL_GEMM_DEBUG=skip_store: timing experiments only
        } else if (vec) {
          if (ESZ == 4)
            *(f32x4*)dst = (f32x4){v[0], v[1 % CW], v[2 % CW], v[3 % CW]};
          else
            *(bf16x8*)dst = (bf16x8){(bf16)v[0], (bf16)v[1 % CW], (bf16)v[2 % CW], (bf16)v[3 % CW],
                                     (bf16)v[4 % CW], (bf16)v[5 % CW], (bf16)v[6 % CW], (bf16)v[7 % CW]};
        } else {
#pragma unroll
          for (int e = 0; e < CW; ++e)
            if (j + e < p.N) {
              if (ESZ == 4) ((float*)dst)[e] = v[e];
              else ((bf16*)dst)[e] = (bf16)v[e];
            }
        }
      }
    };
    // input registers are indexed by iteration: unroll fully; the others keep
    // the loop short (a full unroll of the dropout hash costs I-cache)
    if constexpr (ND > 1 || NF > 1) {
#pragma unroll
      for (int iu = 0; iu < NI; ++iu) body(iu);
    } else {
#pragma unroll 2
      for (int iu = 0; iu < NI; ++iu) body(iu);
    }
   }
   if (EM == EM_RELU_DROP && rmask && colok && ib < p.M) p.relu_mask[midx] = mword;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (sq_on) {
    const double t = wave_sum_d((double)ssq);
    if (lane == 0) p.sq_part[sq_slot] = (float)t;
  }
  if (csum_on) {
    // lanes l, l + LPR, ... share columns: fold them, then LPR lanes write the
    // wave's 64 column sums as one partial row (this wave's 128 rows)
#pragma unroll
    for (int e = 0; e < CW; ++e) {
      // the xor-LPR, 16, 32 butterfly (bit-identical pairs) on DPP / permlane moves
      if (LPR == 8) csum[e] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(csum[e]), 0x128, 0xF, 0xF, false));
      else if (LPR != 16) csum[e] += __shfl_xor(csum[e], LPR);  // row_ror:8 above = lane ^ 8 in a 16-lane row
      csum[e] = sum_xor16(csum[e]);
      csum[e] = sum_xor32(csum[e]);
    }
    if (lane < LPR && colok) {
      float* dst = p.colsum_part + (int64_t)(row0 >> 7) * p.N + j;
#pragma unroll
      for (int e = 0; e < CW; ++e)
        if (j + e < p.N) dst[e] = csum[e];
    }
  }
}

// generic fallback (any epilogue op, beta, dtype): per 4-column group epi_store4
NSTL_DEV void ring_epi_generic(const GemmParams& p, const f32x4 (&acc)[8][4], int row0, int col0, int lane,
                               char* scr) {
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    stage_half(acc, half, p, row0, lane, scr);
#pragma unroll 1
    for (int it = 0; it < 16; ++it) {
      const int r = it * 4 + (lane >> 4), c = (lane & 15) * 4;
      const int i = row0 + half * 64 + r;
      if (i < p.M && col0 + c < p.N) epi_store4(p, i, col0 + c, *(const f32x4*)(scr + r * RING_EPI_RB + c * 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// EM_BF16 on a full tile without the LDS staging pass.  Lane (g, c) holds row
// 16a + c, columns 16b + 4g .. +3 of acc[a][b]; after the bias and the bf16 packing,
// a permlane16 swap of the chunks of b and b + 1 (odd 16-lane rows of the first
// operand <-> even rows of the second) leaves lane g even with columns 16b + 4g .. +7
// and lane g odd with 16(b + 1) + 4(g - 1) .. +7: one 16-byte store per lane and
// pair of column blocks, 64 contiguous bytes per row per wave instruction.  The
// ring is not reused, so no barrier precedes it.
NSTL_DEV uint32_t pack_bf16x2(float lo, float hi) {
  const bf16 a = (bf16)lo, b = (bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}
NSTL_DEV void load_bias16(float (&bias)[4][4], const GemmParams& p, int col0, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[b][e] = p.bias != nullptr ? p.bias[col0 + 16 * b + 4 * g + e] : 0.f;
}
NSTL_DEV void ring_epi_bf16_direct_b(const GemmParams& p, const f32x4 (&acc)[8][4], const float (&bias)[4][4],
                                     int row0, int col0, int lane);
NSTL_DEV void ring_epi_bf16_direct(const GemmParams& p, const f32x4 (&acc)[8][4], int row0, int col0, int lane) {
  float bias[4][4];
  load_bias16(bias, p, col0, lane);
  ring_epi_bf16_direct_b(p, acc, bias, row0, col0, lane);
}
NSTL_DEV void ring_epi_bf16_direct_b(const GemmParams& p, const f32x4 (&acc)[8][4], const float (&bias)[4][4],
                                     int row0, int col0, int lane) {
  const int g = lane >> 4, c = lane & 15, odd = g & 1;
  const float alpha = p.alpha;
  bf16* const cbase = (bf16*)p.C + (int64_t)(row0 + c) * p.ldc + col0;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    bf16* crow = cbase + (int64_t)(16 * a) * p.ldc;
#pragma unroll
    for (int bp = 0; bp < 4; bp += 2) {
      const f32x4 u = acc[a][bp], v = acc[a][bp + 1];
      uint32_t x0 = pack_bf16x2(u[0] * alpha + bias[bp][0], u[1] * alpha + bias[bp][1]);
      uint32_t x1 = pack_bf16x2(u[2] * alpha + bias[bp][2], u[3] * alpha + bias[bp][3]);
      uint32_t y0 = pack_bf16x2(v[0] * alpha + bias[bp + 1][0], v[1] * alpha + bias[bp + 1][1]);
      uint32_t y1 = pack_bf16x2(v[2] * alpha + bias[bp + 1][2], v[3] * alpha + bias[bp + 1][3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      const int col = 16 * (bp + odd) + 4 * (g - odd);
      if (p.debug_skip_epilogue != 2)
        *(uint4*)(crow + col) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
  }
}

constexpr int R_SMEM = R_STAGES * R_SLOT;
static_assert(8 * RING_EPI_WAVE <= R_SMEM, "epilogue scratch must fit in the ring");

// Diagnostic build only (make stamps -> libnstl_hip_stamps.so, tools/gemm_timeline.py):
// wave 0 of every ring-GEMM workgroup records the global 100 MHz clock at tile
// entry, after the prologue, after the K loop and after its epilogue stores have
// retired, plus where it ran (HW_ID, XCC_ID).  No product build executes a stamp.
#ifdef NSTL_STAMPS
constexpr int STAMP_MAX = 1 << 16, STAMP_W = 8;
__device__ unsigned long long g_nstl_stamps[STAMP_MAX * STAMP_W];
NSTL_DEV unsigned long long rt_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define NSTL_STAMP(var) const unsigned long long var = rt_stamp()
#else
#define NSTL_STAMP(var)
#endif

// One 256 x 256 output tile of p: `id` is the tile's linear index in p's grid
// (already XCD-remapped by the caller), `kz` its split-K chunk.
template <bool AK, bool BKM, int EM>
NSTL_DEV void ring_tile(const GemmParams& p, int id, int kz0, int kz1, char* smem) {
  NSTL_STAMP(st_entry);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nt_n = (p.N + BIG - 1) / BIG, nt_m = (p.M + BIG - 1) / BIG;
  // grouped order (GROUP_M row tiles per group, column-fastest inside) over
  // XCD-contiguous id ranges: an XCD's 32 co-resident blocks cover ~4 x 8 tiles
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * nt_n;
  const int first_m = (id / per_group) * GROUP_M;
  const int gm = min(nt_m - first_m, GROUP_M);
  const int in_g = id % per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const int m0 = tm * BIG, n0 = tn * BIG;
  const int nk = (kz1 - kz0) / R_BK;
  const uint32_t smem_u32 = lds_u32(smem);
  const RingSrc rs = ring_src<AK, BKM>(p, m0, n0, wave, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: tiles 0..2 in flight, tile 0 landed everywhere
#pragma unroll
  for (int s = 0; s < 3; ++s)
    if (s < nk) ring_stage(smem + s * R_SLOT, rs, kz0 + s * R_BK, wave);
  if (nk >= 3) NSTL_VMCNT(8);
  else if (nk == 2) NSTL_VMCNT(4);
  else NSTL_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  NSTL_STAMP(st_prologue);
  if (wm == 1) __builtin_amdgcn_s_barrier();  // the stagger

  // Branch-free steps (as the fp8 kernel): in the main loop both groups wait
  // vmcnt(8) at both of their wait points (the earlier retires stage kt+1 for
  // group 1, the later for group 0; the other is then already satisfied or
  // nearly so), with the count a constant of each call (8 while a stage is
  // issued three ahead, then 4, 0, 0), instead of the per-step branch chain of
  // retire_next.
  int slot = 0;
  auto step = [&](int kt, bool stage3, int wait) {
    // ---- R(kt)
    const uint32_t Ai = smem_u32 + slot * R_SLOT;
    const uint32_t Bi = Ai + R_SLOT / 2;
    bf16x8 fb[4], fa[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (BKM) asm_frag_k64(fb[t], Bi, wn * 64 + t * 16 + (lane & 15), 8 * (lane >> 4));
      else asm_frag_mn512(fb[t], Bi, wn * 64 + t * 16, lane);
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (AK) asm_frag_k64(fa[a], Ai, wm * 128 + a * 16 + (lane & 15), 8 * (lane >> 4));
      else asm_frag_mn512(fa[a], Ai, wm * 128 + a * 16, lane);
    }
    if (stage3) {
      int s3 = slot + 3;
      if (s3 >= R_STAGES) s3 -= R_STAGES;
      ring_stage(smem + s3 * R_SLOT, rs, kz0 + (kt + 3) * R_BK, wave);
    }
    if (wait == 8) NSTL_VMCNT(8);
    else if (wait == 4) NSTL_VMCNT(4);
    else if (wait == 0) NSTL_VMCNT(0);
    else if (wm == 1) retire_next(kt, nk);
    __builtin_amdgcn_s_barrier();
    // ---- M(kt)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    // operands swapped: acc[a][b] takes C^T's register layout, i.e. lane l owns
    // row 16a + (l & 15) and the four consecutive columns 16b + 4(l >> 4) + 0..3
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) mma16(acc[a][b], fb[b], fa[a]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    if (wait == 8) NSTL_VMCNT(8);
    else if (wait == 4) NSTL_VMCNT(4);
    else if (wait == 0) NSTL_VMCNT(0);
    else if (wm == 0) retire_next(kt, nk);
    __builtin_amdgcn_s_barrier();
    slot = slot + 1 == R_STAGES ? 0 : slot + 1;
  };
  if (nk >= 3) {
    for (int kt = 0; kt + 3 < nk; ++kt) step(kt, true, 8);
    step(nk - 3, false, 4);
    step(nk - 2, false, 0);
    step(nk - 1, false, 0);
  } else {
    for (int kt = 0; kt < nk; ++kt) step(kt, false, -1);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // close the stagger
  NSTL_STAMP(st_kloop);
  if (p.debug_skip_epilogue == 1) {  // timing experiments only (NSTL_GEMM_DEBUG=skip_epi)
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) asm volatile("" ::"v"(acc[a][b]));
  } else if (EM == EM_BF16 && p.direct_epi && m0 + BIG <= p.M && n0 + BIG <= p.N) {
    ring_epi_bf16_direct(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
  } else {
    __syncthreads();  // every wave is done with the ring: it becomes scratch
    char* scr = smem + wave * RING_EPI_WAVE;
    const int row0 = m0 + wm * 128, col0 = n0 + wn * 64;
    if (EM == EM_GENERIC) ring_epi_generic(p, acc, row0, col0, lane, scr);
    else ring_epi<EM, false>(p, acc, row0, col0, lane, scr, id * 8 + wave);
  }
#ifdef NSTL_STAMPS
  NSTL_VMCNT(0);
  NSTL_STAMP(st_epi);
  if (wave == 0 && lane == 0) {
    // slot: tile id (+ 2^15 for the second piece of a split tile)
    const int slot = (id + blockIdx.y * gridDim.x + (kz0 > 0 && blockIdx.y == 0 ? 32768 : 0)) % STAMP_MAX;
    unsigned long long* s = g_nstl_stamps + (int64_t)slot * STAMP_W;
    s[0] = st_entry; s[1] = st_prologue; s[2] = st_kloop; s[3] = st_epi;
    s[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    s[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    s[6] = id; s[7] = nk;
  }
#endif
}

template <bool AK, bool BKM, int EM>
__global__ __launch_bounds__(BIG_NT, 1) void gemm256r_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[R_SMEM];
  const int nt = ((p.M + BIG - 1) / BIG) * ((p.N + BIG - 1) / BIG);
  const int kb = blockIdx.y * p.k_chunk;
  ring_tile<AK, BKM, EM>(p, xcd_remap(blockIdx.x, nt), kb, min(p.K, kb + p.k_chunk), smem);
}

// ===========================================================================
// FP8 forward GEMM (BASELINE config C5: fp8 QKV/FFN projections):
//   C[i][j] = sa[i] * sb[j] * sum_r qa[i][r] qb[j][r]  (+ epilogue)
// with A [M][K], B [N][K] OCP e4m3 bytes (K-major) and f32 row scales sa (per
// row of A = token) and sb (per row of B = output channel) from
// nstl_fp8_quant_rows.  The products run on v_mfma_scale_f32_32x32x64_f8f6f4
// with unit E8M0 block scales (K = 64 per instruction: twice the bf16 rate per
// clock, MI355X_MICROARCH.md "Matrix cores"; the non-scaled fp8 MFMAs only run
// at the bf16 rate); the row scales are applied by the epilogue, so the K loop
// moves nothing but operand bytes.
// The bf16 ring kernel's structure is kept as is: 256x256 tile, 8 waves (2 x 4,
// 128 x 64 each), a ring of five 32 KB LDS-DMA stages issued three ahead, the
// two wave groups one barrier apart, the same vmcnt/barrier protocol.  A stage
// holds 64 K-bytes of A and of B (256 rows x 64 B each; 16-byte chunk c of row
// r sits at c ^ ((r >> 2) & 3), which puts every ds_read_b128 lane group of the
// fragment reads on 16 distinct bank slots).  Per stage a wave issues 8 MFMAs
// (4 A fragments of 32 rows x 2 B fragments of 32 columns): the same 512 MFMA
// cycles as a bf16 stage, for twice the K.
constexpr int F8_BK = 64;        // K bytes (= elements) per fp8 stage
constexpr int F8_UNIT = 0x7f7f7f7f;  // E8M0 127 = 2^0 in every byte


// per-lane sources of one fp8 stage, once per tile (K-major rows: a K-step adds k0 bytes)
NSTL_DEV void glds_src_f8(const char* (&src)[2], const char* base, int64_t ld, int row0, int rows_total, int wave,
                          int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int row = 16 * (wave * 2 + s) + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);
    src[s] = base + (int64_t)min(row0 + row, rows_total - 1) * ld + c * 16;
  }
}

NSTL_DEV RingSrc ring_src_f8(const GemmParams& p, int m0, int n0, int wave, int lane) {
  RingSrc r;
  glds_src_f8(r.a, p.A, p.lda, m0, p.M, wave, lane);
  glds_src_f8(r.b, p.B, p.ldb, n0, p.N, wave, lane);
  r.a_kb = r.b_kb = 1;
  return r;
}

// one 32 x 64 fp8 fragment: lane l holds row (l & 31), K bytes 32 (l >> 5) .. +31
NSTL_DEV void asm_frag_f8(i32x8& f, uint32_t img, int row, int lane) {
  const int h = lane >> 5, x = (row >> 2) & 3;
  i32x4_t v0, v1;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v0) : "v"(img + row * 64 + (((2 * h) ^ x) << 4)));
  asm volatile("ds_read_b128 %0, %1" : "=v"(v1) : "v"(img + row * 64 + (((2 * h + 1) ^ x) << 4)));
  f = (i32x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
}

// operands swapped as in the bf16 kernel (weights first, so acc takes C^T's layout)
NSTL_DEV void mma_f8(f32x16& acc, const i32x8& w, const i32x8& x) {
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(w, x, acc, 0, 0, 0, F8_UNIT, 0, F8_UNIT);
}

template <int EM>
NSTL_DEV void ring_tile_f8(const GemmParams& p, int id, char* smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nt_n = (p.N + BIG - 1) / BIG, nt_m = (p.M + BIG - 1) / BIG;
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * nt_n;
  const int first_m = (id / per_group) * GROUP_M;
  const int gm = min(nt_m - first_m, GROUP_M);
  const int in_g = id % per_group;
  const int tm = first_m + in_g % gm, tn = in_g / gm;
  const int m0 = tm * BIG, n0 = tn * BIG;
  const int nk = p.K / F8_BK;
  const uint32_t smem_u32 = lds_u32(smem);
  const RingSrc rs = ring_src_f8(p, m0, n0, wave, lane);

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

#pragma unroll
  for (int s = 0; s < 3; ++s)
    if (s < nk) ring_stage(smem + s * R_SLOT, rs, s * F8_BK, wave);
  if (nk >= 3) NSTL_VMCNT(8);
  else if (nk == 2) NSTL_VMCNT(4);
  else NSTL_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // the stagger

  // Branch-free steps: both groups retire stage kt+1 at both of their waits
  // (the earlier is group 1's, the later group 0's; the other is then already
  // satisfied or nearly so), with the count a constant of each call (8 while a
  // stage is issued three ahead, then 4, 0, 0).  With a branch between the MFMAs
  // and the barrier, LLVM sinks the scaled MFMAs (unlike the bf16 ones) past it,
  // out of the prioritised phase.
  int slot = 0;
  // wait: the vmcnt both groups use (-1: the per-group retire_next, short K)
  auto step = [&](int kt, bool stage3, int wait) {
    // ---- R(kt)
    const uint32_t Ai = smem_u32 + slot * R_SLOT;
    const uint32_t Bi = Ai + R_SLOT / 2;
    i32x8 fb[2], fa[4];
#pragma unroll
    for (int t = 0; t < 2; ++t) asm_frag_f8(fb[t], Bi, wn * 64 + t * 32 + (lane & 31), lane);
#pragma unroll
    for (int a = 0; a < 4; ++a) asm_frag_f8(fa[a], Ai, wm * 128 + a * 32 + (lane & 31), lane);
    if (stage3) {
      int s3 = slot + 3;
      if (s3 >= R_STAGES) s3 -= R_STAGES;
      ring_stage(smem + s3 * R_SLOT, rs, (kt + 3) * F8_BK, wave);
    }
    if (wait == 8) NSTL_VMCNT(8);
    else if (wait == 4) NSTL_VMCNT(4);
    else if (wait == 0) NSTL_VMCNT(0);
    else if (wm == 1) retire_next(kt, nk);
    __builtin_amdgcn_s_barrier();
    // ---- M(kt)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) mma_f8(acc[a][b], fb[b], fa[a]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    if (wait == 8) NSTL_VMCNT(8);
    else if (wait == 4) NSTL_VMCNT(4);
    else if (wait == 0) NSTL_VMCNT(0);
    else if (wm == 0) retire_next(kt, nk);
    __builtin_amdgcn_s_barrier();
    slot = slot + 1 == R_STAGES ? 0 : slot + 1;
  };
  if (nk >= 3) {
    for (int kt = 0; kt + 3 < nk; ++kt) step(kt, true, 8);
    step(nk - 3, false, 4);
    step(nk - 2, false, 0);
    step(nk - 1, false, 0);
  } else {
    for (int kt = 0; kt < nk; ++kt) step(kt, false, -1);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // close the stagger
  if (p.debug_skip_epilogue == 1) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) asm volatile("" ::"v"(acc[a][b]));
    return;
  }
  __syncthreads();  // every wave is done with the ring: it becomes scratch
  char* scr = smem + wave * RING_EPI_WAVE;
  ring_epi<EM, true>(p, acc, m0 + wm * 128, n0 + wn * 64, lane, scr);
}

template <int EM>
__global__ __launch_bounds__(BIG_NT, 1) void gemm256f8_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[R_SMEM];
  const int nt = ((p.M + BIG - 1) / BIG) * ((p.N + BIG - 1) / BIG);
  ring_tile_f8<EM>(p, xcd_remap(blockIdx.x, nt), smem);
}

// which lean epilogue fits this call (EM_GENERIC when none does)
int ring_epi_mode(const nstl_gemm_args* a, const GemmParams& p) {
  if (p.ws != nullptr) return EM_WS;
  if (p.c_f32) return a->epilogue == NSTL_EPI_NONE ? EM_F32 : EM_GENERIC;
  if (p.beta != 0.f) return EM_GENERIC;
  switch (a->epilogue) {
    case NSTL_EPI_NONE:
    case NSTL_EPI_BIAS: return EM_BF16;
    case NSTL_EPI_BIAS_RELU_DROP: return (a->N % 2 == 0) ? EM_RELU_DROP : EM_GENERIC;
    case NSTL_EPI_BIAS_ROPE: return EM_ROPE;
    case NSTL_EPI_DRELU_DROP: return a->dtype == NSTL_BF16 || a->dtype == NSTL_FP8 ? EM_DRELU : EM_GENERIC;
  }
  return EM_GENERIC;
}

template <bool AK, bool BKM>
void launch_ring_em(int em, dim3 grid, dim3 block, hipStream_t st, const GemmParams& p) {
  switch (em) {
    case EM_BF16: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_BF16>), grid, block, 0, st, p); break;
    case EM_RELU_DROP: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_RELU_DROP>), grid, block, 0, st, p); break;
    case EM_ROPE: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_ROPE>), grid, block, 0, st, p); break;
    case EM_DRELU: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_DRELU>), grid, block, 0, st, p); break;
    case EM_F32: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_F32>), grid, block, 0, st, p); break;
    case EM_WS: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_WS>), grid, block, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, EM_GENERIC>), grid, block, 0, st, p); break;
  }
}

// split-K combine: C = sum_z ws[z] (+bias) (+beta*C)
__global__ void splitk_reduce(const float* ws, int splits, int M, int N, char* C, int64_t ldc, int c_f32,
                              float beta, const float* bias) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[(int64_t)z * total + e];
    const int i = (int)(e / N), j = (int)(e % N);
    if (bias) v += bias[j];
    const int64_t o = (int64_t)i * ldc + j;
    if (c_f32) {
      float* c = (float*)C + o;
      if (beta != 0.f) v += beta * *c;
      *c = v;
    } else {
      bf16* c = (bf16*)C + o;
      if (beta != 0.f) v += beta * (float)*c;
      *c = (bf16)v;
    }
  }
}

int launch_big(const nstl_gemm_args* a, GemmParams& p, int splits, hipStream_t st) {
  const int nt = ((a->M + BIG - 1) / BIG) * ((a->N + BIG - 1) / BIG);
  dim3 grid(nt, splits), block(BIG_NT);
  const int em = ring_epi_mode(a, p);
  if (a->a_kmajor && a->b_kmajor) launch_ring_em<true, true>(em, grid, block, st, p);
  else if (a->a_kmajor && !a->b_kmajor) launch_ring_em<true, false>(em, grid, block, st, p);
  else if (!a->a_kmajor && !a->b_kmajor) launch_ring_em<false, false>(em, grid, block, st, p);
  else launch_ring_em<false, true>(em, grid, block, st, p);
  NSTL_LAUNCH_CHECK("nstl_gemm (256 ring)");
  nstl::count(NSTL_K_GEMM_RING);
  nstl::count(NSTL_K_GEMM_RING_TILES, (long long)nt * splits);
  return 0;
}

template <typename T>
int launch_typed(const nstl_gemm_args* a, GemmParams& p, int splits, hipStream_t st) {
  const int nt = ((a->M + BM - 1) / BM) * ((a->N + BN - 1) / BN);
  dim3 grid(nt, splits), block(NTHREADS);
  if (a->a_kmajor && a->b_kmajor)
    hipLaunchKernelGGL((gemm_kernel<T, true, true>), grid, block, 0, st, p);
  else if (a->a_kmajor && !a->b_kmajor)
    hipLaunchKernelGGL((gemm_kernel<T, true, false>), grid, block, 0, st, p);
  else if (!a->a_kmajor && !a->b_kmajor)
    hipLaunchKernelGGL((gemm_kernel<T, false, false>), grid, block, 0, st, p);
  else
    hipLaunchKernelGGL((gemm_kernel<T, false, true>), grid, block, 0, st, p);
  NSTL_LAUNCH_CHECK("nstl_gemm");
  nstl::count(NSTL_K_GEMM128);
  return 0;
}

// NSTL_GEMM_DEBUG=skip_epi / skip_store: the ring kernel computes no epilogue /
// stores nothing (timing experiments only: wrong results)
int getenv_debug_skip_epi() {
  static const int v = [] {
    const char* e = getenv("NSTL_GEMM_DEBUG");
    return !e ? 0 : std::string(e) == "skip_epi" ? 1 : std::string(e) == "skip_store" ? 2 : 0;
  }();
  return v;
}

// NSTL_GEMM_SMALL=1 forces the 128x128 kernel (A/B comparisons, debugging)
bool getenv_small_gemm() {
  static const int v = [] {
    const char* e = getenv("NSTL_GEMM_SMALL");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return v != 0;
}

}  // namespace

extern "C" int64_t nstl_gemm_workspace_bytes(int M, int N, int split_k) {
  return split_k > 1 ? (int64_t)split_k * M * N * 4 : 0;
}

namespace {

// validate one problem and fill its kernel parameters (no split-K decisions)
int make_params(const nstl_gemm_args* a, GemmParams& p) {
  NSTL_CHECK_ARG(a != nullptr, "nstl_gemm: null args");
  NSTL_CHECK_ARG(a->dtype == NSTL_F32 || a->dtype == NSTL_BF16 || a->dtype == NSTL_FP8, "nstl_gemm: bad dtype %d",
                 a->dtype);
  NSTL_CHECK_ARG(a->c_dtype == NSTL_F32 || a->c_dtype == NSTL_BF16, "nstl_gemm: bad c_dtype");
  NSTL_CHECK_ARG(a->M > 0 && a->N > 0 && a->K > 0, "nstl_gemm: empty problem %dx%dx%d", a->M, a->N, a->K);
  const int esz = a->dtype == NSTL_F32 ? 4 : a->dtype == NSTL_BF16 ? 2 : 1;
  const int vec = 16 / esz;
  NSTL_CHECK_ARG(((uintptr_t)a->A % 16) == 0 && ((uintptr_t)a->B % 16) == 0,
                 "nstl_gemm: A and B must be 16-byte aligned");
  NSTL_CHECK_ARG(a->lda % vec == 0 && a->ldb % vec == 0, "nstl_gemm: lda/ldb must be multiples of %d", vec);
  // K-major rows are read in 16-byte chunks: the reduction extent is rounded up to
  // a chunk and must be readable (zero-padded) up to lda/ldb.
  NSTL_CHECK_ARG(!a->a_kmajor || a->lda >= ((a->K + vec - 1) / vec) * vec, "nstl_gemm: lda < K");
  NSTL_CHECK_ARG(!a->b_kmajor || a->ldb >= ((a->K + vec - 1) / vec) * vec, "nstl_gemm: ldb < K");
  NSTL_CHECK_ARG(a->a_kmajor || a->lda >= ((a->M + vec - 1) / vec) * vec, "nstl_gemm: lda < M");
  NSTL_CHECK_ARG(a->b_kmajor || a->ldb >= ((a->N + vec - 1) / vec) * vec, "nstl_gemm: ldb < N");
  NSTL_CHECK_ARG(a->ldc >= a->N, "nstl_gemm: ldc < N");
  NSTL_CHECK_ARG(a->epilogue >= 0 && a->epilogue <= 4, "nstl_gemm: bad epilogue %d", a->epilogue);
  if (a->epilogue == NSTL_EPI_BIAS_ROPE) {
    NSTL_CHECK_ARG(a->rope_cos && a->rope_sin && a->rope_T > 0 && a->rope_dim > 0 && a->rope_dim % 2 == 0,
                   "nstl_gemm: rope tables missing");
    NSTL_CHECK_ARG(a->rope_cols % 16 == 0, "nstl_gemm: rope_cols must be a multiple of 16");
  }
  if (a->epilogue == NSTL_EPI_DRELU_DROP) NSTL_CHECK_ARG(a->aux != nullptr, "nstl_gemm: aux missing");
  NSTL_CHECK_ARG(a->p_drop >= 0.f && a->p_drop < 1.f, "nstl_gemm: p_drop out of range");
  NSTL_CHECK_ARG(a->p_drop == 0.f || nstl_pair_index32_ok((uint64_t)a->M * a->N),
                 "nstl_gemm: M*N past 2^33 dropout elements (32-bit pair index)");

  p.A = (const char*)a->A; p.lda = a->lda;
  p.B = (const char*)a->B; p.ldb = a->ldb;
  p.C = (char*)a->C; p.ldc = a->ldc;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.c_f32 = a->c_dtype == NSTL_F32;
  p.alpha = a->alpha; p.beta = a->beta;
  p.epi = a->epilogue;
  p.bias = a->bias;
  p.aux = (const char*)a->aux; p.ld_aux = a->ld_aux; p.aux_f32 = a->dtype == NSTL_F32;
  p.thresh = nstl_drop_thresh(a->p_drop);
  p.inv_keep = 1.0f / (1.0f - a->p_drop);
  p.seed = a->seed;
  p.rope_cos = a->rope_cos; p.rope_sin = a->rope_sin;
  p.rope_T = a->rope_T; p.rope_dim = a->rope_dim; p.rope_cols = a->rope_cols;
  {
    // NSTL_GEMM_ROPE=fast (A/B, read per call): the bf16 ring epilogue recomputes the
    // RoPE angles (v_sin / v_cos, as the attention backward does) instead of loading
    // 2 x 16 B of table per row; the f32 parity-mode kernels always use the tables
    const char* e = getenv("NSTL_GEMM_ROPE");
    p.rope_fast = e != nullptr && strcmp(e, "fast") == 0;
  }
  p.ws = nullptr;
  p.debug_skip_epilogue = getenv_debug_skip_epi();
  // NSTL_GEMM_DIRECT=0: the LDS-staged EM_BF16 epilogue (A/B; read per call).  The
  // direct one needs 16-byte aligned rows of C.
  {
    const char* e = getenv("NSTL_GEMM_DIRECT");
    p.direct_epi = !(e && e[0] == '0') && (a->ldc % 8) == 0 && ((uintptr_t)a->C % 16) == 0;
  }
  p.k_chunk = a->K;
  p.colsum_part = a->colsum_part;
  p.relu_mask = a->relu_mask;
  p.a_scale = a->a_scale;
  p.b_scale = a->b_scale;
  p.sq_part = a->sq_part;
  return 0;
}

}  // namespace
namespace nstl {
int gemm4_f8(const nstl_gemm_args* a, hipStream_t st, int* handled);  // gemm4.hip
}
namespace {

// FP8 operands: the 4-wave kernel for full tiles (gemm4f8_kernel), the fp8 ring
// kernel otherwise (K-major A and B, K % 64 == 0, no split-K)
int gemm_f8(const nstl_gemm_args* a, GemmParams& p, hipStream_t st) {
  NSTL_CHECK_ARG(a->a_kmajor && a->b_kmajor, "nstl_gemm: FP8 needs K-major A and B (Y = X W^T)");
  NSTL_CHECK_ARG(a->K % 64 == 0, "nstl_gemm: FP8 needs K %% 64 == 0 (got %d)", a->K);
  NSTL_CHECK_ARG(a->a_scale && a->b_scale, "nstl_gemm: FP8 needs the row scales a_scale [M] and b_scale [N]");
  NSTL_CHECK_ARG(a->split_k <= 1, "nstl_gemm: FP8: no split-K");
  {
    int handled = 0;
    if (int rc = nstl::gemm4_f8(a, st, &handled)) return rc;
    if (handled) return 0;
  }
  const int em = ring_epi_mode(a, p);
  NSTL_CHECK_ARG(em == EM_BF16 || em == EM_RELU_DROP || em == EM_ROPE || em == EM_DRELU || em == EM_F32,
                 "nstl_gemm: FP8 supports the NONE / BIAS / BIAS_RELU_DROP / BIAS_ROPE / DRELU_DROP epilogues "
                 "(bf16 out without beta, or f32 out without epilogue)");
  NSTL_CHECK_ARG(!a->relu_mask || em == EM_RELU_DROP || em == EM_DRELU,
                 "nstl_gemm: relu_mask needs the ReLU-dropout / dReLU epilogue");
  NSTL_CHECK_ARG(!a->colsum_part || em == EM_DRELU, "nstl_gemm: FP8: colsum_part needs the dReLU epilogue");
  const int nt = ((a->M + BIG - 1) / BIG) * ((a->N + BIG - 1) / BIG);
  dim3 grid(nt), block(BIG_NT);
  switch (em) {
    case EM_BF16: hipLaunchKernelGGL((gemm256f8_kernel<EM_BF16>), grid, block, 0, st, p); break;
    case EM_RELU_DROP: hipLaunchKernelGGL((gemm256f8_kernel<EM_RELU_DROP>), grid, block, 0, st, p); break;
    case EM_ROPE: hipLaunchKernelGGL((gemm256f8_kernel<EM_ROPE>), grid, block, 0, st, p); break;
    case EM_DRELU: hipLaunchKernelGGL((gemm256f8_kernel<EM_DRELU>), grid, block, 0, st, p); break;
    default: hipLaunchKernelGGL((gemm256f8_kernel<EM_F32>), grid, block, 0, st, p); break;
  }
  NSTL_LAUNCH_CHECK("nstl_gemm (FP8)");
  nstl::count(NSTL_K_GEMM_FP8);
  if (em == EM_ROPE) nstl::count(NSTL_K_GEMM_FP8_ROPE);
  return 0;
}

bool big_ok(const nstl_gemm_args* a) {
  const int64_t big_tiles = (int64_t)((a->M + BIG - 1) / BIG) * ((a->N + BIG - 1) / BIG);
  return a->dtype == NSTL_BF16 && a->K % 64 == 0 && a->M >= BIG && a->N >= BIG && big_tiles >= 32 &&
         !getenv_small_gemm();
}

}  // namespace

namespace nstl {
int gemm4(const nstl_gemm_args* a, hipStream_t st, int* handled);                   // gemm4.hip
int gemm4_grouped(const nstl_gemm_args* args, int n, hipStream_t st, int* handled);  // gemm4.hip
}

extern "C" int nstl_gemm(const nstl_gemm_args* a, void* stream) {
  GemmParams p;
  if (int rc = make_params(a, p)) return rc;
  NSTL_CHECK_ARG(!a->sq_part, "nstl_gemm: sq_part is produced by nstl_gemm_grouped only");
  if (a->dtype == NSTL_FP8) return gemm_f8(a, p, (hipStream_t)stream);
  {  // full 256^2 tiles: the 4-wave persistent kernel (gemm4.hip); the rest below
    int handled = 0;
    if (int rc = nstl::gemm4(a, (hipStream_t)stream, &handled)) return rc;
    if (handled) return 0;
  }
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;

  // the 256x256 LDS-DMA kernel: bf16, K a multiple of its 64-deep K tile, and at
  // least 32 of its tiles (measured on the 228M step's shapes, tools/bench_gemm.py;
  // smaller/odd problems take the 128 kernel.  A 1024^2 dW split 16 ways on the
  // 256 kernel ties the 128 kernel split 8 ways: 60 vs 61 us, tools/bench_gemm_epi.py)
  const bool big = big_ok(a);
  NSTL_CHECK_ARG(!a->colsum_part || (big && a->epilogue == NSTL_EPI_DRELU_DROP && a->split_k <= 1 &&
                                      ring_epi_mode(a, p) == EM_DRELU),
                 "nstl_gemm: colsum_part needs the 256 kernel's dReLU epilogue (nstl_gemm_colsum_rows)");
  NSTL_CHECK_ARG(!a->relu_mask || nstl_gemm_relu_mask_words(a) > 0,
                 "nstl_gemm: relu_mask needs the 256 kernel's ReLU-dropout / dReLU epilogue (nstl_gemm_relu_mask_words)");
  const int BKe = big ? 64 : 128 / esz;
  int splits = a->split_k > 1 ? a->split_k : 1;
  if (splits > 1) {
    NSTL_CHECK_ARG(a->epilogue == NSTL_EPI_NONE || a->epilogue == NSTL_EPI_BIAS,
                   "nstl_gemm: split-K supports NONE/BIAS epilogues only");
    NSTL_CHECK_ARG(a->workspace != nullptr && a->workspace_bytes >= nstl_gemm_workspace_bytes(a->M, a->N, splits),
                   "nstl_gemm: split-K workspace too small");
    p.ws = (float*)a->workspace;
  }
  int chunk = (a->K + splits - 1) / splits;
  chunk = ((chunk + BKe - 1) / BKe) * BKe;
  splits = (a->K + chunk - 1) / chunk;
  p.k_chunk = chunk;
  if (splits == 1) p.ws = nullptr;

  hipStream_t st = (hipStream_t)stream;
  int rc = big ? launch_big(a, p, splits, st)
               : a->dtype == NSTL_BF16 ? launch_typed<bf16>(a, p, splits, st) : launch_typed<float>(a, p, splits, st);
  if (rc) return rc;
  if (p.ws != nullptr) {
    const int64_t total = (int64_t)a->M * a->N;
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, st, p.ws, splits, a->M, a->N, p.C, a->ldc,
                       p.c_f32, a->beta, a->epilogue == NSTL_EPI_BIAS ? a->bias : nullptr);
    NSTL_LAUNCH_CHECK("nstl_gemm splitk_reduce");
    nstl::count(NSTL_K_GEMM_SPLITK_REDUCE);
  }
  return 0;
}

extern "C" int nstl_gemm_grouped(const nstl_gemm_args* args, int n, void* stream) {
  NSTL_CHECK_ARG(args != nullptr && n >= 1 && n <= NSTL_GEMM_GROUP_MAX, "nstl_gemm_grouped: 1..%d problems (got %d)",
                 NSTL_GEMM_GROUP_MAX, n);
  for (int g = 0; g < n; ++g) {
    const nstl_gemm_args* a = args + g;
    GemmParams p;
    if (int rc = make_params(a, p)) return rc;
    NSTL_CHECK_ARG(a->dtype == NSTL_BF16 && a->K % 64 == 0 && a->M >= BIG && a->N >= BIG,
                   "nstl_gemm_grouped: problem %d is not a 256-kernel problem (bf16, M, N >= 256, K %% 64 == 0)", g);
    // no epilogue (the weight gradients), or bias + RoPE with one shared table
    // (the decoder's cross-attention k|v projections of every layer at once)
    NSTL_CHECK_ARG((a->epilogue == NSTL_EPI_NONE || a->epilogue == NSTL_EPI_BIAS_ROPE) &&
                       a->epilogue == args[0].epilogue && a->split_k <= 1 && !a->colsum_part && !a->relu_mask,
                   "nstl_gemm_grouped: problem %d: no epilogue or bias + RoPE (the same for all), no split-K", g);
    NSTL_CHECK_ARG(a->a_kmajor == args[0].a_kmajor && a->b_kmajor == args[0].b_kmajor &&
                       a->c_dtype == args[0].c_dtype && (a->beta != 0.f) == (args[0].beta != 0.f),
                   "nstl_gemm_grouped: problem %d differs in layout, output type or beta use", g);
    NSTL_CHECK_ARG(a->epilogue != NSTL_EPI_BIAS_ROPE ||
                       (a->rope_cos == args[0].rope_cos && a->rope_sin == args[0].rope_sin &&
                        a->rope_T == args[0].rope_T && a->rope_dim == args[0].rope_dim),
                   "nstl_gemm_grouped: problem %d: RoPE problems share one table (cos, sin, T, dim)", g);
    const int em = ring_epi_mode(a, p);
    NSTL_CHECK_ARG(em == EM_F32 || em == EM_BF16 || (em == EM_ROPE && a->epilogue == NSTL_EPI_BIAS_ROPE),
                   "nstl_gemm_grouped: f32 output, or bf16 without beta");
    NSTL_CHECK_ARG(!a->sq_part || em == EM_F32, "nstl_gemm_grouped: sq_part needs f32 output");
  }
  hipStream_t st = (hipStream_t)stream;
  {  // full tiles, beta 0: one launch of the 4-wave persistent kernel (gemm4.hip)
    int handled = 0;
    if (int rc = nstl::gemm4_grouped(args, n, st, &handled)) return rc;
    if (handled) return 0;
  }
  // anything else (partial tiles, beta != 0, K % 128 != 0, NSTL_GEMM4=0): one
  // 8-wave ring launch per problem, in order, whatever its tile count (the ring
  // epilogue writes sq_part, one slot per (tile, wave), as the grouped kernel did)
  for (int g = 0; g < n; ++g) {
    GemmParams p;
    if (int rc = make_params(args + g, p)) return rc;
    if (int rc = launch_big(args + g, p, 1, st)) return rc;
  }
  return 0;
}

extern "C" int nstl_gemm_colsum_rows(const nstl_gemm_args* a) {
  GemmParams p;
  if (a == nullptr || make_params(a, p) != 0) return 0;
  if (a->dtype == NSTL_FP8)  // the fp8 ring kernel's dReLU epilogue (same 128-row partial layout)
    return a->epilogue == NSTL_EPI_DRELU_DROP && a->split_k <= 1 && a->c_dtype == NSTL_BF16 &&
                   ring_epi_mode(a, p) == EM_DRELU ? (a->M + 127) / 128 : 0;
  if (!big_ok(a) || a->epilogue != NSTL_EPI_DRELU_DROP || a->split_k > 1) return 0;
  if (ring_epi_mode(a, p) != EM_DRELU) return 0;
  return (a->M + 127) / 128;
}

extern "C" int64_t nstl_gemm_relu_mask_words(const nstl_gemm_args* a) {
  GemmParams p;
  if (a == nullptr || make_params(a, p) != 0) return 0;
  if (a->dtype == NSTL_FP8) {
    const int em = ring_epi_mode(a, p);
    if (a->split_k > 1 || a->c_dtype != NSTL_BF16 || (em != EM_RELU_DROP && em != EM_DRELU)) return 0;
    return (int64_t)((a->M + 63) / 64) * 8 * ((a->N + 7) / 8);
  }
  if (!big_ok(a) || a->split_k > 1 || a->dtype != NSTL_BF16 || a->c_dtype != NSTL_BF16) return 0;
  const int em = ring_epi_mode(a, p);
  if (em != EM_RELU_DROP && em != EM_DRELU) return 0;
  return (int64_t)((a->M + 63) / 64) * 8 * ((a->N + 7) / 8);
}

#ifdef NSTL_STAMPS
// diagnostic build only (not declared in include/nstl.h): copy / clear the stamps
extern "C" int nstl_debug_gemm_stamps(unsigned long long* host, int64_t n) {
  n = std::min<int64_t>(n, (int64_t)STAMP_MAX * STAMP_W);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nstl_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" int nstl_debug_gemm_stamps_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_nstl_stamps)) != hipSuccess) return 1;
  return hipMemset(p, 0, sizeof(unsigned long long) * STAMP_MAX * STAMP_W) == hipSuccess ? 0 : 1;
}
#endif
