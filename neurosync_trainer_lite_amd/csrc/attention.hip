// Multi-head attention forward/backward for the NeuroSync Seq2Seq
// (replaces F.scaled_dot_product_attention, utils/model.py:126-127, and its
// autograd backward; RoPE (apply_rope_qk, :60-83) is applied to q/k by the
// projection epilogue, and rotated back here on dq/dk).
//
// Shapes are short: T <= 256 frames, dh = 64.  A whole (batch, head) key/value
// sequence fits in LDS, so there is no online softmax and no cross-workgroup
// reduction:
//   forward : workgroup = (b, h, 128 queries); each wave 16 queries; scores for
//             all keys live in MFMA accumulators (S^T layout); exact softmax;
//             P feeds P.V straight from the score registers (acc_frag).
//   backward: dQ kernel (workgroup = b, h, 128 queries) and dK/dV kernel
//             (b, h, 128 keys); scores recomputed from the saved LSE, dS / P^T
//             again used as register operands.
// K/V (forward, dQ) and Q/dO (dK/dV) arrive by LDS-DMA (global_load_lds_dwordx4,
// bank swizzle applied on the source address); a wave's own 16 rows come from
// global memory straight into MFMA fragments.  Dropout keep-mask: a counter
// hash of (b, h, query, key), or the bits the forward stored (mask_bits).
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
  int rope_fast;  // bf16 backward: RoPE^T angles recomputed with v_sin / v_cos instead of the tables
  int B, T, H, dh;
  float scale;
  uint32_t thresh; float inv_keep; uint64_t seed;
};

// 2^x as one v_exp_f32 (exp2f adds a denormal-range fix-up: 4 more vector
// instructions per call; every argument here is <= 0 and a probability below
// 2^-126 is 0 either way)
NSTL_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int N>
NSTL_DEV void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The 128-byte-row (bf16) K / V / Q / dO images of this file: 16-byte chunk c
// of row r at c ^ att_x(r).  They are read both ways: by rows (ds_read_b128, 16
// rows at one chunk per lane group) and transposed (ds_read_b64_tr_b16, 8 rows x
// 32 bytes per 32-lane group).  ImgK<128>'s x = (r >> 1) & 7 serves the row reads
// but puts rows r and r + 2 of a transposed read on the same banks (2 LDS cycles
// per 32-lane group instead of 1: the backward's largest bank-conflict term).
// This x -- row bit 1 to chunk bit 2, row bit 2 to chunk bit 1 -- is
// conflict-free for both (checked for every read pattern of the kernels below by
// a bank simulation of the ds_read_b128 / ds_read_b64_tr_b16 lane groups).
// 256-byte rows (f32) keep ImgK<256>.
NSTL_DEV int att_x(int row) { return (((row >> 2) & 1) << 1) | (((row >> 1) & 1) << 2); }
template <int RB> struct ImgAtt {
  static NSTL_DEV int off(int row, int byte) {
    const int chunk = byte >> 4;
    const int x = RB == 128 ? att_x(row) : (row & 15);
    return row * RB + (((chunk ^ x) << 4) | (byte & 15));
  }
};

// LDS-DMA rows [0, nrows) of a (b, h) slice (64 elements per row) into an
// ImgAtt<RB> image.  One wave instruction moves 1 KB = 1024/RB rows; the image
// swizzle is applied to the per-lane source chunk.
template <int RB, int NW = NT / 64>
NSTL_DEV void dma_rows(char* img, const char* g, int64_t ld_bytes, int nrows, int wave, int lane) {
  constexpr int RPK = 1024 / RB, CPR = RB / 16;
  const int ninst = nrows / RPK;
  for (int q = wave; q < ninst; q += NW) {
    const int row = q * RPK + lane / CPR, pc = lane % CPR;
    const int x = RB == 128 ? att_x(row) : (row & 15);
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

// dropout element index: query-major, so the key pair (k, k+1) of one query
// shares a hash (the MFMA kernels hold 4 consecutive keys of a query per lane)
NSTL_DEV uint64_t drop_idx(int bh, int T, int q, int k) { return ((uint64_t)bh * T + q) * T + k; }

// Stored keep bits (MFMA path): one 64-bit word per (query tile qt, key tile kt,
// key % 4) of a head, bit 16 * ((key % 16) / 4) + query % 16 -- the ballot of
// one score register r over a wave in the forward / dQ layout (lane 16g + c:
// query c, key 4g + r).  A head's words are [qt][kt][4] (T*T/64 of them).
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

// ---------------------------------------------------------------------------
// Register-operand layout.  Scores are computed TRANSPOSED where the next
// product reduces over them: mma16(acc, X, Y) gives lane (g, c = lane & 15)
// the elements (row 4g + r, column c), so with X = keys and Y = queries a lane
// owns keys 16kt + 4g + r of ITS query c -- exactly what it must supply as the
// A operand (row c) of a product that sums over keys.  Two score registers
// (tiles 2j, 2j+1) form one A fragment whose 8 reduction slots are the keys
// {32j + 4g + 0..3, 32j + 16 + 4g + 0..3}; the B operand is read from its LDS
// image in that same order (frag_col2), so P / dS never go through LDS.
template <typename T> NSTL_DEV typename FragT<T>::type acc_frag(const f32x4& a, const f32x4& b);
template <> NSTL_DEV bf16x8 acc_frag<bf16>(const f32x4& a, const f32x4& b) {
  return (bf16x8){(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}
template <> NSTL_DEV f32x8 acc_frag<float>(const f32x4& a, const f32x4& b) {
  return (f32x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// column col16 + (lane & 15) of an image whose rows are the reduction index, rows
// r0 + 4g + 0..3 then r0 + 16 + 4g + 0..3 (acc_frag's order): two gfx950
// transpose reads (bf16) / eight element reads (f32)
template <class Img>
NSTL_DEV void frag_col2(bf16x8& f, const char* img, int col16, int r0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int byte = (col16 + 4 * p) * 2;
  const lds_char* base = (const lds_char*)img;
  s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + Img::off(r0 + 4 * g + q, byte)));
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + Img::off(r0 + 16 + 4 * g + q, byte)));
  const bf16x4 b0 = __builtin_bit_cast(bf16x4, v0), b1 = __builtin_bit_cast(bf16x4, v1);
  f = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
}
template <class Img>
NSTL_DEV void frag_col2(f32x8& f, const char* img, int col16, int r0, int lane) {
  const int g = lane >> 4, byte = (col16 + (lane & 15)) * 4;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = *(const float*)(img + Img::off(r0 + 4 * g + (j & 3) + 16 * (j >> 2), byte));
}

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

// four consecutive elements of a row: one 8-byte (bf16) / 16-byte (f32) store
template <typename T> NSTL_DEV void store4(T* dst, const f32x4& v);
template <> NSTL_DEV void store4<bf16>(bf16* dst, const f32x4& v) {
  *(bf16x4*)dst = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}
template <> NSTL_DEV void store4<float>(float* dst, const f32x4& v) { *(f32x4*)dst = v; }

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

// ----------------------------------------------------------------------------
// Forward: one workgroup of 8 waves per (b, h) and 128 queries (all of T=128),
// so K and V are staged once per (b, h) by LDS-DMA; each wave owns 16 queries,
// loaded straight from global memory as MFMA fragments.  S^T = K Q^T in
// accumulators, exact softmax over the keys (a lane holds 4*T/16 of its
// query's scores; the rest are in the lanes of the same column, 2 shuffles),
// dropout, then O = P V with P taken from the score registers (acc_frag).
constexpr int FWD_NT = 512, FWD_QB = 16 * FWD_NT / 64;

// One wave's 16 queries q0 .. q0+15 of head bh (tokens from tok0, head column
// h*DH) against all keys of the K / V images: scores, exact softmax, dropout
// (keep bits to p.mask), O and the LSE.  fq: the wave's Q fragments.
// ImgAtt<128> fragment reads as inline asm (bf16): with a prefetch DMA in flight
// into the other buffer the compiler would put vmcnt(0) in front of its own LDS
// reads (it cannot tell the images apart), draining the prefetch; the caller
// orders them with an explicit lgkmcnt(0) + sched_barrier before the MFMAs.
NSTL_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p; }
typedef int i32x4a __attribute__((ext_vector_type(4)));
typedef int i32x2a __attribute__((ext_vector_type(2)));
NSTL_DEV void asm_row128(bf16x8& f, const char* img, int row, int r) {
  i32x4a v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(img + ImgAtt<128>::off(row, r * 2))));
  f = __builtin_bit_cast(bf16x8, v);
}
NSTL_DEV void asm_col2_128(bf16x8& f, const char* img, int col16, int r0, int lane) {  // frag_col2<ImgAtt<128>>
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int byte = (col16 + 4 * pp) * 2;
  i32x2a v0, v1;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v0) : "v"(lds_addr(img + ImgAtt<128>::off(r0 + 4 * g + q, byte))));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v1) : "v"(lds_addr(img + ImgAtt<128>::off(r0 + 16 + 4 * g + q, byte))));
  const bf16x4 b0 = __builtin_bit_cast(bf16x4, v0), b1 = __builtin_bit_cast(bf16x4, v1);
  f = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
}
NSTL_DEV void lgkm_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// rows [tok0, tok0 + T) of a head's 64 columns (h * DH) of a bf16 [*, ld] operand
// as a buffer resource (host-checked: T * ld * 2 < 2^31)
NSTL_DEV __amdgpu_buffer_rsrc_t head_rsrc(const char* base, int64_t ld, int64_t tok0, int h, int T) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (tok0 * ld + h * DH) * 2), 0, (int)((uint32_t)T * ld * 2),
                                           0x00020000);
}
struct NoHook {
  NSTL_DEV void operator()() const {}
};

// AR: the Q fragments come from the wave's 16-row Q image Qw (ImgAtt<128>) and
// every K / V / Q fragment read is inline asm (bf16 only; the persistent kernel);
// after_qk() runs once the wave is done with its Q image (the S products)
template <typename T, int NKT, bool AR = false, typename Hook = NoHook>
NSTL_DEV void fwd_queries(const AttnParams& p, const char* Kimg, const char* Vimg,
                          const typename FragT<T>::type (&fq_in)[2], const char* Qw, int bh, int h, int64_t tok0,
                          int q0, int lane, Hook after_qk = Hook()) {
  typedef typename FragT<T>::type Frag;
  constexpr int RBK = DH * (int)sizeof(T);
  typedef ImgAtt<RBK> Img;
  constexpr int nkt = NKT;
  const int T_ = p.T, g = lane >> 4, c = lane & 15;
  // s[kt][r] = score(query q0 + c, key 16kt + 4g + r)
  f32x4 s[NKT];
  if constexpr (AR) {
    static_assert(sizeof(T) == 2 && NKT % 2 == 0, "asm reads: bf16");
    Frag fq[2];
    asm_row128(fq[0], Qw, c, 8 * g);
    asm_row128(fq[1], Qw, c, 32 + 8 * g);
#pragma unroll
    for (int kt = 0; kt < NKT; kt += 2) {  // two key tiles (4 reads) per wait
      Frag fk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) asm_row128(fk[u], Kimg, (kt + (u >> 1)) * 16 + c, 32 * (u & 1) + 8 * g);
      lgkm_fence();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        s[kt + u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        mma16(s[kt + u], fk[2 * u], fq[0]);
        mma16(s[kt + u], fk[2 * u + 1], fq[1]);
      }
    }
    after_qk();
  } else {
    const Frag(&fq)[2] = fq_in;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (kt < nkt) {
        Frag fk;
        frag_row<Img>(fk, Kimg, kt * 16 + c, 8 * g);
        mma16(s[kt], fk, fq[0]);
        frag_row<Img>(fk, Kimg, kt * 16 + c, 32 + 8 * g);
        mma16(s[kt], fk, fq[1]);
      }
    }
  }
  const float c2 = p.scale * LOG2E;
  float m = -INFINITY;
  float sum = 0.f;
  if constexpr (sizeof(T) == 2) {
    // bf16: the max as two v_max3 per key tile; 2^(s*c2 - m*c2) as packed FMAs
    // (one per two scores, instead of a subtract and a multiply per score) and
    // the row sum as packed adds over two partial sums
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      if (kt < nkt) m = fmaxf(fmaxf(m, fmaxf(fmaxf(s[kt][0], s[kt][1]), s[kt][2])), s[kt][3]);
    m = max_xor16(m);
    m = max_xor32(m);
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 c2v = {c2, c2}, nmc = {-m * c2, -m * c2};
    f32x2 sum2 = {0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 x = __builtin_elementwise_fma((f32x2){s[kt][r], s[kt][r + 1]}, c2v, nmc);
          const f32x2 e = {fast_exp2(x[0]), fast_exp2(x[1])};
          s[kt][r] = e[0];
          s[kt][r + 1] = e[1];
          sum2 += e;
        }
      }
    sum = sum2[0] + sum2[1];
  } else {
    // f32 (parity mode) keeps (s - m)*c2: s - m is exact near the max, where the
    // rounded m*c2 of the FMA form would cancel (the fp32 gradient norm moved by 1e-4)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      if (kt < nkt) m = fmaxf(fmaxf(fmaxf(m, s[kt][0]), fmaxf(s[kt][1], s[kt][2])), s[kt][3]);
    m = max_xor16(m);
    m = max_xor32(m);
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = fast_exp2((s[kt][r] - m) * c2);
          s[kt][r] = e;
          sum += e;
        }
      }
  }
  sum = sum_xor16(sum);
  sum = sum_xor32(sum);
  if (p.thresh) {
    // dropout on P: keys (r, r+1) of this lane's query share one hash.  The keep
    // compare is an SGPR lane mask already -- the ballot of (kt, r) -- and lane
    // kt*4 + r takes it by v_writelane (the select-by-lane-index form cost ~7
    // vector instructions per ballot).  The hashes go first, all of them (their
    // multiplies interleave); then one key tile's compares, selects and ballots
    // at a time (sched_barrier): left free, the compiler formed all 32 ballot
    // masks before the first v_writelane and spilled SGPRs into VGPR lanes.
    const int q = q0 + c;
    // pair index of drop_idx(bh, T, q, 4g) (even): 32-bit, checked by the launcher
    const uint32_t pair0 = ((uint32_t)bh * T_ + q) * (uint32_t)(T_ >> 1) + 2 * g;
    const uint32_t st = nstl_seed_term(p.seed);
    uint32_t hs[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      hs[kt][0] = nstl_pair_hash32(st, pair0 + kt * 8);
      hs[kt][1] = nstl_pair_hash32(st, pair0 + kt * 8 + 1);
    }
    uint32_t mlo = 0, mhi = 0;  // lane kt*4 + r: keep bits of (kt, r)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
        const uint32_t h0 = hs[kt][0], h1 = hs[kt][1];
        const bool k[4] = {(h0 & 0xFFFFu) >= p.thresh, (h0 >> 16) >= p.thresh, (h1 & 0xFFFFu) >= p.thresh,
                           (h1 >> 16) >= p.thresh};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kt][r] = k[r] ? s[kt][r] : 0.f;  // 1/(1-p): in the normalisation
          // in the compare's own block: the ballot IS its SGPR mask (under a branch
          // the compiler rebuilds the mask from a materialised bool)
          const uint64_t bal = __builtin_amdgcn_ballot_w64(k[r]);
          mlo = nstl_writelane_i32((int)(uint32_t)bal, kt * 4 + r, (int)mlo);
          mhi = nstl_writelane_i32((int)(uint32_t)(bal >> 32), kt * 4 + r, (int)mhi);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (p.mask && lane < nkt * 4) p.mask[mask_word(bh, nkt, q0 >> 4, 0, 0) + lane] = ((uint64_t)mhi << 32) | mlo;
  }
  // O^T = V^T P^T over 32-key chunks (V^T the A operand, the score registers
  // the B operand): o[dt][r] = O(query q0 + c, d = 16dt + 4g + r), so a lane
  // holds 4 consecutive dims of ITS query, whose softmax sum it already has, and
  // stores them straight from registers (no LDS round trip).
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NKT / 2; ++j) {
    const Frag fp = acc_frag<T>(s[2 * j], s[2 * j + 1]);
    if constexpr (AR) {
      Frag fv[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) asm_col2_128(fv[dt], Vimg, dt * 16, 32 * j, lane);
      lgkm_fence();
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) mma16(o[dt], fv[dt], fp);
    } else {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        Frag fv;
        frag_col2<Img>(fv, Vimg, dt * 16, 32 * j, lane);
        mma16(o[dt], fv, fp);
      }
    }
  }
  // normalise (dropout's 1/(1-p) applied to O instead of P) and store
  const float inv = (p.thresh ? p.inv_keep : 1.f) * __builtin_amdgcn_rcpf(sum);
  if constexpr (AR) {  // the head's O rows as a buffer: 32-bit offsets (one store per dt, as store4)
    const __amdgpu_buffer_rsrc_t ro = head_rsrc(p.o, p.o_ld, tok0, h, T_);
    const uint32_t ob = ((uint32_t)(q0 + c) * (uint32_t)p.o_ld + 4 * g) * 2;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 x = o[dt] * inv;
      const bf16x4 b = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2a, b), ro, ob + 32 * dt, 0, 0);
    }
  } else {
    T* orow = (T*)p.o + (tok0 + q0 + c) * p.o_ld + h * DH + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store4<T>(orow + 16 * dt, o[dt] * inv);
  }
  if (g == 0) p.lse[(int64_t)bh * T_ + q0 + c] = m * p.scale + logf(sum);
}

// NKT = T/16 key tiles (score registers sized to T); T <= 128: 6 waves per SIMD (3
// workgroups per CU) without spills; longer T: 4 / 3
template <typename T, int NKT>
__global__ __launch_bounds__(FWD_NT, NKT <= 8 ? 6 : (NKT <= 12 ? 4 : 3)) void attn_fwd_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;   // 128 (bf16) / 256 (f32)
  constexpr int NW = FWD_NT / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T;
  char* Kimg = smem;
  char* Vimg = Kimg + T_ * RBK;

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int qb0 = blockIdx.x * FWD_QB;
  const int nq = min(FWD_QB, T_ - qb0);
  const int64_t tok0 = (int64_t)b * T_;

  dma_rows<RBK, NW>(Kimg, p.k + (tok0 * p.k_ld + h * DH) * ESZ, p.k_ld * ESZ, T_, w, lane);
  dma_rows<RBK, NW>(Vimg, p.v + (tok0 * p.v_ld + h * DH) * ESZ, p.v_ld * ESZ, T_, w, lane);
  const int q0 = qb0 + w * 16;  // this wave's first query
  const bool act = w * 16 < nq;
  Frag fq[2];
  if (act) {
    const T* qrow = (const T*)p.q + (tok0 + q0 + c) * p.q_ld + h * DH;
    gload_frag<T>(fq[0], qrow, 8 * g);
    gload_frag<T>(fq[1], qrow, 32 + 8 * g);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!act) return;
  fwd_queries<T, NKT>(p, Kimg, Vimg, fq, nullptr, bh, h, tok0, q0, lane);
}

// Persistent form for the production shape (bf16, T = 128: one workgroup's 8
// waves cover a head's 128 queries).  The one-shot grid above runs 2048 (b, h)
// workgroups, 3 per CU, each of which loads its K / V / Q, waits, computes and
// stores: every workgroup pays a full memory latency with nothing of its own to
// overlap, and the 2.7 rounds of workgroups leave the last one a third empty.
// Here a grid of 2 workgroups per CU walks the heads (item = blockIdx.x + i * G)
// with two K / V image buffers and one Q image (2 KB per wave), all filled by
// LDS-DMA: the next head's K / V are issued before the current head is
// computed, a wave's next Q rows as soon as its S products no longer need its
// Q image, and the O / LSE / keep-bit stores stay in flight across the next
// head's wait (the counted vmcnt retires only the loads issued before them).
// No operand goes to VGPRs by a load the compiler tracks, so it adds no wait
// of its own.  LDS: 2 x 32 KB + 16 KB = 80 KB, two workgroups per CU.
// Per wave and head: 4 K / V + 2 Q DMA, 4 O + 1 LSE (+ 1 keep-bit word with
// MK) stores.
constexpr int PF_T = 128, PF_IMG = PF_T * DH * 2, PF_KV = 4;
constexpr size_t PF_LDS = 2 * 2 * (size_t)PF_IMG + 8 * 2048;
// raw barrier: __syncthreads() would also wait for every outstanding memory
// operation (vmcnt(0)), i.e. for the next head's prefetch
NSTL_DEV void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
NSTL_DEV void dma1k(const char* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
}
template <bool MK>
__global__ __launch_bounds__(FWD_NT, 4) void attn_fwd_persist_kernel(AttnParams p, int nitems) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PF_STORES = MK ? 6 : 5;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  char* const Qw = smem + 4 * PF_IMG + w * 2048;
  // per-lane byte offsets inside a head's slab, once (ImgAtt<128> swizzle on the
  // source chunk, as dma_rows): the wave's two 1 KB pieces of the K and V
  // images (rows 8(w + 8u) ..) and of its own Q rows (16w + 8u ..)
  uint32_t offk[2], offv[2], offq[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int row = (w + 8 * u) * 8 + (lane >> 3), lc = (lane & 7) ^ att_x(row);
    offk[u] = (uint32_t)(row * p.k_ld * 2 + lc * 16);
    offv[u] = (uint32_t)(row * p.v_ld * 2 + lc * 16);
    const int qr = 8 * u + (lane >> 3), qc = (lane & 7) ^ att_x(qr);
    offq[u] = (uint32_t)((w * 16 + qr) * p.q_ld * 2 + qc * 16);
  }
  auto head = [&](int it, const char* base, int64_t ld) {
    const int b = it / p.H, h = it % p.H;
    return base + ((int64_t)b * PF_T * ld + h * DH) * 2;
  };
  // heads as buffer resources (base in SGPRs, the per-lane offsets above as 32-bit
  // voffsets: no 64-bit address per piece)
  auto hbuf = [&](int it, const char* base, int64_t ld) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)head(it, base, ld), 0, (int)((uint32_t)PF_T * ld * 2), 0x00020000);
  };
  auto dma_buf = [](__amdgpu_buffer_rsrc_t r, uint32_t off, char* dst) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, off, 0, 0, 0);
  };
  auto issue_kv = [&](int it, int buf) {
    const __amdgpu_buffer_rsrc_t rk = hbuf(it, p.k, p.k_ld), rv = hbuf(it, p.v, p.v_ld);
    char* img = smem + buf * 2 * PF_IMG;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      dma_buf(rk, offk[u], img + (w + 8 * u) * 1024);
      dma_buf(rv, offv[u], img + PF_IMG + (w + 8 * u) * 1024);
    }
  };
  auto issue_q = [&](int it) {
    const __amdgpu_buffer_rsrc_t rq = hbuf(it, p.q, p.q_ld);
#pragma unroll
    for (int u = 0; u < 2; ++u) dma_buf(rq, offq[u], Qw + u * 1024);
  };
  int it = blockIdx.x;
  if (it >= nitems) return;
  issue_kv(it, 0);
  issue_q(it);
  const bf16x8 nofq[2] = {};
  for (int i = 0; it < nitems; ++i, it += G) {
    const int buf = i & 1;
    const bool next = it + G < nitems;
    if (next) issue_kv(it + G, buf ^ 1);  // buffer of head i-1: free since the barrier ending it
    // retire head i's K / V / Q: younger are head i-1's stores (i > 0) and head i+1's K / V
    if (i == 0) {
      if (next) vmcnt_wait<PF_KV>();
      else vmcnt_wait<0>();
    } else {
      if (next) vmcnt_wait<PF_KV + PF_STORES>();
      else vmcnt_wait<PF_STORES>();
    }
    raw_barrier();  // every wave's DMA share of head i has landed
    const int b = it / p.H, h = it % p.H;
    const char* img = smem + buf * 2 * PF_IMG;
    auto after_qk = [&]() {
      if (next) issue_q(it + G);  // this wave's own Q image: no other wave reads it
    };
    fwd_queries<bf16, PF_T / 16, true>(p, img, img + PF_IMG, nofq, Qw, it, h, (int64_t)b * PF_T, w * 16, lane,
                                       after_qk);
    raw_barrier();  // every wave is done reading buffer `buf`
  }
}

// RoPE^T: rotate (row t, col d) accumulator elements back by -theta
// partner element of a RoPE pair: lane c <-> c ^ 1 (DPP quad_perm [1,0,3,2], no LDS)
NSTL_DEV float swap_pair(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
// RoPE^T over a lane's 16 x 64 tile elements v[dt][r] = (row0 + r, d = 16 dt + c):
// the 32 table reads are issued together (rope_tab), the pair swaps are DPP
// moves (the per-element form waited on one ds_bpermute and two table reads at
// a time).  Tables [T][RS] with row stride RS floats (32 in global memory, 36
// in the fused kernel's LDS copy: the rows 4g + r of a wave's four lane groups
// then fall on distinct banks).  The sin table comes out with the lane's sign
// folded in (ts = -sin on odd lanes), so every element is x cos + partner ts:
// one multiply and one FMA.  rope_apply needs every lane of the wave active.
template <int RS>
NSTL_DEV void rope_tab(float (&tc)[4][4], float (&ts)[4][4], int row0, int c, const float* cs, const float* sn) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int i = (row0 + r) * RS + dt * 8 + (c >> 1);
      tc[dt][r] = cs[i];
      ts[dt][r] = (c & 1) ? -sn[i] : sn[i];
    }
}
NSTL_DEV void rope_apply(float (&v)[4][4], const float (&tc)[4][4], const float (&ts)[4][4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const float x = v[dt][r], partner = swap_pair(x);
      v[dt][r] = fmaf(partner, ts[dt][r], x * tc[dt][r]);
    }
}
// The same cos / sin values recomputed: angle = float(t) * inv_freq_i as
// rotation_tables() forms it (f32 product; inv_freq by the hardware exp), then
// the hardware sin / cos (v_sin_f32 / v_cos_f32 on angle / 2pi).  Against the
// f32 tables the error is ~1e-6 absolute, far below the bf16 rounding of the
// dQ / dK it rotates.
// The angle goes to v_sin / v_cos in revolutions, t * (inv_freq / 2pi), with the
// lane's sign folded into the factor (sin is odd, cos even): one multiply per
// angle instead of three (angle, 1/2pi for each of sin and cos, the sign).
NSTL_DEV void rope_tab_fast(float (&tc)[4][4], float (&ts)[4][4], int row0, int c) {
  const float sgn_rev = ((c & 1) ? -1.f : 1.f) * 0.15915494309189535f;  // +-1/(2pi)
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const float two_i = (float)(2 * (dt * 8 + (c >> 1)));
    const float inv_freq = __expf(-9.21034049987793f * two_i / (float)DH);  // f32(ln 10000)
    const float f = inv_freq * sgn_rev;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = (float)(row0 + r) * f;
      ts[dt][r] = __builtin_amdgcn_sinf(a);
      tc[dt][r] = __builtin_amdgcn_cosf(a);
    }
  }
}
// fast: the angles recomputed (rope_tab_fast) instead of per-element table reads
// from global memory (16 dependent L2 round trips per wave at the end of the split
// kernels; bf16 only -- the f32 parity mode keeps the tables' exact values)
NSTL_DEV void rope_back_tile(float (&v)[4][4], int row0, int c, const float* cs, const float* sn, bool fast = false) {
  float tc[4][4], ts[4][4];
  if (fast) rope_tab_fast(tc, ts, row0, c);
  else rope_tab<DH / 2>(tc, ts, row0, c, cs, sn);
  rope_apply(v, tc, ts);
}

// Bias gradients fused into the backward stores: column sums of a wave's stored
// 16 x 64 tile (rounded to T, as colsum() of the stored tensor would see it) go
// to red[w][64]; the LAST wave to finish (an LDS arrival counter, no barrier,
// so early waves leave at once) adds the block's waves in fixed order and
// writes one partial row: deterministic, no float atomics.
template <typename T>
NSTL_DEV void wave_colsum16x64(const float (&v)[4][4], float* red, int w, int lane) {
  if constexpr (sizeof(T) == 2) {
    // bf16: one v_mfma_f32_16x16x16_bf16 per 16 columns, ones x tile: the lane's
    // four rows 4g + r of column 16 dt + c are exactly its B operand, and every
    // result row is the column sum of the stored (bf16) values -- lane c of lane
    // group 0 holds column 16 dt + c, no cross-lane reduction
    const s16x4 ones = __builtin_bit_cast(s16x4, (bf16x4){(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f});
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x4 x = {(bf16)v[dt][0], (bf16)v[dt][1], (bf16)v[dt][2], (bf16)v[dt][3]};
      const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ones, __builtin_bit_cast(s16x4, x),
                                                                (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if (lane < 16) red[w * 64 + dt * 16 + lane] = d[0];
    }
    return;
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) cs += to_f32(from_f32<T>(v[dt][r]));
    cs = sum_xor16(cs);
    cs = sum_xor32(cs);
    if (lane < 16) red[w * 64 + dt * 16 + lane] = cs;
  }
}
NSTL_DEV bool last_to_arrive(unsigned* cnt, int nw, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's red[] writes are done
  unsigned old = 0;
  if (lane == 0) old = atomicAdd(cnt, 1u);
  return __shfl(old, 0) == (unsigned)(nw - 1);
}
NSTL_DEV void wave_sum_out(const float* red, int nw, float* out, int lane) {
  float cs = 0.f;
  for (int k = 0; k < nw; ++k) cs += red[k * 64 + lane];
  out[lane] = cs;
}

// ---------------------------------------------------------------------------
// Backward, as two kernels (8 waves, 128 rows: all of T=128, so each (b, h)
// operand is staged once):
//   attn_bwd_dq : workgroup = (b, h, 128 queries); K, V of (b, h) in LDS; a wave
//                 owns 16 queries (fragments from global): D = rowsum(dO * O)
//                 (also written to p.dsum for the second kernel), S^T and dP^T
//                 over all keys, dS^T in registers -> dQ = dS K (RoPE^T).
//   attn_bwd_dkv: workgroup = (b, h, 128 keys); Q, dO of (b, h) in LDS; a wave
//                 owns 16 keys: S and dP (query rows), P^T / dS^T in registers
//                 -> dV = P_drop^T dO, dK = dS^T Q (RoPE^T).
constexpr int BWD_NT = 512, BWD_ROWS = 16 * BWD_NT / 64;  // 8 waves, 128 rows

// (BWD_NT, 6): 6 waves per SIMD = 3 workgroups per CU (bf16: 78 VGPRs, no spill)
// DM: dropout mode as in attn_bwd_fused_kernel (0 none, 1 stored bits, 2 re-hash)
template <typename T, int DM>
__global__ __launch_bounds__(BWD_NT, 6) void attn_bwd_dq_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;
  typedef ImgAtt<RBK> Img;
  constexpr int NW = BWD_NT / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Kimg = smem;
  char* Vimg = Kimg + T_ * RBK;
  // T % 128 == 0 (every wave active): the output staging reuses the K image after
  // a barrier (bwd_lds_bytes), so T = 256 fits two workgroups per CU
  const bool alias = T_ % BWD_ROWS == 0;
  char* scratch = alias ? smem : Vimg + T_ * RBK;  // [NW][16][RBK] output staging
  float* red = (float*)(alias ? Vimg + T_ * RBK : scratch + NW * 16 * RBK);  // [NW][64] bias partials
  unsigned* arrived = (unsigned*)(red + 2 * NW * 64);

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;
  const int q0 = blockIdx.x * BWD_ROWS + w * 16;
  dma_rows<RBK, NW>(Kimg, p.k + (tok0 * p.k_ld + h * DH) * ESZ, p.k_ld * ESZ, T_, w, lane);
  dma_rows<RBK, NW>(Vimg, p.v + (tok0 * p.v_ld + h * DH) * ESZ, p.v_ld * ESZ, T_, w, lane);
  const bool act = q0 < T_;
  Frag fq[2], fo[2];
  float lq = 0.f, dqv = 0.f;  // LSE (log2 units) and D of this lane's query q0 + c
  if (act) {
    const int qr = q0 + c;
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
    float dpart = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) dpart += to_f32(fo[u][e]) * to_f32(oo[u][e]);
    dpart = sum_xor16(dpart);
    dpart = sum_xor32(dpart);
    if (g == 0) p.dsum[(int64_t)bh * T_ + qr] = dpart;
    dqv = dpart;
    lq = p.lse[(int64_t)bh * T_ + qr] * LOG2E;
  }
  if (tid == 0) *arrived = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* bias_row = p.dbias ? p.dbias + (int64_t)(b * gridDim.x + blockIdx.x) * 3 * p.H * DH : nullptr;
  if (!act) {
    if (bias_row) {
      red[w * 64 + lane] = 0.f;
      if (last_to_arrive(arrived, NW, lane)) wave_sum_out(red, NW, bias_row + h * DH, lane);
    }
    return;
  }

  const float c2 = p.scale * LOG2E;
  // stored keep bits of this wave's 16 queries: lane kt*4 + r holds word (kt, r)
  uint64_t mword = 0;
  if (DM == 1 && lane < nkt * 4) mword = p.mask[mask_word(bh, nkt, q0 >> 4, 0, 0) + lane];
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nkt / 2; ++j) {  // 32-key chunks
    f32x4 dsv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kt = 2 * j + u;
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      Frag fb;
      frag_row<Img>(fb, Kimg, kt * 16 + c, 8 * g);
      mma16(sc, fb, fq[0]);
      frag_row<Img>(fb, Kimg, kt * 16 + c, 32 + 8 * g);
      mma16(sc, fb, fq[1]);
      frag_row<Img>(fb, Vimg, kt * 16 + c, 8 * g);
      mma16(dp, fb, fo[0]);
      frag_row<Img>(fb, Vimg, kt * 16 + c, 32 + 8 * g);
      mma16(dp, fb, fo[1]);
      // sc[r] / dp[r]: S^T / dP^T at (key 16kt + 4g + r, query q0 + c)
      bool keep[4] = {true, true, true, true};
      if constexpr (DM == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) keep[r] = (readlane64(mword, kt * 4 + r) >> lane) & 1;
      } else if constexpr (DM == 2) {
        const uint64_t idx = drop_idx(bh, T_, q0 + c, kt * 16 + 4 * g);
        nstl_keep2(p.seed, idx, p.thresh, keep[0], keep[1]);
        nstl_keep2(p.seed, idx + 2, p.thresh, keep[2], keep[3]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = fast_exp2(sc[r] * c2 - lq);
        float dpd = dp[r];
        if constexpr (DM != 0) dpd = keep[r] ? dpd * p.inv_keep : 0.f;
        dsv[u][r] = pv * (dpd - dqv);
      }
    }
    const Frag fa = acc_frag<T>(dsv[0], dsv[1]);  // dS, row = query q0 + c
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      Frag fb;
      frag_col2<Img>(fb, Kimg, dt * 16, 32 * j, lane);
      mma16(dq[dt], fa, fb);
    }
  }
  float vq[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vq[dt][r] = dq[dt][r] * p.scale;
  if (p.rope_q) rope_back_tile(vq, q0 + 4 * g, c, p.rope_cos, p.rope_sin, sizeof(T) == 2 && p.rope_fast);
  if (alias) __syncthreads();  // every wave is done with the K / V images
  store_tile16x64<T>(vq, scratch + w * 16 * RBK, p.dq + ((tok0 + q0) * p.dq_ld + h * DH) * ESZ, p.dq_ld, lane);
  if (bias_row) {
    wave_colsum16x64<T>(vq, red, w, lane);
    if (last_to_arrive(arrived, NW, lane)) wave_sum_out(red, NW, bias_row + h * DH, lane);
  }
}

template <typename T, int DM>
__global__ __launch_bounds__(BWD_NT) void attn_bwd_dkv_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int ESZ = (int)sizeof(T);
  constexpr int RBK = DH * ESZ;
  typedef ImgAtt<RBK> Img;
  constexpr int NW = BWD_NT / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Qimg = smem;
  char* Dimg = Qimg + T_ * RBK;
  float* lse_s = (float*)(Dimg + T_ * RBK);
  float* dq_s = lse_s + T_;
  const bool alias = T_ % BWD_ROWS == 0;           // as in attn_bwd_dq_kernel: staging over the Q image
  char* scratch = alias ? smem : (char*)(dq_s + T_);  // [NW][16][RBK] output staging
  float* red = alias ? dq_s + T_ : (float*)(scratch + NW * 16 * RBK);  // [2][NW][64] bias partials
  unsigned* arrived = (unsigned*)(red + 2 * NW * 64);

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;
  const int k0 = blockIdx.x * BWD_ROWS + w * 16;
  dma_rows<RBK, NW>(Qimg, p.q + (tok0 * p.q_ld + h * DH) * ESZ, p.q_ld * ESZ, T_, w, lane);
  dma_rows<RBK, NW>(Dimg, p.dout + (tok0 * p.dout_ld + h * DH) * ESZ, p.dout_ld * ESZ, T_, w, lane);
  for (int i = tid; i < T_; i += BWD_NT) {
    lse_s[i] = p.lse[(int64_t)bh * T_ + i] * LOG2E;
    dq_s[i] = p.dsum[(int64_t)bh * T_ + i];
  }
  const bool act = k0 < T_;
  Frag fk[2], fv[2];
  if (act) {
    const int kr = k0 + c;
    const T* krow = (const T*)p.k + (tok0 + kr) * p.k_ld + h * DH;
    const T* vrow = (const T*)p.v + (tok0 + kr) * p.v_ld + h * DH;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gload_frag<T>(fk[u], krow, 32 * u + 8 * g);
      gload_frag<T>(fv[u], vrow, 32 * u + 8 * g);
    }
  }
  if (tid == 0) *arrived = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* bias_row = p.dbias ? p.dbias + (int64_t)(b * gridDim.x + blockIdx.x) * 3 * p.H * DH : nullptr;
  if (!act) {
    if (bias_row) {
      red[w * 64 + lane] = 0.f;
      red[NW * 64 + w * 64 + lane] = 0.f;
      if (last_to_arrive(arrived, NW, lane)) {
        wave_sum_out(red, NW, bias_row + p.H * DH + h * DH, lane);
        wave_sum_out(red + NW * 64, NW, bias_row + 2 * p.H * DH + h * DH, lane);
      }
    }
    return;
  }

  const float c2 = p.scale * LOG2E;
  // stored keep bits for this wave's 16 keys: lane 4*qt + r holds word (qt, k0/16, r)
  uint64_t mword = 0;
  if (DM == 1 && (lane >> 2) < nkt) mword = p.mask[mask_word(bh, nkt, lane >> 2, k0 >> 4, lane & 3)];
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nkt / 2; ++j) {  // 32-query chunks
    f32x4 pdv[2], dsv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qt = 2 * j + u;
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
      Frag fb;
      frag_row<Img>(fb, Qimg, qt * 16 + c, 8 * g);
      mma16(st, fb, fk[0]);
      frag_row<Img>(fb, Qimg, qt * 16 + c, 32 + 8 * g);
      mma16(st, fb, fk[1]);
      frag_row<Img>(fb, Dimg, qt * 16 + c, 8 * g);
      mma16(dpt, fb, fv[0]);
      frag_row<Img>(fb, Dimg, qt * 16 + c, 32 + 8 * g);
      mma16(dpt, fb, fv[1]);
      // st[r] / dpt[r]: S / dP at (query 16qt + 4g + r, key k0 + c)
      // its keep bits: 4 consecutive bits of word (qt, k0/16, key % 4)
      uint32_t nib = 0;
      if (DM == 1) nib = (uint32_t)(shfl64(mword, 4 * qt + (lane & 3)) >> (16 * (c >> 2) + 4 * g));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = qt * 16 + 4 * g + r;
        const float pv = fast_exp2(st[r] * c2 - lse_s[q]);
        float pdr = pv, dpd = dpt[r];
        if constexpr (DM != 0) {  // P_drop's 1/(1-p) goes onto dV at the end
          const bool keep = DM == 1 ? ((nib >> r) & 1) : nstl_keep(p.seed, drop_idx(bh, T_, q, k0 + c), p.thresh);
          pdr = keep ? pv : 0.f;
          dpd = keep ? dpd * p.inv_keep : 0.f;
        }
        pdv[u][r] = pdr;
        dsv[u][r] = pv * (dpd - dq_s[q]);
      }
    }
    const Frag fa1 = acc_frag<T>(pdv[0], pdv[1]);  // P_drop^T, row = key k0 + c
    const Frag fa2 = acc_frag<T>(dsv[0], dsv[1]);  // dS^T
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      Frag fb;
      frag_col2<Img>(fb, Dimg, dt * 16, 32 * j, lane);
      mma16(dv[dt], fa1, fb);
      frag_col2<Img>(fb, Qimg, dt * 16, 32 * j, lane);
      mma16(dk[dt], fa2, fb);
    }
  }
  float vk[4][4], vv[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      vk[dt][r] = dk[dt][r] * p.scale;
      vv[dt][r] = DM != 0 ? dv[dt][r] * p.inv_keep : dv[dt][r];
    }
  if (p.rope_k) rope_back_tile(vk, k0 + 4 * g, c, p.rope_cos, p.rope_sin, sizeof(T) == 2 && p.rope_fast);
  if (alias) __syncthreads();  // every wave is done with the Q / dO images
  char* scr = scratch + w * 16 * RBK;
  store_tile16x64<T>(vk, scr, p.dk + ((tok0 + k0) * p.dk_ld + h * DH) * ESZ, p.dk_ld, lane);
  store_tile16x64<T>(vv, scr, p.dv + ((tok0 + k0) * p.dv_ld + h * DH) * ESZ, p.dv_ld, lane);
  if (bias_row) {
    wave_colsum16x64<T>(vk, red, w, lane);
    wave_colsum16x64<T>(vv, red + NW * 64, w, lane);
    if (last_to_arrive(arrived, NW, lane)) {
      wave_sum_out(red, NW, bias_row + p.H * DH + h * DH, lane);
      wave_sum_out(red + NW * 64, NW, bias_row + 2 * p.H * DH + h * DH, lane);
    }
  }
}

// ---------------------------------------------------------------------------
// Fused backward (bf16, T <= 128): ONE workgroup per (b, h) produces dQ, dK and
// dV, so Q, dO, K and V are read once (the split kernels read Q, K, V and dO
// twice: 384 -> 256 MB per call at the 228M shape).  A wave owns 16 keys, as in
// attn_bwd_dkv: S / dP with query rows, P^T / dS^T in registers -> dV, dK.  The
// dS^T fragments (bf16, what the dK product consumed) stay in registers until
// every wave is done with the Q / dO images, then go to an LDS image over them
// (rows = keys, the reduction index of dQ = dS K), and each wave computes dQ for
// 16 queries from that image and the K image.  LDS: Q | dO (later dS^T, 32 KB),
// K (16 KB), lse / D (1 KB); the output staging and bias partials reuse the
// first 22 KB once dQ is done.  49 KB: up to 3 workgroups per CU by LDS.
//   prologue: DMA Q, dO, K images; own K / V rows and own-query O rows from
//             global; lse -> LDS; barrier; D = rowsum(dO * O) of own queries
//             (dO from its image) -> LDS; barrier
//   phase 1 : S, dP over the 8 query tiles; dV += P_drop^T dO, dK += dS^T Q
//   phase 2 : barrier; dS^T -> image; barrier; dQ = dS K
//   stores  : barrier; dQ, dK, dV rows (+ bias column sums, last wave out)
constexpr int FUSED_MAX_T = 128;
// Output staging of one wave (store_tile16x64_buf): its 16 rows in four groups of
// 4 rows (lane group g's rows 4g + r), each group padded by 32 bytes.  With
// 128-byte rows and no padding the four lane groups' 2-byte writes land on the
// same 8 banks (4-way conflicts on every element write: the fused backward's
// largest remaining conflict term); the 32-byte pad puts group g on banks
// 8g .. 8g + 7, and the address stays one per-lane base + immediate offsets.
constexpr int FUSED_SCR_G = 4 * DH * 2 + 32, FUSED_SCR = 4 * FUSED_SCR_G;
// LDS map after phase 2: staging [0, 17 KB), bias partials [17 KB, 23 KB), RoPE
// tables [23 KB, 59 KB) over the dead K image / lse / D, then the counter
constexpr int FUSED_ROPE_OFF = 8 * FUSED_SCR + 3 * 8 * 64 * 4;
constexpr int FUSED_RS = DH / 2 + 4;  // padded table row (floats): 144 B, 16-byte aligned
constexpr int FUSED_ARRIVED_OFF = FUSED_ROPE_OFF + 2 * FUSED_MAX_T * FUSED_RS * 4;
constexpr int FUSED_DS_RB = FUSED_MAX_T * 2;  // dS^T image row: 128 queries (bf16)
// The dS^T image: written by rows (ds_write_b64, 16 lanes on 16 consecutive rows at one
// column) and read transposed (frag_col2: 8 consecutive rows x 32 bytes per 32-lane
// group).  16-byte chunk c of row r at c ^ x, x = (r & 7) << 1 | (r >> 3) & 1: the
// transposed reads are conflict-free and the writes 2-way (16-byte chunk swizzles
// cannot place 16 rows' 8-byte halves on distinct banks).  ImgMN<256>, made for
// frag_col's row pattern, cost 4-way writes and 2-way reads here.
struct DsImg {
  static NSTL_DEV int off(int row, int byte) {
    const int x = ((row & 7) << 1) | ((row >> 3) & 1);
    return row * FUSED_DS_RB + ((((byte >> 4) ^ x) << 4) | (byte & 15));
  }
};

// 16-byte chunk idx of the concatenated cos | sin tables (nchunk chunks each);
// past the end it re-reads the last chunk (the caller does not store it)
NSTL_DEV uint4 rope_chunk(const AttnParams& p, int idx, int nchunk) {
  idx = min(idx, 2 * nchunk - 1);
  const uint4* src = idx < nchunk ? (const uint4*)p.rope_cos + idx : (const uint4*)p.rope_sin + (idx - nchunk);
  return *src;
}

// dma_rows (ImgAtt<128>, bf16) from a head buffer: 8 rows per 1 KB wave instruction
template <int NW>
NSTL_DEV void dma_rows_buf(char* img, __amdgpu_buffer_rsrc_t r, uint32_t ld_bytes, int nrows, int wave, int lane) {
  const int ninst = nrows / 8;
  for (int q = wave; q < ninst; q += NW) {
    const int row = q * 8 + (lane >> 3), lc = (lane & 7) ^ att_x(row);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(img + q * 1024), 16,
                                             (uint32_t)row * ld_bytes + lc * 16, 0, 0, 0);
  }
}
typedef int i32x4b __attribute__((ext_vector_type(4)));
// store_tile16x64<bf16> into a head buffer (head_rsrc of the output), the tile's
// first row at byte offset off0: 32-bit offsets instead of 64-bit addresses.  The
// wave's staging image is FUSED_SCR bytes, rows grouped by 4 with a 32-byte pad.
NSTL_DEV void store_tile16x64_buf(const float (&v)[4][4], char* scr, __amdgpu_buffer_rsrc_t r, uint32_t off0,
                                  uint32_t ld_bytes, int lane) {
  constexpr int RB = DH * 2, CPR = RB / 16;
  const int g = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      *(bf16*)(scr + g * FUSED_SCR_G + rr * RB + (dt * 16 + (lane & 15)) * 2) = (bf16)v[dt][rr];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int row = c / CPR, ch = c % CPR;
    __builtin_amdgcn_raw_buffer_store_b128(*(const i32x4b*)(scr + (row >> 2) * FUSED_SCR_G + (row & 3) * RB + ch * 16), r,
                                           off0 + (uint32_t)row * ld_bytes + ch * 16, 0, 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
NSTL_DEV bf16x8 buf_frag(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
// D's row part: sum_e a[e] b[e] over one fragment pair, two products per
// v_dot2_f32_bf16 (unpacked, each product cost two conversions and an FMA)
NSTL_DEV float dot8_bf16(const bf16x8& a, const bf16x8& b, float acc) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int e = 0; e < 8; e += 2)
    acc = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){a[e], a[e + 1]}, (bf16x2){b[e], b[e + 1]}, acc, false);
  return acc;
}
// stored keep bit r of a nibble as an all-ones / zero lane mask (one v_bfe_i32):
// P_drop and dP_drop then take it by AND instead of a compare and two selects
NSTL_DEV uint32_t keep_mask(uint32_t nib, int r) { return (uint32_t)((int)(nib << (31 - r)) >> 31); }
NSTL_DEV float and_mask(float x, uint32_t m) { return __uint_as_float(__float_as_uint(x) & m); }

// DM: dropout mode, fixed per launch so the per-element loop carries no branch:
// 0 none, 1 the forward's stored keep bits, 2 re-hashed (seed, element)
// TC: T as a compile-time constant (the production T = 128; 0: p.T)
template <int DM, int TC = 0>
__global__ __launch_bounds__(BWD_NT, 4) void attn_bwd_fused_kernel(AttnParams p) {
  typedef bf16x8 Frag;
  constexpr int RBK = DH * 2;
  typedef ImgAtt<RBK> Img;
  constexpr int NW = BWD_NT / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = TC ? TC : p.T, nkt = T_ / 16;
  char* Qimg = smem;                                           // [128][128 B]
  char* Dimg = Qimg + FUSED_MAX_T * RBK;                       // [128][128 B]
  char* DSimg = smem;                                          // over Q | dO after phase 1
  char* Kimg = smem + 2 * FUSED_MAX_T * RBK;                   // [128][128 B]
  float* lse_s = (float*)(Kimg + FUSED_MAX_T * RBK);
  float* d_s = lse_s + FUSED_MAX_T;
  char* scratch = smem;                                        // after phase 2: [NW][FUSED_SCR]
  float* red = (float*)(smem + NW * FUSED_SCR);                // after phase 2: [3][NW][64]
  float* cos_s = (float*)(smem + FUSED_ROPE_OFF);              // after phase 2: RoPE tables [T][DH/2] x 2
  float* sin_s = cos_s + T_ * FUSED_RS;
  unsigned* arrived = (unsigned*)(smem + FUSED_ARRIVED_OFF);

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;
  const int k0 = w * 16;     // this wave's keys (phase 1) and queries (D, phase 2)
  const bool act = TC == FUSED_MAX_T || k0 < T_;
  // the head's rows of each operand as a buffer (base in SGPRs, per-lane 32-bit
  // offsets; 64-bit per-lane addresses were ~100 of the wave's vector instructions)
  const __amdgpu_buffer_rsrc_t rq = head_rsrc(p.q, p.q_ld, tok0, h, T_), rd = head_rsrc(p.dout, p.dout_ld, tok0, h, T_),
                               rk = head_rsrc(p.k, p.k_ld, tok0, h, T_), rv = head_rsrc(p.v, p.v_ld, tok0, h, T_),
                               ro = head_rsrc(p.o, p.o_ld, tok0, h, T_);
  dma_rows_buf<NW>(Qimg, rq, (uint32_t)p.q_ld * 2, T_, w, lane);
  dma_rows_buf<NW>(Dimg, rd, (uint32_t)p.dout_ld * 2, T_, w, lane);
  dma_rows_buf<NW>(Kimg, rk, (uint32_t)p.k_ld * 2, T_, w, lane);
  for (int i = tid; i < T_; i += BWD_NT) lse_s[i] = p.lse[(int64_t)bh * T_ + i] * LOG2E;
  if (tid == 0) *arrived = 0u;
  Frag fk[2], fv[2], oo[2];
  if (act) {
    const uint32_t r = (uint32_t)(k0 + c);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t col = (uint32_t)(32 * u + 8 * g) * 2;
      fk[u] = buf_frag(rk, r * (uint32_t)p.k_ld * 2 + col);
      fv[u] = buf_frag(rv, r * (uint32_t)p.v_ld * 2 + col);
      oo[u] = buf_frag(ro, r * (uint32_t)p.o_ld * 2 + col);
    }
  }
  // stored keep bits for this wave's 16 keys: lane 4*qt + r holds word (qt, k0/16, r)
  uint64_t mword = 0;
  if (DM == 1 && act && (lane >> 2) < nkt) mword = p.mask[mask_word(bh, nkt, lane >> 2, k0 >> 4, lane & 3)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (act) {  // D of queries k0 + c (dO from its image, O from registers)
    float dpart = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      Frag fo;
      frag_row<Img>(fo, Dimg, k0 + c, 32 * u + 8 * g);
      dpart = dot8_bf16(fo, oo[u], dpart);
    }
    dpart = sum_xor16(dpart);
    dpart = sum_xor32(dpart);
    if (g == 0) d_s[k0 + c] = dpart;
  }
  __syncthreads();

  const float c2 = p.scale * LOG2E;
  f32x4 dk[4], dv[4];
  Frag dsf[FUSED_MAX_T / 32];  // dS^T fragments (acc_frag order), kept for dQ
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (act) {
#pragma unroll
    for (int j = 0; j < FUSED_MAX_T / 32; ++j) {  // 32-query chunks
      if (j < nkt / 2) {
        f32x4 pdv[2], dsv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int qt = 2 * j + u;
          f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
          Frag fb;
          frag_row<Img>(fb, Qimg, qt * 16 + c, 8 * g);
          mma16(st, fb, fk[0]);
          frag_row<Img>(fb, Qimg, qt * 16 + c, 32 + 8 * g);
          mma16(st, fb, fk[1]);
          frag_row<Img>(fb, Dimg, qt * 16 + c, 8 * g);
          mma16(dpt, fb, fv[0]);
          frag_row<Img>(fb, Dimg, qt * 16 + c, 32 + 8 * g);
          mma16(dpt, fb, fv[1]);
          // st[r] / dpt[r]: S / dP at (query 16qt + 4g + r, key k0 + c)
          uint32_t nib = 0;
          if (DM == 1) nib = (uint32_t)(shfl64(mword, 4 * qt + (lane & 3)) >> (16 * (c >> 2) + 4 * g));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = qt * 16 + 4 * g + r;
            const float pv = fast_exp2(st[r] * c2 - lse_s[q]);
            float pdr = pv, dpd = dpt[r];
            if constexpr (DM == 1) {  // P_drop's 1/(1-p) goes onto dV at the end
              const uint32_t km = keep_mask(nib, r);
              pdr = and_mask(pv, km);
              dpd = and_mask(dpd * p.inv_keep, km);
            } else if constexpr (DM == 2) {
              const bool keep = nstl_keep(p.seed, drop_idx(bh, T_, q, k0 + c), p.thresh);
              pdr = keep ? pv : 0.f;
              dpd = keep ? dpd * p.inv_keep : 0.f;
            }
            pdv[u][r] = pdr;
            dsv[u][r] = pv * (dpd - d_s[q]);
          }
        }
        const Frag fa1 = acc_frag<bf16>(pdv[0], pdv[1]);  // P_drop^T, row = key k0 + c
        dsf[j] = acc_frag<bf16>(dsv[0], dsv[1]);          // dS^T
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          Frag fb;
          frag_col2<Img>(fb, Dimg, dt * 16, 32 * j, lane);
          mma16(dv[dt], fa1, fb);
          frag_col2<Img>(fb, Qimg, dt * 16, 32 * j, lane);
          mma16(dk[dt], dsf[j], fb);
        }
      }
    }
  }
  __syncthreads();  // every wave is done with the Q / dO images
  // RoPE tables for the epilogue's rope_back: 16-byte loads issued now, their
  // latency hidden under the dS^T write and dQ; to LDS once the K image is
  // dead.  (Read per element from global memory they cost ~16 dependent L2
  // round trips per wave: 95 -> 79 us per call with RoPE^T off.)
  const bool rope = p.rope_q || p.rope_k, rope_tabs = rope && !p.rope_fast;
  const int nchunk = T_ * (DH / 2) / 4;  // 16-byte chunks per table
  uint4 rt0 = {}, rt1 = {}, rt2 = {}, rt3 = {};
  if (rope_tabs) {
    rt0 = rope_chunk(p, tid, nchunk);
    rt1 = rope_chunk(p, tid + BWD_NT, nchunk);
    rt2 = rope_chunk(p, tid + 2 * BWD_NT, nchunk);
    rt3 = rope_chunk(p, tid + 3 * BWD_NT, nchunk);
  }
  if (act) {
    // dS^T row = key k0 + c; fragment j holds queries 32j + 4g + 0..3 and 32j + 16 + 4g + 0..3
#pragma unroll
    for (int j = 0; j < FUSED_MAX_T / 32; ++j) {
      if (j < nkt / 2) {
        const bf16x8 f = dsf[j];
        *(bf16x4*)(DSimg + DsImg::off(k0 + c, (32 * j + 4 * g) * 2)) = (bf16x4){f[0], f[1], f[2], f[3]};
        *(bf16x4*)(DSimg + DsImg::off(k0 + c, (32 * j + 16 + 4 * g) * 2)) = (bf16x4){f[4], f[5], f[6], f[7]};
      }
    }
  }
  __syncthreads();
  // dQ(query k0 + 4g + r, d = 16dt + c) = sum_key dS(query, key) K(key, d)
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (act) {
#pragma unroll
    for (int j = 0; j < FUSED_MAX_T / 32; ++j) {
      if (j < nkt / 2) {
        Frag fa;
        frag_col2<DsImg>(fa, DSimg, k0, 32 * j, lane);  // dS, row = query k0 + c
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          Frag fb;
          frag_col2<Img>(fb, Kimg, dt * 16, 32 * j, lane);
          mma16(dq[dt], fa, fb);
        }
      }
    }
  }
  __syncthreads();  // the dS^T / K images become output staging and RoPE tables
  if (rope_tabs) {
    // chunk idx (8 per 32-float table row) -> row-padded image, sin_s = cos_s + T * FUSED_RS
    auto put = [&](int idx, const uint4& v) {
      if (idx < 2 * nchunk) {
        const int t = idx < nchunk ? idx : idx - nchunk;
        *(uint4*)(cos_s + (idx < nchunk ? 0 : T_ * FUSED_RS) + (t >> 3) * FUSED_RS + (t & 7) * 4) = v;
      }
    };
    put(tid, rt0);
    put(tid + BWD_NT, rt1);
    put(tid + 2 * BWD_NT, rt2);
    put(tid + 3 * BWD_NT, rt3);
    __syncthreads();
  }
  float vq[4][4], vk[4][4], vv[4][4];
  float* bias_row = p.dbias ? p.dbias + (int64_t)b * 3 * p.H * DH : nullptr;
  if (act) {  // wave-uniform: rope_back_tile's DPP swaps see the whole wave
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        vq[dt][r] = dq[dt][r] * p.scale;
        vk[dt][r] = dk[dt][r] * p.scale;
        vv[dt][r] = DM != 0 ? dv[dt][r] * p.inv_keep : dv[dt][r];
      }
    if (rope) {  // dQ and dK rows are the same 16: one table read for both
      float tc[4][4], ts[4][4];
      if (rope_tabs) rope_tab<FUSED_RS>(tc, ts, k0 + 4 * g, c, cos_s, sin_s);
      else rope_tab_fast(tc, ts, k0 + 4 * g, c);
      if (p.rope_q) rope_apply(vq, tc, ts);
      if (p.rope_k) rope_apply(vk, tc, ts);
    }
    char* scr = scratch + w * FUSED_SCR;
    store_tile16x64_buf(vq, scr, head_rsrc(p.dq, p.dq_ld, tok0, h, T_), (uint32_t)k0 * p.dq_ld * 2, p.dq_ld * 2, lane);
    store_tile16x64_buf(vk, scr, head_rsrc(p.dk, p.dk_ld, tok0, h, T_), (uint32_t)k0 * p.dk_ld * 2, p.dk_ld * 2, lane);
    store_tile16x64_buf(vv, scr, head_rsrc(p.dv, p.dv_ld, tok0, h, T_), (uint32_t)k0 * p.dv_ld * 2, p.dv_ld * 2, lane);
  }
  if (bias_row) {
    if (act) {
      wave_colsum16x64<bf16>(vq, red, w, lane);
      wave_colsum16x64<bf16>(vk, red + NW * 64, w, lane);
      wave_colsum16x64<bf16>(vv, red + 2 * NW * 64, w, lane);
    } else {
      red[w * 64 + lane] = 0.f;
      red[NW * 64 + w * 64 + lane] = 0.f;
      red[2 * NW * 64 + w * 64 + lane] = 0.f;
    }
    if (last_to_arrive(arrived, NW, lane)) {
#pragma unroll
      for (int m = 0; m < 3; ++m) wave_sum_out(red + m * NW * 64, NW, bias_row + m * p.H * DH + h * DH, lane);
    }
  }
}
constexpr size_t FUSED_LDS = FUSED_ARRIVED_OFF + 16;  // 58 KB: two workgroups per CU
static_assert(FUSED_ARRIVED_OFF >= 3 * FUSED_MAX_T * DH * 2 + 2 * FUSED_MAX_T * 4, "counter past the images");
static_assert(FUSED_ROPE_OFF % 16 == 0, "16-byte table chunks");
static_assert(8 * FUSED_SCR + 3 * 8 * 64 * 4 <= 3 * FUSED_MAX_T * DH * 2, "staging must fit in the images");
static_assert(BWD_NT / 64 == 8, "the staging map assumes 8 waves");


size_t fwd_lds_bytes(int T, int esz) {  // K, V images (the output leaves from registers)
  return (size_t)2 * T * DH * esz;
}
size_t bwd_lds_bytes(int T, int esz) {  // either backward kernel (+ 2 x [8][64] f32 bias partials + counter)
  // T % BWD_ROWS == 0: the output staging reuses the first operand image
  const size_t staging = T % BWD_ROWS == 0 ? 0 : (size_t)(BWD_NT / 64) * 16 * DH * esz;
  return (size_t)2 * T * DH * esz + 2 * T * 4 + staging + 2 * (BWD_NT / 64) * 64 * 4 + 16;
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

// the fused backward (bf16, T <= 128); NSTL_ATTN_BWD=split selects the two
// kernels (A/B comparisons; read per call so a test can switch it)
bool use_fused_bwd(const nstl_attn_args* a) {
  const char* e = getenv("NSTL_ATTN_BWD");
  if (e && e[0] == 's') return false;
  return use_fast(a) && a->dtype == NSTL_BF16 && a->T <= FUSED_MAX_T;
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
  {  // NSTL_ROPE_BWD=table: the bf16 backward kernels read the tables (A/B; read per call)
    const char* e = getenv("NSTL_ROPE_BWD");
    p.rope_fast = !(e && e[0] == 't');
  }
  p.B = a->B; p.T = a->T; p.H = a->H; p.dh = a->dh;
  p.scale = 1.0f / sqrtf((float)a->dh);
  p.thresh = nstl_drop_thresh(a->p_drop);
  p.inv_keep = 1.0f / (1.0f - a->p_drop);
  p.seed = a->seed;
  NSTL_CHECK_ARG(!p.thresh || nstl_pair_index32_ok((uint64_t)a->B * a->H * a->T * a->T),
                 "nstl_attn: B*H*T*T past 2^33 dropout elements (32-bit pair index)");
  return 0;
}

template <typename K, typename... X>
int launch(K kern, dim3 grid, size_t lds, hipStream_t st, const AttnParams& p, const char* what, int nt = NT,
           X... extra) {
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return nstl::fail((int)e, "%s: LDS request %zu: %s", what, lds, hipGetErrorString(e));
  hipLaunchKernelGGL(kern, grid, dim3(nt), lds, st, p, extra...);
  NSTL_LAUNCH_CHECK(what);
  return 0;
}


// the persistent forward (bf16, T = 128, enough heads to fill the grid);
// NSTL_ATTN_FWD=oneshot selects the one-workgroup-per-head kernel (A/B; read per call)
bool use_persist_fwd(const nstl_attn_args* a) {
  const char* e = getenv("NSTL_ATTN_FWD");
  if (e && e[0] == 'o') return false;
  return a->dtype == NSTL_BF16 && a->T == PF_T && a->dh == DH;
}

// the split backward: dQ (also writes D = rowsum(dO * O)), then dK / dV
template <typename T, int DM>
int launch_split(dim3 grid, size_t lds, hipStream_t st, const AttnParams& p) {
  nstl::count(NSTL_K_ATTN_BWD_SPLIT);
  int rc = launch(attn_bwd_dq_kernel<T, DM>, grid, lds, st, p, "nstl_attn_bwd dq", BWD_NT);
  if (rc) return rc;
  return launch(attn_bwd_dkv_kernel<T, DM>, grid, lds, st, p, "nstl_attn_bwd dkv", BWD_NT);
}

}  // namespace

extern "C" int nstl_attn_fwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, false);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  hipStream_t st = (hipStream_t)stream;
  if (!use_fast(a)) {
    nstl::count(NSTL_K_ATTN_FWD_GENERIC);
    dim3 grid((a->T + 3) / 4, a->B * a->H);
    const size_t lds = 4 * (size_t)(a->dh + a->T) * 4;
    if (a->dtype == NSTL_BF16) return launch(attn_fwd_generic<bf16>, grid, lds, st, p, "nstl_attn_fwd generic");
    return launch(attn_fwd_generic<float>, grid, lds, st, p, "nstl_attn_fwd generic");
  }
  nstl::count(NSTL_K_ATTN_FWD);
  if (use_persist_fwd(a)) {
    // head buffers (q, k, v, o): T rows of each as one 32-bit extent
    NSTL_CHECK_ARG((int64_t)a->T * std::max(std::max(a->q_ld, a->k_ld), std::max(a->v_ld, a->o_ld)) * 2 < (1ll << 31),
                   "nstl_attn_fwd: T x row stride past 2^31 bytes");
    const int nitems = a->B * a->H;
    const int G = std::min(nitems, std::max(2, 2 * nstl::stream_cus(st)));  // two workgroups per CU the stream may use
    const size_t lds = PF_LDS;
    if (p.thresh && p.mask)
      return launch(attn_fwd_persist_kernel<true>, dim3(G), lds, st, p, "nstl_attn_fwd persistent", FWD_NT, nitems);
    return launch(attn_fwd_persist_kernel<false>, dim3(G), lds, st, p, "nstl_attn_fwd persistent", FWD_NT, nitems);
  }
  dim3 grid((a->T + FWD_QB - 1) / FWD_QB, a->B * a->H);
  const size_t lds = fwd_lds_bytes(a->T, esz);
  // T % 32 == 0 and T <= 256 on this path: NKT in {2, 4, ..., 16}
#define NSTL_FWD_CASE(N)                                                                              \
  case N:                                                                                             \
    return a->dtype == NSTL_BF16 ? launch(attn_fwd_kernel<bf16, N>, grid, lds, st, p, "nstl_attn_fwd", FWD_NT) \
                                 : launch(attn_fwd_kernel<float, N>, grid, lds, st, p, "nstl_attn_fwd", FWD_NT);
  switch (a->T / 16) {
    NSTL_FWD_CASE(2) NSTL_FWD_CASE(4) NSTL_FWD_CASE(6) NSTL_FWD_CASE(8)
    NSTL_FWD_CASE(10) NSTL_FWD_CASE(12) NSTL_FWD_CASE(14) NSTL_FWD_CASE(16)
  }
#undef NSTL_FWD_CASE
  return nstl::fail((int)hipErrorInvalidValue, "nstl_attn_fwd: T=%d off the MFMA path", a->T);
}

extern "C" int nstl_attn_bwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, true);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  hipStream_t st = (hipStream_t)stream;
  if (!use_fast(a)) {
    nstl::count(NSTL_K_ATTN_BWD_GENERIC);
    dim3 grid((a->T + 3) / 4, a->B * a->H);
    const size_t lq = 4 * (size_t)(2 * a->dh + a->T) * 4, lkv = 4 * (size_t)(2 * a->dh + 2 * a->T) * 4;
    if (a->dtype == NSTL_BF16) {
      if ((rc = launch(attn_bwd_dq_generic<bf16>, grid, lq, st, p, "nstl_attn_bwd generic dq"))) return rc;
      return launch(attn_bwd_dkv_generic<bf16>, grid, lkv, st, p, "nstl_attn_bwd generic dkv");
    }
    if ((rc = launch(attn_bwd_dq_generic<float>, grid, lq, st, p, "nstl_attn_bwd generic dq"))) return rc;
    return launch(attn_bwd_dkv_generic<float>, grid, lkv, st, p, "nstl_attn_bwd generic dkv");
  }
  if (use_fused_bwd(a)) {
    NSTL_CHECK_ARG(!(a->rope_q || a->rope_k) || ((((uintptr_t)a->rope_cos) | ((uintptr_t)a->rope_sin)) & 15) == 0,
                   "nstl_attn_bwd: RoPE tables must be 16-byte aligned");
    // head_rsrc: T rows of each operand as one buffer (32-bit extent)
    const int64_t ld_max = std::max(std::max(std::max(a->q_ld, a->k_ld), std::max(std::max(a->v_ld, a->o_ld), a->dout_ld)),
                                    std::max(std::max(a->dq_ld, a->dk_ld), a->dv_ld));
    NSTL_CHECK_ARG((int64_t)a->T * ld_max * 2 < (1ll << 31), "nstl_attn_bwd: T x row stride past 2^31 bytes");
    nstl::count(NSTL_K_ATTN_BWD_FUSED);
    const dim3 grid(1, a->B * a->H);
    if (a->T == FUSED_MAX_T) {  // the production shape: T a compile-time constant
      if (!p.thresh) return launch(attn_bwd_fused_kernel<0, FUSED_MAX_T>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
      if (p.mask) return launch(attn_bwd_fused_kernel<1, FUSED_MAX_T>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
      return launch(attn_bwd_fused_kernel<2, FUSED_MAX_T>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
    }
    if (!p.thresh) return launch(attn_bwd_fused_kernel<0>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
    if (p.mask) return launch(attn_bwd_fused_kernel<1>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
    return launch(attn_bwd_fused_kernel<2>, grid, FUSED_LDS, st, p, "nstl_attn_bwd fused", BWD_NT);
  }
  dim3 grid((a->T + BWD_ROWS - 1) / BWD_ROWS, a->B * a->H);
  const size_t lds = bwd_lds_bytes(a->T, esz);
  const int dm = !p.thresh ? 0 : (p.mask ? 1 : 2);
  if (a->dtype == NSTL_BF16) {
    if (dm == 0) return launch_split<bf16, 0>(grid, lds, st, p);
    if (dm == 1) return launch_split<bf16, 1>(grid, lds, st, p);
    return launch_split<bf16, 2>(grid, lds, st, p);
  }
  if (dm == 0) return launch_split<float, 0>(grid, lds, st, p);
  if (dm == 1) return launch_split<float, 1>(grid, lds, st, p);
  return launch_split<float, 2>(grid, lds, st, p);
}

extern "C" int nstl_attn_bias_rows(const nstl_attn_args* a) {
  if (a == nullptr || !use_fast(a)) return 0;
  return a->B * ((a->T + BWD_ROWS - 1) / BWD_ROWS);
}
