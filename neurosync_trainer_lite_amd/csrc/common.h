// Shared device helpers for the NeuroSync Trainer Lite MI355X (gfx950) kernels.
//
// Fragment convention (all MFMA users in this library):
//   a "fragment" is what one lane contributes to one 16x16xK32 MFMA step:
//   8 consecutive reduction-index elements r = 8*(lane>>4) + 0..7 of row
//   (lane & 15).  For bf16 that is ONE v_mfma_f32_16x16x32_bf16; for f32 it is
//   EIGHT v_mfma_f32_16x16x4_f32, step s taking element s (the reduction index
//   is permuted identically on A and B, so the sum is the same).
//   C/D layout (both): col = lane & 15, row = 4*(lane>>4) + reg.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NSTL_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <typename T> struct FragT;
template <> struct FragT<bf16> { typedef bf16x8 type; };
template <> struct FragT<float> { typedef f32x8 type; };

NSTL_DEV void mma16(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}
NSTL_DEV void mma16(f32x4& acc, const f32x8& a, const f32x8& b) {
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
}

NSTL_DEV float to_f32(float x) { return x; }
NSTL_DEV float to_f32(bf16 x) { return (float)x; }
template <typename T> NSTL_DEV T from_f32(float x);
template <> NSTL_DEV float from_f32<float>(float x) { return x; }
template <> NSTL_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

typedef __attribute__((address_space(3))) char lds_char;

// ---------------------------------------------------------------------------
// LDS images.  All staging is 16-byte chunks; swizzles permute whole chunks so
// a 16-byte store/load never straddles.  An image policy maps (row, byte in
// row) -> byte offset; writers and readers of one image use the same policy.
//
// ImgK<RB>: rows of RB bytes read mainly as 16-byte row chunks (ds_read_b128
// by 16 lanes on 16 different rows).  RB=128: chunk ^ ((row>>1)&7); RB=256:
// chunk ^ (row&15); either way 16 consecutive rows at one chunk land on 16
// distinct 16-byte bank slots.
template <int RB> struct ImgK {
  static NSTL_DEV int off(int row, int byte) {
    const int chunk = byte >> 4;
    int x;
    if constexpr (RB == 64) x = 0;  // 16 rows x 64 B = one contiguous KB: conflict-free as is
    else if constexpr (RB == 128) x = (row >> 1) & 7;
    else x = row & 15;
    return row * RB + (((chunk ^ x) << 4) | (byte & 15));
  }
};
// ImgMN<RB>: rows = reduction index, read with transpose reads (4 rows x 32
// bytes per 16-lane group; one 32-lane half touches rows {r0..r0+3, r0+8..r0+11}).
// The XOR keeps chunk pairs adjacent and puts those 8 rows on 8 distinct 32-byte
// bank slots.  RB=128: x = ((row>>1)&1) | ((row>>3)&1)<<1; RB>=256:
// x = (row&3) | ((row>>3)&1)<<2.
template <int RB> struct ImgMN {
  static NSTL_DEV int off(int row, int byte) {
    const int chunk = byte >> 4;
    int x;
    if constexpr (RB == 128) x = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    else x = (row & 3) | (((row >> 3) & 1) << 2);
    return row * RB + (((chunk ^ (x << 1)) << 4) | (byte & 15));
  }
};
// Plain padded rows (scratch images written element-wise).
template <int RB> struct ImgPlain {
  static NSTL_DEV int off(int row, int byte) { return row * RB + byte; }
};

// Fragment from an image whose rows are the fragment rows: element
// (row, r..r+7), r a multiple of 8 (one/two 16-byte reads).
template <class Img> NSTL_DEV void frag_row(bf16x8& f, const char* img, int row, int r) {
  f = *(const bf16x8*)(img + Img::off(row, r * 2));
}
template <class Img> NSTL_DEV void frag_row(f32x8& f, const char* img, int row, int r) {
  f32x4 lo = *(const f32x4*)(img + Img::off(row, r * 4));
  f32x4 hi = *(const f32x4*)(img + Img::off(row, r * 4 + 16));
  f = (f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Fragment from an image whose rows are the reduction index: element
// (col = col16 + (lane&15), r..r+7) with r = r0 + 8*(lane>>4).
// bf16: two ds_read_b64_tr_b16 (gfx950 transpose read: per 16-lane group a
// block of 4 rows x 16 columns, lane 4q+p supplying row q, columns 4p..4p+3,
// lane i receiving column i).
template <class Img>
NSTL_DEV void frag_col(bf16x8& f, const char* img, int col16, int r0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int rb = r0 + 8 * g;
  const int byte = (col16 + 4 * p) * 2;
  const lds_char* base = (const lds_char*)img;
  s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + Img::off(rb + q, byte)));
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + Img::off(rb + 4 + q, byte)));
  bf16x4 b0 = __builtin_bit_cast(bf16x4, v0);
  bf16x4 b1 = __builtin_bit_cast(bf16x4, v1);
  f = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
}
template <class Img>
NSTL_DEV void frag_col(f32x8& f, const char* img, int col16, int r0, int lane) {
  const int rb = r0 + 8 * (lane >> 4);
  const int byte = (col16 + (lane & 15)) * 4;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = *(const float*)(img + Img::off(rb + j, byte));
}

// ---------------------------------------------------------------------------
// Counter-based dropout RNG: keep(seed, idx) is a pure function of its inputs,
// so forward and backward regenerate the same mask without storing it.
// One 32-bit fmix (murmur3 finaliser) of the seed-keyed pair index gives two
// 16-bit uniforms: elements 2k and 2k+1 take the low / high half.  The drop
// probability is quantised to 1/65536 (0.3 -> 0.300003).
NSTL_DEV uint32_t nstl_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
// Two 32-bit multiplies per pair (the fmix), both on the vector path; the
// seed term is wave-uniform (scalar).  Pair indices past 2^32 (elements past
// 2^33, far beyond any tensor of this model) fold their high word in by a
// rotation, no multiply: v_mul_lo_u32 is the costly instruction here (the
// attention forward spent ~7 us per call on 4 of them per pair).
NSTL_DEV uint32_t nstl_pair_hash(uint64_t seed, uint64_t idx) {
  const uint32_t hi = (uint32_t)(idx >> 33);
  const uint32_t s = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27D4EB2Fu) ^ ((hi << 17) | (hi >> 15));
  return nstl_fmix32((uint32_t)(idx >> 1) ^ s);
}
NSTL_DEV bool nstl_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  const uint32_t h = nstl_pair_hash(seed, idx);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thresh;
}
// keep decisions for the pair (idx, idx+1), idx even: one hash
NSTL_DEV void nstl_keep2(uint64_t seed, uint64_t idx, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = nstl_pair_hash(seed, idx);
  k0 = (h & 0xFFFFu) >= thresh;
  k1 = (h >> 16) >= thresh;
}
// The same hash with the index already in 32-bit pair form.  For element
// indices below 2^33 (hi == 0 above) nstl_pair_hash(seed, idx) ==
// nstl_pair_hash32(nstl_seed_term(seed), idx >> 1): identical masks, but a hot
// loop then forms its pair indices with 32-bit adds instead of 64-bit element
// indices, shifts and the high-word fold (the attention forward built its 16
// hashes per lane from ~18 vector instructions each, the fmix being 8 of them).
// Launchers that use it check nstl_pair_index32_ok on the tensor's element count.
NSTL_DEV uint32_t nstl_seed_term(uint64_t seed) { return (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27D4EB2Fu); }
NSTL_DEV uint32_t nstl_pair_hash32(uint32_t seed_term, uint32_t pair) { return nstl_fmix32(pair ^ seed_term); }
NSTL_DEV void nstl_keep2_32(uint32_t seed_term, uint32_t pair, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = nstl_pair_hash32(seed_term, pair);
  k0 = (h & 0xFFFFu) >= thresh;
  k1 = (h >> 16) >= thresh;
}
static inline bool nstl_pair_index32_ok(uint64_t elements) { return elements <= (1ull << 33); }

// threshold on a 16-bit uniform; 0 = no dropout
static inline uint32_t nstl_drop_thresh(float p) {
  double t = (double)p * 65536.0 + 0.5;
  if (p <= 0.f) return 0;
  if (t >= 65536.0) return 65536u;
  return (uint32_t)t;
}

// v_writelane_b32 through the LLVM intrinsic (hipcc exposes no clang builtin for
// it): lane `lane` of `old` takes the wave-uniform `val`; the backend inserts the
// VALU-writes-SGPR -> v_writelane wait states (inline asm would not)
__device__ int nstl_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// x (op) x[lane ^ 16] and x (op) x[lane ^ 32] with the gfx950 permlane swaps: one
// VALU exchange each (the compiler pads its hazard), where __shfl_xor is an LDS
// ds_bpermute plus its address arithmetic.  The pairs are the same, so the
// results equal the __shfl_xor forms bit for bit.  Every lane must be active.
NSTL_DEV float sum_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
NSTL_DEV float sum_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
NSTL_DEV float max_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
NSTL_DEV float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// x[lane ^ 1], x[lane ^ 2] (quad_perm) and the 8- / 16-lane mirrors (row_half_mirror,
// row_mirror) as DPP moves: inside a 16-lane row, after the quad steps every quad
// holds one value, so the mirrors pair quad 0 with 1 and half 0 with 1.
#define NSTL_DPP(x, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), ctrl, 0xF, 0xF, false))

// wave-level reductions (64 lanes): four DPP steps inside 16-lane rows, then the two
// permlane swaps; every lane ends with the result
NSTL_DEV float wave_sum(float v) {
  v += NSTL_DPP(v, 0xB1);   // quad_perm [1, 0, 3, 2]
  v += NSTL_DPP(v, 0x4E);   // quad_perm [2, 3, 0, 1]
  v += NSTL_DPP(v, 0x141);  // row_half_mirror
  v += NSTL_DPP(v, 0x140);  // row_mirror
  v = sum_xor16(v);
  return sum_xor32(v);
}
NSTL_DEV float wave_max(float v) {
  v = fmaxf(v, NSTL_DPP(v, 0xB1));
  v = fmaxf(v, NSTL_DPP(v, 0x4E));
  v = fmaxf(v, NSTL_DPP(v, 0x141));
  v = fmaxf(v, NSTL_DPP(v, 0x140));
  v = max_xor16(v);
  return max_xor32(v);
}
NSTL_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// bijective XCD-aware remap: blocks b and b+8 share an XCD (observed round-robin
// dealing); give each XCD a contiguous range of logical tile ids.
NSTL_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int x = bid & 7, k = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

