// 4-wave persistent 256 x 256 MFMA GEMM for gfx950 (device code, shared by
// gemm4.hip and tools/micro/gemm4_bench.hip).
//
//   C[i, j] = alpha * sum_r A(i, r) B(j, r)  (+ epilogue)
//
// For full 256 x 256 tiles it replaces the 8-wave ring kernel (gemm.hip) and
// the library dispatch of round 3.
//
// Wave layout.  One workgroup = 4 waves, one per SIMD; wave (wm, wn) owns the
// 128 x 128 block (wm, wn) of the tile: 8 x 8 accumulators of
// v_mfma_f32_16x16x32_bf16 (operands swapped, so lane (g = l >> 4, c = l & 15)
// holds row 16a + c, columns 16b + 4g .. +3 of acc[a][b]), 256 f32 per lane in
// AGPRs.  A wave reads 16 fragments per 64 MFMAs (the 8-wave ring: 12 per 32).
//
// K loop (BK = 64).  Two 64 KB stages; A slots at [0, 32K) / [32K, 64K), B at
// [64K, 96K) / [96K, 128K).  K-major images have 128-byte rows (one whole cache
// line per row and stage: with 64-byte rows every DMA piece fetched half lines,
// and the K loop ran 8-12 % slower, tools/micro/gemm4_bench.hip); chunk c of row
// r sits at c ^ ((r >> 1) & 7).  MN-major images are 64 rows (k) x 512 B
// (ImgMN<512>, transpose reads).  A step is two half-steps of 64 MFMAs: h = 0
// computes k 0..31 of stage s (register set F0) while reading k 32..63 into F1;
// h = 1 computes F1 while reading stage s + 1's k 0..31 into F0 and issuing
// stage s + 2's 16 LDS-DMA pieces (buffer_load ... lds; per-lane 32-bit source
// offsets fixed per tile, the K advance a scalar offset) into the slot stage s
// just vacated.  One barrier per step, before h = 1: the counted vmcnt retires
// this wave's pieces of stage s + 1, the barrier publishes every wave's, and
// every wave is done reading stage s.  Reads and DMA pieces are interleaved with
// the MFMAs in a fixed order (sched_barrier): one wave per SIMD has no partner
// wave to hide them.
//
// Persistent tiles.  Workgroup w runs tiles w, w + G, ... (XCD-aware order).
// The stage sequence runs on across tiles: the last two steps of a tile stage
// the next tile's first two stages and its last half-step reads the next tile's
// first fragments, so the next K loop starts with no fill.  The first half-step
// of a tile takes C = 0 (no accumulator zeroing).  The epilogue runs from
// registers (no LDS staging, no barrier).  Its stores are the youngest VMEM
// operations when the next tile's step 0 waits for its stage 1, so that wait
// is counted past them (vmcnt retires in issue order) and they drain under the
// next tile's first step.
#pragma once
#include "common.h"
#include <type_traits>

namespace g4 {

constexpr int NT = 256;
constexpr int TILE = 256;
constexpr int BK = 64;
constexpr int OPS = 32768;         // one operand's stage image
constexpr int SMEM = 4 * OPS;      // 128 KB of stages
constexpr int ROPE_LDS = 32768;    // RoPE tables (EM_ROPE): T * rope_dim * 4 bytes at most
constexpr int GROUP_MAX = 16;

// epilogue kinds (the ring kernel's EM_* numbering)
enum { EM_BF16 = 1, EM_RELU_DROP = 2, EM_ROPE = 3, EM_DRELU = 4, EM_F32 = 5 };

struct Params {
  const char* A; int64_t lda;
  const char* B; int64_t ldb;
  char* C; int64_t ldc;
  int M, N, K;
  float alpha;
  const float* bias;               // [N] or null (BF16, RELU_DROP, ROPE)
  float inv_keep; uint32_t thresh; uint64_t seed;
  const float* rope_cos; const float* rope_sin; int rope_T, rope_dim, rope_cols;
  float* colsum_part;              // [M / 128][N] (DRELU)
  uint64_t* relu_mask;             // keep & positive bits, the ring layout (RELU_DROP writes, DRELU reads)
  float* sq_part;                  // [tiles][8] sums of squares of C (F32)
  const float* a_scale;            // fp8 (gemm4f8_kernel): f32 row scales of A [M] and of B [N]
  const float* b_scale;
  int rope_bf16;                   // EM_ROPE: the LDS table holds bf16 (cos, sin) (fp8 at T = 256)
  uint32_t a_bytes, b_bytes;       // extents of A and B (buffer range checks)
  int tiles_m, tiles_n;
};

// Stream-K tail (slab != nullptr): when the tile count T is not a multiple of
// the grid G (a compute stream that cedes CUs), tiles [0, dp_tiles) are dealt
// whole (w, w + G, ...; dp_tiles = (T / G - 1) G) and the last G + T % G tiles
// are cut into 256-deep K units and dealt as G equal contiguous unit ranges.  A
// range spans at least one tile, so a tile has at most two contributors: each
// writes its partial accumulators to its slab (write-through sc1 stores), takes
// a ticket, and the second one adds the other's slab (sc1 loads) and runs the
// epilogue.  x + y == y + x: the result does not depend on who arrives last.
struct StreamK {
  float* slab;          // [2 G slots][4 waves][64 (a, b)][64 lanes] f32x4 = 256 KB per slot
  unsigned* cnt;        // [G + T % G][4 waves] tickets, zero between launches (the second arriver resets)
  uint32_t slab_bytes;
  int dp_tiles;
  int units;            // 256-deep K units per tile (every problem the same K)
};

struct GroupParams {
  Params g[GROUP_MAX];
  int tile_end[GROUP_MAX];
  int n;
  StreamK sk;
};
static_assert(sizeof(GroupParams) <= 4096, "kernel arguments");

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

NSTL_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p; }

#define G4_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define G4_SB() __builtin_amdgcn_sched_barrier(0)
#define G4_LGKM0()                                      \
  do {                                                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    G4_SB();                                            \
  } while (0)

// one 1 KB DMA piece: lane l writes bytes [16 l, 16 l + 16) of `lds`
NSTL_DEV void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, soff, 0, 0);
}

// Epilogue side data in LDS (round 5): a wave's bias columns (BF16, RELU_DROP)
// or dReLU keep-bit words (DRELU), DMA'd into its own 2 KB at the tile's start.
// Loaded in the epilogue instead, they sat behind the next tile's stage pieces
// in vmcnt order (issued during the last two steps), so the epilogue began with
// a wait for those, and the keep-bit words come cold from HBM.  Issued at the
// tile's start they are older than every stage piece a K step waits for, so they
// have landed by the epilogue, which reads them by inline asm (a plain LDS load
// would make the compiler wait for the DMA in flight).
constexpr int SIDE_W = 2048;             // per wave
constexpr int SIDE_LDS = 4 * SIDE_W;
// side layout: bias floats [128] (columns col0 ..); keep-bit words [hb][r0][16]
// (word (row block hb, row & 7 = r0, column group k of the wave's 16) at
// hb * 1024 + r0 * 128 + 8 k).  side_dma follows mask_word.

// Per-lane DMA source offsets of this wave's 8 pieces of one operand's stage,
// relative to the tile's first row (K-major) / column (MN-major): fixed per
// problem.  The tile's offset and the K advance go in the scalar offset.
// Full tiles only: no row clamping.
template <bool KMAJ>
NSTL_DEV void dma_lane_offsets(uint32_t (&vo)[8], int64_t ld, int wave, int lane) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int q = wave * 8 + s;
    if (KMAJ) {  // 128-byte rows (64 k), 8 rows per piece
      const int row = 8 * q + (lane >> 3), pc = lane & 7;
      const int lc = pc ^ ((row >> 1) & 7);
      vo[s] = (uint32_t)(((int64_t)row * ld + lc * 8) * 2);
    } else {     // 512-byte rows (256 m/n), 2 rows (k) per piece, ImgMN<512>
      const int row = 2 * q + (lane >> 5), pc = lane & 31;
      const int x = (row & 3) | (((row >> 3) & 1) << 2);
      const int lc = pc ^ (x << 1);
      vo[s] = (uint32_t)(((int64_t)row * ld + lc * 8) * 2);
    }
  }
}

// LDS fragment reads as inline asm: the compiler would otherwise wait vmcnt(0)
// before LDS reads that may alias an in-flight DMA (gemm.hip).  Offsets are
// immediates; the caller orders them with lgkmcnt + sched_barrier.
template <int OFF>
NSTL_DEV void ds_b128(bf16x8& f, uint32_t addr) {
  i32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  f = __builtin_bit_cast(bf16x8, v);
}
// the two transpose reads of an MN-major fragment: rows 8g + q and 8g + 4 + q of
// the image, 4 rows = 2048 bytes apart (the ImgMN<512> swizzle does not depend on
// row bit 2), so one address serves both
template <int OFF>
NSTL_DEV void ds_tr2(bf16x8& f, uint32_t a0) {
  i32x2_t v0, v1;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v0) : "v"(a0), "i"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v1) : "v"(a0), "i"(OFF + 2048));
  const bf16x4 b0 = __builtin_bit_cast(bf16x4, v0), b1 = __builtin_bit_cast(bf16x4, v1);
  f = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
}

// Per-lane LDS read addresses of one operand, slot 0.  K-major: one base per
// half-step (the swizzle makes h a lane-dependent offset), row block j at
// + 2048 j.  MN-major: 8 x 2 transpose-read addresses (block j), h at + 16 KB.
template <bool KMAJ>
struct RdAddr {
  uint32_t k[2];
  uint32_t t[8];
};
template <bool KMAJ>
NSTL_DEV void rd_addr(RdAddr<KMAJ>& r, uint32_t img, int blk0, int lane) {
  if (KMAJ) {
    const int row = blk0 + (lane & 15), sw = (row >> 1) & 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) r.k[h] = img + row * 128 + (((4 * h + (lane >> 4)) ^ sw) << 4);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.t[j] = img + ImgMN<512>::off(8 * g + q, (blk0 + 16 * j + 4 * pp) * 2);
  }
}
// Read slots of one half-step in issue order: A block 0..7, then B block 0..7; a
// K-major block is one ds_read_b128, an MN-major block two transpose reads (sub 0,
// 1).  Slot offsets are immediates (SO: the stage slot's byte offset).
template <bool AK, bool BKM>
constexpr int n_reads() { return (AK ? 8 : 16) + (BKM ? 8 : 16); }
template <int SO, bool KMAJ, int H, int J, int SUB>
NSTL_DEV void rd_one(bf16x8& f, const RdAddr<KMAJ>& r) {
  if constexpr (KMAJ) {
    i32x4_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(r.k[H]), "i"(SO + J * 2048));
    f = __builtin_bit_cast(bf16x8, v);
  } else {
    // two transpose reads, 4 rows = 2048 bytes apart, fill the halves of f
    i32x2_t v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(r.t[J]), "i"(SO + H * 16384 + SUB * 2048));
    const bf16x4 b = __builtin_bit_cast(bf16x4, v);
    if constexpr (SUB == 0) f = (bf16x8){b[0], b[1], b[2], b[3], f[4], f[5], f[6], f[7]};
    else f = (bf16x8){f[0], f[1], f[2], f[3], b[0], b[1], b[2], b[3]};
  }
}
// read slot R of the half-step (SOA / SOB: the A / B stage slot's byte offset)
template <bool AK, bool BKM, int SOA, int SOB, int H, int R>
NSTL_DEV void rd_slot(bf16x8 (&fa)[8], bf16x8 (&fb)[8], const RdAddr<AK>& ra, const RdAddr<BKM>& rb) {
  constexpr int NA = AK ? 8 : 16;
  if constexpr (R < NA) {
    constexpr int J = AK ? R : R / 2, SUB = AK ? 0 : R % 2;
    rd_one<SOA, AK, H, J, SUB>(fa[J], ra);
  } else {
    constexpr int Q = R - NA;
    constexpr int J = BKM ? Q : Q / 2, SUB = BKM ? 0 : Q % 2;
    rd_one<SOB, BKM, H, J, SUB>(fb[J], rb);
  }
}

// DMA state: buffer resources and per-lane offsets (per problem), the tile's
// scalar byte offsets, the bytes per 64-deep stage
struct Dma {
  __amdgpu_buffer_rsrc_t ra, rb;
  uint32_t va[8], vb[8];
  uint32_t ta, tb;
  uint32_t a_kb, b_kb;
};
template <bool AK, bool BKM>
NSTL_DEV void dma_lanes(Dma& d, const Params& p, int wave, int lane) {
  dma_lane_offsets<AK>(d.va, p.lda, wave, lane);
  dma_lane_offsets<BKM>(d.vb, p.ldb, wave, lane);
}
// the scalar part of a tile (resources rebuilt from the kernel arguments every
// tile: a resource chosen by a branch is not provably uniform, and the compiler
// would wrap every DMA in a readfirstlane loop)
// (ks: the first 256-deep K unit of a stream-K segment)
template <bool AK, bool BKM>
// live = false: the refill after a workgroup's last tile, with empty buffer
// ranges (its pieces return zeros without touching memory: no HBM / L2 traffic
// beside the last epilogue's stores, and the exit drain waits for less)
NSTL_DEV void dma_tile(Dma& d, const Params& p, int m0, int n0, int ks, bool live = true) {
  d.ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, live ? (int)p.a_bytes : 0, 0x00020000);
  d.rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, live ? (int)p.b_bytes : 0, 0x00020000);
  d.a_kb = AK ? 2 * BK : (uint32_t)(2 * BK * p.lda);
  d.b_kb = BKM ? 2 * BK : (uint32_t)(2 * BK * p.ldb);
  const uint32_t k0 = (uint32_t)ks * 4u;  // stages
  d.ta = __builtin_amdgcn_readfirstlane((AK ? (uint32_t)(m0 * p.lda * 2) : (uint32_t)(m0 * 2)) + k0 * d.a_kb);
  d.tb = __builtin_amdgcn_readfirstlane((BKM ? (uint32_t)(n0 * p.ldb * 2) : (uint32_t)(n0 * 2)) + k0 * d.b_kb);
}

// a tile's first MFMA on each block: C = 0 (an inline constant), so the epilogue
// need not zero the accumulators it reads (256 v_accvgpr_write per tile and wave)
NSTL_DEV void mma16z(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}

// every read slot of a half-step (slot 0, h = 0): the first tile's prologue
template <bool AK, bool BKM, int R>
NSTL_DEV void rd_all(bf16x8 (&fa)[8], bf16x8 (&fb)[8], const RdAddr<AK>& ra, const RdAddr<BKM>& rb) {
  if constexpr (R < n_reads<AK, BKM>()) {
    rd_slot<AK, BKM, 0, 0, 0, R>(fa, fb, ra, rb);
    rd_all<AK, BKM, R + 1>(fa, fb, ra, rb);
  }
}

// One half-step: 64 MFMAs on (ca, cb); if RD, the half-step's reads (16 to 32
// instructions: read slots, rd_slot) into (na, nb) spread over MFMAs 1 .. 46 (read
// slot r after MFMA 1 + 46 r / R: each transpose read gets a gap of its own as far
// as the count allows, and the last read has 17 MFMAs to land before the closing
// lgkmcnt(0)).  DMAM: the stage DMA this half-step issues -- 0 none; 1 all 16
// pieces of the stage after MFMAs 2, 6, ..., 62 (A pieces to adst, B pieces to
// bdst, stage offsets sa / sb; the two-stage ring); 2 the 8 A pieces, 3 the 8 B
// pieces, after MFMAs 2, 10, ..., 58 (the A3/B2 ring: one operand per half-step).
// RSOA / RSOB: the read slots' byte offsets.
// DBG (timing experiments only, wrong results): 1 no DMA, 2 no reads, 8 no MFMA.
// (experiments, profiles/r4_gemm4_read_spread.txt: DBG & 256 spreads the reads over
// MFMAs 1 .. 56, DBG & 512 over 1 .. 32, DBG & 1024 over 1 .. 24)
template <bool AK, bool BKM, int RSOA, int RSOB, int RH, int I, int R, int SPAN = 46>
NSTL_DEV void rd_after(bf16x8 (&na)[8], bf16x8 (&nb)[8], const RdAddr<AK>& ra, const RdAddr<BKM>& rb) {
  constexpr int NR = n_reads<AK, BKM>();
  if constexpr (R < NR) {
    if constexpr (1 + (SPAN * R) / NR == I) {
      rd_slot<AK, BKM, RSOA, RSOB, RH, R>(na, nb, ra, rb);
      G4_SB();
      rd_after<AK, BKM, RSOA, RSOB, RH, I, R + 1, SPAN>(na, nb, ra, rb);
    } else if constexpr (1 + (SPAN * R) / NR < I) {
      rd_after<AK, BKM, RSOA, RSOB, RH, I, R + 1, SPAN>(na, nb, ra, rb);
    }
  }
}
template <bool AK, bool BKM, bool RD, int RSOA, int RSOB, int RH, int DMAM, int DBG, bool Z = false, int I = 0>
NSTL_DEV void half_step(f32x4 (&acc)[8][8], const bf16x8 (&ca)[8], const bf16x8 (&cb)[8], bf16x8 (&na)[8],
                        bf16x8 (&nb)[8], const RdAddr<AK>& ra, const RdAddr<BKM>& rb, const Dma& d, char* adst,
                        char* bdst, uint32_t sa, uint32_t sb) {
  if constexpr (I < 64) {
    if constexpr (!(DBG & 8)) {
      if constexpr (Z) mma16z(acc[I >> 3][I & 7], cb[I & 7], ca[I >> 3]);
      else mma16(acc[I >> 3][I & 7], cb[I & 7], ca[I >> 3]);
    }
    G4_SB();
    if constexpr (RD && !(DBG & 2))
      rd_after<AK, BKM, RSOA, RSOB, RH, I, 0, (DBG & 256) ? 56 : (DBG & 512) ? 32 : (DBG & 1024) ? 24 : 46>(na, nb, ra,
                                                                                                       rb);
    if constexpr ((DMAM == 2 || DMAM == 3) && !(DBG & 1) && (I & 7) == ((DBG & 2048) ? 6 : 2)) {
      constexpr int q = I >> 3;
      if constexpr (DMAM == 2) dma16(d.ra, adst + q * 1024, d.va[q], d.ta + sa);
      else dma16(d.rb, bdst + q * 1024, d.vb[q], d.tb + sb);
      G4_SB();
    }
    // the 16 DMA pieces: after MFMAs 2, 6, ..., 62, or (experiments) after MFMAs
    // 0 .. 15 (DBG & 16) / 0, 2, ..., 30 (DBG & 32): issued earlier in h = 1; after
    // MFMAs 32, 34, ..., 62 (DBG & 64) / 47 .. 62 (DBG & 128): later
    constexpr bool DMA_HERE = (DBG & 16)    ? I < 16
                              : (DBG & 32)  ? (I < 32 && (I & 1) == 0)
                              : (DBG & 64)  ? (I >= 32 && (I & 1) == 0)
                              : (DBG & 128) ? (I >= 47 && I < 63)
                                            : (I & 3) == 2;
    if constexpr (DMAM == 1 && !(DBG & 1) && DMA_HERE) {
      constexpr int q = (DBG & 16)    ? I
                        : (DBG & 32)  ? I >> 1
                        : (DBG & 64)  ? (I - 32) >> 1
                        : (DBG & 128) ? I - 47
                                      : I >> 2;
      if constexpr (q < 8) dma16(d.ra, adst + q * 1024, d.va[q], d.ta + sa);
      else dma16(d.rb, bdst + (q - 8) * 1024, d.vb[q - 8], d.tb + sb);
      G4_SB();
    }
    half_step<AK, BKM, RD, RSOA, RSOB, RH, DMAM, DBG, Z, I + 1>(acc, ca, cb, na, nb, ra, rb, d, adst, bdst, sa, sb);
  }
}

// grouped tile order over XCD-contiguous id ranges (as the ring kernel)
NSTL_DEV void tile_coords(int id, int nt_m, int nt_n, int& m0, int& n0) {
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * nt_n;
  const int first_m = (id / per_group) * GROUP_M;
  const int gm = min(nt_m - first_m, GROUP_M);
  const int in_g = id % per_group;
  m0 = (first_m + in_g % gm) * TILE;
  n0 = (in_g / gm) * TILE;
}

// (lo, hi) -> two bf16 (round to nearest even) in one word: ONE v_cvt_pk_bf16_f32
// (two scalar casts cost two conversions, a shift and an SDWA or per pair: a
// third of the plain epilogue's vector instructions)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
NSTL_DEV uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
// the two bf16 of a packed word back to f32 (exact)
NSTL_DEV float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
NSTL_DEV float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
// dropout keep masks of an element pair from its hash: all ones where the 16-bit
// uniform is >= thresh (thresh in 1 .. 65536), else 0 -- the compare of
// nstl_keep2_32 as integer arithmetic, so the select is an AND (a compare writes
// VCC, and every VCC-reading select behind it costs a hazard s_nop)
// (the shift and the min below are asm: written in C the compiler turns them back
// into a compare and a select)
NSTL_DEV uint32_t asr31(uint32_t x) {
  uint32_t r;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(r) : "v"(x));
  return r;
}
NSTL_DEV uint32_t min1(uint32_t x) {
  uint32_t r;
  asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(x));
  return r;
}
NSTL_DEV uint32_t keep_lo_mask(uint32_t h, uint32_t thresh) { return asr31(thresh - 1u - (h & 0xFFFFu)); }
NSTL_DEV uint32_t keep_hi_mask(uint32_t h, uint32_t thresh) { return asr31(thresh - 1u - (h >> 16)); }
NSTL_DEV float and_mask(float x, uint32_t m) { return __uint_as_float(__float_as_uint(x) & m); }
// ReLU-mask bits of a packed pair of non-negative bf16 (after max(., 0)): bit 0
// for the low element, bit 1 for the high one, set where the stored value is
// not zero (+0 or -0) -- "(bf16)v > 0" for v >= 0
NSTL_DEV uint32_t pos_bits2(uint32_t w) {
  const uint32_t t = w & 0x7FFF7FFFu;
  return min1(t & 0xFFFFu) | (min1(t >> 16) << 1);
}

// ReLU keep&positive bits in the ring kernel's word layout (gemm.hip
// relu_mask_index): word ((row >> 6) * 8 + (row & 7)) * ceil(N / 8) + col / 8,
// byte (row & 63) >> 3, bit col & 7.  Lane (g, c) of acc[a][b] holds rows
// 16a + c: byte 2(a & 3) + (c >> 3) of word (row block a >> 2, r0 = c & 7, column
// group 2b + (g >> 1)), bits 4(g & 1) .. +3.
NSTL_DEV int64_t mask_word(int N, int row, int col) {
  return ((int64_t)(row >> 6) * 8 + (row & 7)) * ((N + 7) >> 3) + (col >> 3);
}

// the fp8 kernel's side area (SC): its row and column scales first (1 KB each,
// the wave's 128 in the first 512 B), then the bias / keep-bit words
constexpr int SIDE_SC_OFF = 2048;
constexpr int SIDE_W_SC = SIDE_SC_OFF + SIDE_W;

// the wave's side data of its 128 x 128 block (row0, col0) (see SIDE_W); SC: the
// fp8 scales too, and the rest at SIDE_SC_OFF
template <int EM, bool SC = false>
NSTL_DEV void side_dma(const Params& p, char* side, int row0, int col0, int lane) {
  if constexpr (SC) {
    // 128 row scales from lanes 0..31 (lanes 32..63: the next 128, zeros past M)
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.a_scale, 0, (int)((uint32_t)p.M * 4u), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)side, 16, (uint32_t)lane * 16u,
                                             __builtin_amdgcn_readfirstlane((uint32_t)row0 * 4u), 0, 0);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.b_scale, 0, (int)((uint32_t)p.N * 4u), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)(side + 1024), 16, (uint32_t)lane * 16u,
                                             __builtin_amdgcn_readfirstlane((uint32_t)col0 * 4u), 0, 0);
    side += SIDE_SC_OFF;
  }
  if constexpr (EM == EM_DRELU) {
    // 2 x 8 rows of 16 words (128 B): lane l of piece j loads words 2 (l & 7),
    // + 1 of row (j, l >> 3)
    const uint32_t wpr = (uint32_t)((p.N + 7) >> 3);  // words per mask row
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.relu_mask, 0, (int)((uint32_t)(p.M >> 6) * 8u * wpr * 8u), 0x00020000);
    // the lane's part in the vector offset, the block's in the scalar one
    const uint32_t vo = ((uint32_t)(lane >> 3) * wpr + 2u * (uint32_t)(lane & 7)) * 8u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t so =
          __builtin_amdgcn_readfirstlane((((uint32_t)((row0 >> 6) + j) * 8u) * wpr + (uint32_t)(col0 >> 3)) * 8u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(side + j * 1024), 16, vo, so, 0, 0);
    }
  } else if (p.bias != nullptr) {
    // 128 floats from lanes 0..31; lanes 32..63 read the next 128 (zeros past N)
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, 0, (int)((uint32_t)p.N * 4u), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)side, 16, (uint32_t)lane * 16u,
                                             __builtin_amdgcn_readfirstlane((uint32_t)col0 * 4u), 0, 0);
  }
}

// RoPE tables in LDS (EM_ROPE): row t holds rope_dim / 2 (cos, sin) pairs,
// 16-byte chunk k (pairs 2k, 2k + 1) at k ^ (t & m): the 16 lanes of a read
// (16 consecutive positions, one chunk) hit 16 distinct bank slots when the row
// has 16 or more chunks.  m (rope_swz) keeps the XOR inside the row: the low bit
// of the chunk count, at most 16, minus one (rope_dim 64: 15; 32: 7; 96: 7; a
// chunk count with bit 0 set: 0, no swizzle).  With m = 15 and fewer than 16
// chunks, rows wrote into their neighbours' slots.
NSTL_DEV int rope_swz(int rope_dim) {
  const int chunks = rope_dim >> 2;
  const int low = chunks & -chunks;
  return (low < 16 ? low : 16) - 1;
}
NSTL_DEV int rope_off(int t, int chunk, int row_bytes, int swz) { return t * row_bytes + ((chunk ^ (t & swz)) << 4); }
// the bf16 table: 8-byte chunks
NSTL_DEV int rope_off8(int t, int chunk, int row_bytes, int swz) { return t * row_bytes + ((chunk ^ (t & swz)) << 3); }

// An accumulator tile read out of the AGPRs at the point of use ...  Left to the
// compiler, the epilogue's VALU uses split the accumulators' live range at the
// epilogue entry: all 256 are copied to VGPRs at once and the DMA offsets and
// next fragments spill around them.
// ZW: ... and zeroed in place for the next tile.  Kernels whose tiles start with
// C = 0 MFMAs (mma16z: the dX / dW layouts and fp8) read without zeroing (256
// fewer v_accvgpr_write per tile and wave); the K-major-B (forward) and stream-K
// instantiations keep the zeroing: with C = 0 their register allocation spilled.
// ZW 2: zeroed by one MFMA on zero operands (0 x 0 + 0) instead of four
// v_accvgpr_write (half the issue cycles; the next reader of x is the next tile's
// first MFMA, far past any MFMA-result hazard window) -- the forward
// instantiations; 1: the four writes (stream-K: with the MFMA form it spilled)
// z: the zero operand of the ZW 2 form, from zero_operand() -- written by asm
// followed by wait states of its own: the compiler cannot see that the asm below
// is an MFMA, so it would not separate a VALU write of a zero it materialised
// itself from the MFMA's read (that missing hazard wait gave NaN)
NSTL_DEV s16x4 zero_operand() {
  uint64_t zz;
  asm volatile("v_mov_b64 %0, 0\n\ts_nop 4" : "=v"(zz));
  return __builtin_bit_cast(s16x4, zz);
}
template <int ZW = 1>
NSTL_DEV f32x4 rd_acc(f32x4& x, s16x4 z = {}) {
  float r0, r1, r2, r3;
  if constexpr (ZW == 2) {
    asm volatile(
        "v_accvgpr_read_b32 %0, %4\n\t"
        "v_accvgpr_read_b32 %1, %5\n\t"
        "v_accvgpr_read_b32 %2, %6\n\t"
        "v_accvgpr_read_b32 %3, %7"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
        : "a"(x[0]), "a"(x[1]), "a"(x[2]), "a"(x[3]));
    asm volatile("v_mfma_f32_16x16x16_bf16 %0, %1, %1, 0" : "+a"(x) : "v"(z));
  } else if constexpr (ZW == 1) {
    asm volatile(
        "v_accvgpr_read_b32 %0, %4\n\t"
        "v_accvgpr_read_b32 %1, %5\n\t"
        "v_accvgpr_read_b32 %2, %6\n\t"
        "v_accvgpr_read_b32 %3, %7\n\t"
        "v_accvgpr_write_b32 %4, 0\n\t"
        "v_accvgpr_write_b32 %5, 0\n\t"
        "v_accvgpr_write_b32 %6, 0\n\t"
        "v_accvgpr_write_b32 %7, 0"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "+a"(x[0]), "+a"(x[1]), "+a"(x[2]), "+a"(x[3]));
  } else {
    asm volatile(
        "v_accvgpr_read_b32 %0, %4\n\t"
        "v_accvgpr_read_b32 %1, %5\n\t"
        "v_accvgpr_read_b32 %2, %6\n\t"
        "v_accvgpr_read_b32 %3, %7"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
        : "a"(x[0]), "a"(x[1]), "a"(x[2]), "a"(x[3]));
  }
  return (f32x4){r0, r1, r2, r3};
}

// read without zeroing (a stream-K partial, kept for the sum)
NSTL_DEV f32x4 rd_acc_keep(const f32x4& x) {
  float r0, r1, r2, r3;
  asm volatile(
      "v_accvgpr_read_b32 %0, %4\n\t"
      "v_accvgpr_read_b32 %1, %5\n\t"
      "v_accvgpr_read_b32 %2, %6\n\t"
      "v_accvgpr_read_b32 %3, %7"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "a"(x[0]), "a"(x[1]), "a"(x[2]), "a"(x[3]));
  return (f32x4){r0, r1, r2, r3};
}
// x += y in place
NSTL_DEV void add_acc(f32x4& x, const f32x4 y) {
  float t0, t1, t2, t3;
  asm volatile(
      "v_accvgpr_read_b32 %0, %4\n\t"
      "v_accvgpr_read_b32 %1, %5\n\t"
      "v_accvgpr_read_b32 %2, %6\n\t"
      "v_accvgpr_read_b32 %3, %7\n\t"
      "v_add_f32 %0, %0, %8\n\t"
      "v_add_f32 %1, %1, %9\n\t"
      "v_add_f32 %2, %2, %10\n\t"
      "v_add_f32 %3, %3, %11\n\t"
      "v_accvgpr_write_b32 %4, %0\n\t"
      "v_accvgpr_write_b32 %5, %1\n\t"
      "v_accvgpr_write_b32 %6, %2\n\t"
      "v_accvgpr_write_b32 %7, %3"
      : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+a"(x[0]), "+a"(x[1]), "+a"(x[2]), "+a"(x[3])
      : "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]));
}

// The work of workgroup w: its whole tiles, then its stream-K unit range.  A
// segment is tile t, K units [ks, ke) (ke < 0: the whole tile, any K).
struct Seg {
  int t, ks, ke;
};
// The tail's unit ranges go to the workgroups in XCD-contiguous order (rank =
// xcd_remap(w)): the workgroups of one XCD take consecutive tiles, which
// tile_coords lays out as a patch sharing A and B panels in that XCD's L2 (dealt
// in workgroup order, an XCD's tiles were scattered over the whole output and
// the GEMM ran 40-70 % slower).  Slab slots and the hand-off partner go by rank.
struct Walker {
  int t_dp, G, dp_tiles, U;
  int rank;      // position of this workgroup's range in the tail
  int pos, end;  // units: at most 2 G tiles x 64 (K = 16384) in the tail
  NSTL_DEV void init(const GroupParams& gp, int T, int w, int G_, bool sk) {
    G = G_;
    t_dp = w;
    rank = w;
    if (sk) {
      dp_tiles = gp.sk.dp_tiles;
      U = gp.sk.units;
      if (G % 8 == 0) rank = xcd_remap(w, G);
      const int I = (T - dp_tiles) * U;
      pos = rank * I / G;
      end = (rank + 1) * I / G;
    } else {
      dp_tiles = T;
      U = 1;
      pos = end = 0;
    }
  }
  NSTL_DEV bool next(Seg& s) {
    if (t_dp < dp_tiles) {
      s.t = t_dp;
      s.ks = 0;
      s.ke = -1;
      t_dp += G;
      return true;
    }
    if (pos >= end) return false;
    s.t = dp_tiles + pos / U;
    s.ks = pos % U;
    s.ke = s.ks + end - pos < U ? s.ks + end - pos : U;
    pos += s.ke - s.ks;
    return true;
  }
};

// The stream-K hand-off at the end of a segment, per wave (a wave's 128 x 128
// block is its own: slab part, ticket and epilogue).  Returns whether this wave
// finishes the block: a whole tile, or the second contributor (its accumulators
// then hold the sum); the first contributor's epilogue runs with its stores off
// (it zeroes the accumulators for the next segment).  The tile's head [0, ks)
// belongs to the previous range's workgroup (its last segment, slot
// 2 (w - 1) + 1; w: the range's rank), its tail to the next one's (first
// segment, slot 2 (w + 1)).
// One straight-line pass whatever the case -- a branch over the accumulators
// splits their live ranges and spills: stores and loads that do not apply go
// through an empty buffer range (dropped; loads return 0).
NSTL_DEV bool sk_handoff(const StreamK& sk, f32x4 (&acc)[8][8], const Seg& s, int w, int wave, int lane) {
  const bool part = !(s.ke < 0 || (s.ks == 0 && s.ke == sk.units));
  const bool tail = s.ks > 0;
  const uint32_t mine = (uint32_t)(tail ? 2 * w : 2 * w + 1), other = (uint32_t)(tail ? 2 * w - 1 : 2 * w + 2);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)sk.slab, 0, part ? (int)sk.slab_bytes : 0, 0x00020000);
  const uint32_t wsoff = (uint32_t)wave * 65536u;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const f32x4 v = rd_acc_keep(acc[a][b]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), r, lane * 16 + (a * 8 + b) * 1024,
                                             mine * 262144u + wsoff, 16 /* sc1: write-through */);
      G4_SB();
    }
  G4_VMCNT(0);  // the slab part is written through before the ticket
  unsigned old = 0;
  if (part && lane == 0) {
    unsigned* c = sk.cnt + 4 * (s.t - sk.dp_tiles) + wave;
    old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 1u) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool last = __builtin_amdgcn_readfirstlane(old) == 1u;
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void*)sk.slab, 0, part && last ? (int)sk.slab_bytes : 0, 0x00020000);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    i32x4_t y[8];
#pragma unroll
    for (int b = 0; b < 8; ++b)
      y[b] = __builtin_amdgcn_raw_buffer_load_b128(rl, lane * 16 + (a * 8 + b) * 1024, other * 262144u + wsoff,
                                                   16 /* sc1 */);
#pragma unroll
    for (int b = 0; b < 8; ++b) add_acc(acc[a][b], __builtin_bit_cast(f32x4, y[b]));
    G4_SB();  // one row of blocks (8 loads) in flight at a time
  }
  return !part || last;
}

// ---------------------------------------------------------------------------
// Epilogues, from registers.  row0 / col0: the wave's 128 x 128 block.
// bf16 outputs: per (a, pair of column blocks bp, bp + 1) the elementwise math
// runs on the accumulator layout (lane: 4 columns of block bp and 4 of bp + 1,
// row 16a + c), then a permlane16 swap of the packed pairs gives each lane 8
// consecutive columns: one 16-byte store (16 rows x 64 B per wave instruction).
// No epilogue loads from memory after its first store (vmcnt retires in issue
// order, so such a load would wait for the stores before it): the inputs are
// loaded first (bias, dReLU mask words) or read from LDS (RoPE tables).
// SC (the fp8 kernel): C = a_scale[row] b_scale[col] acc, applied as (acc (a_scale
// alpha)) b_scale -- the fp8 ring kernel's order -- before the bias.
template <int EM, bool SC = false, int EDBG = 0, int ZW = 1, bool SIDE = false>
NSTL_DEV void epilogue(const Params& p, f32x4 (&acc)[8][8], int row0, int col0, int lane, int wave, int tile_id,
                       const char* rope_lds, bool fin = true, const char* side = nullptr) {
  const int g = lane >> 4, c = lane & 15, odd = g & 1;
  const float alpha = p.alpha;
  s16x4 z = {};
  if constexpr (ZW == 2) z = zero_operand();
  float rsc[8], csc[8][4];  // SC: the lane's row scales (times alpha) and column scales
  if constexpr (SC && SIDE) {  // side_dma's copies (SIDE_SC_OFF), read by asm
    const uint32_t ra = lds_addr(side + 4 * c), cb = lds_addr(side + 1024 + 16 * g);
    float rv[8];
    f32x4 cv[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(rv[a]) : "v"(ra), "i"(64 * a));
#pragma unroll
    for (int b = 0; b < 8; ++b) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(cv[b]) : "v"(cb), "i"(64 * b));
    G4_LGKM0();
#pragma unroll
    for (int a = 0; a < 8; ++a) rsc[a] = rv[a] * alpha;
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) csc[b][e] = cv[b][e];
    side += SIDE_SC_OFF;
  } else if constexpr (SC) {
#pragma unroll
    for (int a = 0; a < 8; ++a) rsc[a] = p.a_scale[row0 + 16 * a + c] * alpha;
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) csc[b][e] = p.b_scale[col0 + 16 * b + 4 * g + e];
  }
  if constexpr (EM == EM_F32) {
    // f32 out: lane stores its 4 columns (16 B); sum of squares of the stored
    // values -> sq_part (the clip norm's partial, training_utils.py:73)
    float ssq = 0.f;
    // stores through a buffer whose range is empty when this wave does not finish
    // the block (a stream-K first contributor): no branch around them
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.C, 0, fin ? (int)((uint32_t)p.M * (uint32_t)p.ldc * 4u) : 0, 0x00020000);
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const uint32_t crow = ((uint32_t)(row0 + 16 * a + c) * (uint32_t)p.ldc + col0 + 4 * g) * 4u;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        f32x4 v;
        if constexpr (SC) {
          v = rd_acc<ZW>(acc[a][b], z) * rsc[a];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= csc[b][e];
        } else {
          v = rd_acc<ZW>(acc[a][b], z) * alpha;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) ssq += v[e] * v[e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, v), rc, crow + 64 * b, 0, 0);
        G4_SB();
      }
    }
    // the sum is formed unconditionally (a conditional one kept every stored value
    // alive until after the stores, and spilled them)
    const double tsum = wave_sum_d((double)ssq);
    if (fin && p.sq_part != nullptr && lane == 0) {
      p.sq_part[tile_id * 8 + 2 * wave] = (float)tsum;
      p.sq_part[tile_id * 8 + 2 * wave + 1] = 0.f;
    }
  } else {
    f32x4 bias[8];
    if constexpr (SIDE && EM != EM_DRELU) {  // side_dma's copy (see SIDE_W)
      if (p.bias != nullptr) {
        const uint32_t ba = lds_addr(side + 16 * g);
#pragma unroll
        for (int b = 0; b < 8; ++b) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bias[b]) : "v"(ba), "i"(64 * b));
        G4_LGKM0();
      } else {
#pragma unroll
        for (int b = 0; b < 8; ++b) bias[b] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bias[b][e] = (EM != EM_DRELU && p.bias != nullptr) ? p.bias[col0 + 16 * b + 4 * g + e] : 0.f;
    }
    const uint32_t seed_term = nstl_seed_term(p.seed);
    const bool rmask = (EM == EM_RELU_DROP || EM == EM_DRELU) && p.relu_mask != nullptr;
    // mask nibbles: [row block hb][column block b], 4 rows (a & 3) x 4 bits
    uint32_t mbits[2][8];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int b = 0; b < 8; ++b) mbits[hb][b] = 0;
    if (EM == EM_DRELU) {
      // side_dma's copy: word (hb, c & 7, 2b + (g >> 1)); a row block's 8 reads, one wait
      const uint32_t ma = lds_addr(side + (c & 7) * 128 + (g >> 1) * 8);
      // the lane's nibble of each word: byte 2 a2 + (c >> 3), bits 4 (g & 1)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        i32x2_t sw[8];
        if constexpr (SIDE) {
#pragma unroll
          for (int b = 0; b < 8; ++b)
            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(sw[b]) : "v"(ma), "i"(hb * 1024 + 16 * b));
          G4_LGKM0();
        }
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint64_t w = SIDE ? (((uint64_t)(uint32_t)sw[b][1] << 32) | (uint32_t)sw[b][0])
                                  : p.relu_mask[mask_word(p.N, row0 + 64 * hb + c, col0 + 16 * b + 4 * g)];
          uint32_t s = 0;
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2) s |= ((uint32_t)(w >> (8 * (2 * a2 + (c >> 3)) + 4 * odd)) & 0xF) << (4 * a2);
          mbits[hb][b] = s;
        }
      }
    }
    float csum[8][4];
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[b][e] = 0.f;
    const int rope_rb = p.rope_dim * 4;  // bytes per table row in LDS
    const int rswz = rope_swz(p.rope_dim);
    // RoPE: the lane's table chunk per column block (col % rope_dim) / 4, once
    // per tile (a power-of-two rope_dim, the production case: a mask)
    int rchunk[8];
    if constexpr (EM == EM_ROPE) {
      const bool pow2 = (p.rope_dim & (p.rope_dim - 1)) == 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int col = col0 + 16 * b + 4 * g;
        rchunk[b] = (pow2 ? col & (p.rope_dim - 1) : col % p.rope_dim) >> 2;
      }
    }
    bf16* const cbase = (bf16*)p.C + (int64_t)(row0 + c) * p.ldc + col0;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int row = row0 + 16 * a + c;
      bf16* crow = cbase + (int64_t)(16 * a) * p.ldc;
      // position of the row (a power-of-two T, the production case: a mask)
      const int t = EM != EM_ROPE ? 0 : ((p.rope_T & (p.rope_T - 1)) == 0 ? row & (p.rope_T - 1) : row % p.rope_T);
      // RoPE: the row's 8 table reads issued together (one at the point of use
      // exposed an LDS round trip per 4 outputs)
      // Read by inline asm: a plain LDS load here may alias the next tile's stage
      // DMA in flight, so the compiler put vmcnt(0) in front of every row's reads
      // -- a wait for the stage pieces and for every store of the rows before.
      f32x4 rcs[8];
      if constexpr (EM == EM_ROPE) {
        if (p.rope_bf16) {  // (cos, sin) pairs as bf16 (8-byte chunks): the fp8 kernel at T = 256
          i32x2_t w[8];
#pragma unroll
          for (int b = 0; b < 8; ++b)
            asm volatile("ds_read_b64 %0, %1" : "=v"(w[b]) : "v"(lds_addr(rope_lds + rope_off8(t, rchunk[b], p.rope_dim * 2, rswz))));
          G4_LGKM0();
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const uint32_t x = (uint32_t)w[b][0], y = (uint32_t)w[b][1];
            rcs[b] = (f32x4){__uint_as_float(x << 16), __uint_as_float(x & 0xFFFF0000u), __uint_as_float(y << 16),
                             __uint_as_float(y & 0xFFFF0000u)};
          }
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b)
            asm volatile("ds_read_b128 %0, %1" : "=v"(rcs[b]) : "v"(lds_addr(rope_lds + rope_off(t, rchunk[b], rope_rb, rswz))));
          G4_LGKM0();
        }
      }
#pragma unroll
      for (int bp = 0; bp < 8; bp += 2) {
        f32x4 uv[2] = {rd_acc<ZW>(acc[a][bp], z), rd_acc<ZW>(acc[a][bp + 1], z)};
        if (!fin) {  // a stream-K first contributor: only the zeroing reads above
          G4_SB();
          continue;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int b = bp + s;
          const int col = col0 + 16 * b + 4 * g;
          f32x4 v;
          if constexpr (SC) {
            v = uv[s] * rsc[a];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= csc[b][e];
          } else {
            v = uv[s] * alpha;
          }
          v += bias[b];  // two v_pk_add_f32
          if constexpr (EM == EM_RELU_DROP) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            if (p.thresh) {
              const uint32_t pair = (uint32_t)row * (uint32_t)(p.N >> 1) + (uint32_t)(col >> 1);
#pragma unroll
              for (int e = 0; e < 4; e += 2) {
                const uint32_t h = nstl_pair_hash32(seed_term, pair + (e >> 1));
                v[e] = and_mask(v[e] * p.inv_keep, keep_lo_mask(h, p.thresh));
                v[e + 1] = and_mask(v[e + 1] * p.inv_keep, keep_hi_mask(h, p.thresh));
              }
            }
          } else if constexpr (EM == EM_ROPE) {
            // products rounded before the add, as the reference's f32 elementwise
            // rotation (model.py:60-83); no FMA contraction
#pragma clang fp contract(off)
            if (col < p.rope_cols) {
              // pairs (col, col + 1), (col + 2, col + 3): chunk (col % rope_dim) / 4
              const f32x4 cs = rcs[b];
              const float x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
              v[0] = x0 * cs[0] - x1 * cs[1];
              v[1] = x0 * cs[1] + x1 * cs[0];
              v[2] = x2 * cs[2] - x3 * cs[3];
              v[3] = x2 * cs[3] + x3 * cs[2];
            }
          } else if constexpr (EM == EM_DRELU) {
            const uint32_t nib = mbits[a >> 2][b] >> (4 * (a & 3));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = and_mask(v[e] * p.inv_keep, asr31(nib << (31 - e)));
          }
          uv[s] = v;
        }
        const uint32_t x0 = pack_bf16x2(uv[0][0], uv[0][1]), x1 = pack_bf16x2(uv[0][2], uv[0][3]);
        const uint32_t y0 = pack_bf16x2(uv[1][0], uv[1][1]), y1 = pack_bf16x2(uv[1][2], uv[1][3]);
        if constexpr (EM == EM_RELU_DROP) {
          if (rmask) {  // keep&positive bits of what is stored
            mbits[a >> 2][bp] |= (pos_bits2(x0) | (pos_bits2(x1) << 2)) << (4 * (a & 3));
            mbits[a >> 2][bp + 1] |= (pos_bits2(y0) | (pos_bits2(y1) << 2)) << (4 * (a & 3));
          }
        }
        if constexpr (EM == EM_DRELU) {
          if (p.colsum_part != nullptr) {  // sum what is stored (the bf16 values, exactly)
            csum[bp][0] += bf16_lo(x0); csum[bp][1] += bf16_hi(x0);
            csum[bp][2] += bf16_lo(x1); csum[bp][3] += bf16_hi(x1);
            csum[bp + 1][0] += bf16_lo(y0); csum[bp + 1][1] += bf16_hi(y0);
            csum[bp + 1][2] += bf16_lo(y1); csum[bp + 1][3] += bf16_hi(y1);
          }
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        // EDBG & 1 (experiment: timing only): the stores skipped, the math kept
        if (!(EDBG & 1) || p.ldc < 0) *(uint4*)(crow + 16 * (bp + odd) + 4 * (g - odd)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        G4_SB();  // one (a, bp) group at a time: hoisting the accumulator reads spills
      }
    }
    if (EM == EM_RELU_DROP && rmask) {
      // word (hb, r0 = c & 7, column group 2b + (g >> 1)) = OR over the 4 lanes
      // (g, g ^ 1) x (c, c ^ 8) of their nibbles at byte 2 a2 + (c >> 3), bit 4 (g & 1)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint32_t s = mbits[hb][b];
          uint64_t w = 0;
#pragma unroll
          for (int a2 = 0; a2 < 4; ++a2) w |= (uint64_t)((s >> (4 * a2)) & 0xF) << (8 * (2 * a2 + (c >> 3)) + 4 * odd);
          uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
          lo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0x128, 0xF, 0xF, false);  // c ^ 8 (row_ror:8)
          hi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0x128, 0xF, 0xF, false);
          const auto slo = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // g ^ 1
          const auto shi = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
          lo = slo[0] | slo[1];
          hi = shi[0] | shi[1];
          if (fin && c < 8 && odd == 0)
            p.relu_mask[mask_word(p.N, row0 + 64 * hb + c, col0 + 16 * b + 4 * g)] = ((uint64_t)hi << 32) | lo;
        }
    }
    if (EM == EM_DRELU && p.colsum_part != nullptr) {
      // fold the 16 lanes c of each column inside the 16-lane row (DPP), then lane
      // c == 0 writes the wave's 128-row partial of its 8 x 4 columns
#pragma unroll
      for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = csum[b][e];
          x += NSTL_DPP(x, 0xB1);   // quad_perm [1, 0, 3, 2]
          x += NSTL_DPP(x, 0x4E);   // quad_perm [2, 3, 0, 1]
          x += NSTL_DPP(x, 0x141);  // row_half_mirror
          x += NSTL_DPP(x, 0x140);  // row_mirror
          csum[b][e] = x;
        }
      if (fin && c == 0) {
        float* dst = p.colsum_part + (int64_t)(row0 >> 7) * p.N + col0 + 4 * g;
#pragma unroll
        for (int b = 0; b < 8; ++b) *(f32x4*)(dst + 16 * b) = (f32x4){csum[b][0], csum[b][1], csum[b][2], csum[b][3]};
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The persistent kernel.  Preconditions (host-checked): bf16 operands; every
// problem's M, N multiples of 256, K a multiple of 128 with K >= 256; 16-byte
// aligned rows; operand extents < 2^31 bytes; EM_ROPE: T * rope_dim * 4 <=
// ROPE_LDS and rope_dim % 4 == 0; EM_F32: beta 0.  Tiles of up to 16 problems
// (gp.tile_end; one problem: n = 1).
//
// R3 (round 5): the stage DMA spread over both half-steps.  With two 64 KB
// stages, stage s + 2 can only go into the slot stage s vacates, i.e. after the
// mid-step barrier: all 16 pieces of a step sat in h = 1, beside that half's
// fragment reads, while h = 0 issued none (the pieces' issue slots, not their
// latency, cost the MFMA pipe: DESIGN.md section 4).  R3 gives A a ring of
// three 32 KB slots and B a ring of two (160 KB, the whole LDS; not with the RoPE
// table): in h = 0 of step s the 8 A pieces of stage s + 2 go into the A slot of
// stage s - 1 (free since step s - 1's barrier), in h = 1 the 8 B pieces into
// the B slot of stage s (free since this step's barrier).  The counted wait
// before the barrier then leaves this step's 8 A pieces in flight.  A's slot
// has period 3, so its read addresses carry the slot (one add per address and
// step: 2 for a K-major A, 8 for an MN-major one); B's slot stays an immediate.
template <bool AK, bool BKM, int EM, bool GROUPED, int DBG = 0, bool SK = false, int R3 = 0>
__global__ __launch_bounds__(NT, 1) void gemm4_kernel(const GroupParams gp) {
  // R3 1: A has the ring of three (DMA'd in h = 0), B the ring of two; 2: the reverse
  constexpr bool A3 = R3 == 1, B3 = R3 == 2;
  static_assert(!(R3 && EM == EM_ROPE), "the 3 + 2 ring fills the LDS: no room for the RoPE table");
  // epilogue side data (SIDE_W): not with the 3 + 2 ring (no LDS left) or RoPE,
  // nor for the ReLU-dropout epilogue on an MN-major B (one VGPR short: spills)
  constexpr bool SIDE = !R3 && (EM == EM_BF16 || (EM == EM_RELU_DROP && BKM) || EM == EM_DRELU) && !(DBG & 16384);
  constexpr int SMEM_ALL = R3 ? 5 * OPS : SMEM + (EM == EM_ROPE ? ROPE_LDS : 0) + (SIDE ? SIDE_LDS : 0);
  constexpr int B_BASE = A3 ? 3 * OPS : 2 * OPS;  // B's slot 0
  constexpr bool ZC = !BKM && !SK;                 // tiles start with C = 0 MFMAs (rd_acc)
  __shared__ __attribute__((aligned(16))) char smem[SMEM_ALL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int T = gp.tile_end[gp.n - 1];
  const int G = gridDim.x;
  Walker wk;
  wk.init(gp, T, blockIdx.x, G, SK);
  Seg sg;
  if (!wk.next(sg)) return;
  const uint32_t smem_u32 = lds_addr(smem);
  char* const adst0 = smem + wave * 8 * 1024;
  char* const bdst0 = smem + B_BASE + wave * 8 * 1024;
  const char* rope_lds = smem + SMEM;
  char* const side = smem + SMEM + wave * SIDE_W;  // SIDE
  if constexpr (EM == EM_ROPE) {
    // the whole cos/sin table, once per workgroup (one problem per launch)
    const Params& p0 = gp.g[0];
    const int half = p0.rope_dim >> 1, chunks = p0.rope_dim >> 2, swz = rope_swz(p0.rope_dim);
    for (int i = tid; i < p0.rope_T * chunks; i += NT) {
      const int tt = i / chunks, k = i - tt * chunks;
      const float2 cs = *(const float2*)(p0.rope_cos + tt * half + 2 * k);
      const float2 sn = *(const float2*)(p0.rope_sin + tt * half + 2 * k);
      *(f32x4*)(smem + SMEM + rope_off(tt, k, p0.rope_dim * 4, swz)) = (f32x4){cs.x, sn.x, cs.y, sn.y};
    }
    __syncthreads();
  }

  // tile index -> (problem, m0, n0) and the tile's index within its problem
  // (sq_part is per problem).  The XCD-aware remap runs over the launch's whole
  // list of whole tiles, problems concatenated: XCD x's concurrent tiles are
  // consecutive ids, i.e. one or two problems in compact patches (tile_coords).
  // Remapped per problem instead, every problem was spread over all 8 XCDs, each
  // taking a thin slice that needed most of the problem's A panels: the grouped
  // weight gradients fetched 2.6x their algorithmic bytes.  The stream-K tail is
  // XCD-contiguous by construction (Walker), in tile order.
  const int ndp_all = SK ? gp.sk.dp_tiles : T;
  auto locate = [&](int tt, int& prob, int& m0, int& n0, int& lt) {
    const int gt = tt < ndp_all ? xcd_remap(tt, ndp_all) : tt;
    prob = 0;
    if (GROUPED)
      while (prob + 1 < gp.n && gt >= gp.tile_end[prob]) ++prob;
    const int first = prob ? gp.tile_end[prob - 1] : 0;
    const Params& q = gp.g[prob];
    lt = gt - first;
    tile_coords(lt, q.tiles_m, q.tiles_n, m0, n0);
  };
  int prob, m0, n0, lt;
  locate(sg.t, prob, m0, n0, lt);
  Dma d;
  dma_lanes<AK, BKM>(d, gp.g[prob], wave, lane);
  dma_tile<AK, BKM>(d, gp.g[prob], m0, n0, sg.ks);
  RdAddr<AK> ra;
  RdAddr<BKM> rb;
  rd_addr<AK>(ra, smem_u32, wm * 128, lane);
  rd_addr<BKM>(rb, smem_u32 + B_BASE, wn * 128, lane);

  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 f0a[8], f0b[8], f1a[8], f1b[8];
  // prologue of the first tile: stages 0 and 1 landed (both: step 0's counted
  // wait assumes an epilogue's stores behind stage 1), stage 0's k 0..31 read
  // (R3: A stage s in A slot s % 3, B stage s in B slot s % 2 -- slots 0, 1 here)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma16(d.ra, adst0 + s * OPS + q * 1024, d.va[q], d.ta + (uint32_t)s * d.a_kb);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma16(d.rb, bdst0 + s * OPS + q * 1024, d.vb[q], d.tb + (uint32_t)s * d.b_kb);
  }
  G4_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  G4_SB();
  rd_all<AK, BKM, 0>(f0a, f0b, ra, rb);
  G4_LGKM0();

  // R3: the three-ring operand's slot of the stage this step computes (runtime:
  // period 3); that operand's read addresses carry it (slot 0 + the current slot)
  int s3_cur = 0;
  auto move3 = [&](int from, int to) {  // read addresses: slot `from` -> `to`
    const uint32_t delta = (uint32_t)((to - from) * OPS);
    if constexpr (A3) {
      if constexpr (AK) {
#pragma unroll
        for (int h = 0; h < 2; ++h) ra.k[h] += delta;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) ra.t[j] += delta;
      }
    } else if constexpr (B3) {
      if constexpr (BKM) {
#pragma unroll
        for (int h = 0; h < 2; ++h) rb.k[h] += delta;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) rb.t[j] += delta;
      }
    }
  };

  // step on stage slot S: h = 0 on F0, the counted wait + barrier, h = 1 on F1
  // with the reads of the following stage (slot 1 - S) into F0 and the DMA of
  // stage `dma_stage` of the tile `dd` describes into slot S.  WAITN: how many VMEM
  // operations may stay in flight (issued after this wave's pieces of the stage to
  // retire).  The slot is a template constant: every LDS read takes it as an
  // immediate offset (no address arithmetic in the loop).
  // R3: S is B's slot (period 2); A's slots come from sa_cur (see move_a), and
  // h = 0 issues stage dma_stage's A pieces into A slot (sa_cur + 2) % 3.
  auto step = [&](auto slot_c, auto waitn_c, uint32_t dma_stage, const Dma& dd) {
    constexpr int S = decltype(slot_c)::value;
    constexpr int WAITN = decltype(waitn_c)::value;
    if constexpr (R3 && WAITN != 0 && !(DBG & 4096)) {
      // a tile's first step: h = 0 issues no DMA (it runs right behind the
      // epilogue's stores), h = 1 all 16 pieces -- the three-ring operand's into
      // the slot of stage s - 1, free since the previous step's barrier
      const int s3_dma = s3_cur == 0 ? 2 : s3_cur - 1;
      const int s3_next = s3_cur == 2 ? 0 : s3_cur + 1;
      const uint32_t oa = dma_stage * dd.a_kb, ob = dma_stage * dd.b_kb;
      half_step<AK, BKM, true, A3 ? 0 : S * OPS, B3 ? 0 : S * OPS, 1, 0, DBG, ZC>(acc, f0a, f0b, f1a, f1b, ra, rb,
                                                                               dd, adst0, bdst0, 0, 0);
      G4_LGKM0();
      if constexpr (WAITN == 32) G4_VMCNT(32);
      else G4_VMCNT(63);
      __builtin_amdgcn_s_barrier();
      G4_SB();
      move3(s3_cur, s3_next);
      half_step<AK, BKM, true, A3 ? 0 : (1 - S) * OPS, B3 ? 0 : (1 - S) * OPS, 0, 1, DBG>(
          acc, f1a, f1b, f0a, f0b, ra, rb, dd, adst0 + (A3 ? s3_dma : S) * OPS, bdst0 + (B3 ? s3_dma : S) * OPS, oa,
          ob);
      G4_LGKM0();
      s3_cur = s3_next;
    } else if constexpr (R3) {
      const int s3_dma = s3_cur == 0 ? 2 : s3_cur - 1;  // (s3_cur + 2) % 3
      const int s3_next = s3_cur == 2 ? 0 : s3_cur + 1;
      const uint32_t oa = dma_stage * dd.a_kb, ob = dma_stage * dd.b_kb;
      // h = 0: the three-ring operand's 8 pieces of stage dma_stage
      half_step<AK, BKM, true, A3 ? 0 : S * OPS, B3 ? 0 : S * OPS, 1, A3 ? 2 : 3, DBG, ZC && WAITN != 0>(
          acc, f0a, f0b, f1a, f1b, ra, rb, dd, adst0 + s3_dma * OPS, bdst0 + s3_dma * OPS, oa, ob);
      G4_LGKM0();
      if constexpr (WAITN == 0) G4_VMCNT(8);
      else if constexpr (WAITN == 32) G4_VMCNT(40);
      else G4_VMCNT(63);
      __builtin_amdgcn_s_barrier();
      G4_SB();
      move3(s3_cur, s3_next);
      // h = 1: the two-ring operand's 8 pieces into the slot stage s vacated
      half_step<AK, BKM, true, A3 ? 0 : (1 - S) * OPS, B3 ? 0 : (1 - S) * OPS, 0, A3 ? 3 : 2, DBG>(
          acc, f1a, f1b, f0a, f0b, ra, rb, dd, adst0 + S * OPS, bdst0 + S * OPS, oa, ob);
      G4_LGKM0();
      s3_cur = s3_next;
    } else {
      half_step<AK, BKM, true, S * OPS, S * OPS, 1, 0, DBG, ZC && WAITN != 0>(acc, f0a, f0b, f1a, f1b, ra, rb, dd,
                                                                              adst0, bdst0, 0, 0);
      G4_LGKM0();
      if constexpr (WAITN == 0) G4_VMCNT(0);
      else if constexpr (WAITN == 32) G4_VMCNT(32);
      else G4_VMCNT(63);
      __builtin_amdgcn_s_barrier();
      G4_SB();
      half_step<AK, BKM, true, (1 - S) * OPS, (1 - S) * OPS, 0, 1, DBG>(acc, f1a, f1b, f0a, f0b, ra, rb, dd,
                                                                      adst0 + S * OPS, bdst0 + S * OPS,
                                                                      dma_stage * dd.a_kb, dma_stage * dd.b_kb);
      G4_LGKM0();
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using W0 = std::integral_constant<int, 0>;
  // an epilogue issues at least 32 (bf16: 16 B per lane and 8 columns) or 64 (f32)
  // stores after the next tile's stage 1 pieces
  using WE = std::integral_constant<int, EM == EM_F32 ? 63 : 32>;

  for (;;) {
    const Params& p = gp.g[prob];
    // steps of this segment (a whole tile: K / 64)
    const int nk = sg.ke < 0 ? p.K / BK : 4 * (sg.ke - sg.ks);
    Seg ns;
    const bool has_next = wk.next(ns);
    // the next segment (after the workgroup's last: itself again, an empty-range
    // refill of slots nobody reads afterwards, drained before exit)
    if (!has_next) ns = sg;
    int nprob = prob, nm0 = m0, nn0 = n0, nlt = lt;
    if (has_next) locate(ns.t, nprob, nm0, nn0, nlt);
    // older than every stage piece the steps wait for: landed by the epilogue; the
    // previous epilogue's reads of the side area completed before its values were used
    if constexpr (SIDE) side_dma<EM>(p, side, m0 + wm * 128, n0 + wn * 128, lane);
    // step kt (slot kt & 1: nk is even, so every tile starts on slot 0) stages
    // stage kt + 2: this tile's while kt + 2 < nk, then the next tile's 0 and 1.
    // Three step sites (more make the register allocator give the fragment sets
    // different registers per site, and spill).
    step(S0{}, WE{}, 2u, d);
    for (int kt = 1; kt < nk; kt += 2) {
      step(S1{}, W0{}, (uint32_t)(kt + 2 < nk ? kt + 2 : kt + 2 - nk), d);
      if (kt + 1 < nk) {
        if (kt + 1 == nk - 2) {
          if (GROUPED && nprob != prob) dma_lanes<AK, BKM>(d, gp.g[nprob], wave, lane);
          dma_tile<AK, BKM>(d, gp.g[nprob], nm0, nn0, ns.ks, has_next || (DBG & 32768));
        }
        step(S0{}, W0{}, (uint32_t)(kt + 3 < nk ? kt + 3 : kt + 3 - nk), d);
      }
    }
    bool fin = true;
    if constexpr (SK) fin = sk_handoff(gp.sk, acc, sg, wk.rank, wave, lane);
    epilogue<EM, false, (DBG & 8192) ? 1 : 0, ZC ? 0 : (SK ? 1 : 2), SIDE>(p, acc, m0 + wm * 128, n0 + wn * 128, lane,
                                                                        wave, lt, rope_lds, fin, side);
    if (!has_next) break;
    sg = ns;
    prob = nprob;
    m0 = nm0;
    n0 = nn0;
    lt = nlt;
  }
  G4_VMCNT(0);  // the refill must land before the workgroup's LDS is released
}

// ---------------------------------------------------------------------------
// fp8 (e4m3) on the same structure (BASELINE config C5: the q|k|v / cross q,
// k|v / encoder FFN linear1 forward and FFN linear2 input-gradient GEMMs):
//   C[i, j] = a_scale[i] b_scale[j] sum_r A[i][r] B[j][r]   (+ epilogue)
// A [M][K], B [N][K] OCP e4m3 bytes, K-major (nstl_fp8_quant_rows / _cols), on
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 block scales: 128 K-bytes
// per instruction at twice the bf16 rate per clock, and the 16 x 16
// accumulator layout of the bf16 kernel, so its epilogues (bias, ReLU-dropout +
// keep bits, RoPE, dReLU + column sums, f32) are reused as they are, with the
// row and column scales applied first (SC).
// A stage is 128 K-bytes: 256 rows x 128 B per operand, the bf16 K-major image
// byte for byte (chunk c of row r at c ^ ((r >> 1) & 7)), filled by the same
// LDS-DMA pieces.  A lane's fragment of a 16-row block is 32 K-bytes (chunks
// 2g, 2g + 1 of its row, g = lane >> 4): 8 VGPRs, two ds_read_b128.  A stage's
// 64 MFMAs per wave need all 8 B fragments (64 VGPRs) and 8 A fragments (64),
// so the half-steps split the output rows instead of K: h = 0 computes A row
// blocks 0..3 against all of B while reading blocks 4..7; h = 1 computes 4..7
// while reading the next stage's blocks 0..3 and all of its B into the second
// B set, and issues the stage after next by DMA.  Fragment registers: 2 x 32
// (A) + 2 x 64 (B) = 192.
constexpr int F8_BK = 128;  // K-bytes per stage

typedef int i32x8_t __attribute__((ext_vector_type(8)));

NSTL_DEV void mma_f8(f32x4& acc, const i32x8_t& w, const i32x8_t& x) {
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w, x, acc, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}
NSTL_DEV void mma_f8z(f32x4& acc, const i32x8_t& w, const i32x8_t& x) {  // a tile's first step: C = 0
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(w, x, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0, 0x7f7f7f7f, 0,
                                                          0x7f7f7f7f);
}

// per-lane DMA sources of one operand's stage (K-major, 128-byte rows of bytes)
NSTL_DEV void dma_lane_offsets_f8(uint32_t (&vo)[8], int64_t ld, int wave, int lane) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int q = wave * 8 + s;
    const int row = 8 * q + (lane >> 3), pc = lane & 7;
    const int lc = pc ^ ((row >> 1) & 7);
    vo[s] = (uint32_t)((int64_t)row * ld + lc * 16);
  }
}
NSTL_DEV void dma_tile_f8(Dma& d, const Params& p, int m0, int n0, bool live = true) {  // live: dma_tile
  d.ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, live ? (int)p.a_bytes : 0, 0x00020000);
  d.rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, live ? (int)p.b_bytes : 0, 0x00020000);
  d.a_kb = F8_BK;
  d.b_kb = F8_BK;
  d.ta = __builtin_amdgcn_readfirstlane((uint32_t)(m0 * p.lda));
  d.tb = __builtin_amdgcn_readfirstlane((uint32_t)(n0 * p.ldb));
}

// the two read addresses of a lane's fragment (chunks 2g, 2g + 1 of its row of
// row block 0; block j at + 2048 j)
struct RdAddrF8 {
  uint32_t k[2];
};
NSTL_DEV void rd_addr_f8(RdAddrF8& r, uint32_t img, int blk0, int lane) {
  const int row = blk0 + (lane & 15), sw = (row >> 1) & 7, g = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) r.k[j] = img + row * 128 + (((2 * g + j) ^ sw) << 4);
}
template <int OFF>
NSTL_DEV void rd_f8(i32x8_t& f, const RdAddrF8& r) {
  i32x4_t v0, v1;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v0) : "v"(r.k[0]), "i"(OFF));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v1) : "v"(r.k[1]), "i"(OFF));
  f = (i32x8_t){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
}

// One fp8 half-step: 32 MFMAs, column-major -- for B block b = 0..7, A blocks
// 4H .. 4H + 3 (ca) -- so that in h = 1 B fragment b dies after MFMA 4b + 3 and
// the next stage's B block b is read into its registers right there (one B
// register set, not two).  Reads: h = 0 A blocks 4..7 of the current stage (slot
// offset SO) into na after MFMAs 1, 6, 11, 16; h = 1 the next stage's (SO) A
// blocks 0..3 into na after MFMAs 0, 8, 16, 24 and B block b after MFMA 4b + 3
// (the last, block 7, after the final MFMA: the next h = 0 uses it first at
// MFMA 28 and waits for it there).  DMA (h = 1): the 16 pieces after MFMAs 1, 3,
// ..., 31.  H = 2: h = 1 without any read.
template <int H, int SO, int DBG, bool Z = false, int I = 0>
NSTL_DEV void half_step_f8(f32x4 (&acc)[8][8], const i32x8_t (&ca)[4], i32x8_t (&cb)[8], i32x8_t (&na)[4],
                           const RdAddrF8& ra, const RdAddrF8& rb, const Dma& d, char* adst, char* bdst, uint32_t sa,
                           uint32_t sb) {
  if constexpr (I < 32) {
    constexpr int b = I >> 2, a = I & 3;
    if constexpr (H == 0 && I == 28) {
      // B block 7's read (the previous h = 1's last) is older than the 8 A reads
      // issued since: retire it
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      G4_SB();
    }
    if constexpr (!(DBG & 8)) {
      if constexpr (Z) mma_f8z(acc[4 * (H ? 1 : 0) + a][b], cb[b], ca[a]);
      else mma_f8(acc[4 * (H ? 1 : 0) + a][b], cb[b], ca[a]);
    }
    G4_SB();
    if constexpr (!(DBG & 2)) {
      if constexpr (H == 0 && (I == 1 || I == 6 || I == 11 || I == 16)) {
        constexpr int r = I == 1 ? 0 : I == 6 ? 1 : I == 11 ? 2 : 3;
        rd_f8<SO + (4 + r) * 2048>(na[r], ra);
        G4_SB();
      }
      if constexpr (H == 1 && (I & 7) == 0) {
        rd_f8<SO + (I >> 3) * 2048>(na[I >> 3], ra);
        G4_SB();
      }
      if constexpr (H == 1 && a == 3) {
        rd_f8<SO + b * 2048>(cb[b], rb);
        G4_SB();
      }
    }
    if constexpr (H >= 1 && !(DBG & 1) && (I & 1) == 1) {
      constexpr int q = I >> 1;
      if constexpr (q < 8) dma16(d.ra, adst + q * 1024, d.va[q], d.ta + sa);
      else dma16(d.rb, bdst + (q - 8) * 1024, d.vb[q - 8], d.tb + sb);
      G4_SB();
    }
    half_step_f8<H, SO, DBG, Z, I + 1>(acc, ca, cb, na, ra, rb, d, adst, bdst, sa, sb);
  }
}

// Preconditions (host-checked): e4m3 A [M][K] and B [N][K], M and N multiples of
// 256, K a multiple of 256 with K >= 512 (whole pairs of 128-byte stages, at
// least two pairs), 16-byte aligned rows, operand extents < 2^31 bytes; EM_ROPE:
// the table fits ROPE_LDS as f32 or (rope_bf16) as bf16.
template <int EM, int DBG = 0>
__global__ __launch_bounds__(NT, 1) void gemm4f8_kernel(const GroupParams gp) {
  // epilogue side data (scales, bias / keep-bit words: side_dma<EM, true>); not
  // with the RoPE table (no LDS left)
  constexpr bool SIDE = EM != EM_ROPE && EM != EM_F32 && !(DBG & 16384);
  __shared__ __attribute__((aligned(16))) char smem[SMEM + (EM == EM_ROPE ? ROPE_LDS : 0) + (SIDE ? 4 * SIDE_W_SC : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int T = gp.tile_end[0];
  const int G = gridDim.x;
  const Params& p = gp.g[0];
  Walker wk;
  wk.init(gp, T, blockIdx.x, G, false);
  Seg sg;
  if (!wk.next(sg)) return;
  const uint32_t smem_u32 = lds_addr(smem);
  char* const adst0 = smem + wave * 8 * 1024;
  char* const bdst0 = smem + 2 * OPS + wave * 8 * 1024;
  const char* rope_lds = smem + SMEM;
  char* const side = smem + SMEM + wave * SIDE_W_SC;  // SIDE
  if constexpr (EM == EM_ROPE) {
    const int half = p.rope_dim >> 1, chunks = p.rope_dim >> 2, swz = rope_swz(p.rope_dim);
    for (int i = tid; i < p.rope_T * chunks; i += NT) {
      const int tt = i / chunks, k = i - tt * chunks;
      const float2 cs = *(const float2*)(p.rope_cos + tt * half + 2 * k);
      const float2 sn = *(const float2*)(p.rope_sin + tt * half + 2 * k);
      if (p.rope_bf16) {
        *(uint2*)(smem + SMEM + rope_off8(tt, k, p.rope_dim * 2, swz)) =
            make_uint2(pack_bf16x2(cs.x, sn.x), pack_bf16x2(cs.y, sn.y));
      } else {
        *(f32x4*)(smem + SMEM + rope_off(tt, k, p.rope_dim * 4, swz)) = (f32x4){cs.x, sn.x, cs.y, sn.y};
      }
    }
    __syncthreads();
  }
  int m0, n0;
  tile_coords(xcd_remap(sg.t, T), p.tiles_m, p.tiles_n, m0, n0);
  int lt = 0;
  Dma d;
  dma_lane_offsets_f8(d.va, p.lda, wave, lane);
  dma_lane_offsets_f8(d.vb, p.ldb, wave, lane);
  dma_tile_f8(d, p, m0, n0);
  RdAddrF8 ra, rb;
  rd_addr_f8(ra, smem_u32, wm * 128, lane);
  rd_addr_f8(rb, smem_u32 + 2 * OPS, wn * 128, lane);

  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  i32x8_t fa0[4], fa1[4], fb[8];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma16(d.ra, adst0 + s * OPS + q * 1024, d.va[q], d.ta + (uint32_t)s * d.a_kb);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma16(d.rb, bdst0 + s * OPS + q * 1024, d.vb[q], d.tb + (uint32_t)s * d.b_kb);
  }
  G4_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  G4_SB();
  // stage 0 (slot 0): A blocks 0..3 and all of B
#pragma unroll
  for (int j = 0; j < 4; ++j) rd_f8<0>(fa0[j], (RdAddrF8){{ra.k[0] + j * 2048, ra.k[1] + j * 2048}});
#pragma unroll
  for (int j = 0; j < 8; ++j) rd_f8<0>(fb[j], (RdAddrF8){{rb.k[0] + j * 2048, rb.k[1] + j * 2048}});
  G4_LGKM0();

  // step on stage slot S: h = 0 on A blocks 0..3 (reading blocks 4..7), the
  // counted wait + barrier, h = 1 on blocks 4..7 with the next stage's reads
  // (slot 1 - S) and the DMA of stage `dma_stage` into slot S.  After h = 1 every
  // read but the last B block's has retired (lgkmcnt(2): its two instructions).
  auto step = [&](auto slot_c, auto waitn_c, uint32_t dma_stage) {
    constexpr int S = decltype(slot_c)::value;
    constexpr int WAITN = decltype(waitn_c)::value;
    half_step_f8<0, S * OPS, DBG, WAITN != 0>(acc, fa0, fb, fa1, ra, rb, d, adst0, bdst0, 0, 0);
    G4_LGKM0();
    if constexpr (WAITN == 0) G4_VMCNT(0);
    else if constexpr (WAITN == 32) G4_VMCNT(32);
    else G4_VMCNT(63);
    __builtin_amdgcn_s_barrier();
    G4_SB();
    half_step_f8<1, (1 - S) * OPS, DBG, WAITN != 0>(acc, fa1, fb, fa0, ra, rb, d, adst0 + S * OPS, bdst0 + S * OPS,
                                                    dma_stage * d.a_kb, dma_stage * d.b_kb);
    asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    G4_SB();
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using W0 = std::integral_constant<int, 0>;
  using WE = std::integral_constant<int, EM == EM_F32 ? 63 : 32>;

  const int nk = p.K / F8_BK;
  for (;;) {
    Seg ns;
    const bool has_next = wk.next(ns);
    if (!has_next) ns = sg;
    int nm0 = m0, nn0 = n0;
    if (has_next) tile_coords(xcd_remap(ns.t, T), p.tiles_m, p.tiles_n, nm0, nn0);
    if constexpr (SIDE) side_dma<EM, true>(p, side, m0 + wm * 128, n0 + wn * 128, lane);
    step(S0{}, WE{}, 2u);
    for (int kt = 1; kt < nk; kt += 2) {
      step(S1{}, W0{}, (uint32_t)(kt + 2 < nk ? kt + 2 : kt + 2 - nk));
      if (kt + 1 < nk) {
        if (kt + 1 == nk - 2) dma_tile_f8(d, p, nm0, nn0, has_next);
        step(S0{}, W0{}, (uint32_t)(kt + 3 < nk ? kt + 3 : kt + 3 - nk));
      }
    }
    G4_LGKM0();  // the next tile's last B fragment: before the epilogue's own LDS reads
    lt = sg.t < T ? xcd_remap(sg.t, T) : sg.t;
    epilogue<EM, true, (DBG & 8192) ? 1 : 0, 0, SIDE>(p, acc, m0 + wm * 128, n0 + wn * 128, lane, wave, lt, rope_lds, true,
                                                     side);
    if (!has_next) break;
    if constexpr (EM != EM_BF16) {
      // the per-lane DMA offsets and read addresses, recomputed after every
      // epilogue from a lane index the compiler cannot see through: kept live
      // across it (20 VGPRs) they made the scaled RoPE / dReLU epilogues spill
      // (the plain one is spill-free without, and spills with it)
      int lane_o = lane;
      asm volatile("" : "+v"(lane_o));
      dma_lane_offsets_f8(d.va, p.lda, wave, lane_o);
      dma_lane_offsets_f8(d.vb, p.ldb, wave, lane_o);
      rd_addr_f8(ra, smem_u32, wm * 128, lane_o);
      rd_addr_f8(rb, smem_u32 + 2 * OPS, wn * 128, lane_o);
    }
    sg = ns;
    m0 = nm0;
    n0 = nn0;
  }
  G4_VMCNT(0);
}

}  // namespace g4
