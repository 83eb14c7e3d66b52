// Multi-head attention forward/backward for the NeuroSync Seq2Seq
// (replaces F.scaled_dot_product_attention, utils/model.py:126-127, and its
// autograd backward; RoPE (apply_rope_qk, :60-83) is applied to q/k by the
// projection GEMM epilogue, and rotated back here on dq/dk).
//
// Shapes are short: T <= 256 frames, dh = 64.  A whole (batch, head) key/value
// sequence fits in LDS, so there is no online softmax and no cross-workgroup
// reduction:
//   forward : workgroup = (b, h, 64 query rows); each wave 16 rows; scores for
//             all keys live in MFMA accumulators; exact softmax; P round-trips
//             through a per-wave LDS image to become the A operand of P.V.
//   backward: workgroup = (b, h); phase 1 waves own 16-key tiles and accumulate
//             dK, dV over all queries; phase 2 waves own 16-query tiles and
//             accumulate dQ (scores/probabilities recomputed from the saved LSE).
// Dropout keep-mask is a counter hash of (b, h, q, k): regenerated, never stored.
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
  const char* dout; int64_t dout_ld;
  char* dq; int64_t dq_ld;
  char* dk; int64_t dk_ld;
  char* dv; int64_t dv_ld;
  const float* rope_cos; const float* rope_sin; int rope_q, rope_k;
  int B, T, H;
  float scale;
  uint32_t thresh; float inv_keep; uint64_t seed;
};

// Copy rows [0, nrows) of a (b, h) slice (64 elements per row) into an LDS image.
template <typename T, class Img>
NSTL_DEV void load_rows(char* img, const char* g, int64_t ld, int64_t row0, int col0, int nrows, int tid) {
  constexpr int CPR = DH * (int)sizeof(T) / 16;
  for (int c = tid; c < nrows * CPR; c += NT) {
    const int row = c / CPR, ch = c % CPR;
    const uint4 v = *(const uint4*)(g + (((row0 + row) * ld + col0) * (int64_t)sizeof(T)) + ch * 16);
    *(uint4*)(img + Img::off(row, ch * 16)) = v;
  }
}

template <typename T>
NSTL_DEV void store_elem(char* base, int64_t e, float v) {
  ((T*)base)[e] = from_f32<T>(v);
}

NSTL_DEV uint64_t drop_idx(int bh, int T, int q, int k) { return ((uint64_t)bh * T + q) * T + k; }

// ----------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int RBK = DH * (int)sizeof(T);  // 128 (bf16) / 256 (f32)
  typedef ImgK<RBK> Img;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  const int RBP = T_ * (int)sizeof(T) + 16;
  char* Kimg = smem;
  char* Vimg = Kimg + T_ * RBK;
  char* Qimg = Vimg + T_ * RBK;
  char* Pimg = Qimg + 64 * RBK;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int qb0 = blockIdx.x * 64;
  const int nq = min(64, T_ - qb0);
  const int64_t tok0 = (int64_t)b * T_;

  load_rows<T, Img>(Kimg, p.k, p.k_ld, tok0, h * DH, T_, tid);
  load_rows<T, Img>(Vimg, p.v, p.v_ld, tok0, h * DH, T_, tid);
  load_rows<T, Img>(Qimg, p.q, p.q_ld, tok0 + qb0, h * DH, nq, tid);
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
        Frag fk;
        frag_row<Img>(fk, Kimg, kt * 16 + (lane & 15), 8 * g);
        mma16(s[kt], fq[0], fk);
        frag_row<Img>(fk, Kimg, kt * 16 + (lane & 15), 32 + 8 * g);
        mma16(s[kt], fq[1], fk);
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
    // dropout + write P (unnormalised) into this wave's image [16 rows][T keys]
    char* Pw = Pimg + w * 16 * RBP;
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * g + r, key = kt * 16 + (lane & 15);
          float pv = s[kt][r];
          if (p.thresh)
            pv = nstl_keep(p.seed, drop_idx(bh, T_, qb0 + q0 + row, key), p.thresh) ? pv * p.inv_keep : 0.f;
          *(T*)(Pw + row * RBP + key * (int)sizeof(T)) = from_f32<T>(pv);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nkt / 2; ++ks) {
      Frag fp;
      frag_row<ImgPlain<0>>(fp, Pw + (lane & 15) * RBP, 0, ks * 32 + 8 * g);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        Frag fv;
        frag_col<Img>(fv, Vimg, dt * 16, ks * 32, lane);
        mma16(o[dt], fp, fv);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = qb0 + q0 + 4 * g + r;
      const float inv = 1.f / sum[r];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        store_elem<T>(p.o, (tok0 + q) * p.o_ld + h * DH + dt * 16 + (lane & 15), o[dt][r] * inv);
      if ((lane & 15) == 0) p.lse[(int64_t)bh * T_ + q] = mx[r] * p.scale + logf(sum[r]);
    }
  }
}

// rotate a (row t, col d) accumulator element back by -theta (RoPE^T)
NSTL_DEV float rope_back(float v, int t, int d, const float* cs, const float* sn) {
  const float partner = __shfl_xor(v, 1);
  const float c = cs[t * (DH / 2) + (d >> 1)], s = sn[t * (DH / 2) + (d >> 1)];
  return (d & 1) ? (v * c - partner * s) : (v * c + partner * s);
}

template <typename T>
__global__ __launch_bounds__(NT) void attn_bwd_kernel(AttnParams p) {
  typedef typename FragT<T>::type Frag;
  constexpr int RBK = DH * (int)sizeof(T);
  typedef ImgK<RBK> Img;
  constexpr int RBS = 32 * (int)sizeof(T) + 16;  // per-wave scratch rows (32 elems + pad)
  typedef ImgPlain<RBS> ImgS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T_ = p.T, nkt = T_ / 16;
  char* Qimg = smem;
  char* Kimg = Qimg + T_ * RBK;
  char* Vimg = Kimg + T_ * RBK;
  char* Dimg = Vimg + T_ * RBK;
  float* lse_s = (float*)(Dimg + T_ * RBK);
  float* dq_s = lse_s + T_;
  char* scratch = (char*)(dq_s + T_);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int64_t tok0 = (int64_t)b * T_;

  load_rows<T, Img>(Qimg, p.q, p.q_ld, tok0, h * DH, T_, tid);
  load_rows<T, Img>(Kimg, p.k, p.k_ld, tok0, h * DH, T_, tid);
  load_rows<T, Img>(Vimg, p.v, p.v_ld, tok0, h * DH, T_, tid);
  load_rows<T, Img>(Dimg, p.dout, p.dout_ld, tok0, h * DH, T_, tid);
  // D_q = rowsum(dO * O), one wave per row group
  for (int row = w; row < T_; row += NT / 64) {
    const int64_t eo = (tok0 + row) * p.o_ld + h * DH + lane;
    const int64_t ed = (tok0 + row) * p.dout_ld + h * DH + lane;
    float v = to_f32(((const T*)p.o)[eo]) * to_f32(((const T*)p.dout)[ed]);
    v = wave_sum(v);
    if (lane == 0) {
      dq_s[row] = v;
      lse_s[row] = p.lse[(int64_t)bh * T_ + row];
    }
  }
  __syncthreads();

  const float c2 = p.scale * LOG2E;
  char* S1 = scratch + w * 2 * 16 * RBS;  // Pd^T / dS image A
  char* S2 = S1 + 16 * RBS;               // dS^T image

  // ---------------- phase 1: dK, dV for 16-key tiles ----------------
  for (int kt = w; kt < nkt; kt += 4) {
    Frag fk[2], fv[2];
    frag_row<Img>(fk[0], Kimg, kt * 16 + (lane & 15), 8 * g);
    frag_row<Img>(fk[1], Kimg, kt * 16 + (lane & 15), 32 + 8 * g);
    frag_row<Img>(fv[0], Vimg, kt * 16 + (lane & 15), 8 * g);
    frag_row<Img>(fv[1], Vimg, kt * 16 + (lane & 15), 32 + 8 * g);
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
        const int q = qt * 16 + (lane & 15);
        const float lq = lse_s[q] * LOG2E, dqv = dq_s[q];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kr = 4 * g + r, key = kt * 16 + kr;
          const float pv = exp2f(st[r] * c2 - lq);
          float pd = pv, dpd = dpt[r];
          if (p.thresh) {
            const bool keep = nstl_keep(p.seed, drop_idx(bh, T_, q, key), p.thresh);
            pd = keep ? pv * p.inv_keep : 0.f;
            dpd = keep ? dpd * p.inv_keep : 0.f;
          }
          const float ds = pv * (dpd - dqv);
          *(T*)(S1 + ImgS::off(kr, (u * 16 + (lane & 15)) * (int)sizeof(T))) = from_f32<T>(pd);
          *(T*)(S2 + ImgS::off(kr, (u * 16 + (lane & 15)) * (int)sizeof(T))) = from_f32<T>(ds);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      Frag fa1, fa2;
      frag_row<ImgS>(fa1, S1, lane & 15, 8 * g);
      frag_row<ImgS>(fa2, S2, lane & 15, 8 * g);
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
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = kt * 16 + 4 * g + r;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = dt * 16 + (lane & 15);
        float vk = dk[dt][r] * p.scale;
        if (p.rope_k) vk = rope_back(vk, key, d, p.rope_cos, p.rope_sin);
        store_elem<T>(p.dk, (tok0 + key) * p.dk_ld + h * DH + d, vk);
        store_elem<T>(p.dv, (tok0 + key) * p.dv_ld + h * DH + d, dv[dt][r]);
      }
    }
  }

  // ---------------- phase 2: dQ for 16-query tiles ----------------
  for (int qt = w; qt < nkt; qt += 4) {
    Frag fq[2], fo[2];
    frag_row<Img>(fq[0], Qimg, qt * 16 + (lane & 15), 8 * g);
    frag_row<Img>(fq[1], Qimg, qt * 16 + (lane & 15), 32 + 8 * g);
    frag_row<Img>(fo[0], Dimg, qt * 16 + (lane & 15), 8 * g);
    frag_row<Img>(fo[1], Dimg, qt * 16 + (lane & 15), 32 + 8 * g);
    float lq[4], dqv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      lq[r] = lse_s[qt * 16 + 4 * g + r] * LOG2E;
      dqv[r] = dq_s[qt * 16 + 4 * g + r];
    }
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
        const int key = kt * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qr = 4 * g + r, q = qt * 16 + qr;
          const float pv = exp2f(s[r] * c2 - lq[r]);
          float dpd = dp[r];
          if (p.thresh) dpd = nstl_keep(p.seed, drop_idx(bh, T_, q, key), p.thresh) ? dpd * p.inv_keep : 0.f;
          const float ds = pv * (dpd - dqv[r]);
          *(T*)(S2 + ImgS::off(qr, (u * 16 + (lane & 15)) * (int)sizeof(T))) = from_f32<T>(ds);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      Frag fa;
      frag_row<ImgS>(fa, S2, lane & 15, 8 * g);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        Frag fb;
        frag_col<Img>(fb, Kimg, dt * 16, kc * 32, lane);
        mma16(dq[dt], fa, fb);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = qt * 16 + 4 * g + r;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = dt * 16 + (lane & 15);
        float vq = dq[dt][r] * p.scale;
        if (p.rope_q) vq = rope_back(vq, q, d, p.rope_cos, p.rope_sin);
        store_elem<T>(p.dq, (tok0 + q) * p.dq_ld + h * DH + d, vq);
      }
    }
  }
}

size_t fwd_lds_bytes(int T, int esz) {
  return (size_t)(2 * T + 64) * DH * esz + 4 * 16 * (size_t)(T * esz + 16);
}
size_t bwd_lds_bytes(int T, int esz) {
  return (size_t)4 * T * DH * esz + 2 * T * 4 + 4 * 2 * 16 * (size_t)(32 * esz + 16);
}

int fill(AttnParams& p, const nstl_attn_args* a, bool bwd) {
  NSTL_CHECK_ARG(a != nullptr, "nstl_attn: null args");
  NSTL_CHECK_ARG(a->dtype == NSTL_F32 || a->dtype == NSTL_BF16, "nstl_attn: bad dtype");
  NSTL_CHECK_ARG(a->dh == DH, "nstl_attn: head_dim must be 64 (got %d)", a->dh);
  NSTL_CHECK_ARG(a->T > 0 && a->T % 32 == 0, "nstl_attn: T must be a positive multiple of 32 (got %d)", a->T);
  NSTL_CHECK_ARG(a->T <= (a->dtype == NSTL_BF16 ? 256 : 128), "nstl_attn: T=%d too long for this dtype", a->T);
  NSTL_CHECK_ARG(a->B > 0 && a->H > 0, "nstl_attn: empty batch");
  NSTL_CHECK_ARG(a->q && a->k && a->v && a->o && a->lse, "nstl_attn: null tensor");
  const int vec = a->dtype == NSTL_F32 ? 4 : 8;
  NSTL_CHECK_ARG(a->q_ld % vec == 0 && a->k_ld % vec == 0 && a->v_ld % vec == 0, "nstl_attn: ld alignment");
  NSTL_CHECK_ARG(a->p_drop >= 0.f && a->p_drop < 1.f, "nstl_attn: p_drop out of range");
  if (bwd) {
    NSTL_CHECK_ARG(a->dout && a->dq && a->dk && a->dv, "nstl_attn_bwd: null gradient tensor");
    NSTL_CHECK_ARG(a->dout_ld % vec == 0, "nstl_attn_bwd: dout_ld alignment");
    NSTL_CHECK_ARG(!(a->rope_q || a->rope_k) || (a->rope_cos && a->rope_sin), "nstl_attn_bwd: rope tables");
  }
  p.q = (const char*)a->q; p.q_ld = a->q_ld;
  p.k = (const char*)a->k; p.k_ld = a->k_ld;
  p.v = (const char*)a->v; p.v_ld = a->v_ld;
  p.o = (char*)a->o; p.o_ld = a->o_ld;
  p.lse = a->lse;
  p.dout = (const char*)a->dout; p.dout_ld = a->dout_ld;
  p.dq = (char*)a->dq; p.dq_ld = a->dq_ld;
  p.dk = (char*)a->dk; p.dk_ld = a->dk_ld;
  p.dv = (char*)a->dv; p.dv_ld = a->dv_ld;
  p.rope_cos = a->rope_cos; p.rope_sin = a->rope_sin;
  p.rope_q = a->rope_q; p.rope_k = a->rope_k;
  p.B = a->B; p.T = a->T; p.H = a->H;
  p.scale = 1.0f / sqrtf((float)a->dh);
  p.thresh = nstl_drop_thresh(a->p_drop);
  p.inv_keep = 1.0f / (1.0f - a->p_drop);
  p.seed = a->seed;
  return 0;
}

template <typename K>
int launch(K kern, dim3 grid, size_t lds, hipStream_t st, const AttnParams& p, const char* what) {
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return nstl::fail((int)e, "%s: LDS request %zu: %s", what, lds, hipGetErrorString(e));
  hipLaunchKernelGGL(kern, grid, dim3(NT), lds, st, p);
  NSTL_LAUNCH_CHECK(what);
  return 0;
}

}  // namespace

extern "C" int nstl_attn_fwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, false);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  dim3 grid((a->T + 63) / 64, a->B * a->H);
  const size_t lds = fwd_lds_bytes(a->T, esz);
  if (a->dtype == NSTL_BF16) return launch(attn_fwd_kernel<bf16>, grid, lds, (hipStream_t)stream, p, "nstl_attn_fwd");
  return launch(attn_fwd_kernel<float>, grid, lds, (hipStream_t)stream, p, "nstl_attn_fwd");
}

extern "C" int nstl_attn_bwd(const nstl_attn_args* a, void* stream) {
  AttnParams p;
  int rc = fill(p, a, true);
  if (rc) return rc;
  const int esz = a->dtype == NSTL_F32 ? 4 : 2;
  dim3 grid(a->B * a->H);
  const size_t lds = bwd_lds_bytes(a->T, esz);
  if (a->dtype == NSTL_BF16) return launch(attn_bwd_kernel<bf16>, grid, lds, (hipStream_t)stream, p, "nstl_attn_bwd");
  return launch(attn_bwd_kernel<float>, grid, lds, (hipStream_t)stream, p, "nstl_attn_bwd");
}
