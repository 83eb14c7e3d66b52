// Host side of the 4-wave persistent GEMM (gemm4.h): eligibility, parameters,
// launch.  nstl_gemm / nstl_gemm_grouped (gemm.hip) try it first; problems it
// does not take (partial tiles, split-K, beta != 0, fp8, the dReLU epilogue
// without keep bits, RoPE tables past the LDS budget, ...) stay on the 8-wave
// ring kernel.  NSTL_GEMM4=0 sends everything to the ring kernel (A/B runs).
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <vector>

#include "../../include/nstl.h"
#include "common.h"
#include "gemm4.h"
#include "status.h"

namespace {

// read per call (a getenv per GEMM), so a test can compare both paths in one process
int gemm4_env() {
  const char* e = getenv("NSTL_GEMM4");
  return e ? atoi(e) : 1;
}

// NSTL_GEMM4_SK=1: a stream-K tail when the grid does not divide the tiles
// (default 0: a partial last round of whole tiles, measured faster on every
// shape but the long-K weight gradients, profiles/r4_sk_bench_v2.txt); 2: the
// stream-K instantiation also when the grid divides the tiles (every tail range
// one whole tile: its cost without hand-offs; timing only)
int sk_env() {
  const char* e = getenv("NSTL_GEMM4_SK");
  return e ? atoi(e) : 0;
}

// the stream-K slabs and tickets, per (device, stream): launches on different
// streams never share them.  Tickets start at zero (hipMemset once) and every
// tile's second arriver resets its own.
struct SkSpace {
  float* slab = nullptr;
  unsigned* cnt = nullptr;
  int G = 0;
};
// At most SK_SPACES of them (2 G x 256 KB each, 128 MB at G = 256).  Nothing
// is ever freed on the launch path: a space handed out may still be waiting
// for its launch on another host thread, and a free there would also break
// stream capture.  So a new stream past SK_SPACES gets no space (its launches
// run whole tiles), and a space outgrown by a larger grid is retired, not
// freed (grids change only with a stream's CU mask; stream-K is opt-in).
constexpr size_t SK_SPACES = 4;
bool sk_space(hipStream_t st, int G, g4::StreamK& sk) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, SkSpace> spaces;
  static std::vector<SkSpace> retired;
  const int dev = nstl::stream_device(st);  // the stream's device, not the current one
  std::lock_guard<std::mutex> lk(mu);
  if (spaces.find({dev, st}) == spaces.end() && spaces.size() >= SK_SPACES) return false;
  SkSpace& s = spaces[{dev, st}];
  if (s.G < G) {
    nstl::DeviceGuard on(dev);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    if (s.slab) retired.push_back(s);
    s = SkSpace();
    if (hipMalloc((void**)&s.slab, (size_t)2 * G * 262144) != hipSuccess) return false;
    if (hipMalloc((void**)&s.cnt, (size_t)8 * G * sizeof(unsigned)) != hipSuccess) return false;
    if (hipMemset(s.cnt, 0, (size_t)8 * G * sizeof(unsigned)) != hipSuccess) return false;
    s.G = G;
  }
  sk.slab = s.slab;
  sk.cnt = s.cnt;
  sk.slab_bytes = (uint32_t)((size_t)2 * G * 262144);
  return true;
}

// whole tiles for the first T / G - 1 rounds, stream-K over the rest, when T is
// not a multiple of G (and every problem's K splits into 256-deep units)
void plan_sk(g4::GroupParams& gp, int G, hipStream_t st) {
  memset(&gp.sk, 0, sizeof(gp.sk));
  const int T = gp.tile_end[gp.n - 1];
  const int mode = sk_env();  // 2: the stream-K instantiation even when G divides T (timing only)
  if (T < G || !mode || (T % G == 0 && mode != 2)) return;
  const int K = gp.g[0].K;
  for (int i = 0; i < gp.n; ++i)
    if (gp.g[i].K != K) return;
  if (K % (4 * g4::BK)) return;
  g4::StreamK sk;
  if (!sk_space(st, G, sk)) {
    (void)hipGetLastError();
    return;
  }
  sk.dp_tiles = (T / G - 1) * G;
  sk.units = K / (4 * g4::BK);
  gp.sk = sk;
}

// the epilogue kind this kernel runs for `a`, or 0 (not eligible)
int g4_mode(const nstl_gemm_args* a) {
  if (a->dtype != NSTL_BF16 || a->split_k > 1 || a->beta != 0.f || (a->sq_part != nullptr && a->c_dtype != NSTL_F32))
    return 0;
  const bool bf_out = a->c_dtype == NSTL_BF16;
  // side outputs only with the epilogue that produces them (anything else goes on
  // to nstl_gemm's own argument checks)
  if (a->colsum_part != nullptr && a->epilogue != NSTL_EPI_DRELU_DROP) return 0;
  if (a->relu_mask != nullptr && a->epilogue != NSTL_EPI_BIAS_RELU_DROP && a->epilogue != NSTL_EPI_DRELU_DROP)
    return 0;
  switch (a->epilogue) {
    case NSTL_EPI_NONE:
      return bf_out ? g4::EM_BF16 : g4::EM_F32;
    case NSTL_EPI_BIAS:
      return bf_out ? g4::EM_BF16 : 0;
    case NSTL_EPI_BIAS_RELU_DROP:
      return bf_out && (a->N & 1) == 0 ? g4::EM_RELU_DROP : 0;
    case NSTL_EPI_BIAS_ROPE:
      return bf_out && a->b_kmajor && a->rope_dim % 4 == 0 && a->rope_cols % 16 == 0 &&
                     (int64_t)a->rope_T * a->rope_dim * 4 <= g4::ROPE_LDS
                 ? g4::EM_ROPE
                 : 0;
    case NSTL_EPI_DRELU_DROP:
      return bf_out && a->relu_mask != nullptr ? g4::EM_DRELU : 0;
    default:
      return 0;
  }
}

bool g4_shape_ok(const nstl_gemm_args* a) {
  // K: whole pairs of 64-deep stages (every tile starts on stage slot 0), at least two pairs
  if (a->M % g4::TILE || a->N % g4::TILE || a->K % (2 * g4::BK) || a->K < 4 * g4::BK) return false;
  if (!a->a_kmajor && a->b_kmajor) return false;  // layouts used: TT, TN, NN
  if (((uintptr_t)a->A | (uintptr_t)a->B | (uintptr_t)a->C) % 16) return false;
  if (a->lda % 8 || a->ldb % 8) return false;
  if (a->ldc % (a->c_dtype == NSTL_F32 ? 4 : 8)) return false;
  // operand extents for the 32-bit buffer offsets
  const int64_t ae = a->a_kmajor ? ((int64_t)(a->M - 1) * a->lda + a->K) * 2 : ((int64_t)(a->K - 1) * a->lda + a->M) * 2;
  const int64_t be = a->b_kmajor ? ((int64_t)(a->N - 1) * a->ldb + a->K) * 2 : ((int64_t)(a->K - 1) * a->ldb + a->N) * 2;
  // f32 C through a buffer resource (its epilogue's stores): 32-bit extent
  const int64_t ce = a->c_dtype == NSTL_F32 ? (int64_t)a->M * a->ldc * 4 : 0;
  return ae < (1ll << 31) && be < (1ll << 31) && ce < (1ll << 31);
}

void fill(g4::Params& q, const nstl_gemm_args* a) {
  memset(&q, 0, sizeof(q));
  q.A = (const char*)a->A; q.lda = a->lda;
  q.B = (const char*)a->B; q.ldb = a->ldb;
  q.C = (char*)a->C; q.ldc = a->ldc;
  q.M = a->M; q.N = a->N; q.K = a->K;
  q.alpha = a->alpha;
  q.bias = a->bias;
  q.thresh = nstl_drop_thresh(a->p_drop);
  q.inv_keep = 1.0f / (1.0f - a->p_drop);
  q.seed = a->seed;
  q.rope_cos = a->rope_cos; q.rope_sin = a->rope_sin;
  q.rope_T = a->rope_T; q.rope_dim = a->rope_dim; q.rope_cols = a->rope_cols;
  q.colsum_part = a->colsum_part;
  q.relu_mask = a->relu_mask;
  q.sq_part = a->sq_part;
  q.a_bytes = (uint32_t)(a->a_kmajor ? ((int64_t)(a->M - 1) * a->lda + a->K) * 2 : ((int64_t)(a->K - 1) * a->lda + a->M) * 2);
  q.b_bytes = (uint32_t)(a->b_kmajor ? ((int64_t)(a->N - 1) * a->ldb + a->K) * 2 : ((int64_t)(a->K - 1) * a->ldb + a->N) * 2);
  q.tiles_m = a->M / g4::TILE;
  q.tiles_n = a->N / g4::TILE;
}

// R3 (gemm4.h): the stage DMA spread over both half-steps with a 3 + 2 slot
// ring.  Measured on isolated shapes (profiles/r5_r3_ab.txt, outputs bit-
// identical): the weight gradients (K = 16,384) 3-6 % faster, K = 4096 shapes
// ~1 %, the K = 1024 multi-round forward (FFN1) 4-9 % slower, the rest neutral:
// taken for K >= 2048 (every weight gradient).  NSTL_GEMM4_R3=0: never (A/B).
int r3_env() {
  const char* e = getenv("NSTL_GEMM4_R3");
  return e ? atoi(e) : 1;
}

template <bool AK, bool BKM, bool GROUPED, bool SK, int R3>
void launch_em(int em, dim3 grid, hipStream_t st, const g4::GroupParams& gp) {
  const dim3 block(g4::NT);
  switch (em) {
    case g4::EM_BF16: hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, g4::EM_BF16, GROUPED, 0, SK, R3>), grid, block, 0, st, gp); break;
    case g4::EM_RELU_DROP:
      hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, g4::EM_RELU_DROP, GROUPED, 0, SK, R3>), grid, block, 0, st, gp);
      break;
    case g4::EM_ROPE:  // the q|k|v forward (TT) only: g4_mode takes RoPE with a K-major B; never R3
      if constexpr (BKM && !R3) hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, g4::EM_ROPE, GROUPED, 0, SK>), grid, block, 0, st, gp);
      break;
    case g4::EM_DRELU: hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, g4::EM_DRELU, GROUPED, 0, SK, R3>), grid, block, 0, st, gp); break;
    default: hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, g4::EM_F32, GROUPED, 0, SK, R3>), grid, block, 0, st, gp); break;
  }
}

// the instantiations the step uses: forward and dX (A K-major) with every
// epilogue; the weight gradients (NN) with f32 output, grouped or not; each
// with and without the stream-K tail (R3 only without it)
template <bool SK, int R3>
int launch_sk(int em, bool ak, bool bk, bool grouped, dim3 grid, hipStream_t st, const g4::GroupParams& gp) {
  if (ak && bk) {
    if (grouped) {  // the cross-attention k|v projections of all decoder layers
      if (em != g4::EM_ROPE || SK || R3) return 0;
      hipLaunchKernelGGL((g4::gemm4_kernel<true, true, g4::EM_ROPE, true, 0, false, 0>), grid, dim3(g4::NT), 0, st, gp);
      return 1;
    }
    launch_em<true, true, false, SK, R3>(em, grid, st, gp);
  } else if (ak && !bk) {
    if (grouped) return 0;
    launch_em<true, false, false, SK, R3>(em, grid, st, gp);
  } else {
    if (em != g4::EM_F32) return 0;
    if (grouped) hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, true, 0, SK, R3>), grid, dim3(g4::NT), 0, st, gp);
    else hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 0, SK, R3>), grid, dim3(g4::NT), 0, st, gp);
  }
  return 1;
}

int launch(int em, bool ak, bool bk, bool grouped, int G, hipStream_t st, g4::GroupParams& gp) {
  const int tiles = gp.tile_end[gp.n - 1];
  const dim3 grid(tiles < G ? tiles : G);
  plan_sk(gp, G, st);
  if (!gp.sk.slab) {
    int kmin = gp.g[0].K;
    for (int i = 1; i < gp.n; ++i) kmin = gp.g[i].K < kmin ? gp.g[i].K : kmin;
    if (em != g4::EM_ROPE && kmin >= 2048 && r3_env()) return launch_sk<false, 1>(em, ak, bk, grouped, grid, st, gp);
    return launch_sk<false, 0>(em, ak, bk, grouped, grid, st, gp);
  }
  if (!launch_sk<true, 0>(em, ak, bk, grouped, grid, st, gp)) return 0;
  nstl::count(NSTL_K_GEMM4_SK);
  return 1;
}

// ---------------------------------------------------------------------------
// fp8 (gemm4f8_kernel): e4m3 A [M][K] and B [N][K] with row scales (C5)
int g4f8_mode(const nstl_gemm_args* a) {
  if (a->dtype != NSTL_FP8 || a->split_k > 1 || a->beta != 0.f || !a->a_kmajor || !a->b_kmajor) return 0;
  if (!a->a_scale || !a->b_scale || a->sq_part) return 0;
  const bool bf_out = a->c_dtype == NSTL_BF16;
  if (a->colsum_part != nullptr && a->epilogue != NSTL_EPI_DRELU_DROP) return 0;
  if (a->relu_mask != nullptr && a->epilogue != NSTL_EPI_BIAS_RELU_DROP && a->epilogue != NSTL_EPI_DRELU_DROP)
    return 0;
  switch (a->epilogue) {
    case NSTL_EPI_NONE: return bf_out ? g4::EM_BF16 : 0;  // f32 out: the ring kernel (tests only)
    case NSTL_EPI_BIAS: return bf_out ? g4::EM_BF16 : 0;
    case NSTL_EPI_BIAS_RELU_DROP: return bf_out && (a->N & 1) == 0 ? g4::EM_RELU_DROP : 0;
    case NSTL_EPI_BIAS_ROPE:
      // the table in LDS: f32, or bf16 when only that fits (T = 256 with head dim 64)
      return bf_out && a->rope_dim % 4 == 0 && a->rope_cols % 16 == 0 &&
                     (int64_t)a->rope_T * a->rope_dim * 2 <= g4::ROPE_LDS
                 ? g4::EM_ROPE
                 : 0;
    case NSTL_EPI_DRELU_DROP: return bf_out && a->relu_mask != nullptr ? g4::EM_DRELU : 0;
    default: return 0;
  }
}

bool g4f8_shape_ok(const nstl_gemm_args* a) {
  if (a->M % g4::TILE || a->N % g4::TILE || a->K % (2 * g4::F8_BK) || a->K < 4 * g4::F8_BK) return false;
  if (((uintptr_t)a->A | (uintptr_t)a->B | (uintptr_t)a->C) % 16) return false;
  if (a->lda % 16 || a->ldb % 16) return false;
  if (a->ldc % (a->c_dtype == NSTL_F32 ? 4 : 8)) return false;
  const int64_t ae = (int64_t)(a->M - 1) * a->lda + a->K, be = (int64_t)(a->N - 1) * a->ldb + a->K;
  const int64_t ce = a->c_dtype == NSTL_F32 ? (int64_t)a->M * a->ldc * 4 : 0;
  return ae < (1ll << 31) && be < (1ll << 31) && ce < (1ll << 31);
}

}  // namespace

namespace nstl {

// NSTL_GEMM4_F8=0 keeps every fp8 GEMM on the 8-wave ring kernel (A/B runs; read per call)
int gemm4_f8(const nstl_gemm_args* a, hipStream_t st, int* handled) {
  *handled = 0;
  const char* e = getenv("NSTL_GEMM4_F8");
  if ((e && atoi(e) == 0) || !gemm4_env() || !g4f8_shape_ok(a)) return 0;
  const int em = g4f8_mode(a);
  if (!em) return 0;
  const int G = nstl::stream_cus(st);
  if (G <= 0) return 0;
  g4::GroupParams gp;
  memset(&gp, 0, sizeof(gp));
  g4::Params& q = gp.g[0];
  fill(q, a);
  q.a_bytes = (uint32_t)((int64_t)(a->M - 1) * a->lda + a->K);
  q.b_bytes = (uint32_t)((int64_t)(a->N - 1) * a->ldb + a->K);
  q.a_scale = a->a_scale;
  q.b_scale = a->b_scale;
  q.rope_bf16 = em == g4::EM_ROPE && (int64_t)a->rope_T * a->rope_dim * 4 > g4::ROPE_LDS;
  gp.n = 1;
  gp.tile_end[0] = q.tiles_m * q.tiles_n;
  const dim3 grid(gp.tile_end[0] < G ? gp.tile_end[0] : G), block(g4::NT);
  switch (em) {
    case g4::EM_BF16: hipLaunchKernelGGL((g4::gemm4f8_kernel<g4::EM_BF16>), grid, block, 0, st, gp); break;
    case g4::EM_RELU_DROP: hipLaunchKernelGGL((g4::gemm4f8_kernel<g4::EM_RELU_DROP>), grid, block, 0, st, gp); break;
    case g4::EM_ROPE: hipLaunchKernelGGL((g4::gemm4f8_kernel<g4::EM_ROPE>), grid, block, 0, st, gp); break;
    default: hipLaunchKernelGGL((g4::gemm4f8_kernel<g4::EM_DRELU>), grid, block, 0, st, gp); break;
  }
  NSTL_LAUNCH_CHECK("nstl_gemm (fp8, 4-wave persistent)");
  nstl::count(NSTL_K_GEMM_FP8);  // every fp8 launch, either kernel
  nstl::count(NSTL_K_GEMM4F8);
  if (em == g4::EM_ROPE) nstl::count(NSTL_K_GEMM_FP8_ROPE);
  nstl::count(NSTL_K_GEMM4_TILES, gp.tile_end[0]);
  *handled = 1;
  return 0;
}

// One problem: *handled = 1 when the 4-wave kernel took it.
int gemm4(const nstl_gemm_args* a, hipStream_t st, int* handled) {
  *handled = 0;
  if (!gemm4_env() || !g4_shape_ok(a)) return 0;
  const int em = g4_mode(a);
  if (!em) return 0;
  if (!a->a_kmajor && em != g4::EM_F32) return 0;
  const int G = nstl::stream_cus(st);
  if (G <= 0) return 0;
  g4::GroupParams gp;
  memset(&gp, 0, sizeof(gp));
  fill(gp.g[0], a);
  gp.n = 1;
  gp.tile_end[0] = gp.g[0].tiles_m * gp.g[0].tiles_n;
  if (!launch(em, a->a_kmajor, a->b_kmajor, false, G, st, gp)) return 0;
  NSTL_LAUNCH_CHECK("nstl_gemm (4-wave persistent)");
  nstl::count(NSTL_K_GEMM4);
  nstl::count(NSTL_K_GEMM4_TILES, gp.tile_end[0]);
  *handled = 1;
  return 0;
}

// A group of weight-gradient problems (same layout, f32 output, beta 0), or of
// forward projections with the bias + RoPE epilogue and one shared table (TT:
// the decoder's cross-attention k|v of every layer in one launch; nstl_gemm_grouped
// checked the table is shared).
int gemm4_grouped(const nstl_gemm_args* args, int n, hipStream_t st, int* handled) {
  *handled = 0;
  if (!gemm4_env() || n < 1 || n > g4::GROUP_MAX) return 0;
  const int em = g4_mode(args);
  if (em != g4::EM_F32 && em != g4::EM_ROPE) return 0;
  for (int i = 0; i < n; ++i) {
    const nstl_gemm_args* a = args + i;
    if (!g4_shape_ok(a) || g4_mode(a) != em) return 0;
    if (em == g4::EM_F32 && a->epilogue != NSTL_EPI_NONE) return 0;
    if (a->a_kmajor != args[0].a_kmajor || a->b_kmajor != args[0].b_kmajor) return 0;
  }
  const int G = nstl::stream_cus(st);
  if (G <= 0) return 0;
  g4::GroupParams gp;
  memset(&gp, 0, sizeof(gp));
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    fill(gp.g[i], args + i);
    tiles += gp.g[i].tiles_m * gp.g[i].tiles_n;
    gp.tile_end[i] = tiles;
  }
  gp.n = n;
  if (!launch(em, args[0].a_kmajor, args[0].b_kmajor, true, G, st, gp)) return 0;
  NSTL_LAUNCH_CHECK("nstl_gemm_grouped (4-wave persistent)");
  nstl::count(NSTL_K_GEMM4);
  nstl::count(NSTL_K_GEMM4_TILES, tiles);
  *handled = 1;
  return 0;
}

}  // namespace nstl
