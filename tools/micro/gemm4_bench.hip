// Microbenchmark + check of the 4-wave 256^2 GEMM (csrc/gemm4.h) on the 228M
// step's shapes.  hipcc -O3 --offload-arch=gfx950 -o tools/micro/gemm4_bench \
//   tools/micro/gemm4_bench.hip ; run on the GPU box.
// Each shape: max |C - ref| / max |ref| against an f32 naive GEMM on every 7th
// row, then the median of 20 timed launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "../../neurosync_trainer_lite_amd/csrc/gemm4.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void ref_gemm(const bf16* A, int64_t lda, const bf16* B, int64_t ldb, int bkm, float* C, int M, int N,
                         int K, int rstep) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y * rstep;
  if (j >= N || i >= M) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    const float b = bkm ? (float)B[(int64_t)j * ldb + k] : (float)B[(int64_t)k * ldb + j];
    s += (float)A[(int64_t)i * lda + k] * b;
  }
  C[(int64_t)blockIdx.y * N + j] = s;
}

__global__ void fill(bf16* x, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    x[i] = (bf16)(((float)(h & 0xFFFF) / 65536.f - 0.5f) * 0.2f);
  }
}

template <bool BKM, int DBG = 0>
void launch(const g4::Params& p, hipStream_t st) {
  static int G = 0;
  if (!G) {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    G = getenv("G4_ONESHOT") ? 1 << 30 : prop.multiProcessorCount;
  }
  g4::GroupParams gp{};
  gp.g[0] = p;
  gp.g[0].tiles_m = p.M / 256;
  gp.g[0].tiles_n = p.N / 256;
  gp.n = 1;
  gp.tile_end[0] = gp.g[0].tiles_m * gp.g[0].tiles_n;
  const int grid = std::min(G, gp.tile_end[0]);
  hipLaunchKernelGGL((g4::gemm4_kernel<true, BKM, g4::EM_BF16, false, DBG>), dim3(grid), dim3(g4::NT), 0, st, gp);
}
typedef void (*LaunchFn)(const g4::Params&, hipStream_t);

// the bf16 direct epilogue's store pattern alone (one 256^2 tile per workgroup)
__global__ __launch_bounds__(256, 1) void store_tile(bf16* C, int N, int ldc) {
  const int nt_n = N / 256;
  const int tm = blockIdx.x / nt_n, tn = blockIdx.x % nt_n;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, c = lane & 15, odd = g & 1;
  bf16* cbase = C + (int64_t)(tm * 256 + wm * 128 + c) * ldc + tn * 256 + wn * 128;
  const uint4 v = make_uint4(lane, wave, tm, tn);
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int bp = 0; bp < 8; bp += 2) *(uint4*)(cbase + (int64_t)(16 * a) * ldc + 16 * (bp + odd) + 4 * (g - odd)) = v;
}

// G4_DMA_AB=1: K-loop placement arms (now DBG 0 / 256 / 512, the read spread; the DMA
// placements 16, 32, 64, 128 measured slower, profiles/r4_gemm4_dma_placement.txt)
// alternated over three
// shapes after a warm-up block (the first blocks of a process run slow)
template <bool AK, bool BKM, int EM, int DBG>
void launch_any(const g4::GroupParams& gp, hipStream_t st) {
  hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, EM, false, DBG>), dim3(256), dim3(g4::NT), 0, st, gp);
}
int dma_ab(const bf16* A, const bf16* B, bf16* C, float* Cf, hipStream_t st) {
  struct Case { const char* name; int M, N, K; int kind; };  // kind 0 TT, 1 TN, 2 NN f32 (dW)
  const Case cs[] = {{"fwd ffn2 16384x1024x4096", 16384, 1024, 4096, 0},
                     {"dX  ffn2 16384x1024x4096", 16384, 1024, 4096, 1},
                     {"dW  4096^2 K=16384     ", 4096, 4096, 16384, 2}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  typedef void (*F)(const g4::GroupParams&, hipStream_t);
  const int dbgs[3] = {0, 512, 1024};
  const F fs[3][3] = {{launch_any<true, true, g4::EM_BF16, 0>, launch_any<true, true, g4::EM_BF16, 512>, launch_any<true, true, g4::EM_BF16, 1024>},
                      {launch_any<true, false, g4::EM_BF16, 0>, launch_any<true, false, g4::EM_BF16, 512>, launch_any<true, false, g4::EM_BF16, 1024>},
                      {launch_any<false, false, g4::EM_F32, 0>, launch_any<false, false, g4::EM_F32, 512>, launch_any<false, false, g4::EM_F32, 1024>}};
  for (int round = 0; round < 6; ++round)
    for (const Case& c : cs) {
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.M = c.M; p.N = c.N; p.K = c.K; p.alpha = 1.f;
      if (c.kind == 2) {  // dW = A^T B, A [K][M], B [K][N] (MN-major)
        p.A = (const char*)A; p.lda = c.M; p.B = (const char*)B; p.ldb = c.N; p.C = (char*)Cf; p.ldc = c.N;
        p.a_bytes = (uint32_t)((int64_t)c.K * c.M * 2); p.b_bytes = (uint32_t)((int64_t)c.K * c.N * 2);
      } else {
        p.A = (const char*)A; p.lda = c.K; p.B = (const char*)B; p.ldb = c.kind == 0 ? c.K : c.N; p.C = (char*)C; p.ldc = c.N;
        p.a_bytes = (uint32_t)((int64_t)c.M * c.K * 2); p.b_bytes = (uint32_t)((int64_t)c.N * c.K * 2);
      }
      p.tiles_m = c.M / 256; p.tiles_n = c.N / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      for (int arm = 0; arm < 4; ++arm) {
        const F f = fs[c.kind][arm];
        for (int w = 0; w < 3; ++w) f(gp, st);
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
          CK(hipEventRecord(e0, st)); f(gp, st); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        if (round > 0)
          printf("round %d  %s  dbg %2d  %8.1f us\n", round, c.name, dbgs[arm], ts[7] * 1e3);
        fflush(stdout);
      }
    }
  return 0;
}

// G4_R3_AB=1: the A3/B2 ring (R3: the stage DMA spread over both half-steps)
// against the two-stage ring, alternated after a warm-up block; outputs compared
// bit for bit (same accumulation order)
// R3 arms: 0 two-stage, 1 A3/B2, 2 B3/A2 (a tile's first step: all 16 pieces in h = 1),
// 3 A3/B2 with the first step split like the others (DBG 4096)
template <bool AK, bool BKM, int EM, int R3>
void launch_r3(const g4::GroupParams& gp, hipStream_t st) {
  const int grid = std::min(256, gp.tile_end[0]);
  if constexpr (R3 == 3)
    hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, EM, false, 4096, false, 1>), dim3(grid), dim3(g4::NT), 0, st, gp);
  else
    hipLaunchKernelGGL((g4::gemm4_kernel<AK, BKM, EM, false, 0, false, R3>), dim3(grid), dim3(g4::NT), 0, st, gp);
}
int r3_ab(const bf16* A, const bf16* B, bf16* C, float* Cf, hipStream_t st) {
  struct Case { const char* name; int M, N, K; int kind; };  // kind 0 TT, 1 TN, 2 NN f32 (dW)
  const Case cs[] = {{"fwd out  16384x1024x1024", 16384, 1024, 1024, 0},
                     {"fwd ffn1 16384x4096x1024", 16384, 4096, 1024, 0},
                     {"fwd ffn2 16384x1024x4096", 16384, 1024, 4096, 0},
                     {"dX  ffn2 16384x4096x1024", 16384, 4096, 1024, 1},
                     {"dX  ffn1 16384x1024x4096", 16384, 1024, 4096, 1},
                     {"dW  4096^2 K=16384     ", 4096, 4096, 16384, 2},
                     {"dW  1024x4096 K=16384  ", 1024, 4096, 16384, 2}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  typedef void (*F)(const g4::GroupParams&, hipStream_t);
  const F fs[3][4] = {{launch_r3<true, true, g4::EM_BF16, 0>, launch_r3<true, true, g4::EM_BF16, 1>, launch_r3<true, true, g4::EM_BF16, 2>, launch_r3<true, true, g4::EM_BF16, 3>},
                      {launch_r3<true, false, g4::EM_BF16, 0>, launch_r3<true, false, g4::EM_BF16, 1>, launch_r3<true, false, g4::EM_BF16, 2>, launch_r3<true, false, g4::EM_BF16, 3>},
                      {launch_r3<false, false, g4::EM_F32, 0>, launch_r3<false, false, g4::EM_F32, 1>, launch_r3<false, false, g4::EM_F32, 2>, launch_r3<false, false, g4::EM_F32, 3>}};
  const int64_t cmax = 16384LL * 4096;
  bf16* C2;
  float* Cf2;
  CK(hipMalloc(&C2, cmax * 2));
  CK(hipMalloc(&Cf2, 4096LL * 4096 * 4));
  for (int round = 0; round < 4; ++round)
    for (const Case& c : cs) {
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.M = c.M; p.N = c.N; p.K = c.K; p.alpha = 1.f;
      if (c.kind == 2) {  // dW = A^T B, A [K][M], B [K][N] (MN-major)
        p.A = (const char*)A; p.lda = c.M; p.B = (const char*)B; p.ldb = c.N; p.C = (char*)Cf; p.ldc = c.N;
        p.a_bytes = (uint32_t)((int64_t)c.K * c.M * 2); p.b_bytes = (uint32_t)((int64_t)c.K * c.N * 2);
      } else {
        p.A = (const char*)A; p.lda = c.K; p.B = (const char*)B; p.ldb = c.kind == 0 ? c.K : c.N; p.C = (char*)C; p.ldc = c.N;
        p.a_bytes = (uint32_t)((int64_t)c.M * c.K * 2); p.b_bytes = (uint32_t)((int64_t)c.N * c.K * 2);
      }
      p.tiles_m = c.M / 256; p.tiles_n = c.N / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      if (round == 0) {  // bitwise check: R3 (both assignments) against the two-stage kernel
        fs[c.kind][0](gp, st);
        CK(hipStreamSynchronize(st));
        for (int v = 1; v <= 3; ++v) {
          g4::GroupParams g2 = gp;
          g2.g[0].C = c.kind == 2 ? (char*)Cf2 : (char*)C2;
          CK(hipMemset(g2.g[0].C, 0xFF, (size_t)c.M * c.N * (c.kind == 2 ? 4 : 2)));
          fs[c.kind][v](g2, st);
          CK(hipStreamSynchronize(st));
          const size_t bytes = (size_t)c.M * c.N * (c.kind == 2 ? 4 : 2);
          std::vector<unsigned char> h1(bytes), h2(bytes);
          CK(hipMemcpy(h1.data(), gp.g[0].C, bytes, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h2.data(), g2.g[0].C, bytes, hipMemcpyDeviceToHost));
          size_t diff = 0;
          for (size_t i = 0; i < bytes; ++i) diff += h1[i] != h2[i];
          printf("check %s  R3=%d vs two-stage: %zu differing bytes of %zu %s\n", c.name, v, diff, bytes,
                 diff ? "BAD" : "ok");
        }
        fflush(stdout);
        continue;
      }
      for (int arm = 0; arm < 4; ++arm) {
        const F f = fs[c.kind][arm];
        for (int w = 0; w < 3; ++w) f(gp, st);
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
          CK(hipEventRecord(e0, st)); f(gp, st); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double us = ts[7] * 1e3, fl = 2.0 * c.M * c.N * c.K;
        printf("round %d  %s  %-9s %8.1f us  %7.1f TF/s\n", round, c.name, arm == 0 ? "two-stage" : arm == 1 ? "A3/B2" : arm == 2 ? "B3/A2" : "A3 split1",
               us, fl / us * 1e-6);
        fflush(stdout);
      }
    }
  return 0;
}

// G4_STORE_AB=1: the bf16 epilogue with and without its global stores (DBG 8192,
// timing only): how much of a multi-tile K = 1024 launch the output drain costs
int store_ab(const bf16* A, const bf16* B, bf16* C, hipStream_t st) {
  struct Case { const char* name; int M, N, K; int kind; };  // kind 0 TT, 1 TN
  const Case cs[] = {{"fwd out  16384x1024x1024", 16384, 1024, 1024, 0},
                     {"fwd qkv  16384x3072x1024", 16384, 3072, 1024, 0},
                     {"fwd ffn1 16384x4096x1024", 16384, 4096, 1024, 0},
                     {"dX  ffn2 16384x4096x1024", 16384, 4096, 1024, 1},
                     {"fwd ffn2 16384x1024x4096", 16384, 1024, 4096, 0}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  typedef void (*F)(const g4::GroupParams&, hipStream_t);
  const F fs[2][2] = {{launch_any<true, true, g4::EM_BF16, 0>, launch_any<true, true, g4::EM_BF16, 8192>},
                      {launch_any<true, false, g4::EM_BF16, 0>, launch_any<true, false, g4::EM_BF16, 8192>}};
  for (int round = 0; round < 4; ++round)
    for (const Case& c : cs) {
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.M = c.M; p.N = c.N; p.K = c.K; p.alpha = 1.f;
      p.A = (const char*)A; p.lda = c.K; p.B = (const char*)B; p.ldb = c.kind == 0 ? c.K : c.N; p.C = (char*)C; p.ldc = c.N;
      p.a_bytes = (uint32_t)((int64_t)c.M * c.K * 2); p.b_bytes = (uint32_t)((int64_t)c.N * c.K * 2);
      p.tiles_m = c.M / 256; p.tiles_n = c.N / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      for (int arm = 0; arm < 2; ++arm) {
        const F f = fs[c.kind][arm];
        for (int w = 0; w < 3; ++w) f(gp, st);
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
          CK(hipEventRecord(e0, st)); f(gp, st); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double us = ts[7] * 1e3, fl = 2.0 * c.M * c.N * c.K;
        if (round > 0)
          printf("round %d  %s  %-9s %8.1f us  %7.1f TF/s\n", round, c.name, arm == 0 ? "stores" : "no stores", us, fl / us * 1e-6);
        fflush(stdout);
      }
    }
  return 0;
}

// G4_F8_ABL=1: the fp8 4-wave kernel (gemm4f8_kernel, bf16 out, unit scales) on the
// step's K-major shapes, with ablations (timing only: results are wrong), beside the
// bf16 kernel on the same shape; arms alternated after a warm-up round
__global__ void fill_f8(uint8_t* x, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    const float v = ((float)(h & 0xFFFF) / 65536.f - 0.5f) * 200.f;  // |v| < 100: inside e4m3's range
    x[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false) & 0xFF);
  }
}
__global__ void fill_one(float* x, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = 1.f;
}
template <int DBG>
void launch_f8(const g4::GroupParams& gp, hipStream_t st) {
  hipLaunchKernelGGL((g4::gemm4f8_kernel<g4::EM_BF16, DBG>), dim3(std::min(256, gp.tile_end[0])), dim3(g4::NT), 0, st, gp);
}
int f8_abl(const bf16* A, const bf16* B, bf16* C, hipStream_t st) {
  struct Case { const char* name; int M, N, K; };
  const Case cs[] = {{"fwd out  16384x1024x1024", 16384, 1024, 1024},
                     {"fwd qkv  16384x3072x1024", 16384, 3072, 1024},
                     {"fwd ffn1 16384x4096x1024", 16384, 4096, 1024},
                     {"fwd ffn2 16384x1024x4096", 16384, 1024, 4096},
                     {"sq 4096x4096 K=8192     ", 4096, 4096, 8192}};
  uint8_t *A8, *B8;
  float* ones;
  CK(hipMalloc(&A8, 16384LL * 8192));
  CK(hipMalloc(&B8, 16384LL * 8192));
  CK(hipMalloc(&ones, 16384 * 4));
  hipLaunchKernelGGL(fill_f8, dim3(4096), dim3(256), 0, st, A8, 16384LL * 8192, 3u);
  hipLaunchKernelGGL(fill_f8, dim3(4096), dim3(256), 0, st, B8, 16384LL * 8192, 4u);
  hipLaunchKernelGGL(fill_one, dim3(64), dim3(256), 0, st, ones, 16384);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  typedef void (*F)(const g4::GroupParams&, hipStream_t);
  const int dbgs[7] = {-1, 0, 8192, 1, 2, 3, 8};
  const char* names[7] = {"bf16 gemm4", "fp8", "fp8 no stores", "fp8 no DMA", "fp8 no reads", "fp8 MFMA only", "fp8 no MFMA"};
  const F fs[7] = {launch_any<true, true, g4::EM_BF16, 0>, launch_f8<0>, launch_f8<8192>, launch_f8<1>, launch_f8<2>,
                   launch_f8<3>, launch_f8<8>};
  for (int round = 0; round < 3; ++round)
    for (const Case& c : cs) {
      for (int arm = 0; arm < 7; ++arm) {
        g4::GroupParams gp{};
        g4::Params& p = gp.g[0];
        p.M = c.M; p.N = c.N; p.K = c.K; p.alpha = 1.f; p.C = (char*)C; p.ldc = c.N;
        if (dbgs[arm] < 0) {
          p.A = (const char*)A; p.lda = c.K; p.B = (const char*)B; p.ldb = c.K;
          p.a_bytes = (uint32_t)((int64_t)c.M * c.K * 2); p.b_bytes = (uint32_t)((int64_t)c.N * c.K * 2);
        } else {
          p.A = (const char*)A8; p.lda = c.K; p.B = (const char*)B8; p.ldb = c.K;
          p.a_bytes = (uint32_t)((int64_t)c.M * c.K); p.b_bytes = (uint32_t)((int64_t)c.N * c.K);
          p.a_scale = ones; p.b_scale = ones;
        }
        p.tiles_m = c.M / 256; p.tiles_n = c.N / 256;
        gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
        const F f = fs[arm];
        for (int w = 0; w < 3; ++w) f(gp, st);
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
          CK(hipEventRecord(e0, st)); f(gp, st); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double us = ts[7] * 1e3, fl = 2.0 * c.M * c.N * c.K;
        if (round > 0)
          printf("round %d  %s  %-14s %8.1f us  %7.1f TF/s\n", round, c.name, names[arm], us, fl / us * 1e-6);
        fflush(stdout);
      }
    }
  return 0;
}

// G4_EPI_COST=1: what each fused epilogue costs beside the plain bf16 one on its
// step shape (timing only): FFN1 forward (ReLU, + dropout hash, + keep-bit words),
// FFN2 dX (dReLU from the keep bits, + bias column sums), q|k|v forward (RoPE)
int epi_cost(const bf16* A, const bf16* B, bf16* C, hipStream_t st) {
  uint64_t* mask;
  float *colsum, *rc, *rs;
  CK(hipMalloc(&mask, 16384LL * 4096 / 8));
  CK(hipMemset(mask, 0x5A, 16384LL * 4096 / 8));
  CK(hipMalloc(&colsum, 128LL * 4096 * 4));
  CK(hipMalloc(&rc, 128 * 32 * 4));
  CK(hipMalloc(&rs, 128 * 32 * 4));
  CK(hipMemset(rc, 0, 128 * 32 * 4));
  CK(hipMemset(rs, 0, 128 * 32 * 4));
  float* bias;
  CK(hipMalloc(&bias, 4096 * 4));
  CK(hipMemset(bias, 0, 4096 * 4));
  // cold keep-bit words: 40 copies (320 MB, past the Infinity Cache), one per launch
  uint64_t* cold;
  const int64_t mwords = 16384LL * 4096 / 64;
  CK(hipMalloc(&cold, 40 * mwords * 8));
  CK(hipMemset(cold, 0x5A, 40 * mwords * 8));
  struct Arm { const char* name; int M, N, K; bool bkm; int em; bool drop, msk, csum, bias = false, cold = false; int old = 0; };  // old: 1 DBG 16384 (no side data), 2 DBG 32768 (live refill)
  const Arm arms[] = {{"ffn1 fwd  bf16          ", 16384, 4096, 1024, true, g4::EM_BF16, false, false, false},
                      {"ffn1 fwd  relu          ", 16384, 4096, 1024, true, g4::EM_RELU_DROP, false, false, false},
                      {"ffn1 fwd  relu+drop     ", 16384, 4096, 1024, true, g4::EM_RELU_DROP, true, false, false},
                      {"ffn1 fwd  relu+mask     ", 16384, 4096, 1024, true, g4::EM_RELU_DROP, false, true, false},
                      {"ffn1 fwd  relu+drop+mask", 16384, 4096, 1024, true, g4::EM_RELU_DROP, true, true, false},
                      {"ffn2 dX   bf16          ", 16384, 4096, 1024, false, g4::EM_BF16, false, false, false},
                      {"ffn2 dX   drelu         ", 16384, 4096, 1024, false, g4::EM_DRELU, true, true, false},
                      {"ffn2 dX   drelu+colsum  ", 16384, 4096, 1024, false, g4::EM_DRELU, true, true, true},
                      {"qkv fwd   bf16          ", 16384, 3072, 1024, true, g4::EM_BF16, false, false, false},
                      {"qkv fwd   rope          ", 16384, 3072, 1024, true, g4::EM_ROPE, false, false, false},
                      {"ffn1 fwd  bf16 +bias    ", 16384, 4096, 1024, true, g4::EM_BF16, false, false, false, true},
                      {"ffn1 fwd  r+d+m +bias   ", 16384, 4096, 1024, true, g4::EM_RELU_DROP, true, true, false, true},
                      {"qkv fwd   rope +bias    ", 16384, 3072, 1024, true, g4::EM_ROPE, false, false, false, true},
                      {"ffn2 dX   drelu+cs cold ", 16384, 4096, 1024, false, g4::EM_DRELU, true, true, true, false, true},
                      {"ffn1 fwd  r+d+m +bias OLD", 16384, 4096, 1024, true, g4::EM_RELU_DROP, true, true, false, true, false, true},
                      {"ffn1 fwd  bf16 +bias OLD", 16384, 4096, 1024, true, g4::EM_BF16, false, false, false, true, false, true},
                      {"ffn2 dX   drelu+cs cold OLD", 16384, 4096, 1024, false, g4::EM_DRELU, true, true, true, false, true, true},
                      {"out fwd   bf16 +bias    ", 16384, 1024, 1024, true, g4::EM_BF16, false, false, false, true},
                      {"out fwd   bf16 +bias OLD", 16384, 1024, 1024, true, g4::EM_BF16, false, false, false, true, false, true},
                      {"out fwd   bf16 +bias REFILL", 16384, 1024, 1024, true, g4::EM_BF16, false, false, false, true, false, 2},
                      {"ffn1 fwd  r+d+m +bias REFILL", 16384, 4096, 1024, true, g4::EM_RELU_DROP, true, true, false, true, false, 2},
                      {"out dX    bf16          ", 16384, 1024, 1024, false, g4::EM_BF16, false, false, false},
                      {"out dX    bf16 REFILL   ", 16384, 1024, 1024, false, g4::EM_BF16, false, false, false, false, false, 2}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 4; ++round)
    for (const Arm& c : arms) {
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.M = c.M; p.N = c.N; p.K = c.K; p.alpha = 1.f;
      p.A = (const char*)A; p.lda = c.K; p.B = (const char*)B; p.ldb = c.bkm ? c.K : c.N; p.C = (char*)C; p.ldc = c.N;
      p.a_bytes = (uint32_t)((int64_t)c.M * c.K * 2); p.b_bytes = (uint32_t)((int64_t)c.N * c.K * 2);
      p.inv_keep = 1.f / 0.7f; p.thresh = c.drop ? 19661u : 0u; p.seed = 1234;
      p.relu_mask = c.msk ? mask : nullptr;
      p.bias = c.bias ? bias : nullptr;
      int launch_no = 0;
      p.colsum_part = c.csum ? colsum : nullptr;
      p.rope_cos = rc; p.rope_sin = rs; p.rope_T = 128; p.rope_dim = 64; p.rope_cols = 2048;
      p.tiles_m = c.M / 256; p.tiles_n = c.N / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      typedef void (*F)(const g4::GroupParams&, hipStream_t);
      F f = nullptr;
      if (c.em == g4::EM_BF16)
        f = c.old == 1 ? launch_any<true, true, g4::EM_BF16, 16384>
            : c.old == 2 ? (c.bkm ? launch_any<true, true, g4::EM_BF16, 32768> : launch_any<true, false, g4::EM_BF16, 32768>)
                         : (c.bkm ? launch_any<true, true, g4::EM_BF16, 0> : launch_any<true, false, g4::EM_BF16, 0>);
      if (c.em == g4::EM_RELU_DROP)
        f = c.old == 1 ? launch_any<true, true, g4::EM_RELU_DROP, 16384>
            : c.old == 2 ? launch_any<true, true, g4::EM_RELU_DROP, 32768> : launch_any<true, true, g4::EM_RELU_DROP, 0>;
      if (c.em == g4::EM_DRELU)
        f = c.old ? launch_any<true, false, g4::EM_DRELU, 16384> : launch_any<true, false, g4::EM_DRELU, 0>;
      if (c.em == g4::EM_ROPE) f = launch_any<true, true, g4::EM_ROPE, 0>;
      auto run = [&]() {
        if (c.cold) gp.g[0].relu_mask = cold + (launch_no++ % 40) * mwords;
        f(gp, st);
      };
      for (int w = 0; w < 3; ++w) run();
      std::vector<float> ts;
      for (int r = 0; r < 15; ++r) {
        CK(hipEventRecord(e0, st)); run(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      // sustained: 100 launches back to back (the clock a busy step holds), mean
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < 100; ++r) run();
      CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float msum; CK(hipEventElapsedTime(&msum, e0, e1));
      const double us = ts[7] * 1e3, fl = 2.0 * c.M * c.N * c.K, sus = msum * 10.0;
      if (round > 0) printf("round %d  %s %8.1f us  %7.1f TF/s   sustained %8.1f us  %7.1f TF/s\n", round, c.name, us, fl / us * 1e-6, sus, fl / sus * 1e-6);
      fflush(stdout);
    }
  return 0;
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int M, N, K, bkm; };
  const Shape shapes[] = {
      {"fwd out   16384x1024x1024", 16384, 1024, 1024, 1},
      {"fwd ffn2  16384x1024x4096", 16384, 1024, 4096, 1},
      {"fwd ffn1  16384x4096x1024", 16384, 4096, 1024, 1},
      {"fwd qkv   16384x3072x1024", 16384, 3072, 1024, 1},
      {"dX  out   16384x1024x1024", 16384, 1024, 1024, 0},
      {"dX  ffn2  16384x1024x4096", 16384, 1024, 4096, 0},
      {"dX  ffn1  16384x4096x1024", 16384, 4096, 1024, 0},
      {"sq  4096^3", 4096, 4096, 4096, 1},
  };
  const int reps = 20;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int64_t maxA = 16384LL * 4096, maxB = 4096LL * 4096, maxC = 16384LL * 4096;
  bf16 *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxA * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&R, maxC * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, A, maxA, 1u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, B, maxA, 2u);
  if (getenv("G4_R3_AB")) {
    float* Cf;
    CK(hipMalloc(&Cf, 4096LL * 4096 * 4));
    return r3_ab(A, B, C, Cf, st);
  }
  if (getenv("G4_STORE_AB")) return store_ab(A, B, C, st);
  if (getenv("G4_F8_ABL")) return f8_abl(A, B, C, st);
  if (getenv("G4_EPI_COST")) return epi_cost(A, B, C, st);
  if (getenv("G4_DMA_AB")) {
    float* Cf;
    CK(hipMalloc(&Cf, 4096LL * 4096 * 4));
    return dma_ab(A, B, C, Cf, st);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    g4::Params p{};
    p.A = (const char*)A; p.lda = s.K;
    p.B = (const char*)B; p.ldb = s.bkm ? s.K : s.N;
    p.C = (char*)C; p.ldc = s.N;
    p.M = s.M; p.N = s.N; p.K = s.K;
    p.alpha = 1.f; p.bias = nullptr;
    p.a_bytes = (uint32_t)((int64_t)s.M * s.K * 2);
    p.b_bytes = (uint32_t)((int64_t)s.N * s.K * 2);
    auto run = [&]() { if (s.bkm) launch<true>(p, st); else launch<false>(p, st); };
    run();
    CK(hipStreamSynchronize(st));
    const int rstep = 7, nr = (s.M + rstep - 1) / rstep;
    hipLaunchKernelGGL(ref_gemm, dim3((s.N + 255) / 256, nr), dim3(256), 0, st, A, (int64_t)s.K, B, p.ldb, s.bkm, R,
                       s.M, s.N, s.K, rstep);
    CK(hipStreamSynchronize(st));
    std::vector<bf16> hc((size_t)s.M * s.N);
    std::vector<float> hr((size_t)nr * s.N);
    CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
    double maxd = 0, maxr = 0;
    for (int r = 0; r < nr; ++r)
      for (int j = 0; j < s.N; ++j) {
        const double ref = hr[(size_t)r * s.N + j], got = (float)hc[(size_t)r * rstep * s.N + j];
        maxd = std::max(maxd, fabs(got - ref));
        maxr = std::max(maxr, fabs(ref));
      }
    for (int w = 0; w < 3; ++w) run();
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      run();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[reps / 2] * 1e3, fl = 2.0 * s.M * s.N * s.K;
    printf("%-28s %8.1f us  %7.1f TF/s  err %.2e %s\n", s.name, us, fl / us * 1e-6, maxd / maxr,
           maxd / maxr < 1e-2 ? "ok" : "BAD");
    fflush(stdout);
  }
  for (int n : {1024, 4096}) {
    const int tiles = 16384 / 256 * (n / 256);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_tile, dim3(tiles), dim3(256), 0, st, C, n, n);
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(store_tile, dim3(tiles), dim3(256), 0, st, C, n, n);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[reps / 2] * 1e3;
    printf("store-only 16384x%d (%d tiles): %.1f us, %.2f TB/s\n", n, tiles, us, 16384.0 * n * 2 / us * 1e-6);
  }
  {  // weight-gradient layout (A and B MN-major, f32 out): dW = dY^T X, K = tokens
    const int Mt = 16384;
    struct WS { const char* name; int n, k; };
    const WS ws[] = {{"dW  4096x4096 K=16384", 4096, 4096}, {"dW  1024x4096 K=16384", 1024, 4096},
                     {"dW  1024x1024 K=16384", 1024, 1024}};
    float* Cf;
    CK(hipMalloc(&Cf, 4096LL * 4096 * 4));
    for (const WS& w : ws) {
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.A = (const char*)A; p.lda = w.n; p.B = (const char*)B; p.ldb = w.k;
      p.C = (char*)Cf; p.ldc = w.k; p.M = w.n; p.N = w.k; p.K = Mt; p.alpha = 1.f;
      p.a_bytes = (uint32_t)((int64_t)Mt * w.n * 2); p.b_bytes = (uint32_t)((int64_t)Mt * w.k * 2);
      p.tiles_m = w.n / 256; p.tiles_n = w.k / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      const int grid = std::min(256, gp.tile_end[0]);
      auto run = [&]() {
        hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 0>), dim3(grid), dim3(g4::NT), 0, st, gp);
      };
      if ((int64_t)Mt * std::max(w.n, w.k) > maxA || (int64_t)Mt * w.k > maxA) continue;
      run();
      CK(hipStreamSynchronize(st));
      // check row 0 and row n-1 of the output against a direct sum
      std::vector<bf16> ha((size_t)Mt * w.n), hb((size_t)Mt * w.k);
      std::vector<float> hc((size_t)w.n * w.k);
      CK(hipMemcpy(ha.data(), A, ha.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hb.data(), B, hb.size() * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hc.data(), Cf, hc.size() * 4, hipMemcpyDeviceToHost));
      double maxd = 0, maxr = 0;
      for (int i : {0, w.n / 2 + 3, w.n - 1})
        for (int j = 0; j < w.k; j += 37) {
          double ref = 0;
          for (int r = 0; r < Mt; ++r) ref += (double)(float)ha[(size_t)r * w.n + i] * (double)(float)hb[(size_t)r * w.k + j];
          maxd = std::max(maxd, fabs(hc[(size_t)i * w.k + j] - ref));
          maxr = std::max(maxr, fabs(ref));
        }
      for (int it = 0; it < 3; ++it) run();
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st)); run(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[reps / 2] * 1e3, fl = 2.0 * w.n * w.k * Mt;
      printf("%-28s %8.1f us  %7.1f TF/s  err %.2e %s\n", w.name, us, fl / us * 1e-6, maxd / maxr,
             maxd / maxr < 1e-4 ? "ok" : "BAD");
      fflush(stdout);
    }
  }
  {  // ablations of the weight-gradient layout (dW 4096^2, K = 16384): timing only
    const int Mt = 16384, n = 4096, k = 4096;
    float* Cf;
    CK(hipMalloc(&Cf, (size_t)n * k * 4));
    g4::GroupParams gp{};
    g4::Params& p = gp.g[0];
    p.A = (const char*)A; p.lda = n; p.B = (const char*)B; p.ldb = k;
    p.C = (char*)Cf; p.ldc = k; p.M = n; p.N = k; p.K = Mt; p.alpha = 1.f;
    p.a_bytes = (uint32_t)((int64_t)Mt * n * 2); p.b_bytes = (uint32_t)((int64_t)Mt * k * 2);
    p.tiles_m = n / 256; p.tiles_n = k / 256;
    gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
    struct AblMM { int dbg; void (*f)(const g4::GroupParams&, hipStream_t); const char* what; };
    const AblMM am[] = {
        {0, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 0>), dim3(256), dim3(256), 0, s, g); }, "baseline"},
        {1, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 1>), dim3(256), dim3(256), 0, s, g); }, "no DMA in loop"},
        {2, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 2>), dim3(256), dim3(256), 0, s, g); }, "no frag reads"},
        {3, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 3>), dim3(256), dim3(256), 0, s, g); }, "no DMA, no reads"},
        {8, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 8>), dim3(256), dim3(256), 0, s, g); }, "no MFMA"},
        {16, [](const g4::GroupParams& g, hipStream_t s) { hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 16>), dim3(256), dim3(256), 0, s, g); }, "DMA early in h1"},
    };
    for (const AblMM& a : am) {
      for (int w = 0; w < 3; ++w) a.f(gp, st);
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st)); a.f(gp, st); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[reps / 2] * 1e3, fl = 2.0 * n * k * Mt;
      printf("  abl dW 4096^2 K=16384 dbg %d %-20s %8.1f us  %7.1f TF/s\n", a.dbg, a.what, us, fl / us * 1e-6);
    }
  }
  {  // dW 4096^2 (K = 15360 tokens) with padded operand row strides: do power-of-two
     // strides of the MN-major operands (the token rows) cost DMA intake?  timing only
    const int Mt = 15360, n = 4096, k = 4096;
    float* Cf;
    CK(hipMalloc(&Cf, (size_t)n * k * 4));
    for (int pad : {0, 64, 128, 256}) {
      // both operands live in maxA-element buffers: a padded stride must still fit
      // (a range past the allocation reads unmapped memory and faults the card)
      if ((int64_t)Mt * (std::max(n, k) + pad) > maxA) continue;
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.A = (const char*)A; p.lda = n + pad; p.B = (const char*)B; p.ldb = k + pad;
      p.C = (char*)Cf; p.ldc = k; p.M = n; p.N = k; p.K = Mt; p.alpha = 1.f;
      p.a_bytes = (uint32_t)((int64_t)Mt * (n + pad) * 2); p.b_bytes = (uint32_t)((int64_t)Mt * (k + pad) * 2);
      p.tiles_m = n / 256; p.tiles_n = k / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      auto run = [&]() {
        hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 0>), dim3(256), dim3(g4::NT), 0, st, gp);
      };
      for (int w = 0; w < 3; ++w) run();
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st)); run(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[reps / 2] * 1e3, fl = 2.0 * n * k * Mt;
      printf("  dW 4096^2 K=15360 operand stride +%3d elements %8.1f us  %7.1f TF/s\n", pad, us, fl / us * 1e-6);
      fflush(stdout);
    }
  }
  {  // dW at K = 16384 vs 15360 and 3840^2 vs 4096^2: is the K = 16384 slowdown the
     // operands' size (256 MB, the Infinity Cache) or the K extent?  timing only
    struct DS { int n, Mt; };
    const DS ds[] = {{4096, 16384}, {4096, 15360}, {3840, 16384}, {3840, 15360}, {4096, 8192}};
    float* Cf;
    CK(hipMalloc(&Cf, (size_t)4096 * 4096 * 4));
    for (const DS& d : ds) {
      if ((int64_t)d.Mt * d.n > maxA) continue;  // both operands live in maxA-element buffers
      g4::GroupParams gp{};
      g4::Params& p = gp.g[0];
      p.A = (const char*)A; p.lda = d.n; p.B = (const char*)B; p.ldb = d.n;
      p.C = (char*)Cf; p.ldc = d.n; p.M = d.n; p.N = d.n; p.K = d.Mt; p.alpha = 1.f;
      p.a_bytes = (uint32_t)((int64_t)d.Mt * d.n * 2); p.b_bytes = p.a_bytes;
      p.tiles_m = d.n / 256; p.tiles_n = d.n / 256;
      gp.n = 1; gp.tile_end[0] = p.tiles_m * p.tiles_n;
      const int grid = std::min(256, gp.tile_end[0]);
      auto run = [&]() {
        hipLaunchKernelGGL((g4::gemm4_kernel<false, false, g4::EM_F32, false, 0>), dim3(grid), dim3(g4::NT), 0, st, gp);
      };
      for (int w = 0; w < 3; ++w) run();
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st)); run(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[reps / 2] * 1e3, fl = 2.0 * d.n * d.n * d.Mt;
      printf("  dW %dx%d K=%d (operands %.0f MB)  %8.1f us  %7.1f TF/s\n", d.n, d.n, d.Mt,
             2.0 * d.Mt * d.n * 2 / 1048576.0, us, fl / us * 1e-6);
      fflush(stdout);
    }
  }
  {  // early DMA on the forward / dX shapes
    for (int bkm = 1; bkm >= 0; --bkm)
      for (int dbg : {0, 16}) {
        g4::Params p{};
        const int M = 16384, N = 1024, Kd = 4096;
        p.A = (const char*)A; p.lda = Kd; p.B = (const char*)B; p.ldb = bkm ? Kd : N;
        p.C = (char*)C; p.ldc = N; p.M = M; p.N = N; p.K = Kd; p.alpha = 1.f;
        p.a_bytes = (uint32_t)((int64_t)M * Kd * 2); p.b_bytes = (uint32_t)((int64_t)N * Kd * 2);
        auto f = [&]() {
          if (bkm) { if (dbg) launch<true, 16>(p, st); else launch<true, 0>(p, st); }
          else { if (dbg) launch<false, 16>(p, st); else launch<false, 0>(p, st); }
        };
        for (int w = 0; w < 3; ++w) f();
        std::vector<float> ts;
        for (int r = 0; r < reps; ++r) {
          CK(hipEventRecord(e0, st)); f(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double us = ts[reps / 2] * 1e3, fl = 2.0 * M * N * Kd;
        printf("  %s ffn2 16384x1024x4096 dbg %2d %8.1f us  %7.1f TF/s\n", bkm ? "fwd" : "dX ", dbg, us, fl / us * 1e-6);
      }
  }
  if (getenv("G4_NO_ABL")) return 0;
  // ablations on two single-round shapes (timing only: results are wrong)
  struct Abl { int dbg; LaunchFn f; const char* what; };
  const Abl abl[] = {
      {0, launch<true, 0>, "baseline"},
      {1, launch<true, 1>, "no DMA in loop"},
      {2, launch<true, 2>, "no frag reads"},
      {3, launch<true, 3>, "no DMA, no reads"},
      {7, launch<true, 7>, "MFMA only"},
      {8, launch<true, 8>, "no MFMA"},
  };
  const Shape ash[] = {{"fwd ffn2  16384x1024x4096", 16384, 1024, 4096, 1}, {"sq  4096^3", 4096, 4096, 4096, 1}};
  for (const Shape& s : ash) {
    g4::Params p{};
    p.A = (const char*)A; p.lda = s.K;
    p.B = (const char*)B; p.ldb = s.K;
    p.C = (char*)C; p.ldc = s.N;
    p.M = s.M; p.N = s.N; p.K = s.K;
    p.alpha = 1.f;
    p.a_bytes = (uint32_t)((int64_t)s.M * s.K * 2);
    p.b_bytes = (uint32_t)((int64_t)s.N * s.K * 2);
    for (const Abl& a : abl) {
      for (int w = 0; w < 3; ++w) a.f(p, st);
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st));
        a.f(p, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[reps / 2] * 1e3, fl = 2.0 * s.M * s.N * s.K;
      printf("  abl %-28s dbg %d %-22s %8.1f us  %7.1f TF/s\n", s.name, a.dbg, a.what, us, fl / us * 1e-6);
      fflush(stdout);
    }
  }
  return 0;
}
