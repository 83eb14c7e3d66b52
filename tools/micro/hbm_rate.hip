// HBM stream rates of the access patterns the step's memory-bound kernels use
// (round 6): what a plain 16-byte-per-lane stream kernel reaches on this box
// for R read streams + W write streams of one size, against the production
// kernels' rates (Adam: 4 f32 reads + 3 f32 writes + 1 bf16 write per element;
// LayerNorm backward: 2 bf16 + 1 f32 reads, 1 f32 + 1 bf16 writes).  Each
// kernel is a grid-stride loop, U 16-byte elements per lane in flight per
// pass; grids of 256 x k workgroups.  Median of 9 launches after 3 warm-ups.
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/hbm_rate tools/micro/hbm_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// R reads, W writes of n16 16-byte elements each; NT: nontemporal loads/stores
template <int R, int W, int U, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const f4* __restrict__ in, f4* __restrict__ out, long n16) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + (long)u * 256;
      f4 s = {0.f, 0.f, 0.f, 0.f};
      if (i < n16) {
#pragma unroll
        for (int r = 0; r < R; ++r) s += NT ? __builtin_nontemporal_load(in + (long)r * n16 + i) : in[(long)r * n16 + i];
      }
      v[u] = s;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + (long)u * 256;
      if (i < n16) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
          if (NT) __builtin_nontemporal_store(v[u] + (float)w, out + (long)w * n16 + i);
          else out[(long)w * n16 + i] = v[u] + (float)w;
        }
      }
    }
  }
}

template <int R, int W, int U, bool NT>
void run(const char* name, f4* in, f4* out, long n16, int grid_mult, hipStream_t st) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * grid_mult;
  std::vector<float> ts;
  for (int it = 0; it < 12; ++it) {
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL((stream_kernel<R, W, U, NT>), dim3(grid), dim3(256), 0, st, in, out, n16);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  const double bytes = (double)(R + W) * n16 * 16;
  printf("%-34s grid 256x%-2d U=%d %s  %8.1f us  %6.2f TB/s  (%.0f MB)\n", name, grid_mult, U, NT ? "nt" : "  ",
         ts[ts.size() / 2] * 1e3, bytes / (ts[ts.size() / 2] * 1e-3) / 1e12, bytes / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  // 235 M f32 = the 228M model's arena (Adam's element count); 16 M x 1024 / 4 for a
  // LayerNorm-sized stream
  const long n_adam16 = 235000000L / 4, n_ln16 = 16384L * 1024 / 4;
  f4 *in, *out;
  CK(hipMalloc(&in, 8 * n_adam16 * 16));
  CK(hipMalloc(&out, 4 * n_adam16 * 16));
  CK(hipMemset(in, 0, 8 * n_adam16 * 16));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int rep = 0; rep < 2; ++rep) {
    printf("# rep %d\n", rep);
    for (int gm : {4, 8, 16}) {
      run<1, 1, 4, false>("copy 940 MB (1R 1W)", in, out, n_adam16, gm, st);
      run<1, 1, 4, true>("copy 940 MB (1R 1W)", in, out, n_adam16, gm, st);
    }
    run<1, 1, 2, false>("copy 940 MB (1R 1W)", in, out, n_adam16, 8, st);
    run<1, 1, 8, false>("copy 940 MB (1R 1W)", in, out, n_adam16, 8, st);
    run<1, 0, 4, false>("read 940 MB (1R)", in, out, n_adam16, 8, st);
    run<0, 1, 4, false>("write 940 MB (1W)", in, out, n_adam16, 8, st);
    // Adam: 16 B/elem read (p, g, m, v f32) + 14 B written (p, m, v f32, p16 bf16) ~ 4R 3.5W
    run<4, 3, 2, false>("adam-like 4R 3W (940 MB each)", in, out, n_adam16, 8, st);
    run<4, 3, 2, true>("adam-like 4R 3W (940 MB each)", in, out, n_adam16, 8, st);
    run<4, 3, 1, true>("adam-like 4R 3W (940 MB each)", in, out, n_adam16, 8, st);
    run<4, 3, 2, true>("adam-like 4R 3W (940 MB each)", in, out, n_adam16, 16, st);
    // LayerNorm backward: ~2 f32-sized reads + 1.5 f32-sized writes on 16384 x 1024
    run<3, 2, 4, false>("ln-bwd-like 3R 2W (67 MB each)", in, out, n_ln16, 8, st);
    run<3, 2, 4, true>("ln-bwd-like 3R 2W (67 MB each)", in, out, n_ln16, 8, st);
    run<2, 2, 4, false>("ln-fwd-like 2R 2W (33 MB each)", in, out, n_ln16 / 2, 8, st);
  }
  return 0;
}
