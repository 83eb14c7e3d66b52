// Microbenchmark: the GEMM epilogue's store pattern alone.  1024 workgroups of
// 512 threads each write a 256 x 256 bf16 tile of a 16384 x 4096 matrix, 16 B
// per lane, a wave instruction covering 8 rows x 128 B (the ring kernel's
// layout), vs. contiguous 512 B row segments.  hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(512) void store_gemm_pattern(uint4* C, int N) {
  const int nt_n = N / 256;
  const int tm = blockIdx.x / nt_n, tn = blockIdx.x % nt_n;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const uint4 v = make_uint4(lane, wave, tm, tn);
  for (int it = 0; it < 16; ++it) {
    const int r = tm * 256 + wm * 128 + it * 8 + lane / 8;
    const int c = tn * 256 + wn * 64 + (lane % 8) * 8;
    C[((size_t)r * N + c) / 8] = v;
  }
}

__global__ __launch_bounds__(512) void store_rows(uint4* C, int N) {
  const int nt_n = N / 256;
  const int tm = blockIdx.x / nt_n, tn = blockIdx.x % nt_n;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint4 v = make_uint4(lane, wave, tm, tn);
  for (int it = 0; it < 16; ++it) {  // wave instr: 2 rows x 512 B
    const int r = tm * 256 + (wave * 16 + it) * 2 + lane / 32;
    const int c = tn * 256 + (lane % 32) * 8;
    C[((size_t)r * N + c) / 8] = v;
  }
}

int main() {
  const int M = 16384, N = 4096;
  uint4* C;
  hipMalloc(&C, (size_t)M * N * 2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int k = 0; k < 2; ++k) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k ? store_rows : store_gemm_pattern, dim3(1024), dim3(512), 0, 0, C, N);
    hipEventRecord(a);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k ? store_rows : store_gemm_pattern, dim3(1024), dim3(512), 0, 0, C, N);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%s: %.1f us per 128 MB (%.2f TB/s)\n", k ? "row segments" : "gemm pattern", ms / 20 * 1e3,
           (double)M * N * 2 / (ms / 20 * 1e-3) / 1e12);
  }
  return 0;
}
