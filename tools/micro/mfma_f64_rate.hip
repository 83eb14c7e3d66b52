// Throughput of v_mfma_f64_16x16x4_f64 vs v_fma_f64 on this GPU (TF/s), to price
// the autocorrelation kernels.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double a, double b) {
  d4 acc[8];
  for (int t = 0; t < 8; ++t) acc[t] = d4{0, 0, 0, 0};
  double x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[t], 0, 0, 0);
  double s = 0;
  for (int t = 0; t < 8; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void fma_loop(double* out, int iters, double a, double b) {
  double acc[16];
  for (int t = 0; t < 16; ++t) acc[t] = t;
  double x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = fma(x, y, acc[t]);
  double s = 0;
  for (int t = 0; t < 16; ++t) s += acc[t];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NM, int NF>
__global__ __launch_bounds__(256) void mix_loop(double* out, int iters, double a, double b) {
  d4 acc[NM > 0 ? NM : 1];
  double f[NF > 0 ? NF : 1];
  for (int t = 0; t < NM; ++t) acc[t] = d4{0, 0, 0, 0};
  for (int t = 0; t < NF; ++t) f[t] = t;
  double x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < NM; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[t], 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int t = 0; t < NF; ++t) f[t] = fma(x, y, f[t]);
  }
  double s = 0;
  for (int t = 0; t < NM; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  for (int t = 0; t < NF; ++t) s += f[t];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NM, int NF>
void run_mix(double* out, int wg, int iters, hipEvent_t e0, hipEvent_t e1) {
  float ms = 0;
  hipLaunchKernelGGL((mix_loop<NM, NF>), dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((mix_loop<NM, NF>), dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double fm = (double)wg * 4 * iters * NM * 2048, ff = (double)wg * 256 * iters * 3 * NF * 2;
  printf("mix %d mfma + %d fma per iter: %.3f ms, mfma %.1f + fma %.1f = %.1f TF/s\n", NM, 3 * NF, ms,
         fm / ms / 1e9, ff / ms / 1e9, (fm + ff) / ms / 1e9);
}
int main() {
  const int wg = 256 * 8, iters = 2000;
  double* out;
  if (hipMalloc(&out, (size_t)wg * 256 * 8) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    float ms = 0;
    hipLaunchKernelGGL(mfma_loop, dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl_m = (double)wg * 4 * iters * 8 * 2048;
    printf("mfma_f64_16x16x4: %.3f ms, %.1f TF/s\n", ms, fl_m / ms / 1e9);
    hipLaunchKernelGGL(fma_loop, dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(fma_loop, dim3(wg), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl_f = (double)wg * 256 * iters * 16 * 2;
    printf("v_fma_f64:        %.3f ms, %.1f TF/s\n", ms, fl_f / ms / 1e9);
  }
  run_mix<4, 0>(out, wg, 1000, e0, e1);
  run_mix<0, 16>(out, wg, 1000, e0, e1);
  run_mix<4, 16>(out, wg, 1000, e0, e1);
  run_mix<4, 32>(out, wg, 1000, e0, e1);
  run_mix<2, 32>(out, wg, 1000, e0, e1);
  return hipDeviceSynchronize() != hipSuccess;
}
