// Issue cost of the vector integer ops a dropout hash is built from, for one
// wave alone on its SIMD (the 4-wave GEMM's epilogue situation): 16 independent
// chains of one instruction, timed with s_memtime inside the kernel.
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/valu_rate tools/micro/valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(512) void rate(unsigned* out, unsigned seed, int iters) {
  unsigned v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed + threadIdx.x * 16 + i;
  const unsigned c = seed | 0x9E3779B1u;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#define STEP(i)                                                                                     \
  if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "s"(c));              \
  if constexpr (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "s"(c));             \
  if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "s"(c));                 \
  if constexpr (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "s"(c));              \
  if constexpr (OP == 4) asm volatile("v_lshrrev_b32 %0, 13, %0\n\tv_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(v[(i + 1) & 15]));
    REP16(STEP)
#undef STEP
  }
  const long long t1 = clock64();
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= v[i];
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = (unsigned)(t1 - t0);
    out[2 * blockIdx.x + 1] = acc;
  }
}

int main(int argc, char** argv) {
  // argv[1]: waves per workgroup (one workgroup per CU: 1 = one wave alone on a SIMD, 8 = two per SIMD)
  const int waves = argc > 1 ? atoi(argv[1]) : 1;
  unsigned* d;
  hipMalloc(&d, 2 * 256 * sizeof(unsigned));
  unsigned h[512];
  const int iters = 4096;
  const char* names[] = {"v_mul_lo_u32", "v_mul_u32_u24", "v_add_u32", "v_mul_hi_u32", "v_lshrrev+v_xor (2 ops)"};
  void (*ks[])(unsigned*, unsigned, int) = {rate<0>, rate<1>, rate<2>, rate<3>, rate<4>};
  for (int rep = 0; rep < 2; ++rep)
    for (int k = 0; k < 5; ++k) {
      hipLaunchKernelGGL(ks[k], dim3(256), dim3(64 * waves), 0, 0, d, 12345u + rep, iters);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < 256; ++b) s += h[2 * b];
      // s_memtime counts at the shader clock
      printf("rep %d  %d waves/CU  %-26s %6.2f cycles per instruction and wave\n", rep, waves, names[k],
             s / 256.0 / ((double)iters * 16 * (k == 4 ? 2 : 1)));
    }
  return 0;
}
