// CU occupancy probe: nblocks workgroups that spin on the clock for `cycles`,
// each holding `lds_bytes` of LDS, on the given stream.  Used to measure how a
// training step degrades when another kernel (e.g. an RCCL all-reduce channel)
// holds some CUs while the step's 1-workgroup-per-CU GEMMs run.
#include <hip/hip_runtime.h>

__global__ void spin_kernel(long long cycles) {
  extern __shared__ char lds[];
  const long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < cycles) {
    if (threadIdx.x == 0) lds[0] = (char)t0;
    __builtin_amdgcn_s_sleep(8);
  }
}

extern "C" int cu_hog(int nblocks, int lds_bytes, long long cycles, void* stream) {
  hipLaunchKernelGGL(spin_kernel, dim3(nblocks), dim3(256), lds_bytes, (hipStream_t)stream, cycles);
  return (int)hipGetLastError();
}
