// Which physical CU (XCC, SE, SH, CU from the hardware id registers) each bit of a
// stream CU mask (hipExtStreamCreateWithCUMask) controls: for every bit i, a
// stream with all bits but i set runs 8192 short workgroups that record where
// they ran; the one (xcc, se, sh, cu) missing from the unmasked run's set is bit
// i's CU.  Prints "bit i -> xcc x se s sh h cu c" per bit and the per-XCC count
// of bits.  hipcc --offload-arch=gfx950 -O2 cu_probe.hip -o cu_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <set>
#include <vector>

__global__ void where(unsigned* out) {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // a few microseconds of work so the workgroups spread over every CU
  float x = threadIdx.x;
  for (int i = 0; i < 2000; ++i) x = x * 0.999f + 1.0f;
  if (threadIdx.x == 0) out[blockIdx.x] = ((xcc & 0xF) << 16) | (hw & 0xFFFF) | (x < 0 ? 1u << 31 : 0u);
}

static unsigned key(unsigned v) {  // xcc, se, sh, cu
  const unsigned hw = v & 0xFFFF, xcc = (v >> 16) & 0xF;
  const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
  return (xcc << 12) | (se << 8) | (sh << 4) | cu;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int NB = 8192;
  unsigned* d;
  hipMalloc(&d, NB * 4);
  std::vector<unsigned> h(NB);
  auto run = [&](hipStream_t s, std::set<unsigned>& seen) {
    hipLaunchKernelGGL(where, dim3(NB), dim3(64), 0, s, d);
    if (hipStreamSynchronize(s) != hipSuccess) { printf("sync failed\n"); exit(1); }
    hipMemcpy(h.data(), d, NB * 4, hipMemcpyDeviceToHost);
    for (unsigned v : h) seen.insert(key(v));
  };
  std::set<unsigned> all;
  run(0, all);
  printf("unmasked: %zu distinct CUs (device reports %d)\n", all.size(), ncu);
  const int words = (ncu + 31) / 32;
  int per_xcc[16] = {0};
  for (int i = 0; i < ncu; ++i) {
    std::vector<uint32_t> m(words, 0);
    for (int c = 0; c < ncu; ++c)
      if (c != i) m[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) { printf("mask %d: create failed\n", i); return 1; }
    std::set<unsigned> seen;
    run(s, seen);
    hipStreamDestroy(s);
    std::vector<unsigned> miss;
    for (unsigned k : all)
      if (!seen.count(k)) miss.push_back(k);
    printf("bit %3d ->", i);
    for (unsigned k : miss) printf(" xcc %u se %u sh %u cu %u", k >> 12, (k >> 8) & 0xF, (k >> 4) & 1, k & 0xF);
    if (miss.size() == 1) per_xcc[miss[0] >> 12]++;
    printf("%s\n", miss.size() == 1 ? "" : "  (not exactly one)");
  }
  printf("bits per xcc:");
  for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
  printf("\n");
  return 0;
}
