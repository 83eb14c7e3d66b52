// Gradient exchange without compute units (the copy-engine ZeRO-1 reduction,
// parallel.ShardPusher): memory shared between the rank processes of one node
// through HIP IPC handles, and device-to-device copies that run on the copy
// engines (hipMemcpyDeviceToDeviceNoCU: SDMA, no kernel, no CU), so the
// gradient slices move during backward without taking CUs from its persistent
// GEMM grids.  Replaces the reference's per-parameter gather to cuda:0
// (/root/reference/utils/training_utils.py:228-257).  Host code only.
#include <string.h>

#include "../../include/nstl.h"
#include "status.h"

static_assert(sizeof(hipIpcMemHandle_t) == NSTL_IPC_HANDLE_BYTES, "IPC handle size");

// the handle names the whole allocation holding ptr (a caching allocator hands
// out pieces of larger ones): its base is found first, and ptr's offset in it
// is returned beside the handle
extern "C" int nstl_ipc_handle(const void* ptr, void* handle_out, int64_t* offset_out) {
  NSTL_CHECK_ARG(ptr && handle_out && offset_out, "nstl_ipc_handle: null pointer");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
  if (e != hipSuccess) return nstl::fail((int)e, "nstl_ipc_handle: hipMemGetAddressRange: %s", hipGetErrorString(e));
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, (void*)base);
  if (e != hipSuccess) return nstl::fail((int)e, "nstl_ipc_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
  memcpy(handle_out, &h, sizeof(h));
  *offset_out = (int64_t)((const char*)ptr - (const char*)base);
  return 0;
}

extern "C" int nstl_ipc_open(const void* handle, void** ptr_out) {
  NSTL_CHECK_ARG(handle && ptr_out, "nstl_ipc_open: null pointer");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  const hipError_t e = hipIpcOpenMemHandle(ptr_out, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return nstl::fail((int)e, "nstl_ipc_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int nstl_ipc_close(void* ptr) {
  NSTL_CHECK_ARG(ptr, "nstl_ipc_close: null pointer");
  const hipError_t e = hipIpcCloseMemHandle(ptr);
  if (e != hipSuccess) return nstl::fail((int)e, "nstl_ipc_close: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int nstl_copy_engine(void* dst, const void* src, int64_t bytes, void* stream) {
  NSTL_CHECK_ARG(dst && src && bytes >= 0, "nstl_copy_engine: bad args");
  if (bytes == 0) return 0;
  const hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDeviceNoCU, (hipStream_t)stream);
  if (e != hipSuccess) return nstl::fail((int)e, "nstl_copy_engine: hipMemcpyAsync: %s", hipGetErrorString(e));
  return 0;
}
