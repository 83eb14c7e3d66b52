// Error plumbing for the C ABI: no exception crosses it; the last error text is
// kept per host thread.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string>

namespace nstl {
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...);
void count(int which, long long n = 1);  // nstl_kernel_counts (NSTL_K_*)
// Workgroups a persistent one-per-CU grid may launch on stream `st`: 32 x the
// fewest CUs the stream's CU mask leaves on any (XCD, shader engine) pair (mask
// bit i is a CU of XCD i % 8, SE (i / 8) % 4, tools/micro/cu_probe.hip;
// workgroups are dealt round-robin over the XCDs and their SEs, so one with
// fewer CUs than its share would run a second round).  NSTL_PERSIST_CUS=<n>
// caps it (tests of the stream-K tail).
int stream_cus(hipStream_t st);
// The device a stream belongs to (hipStreamGetDevice; the current device for
// the null stream or on failure): per-device workspaces are keyed and allocated
// on it, not on whatever device is current when a call is made.
int stream_device(hipStream_t st);
// makes `dev` current for its scope (allocations for another device's stream)
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace nstl

#define NSTL_CHECK_ARG(cond, ...)                                         \
  do {                                                                    \
    if (!(cond)) return nstl::fail((int)hipErrorInvalidValue, __VA_ARGS__); \
  } while (0)

#define NSTL_LAUNCH_CHECK(what)                                            \
  do {                                                                     \
    hipError_t e__ = hipGetLastError();                                    \
    if (e__ != hipSuccess)                                                 \
      return nstl::fail((int)e__, "%s: launch failed: %s", what, hipGetErrorString(e__)); \
  } while (0)
