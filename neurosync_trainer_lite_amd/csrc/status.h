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
