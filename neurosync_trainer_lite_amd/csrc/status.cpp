#include "status.h"

#include <stdarg.h>

#include <atomic>

#include "../../include/nstl.h"

namespace nstl {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code == 0 ? 1 : code;
}
static std::atomic<long long> g_counts[NSTL_K_COUNT];

void count(int which, long long n) {
  if (which >= 0 && which < NSTL_K_COUNT) g_counts[which].fetch_add(n, std::memory_order_relaxed);
}
}  // namespace nstl

extern "C" int nstl_kernel_counts(int64_t* out, int n) {
  for (int i = 0; out != nullptr && i < n && i < NSTL_K_COUNT; ++i)
    out[i] = nstl::g_counts[i].load(std::memory_order_relaxed);
  return NSTL_K_COUNT;
}

extern "C" void nstl_kernel_counts_reset(void) {
  for (auto& c : nstl::g_counts) c.store(0, std::memory_order_relaxed);
}

extern "C" const char* nstl_last_error_string(void) { return nstl::g_last_error.c_str(); }
extern "C" int nstl_version(void) { return 1; }
