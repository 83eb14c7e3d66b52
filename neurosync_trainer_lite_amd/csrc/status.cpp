#include "status.h"

#include <stdarg.h>

#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <map>

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

// mask bit i: XCD i % 8, shader engine (i / 8) % 4 (tools/micro/cu_probe.hip);
// workgroups are dealt round-robin over the XCDs and, inside one, over its 4
// shader engines, so a one-per-CU grid is 32 x the fewest CUs of any (XCD, SE)
extern "C" int nstl_mask_grid(const uint32_t* mask, int ncu) {
  if (mask == nullptr || ncu <= 0 || ncu % 32) return 0;
  int per[32] = {0};
  for (int i = 0; i < ncu; ++i) per[(i % 8) * 4 + (i / 8) % 4] += (mask[i / 32] >> (i % 32)) & 1;
  int lo = per[0];
  for (int x = 1; x < 32; ++x) lo = per[x] < lo ? per[x] : lo;
  return 32 * lo;
}

namespace nstl {
int stream_device(hipStream_t st) {
  int dev = 0;
  if (st != nullptr && hipStreamGetDevice(st, &dev) == hipSuccess) return dev;
  (void)hipGetLastError();
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  return dev;
}

static int stream_cus_query(hipStream_t st) {
  static int cus[64] = {0};
  const int dev = stream_device(st);
  if (dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 0;
    cus[dev] = n;
  }
  const int ncu = cus[dev];
  int g = ncu;
  uint32_t m[32] = {0};
  const int words = (ncu + 31) / 32;
  if (ncu % 32 == 0 && words <= 32 && hipExtStreamGetCUMask(st, (uint32_t)words, m) == hipSuccess) {
    const int mg = nstl_mask_grid(m, ncu);
    if (mg > 0) g = mg;
  } else {
    (void)hipGetLastError();  // no mask (or not queryable): every CU
  }
  return g;
}

// NSTL_PERSIST_CUS caps the grid (tests of the stream-K tail; read per call)
static int persist_cap(int g) {
  const char* e = getenv("NSTL_PERSIST_CUS");
  const int cap = e ? atoi(e) : 0;
  return cap > 0 && cap < g ? cap : g;
}

// A stream's CU mask is fixed when it is created, so the grid is cached per
// stream handle (the query is a runtime call per GEMM launch otherwise).  A
// handle reused by a new stream with another mask would keep the old grid: a
// speed matter only, every persistent kernel runs any grid size correctly.
// (The null stream is per device: keyed by the current device.)
int stream_cus(hipStream_t st) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, int> cache;
  int dev = -1;
  if (st == nullptr && hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return persist_cap(stream_cus_query(st));
  }
  const std::pair<int, hipStream_t> key(dev, st);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return persist_cap(it->second);
  }
  const int g = stream_cus_query(st);
  if (g > 0) {
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 1024) cache.clear();
    cache[key] = g;
  }
  return persist_cap(g);
}
}  // namespace nstl

extern "C" int nstl_kernel_counts(int64_t* out, int n) {
  for (int i = 0; out != nullptr && i < n && i < NSTL_K_COUNT; ++i)
    out[i] = nstl::g_counts[i].load(std::memory_order_relaxed);
  return NSTL_K_COUNT;
}

extern "C" int nstl_stream_cus(void* stream) { return nstl::stream_cus((hipStream_t)stream); }

extern "C" void nstl_kernel_counts_reset(void) {
  for (auto& c : nstl::g_counts) c.store(0, std::memory_order_relaxed);
}

extern "C" const char* nstl_last_error_string(void) { return nstl::g_last_error.c_str(); }
extern "C" int nstl_version(void) { return 1; }
