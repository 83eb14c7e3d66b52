#include "status.h"

#include <stdarg.h>

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
}  // namespace nstl

extern "C" const char* nstl_last_error_string(void) { return nstl::g_last_error.c_str(); }
extern "C" int nstl_version(void) { return 1; }
