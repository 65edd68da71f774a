// C-ABI glue: version and thread-local error reporting for libkgx.
#include <cstdarg>
#include <cstdio>

#include "kgx.h"

namespace kgx {
namespace {
thread_local char g_err[1024] = "";
}
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace kgx

extern "C" int kgx_version(void) { return 1; }
extern "C" const char* kgx_last_error(void) { return kgx::g_err; }
