// errors.cpp — thread-local last-error buffer behind ofx_last_error().
#include <string.h>

#include "ofx_internal.h"

namespace {
thread_local char g_last_error[1024] = {0};
}

namespace ofx {
int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}
void clear_error() { g_last_error[0] = 0; }
}  // namespace ofx

extern "C" const char* ofx_last_error(void) { return g_last_error; }
extern "C" const char* ofx_version(void) { return "ofx-spmm 0.1.0 gfx950"; }
