// svk runtime: error reporting and version for the C ABI.
#include <stdarg.h>
#include <stdio.h>

#include "svk_common.h"

namespace svk {

static thread_local char g_err[512] = "";
static thread_local const char* g_last_kernel = "";

void set_last_kernel(const char* name) { g_last_kernel = name; }

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SVK_ELAUNCH;
  }
  return SVK_OK;
}

}  // namespace svk

extern "C" const char* svk_version(void) { return "svk 0.1.0 gfx950"; }
extern "C" const char* svk_last_error(void) { return svk::g_err; }
extern "C" const char* svk_last_kernel(void) { return svk::g_last_kernel; }
