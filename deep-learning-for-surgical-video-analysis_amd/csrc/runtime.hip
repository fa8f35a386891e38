// svk runtime: error reporting and version for the C ABI.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "svk_common.h"

namespace svk {

static thread_local char g_err[512] = "";
static thread_local const char* g_last_kernel = "";

void set_last_kernel(const char* name) { g_last_kernel = name; }
static thread_local const char* g_pk_reject = "";
void set_pk_reject(const char* why) { g_pk_reject = why; }
const char* pk_reject() { return g_pk_reject; }

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

// Tuning knobs (tile configuration / kernel variant overrides for A/B measurements in one process);
// initial values from the environment, -1 = automatic choice.  Every value selects a complete kernel variant.
static const char* const k_knob_names[TUNE_NKNOBS] = {"pk_cfg", "pk_elds", "dw_lds", "dw_rows", "attn_cfg"};
static const char* const k_knob_env[TUNE_NKNOBS] = {"SVK_PK_CFG", "SVK_PK_ELDS", "SVK_DW_LDS", "SVK_DW_LR", "SVK_ATTN_CFG"};
static int init_knob(int i) {
  const char* e = getenv(k_knob_env[i]);
  return e ? atoi(e) : -1;
}
int g_tune[TUNE_NKNOBS] = {init_knob(0), init_knob(1), init_knob(2), init_knob(3), init_knob(4)};

#ifdef SVK_DIAG
int diag_knob(const char* env) {
  const char* e = getenv(env);
  return e ? atoi(e) : 0;
}
#endif

}  // namespace svk

extern "C" int svk_tune(const char* knob, int value) {
  for (int i = 0; i < svk::TUNE_NKNOBS; ++i)
    if (knob && strcmp(knob, svk::k_knob_names[i]) == 0) {
      svk::g_tune[i] = value;
      return SVK_OK;
    }
  svk::set_error("svk_tune: unknown knob %s", knob ? knob : "(null)");
  return SVK_EINVAL;
}

extern "C" const char* svk_version(void) { return "svk 0.1.0 gfx950"; }
extern "C" const char* svk_last_error(void) { return svk::g_err; }
extern "C" const char* svk_last_kernel(void) { return svk::g_last_kernel; }
