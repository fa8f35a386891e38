// svk runtime: error reporting and version for the C ABI.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <mutex>

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
// initial values from the environment, -1 = automatic choice.
static const char* const k_knob_names[TUNE_NKNOBS] = {"pk_cfg", "pk_elds", "dw_lds", "dw_rows", "ffn_diag", "pk_diag"};
static const char* const k_knob_env[TUNE_NKNOBS] = {"SVK_PK_CFG", "SVK_PK_ELDS", "SVK_DW_LDS", "SVK_DW_LR", "SVK_FFN_DIAG", "SVK_PK_DIAG"};
static int init_knob(int i) {
  const char* e = getenv(k_knob_env[i]);
  return e ? atoi(e) : -1;
}
int g_tune[TUNE_NKNOBS] = {init_knob(0), init_knob(1), init_knob(2), init_knob(3), init_knob(4), init_knob(5)};

// Caller-owned per-stream workspaces (svk_set_stream_workspace): the stream-K GEMM's partial sums and flags.
struct StreamWs { hipStream_t st; void* part; long bytes; int* flags; int nflags; };
static StreamWs g_ws[16];
static int g_nws = 0, g_ws_next = 0;   // full table: entries are replaced oldest first
static std::mutex g_ws_mu;

bool stream_workspace(hipStream_t st, void** part, long* bytes, int** flags, int* nflags) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  for (int i = 0; i < g_nws; ++i)
    if (g_ws[i].st == st) {
      *part = g_ws[i].part; *bytes = g_ws[i].bytes; *flags = g_ws[i].flags; *nflags = g_ws[i].nflags;
      return true;
    }
  return false;
}

}  // namespace svk

extern "C" int svk_set_stream_workspace(void* stream, void* part, long part_bytes, int* flags, int nflags) {
  if ((part && part_bytes <= 0) || (flags && nflags <= 0) || ((uintptr_t)part & 15)) {
    svk::set_error("svk_set_stream_workspace: bad args"); return SVK_EINVAL;
  }
  std::lock_guard<std::mutex> lk(svk::g_ws_mu);
  hipStream_t st = (hipStream_t)stream;
  for (int i = 0; i < svk::g_nws; ++i)
    if (svk::g_ws[i].st == st) {
      svk::g_ws[i] = svk::StreamWs{st, part, part_bytes, flags, nflags};
      return SVK_OK;
    }
  if (svk::g_nws == 16) {                 // evict the oldest registration instead of failing the 17th stream
    svk::g_ws[svk::g_ws_next] = svk::StreamWs{st, part, part_bytes, flags, nflags};
    svk::g_ws_next = (svk::g_ws_next + 1) % 16;
    return SVK_OK;
  }
  svk::g_ws[svk::g_nws++] = svk::StreamWs{st, part, part_bytes, flags, nflags};
  return SVK_OK;
}

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
