// Phase-anticipation regression targets (generate_phase_anticipation.py:10-34): for each phase p, walking
// the video backwards, count = 0 where the phase is present, else min(horizon, count + 1/1500) (minutes at
// 25 fps annotation rate), starting from count = horizon; target = float(count) / horizon.  The count is a
// double (Python float) exactly as the reference accumulates it; the stored value is rounded to f32 and
// divided in f32 like torch's FloatTensor / horizon.  The recurrence is sequential in time, so one thread
// owns one (video, phase) series; output is the reference's [T, P] (after its permute(1, 0)).
#include "svk_common.h"

namespace svk {

__global__ __launch_bounds__(64) void anticipation_gt_kernel(const long long* __restrict__ phases, long ldp, int P,
                                                             int T, double horizon, float* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const long long* code = phases + (long)p * ldp;
  const float hf = (float)horizon;
  double count = horizon;
  for (int i = T - 1; i >= 0; --i) {
    if (code[i] != 0) count = 0.0;
    else count = fmin(horizon, count + 1.0 / 1500.0);
    out[(long)i * P + p] = __fdiv_rn((float)count, hf);
  }
}

}  // namespace svk

using namespace svk;

extern "C" int svk_anticipation_gt(const long long* phases, long ldp, int P, int T, double horizon, float* out,
                                   void* stream) {
  if (P <= 0 || T < 0 || ldp < T || !phases || !out || !(horizon > 0.0)) {
    set_error("svk_anticipation_gt: bad args (P=%d T=%d ldp=%ld horizon=%g)", P, T, ldp, horizon);
    return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  hipLaunchKernelGGL(anticipation_gt_kernel, dim3((P + 63) / 64), dim3(64), 0, (hipStream_t)stream, phases, ldp, P, T,
                     horizon, out);
  return check_launch("anticipation_gt");
}
