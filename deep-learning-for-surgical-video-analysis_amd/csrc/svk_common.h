// svk — surgical-video kernels for MI355X (gfx950 / CDNA4).  Shared device helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/svk.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace svk {

// Thread-local last-error string (svk_last_error); set by the host wrappers only.
void set_error(const char* fmt, ...);
int check_launch(const char* what);

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case SVK_ACT_GELU: return gelu_erf(v);
    case SVK_ACT_RELU: return v > 0.f ? v : 0.f;
    case SVK_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace svk

#define SVK_DISPATCH_DTYPE(dt, T, ...)                                   \
  do {                                                                   \
    if ((dt) == SVK_F32) { typedef float T; __VA_ARGS__; }               \
    else if ((dt) == SVK_BF16) { typedef bf16 T; __VA_ARGS__; }          \
    else { svk::set_error("unsupported dtype %d", (int)(dt)); return SVK_EINVAL; } \
  } while (0)
