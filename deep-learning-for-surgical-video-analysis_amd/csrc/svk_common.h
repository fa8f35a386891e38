// svk — surgical-video kernels for MI355X (gfx950 / CDNA4).  Shared device helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>

#include "../../include/svk.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace svk {

// Thread-local last-error string (svk_last_error); set by the host wrappers only.
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// Tuning knobs set through svk_tune (runtime.hip); -1 = automatic.
enum { TUNE_PK_CFG = 0, TUNE_PK_ELDS = 1, TUNE_DW_LDS = 2, TUNE_DW_ROWS = 3, TUNE_ATTN_CFG = 4, TUNE_NKNOBS = 5 };
extern int g_tune[TUNE_NKNOBS];
#ifdef SVK_DIAG
// Timing-ablation switch of the diagnostic build only (-DSVK_DIAG: SVK_FFN_DIAG / SVK_PK_DIAG in the environment);
// the product library has no code path that skips work or stores.
int diag_knob(const char* env);
#endif
// Name of the kernel instantiation the calling thread launched last (svk_last_kernel; profiling).
void set_last_kernel(const char* name);
void set_pk_reject(const char* why);   // why the last GEMM call missed gemm_pk (fallback kernel names)
const char* pk_reject();
// norm.hip: Y = LN(sum of ks f32 split-K slabs [ks][M][C] + bias), bf16 out (svk_conv2d_ln_nhwc)
template <typename T>
int splitk_layernorm(const float* S, int ks, const float* bias, T* Y, int M, int C, const float* gamma,
                     const float* beta, float eps, hipStream_t st);
// gemm.hip: batched split-M weight-gradient reduction dW[z] += dY[z]^T X[z] (f32 atomics)
int wgrad_batched(int dtype, const void* dY, long ldy, long sa_o, long sa_i, const void* X, long ldx, long sx_o,
                  long sx_i, float* dW, long lddw, long sw_o, long sw_i, int Z, int nzi, int M, int N, int K,
                  hipStream_t st);

// mixffn_rw.hip: register-window fc1 + dwconv3x3 + GELU (f16, stage-2 shape); returns 1 when not eligible
int fc1dw_rw_try(int dtype, const void* XN, const void* W1, const float* b1, const float* taps, const float* dbias,
                 void* G, int B, int H, int W, int C, int hidden, int act, hipStream_t st);

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }

// 16-bit storage types of the MFMA path: bf16 (8 significant bits) and f16 (11 significant bits,
// the reference's torch.autocast(float16) precision, train_evp.py:493/637/760).  Both run the
// 16x16x32 MFMA at the same rate on gfx950; accumulation is f32 either way.
template <typename T> struct VT;
template <> struct VT<bf16> { typedef bf16x8 x8; typedef bf16x4 x4; };
template <> struct VT<f16> { typedef f16x8 x8; typedef f16x4 x4; };
template <typename T> using v8_t = typename VT<T>::x8;
template <typename T> using v4_t = typename VT<T>::x4;
template <typename T> constexpr const char* type_name() {
  return sizeof(T) == 4 ? "float" : (__is_same(T, bf16) ? "__bf16" : "_Float16");
}

__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// The two 16-bit elements of a 32-bit word (element 0 in the low half) as f32.
template <typename T> __device__ __forceinline__ f32x2 unpack2(uint32_t u);
template <> __device__ __forceinline__ f32x2 unpack2<bf16>(uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}
template <> __device__ __forceinline__ f32x2 unpack2<f16>(uint32_t u) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2, u), f32x2);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// ---- packed-f32 VALU (v_pk_fma / v_pk_mul / v_pk_add_f32: two f32 lanes per instruction, the rate of one
// v_fma_f32).  hipcc is built with -packed-fp32-ops (Makefile: on gfx950 a v_pk_*_f32 whose low lane reads,
// THROUGH op_sel, a VGPR the preceding VALU wrote is stale in lanes 48-63 under MFMA load), so packed f32
// arithmetic is written by hand here: natural register pairs and the default op_sel only — the form
// tools/hazard/pk_hazard.hip (variant 7: the same dependency without op_sel, MFMA load on the SIMD) measured
// exact over 10.5 M lane results (profiles/r03/pk_hazard/pk_hazard.log).  csrc/isa_check.py admits v_pk_*_f32
// only without op_sel / op_sel_hi.  A 64-bit SGPR pair is a legal packed source (one scalar operand per
// instruction): constants are passed that way.
// The hazard recognizer does not see inside inline asm: a VALU read of a TRANSCENDENTAL result (v_rcp / v_exp
// ...) needs one wait state on gfx950 (the compiler adds it for its own instructions, not for an asm consumer —
// the first build of gelu_pk read stale rcp / exp results and failed every GELU test, r06c), so the helpers that
// consume rcp / exp2 outputs (pk_fma_tr, pk_rsub) open with s_nop 0.
constexpr unsigned long long kpair(float f) { return (unsigned long long)__builtin_bit_cast(unsigned, f) * 0x100000001ull; }
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, unsigned long long c) {   // c: SGPR pair
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, unsigned long long b, f32x2 c) {   // b: SGPR pair
  f32x2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul(f32x2 a, f32x2 b) {
  f32x2 d;
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ f32x2 pk_mul(f32x2 a, unsigned long long b) {
  f32x2 d;
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "s"(b));
  return d;
}
__device__ __forceinline__ f32x2 pk_rsub(unsigned long long a, f32x2 b) {   // a - b, a: SGPR pair; b may be a trans result
  f32x2 d;
  asm("s_nop 0\n\tv_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "s"(a), "v"(b));
  return d;
}
// fma whose first / second operand may be a transcendental result: one wait state first (see above)
__device__ __forceinline__ f32x2 pk_fma_tr(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  asm("s_nop 0\n\tv_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ f32x2 pk_fma_tr(f32x2 a, unsigned long long b, f32x2 c) {
  f32x2 d;
  asm("s_nop 0\n\tv_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
  return d;
}

// GELU on a pair, erf form: relu(x) - |x| * 0.5 erfc(|x| / sqrt 2) with erfc(z) = t q(t) exp(-z^2),
// t = 1 / (1 + c z).  |x| t = (1 - t) / c' (c' = c / sqrt 2), so the correction is (1 - t) (q(t) / c')
// exp(-x^2 / 2): the rcp / exp2 / relu / x^2 per element, everything else packed — per pair 6 VALU + 6 (NQ = 3)
// or 8 (NQ = 5) packed + 4 transcendental + 3 s_nop, against 2 x (9 or 11) VALU + 4 transcendental element-wise.
//   NQ = 3: Abramowitz & Stegun 7.1.25 (|erf err| <= 2.5e-5: mixffn_rw's gelu_rw);
//   NQ = 5: 7.1.26 (|err| <= 1.5e-7: stencil / dw_fc2's gelu_rl).
// (1 - t) loses relative precision as |x| -> 0, where the correction itself -> 0.5 |x|: its absolute error
// stays within an f32 ulp of 1 times 0.5 |x| / (c' |x|) ~ 1.3e-7 — far below the 16-bit output rounding.
// host switch: SVK_GELU_PK=0 selects the element-wise GELU kernels (A/B runs)
inline bool gelu_pk_on() {
  static const bool on = getenv("SVK_GELU_PK") ? atoi(getenv("SVK_GELU_PK")) != 0 : true;
  return on;
}
template <int NQ>
__device__ __forceinline__ f32x2 gelu_pk(f32x2 x) {
  constexpr float c = NQ == 3 ? 0.47047f * 0.70710678118654752f : 0.3275911f * 0.70710678118654752f;
  // q(t) / c, coefficients of -0.5 (a_1 + a_2 t + ...) (the 0.5 of Phi and the sign of the correction)
  constexpr float s = -0.5f / c;
  constexpr float a1 = NQ == 3 ? 0.3480242f : 0.254829592f, a2 = NQ == 3 ? -0.0958798f : -0.284496736f;
  constexpr float a3 = NQ == 3 ? 0.7478556f : 1.421413741f, a4 = -1.453152027f, a5 = 1.061405429f;
  f32x2 u, t, e;
  u.x = fmaf(c, fabsf(x.x), 1.0f);
  u.y = fmaf(c, fabsf(x.y), 1.0f);
  t.x = __builtin_amdgcn_rcpf(u.x);
  t.y = __builtin_amdgcn_rcpf(u.y);
  f32x2 q;
  if constexpr (NQ == 3) {
    q = pk_fma_tr(t, kpair(s * a3), f32x2{s * a2, s * a2});
  } else {
    q = pk_fma_tr(t, kpair(s * a5), f32x2{s * a4, s * a4});
    q = pk_fma(q, t, kpair(s * a3));
    q = pk_fma(q, t, kpair(s * a2));
  }
  q = pk_fma(q, t, kpair(s * a1));
  const f32x2 a = pk_mul(pk_rsub(kpair(1.0f), t), q);
  // x itself is read only by compiler-generated instructions (x may be an MFMA result, whose read-after-write wait
  // the hazard recognizer inserts for its own instructions only)
  const f32x2 w = pk_mul(f32x2{x.x * x.x, x.y * x.y}, kpair(-0.72134752044448170f));     // -x^2 / 2 * log2(e)
  e.x = __builtin_amdgcn_exp2f(w.x);
  e.y = __builtin_amdgcn_exp2f(w.y);
  return pk_fma_tr(a, e, f32x2{fmaxf(x.x, 0.f), fmaxf(x.y, 0.f)});
}

// Branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 absolute): one rcp, one exp, five
// FMAs — no range-split branches, so a wave never diverges.  Used by the bf16 kernels, whose outputs
// are rounded to 8 significant bits anyway; the f32 parity path keeps erff.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-ax * ax);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case SVK_ACT_GELU: return gelu_erf(v);
    case SVK_ACT_RELU: return v > 0.f ? v : 0.f;
    case SVK_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// bf16 kernels: the output is rounded to 8 significant bits, so the GELU uses the branch-free erf.
__device__ __forceinline__ float apply_act_fast(float v, int act) {
  switch (act) {
    case SVK_ACT_GELU: return gelu_fast(v);
    case SVK_ACT_RELU: return v > 0.f ? v : 0.f;
    case SVK_ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// d act(u) / du (activation backward): GELU (erf form), ReLU, tanh.  The GELU derivative uses the
// branch-free erf (|err| <= 1.5e-7, below bf16 resolution and f32-parity tolerance).
__device__ __forceinline__ float act_grad(float u, int act) {
  switch (act) {
    case SVK_ACT_GELU: {
      const float e = __expf(-0.5f * u * u);
      const float x = u * 0.70710678118654752f, ax = fabsf(x);
      const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
      float p = fmaf(1.061405429f, t, -1.453152027f);
      p = fmaf(p, t, 1.421413741f);
      p = fmaf(p, t, -0.284496736f);
      p = fmaf(p, t, 0.254829592f);
      const float erf_ = copysignf(1.0f - p * t * e, x);      // exp(-x^2) == exp(-u^2 / 2) = e
      return 0.5f * (1.0f + erf_) + u * 0.3989422804014327f * e;
    }
    case SVK_ACT_RELU: return u > 0.f ? 1.f : 0.f;
    case SVK_ACT_TANH: { const float t = tanhf(u); return 1.f - t * t; }
    default: return 1.f;
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
    else if ((dt) == SVK_F16) { typedef f16 T; __VA_ARGS__; }            \
    else { svk::set_error("unsupported dtype %d", (int)(dt)); return SVK_EINVAL; } \
  } while (0)

// 16-bit MFMA-only paths (bf16 / f16)
#define SVK_DISPATCH_H16(dt, T, ...)                                     \
  do {                                                                   \
    if ((dt) == SVK_BF16) { typedef bf16 T; __VA_ARGS__; }               \
    else if ((dt) == SVK_F16) { typedef f16 T; __VA_ARGS__; }            \
    else { svk::set_error("dtype %d: bf16 / f16 only", (int)(dt)); return SVK_EUNSUPPORTED; } \
  } while (0)
