// Row-wise normalisation / reduction kernels: LayerNorm, softmax over channels, row-mean pool.
#include "svk_common.h"
#include <type_traits>

namespace svk {

// One wave per row; PER = ceil(C / 64) values per lane kept in registers (two-pass mean/var,
// biased variance, f32 statistics — nn.LayerNorm semantics).  PER == 0: generic loop.
template <typename T, int PER>
__global__ __launch_bounds__(256) void layernorm_kernel(const T* __restrict__ X, long ldx, T* __restrict__ Y, long ldy,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        int M, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* x = X + row * ldx;
  T* y = Y + row * ldy;
  if constexpr (PER > 0) {
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + 64 * i;
      v[i] = c < C ? to_f(x[c]) : 0.f;
      s += v[i];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + 64 * i;
      float d = c < C ? v[i] - mean : 0.f;
      q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + 64 * i;
      if (c < C) y[c] = from_f<T>((v[i] - mean) * rstd * g[c] + b[c]);
    }
  } else {
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += to_f(x[c]);
    const float mean = wave_sum(s) / C;
    float q = 0.f;
    for (int c = lane; c < C; c += 64) { float d = to_f(x[c]) - mean; q += d * d; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    for (int c = lane; c < C; c += 64) y[c] = from_f<T>((to_f(x[c]) - mean) * rstd * g[c] + b[c]);
  }
}

// Vectorised LayerNorm: each lane owns NCH 8-channel chunks (16-byte bf16 / 32-byte f32 loads),
// LPR lanes cooperate on one row (LPR = power of two >= C/8), 64/LPR rows per wave; the row
// reductions are xor-shuffles inside the LPR-lane group.  Used when C % 8 == 0 and rows are
// 16-byte aligned (every LayerNorm of the MiT path: C = 16..512).
template <typename T, int LPR, int NCH>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const T* __restrict__ X, long ldx, T* __restrict__ Y,
                                                            long ldy, const float* __restrict__ g,
                                                            const float* __restrict__ b, int M, int C, float eps) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool valid = row < M;
  const int nchunks = C >> 3;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
    if (valid && ch < nchunks) {
      const T* src = X + row * ldx + ch * 8;
      T t[8];
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(t) = *reinterpret_cast<const uint4*>(src);
      } else {
        reinterpret_cast<uint4*>(t)[0] = reinterpret_cast<const uint4*>(src)[0];
        reinterpret_cast<uint4*>(t)[1] = reinterpret_cast<const uint4*>(src)[1];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[i][e] = to_f(t[e]); s += v[i][e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
    if (ch < nchunks) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = 1.0f / sqrtf(q / C + eps);
  if (!valid) return;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
    if (ch >= nchunks) continue;
    T t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = ch * 8 + e;
      t[e] = from_f<T>((v[i][e] - mean) * rstd * g[c] + b[c]);
    }
    T* dst = Y + row * ldy + ch * 8;
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(t);
    } else {
      reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(t)[0];
      reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(t)[1];
    }
  }
}

template <typename T, int LPR, int NCH>
static void launch_ln_vec(const T* x, long ldx, T* y, long ldy, const float* g, const float* b, int M, int C,
                          float eps, hipStream_t st) {
  constexpr int RPB = 4 * (64 / LPR);   // rows per 256-thread block
  hipLaunchKernelGGL((layernorm_vec_kernel<T, LPR, NCH>), dim3((M + RPB - 1) / RPB), dim3(256), 0, st, x, ldx, y, ldy,
                     g, b, M, C, eps);
}

// Softmax over C (small) channels per row, one thread per row (MS-TCN's 14-class softmax).
__global__ void softmax_rows_kernel(const float* __restrict__ X, long ldx, float* __restrict__ Y, long ldy, int M, int C) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  const float* x = X + r * ldx;
  float* y = Y + r * ldy;
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, x[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += expf(x[c] - m);
  const float inv = 1.0f / s;
  for (int c = 0; c < C; ++c) y[c] = expf(x[c] - m) * inv;
}

// Y[b, c] = mean over R rows; one thread per (b, c), rows strided by ldx (coalesced over c).
template <typename T>
__global__ void mean_rows_kernel(const T* __restrict__ X, long ldx, float* __restrict__ Y, int B, int R, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (c >= C) return;
  const T* x = X + (long)b * R * ldx + c;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += to_f(x[(long)r * ldx]);
  Y[(long)b * C + c] = s / R;
}

// Split-K reduction + bias + LayerNorm (svk_conv2d_ln_nhwc): Y[m, :] = LN(sum_s S[s][m][:] + bias),
// 16-bit out.  Same lane layout as layernorm_vec_kernel: LPR lanes per row, NCH 8-channel chunks per
// lane, f32 sums, two-pass mean / variance over the row held in registers.
template <typename T, int LPR, int NCH>
__global__ __launch_bounds__(256) void splitk_ln_kernel(const float* __restrict__ S, int ks, const float* __restrict__ bias,
                                                        T* __restrict__ Y, const float* __restrict__ g,
                                                        const float* __restrict__ b, int M, int C, float eps) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool valid = row < M;
  const int nchunks = C >> 3;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    if (valid && ch < nchunks) {
      const float4 b0 = *reinterpret_cast<const float4*>(bias + ch * 8), b1 = *reinterpret_cast<const float4*>(bias + ch * 8 + 4);
      v[i][0] = b0.x; v[i][1] = b0.y; v[i][2] = b0.z; v[i][3] = b0.w;
      v[i][4] = b1.x; v[i][5] = b1.y; v[i][6] = b1.z; v[i][7] = b1.w;
      for (int k = 0; k < ks; ++k) {
        const float* src = S + ((long)k * M + row) * C + ch * 8;
        const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
        v[i][0] += x0.x; v[i][1] += x0.y; v[i][2] += x0.z; v[i][3] += x0.w;
        v[i][4] += x1.x; v[i][5] += x1.y; v[i][6] += x1.z; v[i][7] += x1.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
    if (ch < nchunks) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = 1.0f / sqrtf(q / C + eps);
  if (!valid) return;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = sub + LPR * i;
    if (ch >= nchunks) continue;
    T t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (T)((v[i][e] - mean) * rstd * g[ch * 8 + e] + b[ch * 8 + e]);
    *reinterpret_cast<uint4*>(Y + row * C + ch * 8) = *reinterpret_cast<const uint4*>(t);
  }
}

template <typename T>
int splitk_layernorm(const float* S, int ks, const float* bias, T* Y, int M, int C, const float* gamma,
                     const float* beta, float eps, hipStream_t st) {
  if (C % 8 || C > 4096) { set_error("splitk_layernorm: C %% 8 != 0 or C > 4096"); return SVK_EUNSUPPORTED; }
  const int nch = C / 8;
  auto go = [&](auto lpr_c, auto nch_c) {
    constexpr int LPR = decltype(lpr_c)::value, NCH = decltype(nch_c)::value;
    constexpr int RPB = 4 * (64 / LPR);
    hipLaunchKernelGGL((splitk_ln_kernel<T, LPR, NCH>), dim3((M + RPB - 1) / RPB), dim3(256), 0, st, S, ks, bias, Y, gamma,
                       beta, M, C, eps);
  };
  using I1 = std::integral_constant<int, 1>;
  if (nch <= 8) go(std::integral_constant<int, 8>{}, I1{});
  else if (nch <= 16) go(std::integral_constant<int, 16>{}, I1{});
  else if (nch <= 32) go(std::integral_constant<int, 32>{}, I1{});
  else if (nch <= 64) go(std::integral_constant<int, 64>{}, I1{});
  else if (nch <= 128) go(std::integral_constant<int, 64>{}, std::integral_constant<int, 2>{});
  else if (nch <= 256) go(std::integral_constant<int, 64>{}, std::integral_constant<int, 4>{});
  else go(std::integral_constant<int, 64>{}, std::integral_constant<int, 8>{});
  return check_launch("splitk_ln");
}
template int splitk_layernorm<bf16>(const float*, int, const float*, bf16*, int, int, const float*, const float*, float,
                                    hipStream_t);
template int splitk_layernorm<f16>(const float*, int, const float*, f16*, int, int, const float*, const float*, float,
                                   hipStream_t);

}  // namespace svk

using namespace svk;

extern "C" int svk_layernorm(int dtype, const void* X, long ldx, void* Y, long ldy, const float* gamma,
                             const float* beta, int M, int C, float eps, void* stream) {
  if (M < 0 || C <= 0 || !X || !Y || !gamma || !beta || ldx < C || ldy < C) { set_error("svk_layernorm: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((M + 3) / 4), block(256);
  SVK_DISPATCH_DTYPE(dtype, T, {
    const T* x = (const T*)X; T* y = (T*)Y;
    const long vw = 16 / (long)sizeof(T);
    const bool vec = C % 8 == 0 && C <= 4096 && ldx % vw == 0 && ldy % vw == 0 && ((((uintptr_t)X) | ((uintptr_t)Y)) & 15) == 0;
    if (vec) {
      const int nch = C / 8;
      if (nch <= 1) launch_ln_vec<T, 1, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 2) launch_ln_vec<T, 2, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 4) launch_ln_vec<T, 4, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 8) launch_ln_vec<T, 8, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 16) launch_ln_vec<T, 16, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 32) launch_ln_vec<T, 32, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 64) launch_ln_vec<T, 64, 1>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 128) launch_ln_vec<T, 64, 2>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else if (nch <= 256) launch_ln_vec<T, 64, 4>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      else launch_ln_vec<T, 64, 8>(x, ldx, y, ldy, gamma, beta, M, C, eps, st);
      return check_launch("layernorm");
    }
    if (C <= 64) hipLaunchKernelGGL((layernorm_kernel<T, 1>), grid, block, 0, st, x, ldx, y, ldy, gamma, beta, M, C, eps);
    else if (C <= 128) hipLaunchKernelGGL((layernorm_kernel<T, 2>), grid, block, 0, st, x, ldx, y, ldy, gamma, beta, M, C, eps);
    else if (C <= 256) hipLaunchKernelGGL((layernorm_kernel<T, 4>), grid, block, 0, st, x, ldx, y, ldy, gamma, beta, M, C, eps);
    else if (C <= 512) hipLaunchKernelGGL((layernorm_kernel<T, 8>), grid, block, 0, st, x, ldx, y, ldy, gamma, beta, M, C, eps);
    else hipLaunchKernelGGL((layernorm_kernel<T, 0>), grid, block, 0, st, x, ldx, y, ldy, gamma, beta, M, C, eps);
    return check_launch("layernorm");
  });
}

extern "C" int svk_softmax_rows(const float* X, long ldx, float* Y, long ldy, int M, int C, void* stream) {
  if (M < 0 || C <= 0 || !X || !Y || ldx < C || ldy < C) { set_error("svk_softmax_rows: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((M + 255) / 256), dim3(256), 0, (hipStream_t)stream, X, ldx, Y, ldy, M, C);
  return check_launch("softmax_rows");
}

extern "C" int svk_mean_rows(int dtype, const void* X, long ldx, float* Y, int B, int R, int C, void* stream) {
  if (B < 0 || R <= 0 || C <= 0 || !X || !Y || ldx < C) { set_error("svk_mean_rows: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((mean_rows_kernel<T>), dim3((C + 255) / 256, B), dim3(256), 0, st, (const T*)X, ldx, Y, B, R, C);
    return check_launch("mean_rows");
  });
}
