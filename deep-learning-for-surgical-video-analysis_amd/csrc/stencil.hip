// Memory-bound stencil / layout kernels over NHWC maps: depthwise 3x3 (+bias+GELU),
// input packing NCHW->NHWC, Gaussian 5x5 reflect filter, bilinear resize, window unfold, cast.
#include "svk_common.h"

namespace svk {

// ---- DWConv 3x3, pad 1, + bias + act (MixFFN, mix_transformer_evp.py:22-30, 62-63) ----------
// One thread per (pixel, 8-channel group): 16-byte (bf16) / 32-byte (f32) vector loads along C.
template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3_vec8(const T* __restrict__ X, const float* __restrict__ w,
                                                      const float* __restrict__ bias, T* __restrict__ Y,
                                                      T* __restrict__ Ypre, int B, int H, int W, int C, int act) {
  const int CG = C >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * H * W * CG;
  if (idx >= total) return;
  const int cg = (int)(idx % CG);
  const long pix = idx / CG;
  const int x = (int)(pix % W);
  const long t = pix / W;
  const int y = (int)(t % H);
  const int b = (int)(t / H);
  const int c0 = cg * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = bias[c0 + j];
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = y + dy;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = x + dx;
      if (xx < 0 || xx >= W) continue;
      const T* src = X + (((long)b * H + yy) * W + xx) * C + c0;
      T v[8];
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(v) = *reinterpret_cast<const uint4*>(src);
      } else {
        reinterpret_cast<uint4*>(v)[0] = reinterpret_cast<const uint4*>(src)[0];
        reinterpret_cast<uint4*>(v)[1] = reinterpret_cast<const uint4*>(src)[1];
      }
      const float* wt = w + ((dy + 1) * 3 + (dx + 1)) * C + c0;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += to_f(v[j]) * wt[j];
    }
  }
  T o[8];
  if (Ypre) {   // pre-activation copy (training: the GELU backward needs it)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = from_f<T>(acc[j]);
    T* dp = Ypre + pix * C + c0;
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<uint4*>(dp) = *reinterpret_cast<const uint4*>(o);
    } else {
      reinterpret_cast<uint4*>(dp)[0] = reinterpret_cast<const uint4*>(o)[0];
      reinterpret_cast<uint4*>(dp)[1] = reinterpret_cast<const uint4*>(o)[1];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = from_f<T>(apply_act(acc[j], act));
  T* dst = Y + pix * C + c0;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(o);
  } else {
    reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(o)[0];
    reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(o)[1];
  }
}

template <typename T>
__global__ void dwconv3x3_scalar(const T* __restrict__ X, const float* __restrict__ w, const float* __restrict__ bias,
                                 T* __restrict__ Y, T* __restrict__ Ypre, int B, int H, int W, int C, int act) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * H * W * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int x = (int)(pix % W);
  const long t = pix / W;
  const int y = (int)(t % H);
  const int b = (int)(t / H);
  float acc = bias[c];
  for (int dy = -1; dy <= 1; ++dy)
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = y + dy, xx = x + dx;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      acc += to_f(X[(((long)b * H + yy) * W + xx) * C + c]) * w[((dy + 1) * 3 + (dx + 1)) * C + c];
    }
  if (Ypre) Ypre[idx] = from_f<T>(acc);
  Y[idx] = from_f<T>(apply_act(acc, act));
}

// ---- NCHW f32 -> NHWC T --------------------------------------------------------------------
// One thread per pixel, all C channels: reads coalesced along W within each channel plane.
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ X, T* __restrict__ Y, int B, int C, int H, int W,
                                    int Cpad) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long hw = (long)H * W;
  if (pix >= (long)B * hw) return;
  const long b = pix / hw, p = pix - b * hw;
  const float* src = X + b * C * hw + p;
  T* dst = Y + pix * Cpad;
  for (int c = 0; c < Cpad; ++c) dst[c] = from_f<T>(c < C ? src[(long)c * hw] : 0.f);
}

// ---- GaussianFilter.conv_gauss: reflect pad 2 + binomial 5x5 / 256 (mix_transformer_evp.py:501-514)
__device__ __forceinline__ int reflect(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

// One thread per output pixel, looping over channels: the 25 taps of neighbouring threads are
// neighbouring addresses of one NCHW plane (coalesced), output written NHWC.
template <typename T>
__global__ void gauss5x5_kernel(const float* __restrict__ X, T* __restrict__ Y, int B, int C, int H, int W, int Cpad) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (long)B * H * W) return;
  const int x = (int)(pix % W);
  const long t = pix / W;
  const int y = (int)(t % H);
  const int b = (int)(t / H);
  const float k1[5] = {1.f, 4.f, 6.f, 4.f, 1.f};
  int yy[5], xx[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) { yy[i] = reflect(y + i - 2, H); xx[i] = reflect(x + i - 2, W); }
  for (int c = 0; c < C; ++c) {
    const float* src = X + ((long)b * C + c) * H * W;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) acc += src[(long)yy[i] * W + xx[j]] * (k1[i] * k1[j] * (1.0f / 256.f));
    Y[pix * Cpad + c] = from_f<T>(acc);
  }
  for (int c = C; c < Cpad; ++c) Y[pix * Cpad + c] = from_f<T>(0.f);
}

// ---- bilinear resize, align_corners=False, no antialias (F.interpolate semantics) ----------
__device__ __forceinline__ void src_index(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * (dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - i0;
  l0 = 1.f - l1;
}

template <typename T>
__global__ void resize_bilinear_kernel(const T* __restrict__ X, long ldx, T* __restrict__ Y, long ldy,
                                       int B, int H, int W, int C, int OH, int OW) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * OH * OW * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int ox = (int)(pix % OW);
  const long t = pix / OW;
  const int oy = (int)(t % OH);
  const int b = (int)(t / OH);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  src_index(oy, H, OH, y0, y1, ly0, ly1);
  src_index(ox, W, OW, x0, x1, lx0, lx1);
  const T* base = X + (long)b * H * W * ldx + c;
  auto at = [&](int yy, int xx) { return to_f(base[((long)yy * W + xx) * ldx]); };
  const float v = ly0 * (lx0 * at(y0, x0) + lx1 * at(y0, x1)) + ly1 * (lx0 * at(y1, x0) + lx1 * at(y1, x1));
  Y[((long)b * OH * OW + (long)oy * OW + ox) * ldy + c] = from_f<T>(v);
}

// ---- causal window unfold (adapter_transformer.py:336-343) ---------------------------------
template <typename T>
__global__ void window_unfold_kernel(const T* __restrict__ X, long ldx, const float* __restrict__ pos, T* __restrict__ Y,
                                     int Tn, int C, int len) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Tn * len * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long r = idx / C;
  const int i = (int)(r % len);
  const long t = r / len;
  const long src = t - len + 1 + i;
  float v = src >= 0 ? to_f(X[src * ldx + c]) : 0.f;
  if (pos) v += pos[i * C + c];
  Y[idx] = from_f<T>(v);
}

// Y[r, c] = X[r, c] + P[r % period, c]  (positional-table add, Transformer2_3_1 encoder input)
template <typename T>
__global__ void add_bcast_kernel(const T* __restrict__ X, const float* __restrict__ P, T* __restrict__ Y, long M, int C,
                                 int period) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * C) return;
  const long r = idx / C;
  const int c = (int)(idx - r * C);
  Y[idx] = from_f<T>(to_f(X[idx]) + P[(r % period) * C + c]);
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ X, TO* __restrict__ Y, long n) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) Y[idx] = from_f<TO>(to_f(X[idx]));
}

inline dim3 grid1d(long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

}  // namespace svk

using namespace svk;

extern "C" int svk_dwconv3x3_ex(int dtype, const void* X, const float* w, const float* bias, void* Y, void* Ypre,
                                int B, int H, int W, int C, int act, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || !X || !w || !bias || !Y) { set_error("svk_dwconv3x3: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    const bool vec = (C % 8 == 0) && (((uintptr_t)X | (uintptr_t)Y | (uintptr_t)Ypre) & 15) == 0;
    if (vec) {
      const long n = (long)B * H * W * (C / 8);
      hipLaunchKernelGGL((dwconv3x3_vec8<T>), grid1d(n), dim3(256), 0, st, (const T*)X, w, bias, (T*)Y, (T*)Ypre, B, H,
                         W, C, act);
    } else {
      const long n = (long)B * H * W * C;
      hipLaunchKernelGGL((dwconv3x3_scalar<T>), grid1d(n), dim3(256), 0, st, (const T*)X, w, bias, (T*)Y, (T*)Ypre, B,
                         H, W, C, act);
    }
    return check_launch("dwconv3x3");
  });
}

extern "C" int svk_dwconv3x3(int dtype, const void* X, const float* w, const float* bias, void* Y, int B, int H,
                             int W, int C, int act, void* stream) {
  return svk_dwconv3x3_ex(dtype, X, w, bias, Y, nullptr, B, H, W, C, act, stream);
}

extern "C" int svk_nchw_to_nhwc(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                                void* stream) {
  if (B < 0 || C <= 0 || Cpad < C || H <= 0 || W <= 0 || !X || !Y) { set_error("svk_nchw_to_nhwc: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * H * W;   // one thread per pixel
  SVK_DISPATCH_DTYPE(dtype_out, T, {
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, B, C, H, W, Cpad);
    return check_launch("nchw_to_nhwc");
  });
}

extern "C" int svk_gauss5x5_reflect(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                                    void* stream) {
  if (B < 0 || C <= 0 || Cpad < C || H < 3 || W < 3 || !X || !Y) { set_error("svk_gauss5x5_reflect: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * H * W;   // one thread per pixel
  SVK_DISPATCH_DTYPE(dtype_out, T, {
    hipLaunchKernelGGL((gauss5x5_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, B, C, H, W, Cpad);
    return check_launch("gauss5x5_reflect");
  });
}

extern "C" int svk_resize_bilinear(int dtype, const void* X, long ldx, void* Y, long ldy, int B, int H, int W, int C,
                                   int OH, int OW, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0 || !X || !Y || ldx < C || ldy < C) {
    set_error("svk_resize_bilinear: bad args"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  const long n = (long)B * OH * OW * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((resize_bilinear_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, ldx, (T*)Y,
                       ldy, B, H, W, C, OH, OW);
    return check_launch("resize_bilinear");
  });
}

extern "C" int svk_window_unfold(int dtype, const void* X, long ldx, const float* pos, void* Y, int Tn, int C, int len,
                                 void* stream) {
  if (Tn < 0 || C <= 0 || len <= 0 || !X || !Y || ldx < C) { set_error("svk_window_unfold: bad args"); return SVK_EINVAL; }
  if (Tn == 0) return SVK_OK;
  const long n = (long)Tn * len * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((window_unfold_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, ldx, pos,
                       (T*)Y, Tn, C, len);
    return check_launch("window_unfold");
  });
}

extern "C" int svk_add_bcast(int dtype, const void* X, const float* P, void* Y, long M, int C, int period,
                             void* stream) {
  if (M < 0 || C <= 0 || period <= 0 || !X || !P || !Y) { set_error("svk_add_bcast: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((add_bcast_kernel<T>), grid1d(M * C), dim3(256), 0, (hipStream_t)stream, (const T*)X, P, (T*)Y,
                       M, C, period);
    return check_launch("add_bcast");
  });
}

extern "C" int svk_cast(int dtype_in, const void* X, int dtype_out, void* Y, long n, void* stream) {
  if (n < 0 || !X || !Y) { set_error("svk_cast: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype_in, TI, {
    SVK_DISPATCH_DTYPE(dtype_out, TO, {
      hipLaunchKernelGGL((cast_kernel<TI, TO>), grid1d(n), dim3(256), 0, st, (const TI*)X, (TO*)Y, n);
      return check_launch("cast");
    });
  });
}
