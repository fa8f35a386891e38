// GEMM + bias + residual + LayerNorm over the full output row, 16-bit (round 5):
//
//   X = A W^T + bias + R          (the Block's residual stream after proj / the prompt adapter's shared MLP)
//   H = LayerNorm(X; gamma, beta) (the next norm: Block.norm2 / Block.norm1)
//
// mix_transformer_evp.py:167-171 (x = x + attn(norm1(x)); norm2) and :776-815 (get_prompt, then norm1).  At
// stages 3-4 (N = 320 / 512) the unfused form is a GEMM writing X and a LayerNorm pass reading it back and
// writing H: one launch and 2·M·N·2 bytes more.  Here a workgroup owns BM rows x ALL N columns, so the
// row statistics close inside it:
//
//  * 4 waves split N (N / 4 columns each), every wave covers the BM rows; transposed MFMA (W fragment x A
//    fragment, 16x16x32), a lane ends with 4 consecutive columns of one row;
//  * W comes from a PACKED buffer (svk_gemm_ln_pack: per 32-wide k-step, per wave and n-block, the 64 lanes'
//    16-byte fragments in load order — one contiguous 1 KiB wave-instruction each, L2-resident), A fragments
//    straight from global memory (16 bytes per lane; the four waves' repeats of a row hit L1); a K tail is
//    zero-filled on both sides, so any K % 8 == 0 works (the adapter's K = C / 4 = 80);
//  * epilogue: + bias + residual in f32, rounded to 16 bits (X, as the unfused GEMM stores it), row sums
//    over the lane's columns -> 4 lanes of a row (xor 16 / 32) -> the 4 waves through LDS; mean, then the
//    centred sum of squares the same way (two passes, as layernorm_vec), H = (x - mean) rstd gamma + beta.
#include "svk_common.h"
#include <type_traits>

namespace svk {
namespace gln {

template <int N_, int MB_>
struct Cfg {
  static constexpr int N = N_, MB = MB_, BM = 16 * MB, NT = 256;
  static constexpr int NBW = N / 64;                   // 16-column n-blocks per wave
  static constexpr int PKS = 4 * NBW * 64 * 16;        // packed bytes per 32-wide k-step
  static_assert(N % 64 == 0, "shape");
};

template <typename T, class C>
__global__ __launch_bounds__(256) void gemm_ln_pack(const T* __restrict__ W, int K, uint4* __restrict__ out) {
  const int nks = (K + 31) / 32;
  const long id = (long)blockIdx.x * 256 + threadIdx.x;
  if (id >= (long)nks * (C::PKS / 16)) return;
  const int ks = (int)(id / (C::PKS / 16)), r = (int)(id % (C::PKS / 16));
  const int lane = r % 64, nb = (r / 64) % C::NBW, w = r / (64 * C::NBW);
  const int fr = lane & 15, fq = lane >> 4, k = 32 * ks + 8 * fq;
  const T* src = W + (long)(w * (C::N / 4) + nb * 16 + fr) * K + k;
  uint4 v = {0u, 0u, 0u, 0u};
  if (k < K) v = *reinterpret_cast<const uint4*>(src);   // K % 8 == 0: a fragment is all in or all out
  out[id] = v;
}

template <typename T, class C>
__global__ __launch_bounds__(256, 2) void gemm_ln(const T* __restrict__ A, int M, int K, const char* __restrict__ pk,
                                                 const float* __restrict__ bias, const T* __restrict__ R,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 float eps, T* __restrict__ X, T* __restrict__ Hn) {
  typedef v8_t<T> tx8;
  constexpr int MB = C::MB, NBW = C::NBW, N = C::N;
  __shared__ float red[2][4][C::BM];                   // per-wave row partials: sums, then centred squares
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * C::BM, n0w = wave * (N / 4);
  const int nks = (K + 31) / 32;

  const T* arow[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) arow[mb] = A + (long)min(m0 + 16 * mb + fr, M - 1) * K + 8 * fq;
  const char* pkl = pk + (wave * NBW * 64 + lane) * 16;
  auto load = [&](int ks, tx8 (&af)[MB], tx8 (&wf)[NBW]) __attribute__((always_inline)) {
    const bool kin = 32 * ks + 8 * fq < K;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      tx8 v = *reinterpret_cast<const tx8*>(arow[mb] + (kin ? 32 * ks : 0));
      if (!kin) v = tx8{};
      af[mb] = v;
    }
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) wf[nb] = *reinterpret_cast<const tx8*>(pkl + (long)ks * C::PKS + nb * 1024);
  };
  f32x4 acc[MB][NBW];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const tx8 (&af)[MB], const tx8 (&wf)[NBW]) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = mfma16x16x32(wf[nb], af[mb], acc[mb][nb]);
  };
  // k loop, two register sets (static indices: the loop is unrolled by two), the next step's loads in flight
  tx8 a0[MB], w0[NBW], a1[MB], w1[NBW];
  load(0, a0, w0);
  int ks = 0;
  for (; ks + 2 <= nks; ks += 2) {
    load(ks + 1, a1, w1);
    mma(a0, w0);
    if (ks + 2 < nks) load(ks + 2, a0, w0);
    mma(a1, w1);
  }
  if (ks < nks) mma(a0, w0);

  // ---- epilogue: lane (fr, fq) of (mb, nb) = row m0 + 16 mb + fr, columns n0w + 16 nb + 4 fq .. + 3
  float v[MB][NBW][4];
  float s[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = min(m0 + 16 * mb + fr, M - 1);
    s[mb] = 0.f;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int n = n0w + 16 * nb + 4 * fq;
      const float4 bb = bias ? *reinterpret_cast<const float4*>(bias + n) : float4{0.f, 0.f, 0.f, 0.f};
      float t[4] = {acc[mb][nb][0] + bb.x, acc[mb][nb][1] + bb.y, acc[mb][nb][2] + bb.z, acc[mb][nb][3] + bb.w};
      if (R) {
        const uint2 r = *reinterpret_cast<const uint2*>(R + (long)m * N + n);
        const f32x2 r01 = unpack2<T>(r.x), r23 = unpack2<T>(r.y);
        t[0] += r01.x; t[1] += r01.y; t[2] += r23.x; t[3] += r23.y;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[mb][nb][e] = to_f(from_f<T>(t[e]));           // X as stored; the statistics see the rounded values
        s[mb] += v[mb][nb][e];
      }
    }
  }
  // row partials: the 4 lanes of a row (fq) -> the 4 waves (LDS)
  auto row_reduce = [&](float (&p)[MB], int which) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      p[mb] += __shfl_xor(p[mb], 16, 64);
      p[mb] += __shfl_xor(p[mb], 32, 64);
      if (fq == 0) red[which][wave][16 * mb + fr] = p[mb];
    }
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int row = 16 * mb + fr;
      p[mb] = (red[which][0][row] + red[which][1][row]) + (red[which][2][row] + red[which][3][row]);
    }
  };
  row_reduce(s, 0);
  float mean[MB], q[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    mean[mb] = s[mb] * (1.0f / N);
    q[mb] = 0.f;
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[mb][nb][e] - mean[mb];
        q[mb] += d * d;
      }
  }
  row_reduce(q, 1);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + 16 * mb + fr;
    if (m >= M) continue;
    const float rstd = 1.0f / sqrtf(q[mb] * (1.0f / N) + eps);
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int n = n0w + 16 * nb + 4 * fq;
      const float4 g = *reinterpret_cast<const float4*>(gamma + n), b = *reinterpret_cast<const float4*>(beta + n);
      const float gg[4] = {g.x, g.y, g.z, g.w}, bv[4] = {b.x, b.y, b.z, b.w};
      T xo[4], ho[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xo[e] = from_f<T>(v[mb][nb][e]);
        ho[e] = from_f<T>((v[mb][nb][e] - mean[mb]) * rstd * gg[e] + bv[e]);
      }
      if (X) *reinterpret_cast<uint2*>(X + (long)m * N + n) = *reinterpret_cast<const uint2*>(xo);
      *reinterpret_cast<uint2*>(Hn + (long)m * N + n) = *reinterpret_cast<const uint2*>(ho);
    }
  }
}

template <typename T, class C>
static int launch(const void* A, int M, int K, const void* pk, const float* bias, const void* R, const float* g,
                  const float* b, float eps, void* X, void* H, hipStream_t st) {
  hipLaunchKernelGGL((gemm_ln<T, C>), dim3((M + C::BM - 1) / C::BM), dim3(C::NT), 0, st, (const T*)A, M, K,
                     (const char*)pk, bias, (const T*)R, g, b, eps, (T*)X, (T*)H);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "gemm_ln<%s, Cfg<%d, %d>>", type_name<T>(), C::N, C::BM);
  set_last_kernel(name);
  return check_launch("gemm_ln");
}

}  // namespace gln
}  // namespace svk

using namespace svk;

extern "C" long svk_gemm_ln_packed_bytes(int dtype, int N, int K) {
  if (!(dtype == SVK_F16 || dtype == SVK_BF16) || K <= 0 || K % 8) return 0;
  if (N != 320 && N != 512) return 0;
  return (long)((K + 31) / 32) * 4 * (N / 64) * 64 * 16;
}

extern "C" int svk_gemm_ln_pack(int dtype, const void* W, int N, int K, void* packed, void* stream) {
  if (!W || !packed) { set_error("svk_gemm_ln_pack: bad args"); return SVK_EINVAL; }
  if (svk_gemm_ln_packed_bytes(dtype, N, K) == 0) {
    set_error("svk_gemm_ln_pack: (dtype=%d, N=%d, K=%d) not instantiated", dtype, N, K); return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)W) | ((uintptr_t)packed)) & 15) { set_error("svk_gemm_ln_pack: misaligned operand"); return SVK_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  const long n = svk_gemm_ln_packed_bytes(dtype, N, K) / 16;
  SVK_DISPATCH_H16(dtype, T, {
    if (N == 512)
      hipLaunchKernelGGL((gln::gemm_ln_pack<T, gln::Cfg<512, 2>>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                         (const T*)W, K, (uint4*)packed);
    else
      hipLaunchKernelGGL((gln::gemm_ln_pack<T, gln::Cfg<320, 4>>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                         (const T*)W, K, (uint4*)packed);
    return check_launch("gemm_ln_pack");
  });
}

extern "C" int svk_gemm_ln(int dtype, const void* A, int M, int K, const void* packed, const float* bias, const void* R,
                           const float* gamma, const float* beta, float eps, void* X, void* H, int N, void* stream) {
  if (M < 0 || !A || !packed || !gamma || !beta || !H) { set_error("svk_gemm_ln: bad args"); return SVK_EINVAL; }
  if (svk_gemm_ln_packed_bytes(dtype, N, K) == 0) {
    set_error("svk_gemm_ln: (dtype=%d, N=%d, K=%d) not instantiated", dtype, N, K); return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)A) | ((uintptr_t)packed) | ((uintptr_t)bias) | ((uintptr_t)gamma) | ((uintptr_t)beta)) & 15 ||
      (((uintptr_t)R) | ((uintptr_t)X) | ((uintptr_t)H)) & 7) {
    set_error("svk_gemm_ln: misaligned operand"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    if (N == 512) return gln::launch<T, gln::Cfg<512, 2>>(A, M, K, packed, bias, R, gamma, beta, eps, X, H, st);
    return gln::launch<T, gln::Cfg<320, 4>>(A, M, K, packed, bias, R, gamma, beta, eps, X, H, st);
  });
}
