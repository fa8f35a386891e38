// Multi-head softmax attention with a short key sequence (Nk <= 256, head_dim <= 64).
//
// On this path every attention has a short KV side: the MiT efficient self-attention
// reduces keys to 49 (sequence reduction, mix_transformer_evp.py:114-121), the flow
// cross-attention has 196 / 49 flow tokens, the Transformer2_3_1 window has 30.  So one
// workgroup stages the whole K and V of one (batch, head) in LDS (f32) and streams
// queries: 4 lanes per query, each lane walking every 4th key with an online softmax
// (running max / sum), then the 4 partial states are merged with wave shuffles.
// Q is read once, O written once: the kernel is bound by the Q/O HBM traffic.
#include "svk_common.h"

namespace svk {

template <typename T, int HDMAX>
__global__ __launch_bounds__(256) void attention_kernel(const T* __restrict__ Q, long ldq, long sbq,
                                                        const T* __restrict__ K, long ldk, long sbk,
                                                        const T* __restrict__ V, long ldv, long sbv,
                                                        T* __restrict__ O, long ldo, long sbo,
                                                        int Nq, int Nk, int hd, float scale) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.z, h = blockIdx.y;
  float* sK = smem;                 // [Nk][hd]
  float* sV = smem + Nk * hd;       // [Nk][hd]
  const T* Kb = K + (long)b * sbk + (long)h * hd;
  const T* Vb = V + (long)b * sbv + (long)h * hd;
  for (int e = threadIdx.x; e < Nk * hd; e += blockDim.x) {
    int j = e / hd, d = e - j * hd;
    sK[e] = to_f(Kb[(long)j * ldk + d]);
    sV[e] = to_f(Vb[(long)j * ldv + d]);
  }
  __syncthreads();

  const int sub = threadIdx.x & 3;
  const int qi = blockIdx.x * 64 + (threadIdx.x >> 2);
  const bool active = qi < Nq;
  const T* q = Q + (long)b * sbq + (long)(active ? qi : 0) * ldq + (long)h * hd;
  float qr[HDMAX], o[HDMAX];
#pragma unroll
  for (int d = 0; d < HDMAX; ++d) {
    qr[d] = (d < hd) ? to_f(q[d]) * scale : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = sub; j < Nk; j += 4) {
    const float* kr = sK + j * hd;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HDMAX; ++d) if (d < hd) s += qr[d] * kr[d];
    const float mn = fmaxf(m, s);
    const float corr = expf(m - mn);   // 0 on the first key (m = -inf)
    const float pj = expf(s - mn);
    l = l * corr + pj;
    const float* vr = sV + j * hd;
#pragma unroll
    for (int d = 0; d < HDMAX; ++d) o[d] = o[d] * corr + (d < hd ? pj * vr[d] : 0.f);
    m = mn;
  }
  // merge the 4 lanes of this query
  float mall = fmaxf(m, __shfl_xor(m, 1, 64));
  mall = fmaxf(mall, __shfl_xor(mall, 2, 64));
  const float f = (m == -INFINITY) ? 0.f : expf(m - mall);
  l *= f;
  l += __shfl_xor(l, 1, 64);
  l += __shfl_xor(l, 2, 64);
  const float inv = 1.0f / l;
#pragma unroll
  for (int d = 0; d < HDMAX; ++d) {
    float v = o[d] * f;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    o[d] = v * inv;
  }
  if (!active) return;
  T* out = O + (long)b * sbo + (long)qi * ldo + (long)h * hd;
#pragma unroll
  for (int d = 0; d < HDMAX; ++d)
    if (d < hd && (d & 3) == sub) out[d] = from_f<T>(o[d]);
}

}  // namespace svk

using namespace svk;

extern "C" int svk_attention(int dtype, const void* Q, long ldq, long sbq, const void* K, long ldk, long sbk,
                             const void* V, long ldv, long sbv, void* O, long ldo, long sbo, int B, int Nq,
                             int Nk, int heads, int hd, float scale, void* stream) {
  if (B < 0 || Nq < 0 || Nk <= 0 || Nk > 256 || heads <= 0 || hd <= 0 || hd > 64 || !Q || !K || !V || !O) {
    set_error("svk_attention: bad args (Nk=%d hd=%d; need Nk<=256, hd<=64)", Nk, hd);
    return SVK_EINVAL;
  }
  if (B == 0 || Nq == 0) return SVK_OK;
  if (B > 65535 || heads > 65535) { set_error("svk_attention: grid too large"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((Nq + 63) / 64, heads, B), block(256);
  SVK_DISPATCH_DTYPE(dtype, T, {
    const size_t sm = (size_t)2 * Nk * hd * sizeof(float);
    if (hd <= 32) {
      if (sm > 65536) (void)hipFuncSetAttribute((const void*)attention_kernel<T, 32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
      hipLaunchKernelGGL((attention_kernel<T, 32>), grid, block, sm, st, (const T*)Q, ldq, sbq, (const T*)K, ldk, sbk,
                         (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, scale);
    } else {
      if (sm > 65536) (void)hipFuncSetAttribute((const void*)attention_kernel<T, 64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
      hipLaunchKernelGGL((attention_kernel<T, 64>), grid, block, sm, st, (const T*)Q, ldq, sbq, (const T*)K, ldk, sbk,
                         (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, scale);
    }
    return check_launch("attention");
  });
}
