// Skinny GEMM kernels for the EVP prompt path (PromptGenerator, mix_transformer_evp.py:749-815),
// whose Linears are 16..128 wide over 69k..276k tokens (B = 88..256): the general 64x64/128x64 tiles
// leave most of every tile masked and are latency-bound.
//
// skinny_gemm: C[M, N] = act(A[M, K] W[N, K]^T + bias) * act'(U) + R, N <= 64, K <= 128, bf16 / f16.
//   W lives in LDS for the whole workgroup; each wave streams 16-row blocks of A straight from
//   global memory in the MFMA A-operand layout (lane: row l & 15, 8 consecutive k), so there is no
//   LDS staging of A at all; the 16 x N tile is written back through a per-wave LDS patch as 16-byte
//   row chunks with the epilogue fused.
// skinny_wgrad: dW[N, K] += dY[M, N]^T X[M, K], db[N] += colsum(dY), N, K <= 128, NT * KT <= 16.
//   128-row slabs of dY and X are staged transposed in LDS; wave w reduces rows 32w..32w+31 of each
//   slab into its own full N x K accumulator set, the four waves are summed in LDS and each
//   workgroup adds its partial with one f32 atomic per output element.
#include "svk_common.h"
#include <stdlib.h>

namespace svk {

template <typename T>
struct SkinnyArgs {
  const T* A; long lda;
  const T* W; long ldw;
  const float* bias;
  const T* U; long ldu; int uact;
  const T* R; long ldr;
  T* C; long ldc;
  int M, N, K, act;
};

template <typename T, int NT, int KS>
__global__ __launch_bounds__(256) void skinny_gemm(SkinnyArgs<T> p) {
  typedef v8_t<T> tx8;
  constexpr int NP = NT * 16, KP = KS * 32;
  constexpr int LDW = KP + 8;
  constexpr int LDO = NP + 4;
  __shared__ __attribute__((aligned(16))) T sW[NP][LDW];
  __shared__ __attribute__((aligned(16))) float sO[4][16][LDO];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const T z = (T)0.f;
  for (int i = tid; i < NP * (KP / 8); i += 256) {
    const int n = i / (KP / 8), k8 = (i % (KP / 8)) * 8;
    tx8 v;
    if (n < p.N && k8 < p.K) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = k8 + e < p.K ? p.W[(long)n * p.ldw + k8 + e] : z;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = z;
    }
    *reinterpret_cast<tx8*>(&sW[n][k8]) = v;
  }
  __syncthreads();
  const bool kvec = (p.K % 8) == 0;
  const long nblk = (p.M + 15) / 16;
  for (long blk = (long)blockIdx.x * 4 + w; blk < nblk; blk += (long)gridDim.x * 4) {
    const long m0 = blk * 16;
    const long row = m0 + fr;
    const long rc = row < p.M ? row : p.M - 1;
    tx8 a[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 32 + fg * 8;
      const int kc = k < p.K ? k : 0;
      if (kvec) {
        a[ks] = *reinterpret_cast<const tx8*>(p.A + rc * p.lda + kc);
        if (k >= p.K) {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[ks][e] = z;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[ks][e] = (k + e < p.K) ? p.A[rc * p.lda + k + e] : z;
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const tx8 b = *reinterpret_cast<const tx8*>(&sW[nt * 16 + fr][ks * 32 + fg * 8]);
        acc[nt] = mfma16x16x32(a[ks], b, acc[nt]);
      }
    }
    // C layout: col n = nt * 16 + (lane & 15), row = 4 (lane >> 4) + r  ->  per-wave LDS patch
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nt * 16 + fr;
      const float bn = (p.bias && n < p.N) ? p.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) sO[w][fg * 4 + r][n] = apply_act(acc[nt][r] + bn, p.act);
    }
    __threadfence_block();                  // the wave's own LDS writes complete before its reads
    __builtin_amdgcn_wave_barrier();
    // 16 rows x NP/8 chunks of 8 columns
    for (int c = lane; c < 16 * (NP / 8); c += 64) {
      const int r = c / (NP / 8), c8 = (c % (NP / 8)) * 8;
      const long m = m0 + r;
      if (m >= p.M || c8 >= p.N) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = sO[w][r][c8 + e];
      if (c8 + 8 <= p.N && (p.ldc % 8) == 0 && (!p.U || p.ldu % 8 == 0) && (!p.R || p.ldr % 8 == 0)) {
        if (p.U) {
          const tx8 u = *reinterpret_cast<const tx8*>(p.U + m * p.ldu + c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= act_grad((float)u[e], p.uact);
        }
        if (p.R) {
          const tx8 rr = *reinterpret_cast<const tx8*>(p.R + m * p.ldr + c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rr[e];
        }
        tx8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (T)v[e];
        *reinterpret_cast<tx8*>(p.C + m * p.ldc + c8) = o;
      } else {
        for (int e = 0; e < 8 && c8 + e < p.N; ++e) {
          float x = v[e];
          if (p.U) x *= act_grad((float)p.U[m * p.ldu + c8 + e], p.uact);
          if (p.R) x += (float)p.R[m * p.ldr + c8 + e];
          p.C[m * p.ldc + c8 + e] = (T)x;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

struct SkinnyWgradArgs {
  const bf16* dY; long ldy;
  const bf16* X; long ldx;
  float* dW; long lddw;
  float* db;
  int M, N, K, mchunk;
};

template <int NT, int KT>
__global__ __launch_bounds__(256) void skinny_wgrad(SkinnyWgradArgs p) {
  constexpr int NP = NT * 16, KP = KT * 16;
  constexpr int SL = 128;           // rows per slab
  constexpr int LDT = SL + 8;
  __shared__ __attribute__((aligned(16))) bf16 sA[NP][LDT];
  __shared__ __attribute__((aligned(16))) bf16 sB[KP][LDT];
  __shared__ float sAcc[NP][KP + 1];
  __shared__ float sDb[NP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int mbeg = blockIdx.x * p.mchunk, mend = min(mbeg + p.mchunk, p.M);
  const bf16 z = (bf16)0.f;
  for (int i = tid; i < NP * (KP + 1); i += 256) (&sAcc[0][0])[i] = 0.f;
  if (tid < NP) sDb[tid] = 0.f;
  float dbp = 0.f;                  // thread tid < NP: column sum of dY over this WG's rows
  f32x4 acc[NT][KT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < KT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool av = (p.N % 8) == 0 && (p.ldy % 8) == 0, bv = (p.K % 8) == 0 && (p.ldx % 8) == 0;
  for (int m0 = mbeg; m0 < mend; m0 += SL) {
    __syncthreads();
    // stage dY rows (N wide) and X rows (K wide) transposed: chunk = (row, 8 columns)
    for (int c = tid; c < SL * (NP / 8); c += 256) {
      const int r = c % SL, c8 = (c / SL) * 8;
      const int m = m0 + r;
      bf16x8 v;
      if (m < mend && av && c8 < p.N) v = *reinterpret_cast<const bf16x8*>(p.dY + (long)m * p.ldy + c8);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (m < mend && c8 + e < p.N) ? p.dY[(long)m * p.ldy + c8 + e] : z;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sA[c8 + e][r] = v[e];
    }
    for (int c = tid; c < SL * (KP / 8); c += 256) {
      const int r = c % SL, c8 = (c / SL) * 8;
      const int m = m0 + r;
      bf16x8 v;
      if (m < mend && bv && c8 < p.K) v = *reinterpret_cast<const bf16x8*>(p.X + (long)m * p.ldx + c8);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (m < mend && c8 + e < p.K) ? p.X[(long)m * p.ldx + c8 + e] : z;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sB[c8 + e][r] = v[e];
    }
    __syncthreads();
    bf16x8 fa[NT], fb[KT];
#pragma unroll
    for (int i = 0; i < NT; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(&sA[i * 16 + fr][w * 32 + fg * 8]);
#pragma unroll
    for (int j = 0; j < KT; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(&sB[j * 16 + fr][w * 32 + fg * 8]);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < KT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (p.db && tid < NP) {
      float s = 0.f;
      for (int r = 0; r < SL; r += 8) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(&sA[tid][r]);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)v[e];
      }
      dbp += s;
    }
  }
  // C layout: col k = j * 16 + (lane & 15), row n = i * 16 + 4 (lane >> 4) + r
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < KT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(&sAcc[i * 16 + fg * 4 + r][j * 16 + fr], acc[i][j][r]);
  __syncthreads();
  for (int i = tid; i < NP * KP; i += 256) {
    const int n = i / KP, k = i % KP;
    if (n < p.N && k < p.K) atomicAdd(p.dW + (long)n * p.lddw + k, sAcc[n][k]);
  }
  if (p.db && tid < p.N) atomicAdd(p.db + tid, dbp);
}

}  // namespace svk

using namespace svk;

extern "C" int svk_gemm_skinny(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
                               const void* U, long ldu, int uact, const void* R, long ldr, void* C, long ldc, int M,
                               int N, int K, int act, void* stream) {
  if (M < 0 || N <= 0 || N > 64 || K <= 0 || K > 128 || !A || !W || !C || lda < K || ldw < K || ldc < N ||
      (U && ldu < N) || (R && ldr < N) || ((uintptr_t)A & 15) || (lda % 8 && K % 8 == 0)) {
    set_error("svk_gemm_skinny: bad args (N <= 64, K <= 128, 16-byte aligned A)"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  const long nblk = (M + 15) / 16;
  const int grid = (int)std::min<long>((nblk + 3) / 4, 2048);
  hipStream_t st = (hipStream_t)stream;
  const int nt = (N + 15) / 16, ks = (K + 31) / 32;
  SVK_DISPATCH_H16(dtype, T, {
    SkinnyArgs<T> a{(const T*)A, lda, (const T*)W, ldw, bias, (const T*)U, ldu, uact, (const T*)R, ldr, (T*)C, ldc,
                    M, N, K, act};
    auto go = [&](auto ntc, auto ksc) {
      constexpr int NT = decltype(ntc)::value, KS = decltype(ksc)::value;
      hipLaunchKernelGGL((skinny_gemm<T, NT, KS>), dim3(grid), dim3(256), 0, st, a);
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    auto by_ks = [&](auto ntc) {
      switch (ks) { case 1: go(ntc, I1{}); break; case 2: go(ntc, I2{}); break; case 3: go(ntc, I3{}); break;
                    default: go(ntc, I4{}); break; }
    };
    switch (nt) { case 1: by_ks(I1{}); break; case 2: by_ks(I2{}); break; case 3: by_ks(I3{}); break;
                  default: by_ks(I4{}); break; }
    return check_launch("skinny_gemm");
  });
}

extern "C" int svk_wgrad_skinny(const void* dY, long ldy, const void* X, long ldx, float* dW, long lddw, float* db,
                                int M, int N, int K, void* stream) {
  const int nt = (N + 15) / 16, kt = (K + 15) / 16;
  if (M < 0 || N <= 0 || K <= 0 || nt > 8 || kt > 8 || nt * kt > 16 || !dY || !X || !dW || ldy < N || ldx < K ||
      lddw < K || (((uintptr_t)dY | (uintptr_t)X) & 15)) {
    set_error("svk_wgrad_skinny: bad args (N, K <= 128 with (N/16)*(K/16) <= 16, bf16)"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  // ~512 workgroups, each >= 512 rows, slab-aligned (SVK_SKINNY_WG: the workgroup target, SVK_SKINNY_MINROWS: the
  // row floor — A/B knobs)
  static const long sk_wg = getenv("SVK_SKINNY_WG") ? std::max(1L, atol(getenv("SVK_SKINNY_WG"))) : 512;
  static const long sk_min = getenv("SVK_SKINNY_MINROWS") ? std::max(128L, atol(getenv("SVK_SKINNY_MINROWS"))) : 512;
  long chunk = std::max<long>(sk_min, (M + sk_wg - 1) / sk_wg);
  chunk = (chunk + 127) / 128 * 128;
  const int grid = (int)((M + chunk - 1) / chunk);
  SkinnyWgradArgs a{(const bf16*)dY, ldy, (const bf16*)X, ldx, dW, lddw, db, M, N, K, (int)chunk};
  hipStream_t st = (hipStream_t)stream;
  auto go = [&](auto ntc, auto ktc) {
    constexpr int NT = decltype(ntc)::value, KT = decltype(ktc)::value;
    if constexpr (NT * KT <= 16) hipLaunchKernelGGL((skinny_wgrad<NT, KT>), dim3(grid), dim3(256), 0, st, a);
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  const int ntp = nt <= 1 ? 1 : nt <= 2 ? 2 : nt <= 4 ? 4 : 8;
  const int ktp = kt <= 1 ? 1 : kt <= 2 ? 2 : kt <= 4 ? 4 : 8;
  if (ntp * ktp > 16) { set_error("svk_wgrad_skinny: tile too large"); return SVK_EUNSUPPORTED; }
  auto by_kt = [&](auto ntc) {
    switch (ktp) { case 1: go(ntc, I1{}); break; case 2: go(ntc, I2{}); break; case 4: go(ntc, I4{}); break;
                   default: go(ntc, I8{}); break; }
  };
  switch (ntp) { case 1: by_kt(I1{}); break; case 2: by_kt(I2{}); break; case 4: by_kt(I4{}); break;
                 default: by_kt(I8{}); break; }
  return check_launch("skinny_wgrad");
}
