// Prompt adapter + norm1 of a MiT Block in one kernel, f16 / bf16 (PromptGenerator.get_prompt,
// mix_transformer_evp.py:776-815, followed by Block.norm1, :134-171), for the token-heavy stages 1-2
// (C = 64 / 128, prompt width C4 = C / 4 = 16 / 32):
//
//   f  = GELU(S Wl^T + bl)          S = hc + emb [M, C4] (the stage's summed prompt features)
//   X' = X + f Ws^T + bs            (the prompted block input)
//   H  = LayerNorm(X'; g1, b1)      (norm1: the attention input)
//
// Unfused: the lightweight GEMM writes f, the shared GEMM reads f and X and writes X', the LayerNorm reads
// X' again.  Here per 16-token tile: f^T = Wl . S^T (lane (c, g) ends with f[token c][16 jt + 4 g + r]),
// rounded like the unfused GEMM output, feeds Y^T = Ws . f^T directly as the B operand — the reduction
// index of the shared GEMM permuted to {16 jt + 4 g + r} on both operands (two 8-byte reads of a Ws row) —
// then + bs + x (x tile staged through the wave's LDS patch), rounded, LayerNorm over the 4 lanes that hold
// a token, X' and H out as 16-byte rows.  Wl, Ws resident in LDS; workgroups walk tiles grid-stride.
#include "svk_common.h"
#include <stdio.h>
#include <type_traits>
#include <algorithm>

namespace svk {
namespace pl {

template <int C_>
struct Cfg {
  static constexpr int C = C_, C4 = C / 4, LD = C + 8, NW = 4;
  static constexpr int JT = C4 / 16;             // f tiles (16 prompt channels each)
  static constexpr int KSL = (C4 + 31) / 32;     // lightweight-GEMM k-steps (inputs zero-padded)
  static constexpr int KS2 = (JT + 1) / 2;       // shared-GEMM k-steps (two f tiles each, the last may be half)
  static constexpr int LDW = 32 * (KSL > KS2 ? KSL : KS2) + 8;   // weight row stride (elements)
  static constexpr int CT = C / 16, RC = C / 32;
  static constexpr bool PREF = C <= 128;         // prefetch the x tile into registers (register budget)
  // dynamic LDS carve (bytes)
  static constexpr int OWL = 0, OWS = OWL + C4 * LDW * 2, OP = OWS + C * LDW * 2, OE = OP + NW * 16 * LD * 2;
  static constexpr int BYTES = OE + 4 * C * 4;
};

template <typename T, int C_>
__global__ __launch_bounds__(256) void prompt_ln(const T* __restrict__ S, const T* __restrict__ X,
                                                 const T* __restrict__ Wl, const float* __restrict__ bl,
                                                 const T* __restrict__ Ws, const float* __restrict__ bs,
                                                 const float* __restrict__ g1, const float* __restrict__ b1, float eps,
                                                 T* __restrict__ Xo, T* __restrict__ Ho, int M) {
  typedef Cfg<C_> K;
  typedef v8_t<T> tx8;
  typedef v4_t<T> tx4;
  constexpr int C = K::C, C4 = K::C4, LD = K::LD, LDW = K::LDW, CT = K::CT, RC = K::RC, JT = K::JT;
  extern __shared__ __attribute__((aligned(16))) char smem_pl[];
  T (*sWl)[LDW] = reinterpret_cast<T (*)[LDW]>(smem_pl + K::OWL);   // [out j][in k], k zero-padded
  T (*sWs)[LDW] = reinterpret_cast<T (*)[LDW]>(smem_pl + K::OWS);   // [out n][in j], j zero-padded
  float (*sEp)[C] = reinterpret_cast<float (*)[C]>(smem_pl + K::OE);  // bs, g1, b1 | bl (first C4)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const T zero = (T)0.f;
  for (int e = tid; e < C4 * (LDW - 8); e += 256) {
    const int j = e / (LDW - 8), k = e % (LDW - 8);
    sWl[j][k] = k < C4 ? Wl[j * C4 + k] : zero;
  }
  for (int e = tid; e < C * (LDW - 8); e += 256) {
    const int n = e / (LDW - 8), j = e % (LDW - 8);
    sWs[n][j] = j < C4 ? Ws[n * C4 + j] : zero;
  }
  for (int e = tid; e < 4 * C; e += 256) {
    const int w = e / C, d = e % C;
    sEp[w][d] = w == 0 ? (bs ? bs[d] : 0.f) : (w == 1 ? g1[d] : (w == 2 ? b1[d] : (d < C4 && bl ? bl[d] : 0.f)));
  }
  __syncthreads();
  T (*patch)[LD] = reinterpret_cast<T (*)[LD]>(smem_pl + K::OP + wave * 16 * LD * 2);
  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int ntile = (M + 15) / 16;
  for (int tile = blockIdx.x * K::NW + wave; tile < ntile; tile += gridDim.x * K::NW) {
    const int t0 = tile * 16;
    tx8 xr[K::PREF ? RC : 1];
    if constexpr (K::PREF) {
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int e = lane + 64 * k, row = e / (C / 8);
        xr[k] = *reinterpret_cast<const tx8*>(X + (long)min(t0 + row, M - 1) * C + (e % (C / 8)) * 8);
      }
    }
    // ---- f^T = Wl . S^T (k = the C4 prompt inputs, zero-padded): lane gets f[token c][16 jt + 4 g + r]
    tx8 sb[K::KSL];
    {
      const int tr = min(t0 + c, M - 1);
#pragma unroll
      for (int ks = 0; ks < K::KSL; ++ks) {
        if (32 * ks + 8 * g < C4) sb[ks] = *reinterpret_cast<const tx8*>(S + (long)tr * C4 + 32 * ks + 8 * g);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) sb[ks][j] = zero;
        }
      }
    }
    float fv[JT][4];
#pragma unroll
    for (int jt = 0; jt < JT; ++jt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < K::KSL; ++ks)
        acc = mfma16x16x32(*reinterpret_cast<const tx8*>(&sWl[16 * jt + c][32 * ks + 8 * g]), sb[ks], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) fv[jt][r] = to_f(from_f<T>(gelu_fast(acc[r] + sEp[3][16 * jt + 4 * g + r])));   // as the 16-bit GEMM epilogue
    }
    // ---- Y^T = Ws . f^T: k-step s covers f tiles 2s, 2s + 1 (a missing odd tile is zero on both sides)
    f32x4 ya[CT];
#pragma unroll
    for (int nt = 0; nt < CT; ++nt) ya[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < K::KS2; ++s2) {
      tx8 fb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int jt = 2 * s2 + (j >> 2);
        fb[j] = jt < JT ? (T)fv[jt < JT ? jt : 0][j & 3] : zero;
      }
#pragma unroll
      for (int nt = 0; nt < CT; ++nt) {
        const tx4 w0 = *reinterpret_cast<const tx4*>(&sWs[16 * nt + c][32 * s2 + 4 * g]);
        tx4 w1;
        if (2 * s2 + 1 < JT) w1 = *reinterpret_cast<const tx4*>(&sWs[16 * nt + c][32 * s2 + 16 + 4 * g]);
        else {
#pragma unroll
          for (int j = 0; j < 4; ++j) w1[j] = zero;
        }
        tx8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = w0[j]; a[4 + j] = w1[j]; }
        ya[nt] = mfma16x16x32(a, fb, ya[nt]);      // C[row = n][col = token]
      }
    }
    // ya[nt][r] = Y[token c][n = 16 nt + 4 g + r]; + bs + x (x tile through the patch, row layout)
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k;
      if constexpr (K::PREF) *reinterpret_cast<tx8*>(&patch[e / (C / 8)][(e % (C / 8)) * 8]) = xr[k];
      else
        *reinterpret_cast<tx8*>(&patch[e / (C / 8)][(e % (C / 8)) * 8]) =
            *reinterpret_cast<const tx8*>(X + (long)min(t0 + e / (C / 8), M - 1) * C + (e % (C / 8)) * 8);
    }
    wave_sync();
    float yv[CT][4], sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < CT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * nt + 4 * g + r;
        yv[nt][r] = to_f(from_f<T>(ya[nt][r] + sEp[0][n] + to_f(patch[c][n])));
        sum += yv[nt][r];
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float mean = sum * (1.0f / C);
    float sq = 0.f;
#pragma unroll
    for (int nt = 0; nt < CT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) { const float dd = yv[nt][r] - mean; sq += dd * dd; }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    const float rstd = 1.0f / sqrtf(sq * (1.0f / C) + eps);
    wave_sync();
#pragma unroll
    for (int nt = 0; nt < CT; ++nt) {
      tx4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (T)yv[nt][r];
      *reinterpret_cast<tx4*>(&patch[c][16 * nt + 4 * g]) = v;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k, row = e / (C / 8), c8 = (e % (C / 8)) * 8;
      if (t0 + row < M) *reinterpret_cast<tx8*>(Xo + (long)(t0 + row) * C + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();
#pragma unroll
    for (int nt = 0; nt < CT; ++nt) {
      tx4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * nt + 4 * g + r;
        v[r] = (T)((yv[nt][r] - mean) * rstd * sEp[1][n] + sEp[2][n]);
      }
      *reinterpret_cast<tx4*>(&patch[c][16 * nt + 4 * g]) = v;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k, row = e / (C / 8), c8 = (e % (C / 8)) * 8;
      if (t0 + row < M) *reinterpret_cast<tx8*>(Ho + (long)(t0 + row) * C + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();
  }
}

}  // namespace pl
}  // namespace svk

using namespace svk;

extern "C" int svk_prompt_ln(int dtype, const void* S, const void* X, const void* Wl, const float* bl, const void* Ws,
                             const float* bs, const float* gamma1, const float* beta1, float eps, void* Xo, void* Ho,
                             int M, int C, void* stream) {
  if (M < 0 || (C != 64 && C != 128 && C != 320) || !S || !X || !Wl || !Ws || !gamma1 || !beta1 || !Xo || !Ho) {
    set_error("svk_prompt_ln: bad args (C=%d must be 64, 128 or 320)", C); return SVK_EINVAL;
  }
  if ((((uintptr_t)S) | ((uintptr_t)X) | ((uintptr_t)Xo) | ((uintptr_t)Ho)) & 15) {
    set_error("svk_prompt_ln: S / X / outputs must be 16-byte aligned"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cus = std::max(cus, 1);
  }
  const long ntile = (M + 15) / 16;
  const int grid = (int)std::min<long>((ntile + 3) / 4, (long)cus * 8);
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    auto go = [&](auto c_c) {
      constexpr int CC = decltype(c_c)::value;
      constexpr int LDS = pl::Cfg<CC>::BYTES;
      static bool attr = false;
      if (!attr && LDS > 65536) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pl::prompt_ln<T, CC>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        attr = true;
      }
      hipLaunchKernelGGL((pl::prompt_ln<T, CC>), dim3(grid), dim3(256), LDS, st, (const T*)S, (const T*)X,
                         (const T*)Wl, bl, (const T*)Ws, bs, gamma1, beta1, eps, (T*)Xo, (T*)Ho, M);
    };
    if (C == 64) go(std::integral_constant<int, 64>{});
    else if (C == 128) go(std::integral_constant<int, 128>{});
    else go(std::integral_constant<int, 320>{});
    set_last_kernel(C == 64 ? "prompt_ln<64>" : (C == 128 ? "prompt_ln<128>" : "prompt_ln<320>"));
    return check_launch("prompt_ln");
  });
}
