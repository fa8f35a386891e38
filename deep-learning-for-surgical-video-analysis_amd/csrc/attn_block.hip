// Stage-1 attention half of the MiT Block in one kernel, f16 / bf16 (mix_transformer_evp.py:71-131 Attention
// with one head of 64 channels and sequence reduction, Block :134-171):
//
//   q  = h Wq^T + bq                       h = norm1(x) [B, N, 64] (the sequence-reduced k / v come from kv)
//   o  = softmax(scale q k^T) v            k, v [B, Nk <= 64, 64] (kv = [k | v], row stride ldkv)
//   y  = x + o Wp^T + bp                   (Block residual)
//   h2 = norm2(y)                          (LayerNorm of the MixFFN input)
//
// Unfused, the q GEMM writes q, attention reads it and writes o, the proj GEMM reads o and x and writes y,
// and the LayerNorm reads y again: 9 passes over a [B, 3136, 64] token map (103 MB each at B = 256).  Here
// a 16-query tile goes h -> q -> S -> P -> o -> y -> h2 on chip: h and x are read once, y and h2 written once.
//
// Workgroup = 256 queries of one frame (4 waves walking 16-query tiles); Wq, Wp, K and V^T are staged in LDS
// once per workgroup.  Per tile (16x16x32 MFMAs throughout, f32 accumulation, roundings where the unfused
// path rounds to the storage type: q, o, y):
//   Q^T = Wq . H^T   A = Wq rows (LDS), B = the tile's h rows (16-byte global loads); lane (c, g) ends with
//                    q[query c][d] for d in {16 dt + 4 g + r}: exactly the operand the S MFMA needs when the
//                    reduction index is permuted the same way on the K side (two 8-byte LDS reads per key row).
//   S^T = K . Q^T, in-register softmax over the <= 64 keys, O = P . V  (as attention_mfma_bf16_res).
//   O goes through the wave's LDS patch (C layout -> row layout) and feeds Y = O . Wp^T; the x tile is staged
//   through the same patch; y is rounded, its LayerNorm reduced over the 16 lanes that hold a row, and y / h2
//   leave as 16-byte row pieces through the patch.
#include "svk_common.h"
#include <stdio.h>
#include <type_traits>

namespace svk {
namespace ab {

constexpr int D = 64;          // channels = head dim (one head)
constexpr int KLD = D + 8;     // LDS row stride (elements) of Wq / Wp / K / the patches
constexpr int VLD = 64 + 8;    // V^T row stride (keys padded to 64)
constexpr int QB = 256;   // default queries per workgroup (svk_tune("ffn_diag") 2 / 3: 512 / 1024, sweep)

template <typename T, int QB>
__global__ __launch_bounds__(256) void attn_block_s1(const T* __restrict__ Hn, const T* __restrict__ X,
                                                     const T* __restrict__ KV, long ldkv, const T* __restrict__ Wq,
                                                     const float* __restrict__ bq, const T* __restrict__ Wp,
                                                     const float* __restrict__ bp, const float* __restrict__ g2,
                                                     const float* __restrict__ b2, float eps, T* __restrict__ Y,
                                                     T* __restrict__ H2, int N, int Nk, float scale_log2) {
  typedef v8_t<T> tx8;
  typedef v4_t<T> tx4;
  __shared__ __attribute__((aligned(16))) T sWq[D][KLD];
  __shared__ __attribute__((aligned(16))) T sWp[D][KLD];
  __shared__ __attribute__((aligned(16))) T sK[64][KLD];
  __shared__ __attribute__((aligned(16))) T sVt[D][VLD];
  __shared__ __attribute__((aligned(16))) T sP[4][16][KLD];     // per-wave patch
  __shared__ float sEp[5][D];                                    // bq, bp, gamma, beta (f32), spare

  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const T zero = (T)0.f;
  const T* Hb = Hn + (long)b * N * D;
  const T* Xb = X + (long)b * N * D;
  const T* KVb = KV + (long)b * Nk * ldkv;
  T* Yb = Y + (long)b * N * D;
  T* H2b = H2 + (long)b * N * D;

  for (int e = tid; e < D * (D / 8); e += 256) {
    const int r = e / (D / 8), c8 = (e % (D / 8)) * 8;
    *reinterpret_cast<tx8*>(&sWq[r][c8]) = *reinterpret_cast<const tx8*>(Wq + r * D + c8);
    *reinterpret_cast<tx8*>(&sWp[r][c8]) = *reinterpret_cast<const tx8*>(Wp + r * D + c8);
  }
  for (int e = tid; e < 64 * (D / 8); e += 256) {
    const int key = e / (D / 8), d0 = (e % (D / 8)) * 8;
    tx8 kv, vv;
    if (key < Nk) {
      kv = *reinterpret_cast<const tx8*>(KVb + (long)key * ldkv + d0);
      vv = *reinterpret_cast<const tx8*>(KVb + (long)key * ldkv + D + d0);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { kv[j] = zero; vv[j] = zero; }
    }
    *reinterpret_cast<tx8*>(&sK[key][d0]) = kv;
#pragma unroll
    for (int j = 0; j < 8; ++j) sVt[d0 + j][key] = vv[j];
  }
  for (int e = tid; e < 4 * D; e += 256) {
    const int w = e / D, d = e % D;
    const float* src = w == 0 ? bq : (w == 1 ? bp : (w == 2 ? g2 : b2));
    sEp[w][d] = src ? src[d] : 0.f;
  }
  __syncthreads();

  T (*patch)[KLD] = sP[wave];
  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int qbase = blockIdx.x * QB;
  // software pipeline over the wave's tiles: the next tile's h rows and this tile's x rows are in flight
  // while the current tile computes
  auto load_h = [&](int q0, tx8 (&hb)[2]) {
    const int qr = min(q0 + c, N - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) hb[ks] = *reinterpret_cast<const tx8*>(Hb + (long)qr * D + 32 * ks + 8 * g);
  };
  tx8 hb_next[2];
  if (qbase + wave * 16 < N) load_h(qbase + wave * 16, hb_next);
  for (int qt = wave; qt < QB / 16; qt += 4) {
    const int q0 = qbase + qt * 16;
    if (q0 >= N) break;
    tx8 xr[2];                                     // this tile's x rows (row e >> 3, chunk e & 7 of e = lane + 64 k)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      xr[k] = *reinterpret_cast<const tx8*>(Xb + (long)min(q0 + (e >> 3), N - 1) * D + (e & 7) * 8);
    }
    // ---- Q^T = Wq . H^T: lane (c, g) gets q[query q0 + c][16 dt + 4 g + r]
    f32x4 qa[4];
    {
      tx8 hb[2] = {hb_next[0], hb_next[1]};
      if (q0 + 64 < min(N, qbase + QB)) load_h(q0 + 64, hb_next);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        qa[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const tx8 a = *reinterpret_cast<const tx8*>(&sWq[16 * dt + c][32 * ks + 8 * g]);
          qa[dt] = mfma16x16x32(a, hb[ks], qa[dt]);
        }
      }
    }
    // rounded to the storage type like the unfused q GEMM's output; S-MFMA k-step s takes dt = 2s, 2s + 1
    tx8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int dt = 2 * s + (j >> 2), r = j & 3;
        qf[s][j] = (T)(qa[dt][r] + sEp[0][16 * dt + 4 * g + r]);
      }
    // ---- S^T = K . Q^T (the same d permutation on the K side), softmax over the keys in registers
    f32x4 sc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const tx4 k0 = *reinterpret_cast<const tx4*>(&sK[16 * t + c][16 * (2 * s) + 4 * g]);
        const tx4 k1 = *reinterpret_cast<const tx4*>(&sK[16 * t + c][16 * (2 * s + 1) + 4 * g]);
        tx8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = k0[j]; a[4 + j] = k1[j]; }
        sc[t] = mfma16x16x32(a, qf[s], sc[t]);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * t + 4 * g + r;
        const float v = key < Nk ? sc[t][r] * scale_log2 : -INFINITY;
        sc[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float ps = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(sc[t][r] - mx);
        sc[t][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    // ---- O = P . V: lane holds O[query 4g + r][16 dt + c]
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      tx8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (T)sc[2 * s2][j];
        pa[4 + j] = (T)sc[2 * s2 + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const tx4 v0 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][32 * s2 + 4 * g]);
        const tx4 v1 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][32 * s2 + 16 + 4 * g]);
        tx8 vb;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
        o[dt] = mfma16x16x32(pa, vb, o[dt]);
      }
    }
    // normalised o (rounded like the attention kernel's output) -> patch, row layout
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float inv = 1.0f / __shfl(ps, 4 * g + r, 64);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) patch[4 * g + r][16 * dt + c] = (T)(o[dt][r] * inv);
    }
    wave_sync();
    // ---- Y = O . Wp^T: lane holds y[query 4g + r][16 nt + c]
    f32x4 ya[4];
    {
      tx8 oa[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) oa[ks] = *reinterpret_cast<const tx8*>(&patch[c][32 * ks + 8 * g]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        ya[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const tx8 w = *reinterpret_cast<const tx8*>(&sWp[16 * nt + c][32 * ks + 8 * g]);
          ya[nt] = mfma16x16x32(w, oa[ks], ya[nt]);   // transposed: C[row = n][col = query]
        }
      }
    }
    // ya[nt][r] = Y[query c][n = 16 nt + 4 g + r] (W fragment x O fragment): the lane owns 16 channels
    // {16 nt + 4 g + r} of query c.  Stage the x tile through the patch (row layout) for the residual.
    wave_sync();                                   // the o reads of the patch are done
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      *reinterpret_cast<tx8*>(&patch[e >> 3][(e & 7) * 8]) = xr[k];
    }
    wave_sync();
    float yv[4][4], sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * nt + 4 * g + r;
        const float v = ya[nt][r] + sEp[1][n] + to_f(patch[c][n]);
        yv[nt][r] = to_f(from_f<T>(v));            // the block output as the unfused path stores it
        sum += yv[nt][r];
      }
    // LayerNorm of query c's 64 channels: held by lanes c, c + 16, c + 32, c + 48 (16 each)
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float mean = sum * (1.0f / D);
    float sq = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) { const float dd = yv[nt][r] - mean; sq += dd * dd; }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    const float rstd = 1.0f / sqrtf(sq * (1.0f / D) + eps);
    wave_sync();                                   // the x reads of the patch are done
    // y -> patch -> 16-byte rows; then h2 the same way
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      tx4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (T)yv[nt][r];
      *reinterpret_cast<tx4*>(&patch[c][16 * nt + 4 * g]) = v;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k, row = e >> 3, c8 = (e & 7) * 8;
      if (q0 + row < N) *reinterpret_cast<tx8*>(Yb + (long)(q0 + row) * D + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      tx4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * nt + 4 * g + r;
        v[r] = (T)((yv[nt][r] - mean) * rstd * sEp[2][n] + sEp[3][n]);
      }
      *reinterpret_cast<tx4*>(&patch[c][16 * nt + 4 * g]) = v;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k, row = e >> 3, c8 = (e & 7) * 8;
      if (q0 + row < N) *reinterpret_cast<tx8*>(H2b + (long)(q0 + row) * D + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();                                   // the patch is rewritten by this wave's next tile
  }
}

}  // namespace ab
}  // namespace svk

using namespace svk;

extern "C" int svk_attn_block_s1(int dtype, const void* Hn, const void* X, const void* KV, long ldkv, const void* Wq,
                                 const float* bq, const void* Wp, const float* bp, const float* gamma2,
                                 const float* beta2, float eps, void* Y, void* H2, int B, int N, int Nk, int C,
                                 float scale, void* stream) {
  if (B < 0 || N < 0 || Nk <= 0 || Nk > 64 || C != ab::D || !Hn || !X || !KV || !Wq || !Wp || !Y || !H2 ||
      !gamma2 || !beta2 || ldkv < 2 * C || ldkv % 8) {
    set_error("svk_attn_block_s1: bad args (C=%d must be 64, Nk=%d in 1..64, ldkv=%ld >= 2C, %% 8)", C, Nk, ldkv);
    return SVK_EINVAL;
  }
  if ((((uintptr_t)Hn) | ((uintptr_t)X) | ((uintptr_t)KV) | ((uintptr_t)Wq) | ((uintptr_t)Wp) | ((uintptr_t)Y) |
       ((uintptr_t)H2)) & 15) {
    set_error("svk_attn_block_s1: pointers must be 16-byte aligned"); return SVK_EINVAL;
  }
  if (B == 0 || N == 0) return SVK_OK;
  if (B > 65535) { set_error("svk_attn_block_s1: grid too large"); return SVK_EUNSUPPORTED; }
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t st = (hipStream_t)stream;
  const int qsel = g_tune[TUNE_FFN_DIAG];
  SVK_DISPATCH_H16(dtype, T, {
    auto go = [&](auto qb_c) {
      constexpr int QBv = decltype(qb_c)::value;
      dim3 grid((N + QBv - 1) / QBv, B);
      hipLaunchKernelGGL((ab::attn_block_s1<T, QBv>), grid, dim3(256), 0, st, (const T*)Hn, (const T*)X, (const T*)KV,
                         ldkv, (const T*)Wq, bq, (const T*)Wp, bp, gamma2, beta2, eps, (T*)Y, (T*)H2, N, Nk, sl2);
    };
    if (qsel == 2) go(std::integral_constant<int, 512>{});
    else if (qsel == 3) go(std::integral_constant<int, 1024>{});
    else go(std::integral_constant<int, ab::QB>{});
    set_last_kernel(dtype == SVK_F16 ? "attn_block_s1<_Float16>" : "attn_block_s1<__bf16>");
    return check_launch("attn_block_s1");
  });
}
