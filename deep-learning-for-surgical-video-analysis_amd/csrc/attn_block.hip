// Attention half of a MiT Block in one kernel for the 64-channel-head stages (stage 1: C = 64, one head;
// stage 2: C = 128, two heads), f16 / bf16 (mix_transformer_evp.py:71-131 Attention with sequence
// reduction, Block :134-171):
//
//   q  = h Wq^T + bq                       h = norm1(x) [B, N, C] (the sequence-reduced k / v come from kv)
//   o  = softmax(scale q_h k_h^T) v_h      per 64-channel head h; k, v [B, Nk <= 64, C] (kv = [k | v])
//   y  = x + o Wp^T + bp                   (Block residual)
//   h2 = norm2(y)                          (LayerNorm of the MixFFN input)
//
// Unfused, the q GEMM writes q, attention reads it and writes o, the proj GEMM reads o and x and writes y,
// and the LayerNorm reads y again: 9 passes over a [B, 3136, 64] token map (103 MB each at B = 256).  Here
// a 16-query tile goes h -> q -> S -> P -> o -> y -> h2 on chip: h and x are read once, y and h2 written once.
//
// Workgroup = QB queries of one frame (NW waves walking 16-query tiles); Wq, Wp, K and V^T are staged in LDS
// once per workgroup (stage 2: one 8-wave workgroup per 784-token frame, 139 KB of LDS).  Per tile (16x16x32 MFMAs throughout, f32 accumulation, roundings where the unfused
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

constexpr int HD = 64;         // head dim
constexpr int VLD = 64 + 8;    // V^T row stride (keys padded to 64)

template <int NH, int NW>
struct L {                      // dynamic LDS carve (bytes, 16-byte aligned pieces)
  static constexpr int C = HD * NH, LD = C + 8;
  static constexpr int WQ = 0, WP = WQ + C * LD * 2, K = WP + C * LD * 2, VT = K + 64 * LD * 2;
  static constexpr int PT = VT + C * VLD * 2, EP = PT + NW * 16 * LD * 2, BYTES = EP + 4 * C * 4;
};

template <typename T, int NH, int NW, int QB>
__global__ __launch_bounds__(64 * NW) void attn_block(const T* __restrict__ Hn, const T* __restrict__ X,
                                                      const T* __restrict__ KV, long ldkv, const T* __restrict__ Wq,
                                                      const float* __restrict__ bq, const T* __restrict__ Wp,
                                                      const float* __restrict__ bp, const float* __restrict__ g2,
                                                      const float* __restrict__ b2, float eps, T* __restrict__ Y,
                                                      T* __restrict__ H2, int N, int Nk, float scale_log2) {
  typedef v8_t<T> tx8;
  typedef v4_t<T> tx4;
  typedef L<NH, NW> Lay;
  constexpr int C = Lay::C, LD = Lay::LD, NT = 64 * NW, CT = C / 16, KS = C / 32, RC = C / 32;
  extern __shared__ __attribute__((aligned(16))) char smem_ab[];
  T (*sWq)[LD] = reinterpret_cast<T (*)[LD]>(smem_ab + Lay::WQ);
  T (*sWp)[LD] = reinterpret_cast<T (*)[LD]>(smem_ab + Lay::WP);
  T (*sK)[LD] = reinterpret_cast<T (*)[LD]>(smem_ab + Lay::K);
  T (*sVt)[VLD] = reinterpret_cast<T (*)[VLD]>(smem_ab + Lay::VT);
  float (*sEp)[C] = reinterpret_cast<float (*)[C]>(smem_ab + Lay::EP);

  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const T zero = (T)0.f;
  T (*patch)[LD] = reinterpret_cast<T (*)[LD]>(smem_ab + Lay::PT + wave * 16 * LD * 2);
  const T* Hb = Hn + (long)b * N * C;
  const T* Xb = X + (long)b * N * C;
  const T* KVb = KV + (long)b * Nk * ldkv;
  T* Yb = Y + (long)b * N * C;
  T* H2b = H2 + (long)b * N * C;

  for (int e = tid; e < C * (C / 8); e += NT) {
    const int r = e / (C / 8), c8 = (e % (C / 8)) * 8;
    *reinterpret_cast<tx8*>(&sWq[r][c8]) = *reinterpret_cast<const tx8*>(Wq + r * C + c8);
    *reinterpret_cast<tx8*>(&sWp[r][c8]) = *reinterpret_cast<const tx8*>(Wp + r * C + c8);
  }
  for (int e = tid; e < 64 * (C / 8); e += NT) {
    const int key = e / (C / 8), d0 = (e % (C / 8)) * 8;
    tx8 kv, vv;
    if (key < Nk) {
      kv = *reinterpret_cast<const tx8*>(KVb + (long)key * ldkv + d0);
      vv = *reinterpret_cast<const tx8*>(KVb + (long)key * ldkv + C + d0);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { kv[j] = zero; vv[j] = zero; }
    }
    *reinterpret_cast<tx8*>(&sK[key][d0]) = kv;
#pragma unroll
    for (int j = 0; j < 8; ++j) sVt[d0 + j][key] = vv[j];
  }
  for (int e = tid; e < 4 * C; e += NT) {
    const int w = e / C, d = e % C;
    const float* src = w == 0 ? bq : (w == 1 ? bp : (w == 2 ? g2 : b2));
    sEp[w][d] = src ? src[d] : 0.f;
  }
  __syncthreads();

  auto wave_sync = []() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int qbase = blockIdx.x * QB;
  // software pipeline over the wave's tiles: the next tile's h rows and this tile's x rows are in flight
  // while the current tile computes
  auto load_h = [&](int q0, tx8 (&hb)[KS]) {
    const int qr = min(q0 + c, N - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hb[ks] = *reinterpret_cast<const tx8*>(Hb + (long)qr * C + 32 * ks + 8 * g);
  };
  tx8 hb_next[KS];
  if (qbase + wave * 16 < N) load_h(qbase + wave * 16, hb_next);
  for (int qt = wave; qt < QB / 16; qt += NW) {
    const int q0 = qbase + qt * 16;
    if (q0 >= N) break;
    tx8 xr[RC];                                    // this tile's x rows: chunk e = lane + 64 k, row e / (C/8)
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k, row = e / (C / 8);
      xr[k] = *reinterpret_cast<const tx8*>(Xb + (long)min(q0 + row, N - 1) * C + (e % (C / 8)) * 8);
    }
    // ---- Q^T = Wq . H^T: lane (c, g) gets q[query q0 + c][16 dt + 4 g + r]
    f32x4 qa[CT];
    {
      tx8 hb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) hb[ks] = hb_next[ks];
      if (q0 + 16 * NW < min(N, qbase + QB)) load_h(q0 + 16 * NW, hb_next);
#pragma unroll
      for (int dt = 0; dt < CT; ++dt) {
        qa[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const tx8 a = *reinterpret_cast<const tx8*>(&sWq[16 * dt + c][32 * ks + 8 * g]);
          qa[dt] = mfma16x16x32(a, hb[ks], qa[dt]);
        }
      }
    }
    f32x4 o[CT];
    float ps_h[NH];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      // q of head hh rounded to the storage type like the unfused q GEMM's output; S-MFMA k-step s takes
      // d tiles 4 hh + 2 s and 4 hh + 2 s + 1 (the same permutation of d on the K side)
      tx8 qf[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dt = 4 * hh + 2 * s2 + (j >> 2), r = j & 3;
          qf[s2][j] = (T)(qa[dt][r] + sEp[0][16 * dt + 4 * g + r]);
        }
      f32x4 sc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const tx4 k0 = *reinterpret_cast<const tx4*>(&sK[16 * t + c][HD * hh + 16 * (2 * s2) + 4 * g]);
          const tx4 k1 = *reinterpret_cast<const tx4*>(&sK[16 * t + c][HD * hh + 16 * (2 * s2 + 1) + 4 * g]);
          tx8 a;
#pragma unroll
          for (int j = 0; j < 4; ++j) { a[j] = k0[j]; a[4 + j] = k1[j]; }
          sc[t] = mfma16x16x32(a, qf[s2], sc[t]);
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
      ps_h[hh] = ps;
      // O_h = P . V_h: lane holds O[query 4g + r][64 hh + 16 dt + c]
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[4 * hh + dt] = f32x4{0.f, 0.f, 0.f, 0.f};
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
          const tx4 v0 = *reinterpret_cast<const tx4*>(&sVt[HD * hh + 16 * dt + c][32 * s2 + 4 * g]);
          const tx4 v1 = *reinterpret_cast<const tx4*>(&sVt[HD * hh + 16 * dt + c][32 * s2 + 16 + 4 * g]);
          tx8 vb;
#pragma unroll
          for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
          o[4 * hh + dt] = mfma16x16x32(pa, vb, o[4 * hh + dt]);
        }
      }
    }
    // normalised o (rounded like the attention kernel's output) -> patch, row layout
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float inv = 1.0f / __shfl(ps_h[hh], 4 * g + r, 64);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) patch[4 * g + r][HD * hh + 16 * dt + c] = (T)(o[4 * hh + dt][r] * inv);
      }
    wave_sync();
    // ---- Y = O . Wp^T (transposed MFMA: W fragment x O fragment): ya[nt][r] = Y[query c][16 nt + 4 g + r]
    f32x4 ya[CT];
    {
      tx8 oa[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) oa[ks] = *reinterpret_cast<const tx8*>(&patch[c][32 * ks + 8 * g]);
#pragma unroll
      for (int nt = 0; nt < CT; ++nt) {
        ya[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const tx8 w = *reinterpret_cast<const tx8*>(&sWp[16 * nt + c][32 * ks + 8 * g]);
          ya[nt] = mfma16x16x32(w, oa[ks], ya[nt]);
        }
      }
    }
    wave_sync();                                   // the o reads of the patch are done: x tile in
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k;
      *reinterpret_cast<tx8*>(&patch[e / (C / 8)][(e % (C / 8)) * 8]) = xr[k];
    }
    wave_sync();
    float yv[CT][4], sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < CT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * nt + 4 * g + r;
        const float v = ya[nt][r] + sEp[1][n] + to_f(patch[c][n]);
        yv[nt][r] = to_f(from_f<T>(v));            // the block output as the unfused path stores it
        sum += yv[nt][r];
      }
    // LayerNorm of query c's C channels: held by lanes c, c + 16, c + 32, c + 48 (C / 4 each)
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
    wave_sync();                                   // the x reads of the patch are done
    // y -> patch -> 16-byte rows; then h2 the same way
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
      if (q0 + row < N) *reinterpret_cast<tx8*>(Yb + (long)(q0 + row) * C + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();
#pragma unroll
    for (int nt = 0; nt < CT; ++nt) {
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
    for (int k = 0; k < RC; ++k) {
      const int e = lane + 64 * k, row = e / (C / 8), c8 = (e % (C / 8)) * 8;
      if (q0 + row < N) *reinterpret_cast<tx8*>(H2b + (long)(q0 + row) * C + c8) = *reinterpret_cast<const tx8*>(&patch[row][c8]);
    }
    wave_sync();                                   // the patch is rewritten by this wave's next tile
  }
}

template <typename T, int NH, int NW, int QB>
static void launch(const void* Hn, const void* X, const void* KV, long ldkv, const void* Wq, const float* bq,
                   const void* Wp, const float* bp, const float* g2, const float* b2, float eps, void* Y, void* H2,
                   int B, int N, int Nk, float sl2, hipStream_t st) {
  constexpr int LDS = L<NH, NW>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_block<T, NH, NW, QB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  dim3 grid((N + QB - 1) / QB, B);
  hipLaunchKernelGGL((attn_block<T, NH, NW, QB>), grid, dim3(64 * NW), LDS, st, (const T*)Hn, (const T*)X,
                     (const T*)KV, ldkv, (const T*)Wq, bq, (const T*)Wp, bp, g2, b2, eps, (T*)Y, (T*)H2, N, Nk, sl2);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "attn_block<%s, %d, %d, %d>", type_name<T>(), NH, NW, QB);
  set_last_kernel(name);
}

}  // namespace ab
}  // namespace svk

using namespace svk;

extern "C" int svk_attn_block(int dtype, const void* Hn, const void* X, const void* KV, long ldkv, const void* Wq,
                              const float* bq, const void* Wp, const float* bp, const float* gamma2,
                              const float* beta2, float eps, void* Y, void* H2, int B, int N, int Nk, int C,
                              float scale, void* stream) {
  if (B < 0 || N < 0 || Nk <= 0 || Nk > 64 || (C != 64 && C != 128) || !Hn || !X || !KV || !Wq || !Wp || !Y || !H2 ||
      !gamma2 || !beta2 || ldkv < 2 * C || ldkv % 8) {
    set_error("svk_attn_block: bad args (C=%d must be 64 or 128, Nk=%d in 1..64, ldkv=%ld >= 2C, %% 8)", C, Nk, ldkv);
    return SVK_EINVAL;
  }
  if ((((uintptr_t)Hn) | ((uintptr_t)X) | ((uintptr_t)KV) | ((uintptr_t)Wq) | ((uintptr_t)Wp) | ((uintptr_t)Y) |
       ((uintptr_t)H2)) & 15) {
    set_error("svk_attn_block: pointers must be 16-byte aligned"); return SVK_EINVAL;
  }
  if (B == 0 || N == 0) return SVK_OK;
  if (B > 65535) { set_error("svk_attn_block: grid too large"); return SVK_EUNSUPPORTED; }
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    const int sel = g_tune[TUNE_ATTN_CFG];   // tile-shape sweep (svk_tune("attn_cfg"), tools/attn_block_bench.py)
    // C = 64: 8 waves x 256 queries (same-box whole-step A/B vs 4 waves: +0.25 %, 3 x 3 runs)
    if (C == 64 && sel == 4) ab::launch<T, 1, 8, 512>(Hn, X, KV, ldkv, Wq, bq, Wp, bp, gamma2, beta2, eps, Y, H2, B, N, Nk, sl2, st);
    else if (C == 64 && sel == 6) ab::launch<T, 1, 4, 256>(Hn, X, KV, ldkv, Wq, bq, Wp, bp, gamma2, beta2, eps, Y, H2, B, N, Nk, sl2, st);
    else if (C == 64) ab::launch<T, 1, 8, 256>(Hn, X, KV, ldkv, Wq, bq, Wp, bp, gamma2, beta2, eps, Y, H2, B, N, Nk, sl2, st);
    else ab::launch<T, 2, 8, 784>(Hn, X, KV, ldkv, Wq, bq, Wp, bp, gamma2, beta2, eps, Y, H2, B, N, Nk, sl2, st);
    return check_launch("attn_block");
  });
}
