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
#include <type_traits>

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

// ---------------------------------------------------------------------------------------------
// 16-bit MFMA attention (v_mfma_f32_16x16x32_bf16 / _f16; T = bf16 or f16, f32 softmax state).  Workgroup = 4 waves = 64 queries of one
// (batch, head); each wave owns 16 queries.  Keys are processed in chunks of 64 staged in LDS
// (K row-major, V transposed), with an online softmax across chunks (one chunk for MiT's 49
// reduced keys).
//
// Scores are computed transposed, S^T = K . Q^T (A = K rows from LDS, B = the wave's Q rows held
// in registers), so a lane's accumulator column is ONE query (lane & 15) and its 4 rows are keys
// 16t + 4g + r (g = lane >> 4).  The softmax max/sum over keys is then in-register + 2 shuffles
// (across g), and the exponentiated scores feed the P.V MFMA as its A operand without leaving
// registers: for k-step s the 8 elements of lane group g are keys {32s+4g+j} ++ {32s+16+4g+j}
// (j < 4), a permutation of the 32 keys that the V fragment read from LDS follows exactly.
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attention_mfma_bf16(const T* __restrict__ Q, long ldq, long sbq,
                                                           const T* __restrict__ K, long ldk, long sbk,
                                                           const T* __restrict__ V, long ldv, long sbv,
                                                           T* __restrict__ O, long ldo, long sbo,
                                                           int Nq, int Nk, int hd, float scale_log2) {
  constexpr int KC = 64;
  constexpr int KLD = HDP + 8;   // sK row stride (elements)
  constexpr int VLD = KC + 8;    // sVt row stride (elements)
  constexpr int NKS = HDP / 32;  // k-steps over the head dim
  constexpr int NDT = HDP / 16;  // 16-wide output column tiles
  typedef v8_t<T> tx8;
  typedef v4_t<T> tx4;
  __shared__ __attribute__((aligned(16))) T sK[KC][KLD];
  __shared__ __attribute__((aligned(16))) T sVt[HDP][VLD];

  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int q0 = blockIdx.x * 64 + wave * 16;
  const T* Qb = Q + (long)b * sbq + (long)h * hd;
  const T* Kb = K + (long)b * sbk + (long)h * hd;
  const T* Vb = V + (long)b * sbv + (long)h * hd;
  const bool vec = (hd == HDP) && ((ldq | ldk | ldv) % 8 == 0) &&
                   ((((uintptr_t)Qb) | ((uintptr_t)Kb) | ((uintptr_t)Vb)) & 15) == 0;

  tx8 qf[NKS];
  {
    const int qr = q0 + c;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 32 * ks + 8 * g;
      if (qr < Nq && vec) {
        qf[ks] = *reinterpret_cast<const tx8*>(Qb + (long)qr * ldq + d0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[ks][j] = (qr < Nq && d0 + j < hd) ? Qb[(long)qr * ldq + d0 + j] : (T)0.f;
      }
    }
  }

  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  for (int kc0 = 0; kc0 < Nk; kc0 += KC) {
    __syncthreads();
    for (int e = tid; e < KC * (HDP / 8); e += 256) {
      const int key = e / (HDP / 8), d0 = (e % (HDP / 8)) * 8;
      const int kg = kc0 + key;
      tx8 kv, vv;
      if (kg < Nk && vec) {
        kv = *reinterpret_cast<const tx8*>(Kb + (long)kg * ldk + d0);
        vv = *reinterpret_cast<const tx8*>(Vb + (long)kg * ldv + d0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool ok = kg < Nk && d0 + j < hd;
          kv[j] = ok ? Kb[(long)kg * ldk + d0 + j] : (T)0.f;
          vv[j] = ok ? Vb[(long)kg * ldv + d0 + j] : (T)0.f;
        }
      }
      *reinterpret_cast<tx8*>(&sK[key][d0]) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) sVt[d0 + j][key] = vv[j];
    }
    __syncthreads();

    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const tx8 a = *reinterpret_cast<const tx8*>(&sK[16 * t + c][32 * ks + 8 * g]);
        s[t] = mfma16x16x32(a, qf[ks], s[t]);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kc0 + 16 * t + 4 * g + r;
        const float v = key < Nk ? s[t][r] * scale_log2 : -INFINITY;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);    // 0 on the first chunk
    float ps = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[t][r] - m_new);
        s[t][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l_run = l_run * alpha + ps;
    m_run = m_new;
    if (kc0 > 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) o[dt][r] *= ar;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      tx8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (T)s[2 * s2][j];
        pa[4 + j] = (T)s[2 * s2 + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const tx4 v0 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][32 * s2 + 4 * g]);
        const tx4 v1 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][32 * s2 + 16 + 4 * g]);
        tx8 vb;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
        o[dt] = mfma16x16x32(pa, vb, o[dt]);
      }
    }
  }

  T* Ob = O + (long)b * sbo + (long)h * hd;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 4 * g + r;
    const float inv = 1.0f / __shfl(l_run, 4 * g + r, 64);
    if (qr >= Nq) continue;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int d = 16 * dt + c;
      if (d < hd) Ob[(long)qr * ldo + d] = (T)(o[dt][r] * inv);
    }
  }
}

// Resident-K/V variant for Nk <= 64 * NKC (every attention of the path: 49 reduced keys, 196 / 49 flow
// tokens): the whole K (row-major) and V (transposed) of one (batch, head) are staged in LDS ONCE per
// workgroup of QB = 256 queries — 4x fewer stagings per query than one 64-query block — and each
// wave then walks its 16-query tiles (tile t = wave, wave + 4, ...), the softmax over all keys
// computed chunk by chunk exactly as in attention_mfma_bf16.  The output tile goes through a
// per-wave LDS patch and leaves as 16-byte row pieces (one head row = hd * 2 bytes) instead of
// 2-byte scattered stores.  (Round 6: QB = 64 for the short stage-3 / 4 sequences — one 256-query workgroup per
// (frame, head) leaves its waves 4 / 3 / 3 / 3 tiles at 196 queries — ran the extraction step 0.7 % SLOWER in three
// interleaved pairs, profiles/r06/attn_qb64_ab.txt: the fourfold K / V staging costs more than the balance gains.
// Kept selectable, SVK_ATTN_QB=64, and tested bit-identical.)
template <typename T, int HDP, int NKC, int QB = 256>
__global__ __launch_bounds__(256) void attention_mfma_bf16_res(const T* __restrict__ Q, long ldq, long sbq,
                                                               const T* __restrict__ K, long ldk, long sbk,
                                                               const T* __restrict__ V, long ldv, long sbv,
                                                               T* __restrict__ O, long ldo, long sbo, int Nq,
                                                               int Nk, int hd, float scale_log2) {
  constexpr int KC = 64, NKP = NKC * KC;
  constexpr int KLD = HDP + 8;    // sK row stride (elements)
  constexpr int VLD = NKP + 8;    // sVt row stride (elements)
  constexpr int OLD = HDP + 8;    // per-wave output patch row stride
  constexpr int NKS = HDP / 32, NDT = HDP / 16;
  typedef v8_t<T> tx8;
  typedef v4_t<T> tx4;
  __shared__ __attribute__((aligned(16))) T sK[NKP][KLD];
  __shared__ __attribute__((aligned(16))) T sVt[HDP][VLD];
  __shared__ __attribute__((aligned(16))) T sO[4][16][OLD];

  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const T* Qb = Q + (long)b * sbq + (long)h * hd;
  const T* Kb = K + (long)b * sbk + (long)h * hd;
  const T* Vb = V + (long)b * sbv + (long)h * hd;
  T* Ob = O + (long)b * sbo + (long)h * hd;
  const T zero = (T)0.f;

  // this wave's Q tile rows (zeros past Nq / hd); a tile's rows are loaded one tile ahead (round 6)
  const int qbase = blockIdx.x * QB;
  auto load_q = [&](int qt, tx8 (&qf)[NKS]) {
    const int qr = qbase + qt * 16 + c;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 32 * ks + 8 * g;
      if (qt < QB / 16 && qr < Nq && d0 < hd) {
        qf[ks] = *reinterpret_cast<const tx8*>(Qb + (long)qr * ldq + d0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[ks][j] = zero;
      }
    }
  };
  // stage K [key][d] and V^T [d][key] for all keys (zeros past Nk / hd); with several key chunks (round 6) every
  // thread's K / V pieces are loaded before the first LDS write and each wave's Q tile one tile ahead (at one chunk
  // the extra registers cost more than the overlap gains: 22.6 -> 24.1 us at 196 x 49, profiles/r06/attn_twopass.txt)
  constexpr bool PF = NKC > 1;
  if constexpr (!PF) {
    for (int e = tid; e < NKP * (HDP / 8); e += 256) {
      const int key = e / (HDP / 8), d0 = (e % (HDP / 8)) * 8;
      tx8 kv, vv;
      if (key < Nk && d0 < hd) {
        kv = *reinterpret_cast<const tx8*>(Kb + (long)key * ldk + d0);
        vv = *reinterpret_cast<const tx8*>(Vb + (long)key * ldv + d0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kv[j] = zero; vv[j] = zero; }
      }
      *reinterpret_cast<tx8*>(&sK[key][d0]) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) sVt[d0 + j][key] = vv[j];
    }
  } else {
    constexpr int NST = NKP * (HDP / 8) / 256;
    static_assert(NKP * (HDP / 8) % 256 == 0, "whole staging rounds");
    tx8 kv[NST], vv[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int e = tid + 256 * i, key = e / (HDP / 8), d0 = (e % (HDP / 8)) * 8;
      if (key < Nk && d0 < hd) {
        kv[i] = *reinterpret_cast<const tx8*>(Kb + (long)key * ldk + d0);
        vv[i] = *reinterpret_cast<const tx8*>(Vb + (long)key * ldv + d0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kv[i][j] = zero; vv[i][j] = zero; }
      }
    }
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int e = tid + 256 * i, key = e / (HDP / 8), d0 = (e % (HDP / 8)) * 8;
      *reinterpret_cast<tx8*>(&sK[key][d0]) = kv[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) sVt[d0 + j][key] = vv[i][j];
    }
  }
  tx8 qf[NKS];
  if constexpr (PF) load_q(wave, qf);
  __syncthreads();

  for (int qt = wave; qt < QB / 16; qt += 4) {
    const int q0 = qbase + qt * 16;
    if (q0 >= Nq) break;
    tx8 qn[NKS];
    if constexpr (PF) load_q(qt + 4, qn);
    else load_q(qt, qf);
    f32x4 o[NDT];
    float l_run;
    if constexpr (PF) {
    // all keys are resident, so the softmax takes two passes over registers instead of an online rescale per key
    // chunk (round 6: the rescale, the per-chunk max / sum shuffles and the key mask of every chunk were most of the
    // 4.6 k VALU instructions per wave at 196 keys; only the last chunk can hold padded keys, 64 (NKC - 1) < Nk)
    f32x4 s[NKC][4];
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[ch][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const tx8 a = *reinterpret_cast<const tx8*>(&sK[ch * KC + 16 * t + c][32 * ks + 8 * g]);
          s[ch][t] = mfma16x16x32(a, qf[ks], s[ch][t]);
        }
      }
    float mx = -INFINITY;
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ch < NKC - 1 || ch * KC + 16 * t + 4 * g + r < Nk) mx = fmaxf(mx, s[ch][t][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mb = mx * scale_log2;
    l_run = 0.f;
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool real = ch < NKC - 1 || ch * KC + 16 * t + 4 * g + r < Nk;
          const float p = real ? exp2f(fmaf(s[ch][t][r], scale_log2, -mb)) : 0.f;
          s[ch][t][r] = p;
          l_run += p;
        }
    l_run += __shfl_xor(l_run, 16, 64);
    l_run += __shfl_xor(l_run, 32, 64);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch) {
      const int kc0 = ch * KC;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        tx8 pa;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = (T)s[ch][2 * s2][j];
          pa[4 + j] = (T)s[ch][2 * s2 + 1][j];
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const tx4 v0 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][kc0 + 32 * s2 + 4 * g]);
          const tx4 v1 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][kc0 + 32 * s2 + 16 + 4 * g]);
          tx8 vb;
#pragma unroll
          for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
          o[dt] = mfma16x16x32(pa, vb, o[dt]);
        }
      }
    }
    } else {   // one key chunk: the round-5 online form (one pass)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY;
    l_run = 0.f;
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch) {
      const int kc0 = ch * KC;
      f32x4 s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const tx8 a = *reinterpret_cast<const tx8*>(&sK[kc0 + 16 * t + c][32 * ks + 8 * g]);
          s[t] = mfma16x16x32(a, qf[ks], s[t]);
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kc0 + 16 * t + 4 * g + r;
          const float v = key < Nk ? s[t][r] * scale_log2 : -INFINITY;
          s[t][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = exp2f(m_run - m_new);
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[t][r] - m_new);
          s[t][r] = p;
          ps += p;
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l_run = l_run * alpha + ps;
      m_run = m_new;
      if (ch > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) o[dt][r] *= ar;
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        tx8 pa;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = (T)s[2 * s2][j];
          pa[4 + j] = (T)s[2 * s2 + 1][j];
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const tx4 v0 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][kc0 + 32 * s2 + 4 * g]);
          const tx4 v1 = *reinterpret_cast<const tx4*>(&sVt[16 * dt + c][kc0 + 32 * s2 + 16 + 4 * g]);
          tx8 vb;
#pragma unroll
          for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
          o[dt] = mfma16x16x32(pa, vb, o[dt]);
        }
      }
    }
    }
    // normalise; stage the 16 x hd tile in this wave's LDS patch; 16-byte row pieces out
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float inv = 1.0f / __shfl(l_run, 4 * g + r, 64);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) sO[wave][4 * g + r][16 * dt + c] = (T)(o[dt][r] * inv);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int cpr = hd >> 3;   // 16-byte pieces per row (hd % 8 == 0)
    for (int e = lane; e < 16 * cpr; e += 64) {
      const int row = e / cpr, cc = e - row * cpr;
      const int q = q0 + row;
      if (q < Nq) *reinterpret_cast<uint4*>(Ob + (long)q * ldo + cc * 8) = *reinterpret_cast<const uint4*>(&sO[wave][row][cc * 8]);
    }
    __builtin_amdgcn_wave_barrier();   // the patch is rewritten by this wave's next tile
    if constexpr (PF) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) qf[ks] = qn[ks];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// f32 MFMA attention (v_mfma_f32_16x16x4_f32: f32 operands, exact f32 products, f32 accumulation —
// the parity path of generate_evp_LFB.py's fp32 extraction).  Same structure as the resident-K/V
// 16-bit kernel: the whole K and V of one (batch, head) are staged in LDS (f32, row-major, rows
// padded by 4 floats so the fragment reads of keys 4 apart fall in different banks) once per
// workgroup of 256 queries; each wave walks 16-query tiles.
//   S^T = K . Q^T   A = K rows (lane: key 16t + (lane & 15)), B = the wave's Q rows held in registers;
//                   the reduction index d is assigned d = (HDP / 4) g + ks to lane group g = lane >> 4
//                   (any bijection works when A and B agree), so a lane's 16 K values per key tile are
//                   CONTIGUOUS: 16-byte LDS reads, and its Q fragment is HDP / 4 consecutive floats.
//   C layout: lane column (lane & 15) = query, rows 4g + r = keys -> softmax in registers + 2 shuffles.
//   O = P . V       k-step (t, r) covers keys {16t + 4g + r : g < 4}: lane group g supplies exactly the
//                   P value it holds, and B = V[16t + 4g + r][16 dt + (lane & 15)].
template <int HDP, int NKC>
__global__ __launch_bounds__(256) void attention_mfma_f32(const float* __restrict__ Q, long ldq, long sbq,
                                                          const float* __restrict__ K, long ldk, long sbk,
                                                          const float* __restrict__ V, long ldv, long sbv,
                                                          float* __restrict__ O, long ldo, long sbo, int Nq, int Nk,
                                                          int hd, float scale_log2) {
  constexpr int KC = 64, NKP = NKC * KC, LDR = HDP + 4, QD = HDP / 4, NDT = HDP / 16, QB = 256;
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* sK = smf;                  // [NKP][LDR]
  float* sV = smf + NKP * LDR;      // [NKP][LDR]
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const float* Qb = Q + (long)b * sbq + (long)h * hd;
  const float* Kb = K + (long)b * sbk + (long)h * hd;
  const float* Vb = V + (long)b * sbv + (long)h * hd;
  float* Ob = O + (long)b * sbo + (long)h * hd;

  for (int e = tid; e < NKP * HDP; e += 256) {
    const int key = e / HDP, d = e - key * HDP;
    const bool ok = key < Nk && d < hd;
    sK[key * LDR + d] = ok ? Kb[(long)key * ldk + d] : 0.f;
    sV[key * LDR + d] = ok ? Vb[(long)key * ldv + d] : 0.f;
  }
  __syncthreads();

  const int qbase = blockIdx.x * QB;
  for (int qt = wave; qt < QB / 16; qt += 4) {
    const int q0 = qbase + qt * 16;
    if (q0 >= Nq) break;
    float qf[QD];
    {
      const int qr = q0 + c;
      const float* qp = Qb + (long)(qr < Nq ? qr : 0) * ldq;
#pragma unroll
      for (int ks = 0; ks < QD; ++ks) {
        const int d = QD * g + ks;
        qf[ks] = (qr < Nq && d < hd) ? qp[d] : 0.f;
      }
    }
    f32x4 o[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
#pragma unroll
    for (int ch = 0; ch < NKC; ++ch) {
      const int kc0 = ch * KC;
      f32x4 s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* kr = sK + (kc0 + 16 * t + c) * LDR + QD * g;
#pragma unroll
        for (int k4 = 0; k4 < QD / 4; ++k4) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(kr + 4 * k4);
#pragma unroll
          for (int j = 0; j < 4; ++j) s[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], qf[4 * k4 + j], s[t], 0, 0, 0);
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kc0 + 16 * t + 4 * g + r;
          const float v = key < Nk ? s[t][r] * scale_log2 : -INFINITY;
          s[t][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = exp2f(m_run - m_new);
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[t][r] - m_new);
          s[t][r] = p;
          ps += p;
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l_run = l_run * alpha + ps;
      m_run = m_new;
      if (ch > 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) o[dt][r] *= ar;
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* vr = sV + (kc0 + 16 * t + 4 * g + r) * LDR + c;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(s[t][r], vr[16 * dt], o[dt], 0, 0, 0);
        }
    }
    // lane holds O[query q0 + 4g + r][16 dt + c]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + 4 * g + r;
      const float inv = 1.0f / __shfl(l_run, 4 * g + r, 64);
      if (q < Nq) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int d = 16 * dt + c;
          if (d < hd) Ob[(long)q * ldo + d] = o[dt][r] * inv;
        }
      }
    }
  }
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
  if (dtype == SVK_BF16 || dtype == SVK_F16) {
    const float sl2 = scale * 1.4426950408889634f;   // softmax via exp2
    const bool res_ok = hd % 8 == 0 && ((ldq | ldk | ldv | ldo | sbq | sbk | sbv | sbo) % 8) == 0 &&
                        ((((uintptr_t)Q) | ((uintptr_t)K) | ((uintptr_t)V) | ((uintptr_t)O)) & 15) == 0;
    SVK_DISPATCH_H16(dtype, T, {
      if (res_ok) {
        const int nkc = (Nk + 63) / 64;
        // query block 256; SVK_ATTN_QB=64 selects 64-query blocks (read at every call; measured slower, see the kernel)
        const char* qbe = getenv("SVK_ATTN_QB");
        const int qb = qbe && atoi(qbe) == 64 ? 64 : 256;
        dim3 rgrid((Nq + qb - 1) / qb, heads, B);
        auto go = [&](auto hdp_c, auto nkc_c) {
          constexpr int HDP = decltype(hdp_c)::value, NKC = decltype(nkc_c)::value;
          if (qb == 64)
            hipLaunchKernelGGL((attention_mfma_bf16_res<T, HDP, NKC, 64>), rgrid, block, 0, st, (const T*)Q, ldq, sbq,
                               (const T*)K, ldk, sbk, (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, sl2);
          else
            hipLaunchKernelGGL((attention_mfma_bf16_res<T, HDP, NKC>), rgrid, block, 0, st, (const T*)Q, ldq, sbq,
                               (const T*)K, ldk, sbk, (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, sl2);
        };
        auto by_nkc = [&](auto hdp) {
          switch (nkc) {
            case 1: go(hdp, std::integral_constant<int, 1>{}); break;
            case 2: go(hdp, std::integral_constant<int, 2>{}); break;
            case 3: go(hdp, std::integral_constant<int, 3>{}); break;
            default: go(hdp, std::integral_constant<int, 4>{}); break;
          }
        };
        if (hd <= 32) by_nkc(std::integral_constant<int, 32>{});
        else by_nkc(std::integral_constant<int, 64>{});
        return check_launch("attention_mfma_bf16_res");
      }
      if (hd <= 32)
        hipLaunchKernelGGL((attention_mfma_bf16<T, 32>), grid, block, 0, st, (const T*)Q, ldq, sbq, (const T*)K, ldk,
                           sbk, (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, sl2);
      else
        hipLaunchKernelGGL((attention_mfma_bf16<T, 64>), grid, block, 0, st, (const T*)Q, ldq, sbq, (const T*)K, ldk,
                           sbk, (const T*)V, ldv, sbv, (T*)O, ldo, sbo, Nq, Nk, hd, sl2);
      return check_launch("attention_mfma_bf16");
    });
  }
  static const bool f32_scalar = getenv("SVK_ATTN_F32_SCALAR") != nullptr;   // the exact scalar kernel (A/B checks)
  if (dtype == SVK_F32 && !f32_scalar) {
    const int nkc = (Nk + 63) / 64;
    dim3 rgrid((Nq + 255) / 256, heads, B);
    auto go = [&](auto hdp_c, auto nkc_c) {
      constexpr int HDP = decltype(hdp_c)::value, NKC = decltype(nkc_c)::value;
      constexpr int sm = 2 * NKC * 64 * (HDP + 4) * (int)sizeof(float);
      static bool attr = false;
      if (!attr && sm > 65536) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_mfma_f32<HDP, NKC>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr = true;
      }
      hipLaunchKernelGGL((attention_mfma_f32<HDP, NKC>), rgrid, block, sm, st, (const float*)Q, ldq, sbq,
                         (const float*)K, ldk, sbk, (const float*)V, ldv, sbv, (float*)O, ldo, sbo, Nq, Nk, hd,
                         scale * 1.4426950408889634f);
    };
    auto by_nkc = [&](auto hdp) {
      switch (nkc) {
        case 1: go(hdp, std::integral_constant<int, 1>{}); break;
        case 2: go(hdp, std::integral_constant<int, 2>{}); break;
        case 3: go(hdp, std::integral_constant<int, 3>{}); break;
        default: go(hdp, std::integral_constant<int, 4>{}); break;
      }
    };
    if (hd <= 32) by_nkc(std::integral_constant<int, 32>{});
    else by_nkc(std::integral_constant<int, 64>{});
    return check_launch("attention_mfma_f32");
  }
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

// ---- attention backward ------------------------------------------------------------------------
// One workgroup per (frame, head, QB queries).  K, V (Nk x hd), the QB query rows and their output
// gradients are staged in LDS as f32; P = softmax(scale Q K^T) is recomputed, then
//   dP = dO V^T,  dS = P * (dP - rowsum(dO * O)),  dQ = scale dS K   (written directly, T)
//   dK += scale dS^T Q,  dV += P^T dO                                   (f32 atomics, zeroed by caller)
// The key/value gradients are partial sums over this workgroup's queries.  All contractions are
// LDS-resident scalar FMAs (Nk <= 196 at the model's shapes; an MFMA version is future work).
namespace svk {
template <typename T>
__global__ __launch_bounds__(256) void attention_bwd_kernel(const T* __restrict__ Q, long ldq, long sbq,
                                                            const T* __restrict__ K, long ldk, long sbk,
                                                            const T* __restrict__ V, long ldv, long sbv,
                                                            const T* __restrict__ O, long ldo, long sbo,
                                                            const T* __restrict__ dO, long lddo, long sbdo,
                                                            T* __restrict__ dQ, long lddq, long sbdq,
                                                            float* __restrict__ dK, float* __restrict__ dV, long lddk,
                                                            long sbdk, int Nq, int Nk, int hd, int QB, float scale) {
  extern __shared__ float sm[];
  const int hp = hd + 1, kp = Nk + 1;
  float* sK = sm;
  float* sV = sK + Nk * hp;
  float* sQ = sV + Nk * hp;
  float* sdO = sQ + QB * hp;
  float* sP = sdO + QB * hp;
  float* sdS = sP + QB * kp;
  float* sD = sdS + QB * kp;
  const int tid = threadIdx.x;
  const int q0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
  const long co = (long)h * hd;
  const T* Kb = K + b * sbk + co;
  const T* Vb = V + b * sbv + co;
  for (int idx = tid; idx < Nk * hd; idx += 256) {
    const int j = idx / hd, d = idx - j * hd;
    sK[j * hp + d] = to_f(Kb[(long)j * ldk + d]);
    sV[j * hp + d] = to_f(Vb[(long)j * ldv + d]);
  }
  for (int idx = tid; idx < QB * hd; idx += 256) {
    const int q = idx / hd, d = idx - q * hd;
    const bool ok = q0 + q < Nq;
    sQ[q * hp + d] = ok ? to_f(Q[b * sbq + (long)(q0 + q) * ldq + co + d]) : 0.f;
    sdO[q * hp + d] = ok ? to_f(dO[b * sbdo + (long)(q0 + q) * lddo + co + d]) : 0.f;
  }
  if (tid < QB) {
    float acc = 0.f;
    if (q0 + tid < Nq) {
      const T* o = O + b * sbo + (long)(q0 + tid) * ldo + co;
      const T* g = dO + b * sbdo + (long)(q0 + tid) * lddo + co;
      for (int d = 0; d < hd; ++d) acc += to_f(o[d]) * to_f(g[d]);
    }
    sD[tid] = acc;
  }
  __syncthreads();
  for (int idx = tid; idx < QB * Nk; idx += 256) {
    const int q = idx / Nk, j = idx - q * Nk;
    float s = 0.f;
    for (int d = 0; d < hd; ++d) s += sQ[q * hp + d] * sK[j * hp + d];
    sP[q * kp + j] = s * scale;
  }
  __syncthreads();
  // row softmax: 4 lanes per row
  {
    const int q = tid >> 2, sub = tid & 3;
    if (q < QB) {
      float m = -INFINITY;
      for (int j = sub; j < Nk; j += 4) m = fmaxf(m, sP[q * kp + j]);
      m = fmaxf(m, __shfl_xor(m, 1, 64));
      m = fmaxf(m, __shfl_xor(m, 2, 64));
      float l = 0.f;
      for (int j = sub; j < Nk; j += 4) l += __expf(sP[q * kp + j] - m);
      l += __shfl_xor(l, 1, 64);
      l += __shfl_xor(l, 2, 64);
      const float inv = (q0 + q < Nq) ? 1.f / l : 0.f;
      for (int j = sub; j < Nk; j += 4) sP[q * kp + j] = __expf(sP[q * kp + j] - m) * inv;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < QB * Nk; idx += 256) {
    const int q = idx / Nk, j = idx - q * Nk;
    float dp = 0.f;
    for (int d = 0; d < hd; ++d) dp += sdO[q * hp + d] * sV[j * hp + d];
    sdS[q * kp + j] = sP[q * kp + j] * (dp - sD[q]);
  }
  __syncthreads();
  for (int idx = tid; idx < QB * hd; idx += 256) {
    const int q = idx / hd, d = idx - q * hd;
    if (q0 + q >= Nq) continue;
    float a = 0.f;
    for (int j = 0; j < Nk; ++j) a += sdS[q * kp + j] * sK[j * hp + d];
    dQ[b * sbdq + (long)(q0 + q) * lddq + co + d] = from_f<T>(a * scale);
  }
  const int qn = min(QB, Nq - q0);
  for (int idx = tid; idx < Nk * hd; idx += 256) {
    const int j = idx / hd, d = idx - j * hd;
    float ak = 0.f, av = 0.f;
    for (int q = 0; q < qn; ++q) {
      ak += sdS[q * kp + j] * sQ[q * hp + d];
      av += sP[q * kp + j] * sdO[q * hp + d];
    }
    atomicAdd(dK + b * sbdk + (long)j * lddk + co + d, ak * scale);
    atomicAdd(dV + b * sbdk + (long)j * lddk + co + d, av);
  }
}
}  // namespace svk


// ---- MFMA attention backward (bf16): dQ, and P / dS for the key/value reductions ----------------
// One workgroup per (frame, head, 64 queries); wave w owns queries q0 + 16w .. +15.  Keys are padded
// to NKC x 64 (masked).  Per wave, with 16x16x32 bf16 MFMAs (C layout: col = key (lane & 15),
// row = query 4 (lane >> 4) + r):
//   S = Q K^T, dP = dO V^T (K, V staged in LDS [key][d]); row max / sum over keys by 16-lane
//   xor-shuffles; P = softmax(scale S); dS' = scale P (dP - D), D = rowsum(dO * O);
//   dQ = dS' K  (dS' goes through LDS once to become an A operand; K^T staged in LDS).
// P and dS' are written (bf16, rows padded to NKC x 64 with zeros) to the workspace; dK = dS'^T Q
// and dV = P^T dO are then batched MFMA reductions over the queries (wgrad_batched).
namespace svk {
template <int HDP, int NKC>
__global__ __launch_bounds__(256) void attn_bwd_dq_mfma(const bf16* __restrict__ Q, long ldq, long sbq,
                                                        const bf16* __restrict__ K, long ldk, long sbk,
                                                        const bf16* __restrict__ V, long ldv, long sbv,
                                                        const bf16* __restrict__ O, long ldo, long sbo,
                                                        const bf16* __restrict__ dO, long lddo, long sbdo,
                                                        bf16* __restrict__ dQ, long lddq, long sbdq,
                                                        bf16* __restrict__ Pws, bf16* __restrict__ dSws, int Nq,
                                                        int Nk, int hd, float scale, float4* __restrict__ zacc,
                                                        long nzacc) {
  constexpr int NKP = NKC * 64;
  // zero the dK / dV f32 accumulators the two batched reductions after this kernel add into (round 6: replaces
  // a hipMemsetAsync — one runtime fill launch per attention backward): workgroup slices of nzacc float4
  {
    const long nwg = (long)gridDim.x * gridDim.y * gridDim.z;
    const long wg = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
    const long per = (nzacc + nwg - 1) / nwg, z0 = wg * per, z1 = z0 + per < nzacc ? z0 + per : nzacc;
    for (long i = z0 + threadIdx.x; i < z1; i += 256) zacc[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int LDK = HDP + 8;
  constexpr int LDT = NKP + 8;
  __shared__ __attribute__((aligned(16))) bf16 sK[NKP][LDK];
  __shared__ __attribute__((aligned(16))) bf16 sV[NKP][LDK];
  __shared__ __attribute__((aligned(16))) bf16 sKt[HDP][LDT];
  __shared__ __attribute__((aligned(16))) bf16 sdS[4][16][LDT];
  __shared__ float sD[64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z, heads = gridDim.y;
  const long co = (long)h * hd;
  const bf16 zero = (bf16)0.f;
  // stage K, V, K^T (zero past Nk / hd)
  constexpr int CPR = HDP / 8;
  for (int idx = tid; idx < NKP * CPR; idx += 256) {
    const int key = idx / CPR, c8 = (idx - key * CPR) * 8;
    bf16x8 kv, vv;
    if (key < Nk && c8 < hd) {
      kv = *reinterpret_cast<const bf16x8*>(K + b * sbk + (long)key * ldk + co + c8);
      vv = *reinterpret_cast<const bf16x8*>(V + b * sbv + (long)key * ldv + co + c8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { kv[e] = zero; vv[e] = zero; }
    }
    *reinterpret_cast<bf16x8*>(&sK[key][c8]) = kv;
    *reinterpret_cast<bf16x8*>(&sV[key][c8]) = vv;
#pragma unroll
    for (int e = 0; e < 8; ++e) sKt[c8 + e][key] = kv[e];
  }
  if (tid < 64) {
    const int q = q0 + tid;
    float acc = 0.f;
    if (q < Nq) {
      const bf16* o = O + b * sbo + (long)q * ldo + co;
      const bf16* g = dO + b * sbdo + (long)q * lddo + co;
      for (int d = 0; d < hd; d += 8) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + d);
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + d);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += (float)ov[e] * (float)gv[e];
      }
    }
    sD[tid] = acc;
  }
  // A operands: Q and dO rows of this wave (row = lane & 15, k = 8 (lane >> 4) + j per 32-wide step)
  const int fr = lane & 15, fg = lane >> 4;
  const int qa = q0 + w * 16 + fr;
  bf16x8 aq[HDP / 32], ag[HDP / 32];
#pragma unroll
  for (int ks = 0; ks < HDP / 32; ++ks) {
    const int c = ks * 32 + fg * 8;
    if (qa < Nq && c < hd) {
      aq[ks] = *reinterpret_cast<const bf16x8*>(Q + b * sbq + (long)qa * ldq + co + c);
      ag[ks] = *reinterpret_cast<const bf16x8*>(dO + b * sbdo + (long)qa * lddo + co + c);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { aq[ks][e] = zero; ag[ks][e] = zero; }
    }
  }
  __syncthreads();
  f32x4 S[NKC * 4], dP[NKC * 4];
#pragma unroll
  for (int t = 0; t < NKC * 4; ++t) {
    S[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    dP[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HDP / 32; ++ks) {
      const bf16x8 bk = *reinterpret_cast<const bf16x8*>(&sK[t * 16 + fr][ks * 32 + fg * 8]);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&sV[t * 16 + fr][ks * 32 + fg * 8]);
      S[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[ks], bk, S[t], 0, 0, 0);
      dP[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ag[ks], bv, dP[t], 0, 0, 0);
    }
  }
  // softmax over keys for the 4 query rows this lane holds
  const float sl2 = scale * 1.4426950408889634f;
  float mx[4], inv[4], Dq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NKC * 4; ++t) {
      const int key = t * 16 + fr;
      if (key < Nk) m = fmaxf(m, S[t][r]);
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < NKC * 4; ++t) {
      const int key = t * 16 + fr;
      const float p = key < Nk ? exp2f((S[t][r] - m) * sl2) : 0.f;
      S[t][r] = p;
      l += p;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) l += __shfl_xor(l, o, 64);
    mx[r] = m;
    inv[r] = 1.f / l;
    Dq[r] = sD[w * 16 + fg * 4 + r];
  }
  (void)mx;
  // P, dS' -> workspace (rows of this wave) and dS' -> LDS
  const long zrow = ((long)b * heads + h) * Nq;
#pragma unroll
  for (int t = 0; t < NKC * 4; ++t) {
    const int key = t * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qr = w * 16 + fg * 4 + r;
      const float p = S[t][r] * inv[r];
      const float ds = scale * p * (dP[t][r] - Dq[r]);
      const bf16 dsb = (bf16)ds;
      sdS[w][fg * 4 + r][key] = dsb;
      if (q0 + qr < Nq) {
        const long off = (zrow + q0 + qr) * NKP + key;
        Pws[off] = (bf16)p;
        dSws[off] = dsb;
      }
    }
  }
  __syncthreads();
  // dQ = dS' K: A = dS' rows (LDS), B = K (k = keys, n = d) from sKt
#pragma unroll
  for (int nt = 0; nt < HDP / 16; ++nt) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < NKP / 32; ++kk) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sdS[w][fr][kk * 32 + fg * 8]);
      const bf16x8 bb = *reinterpret_cast<const bf16x8*>(&sKt[nt * 16 + fr][kk * 32 + fg * 8]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc, 0, 0, 0);
    }
    const int d = nt * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + w * 16 + fg * 4 + r;
      if (q < Nq && d < hd) dQ[b * sbdq + (long)q * lddq + co + d] = (bf16)acc[r];
    }
  }
}

// ---- MFMA attention backward with transposed scores (round 6): same outputs as attn_bwd_dq_mfma ----------------
// The scores are computed transposed, S^T = K Q^T and dP^T = V dO^T (A = K / V rows, B = the wave's Q / dO rows
// held in registers; K and V are staged once per workgroup in LDS, row-major), so a lane's accumulator column is ONE
// query (lane & 15) and its rows are the keys 16 t + 4 g + r (g = lane >> 4).  Then
//   * the softmax and D = rowsum(dO * O) reduce in registers plus two shuffles (no LDS, no 64-lane serial loop);
//   * P^T / dS'^T leave as 8-byte pieces (4 consecutive keys of one query) instead of 2-byte stores;
//   * dQ^T = K^T dS'^T takes dS'^T from registers as the B operand, keys permuted {32 s + 4 g + j} ++
//     {32 s + 16 + 4 g + j} as in the forward's P.V, A = K^T gathered from sK: no dS' LDS round trip, no K^T copy.
// LDS is K and V only: 18 KB at NKC = 1, 74 KB at NKC = 4 (the 196-token cross-attention), where the previous kernel
// needed 141 KB and ran one workgroup per CU.  (A first version read the K / V A operands straight from global
// memory, every wave the whole K and V: 0.74 GB of L2 requests at NKC = 4, 41 % missing — slower at <= 64 keys.)
template <int HDP, int NKC>
__global__ __launch_bounds__(256) void attn_bwd_dq_t(const bf16* __restrict__ Q, long ldq, long sbq,
                                                     const bf16* __restrict__ K, long ldk, long sbk,
                                                     const bf16* __restrict__ V, long ldv, long sbv,
                                                     const bf16* __restrict__ O, long ldo, long sbo,
                                                     const bf16* __restrict__ dO, long lddo, long sbdo,
                                                     bf16* __restrict__ dQ, long lddq, long sbdq,
                                                     bf16* __restrict__ Pws, bf16* __restrict__ dSws, int Nq,
                                                     int Nk, int hd, float scale, float4* __restrict__ zacc,
                                                     long nzacc) {
  constexpr int NKP = NKC * 64, NKS = HDP / 32, NDT = HDP / 16, NT = NKC * 4;
  {   // zero this workgroup's slice of the dK / dV accumulators (as attn_bwd_dq_mfma)
    const long nwg = (long)gridDim.x * gridDim.y * gridDim.z;
    const long wg = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
    const long per = (nzacc + nwg - 1) / nwg, z0 = wg * per, z1 = z0 + per < nzacc ? z0 + per : nzacc;
    for (long i = z0 + threadIdx.x; i < z1; i += 256) zacc[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int LDK = HDP + 8;
  __shared__ __attribute__((aligned(16))) bf16 sK[NKP][LDK];
  __shared__ __attribute__((aligned(16))) bf16 sV[NKP][LDK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int q0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z, heads = gridDim.y;
  const long co = (long)h * hd;
  const bf16* Kb = K + b * sbk + co;
  const bf16* Vb = V + b * sbv + co;
  const bf16 zero = (bf16)0.f;
  // K, V [key][d] (zeros past Nk / hd), 16-byte pieces
  for (int idx = tid; idx < NKP * (HDP / 8); idx += 256) {
    const int key = idx / (HDP / 8), c8 = (idx % (HDP / 8)) * 8;
    bf16x8 kv, vv;
    if (key < Nk && c8 < hd) {
      kv = *reinterpret_cast<const bf16x8*>(Kb + (long)key * ldk + c8);
      vv = *reinterpret_cast<const bf16x8*>(Vb + (long)key * ldv + c8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { kv[e] = zero; vv[e] = zero; }
    }
    *reinterpret_cast<bf16x8*>(&sK[key][c8]) = kv;
    *reinterpret_cast<bf16x8*>(&sV[key][c8]) = vv;
  }
  // B operands: this lane's query row of Q and dO (k = d = 32 ks + 8 g + j); D = rowsum(dO * O) from the same pieces
  const int qn = q0 + 16 * w + c;
  const bool qok = qn < Nq;
  bf16x8 bq[NKS], bg[NKS];
  float D = 0.f;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int d0 = 32 * ks + 8 * g;
    if (qok && d0 < hd) {
      bq[ks] = *reinterpret_cast<const bf16x8*>(Q + b * sbq + (long)qn * ldq + co + d0);
      bg[ks] = *reinterpret_cast<const bf16x8*>(dO + b * sbdo + (long)qn * lddo + co + d0);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(O + b * sbo + (long)qn * ldo + co + d0);
#pragma unroll
      for (int e = 0; e < 8; ++e) D += (float)ov[e] * (float)bg[ks][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { bq[ks][e] = zero; bg[ks][e] = zero; }
    }
  }
  D += __shfl_xor(D, 16, 64);
  D += __shfl_xor(D, 32, 64);
  __syncthreads();   // K, V staged
  // S^T, dP^T: A = K / V rows from LDS (key 16 t + c, k = d = 32 ks + 8 g + j)
  f32x4 S[NT], dP[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    S[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    dP[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 ka = *reinterpret_cast<const bf16x8*>(&sK[16 * t + c][32 * ks + 8 * g]);
      const bf16x8 va = *reinterpret_cast<const bf16x8*>(&sV[16 * t + c][32 * ks + 8 * g]);
      S[t] = mfma16x16x32(ka, bq[ks], S[t]);
      dP[t] = mfma16x16x32(va, bg[ks], dP[t]);
    }
  }
  // softmax over keys for this lane's query: in-register over (t, r), then across the 4 lane groups
  const float sl2 = scale * 1.4426950408889634f;
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (16 * t + 4 * g + r < Nk) m = fmaxf(m, S[t][r]);
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = 16 * t + 4 * g + r < Nk ? exp2f((S[t][r] - m) * sl2) : 0.f;
      S[t][r] = p;
      l += p;
    }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  // P^T, dS'^T -> workspace rows [z][query][NKP] (8-byte pieces; padded keys get p = dS' = 0); dS' kept as bf16
  bf16x4 ds4[NT];
  bf16* Prow = Pws + (((long)b * heads + h) * Nq + qn) * NKP;
  bf16* dSrow = dSws + (((long)b * heads + h) * Nq + qn) * NKP;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bf16x4 p4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = S[t][r] * inv;
      p4[r] = (bf16)p;
      ds4[t][r] = (bf16)(scale * p * (dP[t][r] - D));
    }
    if (qok) {
      *reinterpret_cast<bf16x4*>(Prow + 16 * t + 4 * g) = p4;
      *reinterpret_cast<bf16x4*>(dSrow + 16 * t + 4 * g) = ds4[t];
    }
  }
  // dQ^T = K^T dS'^T: k-step s covers keys {32 s + 4 g + j} ++ {32 s + 16 + 4 g + j} (tiles 2 s, 2 s + 1); the A
  // operand (row d = 16 dt + c) gathers K^T from the row-major sK with 2-byte reads (16 lanes read 16 consecutive d
  // of one key row; the 4 lane groups' rows sit 16 banks apart: conflict-free)
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NT / 2; ++s) {
      bf16x8 a, bb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = sK[32 * s + 4 * g + j][16 * dt + c];
        a[4 + j] = sK[32 * s + 16 + 4 * g + j][16 * dt + c];
        bb[j] = ds4[2 * s][j]; bb[4 + j] = ds4[2 * s + 1][j];
      }
      acc = mfma16x16x32(a, bb, acc);
    }
    // C: rows d = 16 dt + 4 g + r, column = this lane's query -> 4 consecutive d (hd % 8 == 0)
    const int d = 16 * dt + 4 * g;
    if (qok && d < hd) {
      bf16x4 o4;
#pragma unroll
      for (int r = 0; r < 4; ++r) o4[r] = (bf16)acc[r];
      *reinterpret_cast<bf16x4*>(dQ + b * sbdq + (long)qn * lddq + co + d) = o4;
    }
  }
}

// ---- fused MFMA attention backward (bf16, <= 64 keys): dQ and the dK / dV reductions in one kernel -------
// One workgroup per (frame, head, query range); it stages K, V, K^T in LDS once and walks its range in
// 64-query chunks (wave w: queries 16w .. 16w + 15 of the chunk).  Per chunk: S = Q K^T, dP = dO V^T,
// softmax, dS' = scale P (dP - D) as in attn_bwd_dq_mfma; then
//   dQ^T = K^T dS'^T          (A = K^T rows d from sKt, B = dS' rows from sdS: a lane ends with 4
//                              consecutive d of one query -> 8-byte stores),
//   dK^T += Q^T dS', dV^T += dO^T P   (A = the chunk's Q^T / dO^T rows d, B = dS'^T / P^T rows key, both
//                              staged transposed in LDS; the 32 16x16 output blocks split 8 per wave and
//                              accumulated in registers over all chunks of the range).
// The dK / dV partial sums reach the f32 accumulators with one atomic per element per workgroup; the
// P / dS' workspace round trip and the two batched reductions of the unfused path are gone.
template <int HDP>
__global__ __launch_bounds__(256) void attn_bwd_fused(const bf16* __restrict__ Q, long ldq, long sbq,
                                                      const bf16* __restrict__ K, long ldk, long sbk,
                                                      const bf16* __restrict__ V, long ldv, long sbv,
                                                      const bf16* __restrict__ O, long ldo, long sbo,
                                                      const bf16* __restrict__ dO, long lddo, long sbdo,
                                                      bf16* __restrict__ dQ, long lddq, long sbdq,
                                                      float* __restrict__ accK, float* __restrict__ accV, int C,
                                                      int Nq, int Nk, int hd, int nchunk, float scale) {
  constexpr int NKP = 64, LD = 72;                   // keys padded to 64; LDS rows padded by 8 (bank spread)
  __shared__ __attribute__((aligned(16))) bf16 sK[NKP][LD], sV[NKP][LD], sKt[HDP][LD];
  __shared__ __attribute__((aligned(16))) bf16 sQt[HDP][LD], sdOt[HDP][LD], sdS[64][LD], sdSt[NKP][LD], sPt[NKP][LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const long co = (long)h * hd;
  const bf16 zero = (bf16)0.f;
  constexpr int CPR = HDP / 8;
  for (int idx = tid; idx < NKP * CPR; idx += 256) {
    const int key = idx / CPR, c8 = (idx - key * CPR) * 8;
    bf16x8 kv, vv;
    if (key < Nk && c8 < hd) {
      kv = *reinterpret_cast<const bf16x8*>(K + b * sbk + (long)key * ldk + co + c8);
      vv = *reinterpret_cast<const bf16x8*>(V + b * sbv + (long)key * ldv + co + c8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { kv[e] = zero; vv[e] = zero; }
    }
    *reinterpret_cast<bf16x8*>(&sK[key][c8]) = kv;
    *reinterpret_cast<bf16x8*>(&sV[key][c8]) = vv;
#pragma unroll
    for (int e = 0; e < 8; ++e) sKt[c8 + e][key] = kv[e];
  }
  const int fr = lane & 15, fg = lane >> 4;
  // this wave's dK^T / dV^T output blocks: blk = 8 w + i -> (matrix blk / 16, d-block (blk / 4) % 4, key-block blk % 4)
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float sl2 = scale * 1.4426950408889634f;
  const int c_end = min((int)((blockIdx.x + 1) * (long)nchunk), (Nq + 63) / 64);
  // this wave's Q / dO / O rows of a chunk (row = query 16 w + (lane & 15), 8 d per lane and 32-wide step),
  // loaded one chunk ahead so their latency hides behind the current chunk's MFMAs
  bf16x8 aq[HDP / 32], ag[HDP / 32], ao[HDP / 32];
  auto load_rows = [&](int ch) __attribute__((always_inline)) {
    const int qa = ch * 64 + w * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < HDP / 32; ++ks) {
      const int c = ks * 32 + fg * 8;
      if (qa < Nq && c < hd) {
        aq[ks] = *reinterpret_cast<const bf16x8*>(Q + b * sbq + (long)qa * ldq + co + c);
        ag[ks] = *reinterpret_cast<const bf16x8*>(dO + b * sbdo + (long)qa * lddo + co + c);
        ao[ks] = *reinterpret_cast<const bf16x8*>(O + b * sbo + (long)qa * ldo + co + c);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { aq[ks][e] = zero; ag[ks][e] = zero; ao[ks][e] = zero; }
      }
    }
  };
  if (blockIdx.x * nchunk < c_end) load_rows(blockIdx.x * nchunk);
  __syncthreads();                       // sK / sV / sKt
  for (int ch = blockIdx.x * nchunk; ch < c_end; ++ch) {
    const int q0 = ch * 64;
    const int ql = w * 16 + fr, qa = q0 + ql;
    // D = rowsum(dO * O) of query fr: the 4 lanes fg hold its 4 d-slices
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < HDP / 32; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += (float)ag[ks][e] * (float)ao[ks][e];
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
#pragma unroll
    for (int ks = 0; ks < HDP / 32; ++ks) {
      const int c = ks * 32 + fg * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) { sQt[c + e][ql] = aq[ks][e]; sdOt[c + e][ql] = ag[ks][e]; }
    }
    f32x4 S[4], dP[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      S[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dP[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < HDP / 32; ++ks) {
        const bf16x8 bk = *reinterpret_cast<const bf16x8*>(&sK[t * 16 + fr][ks * 32 + fg * 8]);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&sV[t * 16 + fr][ks * 32 + fg * 8]);
        S[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[ks], bk, S[t], 0, 0, 0);
        dP[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ag[ks], bv, dP[t], 0, 0, 0);
      }
    }
    if (ch + 1 < c_end) load_rows(ch + 1);   // next chunk's rows (aq / ag are consumed)
    // softmax over keys for the 4 query rows this lane holds (row = query 4 fg + r, col = key t 16 + fr)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t * 16 + fr < Nk) m = fmaxf(m, S[t][r]);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float l = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float p = t * 16 + fr < Nk ? exp2f((S[t][r] - m) * sl2) : 0.f;
        S[t][r] = p;
        l += p;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) l += __shfl_xor(l, o, 64);
      const float inv = 1.f / l, Dq = __shfl(dsum, fg * 4 + r, 64);
      const int qr = w * 16 + fg * 4 + r;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int key = t * 16 + fr;
        const float p = S[t][r] * inv;
        const bf16 dsb = (bf16)(scale * p * (dP[t][r] - Dq));
        sdS[qr][key] = dsb;
        sdSt[key][qr] = dsb;
        sPt[key][qr] = (bf16)p;
      }
    }
    __syncthreads();                     // sdS, sdSt, sPt complete
    // dQ^T [d][q] = sum_key K^T[d][key] dS'[q][key]: this wave's 16 queries, 4 consecutive d per lane
#pragma unroll
    for (int nt = 0; nt < HDP / 16; ++nt) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKP / 32; ++kk) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(&sKt[nt * 16 + fr][kk * 32 + fg * 8]);
        const bf16x8 sb = *reinterpret_cast<const bf16x8*>(&sdS[w * 16 + fr][kk * 32 + fg * 8]);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, sb, a, 0, 0, 0);
      }
      const int d = nt * 16 + fg * 4;
      if (qa < Nq && d < hd) {
        bf16 o4[4] = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
        *reinterpret_cast<uint2*>(dQ + b * sbdq + (long)qa * lddq + co + d) = *reinterpret_cast<const uint2*>(o4);
      }
    }
    // dK^T += Q^T dS', dV^T += dO^T P over the chunk's 64 queries (k = query)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int blk = 8 * w + i, mat = blk >> 4, bd = (blk >> 2) & 3, bk = blk & 3;
      if (bd * 16 >= HDP) continue;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(mat ? &sdOt[bd * 16 + fr][ks * 32 + fg * 8]
                                                                : &sQt[bd * 16 + fr][ks * 32 + fg * 8]);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(mat ? &sPt[bk * 16 + fr][ks * 32 + fg * 8]
                                                                : &sdSt[bk * 16 + fr][ks * 32 + fg * 8]);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
      }
    }
    __syncthreads();                     // the next chunk overwrites sQt / sdOt / sdS / sdSt / sPt
  }
  // lane holds D[d = 16 bd + 4 fg + r][key = 16 bk + fr] of each block
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int blk = 8 * w + i, mat = blk >> 4, bd = (blk >> 2) & 3, bk = blk & 3;
    const int key = bk * 16 + fr;
    if (bd * 16 >= HDP || key >= Nk) continue;
    float* dst = (mat ? accV : accK) + ((long)b * Nk + key) * C + co;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = bd * 16 + fg * 4 + r;
      if (d < hd) atomicAdd(dst + d, acc[i][r]);
    }
  }
}

template <typename T>
__global__ void store_kv_kernel(const float* __restrict__ acc, T* __restrict__ dK, T* __restrict__ dV, long lddk,
                                long sbdk, int B, int Nk, int C) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * Nk * C) return;
  const int c = (int)(i % C);
  const long t = i / C;
  const int j = (int)(t % Nk);
  const int b = (int)(t / Nk);
  const long n = (long)B * Nk * C;
  dK[b * sbdk + (long)j * lddk + c] = from_f<T>(acc[i]);
  dV[b * sbdk + (long)j * lddk + c] = from_f<T>(acc[n + i]);
}
}  // namespace svk

static bool attn_bwd_mfma_ok(int dtype, int Nk, int hd) {
  return dtype == SVK_BF16 && hd % 8 == 0 && hd <= 64 && Nk <= 256;
}

static bool al16(const void* p, long ld, long sb) { return ((uintptr_t)p & 15) == 0 && ld % 8 == 0 && sb % 8 == 0; }

extern "C" long svk_attention_bwd_workspace(int dtype, int B, int Nq, int Nk, int heads, int hd) {
  const long acc = 2L * B * Nk * heads * hd * 4;
  if (!attn_bwd_mfma_ok(dtype, Nk, hd)) return acc;
  const long nkp = (Nk + 63) / 64 * 64;
  return acc + 2L * B * heads * Nq * nkp * 2;
}

extern "C" int svk_attention_bwd(int dtype, const void* Q, long ldq, long sbq, const void* K, long ldk, long sbk,
                                 const void* V, long ldv, long sbv, const void* O, long ldo, long sbo,
                                 const void* dO, long lddo, long sbdo, void* dQ, long lddq, long sbdq, void* dK,
                                 void* dV, long lddk, long sbdk, void* ws, long ws_bytes, int B, int Nq, int Nk,
                                 int heads, int hd, float scale, void* stream) {
  if (B < 0 || Nq < 0 || Nk <= 0 || heads <= 0 || hd <= 0 || hd > 64 || !Q || !K || !V || !O || !dO || !dQ || !dK ||
      !dV || !ws) {
    set_error("svk_attention_bwd: bad args"); return SVK_EINVAL;
  }
  if (B == 0 || Nq == 0) return SVK_OK;
  if (ws_bytes < svk_attention_bwd_workspace(dtype, B, Nq, Nk, heads, hd)) {
    set_error("svk_attention_bwd: workspace too small"); return SVK_EINVAL;
  }
  if (B > 65535 || heads > 65535) { set_error("svk_attention_bwd: grid too large"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  const int C = heads * hd;
  float* acc = static_cast<float*>(ws);                 // [2][B][Nk][C] f32: dK | dV accumulators
  const long nacc = (long)B * Nk * C;
  const bool vec_ok = al16(Q, ldq, sbq) && al16(K, ldk, sbk) && al16(V, ldv, sbv) && al16(O, ldo, sbo) &&
                      al16(dO, lddo, sbdo) && al16(dQ, lddq, sbdq);
  // the MFMA path's dQ kernel zeroes the accumulators itself (16-byte chunks: 2 nacc % 4 == 0 for C % 2 == 0 and
  // a 16-byte aligned workspace); every other path starts from a memset
  const bool zero_in_dq = attn_bwd_mfma_ok(dtype, Nk, hd) && vec_ok && !(getenv("SVK_ATTN_BWD_FUSED") &&
                          getenv("SVK_ATTN_BWD_FUSED")[0] == '1' && Nk <= 64) && (2 * nacc) % 4 == 0 &&
                          ((uintptr_t)acc & 15) == 0;
  if (!zero_in_dq && hipMemsetAsync(acc, 0, 2 * nacc * sizeof(float), st) != hipSuccess) {
    set_error("svk_attention_bwd: memset"); return SVK_ELAUNCH;
  }
  // fused path (opt-in, SVK_ATTN_BWD_FUSED=1): measured 0.35 ms per train step SLOWER than the dQ kernel +
  // two batched reductions below (5 135 vs 5 240 frames/s, same box): its workgroups walk their query
  // chunks serially behind three barriers each, while the unfused dQ kernel's one-chunk workgroups overlap
  // freely.  Kept (and tested) as the starting point for a pipelined version.
  const char* fz = getenv("SVK_ATTN_BWD_FUSED");
  if (attn_bwd_mfma_ok(dtype, Nk, hd) && vec_ok && Nk <= 64 && fz && fz[0] == '1') {
    // query ranges sized so the grid covers the chip about four times over
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      cus = std::max(cus, 1);
    }
    const int chunks = (Nq + 63) / 64;
    const int want = std::max(1, (int)std::min<long>(chunks, (4L * cus + (long)B * heads - 1) / ((long)B * heads)));
    const int nchunk = (chunks + want - 1) / want, nsplit = (chunks + nchunk - 1) / nchunk;
    dim3 grid(nsplit, heads, B);
    if (hd <= 32)
      hipLaunchKernelGGL((attn_bwd_fused<32>), grid, dim3(256), 0, st, (const bf16*)Q, ldq, sbq, (const bf16*)K, ldk, sbk,
                         (const bf16*)V, ldv, sbv, (const bf16*)O, ldo, sbo, (const bf16*)dO, lddo, sbdo, (bf16*)dQ, lddq,
                         sbdq, acc, acc + nacc, C, Nq, Nk, hd, nchunk, scale);
    else
      hipLaunchKernelGGL((attn_bwd_fused<64>), grid, dim3(256), 0, st, (const bf16*)Q, ldq, sbq, (const bf16*)K, ldk, sbk,
                         (const bf16*)V, ldv, sbv, (const bf16*)O, ldo, sbo, (const bf16*)dO, lddo, sbdo, (bf16*)dQ, lddq,
                         sbdq, acc, acc + nacc, C, Nq, Nk, hd, nchunk, scale);
    int rc = check_launch("attn_bwd_fused");
    if (rc) return rc;
  } else if (attn_bwd_mfma_ok(dtype, Nk, hd) && vec_ok) {
    const int nkc = (Nk + 63) / 64;
    const long nkp = nkc * 64L;
    bf16* Pws = reinterpret_cast<bf16*>(acc + 2 * nacc);
    bf16* dSws = Pws + (long)B * heads * Nq * nkp;
    dim3 grid((Nq + 63) / 64, heads, B);
    // transposed-score kernel (round 6, profiles/r06/attn_bwd_t.txt: whole svk_attention_bwd at the train shapes
    // 101 -> 89 us at 3136 queries, 289 -> 213 us for the 196-token cross-attention); SVK_ATTN_BWD_T=0 selects the
    // round-5 kernel (A/B, tests; read at every call like SVK_ATTN_BWD_FUSED)
    const char* tenv = getenv("SVK_ATTN_BWD_T");
    const bool tscore = !(tenv && tenv[0] == '0');
    auto go = [&](auto hdp_c, auto nkc_c) {
      constexpr int HDP = decltype(hdp_c)::value, NKC = decltype(nkc_c)::value;
      if (tscore)
        hipLaunchKernelGGL((attn_bwd_dq_t<HDP, NKC>), grid, dim3(256), 0, st, (const bf16*)Q, ldq, sbq, (const bf16*)K,
                           ldk, sbk, (const bf16*)V, ldv, sbv, (const bf16*)O, ldo, sbo, (const bf16*)dO, lddo, sbdo,
                           (bf16*)dQ, lddq, sbdq, Pws, dSws, Nq, Nk, hd, scale, reinterpret_cast<float4*>(acc),
                           zero_in_dq ? 2 * nacc / 4 : 0L);
      else
        hipLaunchKernelGGL((attn_bwd_dq_mfma<HDP, NKC>), grid, dim3(256), 0, st, (const bf16*)Q, ldq, sbq, (const bf16*)K,
                           ldk, sbk, (const bf16*)V, ldv, sbv, (const bf16*)O, ldo, sbo, (const bf16*)dO, lddo, sbdo,
                           (bf16*)dQ, lddq, sbdq, Pws, dSws, Nq, Nk, hd, scale, reinterpret_cast<float4*>(acc),
                           zero_in_dq ? 2 * nacc / 4 : 0L);
    };
    using H32 = std::integral_constant<int, 32>;
    using H64 = std::integral_constant<int, 64>;
    using N1 = std::integral_constant<int, 1>;
    using N2 = std::integral_constant<int, 2>;
    using N3 = std::integral_constant<int, 3>;
    using N4 = std::integral_constant<int, 4>;
    auto by_nkc = [&](auto hdp) {
      switch (nkc) { case 1: go(hdp, N1{}); break; case 2: go(hdp, N2{}); break;
                     case 3: go(hdp, N3{}); break; default: go(hdp, N4{}); break; }
    };
    if (hd <= 32) by_nkc(H32{}); else by_nkc(H64{});
    int rc = check_launch("attn_bwd_dq_mfma");
    if (rc) return rc;
    // dK[b, :, h] += dS'[z]^T Q[b, :, h];  dV[b, :, h] += P[z]^T dO[b, :, h]   (z = b * heads + h)
    const long zs = (long)Nq * nkp;
    rc = wgrad_batched(SVK_BF16, dSws, nkp, heads * zs, zs, Q, ldq, sbq, hd, acc, C, (long)Nk * C, hd, B * heads, heads,
                       Nq, Nk, hd, st);
    if (rc) return rc;
    rc = wgrad_batched(SVK_BF16, Pws, nkp, heads * zs, zs, dO, lddo, sbdo, hd, acc + nacc, C, (long)Nk * C, hd,
                       B * heads, heads, Nq, Nk, hd, st);
    if (rc) return rc;
  } else {
    auto lds = [&](int qb) { return (size_t)(2 * Nk * (hd + 1) + 2 * qb * (hd + 1) + 2 * qb * (Nk + 1) + qb) * 4; };
    int QB = 32;
    while (QB > 8 && lds(QB) > 160 * 1024) QB >>= 1;
    if (lds(QB) > 160 * 1024) { set_error("svk_attention_bwd: Nk=%d hd=%d exceeds LDS", Nk, hd); return SVK_EUNSUPPORTED; }
    const size_t sm = lds(QB);
    dim3 grid((Nq + QB - 1) / QB, heads, B);
    SVK_DISPATCH_DTYPE(dtype, T, {
      if (sm > 65536)
        (void)hipFuncSetAttribute((const void*)attention_bwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
      hipLaunchKernelGGL((attention_bwd_kernel<T>), grid, dim3(256), sm, st, (const T*)Q, ldq, sbq, (const T*)K, ldk,
                         sbk, (const T*)V, ldv, sbv, (const T*)O, ldo, sbo, (const T*)dO, lddo, sbdo, (T*)dQ, lddq,
                         sbdq, acc, acc + nacc, (long)C, (long)Nk * C, Nq, Nk, hd, QB, scale);
      int rc = check_launch("attention_bwd");
      if (rc) return rc;
    });
  }
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((store_kv_kernel<T>), dim3((unsigned)((nacc + 255) / 256)), dim3(256), 0, st, acc, (T*)dK,
                       (T*)dV, lddk, sbdk, B, Nk, C);
    return check_launch("attention_bwd store");
  });
}
