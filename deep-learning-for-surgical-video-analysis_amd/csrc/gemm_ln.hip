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
//    16-byte fragments in load order — one contiguous 1 KiB wave-instruction each, L2-resident); the A tile is
//    LDS-DMA'd (see the K loop below); a K tail is zero-filled on both sides, so any K % 8 == 0 works (the
//    adapter's K = C / 4 = 80);
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

static __device__ __attribute__((aligned(16))) uint4 g_zero_ln[4];   // DMA source of A's K tail / rows past M
typedef __attribute__((address_space(3))) void* las_ptr;
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// K loop (round 5, second form): the A tile (BM rows x 64 k, 16-byte chunks XOR-swizzled by row on the
// source address) LDS-DMA'd three K-steps ahead into a 3-deep ring, the W fragments (packed, one contiguous
// 1 KiB wave-instruction each) double-buffered in registers two K-steps ahead, all from inline asm so hipcc's
// waitcnt pass never drains the ring; one counted wait + barrier per K-step.  (The first form loaded the A
// fragments straight from global memory with one step of prefetch: 63 us for the stage-3 proj against 48 for
// GEMM + LayerNorm.)
template <typename T, class C>
__global__ __launch_bounds__(256, 2) void gemm_ln(const T* __restrict__ A, int M, int K, const char* __restrict__ pk,
                                                 const float* __restrict__ bias, const T* __restrict__ R,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 float eps, T* __restrict__ X, T* __restrict__ Hn) {
  typedef v8_t<T> tx8;
  constexpr int MB = C::MB, NBW = C::NBW, N = C::N, BM = C::BM;
  constexpr int ABYTES = BM * 128, DPW = BM * 8 / 256;     // A tile per K-step; DMA wave-instructions per wave
  // the output rows are staged through LDS (row stride 2 N + 16 bytes: the 8-byte fragment-layout writes of a
  // wave's 16 rows hit 16 distinct bank pairs) and leave as 16-byte row-contiguous stores — the fragment layout's
  // own 8-byte stores (16 rows x 32 bytes per instruction) made the first forms 1.3x slower than GEMM + LN.  The
  // stage overlays the A ring: it is written after the row-sum barrier, which every wave reaches after the
  // vmcnt(0) that retires its last (clamped) ring DMA
  constexpr int SROW = 2 * N + 16;
  constexpr int SMEM = 3 * ABYTES > BM * SROW ? 3 * ABYTES : BM * SROW;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  __shared__ float red[2][4][BM];                      // per-wave row partials: sums, then centred squares
  char* const stage = smem;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM, n0w = wave * (N / 4);
  const int nk = (K + 63) / 64;

  // ---- A DMA: chunk q = 64 (wave + 4 j) + lane: row q / 8, LDS chunk q % 8 holds global chunk (q % 8) ^ (row & 7)
  const char* zero = reinterpret_cast<const char*>(g_zero_ln);
  const char* asrc[DPW];
  int acol[DPW];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int q = (wave + 4 * j) * 64 + lane, row = q >> 3, c = (q & 7) ^ (row & 7);
    asrc[j] = m0 + row < M ? reinterpret_cast<const char*>(A + (long)(m0 + row) * K + c * 8) : nullptr;
    acol[j] = c * 8;
  }
  auto dma_a = [&](int kt, int slot) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
      dma16(asrc[j] && kt * 64 + acol[j] < K ? asrc[j] + kt * 128 : zero,
            __builtin_amdgcn_readfirstlane(lds0 + slot * ABYTES + (wave + 4 * j) * 1024));
  };
  // ---- W fragments (two register sets, static indices: the loop is unrolled by two)
  const char* pkl = pk + (wave * NBW * 64 + lane) * 16;
  tx8 wf0[2][NBW], wf1[2][NBW];                        // the two sets: [ks][nb]
  auto load_w = [&](int kt, tx8 (&w)[2][NBW]) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb)
        asm volatile("global_load_dwordx4 %0, %1, off"
                     : "=v"(w[ks][nb]) : "v"(pkl + (long)(2 * kt + ks) * C::PKS + nb * 1024) : "memory");
  };
  auto tie_w = [&](tx8 (&w)[2][NBW]) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) asm volatile("" : "+v"(w[ks][nb]));
  };
  f32x4 acc[MB][NBW];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int slot, const tx8 (&w)[2][NBW]) __attribute__((always_inline)) {
    const char* as = smem + slot * ABYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int row = mb * 16 + fr;
        const tx8 a = *reinterpret_cast<const tx8*>(as + row * 128 + (((ks * 4 + fq) ^ (row & 7)) << 4));
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) acc[mb][nb] = mfma16x16x32(w[ks][nb], a, acc[mb][nb]);
      }
  };
  // prologue: A(0..2) in the ring, W(0) / W(1) in the two sets
  dma_a(0, 0);
  dma_a(min(1, nk - 1), 1);
  dma_a(min(2, nk - 1), 2);
  load_w(0, wf0);
  load_w(min(1, nk - 1), wf1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tie_w(wf0);
  tie_w(wf1);
  __syncthreads();
  // iteration kt: MFMAs of K-step kt (A slot kt % 3, W set kt & 1), then W(kt + 2) into that set and the DMA
  // of A(kt + 3) into that slot; the counted wait leaves those in flight (W(kt + 1) and A(kt + 1) retired)
  auto iter = [&](int kt, tx8 (&w)[2][NBW], tx8 (&wn)[2][NBW]) __attribute__((always_inline)) {
    mma(kt % 3, w);
    load_w(min(kt + 2, nk - 1), w);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot kt % 3 are done
    __syncthreads();                                    // everybody's: the slot may be refilled
    dma_a(min(kt + 3, nk - 1), kt % 3);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NBW + DPW) : "memory");
    tie_w(wn);
    __syncthreads();                                    // A(kt + 1) visible to every wave
  };
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    iter(kt, wf0, wf1);
    iter(kt + 1, wf1, wf0);
  }
  if (kt < nk) iter(kt, wf0, wf1);
  // the clamped tail loads / DMA (never used) retire; the ties keep hipcc from handing their registers to other
  // values while those loads are still in flight (an asm load whose output is never read is dead to the compiler)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tie_w(wf0);
  tie_w(wf1);

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
  // X (rounded) into the stage, then the rows leave 16 bytes per lane; H the same way through the same buffer
  auto stage_put = [&](int mb, int nb, const T (&o)[4]) __attribute__((always_inline)) {
    *reinterpret_cast<uint2*>(stage + (16 * mb + fr) * SROW + (n0w + 16 * nb + 4 * fq) * 2) = *reinterpret_cast<const uint2*>(o);
  };
  auto stage_store = [&](T* dst) __attribute__((always_inline)) {
    constexpr int CPR = N / 8, NCH = BM * CPR;        // 16-byte chunks per row / per tile
#pragma unroll
    for (int it = 0; it < (NCH + 255) / 256; ++it) {
      const int c = tid + 256 * it, row = c / CPR, cc = c % CPR;
      if (c < NCH && m0 + row < M)
        *reinterpret_cast<uint4*>(dst + (long)(m0 + row) * N + cc * 8) = *reinterpret_cast<const uint4*>(stage + row * SROW + cc * 16);
    }
  };
  if (X) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        T xo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) xo[e] = from_f<T>(v[mb][nb][e]);
        stage_put(mb, nb, xo);
      }
    __syncthreads();
    stage_store(X);
    __syncthreads();                                   // the stage is rewritten with H next
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const float rstd = 1.0f / sqrtf(q[mb] * (1.0f / N) + eps);
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int n = n0w + 16 * nb + 4 * fq;
      const float4 g = *reinterpret_cast<const float4*>(gamma + n), b = *reinterpret_cast<const float4*>(beta + n);
      const float gg[4] = {g.x, g.y, g.z, g.w}, bv[4] = {b.x, b.y, b.z, b.w};
      T ho[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) ho[e] = from_f<T>((v[mb][nb][e] - mean[mb]) * rstd * gg[e] + bv[e]);
      stage_put(mb, nb, ho);
    }
  }
  __syncthreads();
  stage_store(Hn);
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
  // X and H leave as 16-byte row chunks (stage_store), R is read as 8-byte pieces
  if ((((uintptr_t)A) | ((uintptr_t)packed) | ((uintptr_t)bias) | ((uintptr_t)gamma) | ((uintptr_t)beta) |
       ((uintptr_t)X) | ((uintptr_t)H)) & 15 || ((uintptr_t)R) & 7) {
    set_error("svk_gemm_ln: misaligned operand (A, packed, bias, gamma, beta, X, H: 16 bytes; R: 8)"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    if (N == 512) return gln::launch<T, gln::Cfg<512, 2>>(A, M, K, packed, bias, R, gamma, beta, eps, X, H, st);
    return gln::launch<T, gln::Cfg<320, 4>>(A, M, K, packed, bias, R, gamma, beta, eps, X, H, st);
  });
}
