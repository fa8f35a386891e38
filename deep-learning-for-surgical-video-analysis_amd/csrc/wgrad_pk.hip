// Weight gradient of the training step's token GEMMs (train_evp.py:473-515 backward through the trainable
// head / prompt / flow-encoder / cross-attention layers, and the attention backward's dK / dV):
//
//   dW[n][k] += sum_m dY[m][n] * X[m][k]          (bf16 / f16 operands, f32 accumulation, f32 dW)
//
// Both operands arrive token-major ([m][n], [m][k]); the MFMA wants the reduction index m per lane.
// Here the slabs of 32 token rows are DMA'd into LDS in their natural row layout
// (`global_load_lds_dwordx4`: no VGPR round trip, no per-element transposed LDS writes) and the MFMA
// fragments are read back transposed by the hardware (`ds_read_b64_tr_b16`: a 16-lane group reads a
// 4-row x 16-column block and each lane receives one column).  For the 16x16x32 MFMA, lane (g, i)
// (g = lane >> 4, i = lane & 15) needs A[n = i][m = 8g .. 8g + 7]: two transposed reads of rows
// 8g .. 8g + 3 and 8g + 4 .. 8g + 7 (lane 4q + p of the group addresses row q, columns 4p .. 4p + 3).
// Same for B = X.  The 16-byte chunks of every LDS row are XOR-swizzled (applied on the DMA source
// address, the DMA image being lane-linear) so that a 32-lane half's 8 rows x 2 chunks of a transposed
// read fall into distinct banks.
//
// Tile BN x BK per workgroup (4 waves 2 x 2), the M range split over gridDim.y; each workgroup's
// partial tile is added into dW with f32 atomics (one per element per workgroup; the split count is
// chosen so that the atomic bytes stay well below the operand bytes).  Pipeline per 32-row step:
// DMA(next) -> counted vmcnt -> s_barrier -> transposed reads + MFMAs -> s_barrier (the gemm_pk pattern).
// The bias gradient db[n] = sum_m dY[m][n] is summed from the A fragments already in registers (the
// k-tile-0 workgroups only).  Batching over gridDim.z as in wgrad_kernel (attention dK / dV).
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>

namespace svk {
namespace wgpk {

static __device__ __attribute__((aligned(16))) uint4 g_zero[4];
typedef __attribute__((address_space(3))) void* las_ptr;
typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void barrier_mem() { asm volatile("s_barrier" ::: "memory"); }

template <int BN_, int BK_>
struct Cfg {
  static constexpr int BN = BN_, BK = BK_, NT = 256, BM = 32;
  static constexpr int WN = BN / 2, WK = BK / 2, TM = WN / 16, TN = WK / 16;
  static constexpr int A_BYTES = BM * BN * 2, B_BYTES = BM * BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int A_LD = A_BYTES / (NT * 16), B_LD = B_BYTES / (NT * 16), LD = A_LD + B_LD;
  static_assert(A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "whole DMA rounds");
  static_assert((BN == 64 || BN == 128) && (BK == 64 || BK == 128), "row swizzle defined for 128 / 256-byte rows");
};

// chunk swizzle of row r for rows of CPR 16-byte chunks (8: 128-byte rows, 16: 256-byte rows)
template <int CPR>
__device__ __forceinline__ int swz(int r) {
  if constexpr (CPR == 16) return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
  else return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}

// byte offset of element column `col` (a multiple of 4) of row r in a [32][CPR * 8] 16-bit image
template <int CPR>
__device__ __forceinline__ int img_off(int r, int col) {
  return r * (CPR * 16) + (((col >> 3) ^ swz<CPR>(r)) << 4) + ((col >> 2) & 1) * 8;
}

template <typename T>
__device__ __forceinline__ v8_t<T> tr_frag(const char* img_lo, const char* img_hi) {
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(las_ptr)img_lo);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(las_ptr)img_hi);
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s w = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(v8_t<T>, w);
}

struct Args {
  const void* dY; long ldy;
  const void* X; long ldx;
  float* dW; long lddw;
  float* db;
  int M, N, K, mchunk, nzi;
  long sa_o, sa_i, sx_o, sx_i, sw_o, sw_i;
  int H, Wd, Cin, OH, OW, kw, stride, pad;   // CONV: X is the NHWC input map, row m = output pixel, k = (ky, kx, ci)
};

template <typename T, class C, bool CONV>
__global__ __launch_bounds__(256) void wgrad_pk(Args p) {
  constexpr int BN = C::BN, BK = C::BK, TM = C::TM, TN = C::TN, CPRA = BN / 8, CPRB = BK / 8;
  typedef v8_t<T> tx8;
  __shared__ __attribute__((aligned(1024))) char smem[2 * C::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const int ntk = (p.K + BK - 1) / BK;
  const int n0 = (blockIdx.x / ntk) * BN, k0 = (blockIdx.x % ntk) * BK;
  const int mbeg = blockIdx.y * p.mchunk, mend = min(mbeg + p.mchunk, p.M);
  const int zo = blockIdx.z / p.nzi, zi = blockIdx.z - zo * p.nzi;
  const char* dY = static_cast<const char*>(p.dY) + (zo * p.sa_o + zi * p.sa_i) * (long)sizeof(T);
  const char* X = static_cast<const char*>(p.X) + (zo * p.sx_o + zi * p.sx_i) * (long)sizeof(T);
  float* dW = p.dW + zo * p.sw_o + zi * p.sw_i;
  const char* zero = reinterpret_cast<const char*>(g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;
  const int nsteps = (mend - mbeg + 31) / 32;

  // DMA of one 32-row step into stage `buf`: LDS slot s (16 bytes) = row s / CPR, chunk s % CPR, holding
  // global chunk (s % CPR) ^ swz(row); rows past the chunk's end and columns past N / K read zeros
  auto issue = [&](int step, int buf) {
    const int m0 = mbeg + step * 32;
    const uint32_t sa = lds0 + buf * C::STAGE, sb = sa + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < C::A_LD; ++i) {
      const int s = (wave * C::A_LD + i) * 64 + lane;
      const int r = s / CPRA, c = (s % CPRA) ^ swz<CPRA>(r);
      const int m = m0 + r, n = n0 + c * 8;
      const char* src = (m < mend && n < p.N) ? dY + ((long)m * p.ldy + n) * (long)sizeof(T) : zero;
      dma16(src, __builtin_amdgcn_readfirstlane(sa + (wave * C::A_LD + i) * 1024));
    }
#pragma unroll
    for (int i = 0; i < C::B_LD; ++i) {
      const int s = (wave * C::B_LD + i) * 64 + lane;
      const int r = s / CPRB, c = (s % CPRB) ^ swz<CPRB>(r);
      const int m = m0 + r, k = k0 + c * 8;
      const char* src = zero;
      if constexpr (CONV) {
        // im2col on the fly: 8 consecutive k = 8 channels of one tap (Cin % 8 == 0) = 16 contiguous bytes
        if (m < mend && k < p.K) {
          const int ohw = p.OH * p.OW, b = m / ohw, pix = m - b * ohw, oy = pix / p.OW, ox = pix - oy * p.OW;
          const int t = k / p.Cin, ci = k - t * p.Cin, ky = t / p.kw, kx = t - ky * p.kw;
          const int iy = oy * p.stride - p.pad + ky, ix = ox * p.stride - p.pad + kx;
          if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.Wd)
            src = X + ((((long)b * p.H + iy) * p.Wd + ix) * p.Cin + ci) * (long)sizeof(T);
        }
      } else {
        if (m < mend && k < p.K) src = X + ((long)m * p.ldx + k) * (long)sizeof(T);
      }
      dma16(src, __builtin_amdgcn_readfirstlane(sb + (wave * C::B_LD + i) * 1024));
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_db = p.db != nullptr && k0 == 0 && wk == 0;
  float dbs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) dbs[i] = 0.f;

  // transposed-read addresses: lane (g, q, p) reads rows 8g + q (+ 4), columns base + 4p
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  if (nsteps > 0) issue(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) {
      issue(s + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::LD) : "memory");   // this step's DMA landed (own)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_mem();                                                   // everyone's DMA landed
    const char* sa = smem + buf * C::STAGE;
    const char* sb = sa + C::A_BYTES;
    tx8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int col = wn * C::WN + i * 16 + 4 * pp;
      fa[i] = tr_frag<T>(sa + img_off<CPRA>(8 * g + q, col), sa + img_off<CPRA>(8 * g + 4 + q, col));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wk * C::WK + j * 16 + 4 * pp;
      fb[j] = tr_frag<T>(sb + img_off<CPRB>(8 * g + q, col), sb + img_off<CPRB>(8 * g + 4 + q, col));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
    if (do_db) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) dbs[i] += (float)fa[i][e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_mem();                                                   // nobody still reads `buf`
  }
  // lane holds dW[n = n0 + wn*WN + 16 i + 4 g + r][k = k0 + wk*WK + 16 j + (lane & 15)]
  const int fr = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = k0 + wk * C::WK + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * C::WN + i * 16 + 4 * g + r;
        if (n < p.N && k < p.K) atomicAdd(dW + (long)n * p.lddw + k, acc[i][j][r]);
      }
    }
  if (do_db) {   // lane (g, i16) summed column n = base + i16 over rows 8g .. 8g + 7 of every step
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v = dbs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int n = n0 + wn * C::WN + i * 16 + fr;
      if (g == 0 && n < p.N) atomicAdd(p.db + n, v);
    }
  }
}

template <typename T, class C, bool CONV = false>
static int launch(Args a, int Z, hipStream_t st) {
  const long tiles = (long)((a.N + C::BN - 1) / C::BN) * ((a.K + C::BK - 1) / C::BK);
  // M split: enough workgroups to fill the chip (~2 per CU), each with >= 128 rows (4 steps), and the f32
  // atomic bytes (splits x N x K x 4) at most the operand bytes (M x (N + K) x 2): the training step's
  // weight gradients are mostly short (M = 88 x 49 / 88 x 196 tokens), where the split is what fills the chip.
  // Round 6 (profiles/r06/wgrad_target_ab.txt, train step same box): 512 workgroups 13.61 ms, 1024 13.69, 256 13.75,
  // 2048 13.76, 128 14.30 — past ~2 per CU the extra splits' atomics cost more than the fill gains (SVK_WGRAD_TARGET)
  static const long wg_target = getenv("SVK_WGRAD_TARGET") ? std::max(1L, atol(getenv("SVK_WGRAD_TARGET"))) : 512;
  const long target = std::max<long>(1, wg_target / std::max<long>(1, tiles * Z));
  const long by_rows = std::max<long>(1, a.M / 128);
  const long by_atomics = std::max<long>(1, ((long)a.M * (a.N + a.K) * 2) / std::max<long>(1, (long)a.N * a.K * 4));
  long splits = std::min(target, std::min(by_rows, by_atomics));
  long chunk = (a.M + splits - 1) / splits;
  chunk = (chunk + 31) / 32 * 32;
  splits = (a.M + chunk - 1) / chunk;
  a.mchunk = (int)chunk;
  if (a.nzi <= 0) a.nzi = 1;
  hipLaunchKernelGGL((wgrad_pk<T, C, CONV>), dim3((unsigned)tiles, (unsigned)splits, (unsigned)Z), dim3(256), 0, st, a);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "wgrad_pk<%s, Cfg<%d, %d>%s>", type_name<T>(), C::BN, C::BK, CONV ? ", conv" : "");
  set_last_kernel(name);
  return check_launch("wgrad_pk");
}

}  // namespace wgpk

// dW (+ db) += dY^T X on the transposed-read pipeline.  Returns 1 when not eligible: every row must
// start 16-byte aligned and hold whole 16-byte chunks up to N / K (ldy >= N rounded up to 8, likewise
// ldx; the columns past N / K read there only feed dW rows / columns that are never stored); the caller
// then falls back to wgrad_kernel.
template <typename T>
int wgrad_pk_try(const void* dY, long ldy, long sa_o, long sa_i, const void* X, long ldx, long sx_o, long sx_i,
                 float* dW, long lddw, long sw_o, long sw_i, float* db, int Z, int nzi, int M, int N, int K,
                 hipStream_t st) {
  if (getenv("SVK_NO_WGRAD_PK")) return 1;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const long n8 = (N + 7) / 8 * 8, k8 = (K + 7) / 8 * 8;
  if (ldy % 8 || ldx % 8 || ldy < n8 || ldx < k8 || sa_o % 8 || sa_i % 8 || sx_o % 8 || sx_i % 8 || !al(dY) ||
      !al(X))
    return 1;
  wgpk::Args a{};
  a.dY = dY; a.ldy = ldy; a.X = X; a.ldx = ldx; a.dW = dW; a.lddw = lddw; a.db = db;
  a.M = M; a.N = N; a.K = K; a.nzi = nzi;
  a.sa_o = sa_o; a.sa_i = sa_i; a.sx_o = sx_o; a.sx_i = sx_i; a.sw_o = sw_o; a.sw_i = sw_i;
  if (N <= 64 && K <= 64) return wgpk::launch<T, wgpk::Cfg<64, 64>>(a, Z, st);
  if (N <= 64) return wgpk::launch<T, wgpk::Cfg<64, 128>>(a, Z, st);
  if (K <= 64) return wgpk::launch<T, wgpk::Cfg<128, 64>>(a, Z, st);
  return wgpk::launch<T, wgpk::Cfg<128, 128>>(a, Z, st);
}

// conv weight gradient (svk_conv2d_wgrad_nhwc): dW[co][(ky, kx, ci)] (+ db) over output pixels, X the NHWC map
// (16-byte aligned, Cin % 8 == 0), dY [M, Cout] rows (Cout % 8 == 0).  Returns 1 when not eligible.
template <typename T>
int wgrad_pk_conv_try(const void* X, int B, int H, int W, int Cin, const void* dY, int Cout, int k, int stride, int pad,
                      int OH, int OW, float* dW, float* db, hipStream_t st) {
  if (getenv("SVK_NO_WGRAD_PK") || getenv("SVK_NO_WGRAD_PK_CONV")) return 1;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (Cin % 8 || Cout % 8 || !al(X) || !al(dY)) return 1;
  if ((long)B * H * W * Cin > 0x7fffffffL) return 1;
  wgpk::Args a{};
  a.dY = dY; a.ldy = Cout; a.X = X; a.ldx = 0; a.dW = dW; a.lddw = (long)k * k * Cin; a.db = db;
  a.M = B * OH * OW; a.N = Cout; a.K = k * k * Cin; a.nzi = 1;
  a.H = H; a.Wd = W; a.Cin = Cin; a.OH = OH; a.OW = OW; a.kw = k; a.stride = stride; a.pad = pad;
  if (Cout <= 64 && a.K <= 64) return wgpk::launch<T, wgpk::Cfg<64, 64>, true>(a, 1, st);
  if (Cout <= 64) return wgpk::launch<T, wgpk::Cfg<64, 128>, true>(a, 1, st);
  if (a.K <= 64) return wgpk::launch<T, wgpk::Cfg<128, 64>, true>(a, 1, st);
  return wgpk::launch<T, wgpk::Cfg<128, 128>, true>(a, 1, st);
}

template int wgrad_pk_conv_try<bf16>(const void*, int, int, int, int, const void*, int, int, int, int, int, int, float*,
                                     float*, hipStream_t);
template int wgrad_pk_conv_try<f16>(const void*, int, int, int, int, const void*, int, int, int, int, int, int, float*,
                                    float*, hipStream_t);

template int wgrad_pk_try<bf16>(const void*, long, long, long, const void*, long, long, long, float*, long, long, long,
                                float*, int, int, int, int, int, hipStream_t);
template int wgrad_pk_try<f16>(const void*, long, long, long, const void*, long, long, long, float*, long, long, long,
                               float*, int, int, int, int, int, hipStream_t);

}  // namespace svk
