// Wide-tile persistent GEMM for the long-K / wide-N token GEMMs (f16 / bf16 in and out, f32 accumulate):
//
//   C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]
//
// The shapes it is for (MiT-b2 / b3 at B = 256): the SegFormer head's folded decode-fuse GEMM
// (segformer_head.py:74-80, 158; 12544 x 2048 x 1024), the stage-3 / stage-4 MixFFN fc1 / fc2
// (mix_transformer_evp.py:60-67; 50176 x 1280 x 320, 50176 x 320 x 1280, 12544 x 2048 x 512, 12544 x 512 x 2048)
// and the stage-4 kv projection (:81-90; 12544 x 1024 x 512).
//
// Why not gemm_pk's 128 x 128 tile: there each wave owns 64 x 64 outputs and reads 16 fragment vectors
// (16 KiB per wave) per 32 MFMAs — with both workgroups of a CU computing, that is the LDS's whole
// 256 B/clk at the MFMA rate, so the tile cannot approach the matrix peak.  Here one 256-thread workgroup per
// CU owns a (32 TM) x (32 TN) tile as 2 x 2 waves of (16 TM) x (16 TN): at TM = TN = 8 a wave reads 16
// fragment vectors per 64 MFMAs (4x the reuse), the accumulators (256 registers) sit in the AGPR half of
// the register file, and the LDS traffic is a quarter of the array's rate.
//
//  * LDS: two K-tile stages of A [32 TM][64 k] and W [32 TN][64 k] (128 KiB at TM = TN = 8), filled by
//    LDS-DMA (`global_load_lds_dwordx4`, the XOR swizzle applied on the source address so every
//    ds_read_b128 fragment read is conflict-free; the same image as gemm_pk);
//  * one barrier per 64-deep K-tile: wait own DMA(u) -> barrier -> DMA(u + 1) into the other stage (all
//    reads of it retired before the barrier) -> fragments + 128 MFMAs;
//  * the fragment reads of k-step 0 of a K-tile hide behind the MFMAs of k-step 1 of the previous K-tile
//    (rotated loop), so within a tile the matrix pipe never waits for LDS;
//  * persistent: the grid (one workgroup per CU) walks its tiles; the next tile's first K-tile is DMA'd
//    during the current tile's last, so tile prologues are hidden;
//  * transposed MFMA (W fragment x A fragment): each lane holds 4 consecutive output columns of a row; the
//    epilogue (bias, activation, residual in f32, one rounding) stores 8-byte row pieces from the
//    accumulators.
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>
#include <type_traits>

namespace svk {
namespace wt {

static __device__ __attribute__((aligned(16))) uint4 g_zero[4];   // 64 zero bytes: the K-tail source

typedef __attribute__((address_space(3))) void* las_ptr;

template <int TM_, int TN_>
struct Cfg {
  static constexpr int TM = TM_, TN = TN_;
  static constexpr int WM = 16 * TM, WN = 16 * TN, BM = 2 * WM, BN = 2 * WN, BK = 64, NT = 256;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES, LDS = 2 * STAGE;
  static constexpr int A_LD = A_BYTES / (NT * 16), B_LD = B_BYTES / (NT * 16), LD = A_LD + B_LD;
  static_assert(A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "tile must split into whole DMA rounds");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(LD <= 63, "vmcnt range");
};

// LDS-DMA of one 16-byte chunk per lane: global address = sbase (SGPR pair) + voff (32-bit VGPR), LDS address
// = M0 = lds + IMM (+ lane * 16 by the hardware).  One SGPR pair per operand and one VGPR per instruction: the
// K-tile advance is a scalar add on sbase.  M0 is saved / restored around it.
template <int IMM>
__device__ __forceinline__ void dma16s(const char* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_add_u32 m0, %3, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds), "n"(IMM) : "memory", "scc");
}
// the same with a full 64-bit VGPR address (K tails: a lane past K reads the zero block)
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void barrier() {
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <typename T, class C, bool KTAIL, int ACT>
__global__ __launch_bounds__(256, 1)
void gemm_wt(GemmArgs p, int ntn, int ntiles, int nk) {
  typedef v8_t<T> tx8;
  constexpr int TM = C::TM, TN = C::TN, WM = C::WM, WN = C::WN, BM = C::BM, BN = C::BN;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int first = xcd_remap(blockIdx.x, G);
  if (first >= ntiles) return;
  const char* Ab = static_cast<const char*>(p.A);
  const char* Wb = static_cast<const char*>(p.W);
  const char* zero = reinterpret_cast<const char*>(g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;
  const long ldab = p.lda * 2, ldwb = p.ldw * 2;

  // ---- LDS-DMA of one K-tile (tile, kt) into stage buf: instruction i of wave w moves 16-byte chunks
  // q = (w * LD_ + i) * 64 + lane of the stage image (row q / 8, swizzled chunk).  The per-lane byte offsets
  // (row * ld + chunk) are set once per tile (set_rows); the K-tile enters through the scalar base.
  uint32_t offA[C::A_LD], offB[C::B_LD];
  const int lr = lane >> 3, cq = (lane & 7) ^ (lr & 7);   // chunk q's row within its 8-row group, swizzled chunk
  auto set_rows = [&](int tile) {
    const int m0 = (tile / ntn) * BM + wave * (C::A_LD * 8) + lr, n0 = (tile % ntn) * BN + wave * (C::B_LD * 8) + lr;
#pragma unroll
    for (int i = 0; i < C::A_LD; ++i) offA[i] = (uint32_t)min(m0 + i * 8, p.M - 1) * (uint32_t)ldab + cq * 16;
#pragma unroll
    for (int i = 0; i < C::B_LD; ++i) offB[i] = (uint32_t)min(n0 + i * 8, p.N - 1) * (uint32_t)ldwb + cq * 16;
  };
  // DMA instruction idx (A rows for idx < A_LD, then W rows) of K-tile kt into stage buf
  auto issue1 = [&](int kt, int buf, int idx) {
    const bool isA = idx < C::A_LD;
    const int i = isA ? idx : idx - C::A_LD;
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds0 + buf * C::STAGE + (isA ? 0 : C::A_BYTES) +
                                                        (wave * (isA ? C::A_LD : C::B_LD) + i) * 1024);
    const uint32_t off = isA ? offA[i] : offB[i - 0];
    const char* base = (isA ? Ab : Wb) + kt * 128;
    if constexpr (KTAIL) {
      dma16(kt * 64 + cq * 8 < p.K ? base + off : zero, lds);
    } else {
      dma16s<0>(base, off, lds);
    }
  };
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int idx = 0; idx < C::LD; ++idx) issue1(kt, buf, idx);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // One K-tile: k-step 0 then 1.  A k-step holds its TN B fragments; the A fragment of row block i + 1 is read
  // while the TN MFMAs of row block i run, and the next k-step's B fragments during the last row block — the
  // groups are fenced (sched_barrier) so hipcc cannot hoist every read to the top (which needs ~190 fragment
  // registers next to the 256 accumulators and spills).
  tx8 fb[2][TN], fa[2];
  auto read_b = [&](int buf, int ks, tx8* dst) {
    const char* sb = smem + buf * C::STAGE + C::A_BYTES;
    const int cc = ((ks * 4 + fq) ^ (fr & 7)) * 16;
#pragma unroll
    for (int j = 0; j < TN; ++j) dst[j] = *reinterpret_cast<const tx8*>(sb + (wn * WN + j * 16 + fr) * 128 + cc);
  };
  auto read_a = [&](int buf, int ks, int i) {
    const char* sa = smem + buf * C::STAGE;
    const int cc = ((ks * 4 + fq) ^ (fr & 7)) * 16;
    return *reinterpret_cast<const tx8*>(sa + (wm * WM + i * 16 + fr) * 128 + cc);
  };
  // dkt_ / dbuf_ < 0: no DMA to interleave.  The next K-tile's LD DMA instructions ride two per row group in the
  // first groups (an LDS-DMA issue costs ~60 cycles among MFMAs: issued back to back at the top of the K-tile
  // they cost ~1k cycles with the matrix pipe idle)
  auto ktile = [&](int buf, int dkt_, int dbuf_) {
    read_b(buf, 0, fb[0]);
    fa[0] = read_a(buf, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s2 = 0; s2 < 2 * TM; ++s2) {
      const int ks = s2 / TM, i = s2 % TM;
      if (dbuf_ >= 0) {
        if (2 * s2 < C::LD) issue1(dkt_, dbuf_, 2 * s2);
        if (2 * s2 + 1 < C::LD) issue1(dkt_, dbuf_, 2 * s2 + 1);
      }
      if (s2 + 1 < 2 * TM) fa[(s2 + 1) & 1] = read_a(buf, (s2 + 1) / TM, (s2 + 1) % TM);
      if (s2 == TM - 2) read_b(buf, 1, fb[1]);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[ks][j], fa[s2 & 1], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const T* R = static_cast<const T*>(p.R);
  T* Cout = static_cast<T*>(p.C);
  auto epilogue = [&](int tile) {
    const int m0 = (tile / ntn) * BM + wm * WM, n0 = (tile % ntn) * BN + wn * WN;
    f32x4 bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = min(n0 + j * 16 + fq * 4, p.N - 4);
      bj[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + i * 16 + fr;
      uint2 res[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = min(n0 + j * 16 + fq * 4, p.N - 4);
        res[j] = R ? *reinterpret_cast<const uint2*>(R + (long)min(m, p.M - 1) * p.ldr + n) : uint2{0u, 0u};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + j * 16 + fq * 4;
        float v[4] = {acc[i][j][0] + bj[j].x, acc[i][j][1] + bj[j].y, acc[i][j][2] + bj[j].z, acc[i][j][3] + bj[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act_fast(v[e], ACT);
        const f32x2 r01 = unpack2<T>(res[j].x), r23 = unpack2<T>(res[j].y);
        v[0] += r01.x;
        v[1] += r01.y;
        v[2] += r23.x;
        v[3] += r23.y;
        T o[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
        if (m < p.M && n < p.N) *reinterpret_cast<uint2*>(Cout + (long)m * p.ldc + n) = *reinterpret_cast<const uint2*>(o);
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  // ---- the (tile, K-tile) stream of this workgroup: tiles first, first + G, ...; the DMA cursor runs one
  // K-tile ahead of the compute cursor.  Past the last unit no DMA is issued.
  int dtile = first, dkt = 0;
  set_rows(dtile);
  issue(dkt, 0);
  if (++dkt == nk) {
    dkt = 0;
    dtile += G;
  }
  int buf = 0;
  bool stores_pending = false;
  // one K-tile step: own DMA of this K-tile landed (the previous tile's epilogue stores, younger, may still fly)
  // and every wave's fragment reads of the other stage retired -> barrier: everyone's DMA landed and the other
  // stage is free -> DMA of the next K-tile into it -> fragments + MFMAs of this one
  auto step = [&]() {
    if (stores_pending) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    stores_pending = false;
    barrier();
    int ikt = -1;
    if (dtile < ntiles) {
      if (dkt == 0) set_rows(dtile);       // (here, behind the step's wait: no drain of a DMA in flight)
      ikt = dkt;
      if (++dkt == nk) {
        dkt = 0;
        dtile += G;
      }
    }
    ktile(buf, ikt, ikt >= 0 ? (buf ^ 1) : -1);
    buf ^= 1;
  };
  for (int tile = first; tile < ntiles; tile += G) {
    // (the epilogue sits outside the K loop: inside it, hipcc hoists the epilogue's per-tile addresses out of the
    // loop and keeps them live next to the accumulators)
    for (int kt = 0; kt < nk; ++kt) step();
    epilogue(tile);
    stores_pending = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int slots_of(const void* fn) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0);
  return std::max(1, cus) * std::max(1, per);
}

template <typename T, int TM, int TN, bool KTAIL, int ACT>
static int launch(const GemmArgs& a, hipStream_t st) {
  typedef Cfg<TM, TN> C;
  const int ntm = (a.M + C::BM - 1) / C::BM, ntn = (a.N + C::BN - 1) / C::BN;
  const long ntiles = (long)ntm * ntn;
  const int nk = (a.K + 63) / 64;
  static const int slots = slots_of(reinterpret_cast<const void*>(&gemm_wt<T, C, KTAIL, ACT>));
  const int grid = (int)std::min<long>(ntiles, slots);
  hipLaunchKernelGGL((gemm_wt<T, C, KTAIL, ACT>), dim3(grid), dim3(256), 0, st, a, ntn, (int)ntiles, nk);
  static char name[80];
  if (!name[0])
    snprintf(name, sizeof(name), "gemm_wt<%s, Cfg<%d, %d>, %s, %d>", type_name<T>(), TM, TN, KTAIL ? "true" : "false", ACT);
  set_last_kernel(name);
  return check_launch("gemm_wt");
}

template <typename T, int TM, int TN>
static int launch_cfg(const GemmArgs& a, hipStream_t st) {
  const bool tail = a.K % 64 != 0;
  switch (a.act) {
    case SVK_ACT_GELU: return tail ? launch<T, TM, TN, true, SVK_ACT_GELU>(a, st) : launch<T, TM, TN, false, SVK_ACT_GELU>(a, st);
    case SVK_ACT_RELU: return tail ? launch<T, TM, TN, true, SVK_ACT_RELU>(a, st) : launch<T, TM, TN, false, SVK_ACT_RELU>(a, st);
    case 0: return tail ? launch<T, TM, TN, true, 0>(a, st) : launch<T, TM, TN, false, 0>(a, st);
    default: return 1;
  }
}

}  // namespace wt

// Dense A only, plain epilogue (bias / GELU / ReLU / residual), K % 8 == 0, N % 4 == 0, 16-byte aligned operand
// rows.  cfg: 0 = 256 x 256 (TM = TN = 8), 1 = 256 x 160, 2 = 256 x 128.  Returns 1 when not eligible.
template <typename T>
int gemm_wt_try(const GemmArgs& a, hipStream_t st, int cfg) {
  auto al = [](const void* q, int b) { return ((uintptr_t)q & (b - 1)) == 0; };
  if (a.K % 8 || a.N % 4 || a.lda % 8 || a.ldw % 8 || a.ldc % 4 || (a.R && a.ldr % 4) || a.out_mode || a.U ||
      a.rscale || a.ksplit > 1)
    return 1;
  if (!al(a.A, 16) || !al(a.W, 16) || !al(a.C, 8) || (a.R && !al(a.R, 8)) || (a.bias && !al(a.bias, 16))) return 1;
  // 32-bit per-lane byte offsets of the DMA rows
  if ((long)a.M * a.lda * 2 + 256 >= (1L << 32) || (long)a.N * a.ldw * 2 + 256 >= (1L << 32)) return 1;
  switch (cfg) {
    case 0: return wt::launch_cfg<T, 8, 8>(a, st);
    case 1: return wt::launch_cfg<T, 8, 5>(a, st);
    case 2: return wt::launch_cfg<T, 8, 4>(a, st);
    default: return 1;
  }
}

template int gemm_wt_try<bf16>(const GemmArgs&, hipStream_t, int);
template int gemm_wt_try<f16>(const GemmArgs&, hipStream_t, int);

}  // namespace svk
