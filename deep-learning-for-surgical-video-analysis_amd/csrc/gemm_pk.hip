// Persistent, LDS-DMA-pipelined bf16 / f16 MFMA GEMM for the token GEMMs of the MiT/SegFormer path.
//
//   C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]        (bf16 or f16 in/out, f32 accumulate)
//
// Why persistent: most of the path's GEMMs have a short reduction (K = 64..512, i.e. 1..8 K-steps of
// 64), so in a one-tile-per-workgroup kernel every tile pays the full global-load latency of its
// first K-step and the drain of its epilogue with nothing to overlap them.  Here a fixed grid of
// (CUs x resident workgroups) walks a continuous stream of (tile, K-step) pairs: the LDS-DMA for the
// NEXT step — which at a tile boundary is the next tile's first step — is in flight while the MFMAs
// of the current step run, so tile prologues are hidden behind the previous tile's last step.
//
// Staging: `global_load_lds_dwordx4` (no VGPR round trip, no ds_write pass).  The DMA writes each
// wave-instruction's 64 x 16 B lane-linearly, so the LDS image is unpadded [rows][64 k] (128-B rows)
// and the bank-conflict swizzle is applied on the SOURCE address: LDS chunk c' of row r holds global
// 16-B chunk c' ^ (r & 7) — which makes every ds_read_b128 fragment read of the 16x16x32 MFMA
// conflict-free (each 16-lane group hits 16 distinct 16-B bank slots).  K tails read a 16-byte
// zero block instead of the operand (no masking instructions); rows past M / N are clamped (their
// outputs are never stored).
//
// The MFMA is issued as W-fragment x A-fragment, i.e. it computes the tile transposed: each lane
// then holds 4 consecutive output COLUMNS of one row, so the fused epilogue (bias, activation,
// residual in f32, one rounding) stores 8-byte row pieces straight from the accumulators — no LDS
// round trip and no extra barrier at tile boundaries.
//
// Synchronisation per K-step: issue DMA(next) -> s_waitcnt vmcnt(#DMA of next) (own DMA of the
// current step landed) -> s_barrier (everyone's landed) -> fragment reads + MFMAs -> s_barrier
// (nobody still reads the buffer the following step's DMA overwrites).  Raw s_barrier, never
// __syncthreads (its fence would drain the in-flight DMA).  Two stages: the DMA runs one step ahead.
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>
#include <type_traits>

namespace svk {

static __device__ __attribute__((aligned(16))) uint4 g_pk_zero[4];   // 64 zero bytes: the K-tail source

typedef __attribute__((address_space(1))) void* gas_ptr;
typedef __attribute__((address_space(3))) void* las_ptr;

// Tile BM x BN x 64, WGM x WGN waves (each owning a (BM/WGM) x (BN/WGN) sub-tile of 16x16 MFMA
// blocks), an NSTAGE-deep ring of LDS stages (the DMA runs NSTAGE-1 steps ahead).
template <int BM_, int BN_, int WGM_, int WGN_, int NSTAGE_>
struct PkCfg {
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, NSTAGE = NSTAGE_;
  static constexpr int NT = 64 * WGM * WGN;
  static constexpr int BK = 64;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int LDS = NSTAGE * STAGE;
  static constexpr int A_LD = A_BYTES / (NT * 16);   // DMA instructions per thread per K-step
  static constexpr int B_LD = B_BYTES / (NT * 16);
  static constexpr int LD = A_LD + B_LD;
  // resident workgroups per CU the register budget is held to (LDS allows 3 for 128x64 / 64x128, 2 for
  // 128x128): without the bound the f16 epilogue's conversions cost hipcc ~20-40 more VGPRs than the
  // bf16 one and drop a workgroup per CU
  // waves per SIMD the LDS allows (workgroups per CU x waves per workgroup / 4 SIMDs): the register
  // budget __launch_bounds__ holds the kernel to, so hipcc's allocation never costs a resident workgroup
  static constexpr int WG_PER_CU = (160 * 1024) / LDS;
  static constexpr int OCC = WG_PER_CU * NT / 256 > 5 ? 5 : (WG_PER_CU * NT / 256 < 1 ? 1 : WG_PER_CU * NT / 256);
  static constexpr bool ELDS_FITS = BM * BN * 2 <= STAGE;    // the staged epilogue tile fits one stage
  // big tiles (one workgroup per CU, accumulators in the AGPR half of the register file): the epilogue
  // operands are loaded in the epilogue itself, block by block (held early they would not fit)
  static constexpr bool LATE = BM * BN > 128 * 160;
  static_assert(A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "tile must split into whole DMA rounds");
  static_assert(LD <= 63, "vmcnt range");
};

// n / d for 0 <= n < 2^31 by multiply-high (d >= 1); host computes (mul, shr).
struct FastDiv {
  uint32_t mul, shr;
  __device__ __forceinline__ int div(int n) const { return (int)((__umulhi((uint32_t)n, mul) + (uint32_t)n) >> shr); }
};
static FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  return FastDiv{(uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l};
}
// implicit-GEMM conv (ASRC == 1): divisors of the row / column decompositions
struct PkConv { FastDiv hw, ow, cin, kw; };

__device__ __forceinline__ int pk_xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// LDS-DMA issued from inline asm: hipcc does not track it, so it neither drains it with vmcnt(0)
// before fragment reads of another stage nor before the next DMA (cdna_hip_programming.md §5.7);
// completion is counted by hand (vmcnt; loads return in order).  M0 is saved/restored around it.
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// the same from an SGPR base + 32-bit per-lane VGPR offset (dense operands without a K tail, round 5): the
// per-lane offsets are computed once per tile and the K-step advance is a scalar add on the base, so a DMA costs
// no vector address arithmetic (the 64-bit form spent ~8 VALU per DMA instruction on it: gemm_pk issued 6.6 VALU
// per MFMA, 27 us of VALU per SIMD in the 76 us stage-3 fc1, profiles/r05/gemm_fc1_pmc.txt)
__device__ __forceinline__ void dma16s(const char* sbase, uint32_t voff, uint32_t lds_dst) {
  const uint64_t b = reinterpret_cast<uint64_t>(sbase);
  // (readfirstlane returns int: widen through uint32_t — a sign-extended low word would corrupt the high one)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  sbase = reinterpret_cast<const char*>(((uint64_t)hi << 32) | (uint64_t)lo);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void barrier_mem() { asm volatile("s_barrier" ::: "memory"); }
// Epilogue operand loads hidden from hipcc's waitcnt pass (see epi_load): completion is covered by the
// counted wait of the tile's last step.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#ifdef SVK_PK_VISIBLE_EPI   // diagnostic build: compiler-visible epilogue loads
__device__ __forceinline__ void gload16(f32x4& v, const char* src) { v = *reinterpret_cast<const f32x4*>(src); }
__device__ __forceinline__ void gload8(u32x2& v, const char* src) { v = *reinterpret_cast<const u32x2*>(src); }
__device__ __forceinline__ void gload4(float& v, const char* src) { v = *reinterpret_cast<const float*>(src); }
#else
__device__ __forceinline__ void gload16(f32x4& v, const char* src) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(src) : "memory");
}
__device__ __forceinline__ void gload8(u32x2& v, const char* src) {
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(src) : "memory");
}
__device__ __forceinline__ void gload4(float& v, const char* src) {
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(src) : "memory");
}
#endif

// SPLIT: split-K — unit u = (tile u / ks, K part u % ks) covers nk K-steps of the tile's ks * nk; the
// epilogue stores raw f32 partial sums to slab part (p.slab + (part * M + m) * N + n) and a separate
// reduction adds the parts (+ bias, LayerNorm: svk_conv2d_ln_nhwc).
//
// -DSVK_DIAG (libsvk_diag.so, tools only): timing ablations from SVK_PK_DIAG — 1 drain the stores after each
// epilogue, 2 no C stores, 4 no MFMAs (loads, barriers and fragment reads only), 8 every DMA re-reads the
// workgroup's first tile's K-step 0 (L2-hot operands).  The product build has no such path.
#ifdef SVK_DIAG
#define PK_DIAG_PARAM , int diag
#define PK_DIAG_ARG , diag_knob("SVK_PK_DIAG")
#else
#define PK_DIAG_PARAM
#define PK_DIAG_ARG
#endif
// PERM (round 6, EXT only): block j's W fragment rows are permuted so that a lane's two blocks 2p, 2p + 1 hold 8
// CONSECUTIVE output columns (32 p + 8 fq .. + 7) instead of two 4-column pieces 16 apart — the epilogue operands
// (bias, residual, the activation-backward source U) then load as 16-byte pieces, 16 rows x 64 bytes per
// wave-instruction instead of 16 x 32.  Each output is the same MFMA reduction as without it (bit-identical).
template <typename T, class Cfg, bool KTAIL, bool ELDS, int ASRC, bool EXT, bool SPLIT = false, bool PERM = false>
__global__ __launch_bounds__(Cfg::NT, Cfg::OCC)
void gemm_pk(GemmArgs p, PkConv cv, int ntn, int ntiles, int nk, int ks PK_DIAG_PARAM) {
#ifndef SVK_DIAG
  constexpr int diag = 0;
#endif
  typedef v8_t<T> tx8;
  constexpr int BM = Cfg::BM, BN = Cfg::BN, NS = Cfg::NSTAGE;
  constexpr int WM = BM / Cfg::WGM, WN = BN / Cfg::WGN, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(1024))) char smem[Cfg::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WGN, wn = wave % Cfg::WGN;
  const T* A = static_cast<const T*>(p.A);
  const T* Wt = static_cast<const T*>(p.W);
  const int G = gridDim.x;
  const int first = pk_xcd_remap(blockIdx.x, G);
  if (first >= ntiles) return;
  const char* zero = reinterpret_cast<const char*>(g_pk_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;

  // this thread's DMA lane covers 16-byte chunk q = (wave * LD + i) * 64 + lane of the stage image
  // ASRC == 1: im2col rows of this thread's A slots (output pixel -> first input tap), per tile
  int crb[Cfg::A_LD], ciy[Cfg::A_LD], cix[Cfg::A_LD];
  // dense, no K tail: per-lane byte offsets of this thread's A / W chunks within the current issue tile
  // (32-bit: the host routes operands of 4 GiB or more to the KTAIL instantiation)
  constexpr bool SOFF = ASRC == 0 && !KTAIL && !SPLIT && Cfg::BM * Cfg::BN <= 128 * 128;   // (bigger tiles: no registers left)
  uint32_t offA[SOFF ? Cfg::A_LD : 1], offB[SOFF ? Cfg::B_LD : 1];
  // live == false: past the workgroup's last (tile, K-step) — the same instructions run (branch-free
  // around the DMA issue) with every source replaced by the zero block
  // W-tile chunk swizzle: chunk c of tile row r sits at LDS position c ^ swzB(r).  PERM reads rows 32 q + 8 a + b
  // (+ 4) per block: (r & 7) takes 4 values over them (a 4-way bank conflict on every fragment read), so PERM tiles
  // swizzle by ((r >> 1) & 1) | ((r >> 3) & 3) << 1, which is 8 distinct values over each parity's 8 rows
  auto swzB = [](int r) { return PERM ? (((r >> 1) & 1) | (((r >> 3) & 3) << 1)) : (r & 7); };
  auto issue = [&](int unit, int kt, int buf, bool live) {
    if (diag & 8) { unit = first; kt = 0; }
    const int tile = SPLIT ? unit / ks : unit, part = unit - tile * ks;
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN, k0 = (SPLIT ? part * nk + kt : kt) * Cfg::BK;
    const uint32_t sa = lds0 + buf * Cfg::STAGE, sb = sa + Cfg::A_BYTES;
    if constexpr (ASRC == 1) {
      // every A slot of a lane has the same 16-byte chunk column c (rows differ by multiples of 8)
      const int c = (lane & 7) ^ ((lane >> 3) & 7);
      if (kt == 0) {
#pragma unroll
        for (int i = 0; i < Cfg::A_LD; ++i) {
          const int r = ((wave * Cfg::A_LD + i) * 64 + lane) >> 3;
          const int m = m0 + r;
          const int mm = m < p.M ? m : 0;
          const int b = cv.hw.div(mm), rem = mm - b * (p.OH * p.OW);
          const int oy = cv.ow.div(rem), ox = rem - oy * p.OW;
          crb[i] = b * p.H * p.Wd * p.Cin;
          ciy[i] = m < p.M ? oy * p.stride - p.pad : -0x40000000;   // invalid row: every tap out of range
          cix[i] = ox * p.stride - p.pad;
        }
      }
      const int k = k0 + c * 8;
      const int kc = k < p.K ? k : 0;
      const int tap = cv.cin.div(kc), ci = kc - tap * p.Cin;
      const int ti = cv.kw.div(tap), tj = tap - ti * p.kw;
#pragma unroll
      for (int i = 0; i < Cfg::A_LD; ++i) {
        const int iy = ciy[i] + ti, ix = cix[i] + tj;
        const bool ok = k < p.K && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.Wd;
        const char* src = ok && live ? reinterpret_cast<const char*>(A + crb[i] + ((long)iy * p.Wd + ix) * p.Cin + ci) : zero;
        dma16(src, __builtin_amdgcn_readfirstlane(sa + (wave * Cfg::A_LD + i) * 1024));
      }
    } else if constexpr (SOFF) {
      // a new tile's first K-step: the per-lane offsets; past the last unit (live == false) the last live tile's
      // offsets stay and the DMA re-reads its K-step 0 into a stage nobody reads any more (in bounds, no select)
      if (live && (kt == 0 || (diag & 8))) {
#pragma unroll
        for (int i = 0; i < Cfg::A_LD; ++i) {
          const int q = (wave * Cfg::A_LD + i) * 64 + lane;
          const int r = q >> 3, c = (q & 7) ^ (r & 7);
          offA[i] = (uint32_t)min(m0 + r, p.M - 1) * (uint32_t)(p.lda * 2) + c * 16;
        }
#pragma unroll
        for (int i = 0; i < Cfg::B_LD; ++i) {
          const int q = (wave * Cfg::B_LD + i) * 64 + lane;
          const int r = q >> 3, c = (q & 7) ^ swzB(r);
          offB[i] = (uint32_t)min(n0 + r, p.N - 1) * (uint32_t)(p.ldw * 2) + c * 16;
        }
      }
      const long kb = live ? (long)k0 * 2 : 0;
#pragma unroll
      for (int i = 0; i < Cfg::A_LD; ++i)
        dma16s(reinterpret_cast<const char*>(A) + kb, offA[i], sa + (wave * Cfg::A_LD + i) * 1024);
#pragma unroll
      for (int i = 0; i < Cfg::B_LD; ++i)
        dma16s(reinterpret_cast<const char*>(Wt) + kb, offB[i], sb + (wave * Cfg::B_LD + i) * 1024);
      return;
    } else {
#pragma unroll
      for (int i = 0; i < Cfg::A_LD; ++i) {
        const int q = (wave * Cfg::A_LD + i) * 64 + lane;
        const int r = q >> 3, c = (q & 7) ^ (r & 7);
        const int m = min(m0 + r, p.M - 1), k = k0 + c * 8;
        const char* src = reinterpret_cast<const char*>(A + (long)m * p.lda + k);
        if constexpr (KTAIL) src = k < p.K ? src : zero;
        src = live ? src : zero;
        dma16(src, __builtin_amdgcn_readfirstlane(sa + (wave * Cfg::A_LD + i) * 1024));
      }
    }
#pragma unroll
    for (int i = 0; i < Cfg::B_LD; ++i) {
      const int q = (wave * Cfg::B_LD + i) * 64 + lane;
      const int r = q >> 3, c = (q & 7) ^ swzB(r);
      const int n = min(n0 + r, p.N - 1), k = k0 + c * 8;
      const char* src = reinterpret_cast<const char*>(Wt + (long)n * p.ldw + k);
      if constexpr (KTAIL) src = k < p.K ? src : zero;
      src = live ? src : zero;
      dma16(src, __builtin_amdgcn_readfirstlane(sb + (wave * Cfg::B_LD + i) * 1024));
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
    const char* sa = smem + buf * Cfg::STAGE;
    const char* sb = sa + Cfg::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cc = ((ks * 4 + fq) ^ (fr & 7)) * 16;   // swizzled chunk of this lane's 8 k
      tx8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const tx8*>(sa + (wm * WM + i * 16 + fr) * 128 + cc);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (PERM) {
          const int rr = wn * WN + 32 * (j >> 1) + 8 * (fr >> 2) + 4 * (j & 1) + (fr & 3);
          fb[j] = *reinterpret_cast<const tx8*>(sb + rr * 128 + (((ks * 4 + fq) ^ swzB(rr)) * 16));
        } else {
          fb[j] = *reinterpret_cast<const tx8*>(sb + (wn * WN + j * 16 + fr) * 128 + cc);
        }
      }
      if (diag & 4) {                   // (diagnostic build) keep the fragment reads alive, skip the MFMAs
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(fb[j]));
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);
    }
  };

  // Epilogue operands (bias, residual, and for EXT the activation-backward source and the row scale)
  // are loaded BEFORE the tile's last K-step, so their latency hides behind that step's DMA wait and
  // MFMAs.  They are issued from inline asm like the DMA: a compiler-visible global_load would make
  // hipcc's waitcnt pass (which cannot see the asm DMA) insert s_waitcnt vmcnt(0) before the next
  // reuse of its registers — draining the NEXT tile's prefetch at every tile.  Being older than that
  // prefetch, they are covered by the last step's counted wait (vector-memory operations, LDS-DMA
  // included, retire in issue order), after which tie_epi() hands the registers back to the compiler.  Absent operands read the zero block (no branches).
  // Lane holds C[m][n .. n+3]: m = row fr of block i, n = 4 fq + r of block j (transposed MFMA).
  constexpr bool LATE = Cfg::LATE;
  static_assert(!(LATE && (EXT || SPLIT)), "big tiles: plain epilogue only");
  static_assert(!PERM || (ASRC == 0 && !LATE && !SPLIT && WN % 32 == 0), "PERM: dense tiles with 32-column wave slices");
  // output column of block j, accumulator r: n0 + wn WN + colj(j) + r
  auto colj = [&](int j) { return PERM ? 32 * (j >> 1) + 8 * fq + 4 * (j & 1) : j * 16 + fq * 4; };
  f32x4 ebias[LATE ? 1 : TN];
  u32x2 eres[LATE || PERM ? 1 : TM][LATE || PERM ? 1 : TN], eu[EXT && !PERM ? TM : 1][EXT && !PERM ? TN : 1];
  f32x4 eres4[PERM ? TM : 1][PERM ? TN / 2 : 1], eu4[PERM && EXT ? TM : 1][PERM && EXT ? TN / 2 : 1];   // 8 columns each
  float ers[EXT ? TM : 1];
  const T* R = static_cast<const T*>(p.R);
  auto epi_load = [&](int unit) {
    if constexpr (PERM) {
      const int m0 = (unit / ntn) * BM, n0 = (unit % ntn) * BN;
      const char* zero = reinterpret_cast<const char*>(g_pk_zero);
      const T* U = static_cast<const T*>(p.U);
#pragma unroll
      for (int q = 0; q < TN / 2; ++q) {
        const int n = min(n0 + wn * WN + 32 * q + 8 * fq, p.N - 8);   // host: N % 8 == 0
        gload16(ebias[2 * q], p.bias ? reinterpret_cast<const char*>(p.bias + n) : zero);
        gload16(ebias[2 * q + 1], p.bias ? reinterpret_cast<const char*>(p.bias + n + 4) : zero);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = min(m0 + wm * WM + i * 16 + fr, p.M - 1);
          gload16(eres4[i][q], R ? reinterpret_cast<const char*>(R + (long)m * p.ldr + n) : zero);
          if constexpr (EXT) gload16(eu4[i][q], U ? reinterpret_cast<const char*>(U + (long)m * p.ldu + n) : zero);
        }
      }
      if constexpr (EXT) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = min(m0 + wm * WM + i * 16 + fr, p.M - 1);
          gload4(ers[i], p.rscale ? reinterpret_cast<const char*>(p.rscale + m / p.rdiv) : zero);
        }
      }
    } else if constexpr (!SPLIT && !LATE) {
      const int m0 = (unit / ntn) * BM, n0 = (unit % ntn) * BN;
      const char* zero = reinterpret_cast<const char*>(g_pk_zero);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = min(n0 + wn * WN + j * 16 + fq * 4, p.N - 4);
        gload16(ebias[j], p.bias ? reinterpret_cast<const char*>(p.bias + n) : zero);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = min(m0 + wm * WM + i * 16 + fr, p.M - 1);
          gload8(eres[i][j], R ? reinterpret_cast<const char*>(R + (long)m * p.ldr + n) : zero);
          if constexpr (EXT) {
            const T* U = static_cast<const T*>(p.U);
            gload8(eu[i][j], U ? reinterpret_cast<const char*>(U + (long)m * p.ldu + n) : zero);
          }
        }
      }
      if constexpr (EXT) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = min(m0 + wm * WM + i * 16 + fr, p.M - 1);
          gload4(ers[i], p.rscale ? reinterpret_cast<const char*>(p.rscale + m / p.rdiv) : zero);
        }
      }
    }
  };
  auto tie_epi = [&]() {
    if constexpr (LATE) return;
    if constexpr (PERM) {
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(ebias[j]));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          asm volatile("" : "+v"(eres4[i][q]));
          if constexpr (EXT) asm volatile("" : "+v"(eu4[i][q]));
        }
      if constexpr (EXT) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(ers[i]));
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      asm volatile("" : "+v"(ebias[j]));
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        asm volatile("" : "+v"(eres[i][j]));
        if constexpr (EXT) asm volatile("" : "+v"(eu[i][j]));
      }
    }
    if constexpr (EXT) {
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(ers[i]));
    }
  };
  constexpr int CPR = BN / 8;            // 16-byte chunks per staged output row
  char* stile = nullptr;                  // ELDS: stage buffer consumed by the tile's last step
  // EXT (training): v = act(acc + bias) * rscale[m / rdiv] * uact'(U[m, n]) + R[m, n]; the template
  // activation is then the BACKWARD one (uact), the forward act stays a runtime switch.
  auto epilogue = [&](int unit, auto act_c) {
    constexpr int ACT = decltype(act_c)::value;
    const int tile = SPLIT ? unit / ks : unit, part = unit - tile * ks;
    const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
    if constexpr (SPLIT) {   // raw partial sums, 16-byte f32 stores (N % 4 == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + fq * 4;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = m0 + wm * WM + i * 16 + fr;
          if (m < p.M && n < p.N) *reinterpret_cast<f32x4*>(p.slab + ((long)part * p.M + m) * p.N + n) = acc[i][j];
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      return;
    }
    T* C = static_cast<T*>(p.C);
    if constexpr (EXT) {
      if (!p.rscale) {
#pragma unroll
        for (int i = 0; i < TM; ++i) ers[i] = 1.f;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + colj(j);
      f32x4 bj;
      if constexpr (LATE) {
        const int nb = min(n, p.N - 4);
        bj = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + nb) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        bj = ebias[j];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * WM + i * 16 + fr;
        u32x2 rij;
        if constexpr (LATE) {
          rij = R ? *reinterpret_cast<const u32x2*>(R + (long)min(m, p.M - 1) * p.ldr + min(n, p.N - 4)) : u32x2{0u, 0u};
        } else if constexpr (PERM) {
          const f32x4 r4 = eres4[i][j >> 1];
          rij = (j & 1) ? u32x2{__float_as_uint(r4.z), __float_as_uint(r4.w)} : u32x2{__float_as_uint(r4.x), __float_as_uint(r4.y)};
        } else {
          rij = eres[i][j];
        }
        float v[4] = {acc[i][j][0] + bj.x, acc[i][j][1] + bj.y, acc[i][j][2] + bj.z, acc[i][j][3] + bj.w};
        if constexpr (EXT) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act_fast(v[e], p.act) * ers[i];
          if (p.U) {
            u32x2 uij;
            if constexpr (PERM) {
              const f32x4 u4 = eu4[i][j >> 1];
              uij = (j & 1) ? u32x2{__float_as_uint(u4.z), __float_as_uint(u4.w)} : u32x2{__float_as_uint(u4.x), __float_as_uint(u4.y)};
            } else {
              uij = eu[i][j];
            }
            const f32x2 u01 = unpack2<T>(uij.x), u23 = unpack2<T>(uij.y);
            v[0] *= act_grad(u01.x, ACT);
            v[1] *= act_grad(u01.y, ACT);
            v[2] *= act_grad(u23.x, ACT);
            v[3] *= act_grad(u23.y, ACT);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act_fast(v[e], ACT);
        }
        {                                  // zero block when there is no residual
          const f32x2 r01 = unpack2<T>(rij.x), r23 = unpack2<T>(rij.y);
          v[0] += r01.x;
          v[1] += r01.y;
          v[2] += r23.x;
          v[3] += r23.y;
        }
        T o[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
        if constexpr (ELDS) {
          const int row = wm * WM + i * 16 + fr, col = wn * WN + colj(j);
          *reinterpret_cast<uint2*>(stile + row * (BN * 2) + (((col >> 3) ^ (row & (CPR - 1))) << 4) + ((col >> 2) & 1) * 8) =
              *reinterpret_cast<const uint2*>(o);
        } else if (m < p.M && n < p.N && !(diag & 2)) {   // N % 4 == 0: a 4-column group is all-in or all-out
          *reinterpret_cast<uint2*>(C + (long)m * p.ldc + n) = *reinterpret_cast<const uint2*>(o);
        }
      }
    }
    if constexpr (ELDS) {
      // the tile, staged as bf16 rows in the stage buffer just consumed, leaves as whole 16-byte row
      // chunks (a wave stores 4 full 256-byte rows per instruction instead of 16 x 32-byte pieces);
      // the raw barrier does not wait for this wave's LDS writes, so retire them first
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_mem();
#pragma unroll
      for (int it = 0; it < (BM * CPR) / Cfg::NT; ++it) {
        const int idx = tid + it * Cfg::NT;
        const int row = idx / CPR, c = idx % CPR;
        const uint4 v = *reinterpret_cast<const uint4*>(stile + row * (BN * 2) + ((c ^ (row & (CPR - 1))) << 4));
        const int m = m0 + row, n = n0 + c * 8;
        if (m < p.M && n < p.N && !(diag & 2)) {
          *reinterpret_cast<uint4*>(C + (long)m * p.ldc + n) = v;
        }
      }
      barrier_mem();   // the next step's DMA overwrites this stage buffer
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // DMA issue cursor: the (tile, K-step) stream of this workgroup.  Every step issues exactly LD
  // LDS-DMA instructions — the next (tile, K-step)'s, or, past the last one, LD copies of the zero block
  // into a stage buffer nobody reads any more — so each wait is ONE unconditional counted
  // `s_waitcnt vmcnt(n)`: no data-dependent branch around it, and the epilogue loads have provably
  // landed before their registers are touched (csrc/isa_check.py audits this on the built code object,
  // counting the vector-memory operations issued after each load on every path).
  static_assert((NS - 1) * Cfg::LD <= 63, "vmcnt range");
  int itile = first, ikt = 0, ibuf = 0, buf = 0;
  auto issue_next = [&]() {
    const bool live = itile < ntiles;
    issue(live ? itile : first, live ? ikt : 1, ibuf, live);
    if (live && ++ikt == nk) { ikt = 0; itile += G; }
    ibuf = ibuf + 1 == NS ? 0 : ibuf + 1;
  };
  // One pipeline step: top up the DMA ring (into the stage computed one step ago), wait for the
  // oldest stage `buf` (the NS - 1 steps issued after it may stay in flight), compute from it.  The
  // epilogue operands of a tile are issued just before the DMA of its step nk - EA (EA = min(NS - 1, 2)
  // steps before its last step), and the last step's wait leaves only the EA youngest DMA steps in flight,
  // so it retires them (the host keeps nk >= EA).  (Round 6: with deeper rings the operands held NS - 1 steps
  // made hipcc move their registers before the wait — isa_check; two steps is what the 3-stage ring always
  // used, and the deep rings pay a shallower wait once per tile.)
  constexpr int EA = NS - 1 < 2 ? NS - 1 : 2;
  auto step = [&](bool last) {
    issue_next();
    if (last) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EA * Cfg::LD) : "memory");
      tie_epi();                       // the epilogue loads are older than the EA steps still in flight
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * Cfg::LD) : "memory");
    }
    barrier_mem();
    compute(buf);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_mem();                     // nobody still reads `buf` when a later DMA overwrites it
    stile = smem + buf * Cfg::STAGE;
    buf = buf + 1 == NS ? 0 : buf + 1;
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue_next();
  for (int tile = first; tile < ntiles; tile += G) {
    for (int kt = 0; kt < nk - 1; ++kt) {
      if (EA > 1 && kt == nk - EA) epi_load(tile);    // (NS > 2) fly during the last EA steps
      step(false);
    }
    if (EA == 1) epi_load(tile);      // epilogue operands fly during the last step's wait and MFMAs
    step(true);
    switch (EXT ? p.uact : p.act) {
      case SVK_ACT_GELU: epilogue(tile, std::integral_constant<int, SVK_ACT_GELU>{}); break;
      case SVK_ACT_RELU: epilogue(tile, std::integral_constant<int, SVK_ACT_RELU>{}); break;
      case SVK_ACT_TANH: epilogue(tile, std::integral_constant<int, SVK_ACT_TANH>{}); break;
      default: epilogue(tile, std::integral_constant<int, 0>{}); break;
    }
    if (diag & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (diagnostic build) drain the stores
  }
  // the last step's zero-block DMA is still in flight: retire it before the wave (and the workgroup's
  // LDS allocation) ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- host side -------------------------------------------------------------------------------
static int pk_slots(const void* fn, int nt) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, nt, 0);
  return std::max(1, cus) * std::max(1, per);
}

template <typename T, class Cfg, bool KTAIL, bool ELDS, int ASRC, bool EXT, bool SPLIT = false, bool PERM = false>
static int launch_pk(const GemmArgs& a, hipStream_t st) {
  const int ntm = (a.M + Cfg::BM - 1) / Cfg::BM, ntn = (a.N + Cfg::BN - 1) / Cfg::BN;
  const int ks = SPLIT ? a.ksplit : 1;
  const long ntiles = (long)ntm * ntn * ks;
  const int nk = (a.K + 63) / 64 / ks;   // K-steps per unit (the caller makes ks divide them)
  constexpr int EA = Cfg::NSTAGE - 1 < 2 ? Cfg::NSTAGE - 1 : 2;
  if (nk < EA) {                          // the epilogue loads are issued EA - 1 steps before a tile's last
    set_error("gemm_pk: %d K-steps per tile, the %d-stage ring needs %d", nk, Cfg::NSTAGE, EA);
    return SVK_EUNSUPPORTED;
  }
  static const int slots =
      pk_slots(reinterpret_cast<const void*>(&gemm_pk<T, Cfg, KTAIL, ELDS, ASRC, EXT, SPLIT, PERM>), Cfg::NT);
  const int grid = (int)std::min<long>(ntiles, slots);
  PkConv cv{};
  if (ASRC == 1) {
    cv.hw = make_fastdiv((uint32_t)(a.OH * a.OW));
    cv.ow = make_fastdiv((uint32_t)a.OW);
    cv.cin = make_fastdiv((uint32_t)a.Cin);
    cv.kw = make_fastdiv((uint32_t)a.kw);
  }
  hipLaunchKernelGGL((gemm_pk<T, Cfg, KTAIL, ELDS, ASRC, EXT, SPLIT, PERM>), dim3(grid), dim3(Cfg::NT), 0, st, a, cv, ntn,
                     (int)ntiles, nk, ks PK_DIAG_ARG);
  static char name[112];
  // the demangled instantiation name without PERM: a PERM launch is the same kernel family for the profiles
  // (tools/pmc_traffic.py kernel_key folds the argument the same way)
  if (!name[0])
    snprintf(name, sizeof(name), "gemm_pk<%s, PkCfg<%d, %d, %d, %d, %d>, %s, %s, %d, %s, %s>", type_name<T>(), Cfg::BM, Cfg::BN,
             Cfg::WGM, Cfg::WGN, Cfg::NSTAGE, KTAIL ? "true" : "false", ELDS ? "true" : "false", ASRC,
             EXT ? "true" : "false", SPLIT ? "true" : "false");
  set_last_kernel(name);
  return check_launch("gemm_pk");
}

// PERM (16-byte epilogue operand pieces, bit-identical): 2 = EXT and plain-residual tiles (default; extraction step
// 6.774 -> 6.715 ms, train 13.59 -> 13.48 same-box, profiles/r06/ext_perm_ab.txt), 1 = EXT only, 0 = off
static const int g_pk_perm = getenv("SVK_PK_PERM") ? atoi(getenv("SVK_PK_PERM")) : 2;
template <typename T, class Cfg, int ASRC>
static int launch_pk_k(const GemmArgs& a, hipStream_t st, bool elds) {
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (g_tune[TUNE_PK_ELDS] >= 0) elds = g_tune[TUNE_PK_ELDS];
  // the staged epilogue swizzles 16-byte chunks within a power-of-two row of chunks, in one stage buffer
  elds = elds && Cfg::ELDS_FITS && (Cfg::BN & (Cfg::BN - 1)) == 0 && a.N % 8 == 0 && a.ldc % 8 == 0 && al16(a.C);
  // (the K-tail instantiation also takes operands whose byte offsets do not fit 32 bits: the dense no-tail path
  // addresses its DMA as SGPR base + 32-bit lane offset)
  const bool big = ASRC == 0 && ((long)a.M * a.lda * 2 >= 0xffffffffL || (long)a.N * a.ldw * 2 >= 0xffffffffL);
  const bool tail = a.K % 64 != 0 || big, ext = a.rscale || a.U;
  // the extended (training) epilogue holds two more operand sets: with 8 waves or 3 stages it spills, so
  // it runs on the 4-wave two-stage 128 x 128 tile
  constexpr bool EXT_OK = Cfg::NT == 256 && Cfg::NSTAGE == 2 && Cfg::BM * Cfg::BN <= 128 * 128;
  if constexpr (ASRC == 1) {
    // the im2col loader zero-fills the A side of a K tail itself, but the weight rows must read the
    // zero block too: the last row's tail would otherwise read past the packed weights, and 0 x a
    // NaN bit pattern found there is NaN.  No extended epilogue for convs.
    if constexpr (Cfg::ELDS_FITS) {
      if (elds) return tail ? launch_pk<T, Cfg, true, true, 1, false>(a, st) : launch_pk<T, Cfg, false, true, 1, false>(a, st);
    }
    return tail ? launch_pk<T, Cfg, true, false, 1, false>(a, st) : launch_pk<T, Cfg, false, false, 1, false>(a, st);
  } else {
    if (ext) {
      if constexpr (!EXT_OK) {
        return launch_pk_k<T, PkCfg<128, 128, 2, 2, 2>, ASRC>(a, st, elds);
      } else {
        // PERM: 16-byte epilogue operand pieces (bias, R, U 16-byte aligned with N, ldr, ldu % 8 == 0)
        // (64 x 64: the PERM epilogue needs one VGPR more than its 5-workgroup occupancy allows — not instantiated)
        constexpr bool PERM_OK = (Cfg::BN / Cfg::WGN) % 32 == 0 && Cfg::BM * Cfg::BN >= 128 * 64;
        const bool perm = g_pk_perm && PERM_OK && a.N % 8 == 0 && (!a.bias || al16(a.bias)) &&
                          (!a.R || (al16(a.R) && a.ldr % 8 == 0)) && (!a.U || (al16(a.U) && a.ldu % 8 == 0));
        if constexpr (PERM_OK) {
          if (perm) {
            if constexpr (Cfg::ELDS_FITS) {
              if (elds) return tail ? launch_pk<T, Cfg, true, true, 0, true, false, true>(a, st)
                                    : launch_pk<T, Cfg, false, true, 0, true, false, true>(a, st);
            }
            return tail ? launch_pk<T, Cfg, true, false, 0, true, false, true>(a, st)
                        : launch_pk<T, Cfg, false, false, 0, true, false, true>(a, st);
          }
        }
        if constexpr (Cfg::ELDS_FITS) {
          if (elds) return tail ? launch_pk<T, Cfg, true, true, 0, true>(a, st) : launch_pk<T, Cfg, false, true, 0, true>(a, st);
        }
        return tail ? launch_pk<T, Cfg, true, false, 0, true>(a, st) : launch_pk<T, Cfg, false, false, 0, true>(a, st);
      }
    }
    // PERM for the plain residual epilogue (SVK_PK_PERM=2, the default)
    {
      constexpr bool PERM_OK = Cfg::NSTAGE == 2 && !Cfg::LATE && (Cfg::BN / Cfg::WGN) % 32 == 0 && Cfg::BM * Cfg::BN >= 128 * 64;
      if constexpr (PERM_OK) {
        if (g_pk_perm == 2 && a.R && a.N % 8 == 0 && (!a.bias || al16(a.bias)) && al16(a.R) && a.ldr % 8 == 0) {
          if constexpr (Cfg::ELDS_FITS) {
            if (elds) return tail ? launch_pk<T, Cfg, true, true, 0, false, false, true>(a, st)
                                  : launch_pk<T, Cfg, false, true, 0, false, false, true>(a, st);
          }
          return tail ? launch_pk<T, Cfg, true, false, 0, false, false, true>(a, st)
                      : launch_pk<T, Cfg, false, false, 0, false, false, true>(a, st);
        }
      }
    }
    if constexpr (Cfg::ELDS_FITS) {
      if (elds) return tail ? launch_pk<T, Cfg, true, true, 0, false>(a, st) : launch_pk<T, Cfg, false, true, 0, false>(a, st);
    }
    // deep rings keep the register epilogue's operands in flight NSTAGE - 1 steps: hipcc then moves those
    // registers before the counted wait retires them (isa_check), so deep rings run with the staged epilogue only
    if constexpr (Cfg::NSTAGE > 2) {
      return launch_pk_k<T, PkCfg<128, 128, 2, 2, 2>, ASRC>(a, st, elds);
    } else {
      return tail ? launch_pk<T, Cfg, true, false, 0, false>(a, st) : launch_pk<T, Cfg, false, false, 0, false>(a, st);
    }
  }
}

// Eligible: bf16, K-contiguous operands (16-byte aligned rows, K % 8 == 0; conv: Cin % 8 == 0),
// plain epilogue, C / R rows 8-byte aligned with N % 4 == 0, bias 16-byte aligned.  Returns 1 when
// not eligible.  asrc: 0 dense A, 1 implicit-GEMM conv (A = NHWC map, GemmArgs conv geometry).
static const int g_pk_policy = getenv("SVK_PK_POLICY") ? atoi(getenv("SVK_PK_POLICY")) : 1;   // 0: round-2 picks
// gemm_pp by policy: off by default — faster in isolation on its shapes, but the graph-replayed extraction step
// ran 8.60 ms with it vs 8.42 ms without (same box, profiles/r04/bench_pp_ab.txt): one 128 KiB-LDS workgroup per
// CU for the whole persistent launch leaves no room for the side stream's kernels to co-run
static const int g_pp_policy = getenv("SVK_PP") ? atoi(getenv("SVK_PP")) : 0;
static const int g_pk_ext_policy = getenv("SVK_PK_EXT_POLICY") ? atoi(getenv("SVK_PK_EXT_POLICY")) : 1;  // A/B switch
template <typename T>
int gemm_pk_try(const GemmArgs& a, hipStream_t st, int asrc) {
  const int force = g_tune[TUNE_PK_CFG];
  if (getenv("SVK_NO_PK")) return 1;
  auto al = [](const void* q, int b) { return ((uintptr_t)q & (b - 1)) == 0; };
  // the reason a call misses this path is kept for the fallback kernel's name (profiling: svk_last_kernel)
  auto no = [](const char* why) { set_pk_reject(why); return 1; };
  if (a.K % 8) return no("K%8");
  if (a.N % 4) return no("N%4");
  if (a.ldw % 8) return no("ldw%8");
  if (a.ldc % 4 || (a.R && a.ldr % 4)) return no("ldc/ldr%4");
  if (a.out_mode) return no("out_mode");
  if (a.U && (a.ldu % 4 || !al(a.U, 8))) return no("U align");
  if (asrc != 0 && (a.U || a.rscale)) return no("conv+U/rscale");
  if (asrc == 0 && a.lda % 8) return no("lda%8");
  if (asrc == 1 && (a.Cin % 8 || (long)a.H * a.Wd * a.Cin * (a.M / (a.OH * a.OW)) > 0x7fffffffL)) return no("conv geometry");
  if (!al(a.A, 16)) return no("A align");
  if (!al(a.W, 16)) return no("W align");
  if (!al(a.C, 8) || (a.R && !al(a.R, 8))) return no("C/R align");
  if (a.bias && !al(a.bias, 16)) return no("bias align");
  int cfg = force;
  // Measured on the MiT-b2 B = 256 shapes, all variants interleaved in one process
  // (tools/tune_bench.py, profiles/r01/tune_r01.txt):
  //  * dense, long K (>= 512) with N % 128 == 0, or few rows (M < 32k, e.g. the stage-4 / head GEMMs
  //    at M = 12544): 128 x 128 tiles with the register epilogue;
  //  * every other dense shape (short K: output-write-bound): 128 x 64 with the LDS-staged epilogue;
  //  * implicit-GEMM convs: 128 x 128 never wins (the im2col DMA address math per tile is the cost);
  //    64 x 64 when the 128-row tiling leaves < 512 tiles and N <= 128 (the k = s patchify convs of
  //    the sequence reduction: 98 row tiles at B = 256), 64 x 128 for N % 128 == 0, else 128 x 64.
  const bool big = a.K >= 512 && a.N % 128 == 0;
  if (cfg < 0) {
    if (asrc == 1) {
      const long t128 = (long)((a.M + 127) / 128) * ((a.N + 63) / 64);
      cfg = (t128 < 512 && a.N <= 128) ? 30 : (a.N % 128 == 0 ? 20 : 10);
      // round 4 (profiles/r04/conv_bench.log, B = 256): 128 x 128 now wins the long-K convs with N % 128 == 0 —
      // stage-2 patch embed 67.3 -> 57.9 us, stage-4 patch embed 72.7 -> 64.5 us
      if (g_pk_policy && cfg == 20 && a.K >= 512) cfg = 0;
    } else {
      cfg = (big || (a.N % 128 == 0 && a.M < 32768)) ? 0 : 10;
      // round 3 (profiles/r03/pk_cfg_sweep_elds.txt): 128 x 128 with the LDS-staged epilogue beats both the
      // register-epilogue 128 x 128 and 128 x 64 wherever N % 128 == 0 and K >= 320 (s3 kv 15.7 -> 13.7 us,
      // s4 fc1 50 -> 43, s4 kv 33 -> 29, s2 fc2 79 -> 70, head 80 -> 77, s3 fc1 91 -> 80)
      if (g_pk_policy && a.N % 128 == 0 && a.K >= 320) cfg = 60;
      // round 4: the 256 x 256 ping-pong kernel (gemm_pp, paired DMA schedule) where its faster tile is neither
      // short of tiles (< 192: most CUs idle, e.g. s4 fc2 / q at N = 512) nor lost to a last partial round:
      // one round, long K, or >= 90 % full rounds (MiT-b2 B = 256: head 75.3 -> 71.7 us, s3 fc1 79.7 -> 71.9,
      // s4 kv 27.9 -> 25.0; s4 fc1 (K = 512, 392 tiles) stays on 128 x 128, profiles/r04/pk_cfg_sweep_pp.txt)
      if (g_pp_policy && a.N % 256 == 0 && a.M >= 8192 && a.K >= 320) {
        const long t256 = (long)((a.M + 255) / 256) * (a.N / 256);
        const long rounds = (t256 + 255) / 256;
        if (t256 >= 192 && (t256 <= 256 || a.K >= 1024 || t256 * 10 >= rounds * 256 * 9)) cfg = 71;
      }
      // (round-2 sweep: 128 x 128 for the stage-3 fc1 and 128 x 160 for its fc2 win 5-7 us each in
      // isolation but lost 2 % of the whole graph-replayed step: kept 128 x 64)
      // round 6, extended epilogue (train backward: DropPath row scale / activation backward from a saved
      // pre-activation; profiles/r06/ext_sweep.txt, bf16 B = 88): the extra U operand makes the register
      // epilogue of 128 x 128 the slowest tile everywhere; 64 x 64 wins where 128 x 128 would leave < 1024 tiles
      // (4312 x 512 x 2048: 30.8 -> 22.5 us, 68992 x 128 x 512: 34.1 -> 30.3), 128 x 64 elsewhere
      // (17248 x 1280 x 320: 49.7 -> 47.2)
      if (g_pk_policy && g_pk_ext_policy && (a.U || a.rscale)) {
        const long t128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128);
        cfg = (a.N % 128 == 0 && t128 < 1024) ? 30 : 10;
      }
    }
  }
  const bool reg_epi = cfg == 0 && (big || a.M < 32768);
  // cfg: 0 = 128x128, 10 = 128x64, 20 = 64x128, 30 = 64x64, 40 = 128x160 (N % 160 == 0), 50 = 256x128 (8 waves).
  // Round-3 sweep (profiles/r03/pk_cfg_sweep.txt, every variant interleaved in one process): three-stage
  // rings (256x128 / 128x64 / 128x128 / 128x256-8-wave) never beat the two-stage tiles on the MiT-b2 shapes
  // and 256x256 with 8 waves spills (128 accumulator + 96 epilogue-operand VGPRs): not instantiated.  The
  // kernel keeps NSTAGE generic (epilogue loads issued min(NSTAGE - 1, 2) steps before a tile's last step).
  if (cfg == 40 && a.N % 160 != 0) cfg = 10;
  // 90 / 91 / 92 / 93: the wide-tile kernel (gemm_wt.hip: 256 x 256 / 256 x 160 / 256 x 128 / 256 x 192)
  if (asrc == 0 && cfg >= 90 && cfg <= 93 && gemm_wt_try<T>(a, st, cfg - 90) == 0) return 0;
  if (cfg >= 90 && cfg <= 93) cfg = 60;
  // 70 / 71 / 72: the 256 x 256 ping-pong kernel (gemm_pp.hip: first / deep DMA schedule / deep + stream-K)
  if (asrc == 0 && cfg >= 70 && cfg <= 72 && gemm_pp_try<T>(a, st, cfg - 70) == 0) return 0;
  if (cfg >= 70 && cfg <= 72) cfg = 60;
  if (asrc == 1) {
    switch (cfg) {
      case 10: return launch_pk_k<T, PkCfg<128, 64, 2, 2, 2>, 1>(a, st, !big);
      case 20: return launch_pk_k<T, PkCfg<64, 128, 2, 2, 2>, 1>(a, st, !big);
      case 30: return launch_pk_k<T, PkCfg<64, 64, 2, 2, 2>, 1>(a, st, !big);
      // (128 x 160 for the N = 320 patch embed: 74.5 vs 88 us in isolation, profiles/r05/conv_sweep.txt, but the
      // conv instantiation spills 2 VGPRs — rejected by isa_check: scratch beside counted DMA waits)
      default: return launch_pk_k<T, PkCfg<128, 128, 2, 2, 2>, 1>(a, st, !reg_epi);
    }
  }
  switch (cfg) {
    case 10: return launch_pk_k<T, PkCfg<128, 64, 2, 2, 2>, 0>(a, st, !big);
    case 20: return launch_pk_k<T, PkCfg<64, 128, 2, 2, 2>, 0>(a, st, !big);
    case 30: return launch_pk_k<T, PkCfg<64, 64, 2, 2, 2>, 0>(a, st, !big);
    case 40: return launch_pk_k<T, PkCfg<128, 160, 2, 2, 2>, 0>(a, st, false);
    case 50: return launch_pk_k<T, PkCfg<256, 128, 4, 2, 2>, 0>(a, st, false);
    case 60: return launch_pk_k<T, PkCfg<128, 128, 2, 2, 2>, 0>(a, st, true);   // 128 x 128, staged epilogue
    // (round 6, measured and not instantiated — profiles/r06/pk_cfg_sweep_*.txt, DESIGN §5: 8-wave 128 x 128 at
    // 2 / 1 workgroups per CU with 2-5-stage rings, 8-wave 128 x 256 with 2 / 3 stages, 4-wave 192 x 128: none beats
    // this 128 x 128 staged-epilogue tile on the MiT-b2 shapes; the deep rings lost 15-25 %, 192 x 128 up to 70 %)
    // (256 x 256 with 4 waves: 512 registers and ~15 VGPR spills, which the counted DMA waits cannot tolerate;
    // 256 x 128 / 128 x 256 at one wave per SIMD run 2-4x slower than 128 x 128, and 256 x 256 with 8 waves of
    // 128 x 64 (225 VGPRs, one workgroup per CU) 1.2-2x slower: per-tile prologue / epilogue / store drain
    // are no longer covered by a second workgroup; not instantiated)
    default: return launch_pk_k<T, PkCfg<128, 128, 2, 2, 2>, 0>(a, st, !reg_epi);
  }
}

// Split-K implicit-GEMM conv into f32 partial slabs (a.ksplit parts, a.slab [ksplit][M][N]): for the
// k = s patchify convs of the sequence reduction, whose 98-row-tile grids (B = 256) cannot fill the
// chip with a long K (2048 / 4096).  Returns 1 when not eligible.
template <typename T>
int gemm_pk_conv_splitk(const GemmArgs& a, hipStream_t st) {
  auto al = [](const void* q, int b) { return ((uintptr_t)q & (b - 1)) == 0; };
  if (a.ksplit < 2 || !a.slab || a.K % 64 || ((a.K / 64) % a.ksplit) || a.N % 4 || a.Cin % 8 || !al(a.A, 16) ||
      !al(a.W, 16) || !al(a.slab, 16) || (long)a.H * a.Wd * a.Cin * (a.M / (a.OH * a.OW)) > 0x7fffffffL)
    return 1;
  if (a.N <= 128 && splitk_bm() == 64) return launch_pk<T, PkCfg<64, 64, 2, 2, 2>, false, false, 1, false, true>(a, st);
  return launch_pk<T, PkCfg<128, 64, 2, 2, 2>, false, false, 1, false, true>(a, st);
}

// one element type per translation unit (gemm_pk_bf16.hip / gemm_pk_f16.hip define SVK_PK_T): the two
// halves of the instantiation set compile in parallel
template int gemm_pk_try<SVK_PK_T>(const GemmArgs&, hipStream_t, int);
template int gemm_pk_conv_splitk<SVK_PK_T>(const GemmArgs&, hipStream_t);

}  // namespace svk
