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
// (16 KiB) per 32 MFMAs — with both workgroups of a CU computing, that is the LDS's whole 256 B/clk at the MFMA
// rate.  Here one 256-thread workgroup per CU owns a (32 TM) x (32 TN) tile as 2 x 2 waves of (16 TM) x (16 TN):
// at TM = TN = 8 a wave reads 16 fragment vectors per 64 MFMAs (4x the reuse) and the 256 accumulator registers
// sit in the AGPR half of the register file.
//
// Pipeline (measured: with one whole 64-deep K-tile issued at the top of each K-tile the LDS-DMA landing time was
// exposed every K-tile; 32-deep stages in a 4-deep ring were slower still — each DMA wave-instruction then covers
// 16 rows x 64 B, twice the cache-line requests per byte, and the chip's LDS-DMA rate is request-bound):
//  * 64-deep stages (128-byte rows, the gemm_pk image: chunk c of row r in slot c ^ (r & 7), conflict-free
//    ds_read_b128 fragments), a ring of NS = 160 KiB / stage stages (2 at 256 x 256 / 256 x 192, 3 at
//    256 x 160 / 256 x 128), filled by LDS-DMA (`global_load_lds_dwordx4`);
//  * one barrier per stage, in the MIDDLE: after the reads of stage u are all issued (row group 2 TM - 2 of the
//    2 TM (k-step, row block) groups) every wave waits for its share of stage u + 1, then the barrier; behind it
//    stage u's slot is refilled (DMA of stage u + NS, spread over the next stage's row groups: an LDS-DMA issue
//    costs ~60 cycles among MFMAs) and the k-step-0 fragments of stage u + 1 are read under the MFMAs of stage u's
//    last row group — the matrix pipe does not wait for LDS at stage boundaries;
//  * persistent: the grid (one workgroup per CU) walks its tiles; the next tile's first stages are in flight
//    during the current tile's last ones and its epilogue;
//  * transposed MFMA (W fragment x A fragment): each lane holds 4 consecutive output columns of a row; the
//    epilogue (bias, activation, residual in f32, one rounding) stores 8-byte row pieces from the accumulators.
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>
#include <type_traits>

namespace svk {
namespace wt {

static __device__ __attribute__((aligned(16))) uint4 g_zero[4];   // 64 zero bytes: K tails, padding DMA

typedef __attribute__((address_space(3))) void* las_ptr;

template <int TM_, int TN_, int NS_>
struct Cfg {
  static constexpr int TM = TM_, TN = TN_, NS = NS_;
  static constexpr int WM = 16 * TM, WN = 16 * TN, BM = 2 * WM, BN = 2 * WN, BK = 64, NT = 256;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  // DMA wave-instructions (1 KiB each) of one stage, dealt round-robin to the 4 waves
  static constexpr int NI_A = A_BYTES / 1024, NI_B = B_BYTES / 1024;
  static constexpr int LDA = NI_A / 4, LDB = NI_B / 4, LD = LDA + LDB;
  static constexpr int STAGE = A_BYTES + B_BYTES, TRASH = NS * STAGE, LDS = NS * STAGE + 1024;
  static_assert(NI_A % 4 == 0 && NI_B % 4 == 0, "tile rows must split into whole DMA rounds");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert((NS - 2) * LD <= 63, "vmcnt range");
  // mid-stage wait right after a tile's epilogue: its TM * TN stores sit between the stage waited for and the
  // younger DMA (capped at the counter's 63: a conservative wait)
  static constexpr int NWAIT = (NS - 2) * LD, NWAIT_ST = (NS - 2) * LD + TM * TN > 63 ? 63 : (NS - 2) * LD + TM * TN;
};

// LDS-DMA of one 16-byte chunk per lane: global address = sbase (SGPR pair) + voff (32-bit VGPR), LDS address
// = M0 = lds (+ lane * 16 by the hardware).  One SGPR pair per operand and one VGPR per instruction: the
// stage advance is a scalar add on sbase.  M0 is saved / restored around it.
__device__ __forceinline__ void dma16s(const char* sbase, uint32_t voff, uint32_t lds) {
  // (the base is uniform; readfirstlane makes that visible, else hipcc may hand the "s" operand a VGPR pair)
  const uint64_t b = reinterpret_cast<uint64_t>(sbase);
  // (readfirstlane returns int: widen through uint32_t, a sign-extended low word would corrupt the high one)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  sbase = reinterpret_cast<const char*>(((uint64_t)hi << 32) | (uint64_t)lo);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
// the same with a full 64-bit VGPR address (K tails / padding: the lane reads the zero block)
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
  constexpr int TM = C::TM, TN = C::TN, WM = C::WM, WN = C::WN, BM = C::BM, BN = C::BN, NS = C::NS, LD = C::LD;
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

  // ---- DMA.  Instruction t of a stage's A (or W) image moves slots q = t * 64 + lane: row 8 t + lane / 8, slot
  // lane % 8 holding chunk (lane % 8) ^ ((lane / 8) & 7) — the same chunk for every t.
  const int lr = lane >> 3, cq = (lane & 7) ^ (lr & 7);
  uint32_t offA[C::LDA], offB[C::LDB];
  auto set_rows = [&](int tile) __attribute__((always_inline)) {
    const int m0 = (tile / ntn) * BM + lr, n0 = (tile % ntn) * BN + lr;
#pragma unroll
    for (int i = 0; i < C::LDA; ++i)
      offA[i] = (uint32_t)min(m0 + 8 * (i * 4 + wave), p.M - 1) * (uint32_t)ldab + cq * 16;
#pragma unroll
    for (int i = 0; i < C::LDB; ++i)
      offB[i] = (uint32_t)min(n0 + 8 * (i * 4 + wave), p.N - 1) * (uint32_t)ldwb + cq * 16;
  };
  // DMA instruction idx (A for idx < LDA, then W) of stage ks (64-deep K slice) into ring slot buf
  auto issue1 = [&](int ks, int buf, int idx) __attribute__((always_inline)) {
    const bool isA = idx < C::LDA;
    const int i = isA ? idx : idx - C::LDA;
    const int t = i * 4 + wave;
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds0 + buf * C::STAGE + (isA ? 0 : C::A_BYTES) + t * 1024);
    dma16s((isA ? Ab : Wb) + ks * 128, isA ? offA[isA ? i : 0] : offB[isA ? 0 : i], lds);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment of 16-row group g of a stage image, k-step ks (32 of the stage's 64): row 16 g + fr, chunk ks 4 + fq
  const int foff0 = fr * 128 + ((0 + fq) ^ (fr & 7)) * 16, foff1 = fr * 128 + ((4 + fq) ^ (fr & 7)) * 16;
  auto frag = [&](int buf, bool isB, int g, int ks) {
    return *reinterpret_cast<const tx8*>(smem + buf * C::STAGE + (isB ? C::A_BYTES : 0) + g * 2048 + (ks ? foff1 : foff0));
  };
  tx8 fb[2][TN], fa[2];
  auto read_b = [&](int buf, int ks) {
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[ks][j] = frag(buf, true, wn * TN + j, ks);
  };

  const T* R = static_cast<const T*>(p.R);
  T* Cout = static_cast<T*>(p.C);
  auto epilogue = [&](int tile) __attribute__((always_inline)) {
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
      __builtin_amdgcn_sched_barrier(0);   // one row block at a time (hoisting every row's loads costs registers)
    }
  };

  // ---- the stage stream of this workgroup: tiles first, first + G, ...; nk stages each.  The DMA cursor (dtile,
  // dks) fills ring slot dbuf.
  int dtile = first, dks = 0, dbuf = 0;
  auto advance = [&]() __attribute__((always_inline)) {
    dbuf = dbuf + 1 == NS ? 0 : dbuf + 1;
    if (++dks == nk) {
      dks = 0;
      dtile += G;
    }
  };
  // the DMA row offsets follow the tile of the DMA actually being issued (a refill of tile t's last stage is
  // still issued after the cursor has moved on to tile t + G)
  int rows_tile = first;
  set_rows(first);
  auto ensure_rows = [&](int t) __attribute__((always_inline)) {
    if (t != rows_tile) {
      set_rows(t);
      rows_tile = t;
    }
  };
  auto pad_dma = [&]() __attribute__((always_inline)) { dma16(zero, __builtin_amdgcn_readfirstlane(lds0 + C::TRASH)); };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (dtile < ntiles) {
      ensure_rows(dtile);
#pragma unroll
      for (int idx = 0; idx < LD; ++idx) issue1(dks, dbuf, idx);
      advance();
    } else {
#pragma unroll
      for (int idx = 0; idx < LD; ++idx) pad_dma();
    }
  }
  // stage 0 landed (NS - 2 younger stages in flight) -> barrier -> its first fragments
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * LD) : "memory");
  barrier();
  int buf = 0;
  read_b(0, 0);
  fa[0] = frag(0, false, wm * TM, 0);
  // the stage whose DMA rides on the current stage's row groups: stage u + NS - 1 into slot (u - 1) % NS (the
  // prologue filled slots 0 .. NS - 2); past the end of the stream, padding DMA keeps every count exact
  int pks = dks, pbuf = dbuf, ptile = dtile;
  bool plive = dtile < ntiles;
  if (plive) advance();
  int stores = 0;        // mid-stage waits left with a tile's epilogue stores younger than the stage they need
  constexpr int NG = 2 * TM;                          // (k-step, row block) groups of a stage
  // refill schedule: FRONT instructions right behind the mid-stage barrier that frees the slot (with a 2-deep ring
  // the stage has only until the next mid-stage wait to land), the rest PER per group from the next stage's start
  constexpr int FRONT = NS == 2 ? (LD + 1) / 2 : 0;
  constexpr int PER = 2;
  static_assert(FRONT + PER * (NG - 1) >= LD, "refill schedule");
  if constexpr (FRONT > 0) {             // the first pending stage's front part (no mid-stage barrier before it)
    if (plive) ensure_rows(ptile);
#pragma unroll
    for (int idx = 0; idx < FRONT; ++idx) {
      if (plive) issue1(pks, pbuf, idx);
      else pad_dma();
    }
  }
  auto stage = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < NG - 1; ++g) {
      const int ks = g / TM, i = g % TM;
      if (g == 0 && plive) ensure_rows(ptile);
#pragma unroll
      for (int r = 0; r < PER; ++r) {
        const int idx = FRONT + g * PER + r;
        if (idx < LD) {
          if (plive) issue1(pks, pbuf, idx);
          else pad_dma();
        }
      }
      if (g == TM - 2) read_b(buf, 1);                // k-step 1's B fragments under k-step 0's last row blocks
      fa[(g + 1) & 1] = frag(buf, false, wm * TM + (g + 1) % TM, (g + 1) / TM);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[ks][j], fa[g & 1], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // mid-stage: every DMA instruction of this stage's refill is out; the next stage must have landed — NS - 2
    // younger stages may stay in flight (a tile's epilogue stores in between: NWAIT_ST) — and every wave's reads
    // of this stage are retired
    if (stores > 0) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C::NWAIT_ST) : "memory");
      --stores;
    } else {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C::NWAIT) : "memory");
    }
    barrier();
    // this stage's slot is free: the next stage's row groups refill it
    plive = dtile < ntiles;
    pks = dks;
    pbuf = dbuf;
    ptile = dtile;
    if (plive) advance();
    if constexpr (FRONT > 0) {
      if (plive) ensure_rows(ptile);
#pragma unroll
      for (int idx = 0; idx < FRONT; ++idx) {
        if (plive) issue1(pks, pbuf, idx);
        else pad_dma();
      }
    }
    // k-step-0 fragments of the next stage (fb[0] is free since this stage's k-step 0) under the last group's
    // MFMAs; past the stream's end they read a stale slot, never used
    const int nbuf = buf + 1 == NS ? 0 : buf + 1;
    read_b(nbuf, 0);
    const tx8 fa_next = frag(nbuf, false, wm * TM, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[TM - 1][j] = mfma16x16x32(fb[1][j], fa[(NG - 1) & 1], acc[TM - 1][j]);
    __builtin_amdgcn_sched_barrier(0);
    fa[0] = fa_next;
    buf = nbuf;
  };
  for (int tile = first; tile < ntiles; tile += G) {
    for (int ks = 0; ks < nk; ++ks) stage();
    // (outside the K loop: inside it hipcc hoists the epilogue's per-tile addresses and keeps them live next to
    // the accumulators)
    epilogue(tile);
    // the stages older than the stores reach NS - 1 ahead of the last one: the next NS - 2 mid-stage waits need
    // one of them
    stores = NS - 2;
  }
  // the padding / refill DMA still in flight lands in LDS this workgroup owns until it ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int slots_of(const void* fn) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0);
  return std::max(1, cus) * std::max(1, per);
}

template <typename T, int TM, int TN, int NS, bool KTAIL, int ACT>
static int launch(const GemmArgs& a, hipStream_t st) {
  typedef Cfg<TM, TN, NS> C;
  const int ntm = (a.M + C::BM - 1) / C::BM, ntn = (a.N + C::BN - 1) / C::BN;
  const long ntiles = (long)ntm * ntn;
  const int nk = (a.K + C::BK - 1) / C::BK;
  static const int slots = slots_of(reinterpret_cast<const void*>(&gemm_wt<T, C, KTAIL, ACT>));
  const int grid = (int)std::min<long>(ntiles, slots);
  hipLaunchKernelGGL((gemm_wt<T, C, KTAIL, ACT>), dim3(grid), dim3(256), 0, st, a, ntn, (int)ntiles, nk);
  static char name[80];
  if (!name[0])
    snprintf(name, sizeof(name), "gemm_wt<%s, Cfg<%d, %d, %d>, %s, %d>", type_name<T>(), TM, TN, NS,
             KTAIL ? "true" : "false", ACT);
  set_last_kernel(name);
  return check_launch("gemm_wt");
}

template <typename T, int TM, int TN, int NS>
static int launch_cfg(const GemmArgs& a, hipStream_t st) {
  const bool tail = false;                        // (K % 64 == 0: no tails)
  switch (a.act) {
    case SVK_ACT_GELU:
      return tail ? launch<T, TM, TN, NS, true, SVK_ACT_GELU>(a, st) : launch<T, TM, TN, NS, false, SVK_ACT_GELU>(a, st);
    case SVK_ACT_RELU:
      return tail ? launch<T, TM, TN, NS, true, SVK_ACT_RELU>(a, st) : launch<T, TM, TN, NS, false, SVK_ACT_RELU>(a, st);
    case 0: return tail ? launch<T, TM, TN, NS, true, 0>(a, st) : launch<T, TM, TN, NS, false, 0>(a, st);
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
  if (a.K % 64) return 1;                         // whole 64-deep stages (no K tails)
  switch (cfg) {
    case 0: return wt::launch_cfg<T, 8, 8, 2>(a, st);
    case 1: return wt::launch_cfg<T, 8, 5, 3>(a, st);
    case 2: return wt::launch_cfg<T, 8, 4, 3>(a, st);
    case 3: return wt::launch_cfg<T, 8, 6, 2>(a, st);
    default: return 1;
  }
}

template int gemm_wt_try<bf16>(const GemmArgs&, hipStream_t, int);
template int gemm_wt_try<f16>(const GemmArgs&, hipStream_t, int);

}  // namespace svk
