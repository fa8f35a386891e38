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
// Pipeline (measured lesson of the first version: with one 64-deep K-tile in flight the LDS-DMA landing time,
// ~1-2 us under load, was exposed every K-tile — 2.6x the MFMA time):
//  * the K axis is cut into 32-deep stages; a ring of NS stages in LDS (NS = 4: 128 KiB at 256 x 256), filled by
//    LDS-DMA (`global_load_lds_dwordx4`), NS - 1 stages in flight — ~1.5 us of landing time at the MFMA rate;
//  * stage image: rows paired into 128-byte "double rows" (row 2d + h, 16-byte k-chunk c of 4 -> chunk slot
//    ((h << 2) | c) ^ (d & 7) of double row d), so every ds_read_b128 fragment read of the 16x16x32 MFMA is
//    bank-conflict-free and a lane's fragment offset inside a 16-row group is a per-lane constant;
//  * one barrier per stage, in the MIDDLE of the stage's row groups: after the reads of stage u are all issued
//    (row group TM - 2) every wave waits for its share of stage u + 1, then the barrier; behind it stage u's
//    buffer is refilled (DMA of stage u + NS, spread over the next row groups: an LDS-DMA issue costs ~60 cycles
//    among MFMAs) and the fragments of stage u + 1 are read under the MFMAs of stage u's last row group — the
//    matrix pipe does not wait for LDS at stage boundaries;
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
  static constexpr int WM = 16 * TM, WN = 16 * TN, BM = 2 * WM, BN = 2 * WN, BK = 32, NT = 256;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  // DMA wave-instructions (1 KiB each) of one stage, dealt round-robin to the 4 waves; a wave whose share is
  // short issues a padding DMA of the zero block into the TRASH KiB, so every wave counts the same LD
  static constexpr int NI_A = A_BYTES / 1024, NI_B = B_BYTES / 1024;
  static constexpr int LDA = (NI_A + 3) / 4, LDB = (NI_B + 3) / 4, LD = LDA + LDB;
  static constexpr bool PAD = NI_A % 4 != 0 || NI_B % 4 != 0;
  // ring, the padding-DMA sink, and the bias vector (f32, up to MAXN columns: loaded once per launch, so the
  // epilogue's bias reads are LDS reads — a compiler-visible global load there would make hipcc wait for every
  // older vector-memory operation, i.e. for the DMA stages in flight)
  static constexpr int MAXN = 4096;
  static constexpr int STAGE = A_BYTES + B_BYTES, TRASH = NS * STAGE, BIAS = TRASH + 1024, LDS = BIAS + MAXN * 4;
  static_assert(A_BYTES % 1024 == 0 && B_BYTES % 1024 == 0, "tile rows must be whole DMA instructions");
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

  // bias -> LDS (before any DMA is in flight: the loads' wait drains nothing else)
  float* sbias = reinterpret_cast<float*>(smem + C::BIAS);
  for (int n = tid; n < p.N; n += 256) sbias[n] = p.bias ? p.bias[n] : 0.f;
  __syncthreads();

  // ---- DMA.  Instruction t of a stage's A (or W) image moves slots q = t * 64 + lane: double row d = q / 8,
  // slot s = q % 8 holds chunk c = s ^ (d & 7) = (h << 2) | kc of row 2d + h.  This lane's (h, kc) is the same
  // for every t (t * 64 moves d by multiples of 8); its row is 16 t + 2 (lane / 8) + h.
  const int dl = lane >> 3, cs = (lane & 7) ^ (dl & 7), hl = cs >> 2, kl = cs & 3;
  uint32_t offA[C::LDA], offB[C::LDB];
  auto set_rows = [&](int tile) __attribute__((always_inline)) {
    const int m0 = (tile / ntn) * BM + 2 * dl + hl, n0 = (tile % ntn) * BN + 2 * dl + hl;
#pragma unroll
    for (int i = 0; i < C::LDA; ++i)
      offA[i] = (uint32_t)min(m0 + 16 * (i * 4 + wave), p.M - 1) * (uint32_t)ldab + kl * 16;
#pragma unroll
    for (int i = 0; i < C::LDB; ++i)
      offB[i] = (uint32_t)min(n0 + 16 * (i * 4 + wave), p.N - 1) * (uint32_t)ldwb + kl * 16;
  };
  // DMA instruction idx (A for idx < LDA, then W) of stage ks (32-deep K slice) into ring slot buf
  auto issue1 = [&](int ks, int buf, int idx) __attribute__((always_inline)) {
    const bool isA = idx < C::LDA;
    const int i = isA ? idx : idx - C::LDA;
    const int t = i * 4 + wave;                                   // the stage's instruction number
    const bool pad = t >= (isA ? C::NI_A : C::NI_B);             // wave-uniform
    const uint32_t lds = __builtin_amdgcn_readfirstlane(
        pad ? lds0 + C::TRASH : lds0 + buf * C::STAGE + (isA ? 0 : C::A_BYTES) + t * 1024);
    const uint32_t off = isA ? offA[isA ? i : 0] : offB[isA ? 0 : i];
    const char* base = (isA ? Ab : Wb) + ks * 64;
    if constexpr (KTAIL || C::PAD) {
      const bool ok = !pad && (!KTAIL || ks * 32 + kl * 8 < p.K);
      dma16(ok ? base + off : zero, lds);
    } else {
      dma16s(base, off, lds);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment of 16-row group g (row0 = 16 g) of a stage image: this lane reads row row0 + fr, k-chunk fq
  const int foff = (fr >> 1) * 128 + ((((fr & 1) << 2) | fq) ^ ((fr >> 1) & 7)) * 16;
  auto frag = [&](int buf, bool isB, int g) {
    return *reinterpret_cast<const tx8*>(smem + buf * C::STAGE + (isB ? C::A_BYTES : 0) + g * 1024 + foff);
  };
  tx8 fb[2][TN], fa[2];
  auto read_b = [&](int buf, tx8* dst) {
#pragma unroll
    for (int j = 0; j < TN; ++j) dst[j] = frag(buf, true, wn * TN + j);
  };

  const T* R = static_cast<const T*>(p.R);
  T* Cout = static_cast<T*>(p.C);
  auto epilogue = [&](int tile) __attribute__((always_inline)) {
    const int m0 = (tile / ntn) * BM + wm * WM, n0 = (tile % ntn) * BN + wn * WN;
    f32x4 bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = min(n0 + j * 16 + fq * 4, p.N - 4);
      bj[j] = *reinterpret_cast<const f32x4*>(sbias + n);
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
  // dks) runs NS stages ahead of the compute cursor; the stage it fills goes to ring slot dbuf.
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
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (dtile < ntiles) {
      ensure_rows(dtile);
#pragma unroll
      for (int idx = 0; idx < LD; ++idx) issue1(dks, dbuf, idx);
      advance();
    } else {
#pragma unroll
      for (int idx = 0; idx < LD; ++idx) dma16(zero, __builtin_amdgcn_readfirstlane(lds0 + C::TRASH));
    }
  }
  // stage 0 landed (NS - 2 younger stages in flight) -> barrier -> its first fragments
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * LD) : "memory");
  barrier();
  int buf = 0;
  read_b(0, fb[0]);
  fa[0] = frag(0, false, wm * TM);
  // the stage whose DMA rides on the current stage's row groups: stage u + NS - 1 into slot (u - 1) % NS (the
  // prologue filled slots 0 .. NS - 2); past the end of the stream, padding DMA keeps every count exact
  int pks = dks, pbuf = dbuf, ptile = dtile;
  bool plive = dtile < ntiles;
  if (plive) advance();
  int stores = 0;        // mid-stage waits left with a tile's epilogue stores younger than the stage they need
  constexpr int PER = (LD + TM - 2) / (TM - 1);   // refill instructions per row group
  // one stage of the stream; CUR = which fb[] holds its B fragments (compile-time: a runtime index would put the
  // fragment arrays in scratch)
  auto stage = [&](auto CUR_) __attribute__((always_inline)) {
    constexpr int CUR = decltype(CUR_)::value;
    // row groups 0 .. TM - 2: the next A fragment read ahead, the refill DMA spread over them
#pragma unroll
    for (int i = 0; i < TM - 1; ++i) {
      if (i == 0 && plive) ensure_rows(ptile);
#pragma unroll
      for (int r = 0; r < PER; ++r) {
        const int idx = i * PER + r;
        if (idx < LD) {
          if (plive) issue1(pks, pbuf, idx);
          else dma16(zero, __builtin_amdgcn_readfirstlane(lds0 + C::TRASH));
        }
      }
      fa[(i + 1) & 1] = frag(buf, false, wm * TM + i + 1);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[CUR][j], fa[i & 1], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // mid-stage: every DMA instruction of this stage's refill is out; the next stage (issued NS - 2 stages ago)
    // must have landed — NS - 2 younger stages may stay in flight (a tile's epilogue stores in between: NWAIT_ST)
    // — and every wave's reads of this stage are retired
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
    // fragments of the next stage under the last row group's MFMAs (past the stream's end they read a stale slot:
    // never used)
    const int nbuf = buf + 1 == NS ? 0 : buf + 1;
    read_b(nbuf, fb[CUR ^ 1]);
    const tx8 fa_next = frag(nbuf, false, wm * TM);
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[TM - 1][j] = mfma16x16x32(fb[CUR][j], fa[(TM - 1) & 1], acc[TM - 1][j]);
    __builtin_amdgcn_sched_barrier(0);
    fa[0] = fa_next;
    buf = nbuf;
  };
  // nk is even (host): stages alternate fb[0] / fb[1] and every tile starts on fb[0]
  for (int tile = first; tile < ntiles; tile += G) {
    for (int ks = 0; ks < nk; ks += 2) {
      stage(std::integral_constant<int, 0>{});
      stage(std::integral_constant<int, 1>{});
    }
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
  if (a.N > 4096) return 1;                       // the bias vector lives in LDS (Cfg::MAXN)
  if (a.K % 64) return 1;                         // an even number of 32-deep stages per tile
  switch (cfg) {
    case 0: return wt::launch_cfg<T, 8, 8, 4>(a, st);
    case 3: return wt::launch_cfg<T, 8, 6, 4>(a, st);
    case 1: return wt::launch_cfg<T, 8, 5, 4>(a, st);
    case 2: return wt::launch_cfg<T, 8, 4, 5>(a, st);
    default: return 1;
  }
}

template int gemm_wt_try<bf16>(const GemmArgs&, hipStream_t, int);
template int gemm_wt_try<f16>(const GemmArgs&, hipStream_t, int);

}  // namespace svk
