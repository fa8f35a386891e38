// Ping-pong 256-row GEMM for the MFMA-bound token GEMMs (f16 / bf16 in and out, f32 accumulate):
//
//   C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]
//
// Why a second GEMM next to gemm_pk: gemm_pk's 128 x 128 tile (4 waves of 64 x 64, two workgroups per CU)
// reads 16 fragment vectors from LDS per 32 MFMAs and synchronises its four waves twice per 64-deep K-step;
// on the long-K / wide-N shapes (the SegFormer head, stage-3 / stage-4 fc1 / fc2 / kv) it peaks near
// 700 TF/s while hipBLASLt runs them 1.15-1.42x faster.  This kernel is the CDNA4 "ping-pong" shape:
//
//  * one 512-thread workgroup per CU, a 256 x BN x 64 tile (BN = 256: 4 x 64-column waves; BN = 320: 4 x 80,
//    so the N = 320 / 640 / 1280 shapes have no padded columns), 8 waves = 2 groups of 4: group g owns rows
//    128 g .. 128 g + 127, wave c of a group owns columns c * BN / 4 ..; a wave's 128 x BN/4 accumulators
//    (128 / 160 registers) live in the AGPR half of the register file;
//  * two K-tile buffers in LDS (128 / 144 KiB), filled by LDS-DMA (`global_load_lds_dwordx4`, the XOR
//    swizzle applied on the source address so every ds_read_b128 fragment read is conflict-free);
//  * the two groups run ONE barrier interval apart (group 1 passes one extra s_barrier first): in every
//    interval one group issues its 16-20 MFMAs while the other reads its next fragments from LDS and issues
//    its share of the next K-tile's DMA, so each SIMD's matrix pipe alternates between its two waves and the
//    fragment reads, DMA issue and barrier waits of one wave hide under the other wave's MFMAs;
//  * a K-tile is 4 phases per group: phase p = MFMA rows 32 p .. 32 p + 31 of the wave's 128 (2 x BN/64
//    blocks x 2 k-steps = 16 / 20 MFMAs); the wave's B fragments (BN/64 blocks x 2 k-steps) are read once per
//    K-tile and kept in registers, A fragments 4 per phase;
//  * persistent: a fixed grid (one workgroup per CU) walks the (tile, K-tile) stream; the next K-tile — at a
//    tile boundary the next tile's first — is DMA'd during the current one, so tile prologues are hidden;
//  * transposed MFMA (W fragment x A fragment): each lane holds 4 consecutive output columns of a row, so the
//    epilogue (bias, activation, residual in f32, one rounding) stores 8-byte row pieces from registers.
//
// Buffer hazards (t = K-tile of the stream, buffer t % 2; interval i of the workgroup's barrier sequence):
//  group 0 reads tile t in intervals 8t, 8t+2, 8t+4, 8t+6, group 1 in 8t+1 .. 8t+7 (odd); a read issued in
//  interval i is retired (lgkmcnt, before the MFMAs that consume it) inside interval i + 1.  The DMA of tile
//  t+1 overwrites tile t-1's buffer, whose last read (group 1, interval 8t-1) retired in 8t: it is issued in
//  intervals 8t+1 / 8t+3 (group 1) and 8t+2 / 8t+4 (group 0), and every wave retires its own DMA
//  (`s_waitcnt vmcnt(0)`) before the barrier that precedes the first read of tile t+1 (interval 8t+8): group 0
//  at the end of its compute interval 8t+7, group 1 at the end of its LOAD interval 8t+7 (its last compute
//  interval of tile t, 8t+8, is already past that barrier).  Raw s_barrier (never __syncthreads, whose fence drains DMA).
#include "svk_common.h"
#include "gemm_args.h"
#include <stdio.h>
#include <type_traits>

namespace svk {
namespace pp {

static __device__ __attribute__((aligned(16))) uint4 g_zero[4];   // zero block: K tails
static __device__ __attribute__((aligned(16))) uint2 g_trash[64];  // sink of the epilogue's out-of-range stores

typedef __attribute__((address_space(3))) void* las_ptr;

template <int BN_>
struct Cfg {
  static constexpr int BM = 256, BN = BN_, BK = 64, NT = 512;
  static constexpr int WN = BN / 4, TM = 8, TN = WN / 16;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES, LDS = 2 * STAGE;
  static constexpr int A_LD = A_BYTES / (NT * 16), B_LD = B_BYTES / (NT * 16);   // DMA instructions per thread
  static_assert(WN % 16 == 0 && A_BYTES % (NT * 16) == 0 && B_BYTES % (NT * 16) == 0, "tile shape");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(BN == 256, "the DMA stream's 8 pieces per K-tile = 4 W pieces (BN / 64) + 4 A pieces");
};

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

template <typename T, class C, bool KTAIL, int ACT, int DEEP>
__global__ __launch_bounds__(512, 2)
void gemm_pp(GemmArgs p, int ntn, int ntiles, int nk) {
  typedef v8_t<T> tx8;
  constexpr int BN = C::BN, WN = C::WN, TM = C::TM, TN = C::TN;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int first = xcd_remap(blockIdx.x, G);         // first tile of this workgroup
  if (first >= ntiles) return;                        // whole workgroup: no barrier is left waiting
  const T* A = static_cast<const T*>(p.A);
  const T* Wt = static_cast<const T*>(p.W);
  const char* zero = reinterpret_cast<const char*>(g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;

  // LDS-DMA stream.  A K-tile is 8 pieces of one `global_load_lds_dwordx4` per thread: B0..B3 (W rows 32 w + 8 i
  // .. of wave w, i = 0..3: the whole 256-row W slab) and A0..A3 (piece A_p = the rows phase p reads: 32 p ..
  // 32 p + 31 of each group's half; wave w loads 8 of them, group g's waves exactly group g's rows).  Every
  // interval of every wave issues exactly ONE piece, in stream order, so `s_waitcnt vmcnt(NW)` at the end of
  // every interval retires each piece NW intervals after its issue (readable one interval later; group 1 issues
  // one interval after group 0).  Issue time of piece k of stream position u: 8u - DD + k (group 0's interval
  // numbering).  Deadlines: the B pieces are read by group 0 from 8u on — group 1's copy must retire by 8u - 1:
  // DD - 3 >= NW + 2; A_p is read by its own group from 8u + 2p: DD - 4 - p >= NW + 1 - 2p.  Buffer reuse (a
  // piece overwrites the same piece of position u - 2): B after 8u - 14 (group 1's reads of u - 2 retired),
  // A_p after 8u - 15 + 2p: DD <= 13.  DEEP = 0: DD = 9, NW = 3 (round-4 first form); DEEP = 1: DD = 13,
  // NW = 8 — each piece gets 8 intervals (~2-4k cycles) to land instead of 3.
  //
  // DEEP = 2 ("paired" schedule, the 8-phase template's placement): the compute intervals issue nothing but their
  // MFMAs; load interval 2p of position u issues TWO pieces of position u + 1 — B0 B1 | B2 B3 | A0 A1 | A2 A3 —
  // and each wave counts its DMA twice per K-tile: at the end of slot 6, vmcnt(2) retires everything but the
  // two pieces just issued (B and A0 A1 of u + 1: B is read by both groups from interval 8(u + 1), group 1's
  // copy retired at the end of 8u + 7, group 0's at 8u + 6; A0 A1 by their own group from slot 0 / 2), and at
  // the end of slot 3 of u + 1, vmcnt(4) retires A2 A3 (read from slot 4) past the four B pieces of u + 2
  // (+ NST when the epilogue's stores sit between them).  Buffer reuse: position u + 1 overwrites u - 1, whose
  // last reads (group 1's A3, interval 8u - 1) retired in interval 8u, the first issue's.
  constexpr int DD = DEEP == 1 ? 13 : 9, NW = DEEP == 1 ? 8 : 3;
  constexpr int OFF = DEEP >= 2 ? 0 : DD & 7;               // slot s issues piece (s + OFF) % 8 ...
  static_assert(DD - 3 >= NW + 2 && DD - 4 >= NW + 1 && DD <= 13, "DMA schedule");
  auto opaque = [](int v) { asm volatile("" : "+s"(v)); return v; };
  const int cq = (lane & 7) ^ ((lane >> 3) & 7);          // this lane's swizzled 16-byte chunk (rows are 8-aligned)
  const long ldab = p.lda * 2, ldwb = p.ldw * 2;
  uint32_t offA[4], offB[4];
  auto set_rows = [&](int tile) {
    tile = opaque(tile);
    const int m0 = (tile / ntn) * C::BM, n0 = (tile % ntn) * BN;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ra = (wave >> 2) * 128 + 32 * q + (wave & 3) * 8 + (lane >> 3);
      const int rb = wave * 32 + 8 * q + (lane >> 3);
      offA[q] = (uint32_t)min(m0 + ra, p.M - 1) * (uint32_t)ldab + cq * 16;
      offB[q] = (uint32_t)min(n0 + rb, p.N - 1) * (uint32_t)ldwb + cq * 16;
    }
  };
  auto issue = [&](int piece, int kt, int buf) {
    const int q = piece & 3;
    const bool isA = piece >= 4;
    const char* base = isA ? reinterpret_cast<const char*>(A) : reinterpret_cast<const char*>(Wt);
    const char* src = base + (isA ? offA[q] : offB[q]) + (uint32_t)kt * 128u;
    if constexpr (KTAIL) src = kt * C::BK + cq * 8 < p.K ? src : zero;
    const uint32_t row0 = isA ? (wave >> 2) * 128 + 32 * q + (wave & 3) * 8 : C::BM + wave * 32 + 8 * q;
    dma16(src, lds0 + buf * C::STAGE + row0 * 128);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  tx8 fb[TN][2], fa[2][2];

  auto read_b = [&](int buf) {
    const char* sb = smem + buf * C::STAGE + C::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cc = ((ks * 4 + fq) ^ (fr & 7)) * 16;
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j][ks] = *reinterpret_cast<const tx8*>(sb + (wc * WN + j * 16 + fr) * 128 + cc);
    }
  };
  auto read_a = [&](int buf, int ph) {
    const char* sa = smem + buf * C::STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cc = ((ks * 4 + fq) ^ (fr & 7)) * 16;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i][ks] = *reinterpret_cast<const tx8*>(sa + (g * 128 + (2 * ph + i) * 16 + fr) * 128 + cc);
    }
  };
  auto mfma_phase = [&](int ph) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[2 * ph + i][j] = mfma16x16x32(fb[j][ks], fa[i][ks], acc[2 * ph + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // epilogue of one tile: lane (fr, fq) of block (i, j) holds C[m0 + 128 g + 16 i + fr][n0 + wc WN + 16 j + 4 fq ..+3].
  // Every lane issues exactly TM * TN stores (out-of-range pieces go to a scratch row): the wait counts after
  // the epilogue assume that number.
  const T* R = static_cast<const T*>(p.R);
  T* Cout = static_cast<T*>(p.C);
  constexpr int NST = TM * TN;
  auto epilogue = [&](int tile) {
    asm volatile("" : "+v"(tile));                   // opaque (see set_rows); a VGPR operand works on every path
    const int m0 = (tile / ntn) * C::BM + g * 128, n0 = (tile % ntn) * BN + wc * WN;
    f32x4 bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = min(n0 + j * 16 + fq * 4, p.N - 4);
      bj[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {                    // two halves of the rows: fewer live residual registers
      uint2 res[TM / 2][TN];
#pragma unroll
      for (int ii = 0; ii < TM / 2; ++ii)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int m = min(m0 + (h * 4 + ii) * 16 + fr, p.M - 1), n = min(n0 + j * 16 + fq * 4, p.N - 4);
          res[ii][j] = R ? *reinterpret_cast<const uint2*>(R + (long)m * p.ldr + n) : uint2{0u, 0u};
        }
#pragma unroll
      for (int ii = 0; ii < TM / 2; ++ii) {
        const int i = h * 4 + ii;
        const int m = m0 + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + j * 16 + fq * 4;
          float v[4] = {acc[i][j][0] + bj[j].x, acc[i][j][1] + bj[j].y, acc[i][j][2] + bj[j].z, acc[i][j][3] + bj[j].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act_fast(v[e], ACT);
          const f32x2 r01 = unpack2<T>(res[ii][j].x), r23 = unpack2<T>(res[ii][j].y);
          v[0] += r01.x;
          v[1] += r01.y;
          v[2] += r23.x;
          v[3] += r23.y;
          T o[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
          uint2* dst = m < p.M && n < p.N ? reinterpret_cast<uint2*>(Cout + (long)m * p.ldc + n) : g_trash + lane;
          *dst = *reinterpret_cast<const uint2*>(o);
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };

  // ---- prologue: stream position 0 whole and the first OFF pieces of position 1 (their nominal issue intervals
  // are negative); position 0 retired before the first barrier
  int dtile = first, dkt = 0, dbuf = 0;
  bool dlive = true;
  // the consumer's cursor starts at stream position 0 (the DMA cursor is moved ahead by the prologue below)
  int tile = dtile, kt = dkt;
  auto advance = [&]() {
    dbuf ^= 1;
    if (++dkt == nk) {
      dkt = 0;
      dtile += G;
      dlive = dtile < ntiles;
      if (dlive) set_rows(dtile);
    }
  };
  set_rows(dtile);
#pragma unroll
  for (int k = 0; k < 8; ++k) issue(k, dkt, 0);
  advance();
#pragma unroll
  for (int k = 0; k < OFF; ++k)
    if (dlive) issue(k, dkt, dbuf);
  if constexpr (DEEP >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OFF) : "memory");
  barrier();
  if (g == 1) barrier();                              // the stagger: group 1 runs one interval behind

  int buf = 0;
  int post = 0;                                       // intervals left in which the epilogue's stores may still fly
  while (tile < ntiles) {
    const bool tlast = kt == nk - 1;
    const bool live = dlive;                          // (DEEP 2) pieces of the next position are issued in this one
    // the 8 intervals of this K-tile, each a compile-time slot (a runtime slot index would put the
    // accumulators in scratch)
    auto slot = [&](auto S_) {
      constexpr int s = decltype(S_)::value, ph = s >> 1, piece = (s + OFF) & 7;
      constexpr bool PAIRED = DEEP >= 2, READS_FIRST = DEEP == 3;
      auto dma = [&]() {
        if constexpr (PAIRED) {
          if constexpr ((s & 1) == 0) {
            if (live) {
              issue(s, dkt, dbuf);
              issue(s + 1, dkt, dbuf);
            }
            if constexpr (s == 6) advance();          // the cursor moves on once position u + 1 is issued
          }
        } else {
          if (piece == 0) advance();                  // the cursor moves to the next stream position
          if (dlive) issue(piece, dkt, dbuf);
        }
      };
      if constexpr (!READS_FIRST) dma();
      if constexpr ((s & 1) == 0) {                   // ---- load interval
        if constexpr (ph == 0) read_b(buf);
        read_a(buf, ph);
        if constexpr (READS_FIRST) {                  // (DEEP 3) fragment reads issued ahead of the DMA pair
          __builtin_amdgcn_sched_barrier(0);
          dma();
        }
      } else {                                        // ---- compute interval
        mfma_phase(ph);
        if (s == 7 && tlast) {
          epilogue(tile);
          post = NW + 1;
        }
      }
      // the epilogue's NST stores are younger than the NW pieces issued before them: for the NW + 1 intervals
      // until the last of those pieces is due, the count leaves them out as well.  Past the end of the stream no
      // piece is issued, so a count of NW would leave the last pieces in flight into their reads: drain.
      if constexpr (PAIRED) {
        if constexpr (s == 3) {
          if (!live) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else if (post > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST + 4) : "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          post = 0;
        } else if constexpr (s == 6) {
          if (!live) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
      } else if (!dlive) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (post > 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST + NW) : "memory");
        --post;
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW) : "memory");
      }
      barrier();
    };
    slot(std::integral_constant<int, 0>{});
    slot(std::integral_constant<int, 1>{});
    slot(std::integral_constant<int, 2>{});
    slot(std::integral_constant<int, 3>{});
    slot(std::integral_constant<int, 4>{});
    slot(std::integral_constant<int, 5>{});
    slot(std::integral_constant<int, 6>{});
    slot(std::integral_constant<int, 7>{});
    buf ^= 1;
    if (tlast) {
      kt = 0;
      tile += G;
    } else {
      ++kt;
    }
  }
  if (g == 0) barrier();                              // equal barrier counts: group 0 matches the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int slots_of(const void* fn) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 512, 0);
  return std::max(1, cus) * std::max(1, per);
}

template <typename T, int BN, bool KTAIL, int ACT, int DEEP>
static int launch(const GemmArgs& a, hipStream_t st) {
  typedef Cfg<BN> C;
  const int ntm = (a.M + C::BM - 1) / C::BM, ntn = (a.N + BN - 1) / BN;
  const long ntiles = (long)ntm * ntn;
  const int nk = (a.K + 63) / 64;
  static const int slots = slots_of(reinterpret_cast<const void*>(&gemm_pp<T, C, KTAIL, ACT, DEEP>));
  const int grid = (int)std::min<long>(ntiles, slots);
  hipLaunchKernelGGL((gemm_pp<T, C, KTAIL, ACT, DEEP>), dim3(grid), dim3(512), 0, st, a, ntn, (int)ntiles, nk);
  static char name[96];
  if (!name[0])
    snprintf(name, sizeof(name), "gemm_pp<%s, Cfg<%d>, %s, %d, %d>", type_name<T>(), BN, KTAIL ? "true" : "false", ACT,
             DEEP);
  set_last_kernel(name);
  return check_launch("gemm_pp");
}

template <typename T, int BN, int DEEP>
static int launch_bn(const GemmArgs& a, hipStream_t st) {
  const bool tail = a.K % 64 != 0;
  switch (a.act) {
    case SVK_ACT_GELU:
      return tail ? launch<T, BN, true, SVK_ACT_GELU, DEEP>(a, st) : launch<T, BN, false, SVK_ACT_GELU, DEEP>(a, st);
    case SVK_ACT_RELU:
      return tail ? launch<T, BN, true, SVK_ACT_RELU, DEEP>(a, st) : launch<T, BN, false, SVK_ACT_RELU, DEEP>(a, st);
    case 0: return tail ? launch<T, BN, true, 0, DEEP>(a, st) : launch<T, BN, false, 0, DEEP>(a, st);
    default: return 1;
  }
}

}  // namespace pp

// Dense A only (asrc 0), plain epilogue (bias / GELU / ReLU / residual), K % 8 == 0, N % 4 == 0, 16-byte
// aligned operand rows.  Returns 1 when not eligible.
template <typename T>
int gemm_pp_try(const GemmArgs& a, hipStream_t st, int variant) {
  auto al = [](const void* q, int b) { return ((uintptr_t)q & (b - 1)) == 0; };
  if (a.K % 8 || a.N % 4 || a.lda % 8 || a.ldw % 8 || a.ldc % 4 || (a.R && a.ldr % 4) || a.out_mode || a.U ||
      a.rscale || a.ksplit > 1)
    return 1;
  if (!al(a.A, 16) || !al(a.W, 16) || !al(a.C, 8) || (a.R && !al(a.R, 8)) || (a.bias && !al(a.bias, 16))) return 1;
  // 32-bit byte offsets of the DMA rows
  if ((long)a.M * a.lda * 2 + 256 >= (1L << 32) || (long)a.N * a.ldw * 2 + 256 >= (1L << 32)) return 1;
  // variant: 0 = first DMA schedule, 1 = deep DMA schedule
  if (variant == 0) return pp::launch_bn<T, 256, 3>(a, st);
  if (variant == 1) return pp::launch_bn<T, 256, 2>(a, st);
  // (round 6: the stream-K variant — f32 partial slabs + per-wave flags in a per-stream workspace — was removed: its
  // in-loop partial-sum path spilled 55-67 VGPRs, a scratch access the counted DMA waits cannot see, so it was never
  // instantiated, and its workspace registry had no caller left)
  return 1;
}

template int gemm_pp_try<bf16>(const GemmArgs&, hipStream_t, int);
template int gemm_pp_try<f16>(const GemmArgs&, hipStream_t, int);

}  // namespace svk
