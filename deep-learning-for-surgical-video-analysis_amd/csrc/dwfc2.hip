// The back half of the stage-3 / stage-4 MixFFN in one kernel (mix_transformer_evp.py:60-67 with DWConv :19-30,
// Block residual :169), 16-bit:
//
//   Y[m, n] = sum_k GELU(dwconv3x3(H)[m, k]) * W2[n, k] + b2[n] + R[m, n]
//
// H is fc1's output [B, WI, WI, K] (hidden K = 4C), W2 [N = C, K], R the Block input.  Unfused this is
// dwconv3x3 (+ GELU) writing the hidden map G (B*WI*WI x K 16-bit values) and fc2 reading it back; here G never
// leaves the chip: every K-step of 64 hidden channels the workgroup builds its 64-token G tile in LDS from a
// halo'd H tile (the tile's tokens +- one image row + 1, flattened indices, neighbours masked at the image
// edges), then runs the fc2 MFMAs on it.
//
//  * workgroup = 4 waves, 64 tokens x all N output channels (so each G value is made once); wave w owns
//    columns N/4 w .. (N = 320: 5 n-blocks of 16, 80 accumulator registers; N = 512: 8 blocks, 128);
//  * G production: thread (token t, 8-channel group cg) for tokens t and t + 32: acc = bias, 9 taps in the
//    dwconv3x3_strip order (fma over f32 taps), GELU (the same gelu_rl), rounded to 16 bits -> LDS, rows
//    XOR-swizzled (16-byte chunk c of row r at c ^ (r & 7)) so the MFMA fragment reads are conflict-free;
//  * software pipeline, one barrier per K-step: iteration k issues the fc2 MFMAs of K-step k (G(k), W2
//    fragments in registers), produces G(k + 1) from the H tile already in LDS, writes the H / tap tiles of
//    k + 2 (register-staged, loaded one iteration earlier) and loads those of k + 3 and the W2 fragments of
//    k + 1 — the MFMA and VALU streams are independent, the scheduler interleaves them;
//  * transposed MFMA (W2 fragment x G fragment): a lane ends with 4 consecutive output channels of a token,
//    the epilogue adds b2 and the residual in f32 and stores 8-byte row pieces.
// Numerics: the dwconv + GELU exactly as dwconv3x3_strip (f32 taps and accumulation, G rounded to 16 bits),
// fc2 as the GEMM (f32 accumulation, bias then residual, one rounding).
#include "svk_common.h"
#include <type_traits>

namespace svk {
namespace dwfc {

__device__ __forceinline__ float gelu_rl(float x) {   // = stencil.hip's gelu_rl (erf form, |err| <= 1.5e-7)
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.0f));
  float q = fmaf(-0.5f * 1.061405429f, t, -0.5f * -1.453152027f);
  q = fmaf(q, t, -0.5f * 1.421413741f);
  q = fmaf(q, t, -0.5f * -0.284496736f);
  q = fmaf(q, t, -0.5f * 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
  return fmaf(ax * t * q, e, fmaxf(x, 0.f));
}

static __device__ __attribute__((aligned(16))) uint4 g_zero[4];   // DMA source of halo rows outside the map
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

template <int N_, int WI_, int BM_>
struct Cfg {
  static constexpr int N = N_, WI = WI_, BM = BM_, BK = 64, NT = 256;
  static constexpr int MB = BM / 16, IT = BM / 32;    // m-blocks per wave, G items per thread
  static constexpr int WNB = N / 64;                  // 16-column n-blocks per wave (4 waves split N)
  static constexpr int HR = BM + 2 * WI + 2;          // halo rows: tokens m0 - WI - 1 .. m0 + BM + WI
  static constexpr int HBYTES = HR * BK * 2;
  static constexpr int HCH = HR * 8;                  // 16-byte chunks of a halo tile
  static constexpr int HBLK = (HCH + 63) / 64;       // 1 KiB DMA blocks of a halo tile
  static constexpr int TBYTES = 10 * BK * 4;          // taps [9][64] + dwconv bias [64], f32
  static constexpr int TCH = TBYTES / 16;
  static constexpr int TBLK = (TCH + 63) / 64;
  static constexpr int GBYTES = BM * BK * 2;
  static constexpr int HSTRIDE = HBLK * 1024, TSTRIDE = TBLK * 1024;   // buffers in whole DMA blocks
  static constexpr int H_OFF = 0, T_OFF = 2 * HSTRIDE, G_OFF = T_OFF + 2 * TSTRIDE;
  static constexpr int LDS = G_OFF + 2 * GBYTES;
  static_assert(N % 64 == 0 && LDS <= 64 * 1024 && BM % 32 == 0, "shape");
};

template <typename T, class C>
__global__ __launch_bounds__(256, 2) void dw_fc2(const T* __restrict__ Hm, const float* __restrict__ taps,
                                               const float* __restrict__ dbias, const T* __restrict__ W2,
                                               const float* __restrict__ b2, const T* __restrict__ R,
                                               T* __restrict__ Y, int M, int K) {
  typedef v8_t<T> tx8;
  constexpr int BM = C::BM, WI = C::WI, WNB = C::WNB, MB = C::MB, IT = C::IT;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int nk = K / C::BK;

  // ---- G production mapping: tokens tok and tok + 32, channels 8 cg .. 8 cg + 7 of the K-step
  const int cg = tid & 7, tok = tid >> 3;
  uint32_t vmask[IT];                                  // bit t: tap t's neighbour is inside the image
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int m = m0 + tok + 32 * i;
    const int pix = m % (WI * WI), y = pix / WI, x = pix - y * WI;
    uint32_t v = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (m < M && yy >= 0 && yy < WI && xx >= 0 && xx < WI) v |= 1u << t;
    }
    vmask[i] = v;
  }

  // ---- halo / tap tiles of K-step kt -> buffer buf by LDS-DMA (lane-linear 1 KiB blocks; halo rows outside
  // [0, M) and the blocks' tail chunks read the zero block: they only feed masked taps)
  const char* zero = reinterpret_cast<const char*>(g_zero);
  auto dma_tiles = [&](int kt, int buf) {
    for (int blk = wave; blk < C::HBLK + C::TBLK; blk += 4) {      // wave-uniform
      const int c = (blk < C::HBLK ? blk : blk - C::HBLK) * 64 + lane;
      const char* src = zero;
      uint32_t dst;
      if (blk < C::HBLK) {
        const int r = c >> 3, q = c & 7, gm = m0 - WI - 1 + r;
        if (c < C::HCH && gm >= 0 && gm < M) src = reinterpret_cast<const char*>(Hm + (long)gm * K + kt * 64 + q * 8);
        dst = lds0 + C::H_OFF + buf * C::HSTRIDE + blk * 1024;
      } else {
        const int t = c >> 4, j = c & 15;                           // tap row t (9: bias), 4 floats
        if (c < C::TCH) src = reinterpret_cast<const char*>(t < 9 ? taps + (long)t * K + kt * 64 + j * 4 : dbias + kt * 64 + j * 4);
        dst = lds0 + C::T_OFF + buf * C::TSTRIDE + (blk - C::HBLK) * 1024;
      }
      dma16(src, __builtin_amdgcn_readfirstlane(dst));
    }
  };

  // ---- G(k) from the halo / tap tiles in buffer hb into G buffer gb
  auto produce = [&](int hb, int gb) {
    const char* hs = smem + C::H_OFF + hb * C::HSTRIDE;
    const float* ts = reinterpret_cast<const float*>(smem + C::T_OFF + hb * C::TSTRIDE) + cg * 8;
    // one token at a time, one tap at a time (sched barriers): hipcc otherwise hoists all 18 halo and 18 tap
    // reads of the step ahead of the FMAs and spills
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      float acc[8];
      {
        const float4 b0 = *reinterpret_cast<const float4*>(ts + 9 * 64), b1 = *reinterpret_cast<const float4*>(ts + 9 * 64 + 4);
        acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w;
        acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 w0 = *reinterpret_cast<const float4*>(ts + t * 64), w1 = *reinterpret_cast<const float4*>(ts + t * 64 + 4);
        const float wt[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const int dr = WI + 1 + (t / 3 - 1) * WI + (t % 3 - 1);
        uint4 h = *reinterpret_cast<const uint4*>(hs + (tok + 32 * i + dr) * 128 + cg * 16);
        if (!((vmask[i] >> t) & 1u)) h = uint4{0u, 0u, 0u, 0u};
        const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x2 p = unpack2<T>(hw[j]);
          acc[2 * j] = fmaf(p.x, wt[2 * j], acc[2 * j]);
          acc[2 * j + 1] = fmaf(p.y, wt[2 * j + 1], acc[2 * j + 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      T o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = (T)gelu_rl(acc[c]);
      const int row = tok + 32 * i;
      *reinterpret_cast<uint4*>(smem + C::G_OFF + gb * C::GBYTES + row * 128 + ((cg ^ (row & 7)) << 4)) =
          *reinterpret_cast<const uint4*>(o);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- fc2: wave's W2 fragments (n-block nb, k-step ks) and the MFMAs over the G tile in buffer gb
  const int n0w = wave * (C::N / 4);
  // W2 fragments one k-step (32 channels) at a time: the ks = 0 set is loaded during the previous step's G
  // production, the ks = 1 set while the ks = 0 MFMAs run (20 registers live instead of 40)
  tx8 w2f[WNB];
  auto load_w2 = [&](int kt, int ks) {
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb)
      w2f[nb] = *reinterpret_cast<const tx8*>(W2 + (long)(n0w + nb * 16 + fr) * K + kt * 64 + ks * 32 + fq * 8);
  };
  f32x4 acc[MB][WNB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int gb, int kt) {
    const char* gs = smem + C::G_OFF + gb * C::GBYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 1) {
        __builtin_amdgcn_sched_barrier(0);
        load_w2(kt, 1);
      }
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int row = mb * 16 + fr;
        const tx8 g = *reinterpret_cast<const tx8*>(gs + row * 128 + (((ks * 4 + fq) ^ (row & 7)) << 4));
#pragma unroll
        for (int nb = 0; nb < WNB; ++nb) acc[mb][nb] = mfma16x16x32(w2f[nb], g, acc[mb][nb]);
      }
    }
  };

  // ---- prologue: tiles 0 and 1 in LDS, G(0), the first W2 fragments
  dma_tiles(0, 0);
  if (nk > 1) dma_tiles(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  produce(0, 0);
  load_w2(0, 0);
  __syncthreads();
  // iteration k: fc2 MFMAs of K-step k (G buffer k & 1), DMA of tile k + 2 into buffer k & 1 (last read producing
  // G(k), before the previous barrier), G(k + 1) from buffer (k + 1) & 1 (DMA'd and waited for one iteration ago)
  for (int k = 0; k < nk; ++k) {
    mma(k & 1, k);
    // the MFMAs have read the W2 fragments: their registers take the next K-step's (one set live, not two)
    __builtin_amdgcn_sched_barrier(0);
    if (k + 2 < nk) dma_tiles(k + 2, k & 1);
    if (k + 1 < nk) {
      load_w2(k + 1, 0);
      produce((k + 1) & 1, (k + 1) & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // this wave's DMA of tile k + 2 landed
    __syncthreads();
  }

  // ---- epilogue: lane (fr, fq) of block (mb, nb) holds Y[m0 + 16 mb + fr][n0w + 16 nb + 4 fq .. + 3]
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + mb * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb) {
      const int n = n0w + nb * 16 + fq * 4;
      const float4 bb = *reinterpret_cast<const float4*>(b2 + n);
      float v[4] = {acc[mb][nb][0] + bb.x, acc[mb][nb][1] + bb.y, acc[mb][nb][2] + bb.z, acc[mb][nb][3] + bb.w};
      if (R) {
        const uint2 r = *reinterpret_cast<const uint2*>(R + (long)m * C::N + n);
        const f32x2 r01 = unpack2<T>(r.x), r23 = unpack2<T>(r.y);
        v[0] += r01.x; v[1] += r01.y; v[2] += r23.x; v[3] += r23.y;
      }
      const T o[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
      *reinterpret_cast<uint2*>(Y + (long)m * C::N + n) = *reinterpret_cast<const uint2*>(o);
    }
  }
}

template <typename T, class C>
static int launch(const void* H, const float* taps, const float* db, const void* W2, const float* b2, const void* R,
                  void* Y, int M, int K, hipStream_t st) {
  const int grid = (M + C::BM - 1) / C::BM;
  hipLaunchKernelGGL((dw_fc2<T, C>), dim3(grid), dim3(C::NT), 0, st, (const T*)H, taps, db, (const T*)W2, b2,
                     (const T*)R, (T*)Y, M, K);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "dw_fc2<%s, Cfg<%d, %d, %d>>", type_name<T>(), C::N, C::WI, C::BM);
  set_last_kernel(name);
  return check_launch("dw_fc2");
}

}  // namespace dwfc
// ---- stage-3 form with the depthwise conv on the MATRIX cores (round 5) -------------
// The LDS-tap form above is LDS-bound (per 64-token K-step it reads 9 halo chunks and 18 tap vectors from
// LDS for every token it produces, ≈ 220 KB).  A register-window VALU form of the same production (taps as
// DPP-fused v_fmac along image rows, measured 174 us vs 187 unfused at B = 256) is VALU-bound: 9 FMAs +
// the GELU per element at two waves per SIMD, with the fc2 MFMAs in a separate phase.  Here the depthwise
// 3x3 runs on MFMA as a block-diagonal implicit GEMM, so the VALU is left with the GELU only:
//
//   Gpre^T[c][tok] = sum_(t, c') Tap^T[c][(t, c')] * Hsh^T[(t, c')][tok],   Tap^T[c][(t, c')] = tap[t][c] [c == c']
//
// per 16-channel block: K = 9 taps x 16 channels = 144, padded to 5 MFMA k-steps (16x16x32); the A fragments
// (one non-zero per lane) are built from the taps each K-step, the B fragments are shifted reads of the H
// tile in LDS (the implicit-GEMM conv gather).  15/16 of those MFMA products are zeros, still cheaper per
// useful MAC than the VALU (512 MAC / 16 cycles vs 16 FMA / 4 cycles per SIMD).
//
//  * tile = (frame, 4 image rows) x all N output channels, m-block = one image row: 16 slots, slot x16 =
//    pixel x16 - 1 (slots 0 / 15 = the conv's zero padding; their outputs are never stored);
//  * H tile per K-step (6 image rows = the 4 output rows +- 1, 16 slots, 64 channels; rows outside the frame
//    and the padding slots from the zero block, 16-byte chunks XOR-swizzled by slot on the source address)
//    LDS-DMA'd three K-steps ahead into a 3-deep ring;
//  * wave w: the dwconv of channels 16 w .. 16 w + 15 for the 4 rows (20 MFMAs), GELU, G (16-bit, as the
//    unfused dwconv stores it) into a [64 slot][64 channel] LDS tile; then fc2 over its N / 4 output columns
//    (transposed MFMA: W2 fragment x G fragment, 40 MFMAs per K-step, a lane ends with 4 consecutive output
//    channels of one token);
//  * software pipeline, one barrier per K-step: iteration k runs the dwconv MFMAs of K-step k + 1, the fc2
//    MFMAs of k (G(k) made one iteration earlier; the W2 fragments of k + 1 are loaded behind each half), the
//    GELU of k + 1 (interleaved with those MFMAs by the scheduler), loads the taps of k + 2, DMAs H(k + 3) and
//    waits for everything but that DMA.
// Numerics: taps rounded to the 16-bit type (as autocast casts the conv weight), products exact and summed in
// f32 from the bias, gelu_rl, G rounded to 16 bits; fc2 as the GEMM (f32, + b2, + residual, one rounding).
namespace dwrw {

// Geometry.  A tile = (frame, R image rows) x all N outputs, 16 NMB token slots = NMB MFMA m-blocks of 16.  The
// H tile in LDS holds rows y0 - 1 .. in SW-slot rows: slot 0 is the conv's left zero padding and slot s the
// pixel s - 1; the right padding is slot W + 1 when SW >= W + 2 (14 x 14: SW = 16, one image row per m-block;
// 28 x 28: SW = 32, half a row per m-block, slots 30 / 31 unused zeros) or the NEXT row's slot 0 when SW = W + 1
// (7 x 7: SW = 8, two image rows per m-block; one extra zero row below).  Token slot t <-> image row
// y0 + t / SW, slot t % SW, so the tap (dy, dx) of slot t is linear slot t + dy SW + dx - 1.  Waves: NW = 4
// (N = 320: 5 fc2 n-blocks each) or 8 (N = 512: 4 each; N = 128: 1 each, 8 m-blocks), the dwconv of channel
// block cb = w % 4 of the K-step for MPW = 4 NMB / NW m-blocks per wave.
template <int N_, int WI_>
struct Cfg {
  static constexpr int N = N_, WI = WI_, BK = 64;
  static constexpr int SW = WI <= 7 ? 8 : (WI <= 14 ? 16 : 32);
  static constexpr int NMB = N == 128 ? 8 : 4, R = 16 * NMB / SW, XROW = SW == WI + 1 ? 1 : 0;
  static constexpr int NW = N == 320 ? 4 : 8, NT = 64 * NW, WNB = N / (16 * NW), MPW = 4 * NMB / NW;
  static constexpr int HROWS = R + 2 + XROW, HCH = HROWS * SW * 8;
  static constexpr int DPW = (HCH + 64 * NW - 1) / (64 * NW);   // DMA wave-instructions per wave per K-step
  // H ring slot: one 128-byte front pad (linear slot -1: the left tap of the tile's first token, a padding
  // lane whose output is never stored) + the DMA'd tile; 1 KiB of slack keeps the slots 1 KiB-aligned
  static constexpr int HBYTES = DPW * NW * 1024, HSTRIDE = HBYTES + 1024, NHB = 3, GBYTES = NMB * 16 * 128;
  static constexpr int H_OFF = 0, G_OFF = NHB * HSTRIDE, LDS = G_OFF + 2 * GBYTES;
  static constexpr int TILES_PER_FRAME = (WI + R - 1) / R;
  // packed operands (svk_mixffn_dw_fc2_pack): per K-step the W2 part [2 ks][NW waves][WNB][64 lanes] x 16 B (fc2 A
  // fragments: every W2 load of the K loop is one contiguous 1 KiB wave-instruction); after the last K-step the
  // taps rounded to T, [9][K], and dbias [K] f32, from which each lane builds its one-non-zero dwconv A fragments.
  // (Round 5 packed those fragments and the biases expanded, 6 KiB per wave per K-step: with W2 that stream
  // ran the kernel at ~14 TB/s of L2 requests, near the L2 limit; round 6 reads 5 two-byte taps + one bias chunk.)
  static constexpr int PK = 2 * NW * WNB * 64 * 16;
  static constexpr long bytes(int K) { return (long)(K / BK) * PK + 9L * K * 2 + 4L * K; }
  static_assert(N % (16 * NW) == 0 && R * SW == 16 * NMB && SW % 8 == 0 && HROWS * SW * 128 <= HBYTES &&
                SW >= WI + 1 && WNB >= 1 && MPW >= 1, "shape");
};

// packed operands: one thread per 16-byte chunk (the W2 part K-step-major, then the T taps, then dbias)
template <typename T, class C>
__global__ __launch_bounds__(256) void dwfc2_pack(const float* __restrict__ taps, const float* __restrict__ dbias,
                                                  const T* __restrict__ W2, int K, uint4* __restrict__ out) {
  const int nk = K / C::BK;
  const long id = (long)blockIdx.x * 256 + threadIdx.x, nw2 = (long)nk * (C::PK / 16), ntap = 9L * K / 8;
  if (id >= nw2 + ntap + K / 4) return;
  if (id >= nw2 + ntap) {                              // dbias, 4 floats per chunk
    const float* d = dbias + (id - nw2 - ntap) * 4;
    out[id] = uint4{__float_as_uint(d[0]), __float_as_uint(d[1]), __float_as_uint(d[2]), __float_as_uint(d[3])};
    return;
  }
  if (id >= nw2) {                                     // taps [9][K] rounded to T (as autocast casts the conv weight)
    const float* t = taps + (id - nw2) * 8;
    T v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = from_f<T>(t[q]);
    out[id] = *reinterpret_cast<const uint4*>(v);
    return;
  }
  const int kt = (int)(id / (C::PK / 16)), rr = (int)(id % (C::PK / 16));
  const int lane = rr % 64, fr = lane & 15, fq = lane >> 4;
  const int nb = (rr / 64) % C::WNB, w = (rr / (64 * C::WNB)) % C::NW, ks = rr / (64 * C::WNB * C::NW);
  out[id] = *reinterpret_cast<const uint4*>(W2 + (long)(w * (C::N / C::NW) + nb * 16 + fr) * K + kt * 64 + ks * 32 + fq * 8);
}

// gelu_rl's formula on two packed pairs (svk_common.h gelu_pk<5>: the polynomial, squares and the final fma
// as v_pk_*_f32, two chains interleaved; round 6) — not bit-identical to gelu_rl (|x| t is formed as (1 - t) / c)
__device__ __forceinline__ f32x4 gelu4_pk(f32x4 x) {
  const f32x2 a = gelu_pk<5>(f32x2{x[0], x[1]}), b = gelu_pk<5>(f32x2{x[2], x[3]});
  return f32x4{a.x, a.y, b.x, b.y};
}
// gelu_rl (dwfc::gelu_rl, bit-identical) on four values in lockstep, so four independent chains interleave
// (measured no faster than the per-element form in this kernel, kept for the explicit schedule)
__device__ __forceinline__ f32x4 gelu4(f32x4 x) {
  f32x4 ax, t, q, e, r;
#pragma unroll
  for (int i = 0; i < 4; ++i) ax[i] = fabsf(x[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = fmaf(0.3275911f * 0.70710678118654752f, ax[i], 1.0f);
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = __builtin_amdgcn_rcpf(t[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = x[i] * x[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = fmaf(-0.5f * 1.061405429f, t[i], -0.5f * -1.453152027f);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = e[i] * -0.72134752044448170f;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = fmaf(q[i], t[i], -0.5f * 1.421413741f);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_exp2f(e[i]);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = fmaf(q[i], t[i], -0.5f * -0.284496736f);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = fmaf(q[i], t[i], -0.5f * 0.254829592f);
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = ax[i] * t[i] * q[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = fmaf(r[i], e[i], fmaxf(x[i], 0.f));
  return r;
}

// GELU = false: the activation is the identity — the data gradient of a frozen MixFFN's DWConv + fc1
// (svk/train.py: dX = (dwconv3x3ᵀ dU) W1, the transposed depthwise conv being the conv with flipped taps)
// Training forward (round 6): U (optional) receives the pre-activation dwconv3x3(H) + dbias as 16-bit [M][K]
// (the GELU backward's source, as dwconv3x3's pre_out writes it), and rscale (optional) scales each token's
// fc2 output by rscale[token / rdiv] before the residual add (DropPath per frame, as gemm's row_scale).
template <typename T, class C, bool GELU = true, bool PKG = false>
__global__ __launch_bounds__(C::NT, 512 / C::NT) void dwfc2_rw(const T* __restrict__ Hm, const char* __restrict__ pk,
                                                               const float* __restrict__ b2, const T* __restrict__ R,
                                                               T* __restrict__ Y, int ntiles, int K, T* __restrict__ U,
                                                               const float* __restrict__ rscale, int rdiv) {
  typedef v8_t<T> tx8;
  constexpr int WI = C::WI, WNB = C::WNB, SW = C::SW, NW = C::NW, MPW = C::MPW, DPW = C::DPW;
  // dynamic LDS (C::LDS bytes, up to 107 KiB for 28 x 28), sized through hipFuncAttributeMaxDynamicSharedMemorySize
  extern __shared__ __attribute__((aligned(16))) uint4 smem_dwrw[];
  char* const smem = reinterpret_cast<char*>(smem_dwrw);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(dwfc::las_ptr)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int cb = wave & 3, mb0 = (wave >> 2) * MPW;    // this wave's dwconv: channel block, first m-block
  const int tile = dwfc::xcd_remap(blockIdx.x, gridDim.x);
  if (tile >= ntiles) return;
  const int frame = tile / C::TILES_PER_FRAME, y0 = (tile % C::TILES_PER_FRAME) * C::R;
  const int nk = K / C::BK;
  const long fbase = (long)frame * WI * WI;            // first token of the frame

  // ---- DMA of the H tile of K-step kt into ring slot hb: chunk q = 64 blk + lane (blk = wave + NW j): linear
  // slot L = q / 8 (row L / SW, slot L % SW), LDS chunk cs = q % 8 holds global chunk cs ^ (L & 7)
  const char* zero = reinterpret_cast<const char*>(dwfc::g_zero);
  const char* hsrc[DPW];
#pragma unroll
  for (int j = 0; j < DPW; ++j) {
    const int q = (wave + NW * j) * 64 + lane, L = q >> 3;
    const int i = L / SW, sl = L % SW, c = (q & 7) ^ (L & 7), y = y0 - 1 + i;
    hsrc[j] = (i < C::HROWS && sl >= 1 && sl <= WI && y >= 0 && y < WI)
                  ? reinterpret_cast<const char*>(Hm + (fbase + (long)y * WI + (sl - 1)) * K + c * 8)
                  : nullptr;
  }
  auto dma_h = [&](int kt, int hb) {
#pragma unroll
    for (int j = 0; j < DPW; ++j)
      dwfc::dma16(hsrc[j] ? hsrc[j] + kt * 128 : zero,
                  __builtin_amdgcn_readfirstlane(lds0 + C::H_OFF + hb * C::HSTRIDE + 128 + (wave + NW * j) * 1024));
  };

  // ---- dwconv on MFMA.  B fragment (kk, mb): lane (fr, fq) reads tap t = 2 kk + (fq >> 1) (t = 9: padding,
  // any address) of token slot u = 16 mb + fr: linear slot L = u + (t / 3) SW + t % 3 - 1 of the H tile, channels
  // 16 cb + 8 (fq & 1) .. + 7.  Padding lanes' own outputs are garbage, never stored; their reads stay inside
  // the workgroup's LDS.  (Round 5: clamping L at 0 instead of the front pad read the wrong left neighbour for
  // a 28 x 28 tile's m-block 1, whose first token is a real pixel.)
  int hoff[5];
#pragma unroll
  for (int kk = 0; kk < 5; ++kk) {
    const int t = min(2 * kk + (fq >> 1), 8), dy = t / 3, dx = t % 3;
    // m-block 0 (+ 16 slots per m-block); L = -1 only for the tile's first token (a padding lane): the front pad
    const int L = fr + dy * SW + dx - 1, c = 2 * cb + (fq & 1);
    hoff[kk] = (L + 1) * 128 + ((c ^ (L & 7)) << 4);
  }
  // dwconv A fragment kk: row = channel 16 cb + fr, k-slot 8 fq + e = (tap 2 kk + (fq >> 1), channel 8 (fq & 1) + e
  // of the block) -> the single non-zero tap[t][16 cb + fr] sits at e = fr - 8 (fq & 1) when 0 <= e < 8 (t = 9 is
  // the padding tap: zero).  Each lane loads its 5 two-byte taps and its 4 dwconv biases (one K-step at a time:
  // right after dwconv(k) has read them, for dwconv(k + 1) one iteration later) and builds the fragments in dwconv.
  const long nk_bytes = (long)(K / C::BK) * C::PK;
  const char* tapl = pk + nk_bytes + (long)(16 * cb + fr) * 2;                 // + (t K + kt 64) * 2
  const char* dbl = pk + nk_bytes + 9L * K * 2 + (16 * cb + 4 * fq) * 4;      // + kt 64 * 4
  const int ae = fr - 8 * (fq & 1);
  const bool a_lane = ae >= 0 && ae < 8;               // this lane holds the non-zero of its fragments
  const uint32_t a_sh = 16u * (ae & 1);
  const int a_dw = (ae >> 1) & 3;
  uint32_t araw[5];
  f32x4 dbv;
  auto load_a = [&](int kt) {
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const int t = min(2 * kk + (fq >> 1), 8);        // (t = 9 loads tap 8; zeroed when the fragment is built)
      asm volatile("global_load_ushort %0, %1, off" : "=v"(araw[kk]) : "v"(tapl + ((long)t * K + kt * 64) * 2) : "memory");
    }
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dbv) : "v"(dbl + kt * 256) : "memory");
  };
  auto tie_a = [&]() {
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) asm volatile("" : "+v"(araw[kk]));
    asm volatile("" : "+v"(dbv));
  };
  f32x4 dacc[MPW];
  auto dwconv = [&](int hb) {
    const char* hs = smem + C::H_OFF + hb * C::HSTRIDE + mb0 * 2048;
    tx8 afr[5];
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const bool nz = a_lane && 2 * kk + (fq >> 1) < 9;
      const uint32_t v = nz ? (araw[kk] & 0xFFFFu) << a_sh : 0u;
      uint4 d;
      d.x = a_dw == 0 ? v : 0u;
      d.y = a_dw == 1 ? v : 0u;
      d.z = a_dw == 2 ? v : 0u;
      d.w = a_dw == 3 ? v : 0u;
      afr[kk] = *reinterpret_cast<const tx8*>(&d);
    }
#pragma unroll
    for (int m = 0; m < MPW; ++m) dacc[m] = dbv;
#pragma unroll
    for (int kk = 0; kk < 5; ++kk)
#pragma unroll
      for (int m = 0; m < MPW; ++m)
        dacc[m] = mfma16x16x32(afr[kk], *reinterpret_cast<const tx8*>(hs + hoff[kk] + m * 2048), dacc[m]);
  };
  // GELU of the dwconv outputs -> G tile gb: lane (fr, fq) of m-block mb = channels 16 cb + 4 fq .. + 3, slot 16 mb + fr
  // (U: the pre-activation of K-step kt to HBM, 8-byte pieces, padding slots skipped)
  auto gelu_store = [&](int gb, int kt) {
    if (U) {
#pragma unroll
      for (int m = 0; m < MPW; ++m) {
        const int t = (mb0 + m) * 16 + fr, y = y0 + t / SW, x = t % SW - 1;
        if (y < WI && x >= 0 && x < WI) {
          const T o[4] = {from_f<T>(dacc[m][0]), from_f<T>(dacc[m][1]), from_f<T>(dacc[m][2]), from_f<T>(dacc[m][3])};
          *reinterpret_cast<uint2*>(U + (fbase + (long)y * WI + x) * K + kt * 64 + 16 * cb + 4 * fq) =
              *reinterpret_cast<const uint2*>(o);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MPW; ++m) {
      const f32x4 gv = GELU ? (PKG ? gelu4_pk(dacc[m]) : gelu4(dacc[m])) : dacc[m];
      const T o[4] = {from_f<T>(gv[0]), from_f<T>(gv[1]), from_f<T>(gv[2]), from_f<T>(gv[3])};
      const int s = (mb0 + m) * 16 + fr, cw = 16 * cb + 4 * fq;
      *reinterpret_cast<uint2*>(smem + C::G_OFF + gb * C::GBYTES + s * 128 + ((((cw >> 3) ^ (s & 7)) << 4) | ((cw & 4) << 1))) =
          *reinterpret_cast<const uint2*>(o);
    }
  };

  // ---- fc2: wave's n-blocks n0w + 16 nb over the 4 m-blocks, W2 fragments of one K-step (2 x 32 channels)
  const int n0w = wave * (C::N / NW);
  tx8 w2f[2][WNB];
  const char* pkl = pk + lane * 16;
  auto load_w2 = [&](int kt, int ks) {
    const char* src = pkl + (long)kt * C::PK + (ks * NW + wave) * WNB * 1024;
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(w2f[ks][nb]) : "v"(src + nb * 1024) : "memory");
  };
  auto tie_w2 = [&]() {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < WNB; ++nb) asm volatile("" : "+v"(w2f[ks][nb]));
  };
  constexpr int NMB = C::NMB;
  f32x4 acc[NMB][WNB];
#pragma unroll
  for (int mb = 0; mb < NMB; ++mb)
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto fc2_half = [&](int gb, int ks) {
    const char* gs = smem + C::G_OFF + gb * C::GBYTES;
#pragma unroll
    for (int mb = 0; mb < NMB; ++mb) {
      const int row = mb * 16 + fr;
      const tx8 g = *reinterpret_cast<const tx8*>(gs + row * 128 + (((ks * 4 + fq) ^ (row & 7)) << 4));
#pragma unroll
      for (int nb = 0; nb < WNB; ++nb) acc[mb][nb] = mfma16x16x32(w2f[ks][nb], g, acc[mb][nb]);
    }
  };

  // ---- prologue: H(0..2) in the ring, A(0) -> G(0), A(1), W2(0)
  load_a(0);
  dma_h(0, 0);
  dma_h(min(1, nk - 1), 1);
  dma_h(min(2, nk - 1), 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tie_a();
  __syncthreads();
  dwconv(0);
  gelu_store(0, 0);
  load_a(min(1, nk - 1));
  load_w2(0, 0);
  load_w2(0, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tie_a();
  tie_w2();
  __syncthreads();
  // iteration kt < nk - 1: dwconv(kt + 1), then A(kt + 2) into the registers it read; fc2(kt) with W2(kt + 1)
  // loaded behind each half; GELU(kt + 1) -> G ring; DMA H(kt + 3) into the slot dwconv(kt) read (before the
  // previous barrier; clamped past the end: never read); the counted wait leaves only that DMA in flight
  for (int kt = 0; kt + 1 < nk; ++kt) {
    dwconv((kt + 1) % 3);
    load_a(min(kt + 2, nk - 1));
    fc2_half(kt & 1, 0);
    load_w2(kt + 1, 0);
    fc2_half(kt & 1, 1);
    load_w2(kt + 1, 1);
    gelu_store((kt + 1) & 1, kt + 1);
    dma_h(min(kt + 3, nk - 1), kt % 3);
    // A(kt + 2) [6] and W2(kt + 1) [2 WNB] retired; the DMA [DPW] not
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
    tie_a();
    tie_w2();
    __syncthreads();
  }
  fc2_half((nk - 1) & 1, 0);
  fc2_half((nk - 1) & 1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the clamped tail DMA (never read) retires

  // ---- epilogue: lane (fr, fq) of block (mb, nb) = token slot 16 mb + fr, channels n .. n + 3
#pragma unroll
  for (int mb = 0; mb < NMB; ++mb) {
    const int t = mb * 16 + fr, y = y0 + t / SW, x = t % SW - 1;
    if (y >= WI || x < 0 || x >= WI) continue;
    const long m = fbase + (long)y * WI + x;
    const float rs = rscale ? rscale[m / rdiv] : 1.f;
#pragma unroll
    for (int nb = 0; nb < WNB; ++nb) {
      const int n = n0w + nb * 16 + fq * 4;
      const float4 bb = *reinterpret_cast<const float4*>(b2 + n);
      float v[4] = {acc[mb][nb][0] + bb.x, acc[mb][nb][1] + bb.y, acc[mb][nb][2] + bb.z, acc[mb][nb][3] + bb.w};
      if (rscale) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= rs;
      }
      if (R) {
        const uint2 r = *reinterpret_cast<const uint2*>(R + m * C::N + n);
        const f32x2 r01 = unpack2<T>(r.x), r23 = unpack2<T>(r.y);
        v[0] += r01.x; v[1] += r01.y; v[2] += r23.x; v[3] += r23.y;
      }
      const T o[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
      *reinterpret_cast<uint2*>(Y + m * C::N + n) = *reinterpret_cast<const uint2*>(o);
    }
  }
}


template <typename T, class C, bool GELU = true>
static int launch(const void* H, const void* pk, const float* b2, const void* R, void* Y, int B, int K, hipStream_t st,
                  void* U = nullptr, const float* rscale = nullptr, int rdiv = 1) {
  const long nt = (long)B * C::TILES_PER_FRAME;
  if (nt > 0x7fffffffL || (long)B * C::WI * C::WI * K > 0x7fffffffL) return SVK_EUNSUPPORTED;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dwfc2_rw<T, C, GELU, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dwfc2_rw<T, C, GELU, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  if (GELU && gelu_pk_on())   // GELU on packed f32 pairs (svk_common.h gelu_pk; SVK_GELU_PK=0: element-wise)
    hipLaunchKernelGGL((dwfc2_rw<T, C, GELU, true>), dim3((unsigned)nt), dim3(C::NT), C::LDS, st, (const T*)H,
                       (const char*)pk, b2, (const T*)R, (T*)Y, (int)nt, K, (T*)U, rscale, rdiv);
  else
    hipLaunchKernelGGL((dwfc2_rw<T, C, GELU, false>), dim3((unsigned)nt), dim3(C::NT), C::LDS, st, (const T*)H,
                       (const char*)pk, b2, (const T*)R, (T*)Y, (int)nt, K, (T*)U, rscale, rdiv);
  static char name[64];
  if (!name[0])
    snprintf(name, sizeof(name), "dw_fc2_mx<%s, Cfg<%d, %d>%s>", type_name<T>(), C::N, C::WI, GELU ? "" : ", identity");
  set_last_kernel(name);
  return check_launch("dw_fc2_mx");
}

template <typename T, class C>
static int pack(const float* taps, const float* db, const void* W2, int K, void* out, hipStream_t st) {
  const long n = C::bytes(K) / 16;
  hipLaunchKernelGGL((dwfc2_pack<T, C>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, taps, db, (const T*)W2, K,
                     (uint4*)out);
  return check_launch("dw_fc2_pack");
}

}  // namespace dwrw
}  // namespace svk

using namespace svk;

extern "C" int svk_mixffn_dw_fc2_supported(int dtype, int W, int N, int K) {
  return (dtype == SVK_F16 || dtype == SVK_BF16) && ((W == 14 && N == 320) || (W == 7 && N == 512)) && K % 64 == 0 &&
         K >= 64;
}

extern "C" int svk_mixffn_dw_fc2(int dtype, const void* H, const float* taps, const float* dbias, const void* W2,
                                 const float* b2, const void* R, void* Y, int B, int Himg, int Wimg, int K, int N,
                                 void* stream) {
  if (B < 0 || Himg <= 0 || Wimg <= 0 || K <= 0 || N <= 0 || !H || !taps || !dbias || !W2 || !b2 || !Y) {
    set_error("svk_mixffn_dw_fc2: bad args"); return SVK_EINVAL;
  }
  if (Himg != Wimg || !svk_mixffn_dw_fc2_supported(dtype, Wimg, N, K)) {
    set_error("svk_mixffn_dw_fc2: (dtype=%d, %dx%d, N=%d, K=%d) not instantiated", dtype, Himg, Wimg, N, K);
    return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)H) | ((uintptr_t)W2) | ((uintptr_t)taps) | ((uintptr_t)dbias) | ((uintptr_t)b2)) & 15 ||
      (((uintptr_t)Y) | ((uintptr_t)R)) & 7) {
    set_error("svk_mixffn_dw_fc2: misaligned operand"); return SVK_EINVAL;
  }
  const long M = (long)B * Himg * Wimg;
  if (M == 0) return SVK_OK;
  if (M * K > 0x7fffffffL) { set_error("svk_mixffn_dw_fc2: too many tokens"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    if (N == 512) return dwfc::launch<T, dwfc::Cfg<512, 7, 32>>(H, taps, dbias, W2, b2, R, Y, (int)M, K, st);
    return dwfc::launch<T, dwfc::Cfg<320, 14, 64>>(H, taps, dbias, W2, b2, R, Y, (int)M, K, st);
  });
}

// ---- the stage-3 form with the depthwise conv on MFMA: operands packed once per weight set -------------
extern "C" long svk_mixffn_dw_fc2_packed_bytes(int dtype, int W, int N, int K) {
  if (!(dtype == SVK_F16 || dtype == SVK_BF16) || K % 64 || K <= 0) return 0;
  if (W == 14 && N == 320) return dwrw::Cfg<320, 14>::bytes(K);
  if (W == 7 && N == 512) return dwrw::Cfg<512, 7>::bytes(K);
  if (W == 28 && N == 128) return dwrw::Cfg<128, 28>::bytes(K);
  return 0;
}

extern "C" int svk_mixffn_dw_fc2_pack(int dtype, const float* taps, const float* dbias, const void* W2, int W, int N,
                                      int K, void* packed, void* stream) {
  if (!taps || !dbias || !W2 || !packed) { set_error("svk_mixffn_dw_fc2_pack: bad args"); return SVK_EINVAL; }
  if (svk_mixffn_dw_fc2_packed_bytes(dtype, W, N, K) == 0) {
    set_error("svk_mixffn_dw_fc2_pack: (dtype=%d, W=%d, N=%d, K=%d) has no packed form", dtype, W, N, K);
    return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)packed) | ((uintptr_t)W2)) & 15) { set_error("svk_mixffn_dw_fc2_pack: misaligned operand"); return SVK_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    if (W == 7) return dwrw::pack<T, dwrw::Cfg<512, 7>>(taps, dbias, W2, K, packed, st);
    if (W == 28) return dwrw::pack<T, dwrw::Cfg<128, 28>>(taps, dbias, W2, K, packed, st);
    return dwrw::pack<T, dwrw::Cfg<320, 14>>(taps, dbias, W2, K, packed, st);
  });
}

extern "C" int svk_mixffn_dw_fc2_packed_act(int dtype, const void* H, const void* packed, const float* b2,
                                            const void* R, void* Y, int B, int Himg, int Wimg, int K, int N, int act,
                                            void* stream);

extern "C" int svk_mixffn_dw_fc2_packed(int dtype, const void* H, const void* packed, const float* b2, const void* R,
                                        void* Y, int B, int Himg, int Wimg, int K, int N, void* stream) {
  return svk_mixffn_dw_fc2_packed_act(dtype, H, packed, b2, R, Y, B, Himg, Wimg, K, N, SVK_ACT_GELU, stream);
}

extern "C" int svk_mixffn_dw_fc2_packed_ex(int dtype, const void* H, const void* packed, const float* b2,
                                           const void* R, void* Y, int B, int Himg, int Wimg, int K, int N, int act,
                                           void* U, const float* rscale, int rdiv, void* stream);

extern "C" int svk_mixffn_dw_fc2_packed_act(int dtype, const void* H, const void* packed, const float* b2,
                                            const void* R, void* Y, int B, int Himg, int Wimg, int K, int N, int act,
                                            void* stream) {
  return svk_mixffn_dw_fc2_packed_ex(dtype, H, packed, b2, R, Y, B, Himg, Wimg, K, N, act, nullptr, nullptr, 1, stream);
}

extern "C" int svk_mixffn_dw_fc2_packed_ex(int dtype, const void* H, const void* packed, const float* b2,
                                           const void* R, void* Y, int B, int Himg, int Wimg, int K, int N, int act,
                                           void* U, const float* rscale, int rdiv, void* stream) {
  if (act != SVK_ACT_GELU && act != SVK_ACT_NONE) { set_error("svk_mixffn_dw_fc2_packed: act must be GELU or NONE"); return SVK_EINVAL; }
  if (B < 0 || Himg <= 0 || Wimg <= 0 || !H || !packed || !b2 || !Y) { set_error("svk_mixffn_dw_fc2_packed: bad args"); return SVK_EINVAL; }
  if (Himg != Wimg || svk_mixffn_dw_fc2_packed_bytes(dtype, Wimg, N, K) == 0) {
    set_error("svk_mixffn_dw_fc2_packed: (dtype=%d, %dx%d, N=%d, K=%d) has no packed form", dtype, Himg, Wimg, N, K);
    return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)H) | ((uintptr_t)packed) | ((uintptr_t)b2)) & 15 || (((uintptr_t)Y) | ((uintptr_t)R) | ((uintptr_t)U)) & 7) {
    set_error("svk_mixffn_dw_fc2_packed: misaligned operand"); return SVK_EINVAL;
  }
  if (rscale && rdiv <= 0) { set_error("svk_mixffn_dw_fc2_packed: rdiv must be positive"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    if (U || rscale) {                 // the training forward (GELU; 14 x 14 / 7 x 7)
      if (act != SVK_ACT_GELU || Wimg == 28) {
        set_error("svk_mixffn_dw_fc2_packed_ex: pre-activation / row scale need act GELU at 14 x 14 or 7 x 7");
        return SVK_EUNSUPPORTED;
      }
      if (Wimg == 7) return dwrw::launch<T, dwrw::Cfg<512, 7>>(H, packed, b2, R, Y, B, K, st, U, rscale, rdiv);
      return dwrw::launch<T, dwrw::Cfg<320, 14>>(H, packed, b2, R, Y, B, K, st, U, rscale, rdiv);
    }
    if (act == SVK_ACT_NONE) {
      if (Wimg == 7) return dwrw::launch<T, dwrw::Cfg<512, 7>, false>(H, packed, b2, R, Y, B, K, st);
      if (Wimg == 28) { set_error("svk_mixffn_dw_fc2_packed: no identity form for 28 x 28"); return SVK_EUNSUPPORTED; }
      return dwrw::launch<T, dwrw::Cfg<320, 14>, false>(H, packed, b2, R, Y, B, K, st);
    }
    if (Wimg == 7) return dwrw::launch<T, dwrw::Cfg<512, 7>>(H, packed, b2, R, Y, B, K, st);
    if (Wimg == 28) return dwrw::launch<T, dwrw::Cfg<128, 28>>(H, packed, b2, R, Y, B, K, st);
    return dwrw::launch<T, dwrw::Cfg<320, 14>>(H, packed, b2, R, Y, B, K, st);
  });
}
