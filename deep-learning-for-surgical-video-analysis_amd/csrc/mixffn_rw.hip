// Whole MixFFN + Block residual (+ the stage LayerNorm) in one kernel, f16, with the depthwise window
// held in REGISTERS (mix_transformer_evp.py:32-67, DWConv :19-30, Block :169, stage norm :370-412):
//
//   Y  = X + fc2( GELU( dwconv3x3( fc1(XN) ) ) )          NHWC [B, H, W, C] f16, hidden 4C
//   Yn = LN(Y)                                            (when gamma != nullptr; Y may then be null)
//
// Why a second design next to mixffn.hip: the wave-specialised kernel there moves the hidden map
// through LDS (fc1 waves write it, dwconv waves read 3x3 neighbourhoods back, fc2 waves read the GELU
// output), with one workgroup per CU and a barrier per 32-channel chunk: its dwconv waves issue VALU
// ~20 % of the time (LDS latency + barrier waits).  Here nothing of the hidden map touches LDS:
//
//   * the MFMA layout IS the conv layout.  fc1 is computed transposed (D = W1 · XNᵀ, 16x16x32), so
//     lane (fr, fq) ends with hidden channels 4fq .. 4fq+3 (of a 16-channel n-tile) of token fr, and a
//     16-token m-tile is 16 consecutive pixels x0-1 .. x0+14 of one image row.  Vertical taps are the
//     previous / next image rows, which the same lane computed in earlier iterations (a 3-row rolling
//     window, f16-rounded values held as f32); horizontal taps are the neighbouring lanes, read through
//     v_fmac_f32's DPP source operand (row_shr:1 / row_shl:1 inside each 16-lane row): 9 full-rate
//     FMAs per output, no shuffle instructions.  Lanes 0 and 15 are the halo columns (14 outputs each).
//   * the GELU output lands directly in the fc2 operand layout: lane (fr, fq) holds 8 hidden values of
//     token fr for each 32-channel k-step — fc2's reduction index is permuted to match (the W2
//     fragments are gathered accordingly once, in the prologue).  fc2 is transposed too, so a lane ends
//     with 4 consecutive output channels of one token.
//   * a workgroup = HID / 64 waves (4 for C = 64) splitting the hidden channels 64 each, so every wave
//     keeps its W1 / W2 fragments in registers for the whole (persistent) kernel; the per-row fc2
//     partial sums of the waves meet once in LDS (f32 slabs, double-buffered, ONE barrier per row),
//     where each wave reduces a quarter of the tokens and runs the epilogue (+ b2 + residual, LayerNorm
//     over the 16 lanes holding a token, 8-byte stores).  The taps (f32, per n-tile and tap row) stream
//     from LDS one step ahead of their use.
//
// Work unit: (frame, 14-column x-tile, strip of R rows); a wave walks the strip top to bottom, software-
// pipelined: row r issues the fc1 MFMAs of hidden row y + 2 and the X loads of row y + 3, then writes the
// fc2 partial sums of row y - 1 and runs its epilogue, then the dwconv + GELU + fc2 MFMAs of row y.
// Measured (B = 256, stage 1): 335 us vs 348 us for the wave-specialised mixffn_ws; rocprofv3 counters:
// each wave issues VALU 44 % of its cycles at 2 waves per SIMD (233 VGPRs) — GELU and the dwconv taps are
// ~60 % of the VALU instructions; the rest of the time is LDS / MFMA latency the two waves do not cover.
// Numerics as mixffn.hip: fc1 output, taps and GELU output rounded to f16 (the reference's autocast
// stores), accumulation / bias / GELU / LayerNorm statistics in f32.
#include "svk_common.h"
#include <type_traits>

namespace svk {
namespace ffnrw {

template <int C_, int W_, int R_, int OCC_ = 2, bool BI_ = true>
struct Cfg {
  static constexpr int C = C_, W = W_, R = R_, OCC = OCC_;
  static constexpr bool BIAS_INIT = BI_;   // fc1's bias as the MFMA accumulator's initial value (else added after)
  static constexpr int HID = 4 * C, NW = HID / 64, NT = 64 * NW;
  static constexpr int KS = C / 32;                 // fc1 k-steps
  static constexpr int NC2 = C / 16;                // fc2 output n-tiles
  static constexpr int XT = (W + 13) / 14;          // 14-column x-tiles
  static constexpr int TPW = 16 / NW;               // epilogue tokens per wave
  static constexpr int LPT = 64 / TPW;              // epilogue lanes per token (4 channels each)
  static constexpr int SROW = C + 4;                // slab row (floats): conflict-free 16-byte writes
  static constexpr int SLAB = 16 * SROW;            // one wave's partial sums of a row
  static constexpr int TBLK = 160;                  // tap block (wave, n-tile, fq): taps [9][4], dwb [4] (f32)
  static constexpr int LDS_TP = HID * 4;             // b1 (f32) | tap blocks | b2, gamma, beta | slabs
  static constexpr int LDS_EP = LDS_TP + NW * 16 * TBLK;
  static constexpr int LDS_T = LDS_EP + 3 * C * 4;
  static constexpr int LDS = LDS_T + 2 * NW * SLAB * 4;
  static_assert(C % 32 == 0 && NW >= 1 && NW <= 4 && LPT * 4 == C, "shape");
};

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk(float lo, float hi) { return __builtin_bit_cast(uint32_t, h2{(_Float16)lo, (_Float16)hi}); }
__device__ __forceinline__ float lo16(uint32_t u) { return (float)__builtin_bit_cast(h2, u).x; }
__device__ __forceinline__ float hi16(uint32_t u) { return (float)__builtin_bit_cast(h2, u).y; }
// value of lane l - 1 / l + 1 inside each 16-lane row (0 at the row ends: halo lanes, never stored)
__device__ __forceinline__ uint32_t from_left(uint32_t v) { return __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true); }
__device__ __forceinline__ uint32_t from_right(uint32_t v) { return __builtin_amdgcn_update_dpp(0u, v, 0x101, 0xf, 0xf, true); }
// acc[c] += h[x-1][c] t[c] + h[x][c] t[4+c] + h[x+1][c] t[8+c]: the horizontal neighbours come through
// v_fmac_f32's DPP source operand (row_shr:1 / row_shl:1 within each 16-lane row, 0 at the row ends).
// The four plain FMAs go first: they give the DPP reads of h the two wait states a VALU write needs.
__device__ __forceinline__ void taps3(float (&acc)[4], const float (&h)[4], const float (&t)[12]) {
  asm("v_fmac_f32 %0, %4, %12\n\t"    // centre taps t[4..7]
      "v_fmac_f32 %1, %5, %13\n\t"
      "v_fmac_f32 %2, %6, %14\n\t"
      "v_fmac_f32 %3, %7, %15\n\t"
      "v_fmac_f32_dpp %0, %4, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %1, %5, %9 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %2, %6, %10 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %3, %7, %11 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %0, %4, %16 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %1, %5, %17 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %2, %6, %18 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %3, %7, %19 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
      : "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3]), "v"(t[4]),
        "v"(t[5]), "v"(t[6]), "v"(t[7]), "v"(t[8]), "v"(t[9]), "v"(t[10]), "v"(t[11]));
}

// gelu(x) = relu(x) - 0.5 |x| t q(t) exp(-x^2 / 2), 1 - erf(z) = t q(t) exp(-z^2) by Abramowitz & Stegun
// 7.1.25 (|error| <= 2.5e-5, 40x below the f16 rounding of the output): 9 VALU + 2 transcendental
__device__ __forceinline__ float gelu_rw(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.47047f * 0.70710678118654752f, ax, 1.0f));
  const float q = fmaf(fmaf(-0.5f * 0.7478556f, t, -0.5f * -0.0958798f), t, -0.5f * 0.3480242f);
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
  return fmaf(ax * t * q, e, fmaxf(x, 0.f));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <class K>
__global__ __launch_bounds__(K::NT, K::OCC) void mixffn_rw(const f16* __restrict__ XN, const f16* __restrict__ X,
                                                     const f16* __restrict__ W1, const float* __restrict__ b1,
                                                     const float* __restrict__ taps, const float* __restrict__ dwb,
                                                     const f16* __restrict__ W2, const float* __restrict__ b2,
                                                     f16* __restrict__ Y, f16* __restrict__ Yn,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, int H, int nstrip, int total) {
  constexpr int C = K::C, W = K::W, R = K::R, HID = K::HID, KS = K::KS, NC2 = K::NC2, NW = K::NW;
  constexpr bool BIAS_INIT = K::BIAS_INIT;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  char* const smem = reinterpret_cast<char*>(smem4);
  float* const slab0 = reinterpret_cast<float*>(smem + K::LDS_T);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- prologue: b1 [HID] f32 and the tap blocks in LDS; W1 / W2 fragments of this wave's 64 hidden
  // channels in registers (4 n-tiles x KS k-steps; 2 k-steps of 32 hidden x NC2 output n-tiles) with
  // fc2's reduction index permuted to the GELU output layout: k-slot 8 fq + s of k-step q <-> hidden
  // 32 q + 4 fq + s (s < 4), 32 q + 16 + 4 fq + s - 4 (s >= 4)
  for (int e = tid; e < HID; e += K::NT) reinterpret_cast<float*>(smem)[e] = b1[e];
  for (int e = tid; e < NW * 16 * 40; e += K::NT) {
    // block blk = (w * 4 + j) * 4 + fq holds channels 4 blk + c: float t * 4 + c = tap t (rounded to f16,
    // as autocast casts the conv weight), then the depthwise bias
    const int blk = e / 40, r = e % 40, t = r / 4, c = r % 4;
    reinterpret_cast<float*>(smem + K::LDS_TP + blk * K::TBLK)[r] =
        t < 9 ? (float)(f16)taps[t * HID + 4 * blk + c] : dwb[4 * blk + c];
  }
  f16x8 w1f[4][KS], w2f[2][NC2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      w1f[j][ks] = *reinterpret_cast<const f16x8*>(W1 + (long)(64 * w + 16 * j + fr) * C + 32 * ks + 8 * fq);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int c = 0; c < NC2; ++c) {
      const f16* src = W2 + (long)(16 * c + fr) * HID + 64 * w + 32 * q + 4 * fq;
      const f16x4 lo = *reinterpret_cast<const f16x4*>(src), hi = *reinterpret_cast<const f16x4*>(src + 16);
      w2f[q][c] = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  float* const sEp = reinterpret_cast<float*>(smem + K::LDS_EP);   // b2 [C], gamma [C], beta [C]
  for (int e = tid; e < 3 * C; e += K::NT)
    sEp[e] = e < C ? b2[e] : (gamma ? (e < 2 * C ? gamma[e - C] : beta[e - 2 * C]) : (e < 2 * C ? 1.f : 0.f));
  // epilogue lane: token et = TPW w + lane / LPT of the m-tile, channels 4 ec .. 4 ec + 3
  const int et = K::TPW * w + lane / K::LPT, ec = lane % K::LPT;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  const float* b1l = reinterpret_cast<const float*>(smem) + 64 * w + 4 * fq;   // + 16 j
  const uint4* tpl = reinterpret_cast<const uint4*>(smem + K::LDS_TP + (w * 16 + fq) * K::TBLK);   // + j * 4 * TBLK / 16
  const int G = gridDim.x;
  int buf = 0;
  for (int u = xcd_remap(blockIdx.x, G); u < total; u += G) {
    const int xt = u % K::XT, rest = u / K::XT, sidx = rest % nstrip, b = rest / nstrip;
    const int y0 = sidx * R, x0 = 14 * xt;
    const int tx = x0 - 1 + fr;                          // this lane's pixel column (fc1 / dwconv)
    const bool xok = tx >= 0 && tx < W;
    const f16* XNb = XN + (long)b * H * W * C + (long)min(max(tx, 0), W - 1) * C + 8 * fq;
    auto load_x = [&](int yy, f16x8 (&xf)[KS]) __attribute__((always_inline)) {
      const f16* src = XNb + (long)min(max(yy, 0), H - 1) * W * C;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xf[ks] = *reinterpret_cast<const f16x8*>(src + 32 * ks);
    };
    // fc1 of hidden row yy: MFMAs issued early, packed (+ b1, f16, zero outside the image) late, so the
    // dwconv of the current row runs while they are in flight
    // (the accumulators start from b1: the bias add rides on the MFMA)
    auto fc1_mma = [&](const f16x8 (&wf)[4][KS], const f16x8 (&xf)[KS], f32x4 (&a)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = BIAS_INIT ? *reinterpret_cast<const f32x4*>(b1l + 16 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a[j] = mfma16x16x32(wf[j][ks], xf[ks], a[j]);
      }
    };
    // hidden values rounded to f16 (the autocast Linear output) and kept as f32: the depthwise taps then
    // run as full-rate v_fmac_f32 with the horizontal shift folded in as a DPP operand
    // the zero padding of the conv: only tiles at the image's left / right edge (lanes 0 / 15 outside) and the
    // rows above / below the image need the mask (a wave-uniform test)
    const bool edge = x0 == 0 || x0 + 15 > W;
    auto fc1_pack = [&](int yy, const f32x4 (&a)[4], float (&hw)[4][4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 bb = BIAS_INIT ? float4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const float4*>(b1l + 16 * j);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) hw[j][c] = (float)(f16)(BIAS_INIT ? a[j][c] : a[j][c] + bv[c]);
      }
      if (edge || yy < 0 || yy >= H) {
        const uint32_t m = (xok && yy >= 0 && yy < H) ? ~0u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 4; ++c) hw[j][c] = __uint_as_float(__float_as_uint(hw[j][c]) & m);
      }
    };
    float win[3][4][4];
    {
      f16x8 xa[KS], xb[KS], xc[KS];
      f32x4 a[4];
      load_x(y0 - 1, xa);
      load_x(y0, xb);
      load_x(y0 + 1, xc);
      fc1_mma(w1f, xa, a);
      fc1_pack(y0 - 1, a, win[0]);
      fc1_mma(w1f, xb, a);
      fc1_pack(y0, a, win[1]);
      fc1_mma(w1f, xc, a);
      fc1_pack(y0 + 1, a, win[2]);
    }
    f16x8 xn[KS];                 // X row of the next new hidden row (y + 2), prefetched a row ahead
    load_x(y0 + 2, xn);
    // epilogue row operands: residual of (row, token et, channels 4 ec..)
    const int etx = x0 - 1 + et;
    const bool eok = et >= 1 && et <= 14 && etx < W;
    const long eoff0 = ((long)b * H * W + min(max(etx, 0), W - 1)) * C + 4 * ec;   // halo lanes: clamped, never stored
    // ---- epilogue of row yy from slab buffer bb: token et, channels 4 ec .. 4 ec + 3
    auto epilogue = [&](int yy, uint2 res, int bb) __attribute__((always_inline)) {
      float4 v = *reinterpret_cast<const float4*>(slab0 + bb * NW * K::SLAB + et * K::SROW + 4 * ec);
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
        const float4 o = *reinterpret_cast<const float4*>(slab0 + (bb * NW + ww) * K::SLAB + et * K::SROW + 4 * ec);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      const f32x2 r01 = unpack2<f16>(res.x), r23 = unpack2<f16>(res.y);
      const float4 eb2 = *reinterpret_cast<const float4*>(sEp + 4 * ec);
      const f16 o0 = (f16)(v.x + eb2.x + r01.x), o1 = (f16)(v.y + eb2.y + r01.y);
      const f16 o2 = (f16)(v.z + eb2.z + r23.x), o3 = (f16)(v.w + eb2.w + r23.y);
      const bool st = eok && yy < H;
      const long oo = eoff0 + (long)yy * W * C;
      if (Y && st) *reinterpret_cast<f16x4*>(Y + oo) = f16x4{o0, o1, o2, o3};
      if (gamma) {   // LayerNorm of the token's C channels: LPT lanes (a power of two, aligned)
        const float f0 = o0, f1 = o1, f2 = o2, f3 = o3;
        float sm = f0 + f1 + f2 + f3;
#pragma unroll
        for (int m = K::LPT / 2; m >= 1; m >>= 1) sm += __shfl_xor(sm, m, 64);
        const float mean = sm * (1.0f / C);
        const float d0 = f0 - mean, d1 = f1 - mean, d2 = f2 - mean, d3 = f3 - mean;
        float q = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
#pragma unroll
        for (int m = K::LPT / 2; m >= 1; m >>= 1) q += __shfl_xor(q, m, 64);
        const float rstd = 1.0f / sqrtf(q * (1.0f / C) + eps);
        const float4 egam = *reinterpret_cast<const float4*>(sEp + C + 4 * ec);
        const float4 ebet = *reinterpret_cast<const float4*>(sEp + 2 * C + 4 * ec);
        if (st)
          *reinterpret_cast<f16x4*>(Yn + oo) = f16x4{(f16)(d0 * rstd * egam.x + ebet.x), (f16)(d1 * rstd * egam.y + ebet.y),
                                                     (f16)(d2 * rstd * egam.z + ebet.z), (f16)(d3 * rstd * egam.w + ebet.w)};
      }
    };
    // fc2 partial sums -> this wave's slab of buffer bb, then the workgroup barrier
    auto slab_sync = [&](const f32x4 (&a2)[NC2], int bb) __attribute__((always_inline)) {
      float* sl = slab0 + (bb * NW + w) * K::SLAB;
#pragma unroll
      for (int c = 0; c < NC2; ++c) *reinterpret_cast<f32x4*>(sl + fr * K::SROW + 16 * c + 4 * fq) = a2[c];
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    // taps of (n-tile j, tap row dy): 12 floats [dx][c]
    auto tload = [&](int jd, float (&t)[12]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const uint4 v = tpl[(jd / 3) * 4 * K::TBLK / 16 + (jd % 3) * 3 + i];
        t[4 * i] = __uint_as_float(v.x); t[4 * i + 1] = __uint_as_float(v.y);
        t[4 * i + 2] = __uint_as_float(v.z); t[4 * i + 3] = __uint_as_float(v.w);
      }
    };
    // Software pipeline over the strip's rows: row r issues the fc1 MFMAs of hidden row y + 2, writes the
    // fc2 partial sums of row y - 1 (MFMAs issued a whole dwconv earlier) and runs its epilogue, then the
    // dwconv + GELU + fc2 MFMAs of row y; the last row's reduction drains after the loop.
    f32x4 a2[NC2];
    uint2 res_prev = {0u, 0u};
    // one row; the 3-row window rotates through the slots instead of being copied: at row r the rows y - 1, y,
    // y + 1 sit in slots (ROT + 0, 1, 2) % 3 with ROT = r % 3, and the new row y + 2 replaces slot ROT
    auto row = [&](int r, auto ROT_) __attribute__((always_inline)) {
      constexpr int ROT = decltype(ROT_)::value;
      const int y = y0 + r;
      // this row's residual (its epilogue runs one row later), then the fc1 MFMAs of hidden row y + 2
      // and the X row of hidden row y + 3, a row ahead of its use
      const uint2 res = *reinterpret_cast<const uint2*>(X + eoff0 + (long)min(y, H - 1) * W * C);
      f32x4 a1[4];
      fc1_mma(w1f, xn, a1);
      load_x(y + 3, xn);          // (clamped; unconditional: no branch for the waitcnt pass to merge)
      // keep the loads here (the scheduler would sink them to save registers)
      __builtin_amdgcn_sched_barrier(0);
      float tq[2][12];
      tload(0, tq[0]);
      if (r > 0) {                // row y - 1: its fc2 results are long retired
        slab_sync(a2, buf ^ 1);
        epilogue(y - 1, res_prev, buf ^ 1);
      }
      // dwconv 3x3 + bias + GELU of row y, straight into fc2's operand layout; the taps of the next
      // (n-tile, tap row) are read from LDS while the current one computes
      f16x8 g[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 db = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(tpl + j * 4 * K::TBLK / 16) + 36);
        float acc[4] = {db.x, db.y, db.z, db.w};
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const int jd = 3 * j + dy;
          if (jd + 1 < 12) tload(jd + 1, tq[(jd + 1) & 1]);
          taps3(acc, win[(ROT + dy) % 3][j], tq[jd & 1]);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) g[j >> 1][4 * (j & 1) + c] = (_Float16)gelu_rw(acc[c]);
      }
      // fc2 partial sums of this wave's 64 hidden channels (lane: channels 16 c + 4 fq + r, token fr)
#pragma unroll
      for (int c = 0; c < NC2; ++c) {
        a2[c] = mfma16x16x32(w2f[0][c], g[0], f32x4{0.f, 0.f, 0.f, 0.f});
        a2[c] = mfma16x16x32(w2f[1][c], g[1], a2[c]);
      }
      fc1_pack(y + 2, a1, win[ROT]);   // the new row y + 2 (its fc1 MFMAs have long retired)
      res_prev = res;
      buf ^= 1;
    };
    for (int r = 0; r + 3 <= R; r += 3) {
      row(r, std::integral_constant<int, 0>{});
      row(r + 1, std::integral_constant<int, 1>{});
      row(r + 2, std::integral_constant<int, 2>{});
    }
    if constexpr (R % 3 >= 1) row(R - R % 3, std::integral_constant<int, 0>{});
    if constexpr (R % 3 == 2) row(R - 1, std::integral_constant<int, 1>{});
    slab_sync(a2, buf ^ 1);
    epilogue(y0 + R - 1, res_prev, buf ^ 1);
  }
}

// ---- second form of the whole stage-1 MixFFN: the depthwise taps as f16-pair dot products.
// The hidden window is kept as f16 PAIRS of vertically adjacent rows, P_y[c] = (h[y][c], h[y+1][c]) in one
// VGPR per channel, so output row y is, per channel and horizontal offset dx,
//   dot2(P_{y-1}, (t[0][dx], t[1][dx])) + dot2(P_y, (0, t[2][dx]))
// — six v_dot2c_f32_f16 (horizontal shift through the DPP source, as taps3) instead of nine v_fmac_f32, a
// 2-row window of 32 VGPRs instead of 48 f32, and 96 tap dwords per row from LDS instead of 144.  The new
// row's pair P_{y+1} = (hi(P_y), f16(fc1)) replaces P_{y-1} once its n-tile's dwconv has read it.  The
// products of the f16 hidden values and f16 taps are exact in f32 (the conv of the reference's autocast
// in f16 with f32 accumulation); only the summation order differs from the f32-FMA form.
template <int C_, int W_, int R_, int OCC_, bool PKG_ = true>
struct DCfg {
  static constexpr int C = C_, W = W_, R = R_, OCC = OCC_;
  static constexpr bool PKG = PKG_;                  // GELU on packed f32 pairs (svk_common.h gelu_pk<3>, round 6)
  static constexpr int HID = 4 * C, NW = HID / 64, NT = 64 * NW;
  static constexpr int KS = C / 32, NC2 = C / 16, XT = (W + 13) / 14;
  static constexpr int TPW = 16 / NW, LPT = 64 / TPW;
  static constexpr int SROW = C + 4, SLAB = 16 * SROW;
  static constexpr int TBLK = 112;                  // tap block (wave, n-tile, fq): [4 ch][6] f16 pairs, dwb [4] f32
  static constexpr int LDS_TP = HID * 4;             // b1 (f32) | tap blocks | b2, gamma, beta | slabs
  static constexpr int LDS_EP = LDS_TP + NW * 16 * TBLK;
  static constexpr int LDS_T = LDS_EP + 3 * C * 4;
  static constexpr int LDS = LDS_T + 2 * NW * SLAB * 4;
  static_assert(C % 32 == 0 && NW >= 1 && NW <= 4 && LPT * 4 == C && R % 2 == 0, "shape");
};

// acc0/1 (channels c0, c1) += the 3x3 taps: p = P_{y-1}, q = P_y pairs; t = [c0: T01 dx0..2, T2 dx0..2,
// c1: the same], T01 = (t[0][dx], t[1][dx]), T2 = (0, t[2][dx]).  The four centre products go first: they
// give the DPP reads the two wait states a VALU write of p / q needs.
__device__ __forceinline__ void taps_d2(float& a0, float& a1, uint32_t p0, uint32_t p1, uint32_t q0, uint32_t q1,
                                        const uint32_t (&t)[12]) {
  asm("v_dot2c_f32_f16 %0, %2, %7\n\t"
      "v_dot2c_f32_f16 %1, %3, %13\n\t"
      "v_dot2c_f32_f16 %0, %4, %10\n\t"
      "v_dot2c_f32_f16 %1, %5, %16\n\t"
      "v_dot2c_f32_f16_dpp %0, %2, %6 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %1, %3, %12 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %0, %4, %9 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %1, %5, %15 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %0, %2, %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %1, %3, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %0, %4, %11 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_dot2c_f32_f16_dpp %1, %5, %17 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(a0), "+v"(a1)
      : "v"(p0), "v"(p1), "v"(q0), "v"(q1), "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3]), "v"(t[4]), "v"(t[5]),
        "v"(t[6]), "v"(t[7]), "v"(t[8]), "v"(t[9]), "v"(t[10]), "v"(t[11]));
}

__device__ __forceinline__ uint32_t hpair(uint32_t lo_from_hi, float v) {   // (hi half of lo_from_hi, f16(v))
  return __builtin_bit_cast(uint32_t, h2{__builtin_bit_cast(h2, lo_from_hi).y, (f16)v});
}

template <class K>
__global__ __launch_bounds__(K::NT, K::OCC) void mixffn_rwd(const f16* __restrict__ XN, const f16* __restrict__ X,
                                                       const f16* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ taps, const float* __restrict__ dwb,
                                                       const f16* __restrict__ W2, const float* __restrict__ b2,
                                                       f16* __restrict__ Y, f16* __restrict__ Yn,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, int H, int nstrip, int total) {
  constexpr int C = K::C, W = K::W, R = K::R, HID = K::HID, KS = K::KS, NC2 = K::NC2, NW = K::NW;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  char* const smem = reinterpret_cast<char*>(smem4);
  float* const slab0 = reinterpret_cast<float*>(smem + K::LDS_T);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- prologue (as mixffn_rw; the tap blocks hold f16 pairs): block blk = (w * 4 + j) * 4 + fq holds
  // channels 4 blk + i: dwords 6 i + s, s < 3: (t[0][s], t[1][s]), s >= 3: (0, t[2][s - 3]); then dwb [4] f32
  for (int e = tid; e < HID; e += K::NT) reinterpret_cast<float*>(smem)[e] = b1[e];
  for (int e = tid; e < NW * 16 * 28; e += K::NT) {
    const int blk = e / 28, r = e % 28;
    uint32_t v;
    if (r < 24) {
      const int i = r / 6, s = r % 6, dx = s % 3, ch = 4 * blk + i;
      const f16 lo = s < 3 ? (f16)taps[dx * HID + ch] : (f16)0.f;
      const f16 hi = s < 3 ? (f16)taps[(3 + dx) * HID + ch] : (f16)taps[(6 + dx) * HID + ch];
      v = __builtin_bit_cast(uint32_t, h2{lo, hi});
    } else {
      v = __float_as_uint(dwb[4 * blk + r - 24]);
    }
    reinterpret_cast<uint32_t*>(smem + K::LDS_TP + blk * K::TBLK)[r] = v;
  }
  f16x8 w1f[4][KS], w2f[2][NC2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      w1f[j][ks] = *reinterpret_cast<const f16x8*>(W1 + (long)(64 * w + 16 * j + fr) * C + 32 * ks + 8 * fq);
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int c = 0; c < NC2; ++c) {
      const f16* src = W2 + (long)(16 * c + fr) * HID + 64 * w + 32 * q + 4 * fq;
      const f16x4 lo = *reinterpret_cast<const f16x4*>(src), hi = *reinterpret_cast<const f16x4*>(src + 16);
      w2f[q][c] = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  float* const sEp = reinterpret_cast<float*>(smem + K::LDS_EP);
  for (int e = tid; e < 3 * C; e += K::NT)
    sEp[e] = e < C ? b2[e] : (gamma ? (e < 2 * C ? gamma[e - C] : beta[e - 2 * C]) : (e < 2 * C ? 1.f : 0.f));
  const int et = K::TPW * w + lane / K::LPT, ec = lane % K::LPT;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  const float* b1l = reinterpret_cast<const float*>(smem) + 64 * w + 4 * fq;
  const char* tpb = smem + K::LDS_TP + (w * 16 + fq) * K::TBLK;   // + j * 4 * TBLK
  const int G = gridDim.x;
  int buf = 0;
  for (int u = xcd_remap(blockIdx.x, G); u < total; u += G) {
    const int xt = u % K::XT, rest = u / K::XT, sidx = rest % nstrip, b = rest / nstrip;
    const int y0 = sidx * R, x0 = 14 * xt;
    const int tx = x0 - 1 + fr;
    const bool xok = tx >= 0 && tx < W;
    const f16* XNb = XN + (long)b * H * W * C + (long)min(max(tx, 0), W - 1) * C + 8 * fq;
    auto load_x = [&](int yy, f16x8 (&xf)[KS]) __attribute__((always_inline)) {
      const f16* src = XNb + (long)min(max(yy, 0), H - 1) * W * C;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xf[ks] = *reinterpret_cast<const f16x8*>(src + 32 * ks);
    };
    auto fc1_mma = [&](const f16x8 (&xf)[KS], f32x4 (&a)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = *reinterpret_cast<const f32x4*>(b1l + 16 * j);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a[j] = mfma16x16x32(w1f[j][ks], xf[ks], a[j]);
      }
    };
    const bool edge = x0 == 0 || x0 + 15 > W;
    // hidden row yy of n-tile j as f32 values zeroed outside the image: a wave-uniform branch (the empty
    // volatile asm keeps hipcc from if-converting it into two selects per value on every row), one select
    // per value on the edge tiles and the rows beyond the map
    auto fc1_val = [&](int yy, const f32x4& a, float (&hv)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int c = 0; c < 4; ++c) hv[c] = a[c];
      if (edge || yy < 0 || yy >= H) {
        asm volatile("");
        const bool ok = xok && yy >= 0 && yy < H;
#pragma unroll
        for (int c = 0; c < 4; ++c) hv[c] = ok ? hv[c] : 0.f;
      }
    };
    uint32_t P[2][4][4];          // the two pair rows; at row r: P_{y-1} in slot r % 2, P_y in slot (r + 1) % 2
    {
      f16x8 xa[KS], xb[KS], xc[KS];
      f32x4 a[4];
      load_x(y0 - 1, xa);
      load_x(y0, xb);
      load_x(y0 + 1, xc);
      fc1_mma(xa, a);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float hv[4];
        fc1_val(y0 - 1, a[j], hv);
#pragma unroll
        for (int c = 0; c < 4; ++c) P[1][j][c] = hpair(0u, hv[c]);          // (0, h[y0-1])
      }
      fc1_mma(xb, a);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float hv[4];
        fc1_val(y0, a[j], hv);
#pragma unroll
        for (int c = 0; c < 4; ++c) P[0][j][c] = hpair(P[1][j][c], hv[c]);   // (h[y0-1], h[y0])
      }
      fc1_mma(xc, a);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float hv[4];
        fc1_val(y0 + 1, a[j], hv);
#pragma unroll
        for (int c = 0; c < 4; ++c) P[1][j][c] = hpair(P[0][j][c], hv[c]);   // (h[y0], h[y0+1])
      }
    }
    f16x8 xn[KS];
    load_x(y0 + 2, xn);
    const int etx = x0 - 1 + et;
    const bool eok = et >= 1 && et <= 14 && etx < W;
    const long eoff0 = ((long)b * H * W + min(max(etx, 0), W - 1)) * C + 4 * ec;
    auto epilogue = [&](int yy, uint2 res, int bb) __attribute__((always_inline)) {
      float4 v = *reinterpret_cast<const float4*>(slab0 + bb * NW * K::SLAB + et * K::SROW + 4 * ec);
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
        const float4 o = *reinterpret_cast<const float4*>(slab0 + (bb * NW + ww) * K::SLAB + et * K::SROW + 4 * ec);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      const f32x2 r01 = unpack2<f16>(res.x), r23 = unpack2<f16>(res.y);
      const float4 eb2 = *reinterpret_cast<const float4*>(sEp + 4 * ec);
      const f16 o0 = (f16)(v.x + eb2.x + r01.x), o1 = (f16)(v.y + eb2.y + r01.y);
      const f16 o2 = (f16)(v.z + eb2.z + r23.x), o3 = (f16)(v.w + eb2.w + r23.y);
      const bool st = eok && yy < H;
      const long oo = eoff0 + (long)yy * W * C;
      if (Y && st) *reinterpret_cast<f16x4*>(Y + oo) = f16x4{o0, o1, o2, o3};
      if (gamma) {
        const float f0 = o0, f1 = o1, f2 = o2, f3 = o3;
        float sm = f0 + f1 + f2 + f3;
#pragma unroll
        for (int m = K::LPT / 2; m >= 1; m >>= 1) sm += __shfl_xor(sm, m, 64);
        const float mean = sm * (1.0f / C);
        const float d0 = f0 - mean, d1 = f1 - mean, d2 = f2 - mean, d3 = f3 - mean;
        float q = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
#pragma unroll
        for (int m = K::LPT / 2; m >= 1; m >>= 1) q += __shfl_xor(q, m, 64);
        const float rstd = 1.0f / sqrtf(q * (1.0f / C) + eps);
        const float4 egam = *reinterpret_cast<const float4*>(sEp + C + 4 * ec);
        const float4 ebet = *reinterpret_cast<const float4*>(sEp + 2 * C + 4 * ec);
        if (st)
          *reinterpret_cast<f16x4*>(Yn + oo) = f16x4{(f16)(d0 * rstd * egam.x + ebet.x), (f16)(d1 * rstd * egam.y + ebet.y),
                                                     (f16)(d2 * rstd * egam.z + ebet.z), (f16)(d3 * rstd * egam.w + ebet.w)};
      }
    };
    // taps of n-tile j, channel half hf (channels 2 hf, 2 hf + 1): 12 dwords
    auto tload = [&](int jh, uint32_t (&t)[12]) __attribute__((always_inline)) {
      const uint4* src = reinterpret_cast<const uint4*>(tpb + (jh >> 1) * 4 * K::TBLK + (jh & 1) * 48);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const uint4 v = src[i];
        t[4 * i] = v.x; t[4 * i + 1] = v.y; t[4 * i + 2] = v.z; t[4 * i + 3] = v.w;
      }
    };
    uint2 res_prev = {0u, 0u};
    f32x4 a2[NC2];
    // one row (software-pipelined as mixffn_rw): the fc1 MFMAs of hidden row y + 2 and the X row of y + 3;
    // the previous row's fc2 sums to the slab (their MFMAs retired a whole dwconv ago) and its epilogue
    // behind the barrier that publishes them; then per n-tile the taps, the new pair row, GELU and (every
    // second n-tile) a k-step of fc2
    auto row = [&](int r, auto ROT_) __attribute__((always_inline)) {
      constexpr int S0 = decltype(ROT_)::value, S1 = S0 ^ 1;   // P_{y-1} in slot S0, P_y in S1
      const int y = y0 + r;
      const uint2 res = *reinterpret_cast<const uint2*>(X + eoff0 + (long)min(y, H - 1) * W * C);
      f32x4 a1[4];
      fc1_mma(xn, a1);
      load_x(y + 3, xn);
      __builtin_amdgcn_sched_barrier(0);
      uint32_t tq[2][12];
      tload(0, tq[0]);
      if (r > 0) {
        float* sl = slab0 + ((buf ^ 1) * NW + w) * K::SLAB;
#pragma unroll
        for (int c = 0; c < NC2; ++c) *reinterpret_cast<f32x4*>(sl + fr * K::SROW + 16 * c + 4 * fq) = a2[c];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        epilogue(y - 1, res_prev, buf ^ 1);
      }
      f16x8 g[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 db = *reinterpret_cast<const float4*>(tpb + j * 4 * K::TBLK + 96);
        float acc[4] = {db.x, db.y, db.z, db.w};
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int jh = 2 * j + hf;
          if (jh + 1 < 8) tload(jh + 1, tq[(jh + 1) & 1]);
          taps_d2(acc[2 * hf], acc[2 * hf + 1], P[S0][j][2 * hf], P[S0][j][2 * hf + 1], P[S1][j][2 * hf],
                  P[S1][j][2 * hf + 1], tq[jh & 1]);
        }
        // n-tile j of the new pair row P_{y+1} = (h[y+1], h[y+2]) into the slot of P_{y-1}, which this
        // n-tile's taps have just read
        {
          float hv[4];
          fc1_val(y + 2, a1[j], hv);
#pragma unroll
          for (int c = 0; c < 4; ++c) P[S0][j][c] = hpair(P[S1][j][c], hv[c]);
        }
        if constexpr (K::PKG) {
          const f32x2 g01 = gelu_pk<3>(f32x2{acc[0], acc[1]}), g23 = gelu_pk<3>(f32x2{acc[2], acc[3]});
          g[j >> 1][4 * (j & 1) + 0] = (_Float16)g01.x;
          g[j >> 1][4 * (j & 1) + 1] = (_Float16)g01.y;
          g[j >> 1][4 * (j & 1) + 2] = (_Float16)g23.x;
          g[j >> 1][4 * (j & 1) + 3] = (_Float16)g23.y;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) g[j >> 1][4 * (j & 1) + c] = (_Float16)gelu_rw(acc[c]);
        }
        if (j & 1) {   // a complete 32-channel k-step of fc2
#pragma unroll
          for (int c = 0; c < NC2; ++c)
            a2[c] = mfma16x16x32(w2f[j >> 1][c], g[j >> 1], j == 1 ? f32x4{0.f, 0.f, 0.f, 0.f} : a2[c]);
        }
      }
      res_prev = res;
      buf ^= 1;
    };
    for (int r = 0; r < R; r += 2) {
      row(r, std::integral_constant<int, 0>{});
      row(r + 1, std::integral_constant<int, 1>{});
    }
    {
      float* sl = slab0 + ((buf ^ 1) * NW + w) * K::SLAB;
#pragma unroll
      for (int c = 0; c < NC2; ++c) *reinterpret_cast<f32x4*>(sl + fr * K::SROW + 16 * c + 4 * fq) = a2[c];
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    epilogue(y0 + R - 1, res_prev, buf ^ 1);
  }
}

// ---- MixFFN front half in the same register-window form: G = GELU(dwconv3x3(fc1(XN))) written to HBM
// (stage 2, C = 128, hidden 512: the whole-MixFFN form would need 128 weight VGPRs per wave).  A wave owns
// 64 hidden channels of a (frame, 14-column x-tile, R-row strip); a workgroup = 4 waves = 256 channels
// and keeps its W1 fragments in registers and its taps / b1 in LDS for the whole persistent kernel (it
// walks only units of its own hidden block).  No cross-wave reduction, no per-row barrier.  Per row and
// wave: 4 KS fc1 MFMAs (hidden row y + 2, X loaded a row ahead), the 3x3 taps as DPP-fused v_fmac (taps
// streamed from LDS one step ahead), GELU, 8-byte f16 stores of the 4 x 4 channels of the lane's token.
template <int C_, int W_, int R_, bool BI_ = true, bool PKG_ = true>
struct DwCfg {
  static constexpr int C = C_, W = W_, R = R_;
  static constexpr bool BIAS_INIT = BI_;
  static constexpr bool PKG = PKG_;                  // GELU on packed f32 pairs (gelu_pk<3>, round 6)
  static constexpr int KS = C / 32, XT = (W + 13) / 14, NT = 256;
  static constexpr int TBLK = 160;                  // tap block (wave, n-tile, fq): taps [9][4], dwb [4] (f32)
  static constexpr int LDS_TP = 256 * 4;            // b1 of the workgroup's 256 channels | tap blocks
  static constexpr int LDS = LDS_TP + 4 * 16 * TBLK;
};

template <class K>
__global__ __launch_bounds__(K::NT, 2) void fc1dw_rw(const f16* __restrict__ XN, const f16* __restrict__ W1,
                                                    const float* __restrict__ b1, const float* __restrict__ taps,
                                                    const float* __restrict__ dwb, f16* __restrict__ G, int H,
                                                    int hid, int nstrip, int nspatial) {
  constexpr int C = K::C, W = K::W, R = K::R, KS = K::KS;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  char* const smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int nhb = hid / 256, hb = blockIdx.x % nhb, ch0 = 256 * hb;   // this workgroup's hidden block
  for (int e = tid; e < 256; e += K::NT) reinterpret_cast<float*>(smem)[e] = b1[ch0 + e];
  for (int e = tid; e < 4 * 16 * 40; e += K::NT) {
    const int blk = e / 40, r = e % 40, t = r / 4, c = r % 4;   // channel ch0 + 4 blk + c
    reinterpret_cast<float*>(smem + K::LDS_TP + blk * K::TBLK)[r] =
        t < 9 ? (float)(f16)taps[t * hid + ch0 + 4 * blk + c] : dwb[ch0 + 4 * blk + c];
  }
  f16x8 w1f[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      w1f[j][ks] = *reinterpret_cast<const f16x8*>(W1 + (long)(ch0 + 64 * w + 16 * j + fr) * C + 32 * ks + 8 * fq);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const float* b1l = reinterpret_cast<const float*>(smem) + 64 * w + 4 * fq;
  const uint4* tpl = reinterpret_cast<const uint4*>(smem + K::LDS_TP + (w * 16 + fq) * K::TBLK);
  const int gs = gridDim.x / nhb;                       // workgroups per hidden block (host: grid % nhb == 0)
  for (int u = blockIdx.x / nhb; u < nspatial; u += gs) {
    const int xt = u % K::XT, rest = u / K::XT, sidx = rest % nstrip, b = rest / nstrip;
    const int y0 = sidx * R, x0 = 14 * xt;
    const int tx = x0 - 1 + fr;
    const bool xok = tx >= 0 && tx < W;
    const bool sok = fr >= 1 && fr <= 14 && tx < W;     // this lane's token is stored
    const f16* XNb = XN + (long)b * H * W * C + (long)min(max(tx, 0), W - 1) * C + 8 * fq;
    f16* Gb = G + ((long)b * H * W + min(max(tx, 0), W - 1)) * hid + ch0 + 64 * w + 4 * fq;
    auto load_x = [&](int yy, f16x8 (&xf)[KS]) __attribute__((always_inline)) {
      const f16* src = XNb + (long)min(max(yy, 0), H - 1) * W * C;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xf[ks] = *reinterpret_cast<const f16x8*>(src + 32 * ks);
    };
    auto fc1_mma = [&](const f16x8 (&xf)[KS], f32x4 (&a)[4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = K::BIAS_INIT ? *reinterpret_cast<const f32x4*>(b1l + 16 * j) : f32x4{0.f, 0.f, 0.f, 0.f};   // bias on the MFMA
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a[j] = mfma16x16x32(w1f[j][ks], xf[ks], a[j]);
      }
    };
    const bool edge = x0 == 0 || x0 + 15 > W;          // (see mixffn_rw)
    auto fc1_pack = [&](int yy, const f32x4 (&a)[4], float (&hw)[4][4]) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 bb = K::BIAS_INIT ? float4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const float4*>(b1l + 16 * j);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) hw[j][c] = (float)(f16)(K::BIAS_INIT ? a[j][c] : a[j][c] + bv[c]);
      }
      if (edge || yy < 0 || yy >= H) {
        const uint32_t m = (xok && yy >= 0 && yy < H) ? ~0u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 4; ++c) hw[j][c] = __uint_as_float(__float_as_uint(hw[j][c]) & m);
      }
    };
    auto tload = [&](int jd, float (&t)[12]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const uint4 v = tpl[(jd / 3) * 4 * K::TBLK / 16 + (jd % 3) * 3 + i];
        t[4 * i] = __uint_as_float(v.x); t[4 * i + 1] = __uint_as_float(v.y);
        t[4 * i + 2] = __uint_as_float(v.z); t[4 * i + 3] = __uint_as_float(v.w);
      }
    };
    float win[3][4][4];
    {
      f16x8 xa[KS], xb[KS], xc[KS];
      f32x4 a[4];
      load_x(y0 - 1, xa);
      load_x(y0, xb);
      load_x(y0 + 1, xc);
      fc1_mma(xa, a);
      fc1_pack(y0 - 1, a, win[0]);
      fc1_mma(xb, a);
      fc1_pack(y0, a, win[1]);
      fc1_mma(xc, a);
      fc1_pack(y0 + 1, a, win[2]);
    }
    f16x8 xn[KS];
    load_x(y0 + 2, xn);
    // (the window rotates through its slots as in mixffn_rw)
    auto row = [&](int r, auto ROT_) __attribute__((always_inline)) {
      constexpr int ROT = decltype(ROT_)::value;
      const int y = y0 + r;
      f32x4 a1[4];
      fc1_mma(xn, a1);
      load_x(y + 3, xn);
      __builtin_amdgcn_sched_barrier(0);
      float tq[2][12];
      tload(0, tq[0]);
      f16* gy = Gb + (long)min(y, H - 1) * W * hid;
      const bool st = sok && y < H;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 db = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(tpl + j * 4 * K::TBLK / 16) + 36);
        float acc[4] = {db.x, db.y, db.z, db.w};
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const int jd = 3 * j + dy;
          if (jd + 1 < 12) tload(jd + 1, tq[(jd + 1) & 1]);
          taps3(acc, win[(ROT + dy) % 3][j], tq[jd & 1]);
        }
        if constexpr (K::PKG) {
          const f32x2 g01 = gelu_pk<3>(f32x2{acc[0], acc[1]}), g23 = gelu_pk<3>(f32x2{acc[2], acc[3]});
          if (st) *reinterpret_cast<f16x4*>(gy + 16 * j) = f16x4{(f16)g01.x, (f16)g01.y, (f16)g23.x, (f16)g23.y};
        } else {
          if (st)
            *reinterpret_cast<f16x4*>(gy + 16 * j) =
                f16x4{(f16)gelu_rw(acc[0]), (f16)gelu_rw(acc[1]), (f16)gelu_rw(acc[2]), (f16)gelu_rw(acc[3])};
        }
      }
      fc1_pack(y + 2, a1, win[ROT]);
    };
    for (int r = 0; r + 3 <= R; r += 3) {
      row(r, std::integral_constant<int, 0>{});
      row(r + 1, std::integral_constant<int, 1>{});
      row(r + 2, std::integral_constant<int, 2>{});
    }
    if constexpr (R % 3 >= 1) row(R - R % 3, std::integral_constant<int, 0>{});
    if constexpr (R % 3 == 2) row(R - 1, std::integral_constant<int, 1>{});
  }
}

template <class K, bool D2 = false>
static int launch(const void* XN, const void* X, const void* W1, const float* b1, const float* taps, const float* dwb,
                  const void* W2, const float* b2, void* Y, void* Yn, const float* gamma, const float* beta, float eps,
                  int B, int H, hipStream_t st) {
  const int nstrip = (H + K::R - 1) / K::R;
  const long total = (long)B * nstrip * K::XT;
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* fn;
    if constexpr (D2) fn = reinterpret_cast<const void*>(&mixffn_rwd<K>);
    else fn = reinterpret_cast<const void*>(&mixffn_rw<K>);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, K::NT, K::LDS);
    slots = std::max(1, cus) * std::max(1, per);
    if (getenv("SVK_RW_VERBOSE")) fprintf(stderr, "mixffn_rw: %d CUs x %d workgroups, LDS %d B\n", cus, per, K::LDS);
  }
  if (total > 0x7fffffffL) { set_error("svk_mixffn_rw: too many strips"); return SVK_EINVAL; }
  static const int force = getenv("SVK_RW_GRID") ? atoi(getenv("SVK_RW_GRID")) : 0;   // debugging: grid size
  const int grid = (int)std::min<long>(total, force > 0 ? force : slots);
  if constexpr (D2)
    hipLaunchKernelGGL((mixffn_rwd<K>), dim3(grid), dim3(K::NT), K::LDS, st, (const f16*)XN, (const f16*)X, (const f16*)W1,
                       b1, taps, dwb, (const f16*)W2, b2, (f16*)Y, (f16*)Yn, gamma, beta, eps, H, nstrip, (int)total);
  else
    hipLaunchKernelGGL((mixffn_rw<K>), dim3(grid), dim3(K::NT), K::LDS, st, (const f16*)XN, (const f16*)X, (const f16*)W1,
                       b1, taps, dwb, (const f16*)W2, b2, (f16*)Y, (f16*)Yn, gamma, beta, eps, H, nstrip, (int)total);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "%s<Cfg<%d, %d, %d>>", D2 ? "mixffn_rwd" : "mixffn_rw", K::C, K::W, K::R);
  set_last_kernel(name);
  return check_launch("mixffn_rw");
}

}  // namespace ffnrw

// svk_mixffn_fc1_dwconv's f16 GELU path for the instantiated shapes; 1 = not eligible
template <class K>
static int fc1dw_rw_launch(int dtype, const void* XN, const void* W1, const float* b1, const float* taps,
                           const float* dbias, void* G, int B, int H, int W, int C, int hidden, int act, hipStream_t st);

int fc1dw_rw_try(int dtype, const void* XN, const void* W1, const float* b1, const float* taps, const float* dbias,
                 void* G, int B, int H, int W, int C, int hidden, int act, hipStream_t st) {
  static const int var = getenv("SVK_RW_VAR") ? atoi(getenv("SVK_RW_VAR")) : 0;   // 2: bias added after the MFMAs
  if (var == 2)
    return fc1dw_rw_launch<ffnrw::DwCfg<128, 28, 28, false>>(dtype, XN, W1, b1, taps, dbias, G, B, H, W, C, hidden, act, st);
  if (var == 4 || !gelu_pk_on())   // element-wise GELU (SVK_GELU_PK=0)
    return fc1dw_rw_launch<ffnrw::DwCfg<128, 28, 28, true, false>>(dtype, XN, W1, b1, taps, dbias, G, B, H, W, C, hidden, act, st);
  return fc1dw_rw_launch<ffnrw::DwCfg<128, 28, 28>>(dtype, XN, W1, b1, taps, dbias, G, B, H, W, C, hidden, act, st);
}

template <class K>
static int fc1dw_rw_launch(int dtype, const void* XN, const void* W1, const float* b1, const float* taps,
                           const float* dbias, void* G, int B, int H, int W, int C, int hidden, int act, hipStream_t st) {
  if (dtype != SVK_F16 || act != SVK_ACT_GELU || W != K::W || C != K::C || hidden % 256 || B <= 0 ||
      ((((uintptr_t)b1) | ((uintptr_t)dbias) | ((uintptr_t)taps)) & 15) || getenv("SVK_NO_FC1DW_RW"))
    return 1;
  const int nstrip = (H + K::R - 1) / K::R, nhb = hidden / 256;
  const long nspatial = (long)B * nstrip * K::XT;
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&ffnrw::fc1dw_rw<K>), K::NT,
                                                       K::LDS);
    slots = std::max(1, cus) * std::max(1, per);
  }
  if (nspatial * nhb > 0x7fffffffL) return 1;
  const int grid = (int)std::min<long>(nspatial, std::max(1, slots / nhb)) * nhb;
  hipLaunchKernelGGL((ffnrw::fc1dw_rw<K>), dim3(grid), dim3(K::NT), K::LDS, st, (const f16*)XN, (const f16*)W1, b1, taps,
                     dbias, (f16*)G, H, hidden, nstrip, (int)nspatial);
  set_last_kernel("fc1dw_rw<DwCfg<128, 28, 28>>");
  return check_launch("fc1dw_rw");
}
}  // namespace svk

using namespace svk;

extern "C" int svk_mixffn_rw_supported(int dtype, int W, int C) {
  return dtype == SVK_F16 && W == 56 && C == 64;
}

extern "C" int svk_mixffn_rw(int dtype, const void* XN, const void* X, const void* W1, const float* b1, const float* taps,
                             const float* dbias, const void* W2, const float* b2, void* Y, void* Yn, const float* gamma,
                             const float* beta, float eps, int B, int H, int W, int C, void* stream) {
  if (B < 0 || H <= 0 || !XN || !X || !W1 || !b1 || !taps || !dbias || !W2 || !b2 || (!Y && !gamma) ||
      (gamma && (!beta || !Yn))) {
    set_error("svk_mixffn_rw: bad args"); return SVK_EINVAL;
  }
  if ((((uintptr_t)XN) | ((uintptr_t)X) | ((uintptr_t)W1) | ((uintptr_t)W2) | ((uintptr_t)Y) | ((uintptr_t)Yn) |
       ((uintptr_t)b1) | ((uintptr_t)b2) | ((uintptr_t)gamma) | ((uintptr_t)beta)) & 15) {
    set_error("svk_mixffn_rw: pointers must be 16-byte aligned"); return SVK_EINVAL;
  }
  if (!svk_mixffn_rw_supported(dtype, W, C)) {
    set_error("svk_mixffn_rw: (dtype=%d, W=%d, C=%d) not instantiated", dtype, W, C); return SVK_EUNSUPPORTED;
  }
  if (B == 0) return SVK_OK;
  static const int var = getenv("SVK_RW_VAR") ? atoi(getenv("SVK_RW_VAR")) : 0;   // tuning variants
  hipStream_t st = (hipStream_t)stream;
  // strips of 28 rows (two per 56-row frame): measured 335 us vs 341 (14 rows), 342 (8 rows) at B = 256
  if (var == 1) return ffnrw::launch<ffnrw::Cfg<64, 56, 14, 2>>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
  if (var == 2) return ffnrw::launch<ffnrw::Cfg<64, 56, 28, 2, false>>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
  // 3: the f32-FMA tap form (mixffn_rw); default: the f16-pair dot-product taps (mixffn_rwd), 310 vs 319 us
  // (profiles/r05/mixffn_rwd.txt; its 3-waves-per-SIMD build spills and ran 440 us)
  if (var == 3) return ffnrw::launch<ffnrw::Cfg<64, 56, 28, 2>>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
  if (var == 4 || !gelu_pk_on())   // element-wise GELU (SVK_GELU_PK=0)
    return ffnrw::launch<ffnrw::DCfg<64, 56, 28, 2, false>, true>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
  if (var == 5)   // whole-frame strips: 2 halo rows of fc1 per 56 rows instead of per 28
    return ffnrw::launch<ffnrw::DCfg<64, 56, 56, 2>, true>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
  return ffnrw::launch<ffnrw::DCfg<64, 56, 28, 2>, true>(XN, X, W1, b1, taps, dbias, W2, b2, Y, Yn, gamma, beta, eps, B, H, st);
}
