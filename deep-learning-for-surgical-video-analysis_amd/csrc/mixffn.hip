// Fused MixFFN for bf16 (mix_transformer_evp.py:32-67 + DWConv :19-30 + the Block residual :169):
//
//   Y = X + fc2( GELU( dwconv3x3( fc1(XN) ) ) )         XN = LN2(X), all maps NHWC [B, H, W, C]
//
// The unfused path writes and re-reads the 4C-wide hidden map three times (fc1 out, dwconv in/out,
// fc2 in): 1.6 GB per stage-1 block at B = 256.  Here a workgroup owns a TH x TW tile of output
// tokens of one frame and keeps the hidden on chip: it stages XN for the tile plus a 1-token halo
// in LDS once, then for each 64-channel hidden chunk
//   (1) fc1 over the (TH+2)(TW+2) halo tokens      -> sH   (MFMA 16x16x32, out-of-image rows = 0,
//                                                          which is the dwconv's zero padding)
//   (2) depthwise 3x3 + bias + GELU over the tile    -> sG   (VALU, 16-byte LDS reads)
//   (3) fc2 partial sums, accumulated in registers across chunks (MFMA)
// and finally adds b2 + the residual and writes Y through an LDS-staged 16-byte epilogue.
// HBM traffic per block: read XN (+halo re-reads from L2), read X, write Y.
//
// Weights: the fc1 B fragments are read straight from global memory (L2-resident, shared by every
// workgroup); the fc2 weight chunk is staged in LDS with a one-chunk register prefetch.
#include "svk_common.h"

namespace svk {

namespace ffn {

constexpr int HC = 64;      // hidden channels per chunk
constexpr int HLD = HC + 8; // sH / sG / sW2 row stride (elements): 144 B rows, conflict-free b128 reads

template <int C, int TH, int TW>
struct Cfg {
  static constexpr int HW_ = TW + 2, HH = TH + 2;
  static constexpr int NH = HH * HW_;               // halo tokens
  static constexpr int MTH = (NH + 15) / 16;        // fc1 M-tiles
  static constexpr int NO = TH * TW;                // output tokens
  static constexpr int MTO = (NO + 15) / 16;        // fc2 M-tiles
  static constexpr int XLD = C + 8;                 // sXN row stride
  static constexpr int KS1 = C / 32;                // fc1 k-steps
  static constexpr int NT2 = C / 16;                // fc2 n-tiles
  static constexpr int HID = 4 * C;
  static constexpr int NCH = HID / HC;
  static constexpr int I1 = (MTH + 3) / 4;          // fc1 M-tiles per wave (max)
  static constexpr int I2 = (MTO + 3) / 4;          // fc2 M-tiles per wave (max)
  static constexpr int SX = MTH * 16 * XLD * 2;     // bytes
  static constexpr int SH = MTH * 16 * HLD * 2;
  static constexpr int SG = MTO * 16 * HLD * 2;
  static constexpr int SW2 = C * HLD * 2;
  static constexpr int STP = 10 * HC * 4;           // taps [9][64] + dwconv bias [64], f32
  static constexpr int SOUT = NO * (C + 4) * 4;     // f32 epilogue tile (aliases sXN.. region)
  static constexpr int MAIN = SX + SH + SG + SW2 + STP;
  static constexpr int BYTES = MAIN > SOUT ? MAIN : SOUT;
  static constexpr int W2CH = C * HC / 8;           // 16-byte chunks of one W2 chunk
  static constexpr int W2PT = (W2CH + 255) / 256;   // per thread
};

template <int C, int TH, int TW>
__global__ __launch_bounds__(256) void mixffn_bf16(const bf16* __restrict__ XN, const bf16* __restrict__ X,
                                                   const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                   const float* __restrict__ taps, const float* __restrict__ db,
                                                   const bf16* __restrict__ W2, const float* __restrict__ b2,
                                                   bf16* __restrict__ Y, int H, int W, int tiles_x, int tiles_y) {
  using K = Cfg<C, TH, TW>;
  __shared__ __attribute__((aligned(16))) char smem[K::BYTES];
  bf16 (*sX)[K::XLD] = reinterpret_cast<bf16 (*)[K::XLD]>(smem);
  bf16 (*sH)[HLD] = reinterpret_cast<bf16 (*)[HLD]>(smem + K::SX);
  bf16 (*sG)[HLD] = reinterpret_cast<bf16 (*)[HLD]>(smem + K::SX + K::SH);
  bf16 (*sW2)[HLD] = reinterpret_cast<bf16 (*)[HLD]>(smem + K::SX + K::SH + K::SG);
  float (*sT)[HC] = reinterpret_cast<float (*)[HC]>(smem + K::SX + K::SH + K::SG + K::SW2);   // [10][64]
  float (*sO)[C + 4] = reinterpret_cast<float (*)[C + 4]>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;
  const long img = (long)b * H * W;

  // ---- stage XN halo tile: halo token r -> (hy, hx) = (r / HW_, r % HW_), image (y0-1+hy, x0-1+hx)
  {
    // all loads issued before any store (a load -> select -> store loop would serialise one HBM
    // round trip per iteration)
    constexpr int CPR = C / 8;
    constexpr int NIT = (K::MTH * 16 * CPR + 255) / 256;
    uint4 v[NIT];
    bool okv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = min(tid + 256 * it, K::MTH * 16 * CPR - 1);
      const int r = e / CPR, c8 = (e % CPR) * 8;
      const int hy = r / K::HW_, hx = r - hy * K::HW_;
      const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
      okv[it] = r < K::NH && iy >= 0 && iy < H && ix >= 0 && ix < W;
      const int iyc = min(max(iy, 0), H - 1), ixc = min(max(ix, 0), W - 1);
      v[it] = *reinterpret_cast<const uint4*>(XN + (img + (long)iyc * W + ixc) * C + c8);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = tid + 256 * it;
      if (e < K::MTH * 16 * CPR) {
        const int r = e / CPR, c8 = (e % CPR) * 8;
        *reinterpret_cast<uint4*>(&sX[r][c8]) = okv[it] ? v[it] : make_uint4(0, 0, 0, 0);
      }
    }
  }
  // W2 chunk loader (register prefetch): W2 [C][HID], chunk hc -> sW2[n][k] = W2[n][hc*64 + k]
  uint4 w2r[K::W2PT];
  float4 tpr;                                   // taps/bias chunk: 160 float4 -> threads 0..159
  auto w2_fetch = [&](int hc) {
#pragma unroll
    for (int i = 0; i < K::W2PT; ++i) {
      const int e = tid + 256 * i;
      const int ec = e < K::W2CH ? e : K::W2CH - 1;
      const int n = ec / (HC / 8), k8 = (ec % (HC / 8)) * 8;
      w2r[i] = *reinterpret_cast<const uint4*>(W2 + (long)n * K::HID + hc * HC + k8);
    }
    const int tt = min(tid, 159), row = tt / 16, c4 = (tt % 16) * 4;
    tpr = *reinterpret_cast<const float4*>((row < 9 ? taps + row * K::HID : db) + hc * HC + c4);
  };
  auto w2_stash = [&]() {
#pragma unroll
    for (int i = 0; i < K::W2PT; ++i) {
      const int e = tid + 256 * i;
      if (e < K::W2CH) {
        const int n = e / (HC / 8), k8 = (e % (HC / 8)) * 8;
        *reinterpret_cast<uint4*>(&sW2[n][k8]) = w2r[i];
      }
    }
    if (tid < 160) *reinterpret_cast<float4*>(&sT[tid / 16][(tid % 16) * 4]) = tpr;
  };
  w2_fetch(0);

  f32x4 acc2[K::I2][K::NT2];
#pragma unroll
  for (int i = 0; i < K::I2; ++i)
#pragma unroll
    for (int j = 0; j < K::NT2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fc1 A fragments (W1 rows of the chunk) and b1 of the chunk live in ONE register set that is
  // refilled for chunk hc+1 as soon as chunk hc's fc1 has consumed it, so the L2/HBM latency of the
  // refill hides under chunk hc's dwconv and fc2 phases (software pipeline, no extra registers).
  bf16x8 wa[K::KS1][4];
  float b1v[4][4];
  auto w1_fetch = [&](int hc) {
#pragma unroll
    for (int ks = 0; ks < K::KS1; ++ks)
#pragma unroll
      for (int jh = 0; jh < 4; ++jh)
        wa[ks][jh] = *reinterpret_cast<const bf16x8*>(W1 + (long)(hc * HC + 16 * jh + fr) * C + 32 * ks + fk);
#pragma unroll
    for (int jh = 0; jh < 4; ++jh)
      *reinterpret_cast<float4*>(&b1v[jh][0]) = *reinterpret_cast<const float4*>(b1 + hc * HC + 16 * jh + (lane >> 4) * 4);
  };
  w1_fetch(0);
  const int c8 = (tid & 7) * 8;      // each thread's dwconv work always covers channel group c8

  for (int hc = 0; hc < K::NCH; ++hc) {
    __syncthreads();                 // previous chunk's fc2 done with sG / sW2; sX staged (hc = 0)
    w2_stash();
    w2_fetch(hc + 1 < K::NCH ? hc + 1 : hc);

    // ---- (1) fc1 chunk over the halo tokens, computed transposed: H^T = W1c . XN^T, so a lane's
    // accumulator holds 4 consecutive hidden channels of one token -> one 8-byte LDS store.
    {
      f32x4 acc1[4][K::I1];
#pragma unroll
      for (int jh = 0; jh < 4; ++jh)
#pragma unroll
        for (int i = 0; i < K::I1; ++i) acc1[jh][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < K::KS1; ++ks) {
#pragma unroll
        for (int i = 0; i < K::I1; ++i) {
          const int t = wave + 4 * i;
          if (t < K::MTH) {
            const bf16x8 xb = *reinterpret_cast<const bf16x8*>(&sX[16 * t + fr][32 * ks + fk]);
#pragma unroll
            for (int jh = 0; jh < 4; ++jh)
              acc1[jh][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][jh], xb, acc1[jh][i], 0, 0, 0);
          }
        }
      }
      // + b1, zero the tokens outside the image (dwconv zero padding) -> sH (bf16, like the unfused path)
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int i = 0; i < K::I1; ++i) {
        const int t = wave + 4 * i;
        if (t >= K::MTH) continue;
        const int row = 16 * t + fr;                 // halo token
        const int hy = row / K::HW_, hx = row - hy * K::HW_;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool ok = row < K::NH && iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
        for (int jh = 0; jh < 4; ++jh) {
          bf16x4 hv;
#pragma unroll
          for (int r = 0; r < 4; ++r) hv[r] = (bf16)(ok ? acc1[jh][i][r] + b1v[jh][r] : 0.f);
          *reinterpret_cast<bf16x4*>(&sH[row][16 * jh + (lane >> 4) * 4]) = hv;
        }
      }
    }
    w1_fetch(hc + 1 < K::NCH ? hc + 1 : hc);   // refill: lands during dwconv + fc2
    __syncthreads();

    // ---- (2) depthwise 3x3 + bias + GELU: thread -> channel group c8, tokens o = tid/8 + 32 i
    {
#pragma unroll
      for (int i = 0; i < (K::MTO * 16 + 31) / 32; ++i) {
        const int o = (tid >> 3) + 32 * i;
        if (o >= K::MTO * 16) break;
        float v[8];
        *reinterpret_cast<float4*>(&v[0]) = *reinterpret_cast<const float4*>(&sT[9][c8]);
        *reinterpret_cast<float4*>(&v[4]) = *reinterpret_cast<const float4*>(&sT[9][c8 + 4]);
        if (o < K::NO) {
          const int oy = o / TW, ox = o - oy * TW;
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const bf16x8 h = *reinterpret_cast<const bf16x8*>(&sH[(oy + dy) * K::HW_ + ox + dx][c8]);
              float w[8];
              *reinterpret_cast<float4*>(&w[0]) = *reinterpret_cast<const float4*>(&sT[dy * 3 + dx][c8]);
              *reinterpret_cast<float4*>(&w[4]) = *reinterpret_cast<const float4*>(&sT[dy * 3 + dx][c8 + 4]);
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] += (float)h[q] * w[q];
            }
        }
        bf16x8 gv;
#pragma unroll
        for (int q = 0; q < 8; ++q) gv[q] = (bf16)gelu_fast(v[q]);
        *reinterpret_cast<bf16x8*>(&sG[o][c8]) = gv;
      }
    }
    __syncthreads();

    // ---- (3) fc2 partial: acc2 += G (tile x 64) . W2[:, chunk]^T
#pragma unroll
    for (int ks = 0; ks < HC / 32; ++ks) {
      bf16x8 bfr[K::NT2];
#pragma unroll
      for (int j = 0; j < K::NT2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(&sW2[16 * j + fr][32 * ks + fk]);
#pragma unroll
      for (int i = 0; i < K::I2; ++i) {
        const int t = wave + 4 * i;
        if (t < K::MTO) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sG[16 * t + fr][32 * ks + fk]);
#pragma unroll
          for (int j = 0; j < K::NT2; ++j) acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[j], acc2[i][j], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();

  // ---- epilogue: + b2 -> f32 tile in LDS -> + residual -> 16-byte stores
#pragma unroll
  for (int i = 0; i < K::I2; ++i) {
    const int t = wave + 4 * i;
    if (t >= K::MTO) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 16 * t + (lane >> 4) * 4 + r;
      if (o >= K::NO) continue;
#pragma unroll
      for (int j = 0; j < K::NT2; ++j) sO[o][16 * j + fr] = acc2[i][j][r] + b2[16 * j + fr];
    }
  }
  __syncthreads();
  constexpr int CPR = C / 8;
  constexpr int NIT = (K::NO * CPR + 255) / 256;
  bf16x8 xr[NIT];
  long offs[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {       // residual loads first, clamped in range
    const int e = min(tid + 256 * it, K::NO * CPR - 1);
    const int o = e / CPR, c8 = (e % CPR) * 8;
    const int oy = o / TW, ox = o - oy * TW;
    const int iy = min(y0 + oy, H - 1), ix = min(x0 + ox, W - 1);
    offs[it] = (img + (long)iy * W + ix) * C + c8;
    xr[it] = *reinterpret_cast<const bf16x8*>(X + offs[it]);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + 256 * it;
    if (e >= K::NO * CPR) continue;
    const int o = e / CPR, c8 = (e % CPR) * 8;
    const int oy = o / TW, ox = o - oy * TW;
    if (y0 + oy >= H || x0 + ox >= W) continue;
    bf16x8 out;
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = (bf16)(sO[o][c8 + q] + (float)xr[it][q]);
    *reinterpret_cast<bf16x8*>(Y + offs[it]) = out;
  }
}

template <int C, int TH, int TW>
static int launch(const void* XN, const void* X, const void* W1, const float* b1, const float* taps, const float* db,
                  const void* W2, const float* b2, void* Y, int B, int H, int W, hipStream_t st) {
  const int tx = (W + TW - 1) / TW, ty = (H + TH - 1) / TH;
  const long nwg = (long)B * tx * ty;
  hipLaunchKernelGGL((mixffn_bf16<C, TH, TW>), dim3((unsigned)nwg), dim3(256), 0, st, (const bf16*)XN, (const bf16*)X,
                     (const bf16*)W1, b1, taps, db, (const bf16*)W2, b2, (bf16*)Y, H, W, tx, ty);
  return check_launch("mixffn_bf16");
}

}  // namespace ffn
}  // namespace svk

using namespace svk;

extern "C" int svk_mixffn_fused(int dtype, const void* XN, const void* X, const void* W1, const float* b1,
                                const float* taps, const float* dbias, const void* W2, const float* b2, void* Y,
                                int B, int H, int W, int C, void* stream) {
  if (dtype != SVK_BF16) { set_error("svk_mixffn_fused: bf16 only"); return SVK_EUNSUPPORTED; }
  if (B < 0 || H <= 0 || W <= 0 || !XN || !X || !W1 || !b1 || !taps || !dbias || !W2 || !b2 || !Y) {
    set_error("svk_mixffn_fused: bad args"); return SVK_EINVAL;
  }
  if ((((uintptr_t)XN) | ((uintptr_t)X) | ((uintptr_t)W1) | ((uintptr_t)W2) | ((uintptr_t)Y)) & 15) {
    set_error("svk_mixffn_fused: pointers must be 16-byte aligned"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  // 4 x 14 output tiles (6 x 16 halo) keep LDS and registers small enough for several workgroups
  // per CU, so one workgroup's VALU dwconv phase overlaps another's MFMA phases; 14x14 maps use 7 x 14.
  const bool rows7 = (H % 4 != 0) && (H % 7 == 0);
  switch (C) {
    case 32: return rows7 ? ffn::launch<32, 7, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st)
                          : ffn::launch<32, 4, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st);
    case 64: return rows7 ? ffn::launch<64, 7, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st)
                          : ffn::launch<64, 4, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st);
    case 128: return rows7 ? ffn::launch<128, 7, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st)
                           : ffn::launch<128, 4, 14>(XN, X, W1, b1, taps, dbias, W2, b2, Y, B, H, W, st);
    default:
      set_error("svk_mixffn_fused: C=%d not instantiated (32/64/128)", C);
      return SVK_EUNSUPPORTED;
  }
}
