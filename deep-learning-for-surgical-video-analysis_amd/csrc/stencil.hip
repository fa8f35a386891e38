// Memory-bound stencil / layout kernels over NHWC maps: depthwise 3x3 (+bias+GELU),
// input packing NCHW->NHWC, Gaussian 5x5 reflect filter, bilinear resize, window unfold, cast.
#include "svk_common.h"
#include <type_traits>

namespace svk {

template <typename T>
__device__ __forceinline__ void store_vec8(T* dst, const T* o) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(o);
  } else {
    reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(o)[0];
    reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(o)[1];
  }
}

// ---- DWConv 3x3, pad 1, + bias + act (MixFFN, mix_transformer_evp.py:22-30, 62-63) ----------
// One thread per (8-channel group, column x, strip of R rows): the 3 x (R + 2) input vectors of the
// strip are all loaded up front (16-byte loads, addresses clamped, out-of-image taps zeroed by a
// select — no branches, every load in flight at once), so each output costs 3(R+2)/R loads instead
// of 9.  Consecutive lanes take consecutive channel groups: a wave reads whole contiguous pixel
// rows.  bf16: products in packed f32 (v_pk_fma_f32), branch-free erf for the GELU.
template <typename T> struct Vec8 { uint32_t u[sizeof(T) * 2]; };

template <typename T>
__device__ __forceinline__ void load8_masked(const T* p, bool ok, Vec8<T>& v) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(v.u) = *reinterpret_cast<const uint4*>(p);
  } else {
    reinterpret_cast<uint4*>(v.u)[0] = reinterpret_cast<const uint4*>(p)[0];
    reinterpret_cast<uint4*>(v.u)[1] = reinterpret_cast<const uint4*>(p)[1];
  }
#pragma unroll
  for (int j = 0; j < (int)(sizeof(T) * 2); ++j) v.u[j] = ok ? v.u[j] : 0u;
}
// element pair (2j, 2j+1) of a vector as f32
template <typename T>
__device__ __forceinline__ f32x2 pair(const Vec8<T>& v, int j) {
  if constexpr (sizeof(T) == 2) {
    return unpack2<T>(v.u[j]);
  } else {
    return f32x2{__uint_as_float(v.u[2 * j]), __uint_as_float(v.u[2 * j + 1])};
  }
}

// GELU (erf form, the A&S 7.1.26 erfc of erf_fast: |err| <= 1.5e-7), rearranged branch- and select-free as
// relu(x) - 0.5 |x| t p(t) exp(-x^2 / 2): 11 VALU + 2 transcendental per element (the packed-f32 form
// compiles to scalar ops in this build; same-box A/B +0.35 % on the extraction step)
__device__ __forceinline__ float gelu_rl(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.0f));
  float q = fmaf(-0.5f * 1.061405429f, t, -0.5f * -1.453152027f);
  q = fmaf(q, t, -0.5f * 1.421413741f);
  q = fmaf(q, t, -0.5f * -0.284496736f);
  q = fmaf(q, t, -0.5f * 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);   // exp(-x^2 / 2)
  return fmaf(ax * t * q, e, fmaxf(x, 0.f));
}
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) { return f32x2{gelu_rl(x.x), gelu_rl(x.y)}; }

// Physical block b runs on XCD b % 8 (observed dispatch order, MI355X_MICROARCH.md: speed only, no
// correctness depends on it).  Returns the logical block so that XCD k walks logical blocks
// [start_k, start_k + count_k) — a bijection on [0, n) for any n.
__device__ __forceinline__ long xcd_group(unsigned b, unsigned n) {
  const unsigned per = n >> 3, rem = n & 7, x = b & 7, slot = b >> 3;
  return x < rem ? (long)x * (per + 1) + slot : (long)rem * (per + 1) + (long)(x - rem) * per + slot;
}

template <typename T, int R>
__global__ __launch_bounds__(256) void dwconv3x3_strip(const T* __restrict__ X, const float* __restrict__ w,
                                                       const float* __restrict__ bias, T* __restrict__ Y,
                                                       T* __restrict__ Ypre, int B, int H, int W, int C, int act,
                                                       int nstrip, int xcd) {
  const int CG = C >> 3;
  // xcd: blocks are dealt round-robin over the 8 XCDs; regroup them so each XCD walks one contiguous
  // range of (image, strip, column) — a column's left / right neighbours and the strip halos then come
  // from the same L2 instead of being fetched again by up to three XCDs
  const long blk = xcd ? xcd_group(blockIdx.x, gridDim.x) : (long)blockIdx.x;
  const long idx = blk * blockDim.x + threadIdx.x;
  const long total = (long)B * nstrip * W * CG;
  if (idx >= total) return;
  const int cg = (int)(idx % CG);
  long t = idx / CG;
  const int x = (int)(t % W);
  t /= W;
  const int s = (int)(t % nstrip);
  const int b = (int)(t / nstrip);
  const int c0 = cg * 8, y0 = s * R;
  const T* base = X + (long)b * H * W * C + c0;
  const int xl = x > 0 ? x - 1 : 0, xr = x < W - 1 ? x + 1 : W - 1;

  Vec8<T> win[R + 2][3];
#pragma unroll
  for (int r = 0; r < R + 2; ++r) {
    const int yy = y0 - 1 + r;
    const bool oky = yy >= 0 && yy < H;
    const int yc = min(max(yy, 0), H - 1);
    const T* row = base + (long)yc * W * C;
    load8_masked(row + (long)xl * C, oky && x > 0, win[r][0]);
    load8_masked(row + (long)x * C, oky, win[r][1]);
    load8_masked(row + (long)xr * C, oky && x < W - 1, win[r][2]);
  }
  f32x2 wt[9][4], bs[4];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wt[k][j] = *reinterpret_cast<const f32x2*>(w + k * C + c0 + 2 * j);
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = *reinterpret_cast<const f32x2*>(bias + c0 + 2 * j);

#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int y = y0 + r;
    if (y >= H) break;
    f32x2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bs[j];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = pair(win[r + dy][dx], j) * wt[dy * 3 + dx][j] + acc[j];
    const long off = (((long)b * H + y) * W + x) * C + c0;
    T o[8];
    if (Ypre) {   // pre-activation copy (training: the GELU backward needs it)
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[2 * j] = from_f<T>(acc[j].x); o[2 * j + 1] = from_f<T>(acc[j].y); }
      store_vec8(Ypre + off, o);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x2 g;
      if (sizeof(T) == 2 && act == SVK_ACT_GELU) g = gelu_fast2(acc[j]);
      else g = f32x2{apply_act(acc[j].x, act), apply_act(acc[j].y, act)};
      o[2 * j] = from_f<T>(g.x);
      o[2 * j + 1] = from_f<T>(g.y);
    }
    store_vec8(Y + off, o);
  }
}

// Rolling-window variant (bf16, C % 4 == 0): one thread per (4-channel group, column x, strip of R
// rows).  Only three input rows (3 columns x 4 channels, 8-byte loads) are live at a time — the next
// row is loaded while the current output row is computed — and the taps are 9 x 4 floats, so the
// kernel needs ~80 VGPRs (6 waves / SIMD) where the all-rows-up-front strip kernel needs ~240 (2 per
// SIMD): the loads' latency is hidden by occupancy instead of by one thread's register window.
template <int R>
__global__ __launch_bounds__(256) void dwconv3x3_roll_bf16(const bf16* __restrict__ X, const float* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ Y,
                                                           bf16* __restrict__ Ypre, int B, int H, int W, int C,
                                                           int act, int nstrip) {
  const int CG = C >> 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * nstrip * W * CG;
  if (idx >= total) return;
  const int cg = (int)(idx % CG);
  long t = idx / CG;
  const int x = (int)(t % W);
  t /= W;
  const int s = (int)(t % nstrip);
  const int b = (int)(t / nstrip);
  const int c0 = cg * 4, y0 = s * R;
  const bf16* base = X + (long)b * H * W * C + c0;
  const int xl = x > 0 ? x - 1 : 0, xr = x < W - 1 ? x + 1 : W - 1;
  f32x2 wt[9][2], bs[2];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j) wt[k][j] = *reinterpret_cast<const f32x2*>(w + k * C + c0 + 2 * j);
#pragma unroll
  for (int j = 0; j < 2; ++j) bs[j] = *reinterpret_cast<const f32x2*>(bias + c0 + 2 * j);

  auto load_row = [&](int yy, uint2* v) {
    const bool oky = yy >= 0 && yy < H;
    const bf16* row = base + (long)min(max(yy, 0), H - 1) * W * C;
    const uint2 a = *reinterpret_cast<const uint2*>(row + (long)xl * C);
    const uint2 m = *reinterpret_cast<const uint2*>(row + (long)x * C);
    const uint2 c = *reinterpret_cast<const uint2*>(row + (long)xr * C);
    const bool okl = oky && x > 0, okr = oky && x < W - 1;
    v[0] = okl ? a : uint2{0u, 0u};
    v[1] = oky ? m : uint2{0u, 0u};
    v[2] = okr ? c : uint2{0u, 0u};
  };
  auto lo = [](uint32_t u) { return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)}; };
  uint2 win[3][3];
  load_row(y0 - 1, win[0]);
  load_row(y0, win[1]);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int y = y0 + r;
    if (y >= H) break;
    load_row(y + 1, win[(r + 2) % 3]);
    f32x2 acc[2] = {bs[0], bs[1]};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const uint2* v = win[(r + dy) % 3];
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        acc[0] = lo(v[dx].x) * wt[dy * 3 + dx][0] + acc[0];
        acc[1] = lo(v[dx].y) * wt[dy * 3 + dx][1] + acc[1];
      }
    }
    const long off = (((long)b * H + y) * W + x) * C + c0;
    if (Ypre) {
      bf16 o[4] = {(bf16)acc[0].x, (bf16)acc[0].y, (bf16)acc[1].x, (bf16)acc[1].y};
      *reinterpret_cast<uint2*>(Ypre + off) = *reinterpret_cast<const uint2*>(o);
    }
    f32x2 g0, g1;
    if (act == SVK_ACT_GELU) {
      g0 = gelu_fast2(acc[0]);
      g1 = gelu_fast2(acc[1]);
    } else {
      g0 = f32x2{apply_act(acc[0].x, act), apply_act(acc[0].y, act)};
      g1 = f32x2{apply_act(acc[1].x, act), apply_act(acc[1].y, act)};
    }
    bf16 o[4] = {(bf16)g0.x, (bf16)g0.y, (bf16)g1.x, (bf16)g1.y};
    *reinterpret_cast<uint2*>(Y + off) = *reinterpret_cast<const uint2*>(o);
  }
}

// ---- MixFFN front half in one kernel: G = act(dwconv3x3(XN W1^T + b1) + db) ------------------------
// (Mlp.fc1 -> DWConv -> GELU, mix_transformer_evp.py:60-63 / 24-30).  One workgroup per (frame, strip
// of R image rows, 64 hidden channels): it computes the fc1 outputs of the strip plus one halo row
// above and below ((R + 2) x W tokens, MFMA 16x16x32 with the W1 chunk in LDS and the XN rows read as
// A fragments straight from global memory), rounds them to bf16 exactly like the unfused fc1 GEMM
// output and keeps them in an LDS halo tile (zero columns / out-of-image rows = the conv's zero
// padding), then runs the depthwise conv + GELU from LDS and writes G.  The hidden map H — the
// largest tensor of the path — never goes to HBM: the unfused path writes it once and reads it
// (through the vector caches) about 1.4 times.  The halo rows cost (R + 2) / R of the fc1 MFMA work.
template <typename T, int KS>   // T = bf16 / f16; K = 32 * KS (fc1 input channels)
__global__ __launch_bounds__(256) void fc1_dwconv(const T* __restrict__ XN, const T* __restrict__ W1,
                                                  const float* __restrict__ b1, const float* __restrict__ taps,
                                                  const float* __restrict__ db, T* __restrict__ G,
                                                  T* __restrict__ Gpre, int H, int W, int K, int HID, int R,
                                                  int nstrip, int act) {
  typedef v8_t<T> tx8;
  extern __shared__ __attribute__((aligned(16))) uint4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int WLD = K + 8;                                   // W1 chunk row stride (elements)
  T* sW = reinterpret_cast<T*>(smem);                      // [64][WLD]
  const int TW = W + 2;
  char* sH = smem + 64 * WLD * 2;                          // [(R + 2)][TW][64] T
  const int nnb = HID >> 6;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int nb = id % nnb, s = (id / nnb) % nstrip, b = id / (nnb * nstrip);
  const int y0 = s * R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  // W1 rows nb*64 .. +63 -> LDS; zero halo columns of the hidden tile
  for (int e = tid; e < 64 * (K >> 3); e += 256) {
    const int n = e / (K >> 3), k8 = (e - n * (K >> 3)) * 8;
    *reinterpret_cast<uint4*>(sW + n * WLD + k8) = *reinterpret_cast<const uint4*>(W1 + (long)(nb * 64 + n) * K + k8);
  }
  for (int e = tid; e < (R + 2) * 2 * 8; e += 256) {
    const int hr = e >> 4, side = (e >> 3) & 1, c = e & 7;
    reinterpret_cast<uint4*>(sH + ((hr * TW + (side ? TW - 1 : 0)) * 64) * 2)[c] = uint4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  // fc1 over the (R + 2) x W halo tokens: lane -> token fr of the 16-token tile, 4 channels 4fq + r of
  // each 16-channel block (W1 fragment as the A operand: the tile comes out transposed)
  const int ntok = (R + 2) * W, mt_n = (ntok + 15) >> 4;
  const T* Xb = XN + (long)b * H * W * K;
  float bias4[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias4[j][r] = b1[nb * 64 + j * 16 + 4 * fq + r];
  // A fragments of this wave's m-tiles, software-pipelined: the next tile's K row is in flight
  // while the current tile's MFMAs run (rows clamped into the image; invalid tokens stored as zeros)
  auto load_a = [&](int mt, tx8* a) {
    const int t = mt * 16 + fr;
    const int hr = t / W, x = t - hr * W;
    const int y = min(max(y0 - 1 + hr, 0), H - 1);
    const T* xr = Xb + ((long)y * W + min(x, W - 1)) * K + fq * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks] = *reinterpret_cast<const tx8*>(xr + ks * 32);
  };
  tx8 anext[KS];
  if (wave < mt_n) load_a(wave, anext);
  for (int mt = wave; mt < mt_n; mt += 4) {
    const int t = mt * 16 + fr;
    const int hr = t / W, x = t - hr * W;
    const int y = y0 - 1 + hr;
    const bool valid = t < ntok && (unsigned)y < (unsigned)H;
    tx8 a[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks] = anext[ks];
    if (mt + 4 < mt_n) load_a(mt + 4, anext);
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const tx8 w = *reinterpret_cast<const tx8*>(sW + (j * 16 + fr) * WLD + ks * 32 + fq * 8);
        acc[j] = mfma16x16x32(w, a[ks], acc[j]);
      }
    if (t < ntok) {
      char* dst = sH + ((hr * TW + x + 1) * 64) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        T o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = valid ? (T)(acc[j][r] + bias4[j][r]) : (T)0.f;
        *reinterpret_cast<uint2*>(dst + (j * 16 + 4 * fq) * 2) = *reinterpret_cast<const uint2*>(o);
      }
    }
  }

  // depthwise 3x3 + bias + act from the LDS tile (same arithmetic order as dwconv3x3_strip)
  const int c = tid & 7, pl = tid >> 3;
  const int c0 = nb * 64 + c * 8;
  f32x2 wt[9][4], bs[4];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wt[k][j] = *reinterpret_cast<const f32x2*>(taps + k * HID + c0 + 2 * j);
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = *reinterpret_cast<const f32x2*>(db + c0 + 2 * j);
  __syncthreads();
  const uint4* tile = reinterpret_cast<const uint4*>(sH);
  const int rows = min(R, H - y0);
  T* Gb = G + (long)b * H * W * HID + c0;
  T* Gpb = Gpre ? Gpre + (long)b * H * W * HID + c0 : nullptr;
  for (int q = pl; q < rows * W; q += 32) {
    const int r = q / W, x = q - r * W;
    f32x2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bs[j];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        Vec8<T> v;
        *reinterpret_cast<uint4*>(v.u) = tile[((r + dy) * TW + x + dx) * 8 + c];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = pair(v, j) * wt[dy * 3 + dx][j] + acc[j];
      }
    T o[8];
    const long off = ((long)(y0 + r) * W + x) * HID;
    if (Gpre) {   // pre-activation copy (training: the GELU backward reads it), rounded like dwconv3x3_strip's
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[2 * j] = (T)acc[j].x; o[2 * j + 1] = (T)acc[j].y; }
      store_vec8(Gpb + off, o);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2 g = act == SVK_ACT_GELU ? gelu_fast2(acc[j]) : f32x2{apply_act(acc[j].x, act), apply_act(acc[j].y, act)};
      o[2 * j] = (T)g.x;
      o[2 * j + 1] = (T)g.y;
    }
    store_vec8(Gb + off, o);
  }
}

// LDS-tiled variant (bf16, C % 64 == 0): one workgroup per (frame, strip of R rows, 64-channel
// block).  The (R + 2) x (W + 2) halo tile of the block's 64 channels is read from HBM once —
// every 16-byte chunk by exactly one lane, out-of-image pixels as zeros (the conv's zero padding),
// addresses clamped so the loads are branch-free — and the 9 taps of every output are then read
// from LDS (a wave's 64 lanes = 8 pixels x 8 channel groups: 1 KiB contiguous per ds_read_b128,
// conflict-free).  The strip kernel above reads each input vector 3 (R + 2) / R times through the
// vector caches instead; here the only re-read is the 2-row halo (2 / R, mostly L2).
// Workgroup ids are XCD-remapped so that consecutive strips of a frame (which share halo rows)
// run on one XCD's L2.
__global__ __launch_bounds__(256) void dwconv3x3_lds_bf16(const bf16* __restrict__ X, const float* __restrict__ w,
                                                          const float* __restrict__ bias, bf16* __restrict__ Y,
                                                          bf16* __restrict__ Ypre, int H, int W, int C, int R,
                                                          int nstrip, int act) {
  extern __shared__ __attribute__((aligned(16))) uint4 tile[];   // [(R + 2)][(W + 2)][8] 16-byte chunks
  const int ncb = C >> 6;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int s = id % nstrip, cb = (id / nstrip) % ncb, b = id / (nstrip * ncb);
  const int y0 = s * R, TW = W + 2;
  const int tid = threadIdx.x;
  const bf16* Xb = X + (long)b * H * W * C + cb * 64;

  // stage the halo tile: chunk i -> (row, col, c); branch-free clamped loads, zeros outside
  const int nchunk = (R + 2) * TW * 8;
  for (int i0 = 0; i0 < nchunk; i0 += 4 * 256) {
    uint4 v[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256 + tid;
      const int row = i / (TW * 8), rem = i - row * (TW * 8), col = rem >> 3, c = rem & 7;
      const int y = y0 - 1 + row, x = col - 1;
      ok[u] = i < nchunk && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const int yc = min(max(y, 0), H - 1), xc = min(max(x, 0), W - 1);
      v[u] = *reinterpret_cast<const uint4*>(Xb + ((long)yc * W + xc) * C + c * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256 + tid;
      if (i < nchunk) tile[i] = ok[u] ? v[u] : uint4{0u, 0u, 0u, 0u};
    }
  }

  const int c = tid & 7, pl = tid >> 3;
  const int c0 = cb * 64 + c * 8;
  f32x2 wt[9][4], bs[4];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wt[k][j] = *reinterpret_cast<const f32x2*>(w + k * C + c0 + 2 * j);
#pragma unroll
  for (int j = 0; j < 4; ++j) bs[j] = *reinterpret_cast<const f32x2*>(bias + c0 + 2 * j);
  __syncthreads();

  const int rows = min(R, H - y0);
  bf16* Yb = Y + (long)b * H * W * C + c0;
  bf16* Pb = Ypre ? Ypre + (long)b * H * W * C + c0 : nullptr;
  for (int q = pl; q < rows * W; q += 32) {
    const int r = q / W, x = q - r * W;
    f32x2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bs[j];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        Vec8<bf16> v;
        *reinterpret_cast<uint4*>(v.u) = tile[((r + dy) * TW + x + dx) * 8 + c];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = pair(v, j) * wt[dy * 3 + dx][j] + acc[j];
      }
    const long off = ((long)(y0 + r) * W + x) * C;
    bf16 o[8];
    if (Pb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[2 * j] = (bf16)acc[j].x; o[2 * j + 1] = (bf16)acc[j].y; }
      store_vec8(Pb + off, o);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2 g = act == SVK_ACT_GELU ? gelu_fast2(acc[j]) : f32x2{apply_act(acc[j].x, act), apply_act(acc[j].y, act)};
      o[2 * j] = (bf16)g.x;
      o[2 * j + 1] = (bf16)g.y;
    }
    store_vec8(Yb + off, o);
  }
}

template <typename T>
__global__ void dwconv3x3_scalar(const T* __restrict__ X, const float* __restrict__ w, const float* __restrict__ bias,
                                 T* __restrict__ Y, T* __restrict__ Ypre, int B, int H, int W, int C, int act) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * H * W * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int x = (int)(pix % W);
  const long t = pix / W;
  const int y = (int)(t % H);
  const int b = (int)(t / H);
  float acc = bias[c];
  for (int dy = -1; dy <= 1; ++dy)
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = y + dy, xx = x + dx;
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      acc += to_f(X[(((long)b * H + yy) * W + xx) * C + c]) * w[((dy + 1) * 3 + (dx + 1)) * C + c];
    }
  if (Ypre) Ypre[idx] = from_f<T>(acc);
  Y[idx] = from_f<T>(apply_act(acc, act));
}

// ---- NCHW f32 -> NHWC T --------------------------------------------------------------------
// One thread per pixel: reads coalesced along W within each channel plane, the pixel's Cpad
// channels written as whole 16-byte vectors (Cpad % 8 == 0) or scalars.
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ X, T* __restrict__ Y, int B, int C, int H, int W,
                                    int Cpad) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long hw = (long)H * W;
  if (pix >= (long)B * hw) return;
  const long b = pix / hw, p = pix - b * hw;
  const float* src = X + b * C * hw + p;
  T* dst = Y + pix * Cpad;
  if ((Cpad & 7) == 0) {
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      T o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = from_f<T>(c0 + j < C ? src[(long)(c0 + j) * hw] : 0.f);
      store_vec8(dst + c0, o);
    }
  } else {
    for (int c = 0; c < Cpad; ++c) dst[c] = from_f<T>(c < C ? src[(long)c * hw] : 0.f);
  }
}

// 4 pixels per thread (H*W % 4 == 0, C <= 8, Cpad == 8): one float4 load per channel plane and four
// 16-byte NHWC stores, so a wave moves 1 KB per instruction instead of 256 B (the input packing of
// frames / flow runs at the HBM rate instead of the one-pixel kernel's load-issue rate)
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc8_x4_kernel(const float* __restrict__ X, T* __restrict__ Y, int C,
                                                              long hw, long npix4) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npix4) return;
  const long pix = q * 4, b = pix / hw, p = pix - b * hw;
  const float* src = X + b * C * hw + p;
  float v[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c < C) {
      const float4 f = *reinterpret_cast<const float4*>(src + (long)c * hw);
      v[c][0] = f.x; v[c][1] = f.y; v[c][2] = f.z; v[c][3] = f.w;
    } else {
      v[c][0] = v[c][1] = v[c][2] = v[c][3] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    T o[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) o[c] = from_f<T>(v[c][k]);
    store_vec8(Y + (pix + k) * 8, o);
  }
}

// ---- stem input as space-to-depth blocks (the k = 7, s = 4 OverlapPatchEmbed / flow conv1 stems) -----
// NCHW f32 [B, C, H, W] -> [B, NBH, NBW, S*S*C]: block (by, bx) holds input rows S*by - pad .. + S - 1 and
// the same columns, channel (dy*S + dx)*C + c, zeros outside the image.  A k <= 2S, stride-S conv with
// padding `pad` is then a 2 x 2, stride-1, unpadded conv over the blocks (weights zero beyond k, see
// svk.pack.conv_w_s2d): K = 4*S*S*C (192 for RGB, 128 for flow) instead of k*k*8 = 392 with the 3 real
// channels padded to 8, and the packed map is 16*C/8*... = 2.7x smaller than the 8-channel NHWC one.
template <typename T, int S, int C>
__global__ __launch_bounds__(256) void nchw_to_s2d_kernel(const float* __restrict__ X, T* __restrict__ Y, int H, int W,
                                                          int pad, int NBH, int NBW, long nblk) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nblk) return;
  const int bx = (int)(q % NBW);
  const long t = q / NBW;
  const int by = (int)(t % NBH);
  const long b = t / NBH;
  const float* src = X + b * C * (long)H * W;
  constexpr int NCH = S * S * C;
  T o[NCH];
#pragma unroll
  for (int dy = 0; dy < S; ++dy) {
    const int y = S * by - pad + dy;
    const bool oky = y >= 0 && y < H;
    const int yc = min(max(y, 0), H - 1);
#pragma unroll
    for (int dx = 0; dx < S; ++dx) {
      const int x = S * bx - pad + dx;
      const bool ok = oky && x >= 0 && x < W;
      const int xc = min(max(x, 0), W - 1);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float v = src[((long)c * H + yc) * W + xc];
        o[(dy * S + dx) * C + c] = from_f<T>(ok ? v : 0.f);
      }
    }
  }
  T* dst = Y + q * NCH;
#pragma unroll
  for (int k = 0; k < NCH / 8; ++k) store_vec8(dst + 8 * k, o + 8 * k);
}

// ---- GaussianFilter.conv_gauss: reflect pad 2 + binomial 5x5 / 256 (mix_transformer_evp.py:501-514)
__device__ __forceinline__ int reflect(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

// One thread per (column x, strip of GR rows): the filter is separable ([1 4 6 4 1] / 16 twice,
// exactly the reference's outer-product kernel), so each of the GR + 4 input rows is filtered
// horizontally once (5 coalesced loads along W) and the strip's outputs are vertical 5-tap sums of
// those row results.  Output NHWC, channels padded to Cpad, 16-byte stores when Cpad % 8 == 0.
constexpr int GR = 8;
template <typename T, int CMAX>
__global__ void gauss5x5_kernel(const float* __restrict__ X, T* __restrict__ Y, int B, int C, int H, int W, int Cpad,
                                int nstrip) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * nstrip * W) return;
  const int x = (int)(idx % W);
  const long t = idx / W;
  const int s = (int)(t % nstrip);
  const int b = (int)(t / nstrip);
  const int y0 = s * GR;
  const float k1[5] = {1.f / 16.f, 4.f / 16.f, 6.f / 16.f, 4.f / 16.f, 1.f / 16.f};
  int xx[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) xx[j] = reflect(x + j - 2, W);
  float out[GR][CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    if (c >= C) {
#pragma unroll
      for (int r = 0; r < GR; ++r) out[r][c] = 0.f;
      continue;
    }
    const float* src = X + ((long)b * C + c) * H * W;
    float h[GR + 4];
#pragma unroll
    for (int r = 0; r < GR + 4; ++r) {
      const int yy = reflect(min(y0 + r - 2, H + 1), H);   // rows past the strip's last valid output: clamp
      const float* row = src + (long)yy * W;
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < 5; ++j) a += row[xx[j]] * k1[j];
      h[r] = a;
    }
#pragma unroll
    for (int r = 0; r < GR; ++r) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) a += h[r + i] * k1[i];
      out[r][c] = a;
    }
  }
#pragma unroll
  for (int r = 0; r < GR; ++r) {
    const int y = y0 + r;
    if (y >= H) break;
    T* dst = Y + (((long)b * H + y) * W + x) * Cpad;
    if ((Cpad & 7) == 0 && CMAX <= 8) {
      T o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = from_f<T>(c < CMAX ? out[r][c < CMAX ? c : 0] : 0.f);
      store_vec8(dst, o);
      for (int c = 8; c < Cpad; c += 8) {
        T z[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) z[j] = from_f<T>(0.f);
        store_vec8(dst + c, z);
      }
    } else {
      for (int c = 0; c < Cpad; ++c) dst[c] = from_f<T>(c < CMAX ? out[r][c < CMAX ? c : 0] : 0.f);
    }
  }
}

// 4-column variant (W % 4 == 0, C <= 3, Cpad == 8, the prompt generator's frame / segmap filter): a thread
// owns 4 consecutive columns x GR rows; each input row piece is three aligned float4 loads (columns x0 - 4 ..
// x0 + 7, reflected at the image edges from the middle block) instead of 5 scalar loads per column, and
// each output pixel leaves as one 16-byte store.  Same arithmetic order as gauss5x5_kernel (bitwise equal).
template <typename T, int GR>
__global__ __launch_bounds__(256) void gauss5x5_x4_kernel(const float* __restrict__ X, T* __restrict__ Y, int B, int C, int H, int W,
                                   int nstrip) {
  const int W4 = W >> 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * nstrip * W4) return;
  const int x0 = (int)(idx % W4) * 4;
  const long t = idx / W4;
  const int s = (int)(t % nstrip);
  const int b = (int)(t / nstrip);
  const int y0 = s * GR;
  const float k1[5] = {1.f / 16.f, 4.f / 16.f, 6.f / 16.f, 4.f / 16.f, 1.f / 16.f};
  const bool left = x0 == 0, right = x0 + 4 == W;
  float out[GR][4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (c >= C) {
#pragma unroll
      for (int r = 0; r < GR; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) out[r][k][c] = 0.f;
      continue;
    }
    const float* src = X + ((long)b * C + c) * H * W;
    float h[GR + 4][4];
#pragma unroll
    for (int r = 0; r < GR + 4; ++r) {
      const int yy = reflect(min(y0 + r - 2, H + 1), H);
      const float* row = src + (long)yy * W + x0;
      const float4 m = *reinterpret_cast<const float4*>(row);
      const float4 l = left ? m : *reinterpret_cast<const float4*>(row - 4);
      const float4 rr = right ? m : *reinterpret_cast<const float4*>(row + 4);
      // window w[j] = column x0 - 2 + j (reflect: -2 -> 2, -1 -> 1, W -> W - 2, W + 1 -> W - 3)
      const float w[8] = {left ? m.z : l.z, left ? m.y : l.w, m.x, m.y, m.z, m.w, right ? m.z : rr.x, right ? m.y : rr.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) a += w[k + j] * k1[j];
        h[r][k] = a;
      }
    }
#pragma unroll
    for (int r = 0; r < GR; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) a += h[r + i][k] * k1[i];
        out[r][k][c] = a;
      }
  }
#pragma unroll
  for (int r = 0; r < GR; ++r) {
    const int y = y0 + r;
    if (y >= H) break;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      T o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) o[c] = from_f<T>(c < 3 ? out[r][k][c < 3 ? c : 0] : 0.f);
      store_vec8(Y + (((long)b * H + y) * W + x0 + k) * 8, o);
    }
  }
}


// ---- bilinear resize, align_corners=False, no antialias (F.interpolate semantics) ----------
__device__ __forceinline__ void src_index(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * (dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - i0;
  l0 = 1.f - l1;
}

template <typename T>
__global__ void resize_bilinear_kernel(const T* __restrict__ X, long ldx, T* __restrict__ Y, long ldy,
                                       int B, int H, int W, int C, int OH, int OW) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * OH * OW * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int ox = (int)(pix % OW);
  const long t = pix / OW;
  const int oy = (int)(t % OH);
  const int b = (int)(t / OH);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  src_index(oy, H, OH, y0, y1, ly0, ly1);
  src_index(ox, W, OW, x0, x1, lx0, lx1);
  const T* base = X + (long)b * H * W * ldx + c;
  auto at = [&](int yy, int xx) { return to_f(base[((long)yy * W + xx) * ldx]); };
  const float v = ly0 * (lx0 * at(y0, x0) + lx1 * at(y0, x1)) + ly1 * (lx0 * at(y1, x0) + lx1 * at(y1, x1));
  Y[((long)b * OH * OW + (long)oy * OW + ox) * ldy + c] = from_f<T>(v);
}

// ---- the head's four pyramid resizes in one launch (segformer_head.py:150-158: c4..c1 resized to the
// c4 grid and concatenated along channels): a thread owns 8 channels of one output pixel of one level,
// 16-byte loads of the four source pixels and one 16-byte store into the concatenated row; the blend is
// resize_bilinear_kernel's expression, so the values are bit-identical to four resize_bilinear calls
struct RsLevels {
  const void* X[4];
  long ldx[4];
  int H[4], W[4], coff[5];   // coff[l]..coff[l+1]: level l's channels in the output row
};

template <typename T>
__global__ void resize_multi_kernel(RsLevels L, int nl, T* __restrict__ Y, long ldy, int B, int OH, int OW) {
  const int nq = L.coff[nl] / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * OH * OW * nq;
  if (idx >= total) return;
  const int q = (int)(idx % nq);
  const long pix = idx / nq;
  const int ox = (int)(pix % OW);
  const long t = pix / OW;
  const int oy = (int)(t % OH);
  const int b = (int)(t / OH);
  const int c0 = 8 * q;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i) l += (i < nl && c0 >= L.coff[i]) ? 1 : 0;
  const int H = L.H[l], W = L.W[l], c = c0 - L.coff[l];
  const long ldx = L.ldx[l];
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  src_index(oy, H, OH, y0, y1, ly0, ly1);
  src_index(ox, W, OW, x0, x1, lx0, lx1);
  const T* base = static_cast<const T*>(L.X[l]) + (long)b * H * W * ldx + c;
  typedef T v8 __attribute__((ext_vector_type(8)));
  const v8 a = *reinterpret_cast<const v8*>(base + ((long)y0 * W + x0) * ldx);
  const v8 bb = *reinterpret_cast<const v8*>(base + ((long)y0 * W + x1) * ldx);
  const v8 cc = *reinterpret_cast<const v8*>(base + ((long)y1 * W + x0) * ldx);
  const v8 d = *reinterpret_cast<const v8*>(base + ((long)y1 * W + x1) * ldx);
  v8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    o[e] = from_f<T>(ly0 * (lx0 * to_f(a[e]) + lx1 * to_f(bb[e])) + ly1 * (lx0 * to_f(cc[e]) + lx1 * to_f(d[e])));
  *reinterpret_cast<v8*>(Y + ((long)b * OH * OW + (long)oy * OW + ox) * ldy + c0) = o;
}

// ---- causal window unfold (adapter_transformer.py:336-343) ---------------------------------
template <typename T>
__global__ void window_unfold_kernel(const T* __restrict__ X, long ldx, const float* __restrict__ pos, T* __restrict__ Y,
                                     int Tn, int C, int len) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Tn * len * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long r = idx / C;
  const int i = (int)(r % len);
  const long t = r / len;
  const long src = t - len + 1 + i;
  float v = src >= 0 ? to_f(X[src * ldx + c]) : 0.f;
  if (pos) v += pos[i * C + c];
  Y[idx] = from_f<T>(v);
}

// Y[r, c] = X[r, c] + P[r % period, c]  (positional-table add, Transformer2_3_1 encoder input)
template <typename T>
__global__ void add_bcast_kernel(const T* __restrict__ X, const float* __restrict__ P, T* __restrict__ Y, long M, int C,
                                 int period) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * C) return;
  const long r = idx / C;
  const int c = (int)(idx - r * C);
  Y[idx] = from_f<T>(to_f(X[idx]) + P[(r % period) * C + c]);
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ X, TO* __restrict__ Y, long n) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) Y[idx] = from_f<TO>(to_f(X[idx]));
}

inline dim3 grid1d(long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

}  // namespace svk

using namespace svk;

extern "C" int svk_dwconv3x3_ex(int dtype, const void* X, const float* w, const float* bias, void* Y, void* Ypre,
                                int B, int H, int W, int C, int act, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || !X || !w || !bias || !Y) { set_error("svk_dwconv3x3: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    const bool vec = (C % 8 == 0) && (((uintptr_t)X | (uintptr_t)Y | (uintptr_t)Ypre) & 15) == 0;
    const int lds_env = g_tune[TUNE_DW_LDS], rows_env = g_tune[TUNE_DW_ROWS];   // svk_tune knobs
    constexpr bool is_bf16 = std::is_same<T, bf16>::value;   // the opt-in variants below are bf16-only
    // rolling window: by default for the bf16 activation-free conv (the train step's dwconv data gradient with
    // flipped taps; round 6, profiles/r06/dw_train.txt: 87.8 -> 78.9 us at 88 x 56 x 56 x 256, 43.0 -> 38.9 at
    // 28 x 28 x 512, 18.0 -> 13.1 at 7 x 7 x 2048), or forced by dw_lds = 2
    // with GELU (the train forward's stages 3-4, + pre-activation store; profiles/r06/dw_train.txt): the rolling window
    // at 7 x 7 (20.1 -> 15.7 us at 2048 channels), the LDS halo tile at 14 x 14 with >= 1024 channels (37.2 -> 33.0)
    const bool auto_roll = lds_env < 0 && (act == SVK_ACT_NONE || W <= 8);
    const bool auto_lds = lds_env < 0 && act != SVK_ACT_NONE && W > 8 && W <= 16 && C >= 1024;
    if (is_bf16 && (lds_env == 2 || auto_roll) && C % 4 == 0 &&
        (((uintptr_t)X | (uintptr_t)Y | (uintptr_t)Ypre) & 7) == 0) {
      constexpr int RR = 8;
      const int nstrip = (H + RR - 1) / RR;
      const long n = (long)B * nstrip * W * (C / 4);
      hipLaunchKernelGGL((dwconv3x3_roll_bf16<RR>), grid1d(n), dim3(256), 0, st, (const bf16*)X, w, bias, (bf16*)Y,
                         (bf16*)Ypre, B, H, W, C, act, nstrip);
      return check_launch("dwconv3x3_roll");
    }
    if (is_bf16 && vec && C % 64 == 0 && (lds_env == 1 || auto_lds)) {
      // strip height: the tallest strip whose halo tile fits 48 KiB (3 workgroups per CU)
      int R = rows_env > 0 ? rows_env : 49152 / ((W + 2) * 128) - 2;
      R = std::max(1, std::min(R, H));
      const size_t lds = (size_t)(R + 2) * (W + 2) * 128;
      if (lds <= 65536) {
        const int nstrip = (H + R - 1) / R;
        const long nwg = (long)B * nstrip * (C / 64);
        if (nwg < 0x7fffffffL) {
          hipLaunchKernelGGL(dwconv3x3_lds_bf16, dim3((unsigned)nwg), dim3(256), lds, st, (const bf16*)X, w, bias,
                             (bf16*)Y, (bf16*)Ypre, H, W, C, R, nstrip, act);
          return check_launch("dwconv3x3_lds");
        }
      }
    }
    if (vec) {
      constexpr int R = sizeof(T) == 2 ? 7 : 2;   // 16-bit: 56 / 28 / 14 / 7-row maps in whole strips
      const int nstrip = (H + R - 1) / R;
      const long n = (long)B * nstrip * W * (C / 8);
      static const int xcd = getenv("SVK_DW_XCD") ? atoi(getenv("SVK_DW_XCD")) : 0;   // A/B: grouping 0.3 % slower
      hipLaunchKernelGGL((dwconv3x3_strip<T, R>), grid1d(n), dim3(256), 0, st, (const T*)X, w, bias, (T*)Y, (T*)Ypre, B,
                         H, W, C, act, nstrip, xcd);
    } else {
      const long n = (long)B * H * W * C;
      hipLaunchKernelGGL((dwconv3x3_scalar<T>), grid1d(n), dim3(256), 0, st, (const T*)X, w, bias, (T*)Y, (T*)Ypre, B,
                         H, W, C, act);
    }
    return check_launch("dwconv3x3");
  });
}

// fc1 + depthwise conv + activation (MixFFN front half) in one pass; see fc1_dwconv.
extern "C" int svk_mixffn_fc1_dwconv_ex(int dtype, const void* XN, const void* W1, const float* b1,
                                        const float* taps, const float* dbias, void* G, void* Gpre, int B, int H,
                                        int W, int C, int hidden, int act, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || hidden <= 0 || !XN || !W1 || !b1 || !taps || !dbias || !G) {
    set_error("svk_mixffn_fc1_dwconv: bad args"); return SVK_EINVAL;
  }
  if ((dtype != SVK_BF16 && dtype != SVK_F16) || (C != 32 && C != 64 && C != 128 && C != 320 && C != 512) ||
      hidden % 64 || ((((uintptr_t)XN) | ((uintptr_t)W1) | ((uintptr_t)G) | ((uintptr_t)Gpre)) & 15)) {
    set_error("svk_mixffn_fc1_dwconv: needs bf16 / f16, C in {32, 64, 128, 320, 512}, hidden %% 64 == 0, "
              "16-byte aligned maps");
    return SVK_EUNSUPPORTED;
  }
  if (B == 0) return SVK_OK;
  if (!Gpre &&
      fc1dw_rw_try(dtype, XN, W1, b1, taps, dbias, G, B, H, W, C, hidden, act, (hipStream_t)stream) == 0) return SVK_OK;
  // strip height: halo tile <= 44 KiB (measured best at B = 256 against 48 KiB for W1 + tile), strips
  // of equal height; the svk_tune "dw_rows" knob overrides it
  int rmax = std::max(1, std::min(H, 45056 / ((W + 2) * 128) - 2));
  if (g_tune[TUNE_DW_ROWS] > 0) rmax = std::min(H, g_tune[TUNE_DW_ROWS]);
  const int nst0 = (H + rmax - 1) / rmax;
  const int R = (H + nst0 - 1) / nst0, nstrip = (H + R - 1) / R;
  const size_t lds = (size_t)64 * (C + 8) * 2 + (size_t)(R + 2) * (W + 2) * 128;
  if (lds > 160 * 1024) { set_error("svk_mixffn_fc1_dwconv: tile too large"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  const long nwg = (long)B * nstrip * (hidden / 64);
  SVK_DISPATCH_H16(dtype, T, {
    auto go = [&](auto ks_c) {
      constexpr int KS = decltype(ks_c)::value;
      if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)fc1_dwconv<T, KS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((fc1_dwconv<T, KS>), dim3((unsigned)nwg), dim3(256), lds, st, (const T*)XN, (const T*)W1, b1,
                         taps, dbias, (T*)G, (T*)Gpre, H, W, C, hidden, R, nstrip, act);
    };
    if (C == 32) go(std::integral_constant<int, 1>{});
    else if (C == 64) go(std::integral_constant<int, 2>{});
    else if (C == 128) go(std::integral_constant<int, 4>{});
    else if (C == 320) go(std::integral_constant<int, 10>{});
    else go(std::integral_constant<int, 16>{});
    return check_launch("fc1_dwconv");
  });
}

extern "C" int svk_mixffn_fc1_dwconv(int dtype, const void* XN, const void* W1, const float* b1, const float* taps,
                                     const float* dbias, void* G, int B, int H, int W, int C, int hidden, int act,
                                     void* stream) {
  return svk_mixffn_fc1_dwconv_ex(dtype, XN, W1, b1, taps, dbias, G, nullptr, B, H, W, C, hidden, act, stream);
}

extern "C" int svk_dwconv3x3(int dtype, const void* X, const float* w, const float* bias, void* Y, int B, int H,
                             int W, int C, int act, void* stream) {
  return svk_dwconv3x3_ex(dtype, X, w, bias, Y, nullptr, B, H, W, C, act, stream);
}

extern "C" int svk_nchw_to_nhwc(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                                void* stream) {
  if (B < 0 || C <= 0 || Cpad < C || H <= 0 || W <= 0 || !X || !Y) { set_error("svk_nchw_to_nhwc: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * H * W;   // one thread per pixel
  if (Cpad == 8 && ((long)H * W) % 4 == 0 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 15) == 0) {
    SVK_DISPATCH_DTYPE(dtype_out, T, {
      hipLaunchKernelGGL((nchw_to_nhwc8_x4_kernel<T>), grid1d(n / 4), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, C,
                         (long)H * W, n / 4);
      return check_launch("nchw_to_nhwc");
    });
  }
  SVK_DISPATCH_DTYPE(dtype_out, T, {
    hipLaunchKernelGGL((nchw_to_nhwc_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, B, C, H, W, Cpad);
    return check_launch("nchw_to_nhwc");
  });
}

// GaussianFilter.conv_gauss written straight into the stem's space-to-depth blocks (4 x 4 pixels, block
// (by, bx) = rows / columns 4*by - pad .., zeros outside the image): one thread per block filters its 16
// pixels from an 8 x 8 reflect-indexed input window per channel, with gauss5x5_x4_kernel's arithmetic
// (horizontal 5-tap sums, then vertical, same order: bitwise equal values).  The handcrafted prompt
// stem then runs as the 2x2 block conv like the frame's stem.
template <typename T>
__global__ __launch_bounds__(256) void gauss5x5_s2d_kernel(const float* __restrict__ X, T* __restrict__ Y, int C, int H,
                                                           int W, int pad, int NBH, int NBW, long nblk) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nblk) return;
  const int bx = (int)(q % NBW);
  const long t = q / NBW;
  const int by = (int)(t % NBH);
  const long b = t / NBH;
  const int py0 = 4 * by - pad, px0 = 4 * bx - pad;        // first output pixel of the block
  const float k1[5] = {1.f / 16.f, 4.f / 16.f, 6.f / 16.f, 4.f / 16.f, 1.f / 16.f};
  int cx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cx[j] = min(max(reflect(min(max(px0 - 2 + j, -2), W + 1), W), 0), W - 1);
  T o[48];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* src = X + ((long)b * C + min(c, C - 1)) * H * W;
    float h[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int yy = min(max(reflect(min(max(py0 - 2 + r, -2), H + 1), H), 0), H - 1);
      const float* row = src + (long)yy * W;
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = row[cx[j]];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) a += w[k + j] * k1[j];
        h[r][k] = a;
      }
    }
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) a += h[dy + i][k] * k1[i];
        const bool ok = c < C && py0 + dy >= 0 && py0 + dy < H && px0 + k >= 0 && px0 + k < W;
        o[(dy * 4 + k) * 3 + c] = from_f<T>(ok ? a : 0.f);
      }
  }
  T* dst = Y + q * 48;
#pragma unroll
  for (int k = 0; k < 6; ++k) store_vec8(dst + 8 * k, o + 8 * k);
}

// The same filter, one 64-lane workgroup per block row: the 8 reflect-mapped input rows of every channel
// are staged in LDS with float4 loads (W % 4 == 0), then each lane filters one block from LDS — the
// per-lane 8-column windows of the direct kernel cost 192 scalar loads per block.  Same arithmetic.
__device__ __forceinline__ void dma16_lds(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <typename T, bool DMA>
__global__ __launch_bounds__(64) void gauss5x5_s2d_lds_kernel(const float* __restrict__ X, T* __restrict__ Y, int C,
                                                              int H, int W, int pad, int NBH, int NBW) {
  extern __shared__ __attribute__((aligned(1024))) float srow[];    // [C][8][W] (+ pad to a 1 KiB multiple)
  const int by = blockIdx.x % NBH;
  const long b = blockIdx.x / NBH;
  const int py0 = 4 * by - pad;
  const int W4 = W >> 2;
  if (DMA) {
    // the 8 reflect-mapped rows x C channels as 16-byte chunks straight into LDS (global_load_lds_dwordx4: lane-
    // linear 1 KiB per instruction), every chunk in flight before one wait — the register-staged loop below
    // waited out one load round trip per iteration (21 per workgroup at 224 x 224)
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)srow;
    const int total = C * 8 * W4;
    for (int e0 = 0; e0 < total; e0 += 64) {
      const int e = min(e0 + (int)threadIdx.x, total - 1);   // tail lanes re-copy the last chunk into the LDS pad
      const int c = e / (8 * W4), r = (e / W4) % 8, x4 = e % W4;
      const int yy = min(max(reflect(min(max(py0 - 2 + r, -2), H + 1), H), 0), H - 1);
      dma16_lds(X + (((long)b * C + c) * H + yy) * W + 4 * x4, __builtin_amdgcn_readfirstlane(lds0 + e0 * 16));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int e = threadIdx.x; e < C * 8 * W4; e += 64) {
      const int c = e / (8 * W4), r = (e / W4) % 8, x4 = e % W4;
      const int yy = min(max(reflect(min(max(py0 - 2 + r, -2), H + 1), H), 0), H - 1);
      reinterpret_cast<float4*>(srow)[(c * 8 + r) * W4 + x4] =
          reinterpret_cast<const float4*>(X + (((long)b * C + c) * H + yy) * W)[x4];
    }
  }
  __syncthreads();
  const int bx = threadIdx.x;
  if (bx >= NBW) return;
  const int px0 = 4 * bx - pad;
  const float k1[5] = {1.f / 16.f, 4.f / 16.f, 6.f / 16.f, 4.f / 16.f, 1.f / 16.f};
  int cx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cx[j] = min(max(reflect(min(max(px0 - 2 + j, -2), W + 1), W), 0), W - 1);
  T o[48];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* src = srow + min(c, C - 1) * 8 * W;
    float h[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = src[r * W + cx[j]];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) a += w[k + j] * k1[j];
        h[r][k] = a;
      }
    }
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) a += h[dy + i][k] * k1[i];
        const bool ok = c < C && py0 + dy >= 0 && py0 + dy < H && px0 + k >= 0 && px0 + k < W;
        o[(dy * 4 + k) * 3 + c] = from_f<T>(ok ? a : 0.f);
      }
  }
  T* dst = Y + ((long)blockIdx.x * NBW + bx) * 48;
#pragma unroll
  for (int k = 0; k < 6; ++k) store_vec8(dst + 8 * k, o + 8 * k);
}

// LDS-staged Gaussian / float4 frame packing for the space-to-depth stems (env SVK_S2D_PACK_VEC=0 = off)
static const bool g_s2d_pack_vec = getenv("SVK_S2D_PACK_VEC") ? atoi(getenv("SVK_S2D_PACK_VEC")) != 0 : true;

extern "C" int svk_gauss5x5_s2d(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int pad, int NBH,
                                int NBW, void* stream) {
  if (B < 0 || C < 1 || C > 3 || H < 3 || W < 3 || NBH <= 0 || NBW <= 0 || pad < 0 || !X || !Y) {
    set_error("svk_gauss5x5_s2d: bad args (1 <= C <= 3)"); return SVK_EINVAL;
  }
  if ((dtype_out != SVK_BF16 && dtype_out != SVK_F16) || ((uintptr_t)Y & 15)) {
    set_error("svk_gauss5x5_s2d: needs bf16 / f16, 16-byte aligned output"); return SVK_EUNSUPPORTED;
  }
  if (B == 0) return SVK_OK;
  const long nblk = (long)B * NBH * NBW;
  const size_t lds = ((size_t)C * 8 * W * sizeof(float) + 1023) / 1024 * 1024;
  static const bool dma = getenv("SVK_GAUSS_DMA") ? atoi(getenv("SVK_GAUSS_DMA")) != 0 : true;
  SVK_DISPATCH_H16(dtype_out, T, {
    if (g_s2d_pack_vec && W % 4 == 0 && NBW <= 64 && ((uintptr_t)X & 15) == 0 && lds <= 65536 &&
        (long)B * NBH < 0x7fffffffL) {
      if (dma)
        hipLaunchKernelGGL((gauss5x5_s2d_lds_kernel<T, true>), dim3((unsigned)(B * NBH)), dim3(64), lds,
                           (hipStream_t)stream, X, (T*)Y, C, H, W, pad, NBH, NBW);
      else
        hipLaunchKernelGGL((gauss5x5_s2d_lds_kernel<T, false>), dim3((unsigned)(B * NBH)), dim3(64), lds,
                           (hipStream_t)stream, X, (T*)Y, C, H, W, pad, NBH, NBW);
      return check_launch("gauss5x5_s2d_lds");
    }
    hipLaunchKernelGGL((gauss5x5_s2d_kernel<T>), grid1d(nblk), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, C, H, W, pad,
                       NBH, NBW, nblk);
    return check_launch("gauss5x5_s2d");
  });
}

// pad = S - 1 = 3 with W % 4 == 0: block columns 4*bx - 3 .. 4*bx straddle two aligned float4 chunks
// (4*bx - 4 .. 4*bx - 1 and 4*bx .. 4*bx + 3), so each (row, channel) costs two 16-byte loads instead of
// four scalar ones (chunk addresses clamped into the row, out-of-image values masked to zero).
template <typename T, int C>
__global__ __launch_bounds__(256) void nchw_to_s2d4_kernel(const float* __restrict__ X, T* __restrict__ Y, int H, int W,
                                                           int NBH, int NBW, long nblk) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nblk) return;
  const int bx = (int)(q % NBW);
  const long t = q / NBW;
  const int by = (int)(t % NBH);
  const long b = t / NBH;
  const float* src = X + b * C * (long)H * W;
  // both chunk addresses clamped into the row: a block column past the image (NBW > W / 4 + 1, e.g. a
  // k = 6 stem) reads in-row bytes whose values are all masked (4 * bx >= W + 4 there, so x >= W + 1)
  const int a0 = min(max(4 * bx - 4, 0), W - 4), a1 = min(4 * bx, W - 4);
  T o[16 * C];
#pragma unroll
  for (int dy = 0; dy < 4; ++dy) {
    const int y = 4 * by - 3 + dy;
    const bool oky = y >= 0 && y < H;
    const int yc = min(max(y, 0), H - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* row = src + ((long)c * H + yc) * W;
      const float4 u = *reinterpret_cast<const float4*>(row + a0);
      const float4 v = *reinterpret_cast<const float4*>(row + a1);
      const float val[4] = {u.y, u.z, u.w, v.x};
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        const int x = 4 * bx - 3 + dx;
        o[(dy * 4 + dx) * C + c] = from_f<T>(oky && x >= 0 && x < W ? val[dx] : 0.f);
      }
    }
  }
  T* dst = Y + q * 16 * C;
#pragma unroll
  for (int k = 0; k < 2 * C; ++k) store_vec8(dst + 8 * k, o + 8 * k);
}

extern "C" int svk_nchw_to_s2d(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int s, int pad,
                               int NBH, int NBW, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || NBH <= 0 || NBW <= 0 || pad < 0 || !X || !Y) {
    set_error("svk_nchw_to_s2d: bad args"); return SVK_EINVAL;
  }
  if (s != 4 || (C != 2 && C != 3) || (dtype_out != SVK_BF16 && dtype_out != SVK_F16) || ((uintptr_t)Y & 15)) {
    set_error("svk_nchw_to_s2d: needs s = 4, C in {2, 3}, bf16 / f16, 16-byte aligned output"); return SVK_EUNSUPPORTED;
  }
  if (B == 0) return SVK_OK;
  const long nblk = (long)B * NBH * NBW;
  SVK_DISPATCH_H16(dtype_out, T, {
    if (g_s2d_pack_vec && pad == 3 && W % 4 == 0 && W >= 4 && ((uintptr_t)X & 15) == 0) {
      if (C == 3)
        hipLaunchKernelGGL((nchw_to_s2d4_kernel<T, 3>), grid1d(nblk), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, H, W,
                           NBH, NBW, nblk);
      else
        hipLaunchKernelGGL((nchw_to_s2d4_kernel<T, 2>), grid1d(nblk), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, H, W,
                           NBH, NBW, nblk);
      return check_launch("nchw_to_s2d4");
    }
    if (C == 3)
      hipLaunchKernelGGL((nchw_to_s2d_kernel<T, 4, 3>), grid1d(nblk), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, H, W,
                         pad, NBH, NBW, nblk);
    else
      hipLaunchKernelGGL((nchw_to_s2d_kernel<T, 4, 2>), grid1d(nblk), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, H, W,
                         pad, NBH, NBW, nblk);
    return check_launch("nchw_to_s2d");
  });
}

extern "C" int svk_gauss5x5_reflect(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                                    void* stream) {
  if (B < 0 || C <= 0 || C > 8 || Cpad < C || H < 3 || W < 3 || !X || !Y) {
    set_error("svk_gauss5x5_reflect: bad args (1 <= C <= 8)"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  const int nstrip = (H + GR - 1) / GR;
  const long n = (long)B * nstrip * W;   // one thread per (column, strip of GR rows)
  if (W % 4 == 0 && W >= 8 && C <= 3 && Cpad == 8 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 15) == 0) {
    // rows per thread: 4 measured 169 us vs 179 (8) and 269 (16) at B = 256 (tools/pack_bench.py)
    static const int gr = getenv("SVK_GAUSS_GR") ? atoi(getenv("SVK_GAUSS_GR")) : 4;
    SVK_DISPATCH_DTYPE(dtype_out, T, {
      auto go = [&](auto g) {
        constexpr int G = decltype(g)::value;
        const int ns = (H + G - 1) / G;
        hipLaunchKernelGGL((gauss5x5_x4_kernel<T, G>), grid1d((long)B * ns * W / 4), dim3(256), 0, (hipStream_t)stream, X,
                           (T*)Y, B, C, H, W, ns);
      };
      if (gr == 4) go(std::integral_constant<int, 4>{});
      else if (gr == 16) go(std::integral_constant<int, 16>{});
      else go(std::integral_constant<int, 8>{});
      return check_launch("gauss5x5_reflect");
    });
  }
  SVK_DISPATCH_DTYPE(dtype_out, T, {
    if (C <= 3)
      hipLaunchKernelGGL((gauss5x5_kernel<T, 3>), grid1d(n), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, B, C, H, W,
                         Cpad, nstrip);
    else
      hipLaunchKernelGGL((gauss5x5_kernel<T, 8>), grid1d(n), dim3(256), 0, (hipStream_t)stream, X, (T*)Y, B, C, H, W,
                         Cpad, nstrip);
    return check_launch("gauss5x5_reflect");
  });
}

extern "C" int svk_resize_bilinear(int dtype, const void* X, long ldx, void* Y, long ldy, int B, int H, int W, int C,
                                   int OH, int OW, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0 || !X || !Y || ldx < C || ldy < C) {
    set_error("svk_resize_bilinear: bad args"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  const long n = (long)B * OH * OW * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((resize_bilinear_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, ldx, (T*)Y,
                       ldy, B, H, W, C, OH, OW);
    return check_launch("resize_bilinear");
  });
}

extern "C" int svk_resize_bilinear_multi(int dtype, int nl, const void* const* X, const long* ldx, const int* H,
                                         const int* W, const int* C, void* Y, long ldy, int B, int OH, int OW,
                                         void* stream) {
  if (nl < 1 || nl > 4 || B < 0 || OH <= 0 || OW <= 0 || !X || !ldx || !H || !W || !C || !Y ||
      (dtype != SVK_F16 && dtype != SVK_BF16)) {
    set_error("svk_resize_bilinear_multi: bad args (1-4 levels, 16-bit)"); return SVK_EINVAL;
  }
  RsLevels L{};
  L.coff[0] = 0;
  for (int l = 0; l < nl; ++l) {
    if (!X[l] || H[l] <= 0 || W[l] <= 0 || C[l] <= 0 || C[l] % 8 || ldx[l] < C[l] || ldx[l] % 8 ||
        ((uintptr_t)X[l] & 15)) {
      set_error("svk_resize_bilinear_multi: level %d needs C %% 8 == 0, ldx %% 8 == 0, 16-byte aligned", l);
      return SVK_EINVAL;
    }
    L.X[l] = X[l]; L.ldx[l] = ldx[l]; L.H[l] = H[l]; L.W[l] = W[l];
    L.coff[l + 1] = L.coff[l] + C[l];
  }
  if (ldy < L.coff[nl] || ldy % 8 || ((uintptr_t)Y & 15)) {
    set_error("svk_resize_bilinear_multi: ldy must cover the levels' channels, ldy %% 8 == 0, Y 16-byte aligned");
    return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  const long n = (long)B * OH * OW * (L.coff[nl] / 8);
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((resize_multi_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, L, nl, (T*)Y, ldy, B,
                       OH, OW);
    return check_launch("resize_bilinear_multi");
  });
}

extern "C" int svk_window_unfold(int dtype, const void* X, long ldx, const float* pos, void* Y, int Tn, int C, int len,
                                 void* stream) {
  if (Tn < 0 || C <= 0 || len <= 0 || !X || !Y || ldx < C) { set_error("svk_window_unfold: bad args"); return SVK_EINVAL; }
  if (Tn == 0) return SVK_OK;
  const long n = (long)Tn * len * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((window_unfold_kernel<T>), grid1d(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, ldx, pos,
                       (T*)Y, Tn, C, len);
    return check_launch("window_unfold");
  });
}

extern "C" int svk_add_bcast(int dtype, const void* X, const float* P, void* Y, long M, int C, int period,
                             void* stream) {
  if (M < 0 || C <= 0 || period <= 0 || !X || !P || !Y) { set_error("svk_add_bcast: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((add_bcast_kernel<T>), grid1d(M * C), dim3(256), 0, (hipStream_t)stream, (const T*)X, P, (T*)Y,
                       M, C, period);
    return check_launch("add_bcast");
  });
}

extern "C" int svk_cast(int dtype_in, const void* X, int dtype_out, void* Y, long n, void* stream) {
  if (n < 0 || !X || !Y) { set_error("svk_cast: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype_in, TI, {
    SVK_DISPATCH_DTYPE(dtype_out, TO, {
      hipLaunchKernelGGL((cast_kernel<TI, TO>), grid1d(n), dim3(256), 0, st, (const TI*)X, (TO*)Y, n);
      return check_launch("cast");
    });
  });
}
