// Frame preprocessing on the GPU: the extraction/eval transform of
// generate_evp_LFB.py:243-247 — transforms.Resize((250, 250)) on the decoded PIL RGB frame, CenterCrop(224),
// ToTensor, Normalize(mean, std) — applied to a batch of decoded uint8 HWC frames (and, identically, to the
// RGB segmaps: CholecFlowDataset applies the same transform to both, data_process.py:455-462).
//
// Resize is Pillow's separable antialiased bilinear resampling for 8-bit images, bit-exact: per output
// coordinate a window [xmin, xmin + n) with fixed-point coefficients (22 fractional bits) that the host
// computes exactly as Pillow does (svk/preproc.py); horizontal pass first, rounded (+2^21) and clipped to
// uint8, then the vertical pass over the horizontal result, rounded and clipped again.  Only the 224x224
// window CenterCrop keeps is produced: the horizontal pass runs for the kept columns, the vertical pass for
// the kept rows.  ToTensor + Normalize are the same f32 operations torch performs (u8 / 255, then
// (v - mean) / std), with correctly-rounded divisions, so the output equals the DataLoader's tensor.
//
// Layout: frames [B, H, W, 3] uint8 (decoder output, row-major HWC); tmp [B, H, CW, 3] uint8 (horizontal
// result, caller-owned workspace); out [B, 3, CH, CW] f32 (the DataLoader's NCHW tensor).
#include "svk_common.h"

namespace svk {

constexpr int PP_PREC = 22;

__device__ __forceinline__ int pp_clip8(int ss) {
  const int v = ss >> PP_PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Horizontal pass: a workgroup owns PP_ROWS consecutive input rows of one frame — one contiguous byte range
// of the HWC frame — and stages it in LDS with 16-byte loads (the range start aligned down to 16 bytes),
// then every thread produces kept columns of those rows from LDS (taps of neighbouring output columns
// overlap, so each input byte is read from HBM once).  Rows beyond H (last block) are skipped.
constexpr int PP_ROWS = 4;     // sweep (B = 256, 480x854): 2 rows 893k, 4 rows 978k, 8 rows 941k frames/s

__global__ __launch_bounds__(256) void pp_resize_h(const uint8_t* __restrict__ in, uint8_t* __restrict__ tmp,
                                                   const int* __restrict__ xb, const int* __restrict__ xk, int ksx,
                                                   int B, int H, int W, int CW, int cx0, const int* __restrict__ prm,
                                                   int pstride) {
  extern __shared__ uint4 pp_lds[];
  uint8_t* rows = reinterpret_cast<uint8_t*>(pp_lds);
  const int blocks_per_frame = (H + PP_ROWS - 1) / PP_ROWS;
  const int b = blockIdx.x / blocks_per_frame;
  const int y0 = (blockIdx.x - b * blocks_per_frame) * PP_ROWS;
  if (prm) cx0 = prm[b * pstride];                             // training: the sample's RandomCrop column offset
  const int nr = min(PP_ROWS, H - y0);
  const long rowbytes = (long)W * 3;
  const long start = ((long)b * H + y0) * rowbytes;
  const long astart = start & ~15L;
  const int lead = (int)(start - astart);
  const long total_bytes = (long)B * H * rowbytes;
  const int nbytes = lead + (int)(nr * rowbytes);
  const int nvec = (nbytes + 15) >> 4;
  const uint4* src = reinterpret_cast<const uint4*>(in + astart);
  const long nvec_full = (total_bytes - astart) >> 4;          // whole 16-byte vectors inside the frames buffer
  for (int v = threadIdx.x; v < nvec; v += 256) {
    if (v < nvec_full) {
      pp_lds[v] = src[v];
    } else {                                                   // the buffer's ragged tail: byte loads
      uint8_t* d = rows + 16 * v;
      for (int q = 0; q < 16; ++q) d[q] = astart + 16L * v + q < total_bytes ? in[astart + 16L * v + q] : 0;
    }
  }
  __syncthreads();
  // thread -> (row, 4 consecutive kept columns): 12 output bytes written as three 4-byte stores
  const int CG = CW >> 2;                                      // CW % 4 == 0 (checked by the launcher)
  for (int e = threadIdx.x; e < nr * CG; e += 256) {
    const int r = e / CG, ox = (e - r * CG) * 4;
    int acc[12];
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int x = cx0 + ox + px;
      const int xmin = xb[2 * x], n = xb[2 * x + 1];
      const int* k = xk + (long)x * ksx;
      const uint8_t* p = rows + lead + r * rowbytes + xmin * 3;
      int s0 = 1 << (PP_PREC - 1), s1 = s0, s2 = s0;
      for (int j = 0; j < n; ++j) {
        const int c = k[j];
        s0 += p[3 * j] * c;
        s1 += p[3 * j + 1] * c;
        s2 += p[3 * j + 2] * c;
      }
      acc[3 * px] = pp_clip8(s0);
      acc[3 * px + 1] = pp_clip8(s1);
      acc[3 * px + 2] = pp_clip8(s2);
    }
    uint32_t* dst = reinterpret_cast<uint32_t*>(tmp + ((((long)b * H + y0 + r) * CW) + ox) * 3);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      dst[q] = (uint32_t)acc[4 * q] | ((uint32_t)acc[4 * q + 1] << 8) | ((uint32_t)acc[4 * q + 2] << 16) |
               ((uint32_t)acc[4 * q + 3] << 24);
  }
}

// one thread per (b, kept row, 4 kept columns): vertical taps over tmp with 3 x 4-byte loads per tap (the 4
// pixels' 12 bytes), then ToTensor + Normalize per channel and one 16-byte store per plane.  Needs CW % 4 == 0
// and 4/16-byte aligned buffers (otherwise the launcher picks PX = 1, one column per thread).
template <int PX>
__global__ __launch_bounds__(256) void pp_resize_v_norm(const uint8_t* __restrict__ tmp, float* __restrict__ out,
                                                        const int* __restrict__ yb, const int* __restrict__ yk,
                                                        int ksy, int B, int H, int CH, int CW, int cy0, float m0,
                                                        float m1, float m2, float s0d, float s1d, float s2d) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int CG = CW / PX;
  const long total = (long)B * CH * CG;
  if (i >= total) return;
  const int ox = (int)(i % CG) * PX;
  const long r = i / CG;
  const int oy = (int)(r % CH);
  const int b = (int)(r / CH);
  const int y = cy0 + oy;
  const int ymin = yb[2 * y], n = yb[2 * y + 1];
  const int* k = yk + (long)y * ksy;
  const uint8_t* src = tmp + (((long)b * H + ymin) * CW + ox) * 3;
  int acc[3 * PX];
#pragma unroll
  for (int q = 0; q < 3 * PX; ++q) acc[q] = 1 << (PP_PREC - 1);
  for (int j = 0; j < n; ++j) {
    const int c = k[j];
    const uint8_t* p = src + (long)j * CW * 3;
    if (PX == 4) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const uint32_t v = w[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[4 * q + e] += (int)((v >> (8 * e)) & 0xff) * c;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 3 * PX; ++q) acc[q] += p[q] * c;
    }
  }
  const long plane = (long)CH * CW;
  float* o = out + (long)b * 3 * plane + (long)oy * CW + ox;
  const float mm[3] = {m0, m1, m2}, ss[3] = {s0d, s1d, s2d};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float v[PX];
#pragma unroll
    for (int px = 0; px < PX; ++px)                 // acc index = pixel * 3 + channel (HWC bytes)
      v[px] = __fdiv_rn(__fdiv_rn((float)pp_clip8(acc[3 * px + ch]), 255.f) - mm[ch], ss[ch]);
    if (PX == 4) *reinterpret_cast<float4*>(o + ch * plane) = make_float4(v[0], v[1], v[2], v[3]);
    else o[ch * plane] = v[0];
  }
}

// Optical-flow transform (CholecFlowDataset, data_process.py:425-447 + the CenterCrop of the transform):
// cv2.resize(flow, (OW, OH), INTER_LINEAR) on the float32 [H, W, 2] .npy field, u *= OW / W, v *= OH / H,
// then CenterCrop.  cv2's float INTER_LINEAR: per output column a source index sx and weights (1 - fx, fx)
// from fx = (float)((dx + 0.5) * scale - 0.5) with edge clamping (host tables, svk/preproc.py); the
// horizontal pass forms each needed source row's value, the vertical pass blends two rows, as separate
// f32 multiplies and adds (this file is compiled with -ffp-contract=off) like OpenCV's scalar path.
__global__ __launch_bounds__(256) void pp_flow(const float* __restrict__ in, float* __restrict__ out,
                                               const int* __restrict__ xo, const float* __restrict__ xa,
                                               const int* __restrict__ yo, const float* __restrict__ ya, int B, int H,
                                               int W, int CH, int CW, int cy0, int cx0, float su, float sv) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * CH * CW;
  if (i >= total) return;
  const int ox = (int)(i % CW);
  const long r = i / CW;
  const int oy = (int)(r % CH);
  const int b = (int)(r / CH);
  const int x = cx0 + ox, y = cy0 + oy;
  const int sx = xo[x], sy = yo[y];
  const int sx1 = min(sx + 1, W - 1), sy1 = min(sy + 1, H - 1);
  const float a0 = xa[2 * x], a1 = xa[2 * x + 1], b0 = ya[2 * y], b1 = ya[2 * y + 1];
  const float2* f = reinterpret_cast<const float2*>(in) + (long)b * H * W;
  const float2 p00 = f[(long)sy * W + sx], p01 = f[(long)sy * W + sx1];
  const float2 p10 = f[(long)sy1 * W + sx], p11 = f[(long)sy1 * W + sx1];
  const float h0u = __fadd_rn(__fmul_rn(p00.x, a0), __fmul_rn(p01.x, a1));
  const float h0v = __fadd_rn(__fmul_rn(p00.y, a0), __fmul_rn(p01.y, a1));
  const float h1u = __fadd_rn(__fmul_rn(p10.x, a0), __fmul_rn(p11.x, a1));
  const float h1v = __fadd_rn(__fmul_rn(p10.y, a0), __fmul_rn(p11.y, a1));
  const float u = __fadd_rn(__fmul_rn(h0u, b0), __fmul_rn(h1u, b1));
  const float v = __fadd_rn(__fmul_rn(h0v, b0), __fmul_rn(h1v, b1));
  const long plane = (long)CH * CW;
  float* o = out + (long)b * 2 * plane + (long)oy * CW + ox;
  o[0] = __fmul_rn(u, su);
  o[plane] = __fmul_rn(v, sv);
}

void pp_resize_h_launch(const uint8_t* in, uint8_t* tmp, const int* xb, const int* xk, int ksx, int B, int H, int W,
                        int CW, int cx0, const int* prm, int pstride, hipStream_t s) {
  const long lds = ((16 + (long)PP_ROWS * W * 3 + 15) / 16) * 16;
  const int bpf = (H + PP_ROWS - 1) / PP_ROWS;
  hipLaunchKernelGGL(pp_resize_h, dim3((unsigned)((long)B * bpf)), dim3(256), (size_t)lds, s, in, tmp, xb, xk, ksx, B, H,
                     W, CW, cx0, prm, pstride);
}

}  // namespace svk

using namespace svk;

extern "C" int svk_frame_preproc(const void* frames, void* tmp, float* out, const int* xbounds, const int* xcoef,
                                 int ksx, const int* ybounds, const int* ycoef, int ksy, int B, int H, int W,
                                 int crop_y0, int crop_x0, int CH, int CW, const float* mean, const float* std,
                                 void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || CH <= 0 || CW <= 0 || crop_y0 < 0 || crop_x0 < 0 || ksx <= 0 || ksy <= 0 ||
      !frames || !tmp || !out || !xbounds || !xcoef || !ybounds || !ycoef || !mean || !std) {
    set_error("svk_frame_preproc: bad args (B=%d H=%d W=%d crop %dx%d at (%d, %d))", B, H, W, CH, CW, crop_y0,
              crop_x0);
    return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  hipStream_t s = (hipStream_t)stream;
  const long tv = (long)B * CH * CW;
  if (CW % 4 != 0 || ((uintptr_t)tmp & 3)) {
    set_error("svk_frame_preproc: crop width %d must be a multiple of 4 (4-byte aligned scratch)", CW);
    return SVK_EUNSUPPORTED;
  }
  const long lds = ((16 + (long)PP_ROWS * W * 3 + 15) / 16) * 16;
  if (lds > 64 * 1024) { set_error("svk_frame_preproc: frame width %d too large (W*3*%d > 64 KiB)", W, PP_ROWS); return SVK_EUNSUPPORTED; }
  pp_resize_h_launch((const uint8_t*)frames, (uint8_t*)tmp, xbounds, xcoef, ksx, B, H, W, CW, crop_x0, nullptr, 0, s);
  const bool vec = CW % 4 == 0 && ((uintptr_t)tmp & 3) == 0 && ((uintptr_t)out & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((pp_resize_v_norm<4>), dim3((unsigned)((tv / 4 + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t*)tmp, out, ybounds, ycoef, ksy, B, H, CH, CW, crop_y0, mean[0], mean[1], mean[2],
                       std[0], std[1], std[2]);
  else
    hipLaunchKernelGGL((pp_resize_v_norm<1>), dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t*)tmp, out, ybounds, ycoef, ksy, B, H, CH, CW, crop_y0, mean[0], mean[1], mean[2],
                       std[0], std[1], std[2]);
  return check_launch("frame_preproc");
}

extern "C" int svk_flow_preproc(const float* flow, float* out, const int* xofs, const float* xalpha, const int* yofs,
                                const float* yalpha, int B, int H, int W, int crop_y0, int crop_x0, int CH, int CW,
                                float scale_u, float scale_v, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || CH <= 0 || CW <= 0 || crop_y0 < 0 || crop_x0 < 0 || !flow || !out || !xofs ||
      !xalpha || !yofs || !yalpha || ((uintptr_t)flow & 7)) {
    set_error("svk_flow_preproc: bad args (B=%d H=%d W=%d, flow 8-byte aligned)", B, H, W);
    return SVK_EINVAL;
  }
  const long tv = (long)B * CH * CW;
  if (tv == 0) return SVK_OK;
  hipLaunchKernelGGL(pp_flow, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, (hipStream_t)stream, flow, out, xofs,
                     xalpha, yofs, yalpha, B, H, W, CH, CW, crop_y0, crop_x0, scale_u, scale_v);
  return check_launch("flow_preproc");
}
