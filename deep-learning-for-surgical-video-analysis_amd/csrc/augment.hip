// Training-time augmentations on the GPU: train_evp.py:146-163's
//
//   Resize((250, 250)) -> RandomCrop(224) -> [ColorJitter(0.1, 0.1, 0.1, 0.05)] -> RandomHorizontalFlip()
//   -> [RandomRotation(5)] -> ToTensor() -> Normalize(mean, std)
//
// on decoded uint8 RGB frames and segmaps (the synced classes of data_process.py:53-186 — one parameter draw
// per sample and image, made on the host by the drop-in classes), and the geometric part on the RAFT flow
// (CholecFlowDataset, data_process.py:425-487).  Bit-exact to Pillow 12.2.0 for the images (oracle/augment.py
// restates each Pillow routine and tests/test_augment_cpu.py pins it against Pillow itself); this file is
// compiled with -ffp-contract=off so every float / double operation rounds where Pillow's C code rounds.
//
//  1. Resize + crop: Pillow's separable 8-bit bilinear (preproc.hip's horizontal pass, per-sample crop
//     column offset) and a vertical pass that writes the 224 x 224 uint8 crop at the sample's row offset.
//  2. aug_luma_sum: one workgroup per image: sum of L(brightness(pixel)) over the crop — ImageEnhance.Contrast's
//     degenerate grey is int(mean + 0.5) of the brightness-adjusted image.
//  3. aug_finish: per output pixel: the rotation's 16.16 fixed-point source (Image.rotate's inverse matrix,
//     ImagingTransformAffine's nearest path), the flip, the crop pixel, then brightness / contrast / colour
//     blends (Image.blend: float multiply + add, truncation), the HSV hue shift (Pillow's rgb2hsv / hsv2rgb with
//     their double promotions), ToTensor (/255) and Normalize — colour ops commute with the gather because they
//     are per pixel given the image mean.  Output NCHW f32, 4 pixels per thread, 16-byte stores per plane.
//  4. aug_flow: per output pixel of the flow crop: the tensor rotation's nearest grid sample (torchvision's
//     affine grid formed in f32, grid_sample's align_corners=False unnormalisation, round-half-even), the flip
//     (u negated), the crop offset, cv2's INTER_LINEAR value of the raw field (preproc.hip's tables) times the
//     displacement scale, then the vector rotation.
#include "svk_common.h"

namespace svk {

constexpr int AUG_PREC = 22;
constexpr int AUG_NP = 16;   // int32 parameters per sample (see svk.h)

__device__ __forceinline__ int aug_clip8(int ss) {
  int v = ss >> AUG_PREC;
  v = v < 0 ? 0 : (v > 255 ? 255 : v);
  // keep hipcc 7.2 from fusing two (shift, clamp, pack) chains into v_ashr_pk_u8_i32: its lowering assumes
  // the instruction zeroes bits 31:16 of the destination, the hardware keeps them (bytes 6 and 10 of each
  // 12-byte group came out OR-ed with a neighbour); isa_check.py rejects the instruction in every object
  asm volatile("" : "+v"(v));
  return v;
}

// vertical Pillow pass over the horizontal result tmp [B, H, CW, 3] (CW = crop width, columns already at the
// sample's crop offset) for crop rows y1 .. y1 + CH - 1: uint8 crop [B, CH, CW, 3], 4 pixels per thread
__global__ __launch_bounds__(256) void aug_resize_v_u8(const uint8_t* __restrict__ tmp, uint8_t* __restrict__ crop,
                                                       const int* __restrict__ yb, const int* __restrict__ yk, int ksy,
                                                       const int* __restrict__ prm, int B, int H, int CH, int CW) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int CG = CW / 4;
  const long total = (long)B * CH * CG;
  if (i >= total) return;
  const int ox = (int)(i % CG) * 4;
  const long r = i / CG;
  const int oy = (int)(r % CH);
  const int b = (int)(r / CH);
  const int y = prm[b * AUG_NP + 1] + oy;
  const int ymin = yb[2 * y], n = yb[2 * y + 1];
  const int* k = yk + (long)y * ksy;
  const uint8_t* src = tmp + (((long)b * H + ymin) * CW + ox) * 3;
  int acc[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) acc[q] = 1 << (AUG_PREC - 1);
  for (int j = 0; j < n; ++j) {
    const int c = k[j];
    const uint32_t* w = reinterpret_cast<const uint32_t*>(src + (long)j * CW * 3);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t v = w[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4 * q + e] += (int)((v >> (8 * e)) & 0xff) * c;
    }
  }
  uint32_t* dst = reinterpret_cast<uint32_t*>(crop + (((long)b * CH + oy) * CW + ox) * 3);
#pragma unroll
  for (int q = 0; q < 3; ++q)
    dst[q] = (uint32_t)aug_clip8(acc[4 * q]) | ((uint32_t)aug_clip8(acc[4 * q + 1]) << 8) |
             ((uint32_t)aug_clip8(acc[4 * q + 2]) << 16) | ((uint32_t)aug_clip8(acc[4 * q + 3]) << 24);
}

// Image.blend(in1, in2, alpha) of one byte: float arithmetic, truncation (interpolation) or clip + truncation
__device__ __forceinline__ int pil_blend(int in1, int in2, float alpha) {
  const float t = __fadd_rn((float)in1, __fmul_rn(alpha, (float)(in2 - in1)));
  if (alpha >= 0.f && alpha <= 1.f) return (int)t;
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)t);
}
__device__ __forceinline__ int pil_luma(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

// Pillow Convert.c rgb2hsv_row / hsv2rgb (float variables, double literals)
__device__ __forceinline__ void pil_rgb2hsv(int r, int g, int b, int& uh, int& us, int& uv) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  uv = maxc;
  if (minc == maxc) { uh = 0; us = 0; return; }
  const float cr = (float)(maxc - minc);
  const float s = __fdiv_rn(cr, (float)maxc);
  const float rc = __fdiv_rn((float)(maxc - r), cr), gc = __fdiv_rn((float)(maxc - g), cr),
              bc = __fdiv_rn((float)(maxc - b), cr);
  float h;
  if (r == maxc) h = __fsub_rn(bc, gc);
  else if (g == maxc) h = (float)__dsub_rn(__dadd_rn(2.0, (double)rc), (double)bc);
  else h = (float)__dsub_rn(__dadd_rn(4.0, (double)gc), (double)rc);
  h = (float)fmod(__dadd_rn(__ddiv_rn((double)h, 6.0), 1.0), 1.0);
  const int ih = (int)__dmul_rn((double)h, 255.0), is = (int)__dmul_rn((double)s, 255.0);
  uh = ih < 0 ? 0 : (ih > 255 ? 255 : ih);
  us = is < 0 ? 0 : (is > 255 ? 255 : is);
}
__device__ __forceinline__ int pil_round_clip(double x) {   // C round() of a non-negative value, CLIP8
  const int v = (int)floor(__dadd_rn(x, 0.5));
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}
__device__ __forceinline__ void pil_hsv2rgb(int h, int s, int v, int& r, int& g, int& b) {
  if (s == 0) { r = g = b = v; return; }
  const double hd = __ddiv_rn(__dmul_rn((double)(float)h, 6.0), 255.0);
  const int i = (int)floor(hd);
  const float f = (float)__dsub_rn(hd, (double)(float)i);
  const float fs = (float)__ddiv_rn((double)(float)s, 255.0);
  const double vf = (double)(float)v;
  const int p = pil_round_clip(__dmul_rn(vf, __dsub_rn(1.0, (double)fs)));
  const int q = pil_round_clip(__dmul_rn(vf, __dsub_rn(1.0, __dmul_rn((double)fs, (double)f))));
  const int t = pil_round_clip(__dmul_rn(vf, __dsub_rn(1.0, __dmul_rn((double)fs, __dsub_rn(1.0, (double)f)))));
  switch (i % 6) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// per image: sum over the crop of L(brightness-blended pixel) (ImageEnhance.Contrast's mean); one workgroup
__global__ __launch_bounds__(1024) void aug_luma_sum(const uint8_t* __restrict__ crop, const int* __restrict__ prm,
                                                     long long* __restrict__ sums, int npix) {
  const int b = blockIdx.x;
  const int* P = prm + b * AUG_NP;
  const float bright = __int_as_float(P[11]);
  const uint8_t* src = crop + (long)b * npix * 3;
  long long s = 0;
  if (P[10]) {
    for (int i = threadIdx.x; i < npix; i += 1024) {
      const int r = pil_blend(0, src[3 * i], bright), g = pil_blend(0, src[3 * i + 1], bright),
                bb = pil_blend(0, src[3 * i + 2], bright);
      s += pil_luma(r, g, bb);
    }
  }
  __shared__ long long red[16];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < 16; ++w) t += red[w];
    sums[b] = t;
  }
}

// colour jitter of one pixel (brightness, contrast about `mean`, colour, hue shift)
__device__ __forceinline__ void jitter_px(int& r, int& g, int& b, float fb, float fc, float fs, int mean, int hshift) {
  r = pil_blend(0, r, fb); g = pil_blend(0, g, fb); b = pil_blend(0, b, fb);
  r = pil_blend(mean, r, fc); g = pil_blend(mean, g, fc); b = pil_blend(mean, b, fc);
  const int L = pil_luma(r, g, b);
  r = pil_blend(L, r, fs); g = pil_blend(L, g, fs); b = pil_blend(L, b, fs);
  int h, s, v;
  pil_rgb2hsv(r, g, b, h, s, v);
  pil_hsv2rgb((h + hshift) & 255, s, v, r, g, b);
}

// output pixel (x, y) of the 224 x 224 result: rotation source (fixed point) in the flipped crop, flip, fetch,
// jitter, normalise.  One thread per 4 pixels of a row; NCHW f32 out.
__global__ __launch_bounds__(256) void aug_finish(const uint8_t* __restrict__ crop, const int* __restrict__ prm,
                                                  const long long* __restrict__ sums, float* __restrict__ out, int B,
                                                  int CH, int CW, float m0, float m1, float m2, float s0, float s1,
                                                  float s2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int CG = CW / 4;
  const long total = (long)B * CH * CG;
  if (i >= total) return;
  const int ox = (int)(i % CG) * 4;
  const long rr = i / CG;
  const int oy = (int)(rr % CH);
  const int b = (int)(rr / CH);
  const int* P = prm + b * AUG_NP;
  const bool flip = P[2] != 0, rot = P[3] != 0, jit = P[10] != 0;
  const float fb = __int_as_float(P[11]), fc = __int_as_float(P[12]), fsat = __int_as_float(P[13]);
  const int hshift = P[14];
  // ImageStat's mean: sum / count in double, int(mean + 0.5)
  const int mean = jit ? (int)__dadd_rn(__ddiv_rn((double)sums[b], (double)(CH * CW)), 0.5) : 0;
  const uint8_t* src = crop + (long)b * CH * CW * 3;
  float v[3][4];
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    const int x = ox + px;
    int sx = x, sy = oy;
    bool ok = true;
    if (rot) {
      sx = (P[6] + P[5] * oy + P[4] * x) >> 16;
      sy = (P[9] + P[8] * oy + P[7] * x) >> 16;
      ok = sx >= 0 && sx < CW && sy >= 0 && sy < CH;
    }
    if (flip) sx = CW - 1 - sx;
    int r = 0, g = 0, bb = 0;
    if (ok) {
      const uint8_t* p = src + ((long)sy * CW + sx) * 3;
      r = p[0]; g = p[1]; bb = p[2];
      if (jit) jitter_px(r, g, bb, fb, fc, fsat, mean, hshift);
    }
    v[0][px] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)r, 255.f), m0), s0);
    v[1][px] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)g, 255.f), m1), s1);
    v[2][px] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)bb, 255.f), m2), s2);
  }
  const long plane = (long)CH * CW;
  float* o = out + (long)b * 3 * plane + (long)oy * CW + ox;
#pragma unroll
  for (int c = 0; c < 3; ++c) *reinterpret_cast<float4*>(o + c * plane) = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
}

// flow: [B, H, W, 2] f32 raw field -> [B, 2, CH, CW]; parameters: x1, y1, flip, rot, t00 t01 t02 t10 t11 t12
// (f32 bits, the rescaled inverse rotation of the affine grid), cos, sin (f32 bits) of the vector rotation
__global__ __launch_bounds__(256) void aug_flow(const float* __restrict__ in, float* __restrict__ out,
                                                const int* __restrict__ xo, const float* __restrict__ xa,
                                                const int* __restrict__ yo, const float* __restrict__ ya,
                                                const int* __restrict__ prm, int B, int H, int W, int CH, int CW,
                                                float su, float sv) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * CH * CW;
  if (i >= total) return;
  const int x = (int)(i % CW);
  const long rr = i / CW;
  const int y = (int)(rr % CH);
  const int b = (int)(rr / CH);
  const int* P = prm + b * AUG_NP;
  const bool flip = P[2] != 0, rot = P[3] != 0;
  int sx = x, sy = y;
  bool ok = true;
  if (rot) {
    const float xb = __fadd_rn(__fsub_rn((float)x, (float)CW * 0.5f), 0.5f);
    const float yb = __fadd_rn(__fsub_rn((float)y, (float)CH * 0.5f), 0.5f);
    const float gx = __fadd_rn(__fadd_rn(__fmul_rn(xb, __int_as_float(P[4])), __fmul_rn(yb, __int_as_float(P[5]))),
                               __int_as_float(P[6]));
    const float gy = __fadd_rn(__fadd_rn(__fmul_rn(xb, __int_as_float(P[7])), __fmul_rn(yb, __int_as_float(P[8]))),
                               __int_as_float(P[9]));
    sx = (int)rintf(__fdiv_rn(__fsub_rn(__fmul_rn(__fadd_rn(gx, 1.f), (float)CW), 1.f), 2.f));
    sy = (int)rintf(__fdiv_rn(__fsub_rn(__fmul_rn(__fadd_rn(gy, 1.f), (float)CH), 1.f), 2.f));
    ok = sx >= 0 && sx < CW && sy >= 0 && sy < CH;
  }
  float u = 0.f, v = 0.f;
  if (ok) {
    if (flip) sx = CW - 1 - sx;
    const int X = P[0] + sx, Y = P[1] + sy;        // in the 250 x 250 resized field
    const int x0 = xo[X], y0 = yo[Y];
    const int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
    const float a0 = xa[2 * X], a1 = xa[2 * X + 1], b0 = ya[2 * Y], b1 = ya[2 * Y + 1];
    const float2* f = reinterpret_cast<const float2*>(in) + (long)b * H * W;
    const float2 p00 = f[(long)y0 * W + x0], p01 = f[(long)y0 * W + x1];
    const float2 p10 = f[(long)y1 * W + x0], p11 = f[(long)y1 * W + x1];
    const float h0u = __fadd_rn(__fmul_rn(p00.x, a0), __fmul_rn(p01.x, a1));
    const float h0v = __fadd_rn(__fmul_rn(p00.y, a0), __fmul_rn(p01.y, a1));
    const float h1u = __fadd_rn(__fmul_rn(p10.x, a0), __fmul_rn(p11.x, a1));
    const float h1v = __fadd_rn(__fmul_rn(p10.y, a0), __fmul_rn(p11.y, a1));
    u = __fmul_rn(__fadd_rn(__fmul_rn(h0u, b0), __fmul_rn(h1u, b1)), su);
    v = __fmul_rn(__fadd_rn(__fmul_rn(h0v, b0), __fmul_rn(h1v, b1)), sv);
    if (flip) u = -u;
  }
  if (rot) {
    const float ca = __int_as_float(P[10]), sa = __int_as_float(P[11]);
    const float nu = __fsub_rn(__fmul_rn(u, ca), __fmul_rn(v, sa));
    const float nv = __fadd_rn(__fmul_rn(u, sa), __fmul_rn(v, ca));
    u = nu;
    v = nv;
  }
  const long plane = (long)CH * CW;
  float* o = out + (long)b * 2 * plane + (long)y * CW + x;
  o[0] = u;
  o[plane] = v;
}

// preproc.hip: the horizontal Pillow pass (per-sample column offsets from prm[b * AUG_NP] when prm != null)
void pp_resize_h_launch(const uint8_t* in, uint8_t* tmp, const int* xb, const int* xk, int ksx, int B, int H, int W,
                        int CW, int cx0, const int* prm, int pstride, hipStream_t s);

}  // namespace svk

using namespace svk;

extern "C" int svk_train_augment(const void* frames, void* tmp, void* crop, long long* sums, float* out,
                                 const int* xbounds, const int* xcoef, int ksx, const int* ybounds, const int* ycoef,
                                 int ksy, const int* params, int B, int H, int W, int RH, int RW, int CH, int CW,
                                 const float* mean, const float* std, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || RH < CH || RW < CW || CH <= 0 || CW <= 0 || ksx <= 0 || ksy <= 0 || !frames ||
      !tmp || !crop || !sums || !out || !xbounds || !xcoef || !ybounds || !ycoef || !params || !mean || !std) {
    set_error("svk_train_augment: bad args (B=%d H=%d W=%d resize %dx%d crop %dx%d)", B, H, W, RH, RW, CH, CW);
    return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  if (CW % 4 || ((uintptr_t)tmp & 3) || ((uintptr_t)crop & 3) || ((uintptr_t)out & 15)) {
    set_error("svk_train_augment: crop width %d must be a multiple of 4, aligned buffers", CW);
    return SVK_EUNSUPPORTED;
  }
  if ((long)W * 3 * 4 + 32 > 64 * 1024) { set_error("svk_train_augment: frame width %d too large", W); return SVK_EUNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  pp_resize_h_launch((const uint8_t*)frames, (uint8_t*)tmp, xbounds, xcoef, ksx, B, H, W, CW, 0, params, AUG_NP, s);
  const long tv = (long)B * CH * (CW / 4);
  hipLaunchKernelGGL(aug_resize_v_u8, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, (const uint8_t*)tmp,
                     (uint8_t*)crop, ybounds, ycoef, ksy, params, B, H, CH, CW);
  hipLaunchKernelGGL(aug_luma_sum, dim3((unsigned)B), dim3(1024), 0, s, (const uint8_t*)crop, params, sums, CH * CW);
  hipLaunchKernelGGL(aug_finish, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, (const uint8_t*)crop, params,
                     (const long long*)sums, out, B, CH, CW, mean[0], mean[1], mean[2], std[0], std[1], std[2]);
  return check_launch("train_augment");
}

extern "C" int svk_train_augment_flow(const float* flow, float* out, const int* xofs, const float* xalpha,
                                      const int* yofs, const float* yalpha, const int* params, int B, int H, int W,
                                      int CH, int CW, float scale_u, float scale_v, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || CH <= 0 || CW <= 0 || !flow || !out || !xofs || !xalpha || !yofs || !yalpha ||
      !params || ((uintptr_t)flow & 7)) {
    set_error("svk_train_augment_flow: bad args (B=%d H=%d W=%d)", B, H, W);
    return SVK_EINVAL;
  }
  const long tv = (long)B * CH * CW;
  if (tv == 0) return SVK_OK;
  hipLaunchKernelGGL(aug_flow, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, (hipStream_t)stream, flow, out, xofs,
                     xalpha, yofs, yalpha, params, B, H, W, CH, CW, scale_u, scale_v);
  return check_launch("train_augment_flow");
}
