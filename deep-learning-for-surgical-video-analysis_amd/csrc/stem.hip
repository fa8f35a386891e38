// Stage-1 patch embedding over space-to-depth blocks + its LayerNorm in one kernel (mix_transformer_evp.py:
// 174-215, OverlapPatchEmbed: Conv2d(k = 7, s = 4, p = 3) -> flatten -> LayerNorm), 16-bit:
//
//   Y[b, oy, ox, :] = LN( sum_{ky, kx < 2} Xs[b, oy + ky, ox + kx, :] . W[:, ky, kx, :] + bias )
//
// Xs is the s2d packing of the frame / segmap / flow / Gaussian image (4 x 4 pixel blocks, CS = 16 Cin channels,
// svk_nchw_to_s2d / svk_gauss5x5_s2d), W the 7x7 kernel re-packed over the 2 x 2 block window (svk.pack.conv_w_s2d).
// The generic implicit-GEMM path (gemm_pk, im2col DMA per 16-byte chunk) ran these at 0.8-1.5 TB/s: K = 4 CS is
// only 3 K-steps per 128-row tile, so the per-tile prologue / epilogue and the im2col address math dominate, and
// the LayerNorm was a second pass over the 64-channel map.  Here:
//  * a workgroup (4 waves) owns 4 consecutive output rows of one image; the 5 input block rows they read are ONE
//    contiguous byte range of the NHWC map, DMA'd into LDS in 1 KiB lane-linear blocks (`global_load_lds_dwordx4`);
//  * each wave computes one output row: 64 pixel slots (OW <= 64) x Cout = 64, K = 4 CS, W fragments resident in
//    registers for the whole persistent kernel, A fragments read from LDS at the window's shifted offsets;
//  * transposed MFMA (W fragment x A fragment): a lane holds 4 consecutive channels of one pixel; the epilogue adds
//    the bias, rounds to 16 bits (the conv output the unfused path stores), LayerNorm over the pixel's 64 channels
//    (the 4 lanes of a pixel reduce with two shuffles), 8-byte stores.
// Persistent grid: workgroups stride over the (image, row group) units.
#include "svk_common.h"

namespace svk {
namespace stem {

typedef __attribute__((address_space(3))) void* las_ptr;
static __device__ __attribute__((aligned(16))) uint4 g_zero[4];

__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <int CS_, int COUT_ = 64>
struct Cfg {
  static constexpr int CS = CS_, COUT = COUT_, NB = COUT_ / 16, ROWS = 4, MAXW = 64;   // NB: 16-channel n-blocks
  static constexpr int KS = 4 * CS / 32;                       // 32-wide k-steps (CS = 32: 4, CS = 48: 6)
  static constexpr int CPT = CS / 8;                           // 16-byte chunks per tap
  static constexpr int LDS = ((ROWS + 1) * (MAXW + 1) * CS * 2 + 1023) / 1024 * 1024;
  static_assert(CS % 16 == 0 && COUT % 16 == 0 && NB >= 1 && NB <= 4, "channels");
};

template <typename T, class C>
__global__ __launch_bounds__(256, 2) void stem_s2d_ln(const T* __restrict__ Xs, const T* __restrict__ W,
                                                    const float* __restrict__ bias, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float eps, T* __restrict__ Y, int B,
                                                    int OH, int OW) {
  typedef v8_t<T> tx8;
  constexpr int CS = C::CS, KS = C::KS, CPT = C::CPT, ROWS = C::ROWS, NB = C::NB;
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(las_ptr)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int WB = OW + 1, HB = OH + 1;

  // W fragments (NB n-blocks x KS k-steps), resident: lane (fr, fq) holds W[16 nb + fr][32 ks + 8 fq .. + 7]
  tx8 wf[NB][KS];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) wf[nb][ks] = *reinterpret_cast<const tx8*>(W + (long)(nb * 16 + fr) * 4 * CS + ks * 32 + fq * 8);
  float bs[NB][4], gm[NB][4], bt[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = nb * 16 + fq * 4 + c;
      bs[nb][c] = bias ? bias[n] : 0.f;
      gm[nb][c] = gamma ? gamma[n] : 1.f;
      bt[nb][c] = gamma ? beta[n] : 0.f;
    }
  // A-fragment LDS offsets of chunk (ks, fq) relative to the wave's pixel (ky, kx, channel group)
  int aoff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int q = ks * 4 + fq, tap = q / CPT, c0 = (q % CPT) * 8;
    aoff[ks] = ((tap >> 1) * WB + (tap & 1)) * CS + c0;          // elements
  }
  const int ngroups = (OH + ROWS - 1) / ROWS, units = B * ngroups;
  const char* zero = reinterpret_cast<const char*>(g_zero);
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int b = u / ngroups, oy0 = (u - b * ngroups) * ROWS;
    // input block rows oy0 .. oy0 + ROWS (clamped to the map): one contiguous byte range
    const int nrows = min(ROWS + 1, HB - oy0);
    const long nbytes = (long)nrows * WB * CS * 2;
    const char* src = reinterpret_cast<const char*>(Xs + ((long)b * HB + oy0) * WB * CS);
    const int nblk = (int)((nbytes + 1023) >> 10);
    __syncthreads();                                             // the previous unit's LDS reads are done
    for (int blk = wave; blk < nblk; blk += 4) {
      const long o = (long)blk * 1024 + lane * 16;
      dma16(o < nbytes ? src + o : zero, __builtin_amdgcn_readfirstlane(lds0 + blk * 1024));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int oy = oy0 + wave;
    if (oy < OH) {                                               // wave-uniform
      f32x4 acc[4][NB];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const T* rowp = reinterpret_cast<const T*>(smem) + (long)wave * WB * CS;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int px = min(mb * 16 + fr, OW - 1);                // slots past OW compute a copy, never stored
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const tx8 a = *reinterpret_cast<const tx8*>(rowp + px * CS + aoff[ks]);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = mfma16x16x32(wf[nb][ks], a, acc[mb][nb]);
        }
      }
      // epilogue per pixel slot: lane (fr, fq) of block (mb, nb) holds channels 16 nb + 4 fq .. + 3 of pixel 16 mb + fr
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int px = mb * 16 + fr;
        float v[NB][4], s = 0.f;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            v[nb][c] = (float)(T)(acc[mb][nb][c] + bs[nb][c]);   // the conv output as the unfused path stores it
            s += v[nb][c];
          }
        T o[NB][4];
        if (gamma) {
          s += __shfl_xor(s, 16, 64);
          s += __shfl_xor(s, 32, 64);
          const float mean = s / C::COUT;
          float q = 0.f;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int c = 0; c < 4; ++c) { const float d = v[nb][c] - mean; q += d * d; }
          q += __shfl_xor(q, 16, 64);
          q += __shfl_xor(q, 32, 64);
          const float rstd = 1.0f / sqrtf(q / C::COUT + eps);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int c = 0; c < 4; ++c) o[nb][c] = (T)((v[nb][c] - mean) * rstd * gm[nb][c] + bt[nb][c]);
        } else {
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int c = 0; c < 4; ++c) o[nb][c] = (T)v[nb][c];
        }
        if (px < OW) {
          T* dst = Y + (((long)b * OH + oy) * OW + px) * C::COUT + fq * 4;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) *reinterpret_cast<uint2*>(dst + nb * 16) = *reinterpret_cast<const uint2*>(o[nb]);
        }
      }
    }
  }
}

template <typename T, class C>
static int launch(const void* Xs, const void* W, const float* bias, const float* gamma, const float* beta, float eps,
                  void* Y, int B, int OH, int OW, hipStream_t st) {
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&stem_s2d_ln<T, C>), 256, 0);
    slots = std::max(1, cus) * std::max(1, per);
  }
  const long units = (long)B * ((OH + C::ROWS - 1) / C::ROWS);
  const int grid = (int)std::min<long>(units, slots);
  hipLaunchKernelGGL((stem_s2d_ln<T, C>), dim3(grid), dim3(256), 0, st, (const T*)Xs, (const T*)W, bias, gamma, beta, eps,
                     (T*)Y, B, OH, OW);
  static char name[64];
  if (!name[0]) snprintf(name, sizeof(name), "stem_s2d_ln<%s, Cfg<%d, %d>>", type_name<T>(), C::CS, C::COUT);
  set_last_kernel(name);
  return check_launch("stem_s2d_ln");
}

}  // namespace stem
}  // namespace svk

using namespace svk;

extern "C" int svk_conv2d_s2d_ln_supported(int dtype, int CS, int Cout, int OW) {
  return (dtype == SVK_F16 || dtype == SVK_BF16) && (CS == 32 || CS == 48) && (Cout == 64 || Cout == 16) && OW >= 1 &&
         OW <= 64;
}

extern "C" int svk_conv2d_s2d_ln(int dtype, const void* Xs, int B, int HB, int WB, int CS, const void* W, const float* bias,
                                 const float* gamma, const float* beta, float eps, void* Y, int Cout, void* stream) {
  if (B < 0 || HB < 2 || WB < 2 || !Xs || !W || !Y || (gamma && !beta)) {
    set_error("svk_conv2d_s2d_ln: bad args"); return SVK_EINVAL;
  }
  if (!svk_conv2d_s2d_ln_supported(dtype, CS, Cout, WB - 1)) {
    set_error("svk_conv2d_s2d_ln: (dtype=%d, CS=%d, Cout=%d, OW=%d) not instantiated", dtype, CS, Cout, WB - 1);
    return SVK_EUNSUPPORTED;
  }
  if ((((uintptr_t)Xs) | ((uintptr_t)W)) & 15 || ((uintptr_t)Y) & 7) {
    set_error("svk_conv2d_s2d_ln: misaligned operand"); return SVK_EINVAL;
  }
  if (B == 0) return SVK_OK;
  if ((long)B * HB * WB * CS > 0x7fffffffL) { set_error("svk_conv2d_s2d_ln: map too large"); return SVK_EUNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_H16(dtype, T, {
    // Cout 16: the handcrafted prompt generator's first stem (embed_dim / scale_factor = 64 / 4 channels)
    if (Cout == 16) {
      if (CS == 32) return stem::launch<T, stem::Cfg<32, 16>>(Xs, W, bias, gamma, beta, eps, Y, B, HB - 1, WB - 1, st);
      return stem::launch<T, stem::Cfg<48, 16>>(Xs, W, bias, gamma, beta, eps, Y, B, HB - 1, WB - 1, st);
    }
    if (CS == 32) return stem::launch<T, stem::Cfg<32>>(Xs, W, bias, gamma, beta, eps, Y, B, HB - 1, WB - 1, st);
    return stem::launch<T, stem::Cfg<48>>(Xs, W, bias, gamma, beta, eps, Y, B, HB - 1, WB - 1, st);
  });
}
