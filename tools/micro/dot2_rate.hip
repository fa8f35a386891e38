// Issue rate of v_dot2c_f32_f16 (DPP row_shr:1 source) vs v_fmac_f32 (DPP) on gfx950: 8 independent
// accumulators per lane, 2048 workgroups x 256 threads, timed with HIP events.  Decides whether the
// stage-1 depthwise taps are cheaper as f16-pair dot products (6 per channel) than as f32 FMAs (9).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE, int NCH = 8>
__global__ __launch_bounds__(256) void k(float* o, const unsigned* a, int iters) {
  float acc[8];
  unsigned x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { acc[i] = 0.f; x[i] = a[(threadIdx.x + i) & 255]; }
  const unsigned y = a[threadIdx.x ^ 7];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i0 = 0; i0 < 8; ++i0) {
      const int i = i0 % NCH;
      if (MODE == 0)
        asm volatile("v_dot2c_f32_f16_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(acc[i]) : "v"(x[i]), "v"(y));
      else if (MODE == 1)
        asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(acc[i]) : "v"(x[i]), "v"(y));
      else if (MODE == 2)
        asm volatile("v_dot2c_f32_f16 %0, %1, %2" : "+v"(acc[i]) : "v"(x[i]), "v"(y));
      else
        asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc[i]) : "v"(x[i]), "v"(y));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i];
  o[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int NCH = 8>
static void run(const char* name, float* o, const unsigned* a, int grid = 2048) {
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k<MODE, NCH>), dim3(grid), dim3(256), 0, 0, o, a, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MODE, NCH>), dim3(grid), dim3(256), 0, 0, o, a, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  const double inst = 5.0 * grid * 4 * (double)iters * 8;   // wave-instructions
  printf("grid %4d %-18s chains %d %8.3f ms  %.3f G wave-instr/s  (%.2f ns per wave-instr per SIMD at 1024 SIMDs)\n", grid, name, NCH, ms,
         inst / ms / 1e6, ms * 1e6 / inst * 1024);
}

int main() {
  float* o; unsigned* a;
  hipMalloc(&o, 2048 * 256 * 4); hipMalloc(&a, 256 * 4);
  unsigned h[256];
  for (int i = 0; i < 256; ++i) h[i] = 0x3c003c00u ^ (i * 0x00010001u & 0x00ff00ffu);
  hipMemcpy(a, h, sizeof(h), hipMemcpyHostToDevice);
  run<0>("dot2c_f32_f16_dpp", o, a);
  run<1>("fmac_f32_dpp", o, a);
  run<2>("dot2c_f32_f16", o, a);
  run<3>("fmac_f32", o, a);
  run<0>("dot2c_f32_f16_dpp", o, a);
  run<1>("fmac_f32_dpp", o, a);
  run<0, 1>("dot2c_f32_f16_dpp", o, a);
  run<0, 2>("dot2c_f32_f16_dpp", o, a);
  run<0, 4>("dot2c_f32_f16_dpp", o, a);
  run<1, 1>("fmac_f32_dpp", o, a);
  run<1, 2>("fmac_f32_dpp", o, a);
  run<1, 4>("fmac_f32_dpp", o, a);
  // one wave per SIMD: the dependent-chain latency shows
  run<0, 1>("dot2c_f32_f16_dpp", o, a, 256);
  run<0, 2>("dot2c_f32_f16_dpp", o, a, 256);
  run<0, 4>("dot2c_f32_f16_dpp", o, a, 256);
  run<0, 8>("dot2c_f32_f16_dpp", o, a, 256);
  run<1, 1>("fmac_f32_dpp", o, a, 256);
  run<1, 2>("fmac_f32_dpp", o, a, 256);
  run<1, 4>("fmac_f32_dpp", o, a, 256);
  run<1, 8>("fmac_f32_dpp", o, a, 256);
  return 0;
}
