// MS-TCN DilatedResidualLayer (mstcn.py:181-214) fused into one kernel over a time-major
// [T, F] f32 map:  h = relu(Wd0 x[t+o0] + Wd1 x[t+o1] + Wd2 x[t+o2] + bd);  y = x + W1 h + b1.
// Causal (pad 2d, trim last 2d): taps o = (-2d, -d, 0); non-causal (pad d): (-d, 0, +d).
//
// A workgroup owns 64 time steps: it stages the three shifted input windows and the
// hidden tile in LDS (rows padded to F+1 floats: lanes walk t, so an unpadded F=32/64
// stride would put a whole wave on one bank), and reads weights through the scalar
// path (every lane of a wave works on the same output channel, so weight reads are
// wave-uniform).
#include "svk_common.h"

namespace svk {

constexpr int TT = 64;

template <int FMAX>
__global__ __launch_bounds__(256) void mstcn_layer_kernel(const float* __restrict__ X, const float* __restrict__ Wd,
                                                          const float* __restrict__ bd, const float* __restrict__ W1,
                                                          const float* __restrict__ b1, float* __restrict__ Y,
                                                          int T, int F, int dil, int causal) {
  constexpr int LD = FMAX + 1;
  __shared__ float xs[3][TT][LD];
  __shared__ float hs[TT][LD];
  const int t0 = blockIdx.x * TT;
  int off[3];
  if (causal) { off[0] = -2 * dil; off[1] = -dil; off[2] = 0; }
  else { off[0] = -dil; off[1] = 0; off[2] = dil; }
  for (int e = threadIdx.x; e < 3 * TT * F; e += blockDim.x) {
    const int j = e / (TT * F);
    const int r = e - j * TT * F;
    const int tl = r / F, c = r - tl * F;
    const int t = t0 + tl + off[j];
    xs[j][tl][c] = (t >= 0 && t < T && t0 + tl < T) ? X[(long)t * F + c] : 0.f;
  }
  __syncthreads();
  const int tl = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;          // 4 groups of output channels
  for (int fo = g; fo < F; fo += 4) {
    float h = bd[fo];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float* w = Wd + ((long)j * F + fo) * F;
      for (int ci = 0; ci < F; ++ci) h += w[ci] * xs[j][tl][ci];
    }
    hs[tl][fo] = h > 0.f ? h : 0.f;
  }
  __syncthreads();
  const int t = t0 + tl;
  for (int fo = g; fo < F; fo += 4) {
    float y = b1[fo];
    const float* w = W1 + (long)fo * F;
    for (int ci = 0; ci < F; ++ci) y += w[ci] * hs[tl][ci];
    if (t < T) Y[(long)t * F + fo] = xs[causal ? 2 : 1][tl][fo] + y;
  }
}

}  // namespace svk

using namespace svk;

extern "C" int svk_mstcn_layer(const float* X, const float* Wd, const float* bd, const float* W1, const float* b1,
                               float* Y, int T, int F, int dilation, int causal, void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !Wd || !bd || !W1 || !b1 || !Y || X == Y) {
    set_error("svk_mstcn_layer: bad args (F=%d must be <= 64, X != Y)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  dim3 grid((T + TT - 1) / TT);
  if (F <= 32) hipLaunchKernelGGL((mstcn_layer_kernel<32>), grid, dim3(256), 0, (hipStream_t)stream, X, Wd, bd, W1, b1, Y, T, F, dilation, causal);
  else hipLaunchKernelGGL((mstcn_layer_kernel<64>), grid, dim3(256), 0, (hipStream_t)stream, X, Wd, bd, W1, b1, Y, T, F, dilation, causal);
  return check_launch("mstcn_layer");
}
