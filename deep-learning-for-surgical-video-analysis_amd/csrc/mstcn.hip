// MS-TCN DilatedResidualLayer (mstcn.py:181-214) fused into one kernel over a time-major
// [T, F] f32 map:  h = relu(Wd0 x[t+o0] + Wd1 x[t+o1] + Wd2 x[t+o2] + bd);  y = x + W1 h + b1.
// Causal (pad 2d, trim last 2d): taps o = (-2d, -d, 0); non-causal (pad d): (-d, 0, +d).
//
// A workgroup owns 64 time steps: it stages the three shifted input windows and the
// hidden tile in LDS (rows padded to F+1 floats: lanes walk t, so an unpadded F=32/64
// stride would put a whole wave on one bank), and reads weights through the scalar
// path (every lane of a wave works on the same output channel, so weight reads are
// wave-uniform).
//
// Training (tecno.py:195-259 trains the MS-TCN variant with its nn.Dropout(p=0.5) active): the forward
// takes a keep mask m (0 or 1/keep, counter-based svk_keep_mask) — y = x + m * (W1 h + b1) — and saves
// h = relu(pre) for the backward, which runs as two kernels per layer:
//   A  (per 64-step tile)  dout = dy * m;  dpre = (dout W1) * [h > 0] -> dPre;  the tile's partial
//                          dW1 = dout^T h, db1, dWd[j] = dpre^T x[t + o_j], dbd reduced in registers
//                          from LDS and added with one f32 atomic per weight per tile;
//   B  (per 64-step tile)  dx[t] = dy[t] + sum_j Wd[j]^T dpre[t - o_j]  (the transposed dilated conv:
//                          the three dPre windows at t - o_j staged in LDS like the forward's).
#include "svk_common.h"

namespace svk {

constexpr int TT = 64;

__device__ __forceinline__ void tap_offsets(int causal, int dil, int* off) {
  if (causal) { off[0] = -2 * dil; off[1] = -dil; off[2] = 0; }
  else { off[0] = -dil; off[1] = 0; off[2] = dil; }
}

template <int FMAX, bool TRAIN>
__global__ __launch_bounds__(256) void mstcn_layer_kernel(const float* __restrict__ X, const float* __restrict__ Wd,
                                                          const float* __restrict__ bd, const float* __restrict__ W1,
                                                          const float* __restrict__ b1, float* __restrict__ Y,
                                                          int T, int F, int dil, int causal,
                                                          const float* __restrict__ mask, float* __restrict__ Hout) {
  constexpr int LD = FMAX + 1;
  __shared__ float xs[3][TT][LD];
  __shared__ float hs[TT][LD];
  const int t0 = blockIdx.x * TT;
  int off[3];
  tap_offsets(causal, dil, off);
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
  const int t = t0 + tl;
  for (int fo = g; fo < F; fo += 4) {
    float h = bd[fo];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float* w = Wd + ((long)j * F + fo) * F;
      for (int ci = 0; ci < F; ++ci) h += w[ci] * xs[j][tl][ci];
    }
    h = h > 0.f ? h : 0.f;
    hs[tl][fo] = h;
    if (TRAIN && t < T) Hout[(long)t * F + fo] = h;
  }
  __syncthreads();
  for (int fo = g; fo < F; fo += 4) {
    float y = b1[fo];
    const float* w = W1 + (long)fo * F;
    for (int ci = 0; ci < F; ++ci) y += w[ci] * hs[tl][ci];
    if (t < T) {
      if (TRAIN) y *= mask[(long)t * F + fo];
      Y[(long)t * F + fo] = xs[causal ? 2 : 1][tl][fo] + y;
    }
  }
}

template <int FMAX>
__global__ __launch_bounds__(256) void mstcn_bwd_a(const float* __restrict__ X, const float* __restrict__ H,
                                                   const float* __restrict__ mask, const float* __restrict__ dY,
                                                   const float* __restrict__ W1, float* __restrict__ dPre,
                                                   float* __restrict__ dWd, float* __restrict__ dbd,
                                                   float* __restrict__ dW1, float* __restrict__ db1, int T, int F,
                                                   int dil, int causal) {
  constexpr int LD = FMAX + 1;
  __shared__ float xs[3][TT][LD];          // x[t + o_j]
  __shared__ float hs[TT][LD];             // h
  __shared__ float ds[TT][LD];             // dout = dy * m
  __shared__ float ps[TT][LD];             // dpre
  const int t0 = blockIdx.x * TT;
  int off[3];
  tap_offsets(causal, dil, off);
  for (int e = threadIdx.x; e < TT * F; e += blockDim.x) {
    const int tl = e / F, c = e - tl * F;
    const int t = t0 + tl;
    const bool ok = t < T;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ts = t + off[j];
      xs[j][tl][c] = (ok && ts >= 0 && ts < T) ? X[(long)ts * F + c] : 0.f;
    }
    hs[tl][c] = ok ? H[(long)t * F + c] : 0.f;
    ds[tl][c] = ok ? dY[(long)t * F + c] * mask[(long)t * F + c] : 0.f;
  }
  __syncthreads();
  const int tl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int t = t0 + tl;
  for (int ci = g; ci < F; ci += 4) {      // dh[t][ci] = sum_fo dout[t][fo] W1[fo][ci]
    float s = 0.f;
    for (int fo = 0; fo < F; ++fo) s += ds[tl][fo] * W1[(long)fo * F + ci];
    const float p = hs[tl][ci] > 0.f ? s : 0.f;
    ps[tl][ci] = p;
    if (t < T) dPre[(long)t * F + ci] = p;
  }
  __syncthreads();
  const int nt = min(TT, T - t0);
  for (int e = threadIdx.x; e < F * F; e += blockDim.x) {
    const int fo = e / F, ci = e - fo * F;
    float w1 = 0.f, w0 = 0.f, wm = 0.f, wp = 0.f;
    for (int k = 0; k < nt; ++k) {
      const float dd = ds[k][fo], pp = ps[k][fo];
      w1 += dd * hs[k][ci];
      w0 += pp * xs[0][k][ci];
      wm += pp * xs[1][k][ci];
      wp += pp * xs[2][k][ci];
    }
    atomicAdd(dW1 + e, w1);
    atomicAdd(dWd + 3 * e, w0);          // nn.Conv1d weight layout [F_out][F_in][3]
    atomicAdd(dWd + 3 * e + 1, wm);
    atomicAdd(dWd + 3 * e + 2, wp);
  }
  if (threadIdx.x < F) {
    const int fo = threadIdx.x;
    float a = 0.f, b = 0.f;
    for (int k = 0; k < nt; ++k) { a += ds[k][fo]; b += ps[k][fo]; }
    atomicAdd(db1 + fo, a);
    atomicAdd(dbd + fo, b);
  }
}

template <int FMAX>
__global__ __launch_bounds__(256) void mstcn_bwd_b(const float* __restrict__ dY, const float* __restrict__ dPre,
                                                   const float* __restrict__ Wd, float* __restrict__ dX, int T, int F,
                                                   int dil, int causal) {
  constexpr int LD = FMAX + 1;
  __shared__ float ps[3][TT][LD];          // dpre[t - o_j]
  const int t0 = blockIdx.x * TT;
  int off[3];
  tap_offsets(causal, dil, off);
  for (int e = threadIdx.x; e < 3 * TT * F; e += blockDim.x) {
    const int j = e / (TT * F);
    const int r = e - j * TT * F;
    const int tl = r / F, c = r - tl * F;
    const int ts = t0 + tl - off[j];
    ps[j][tl][c] = (ts >= 0 && ts < T && t0 + tl < T) ? dPre[(long)ts * F + c] : 0.f;
  }
  __syncthreads();
  const int tl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int t = t0 + tl;
  if (t >= T) return;
  for (int ci = g; ci < F; ci += 4) {
    float s = dY[(long)t * F + ci];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float* w = Wd + (long)j * F * F + ci;        // Wd[j][fo][ci], fo strided by F
      for (int fo = 0; fo < F; ++fo) s += w[(long)fo * F] * ps[j][tl][fo];
    }
    dX[(long)t * F + ci] = s;
  }
}

// softmax over C classes per row: backward dx = p * (dp - sum_c p dp)
__global__ void softmax_rows_bwd_kernel(const float* __restrict__ P, long ldp, const float* __restrict__ dP, long lddp,
                                        const float* __restrict__ R, long ldr, float* __restrict__ dX, long lddx, int M,
                                        int C) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  const float* p = P + r * ldp;
  const float* g = dP + r * lddp;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += p[c] * g[c];
  for (int c = 0; c < C; ++c) dX[r * lddx + c] = p[c] * (g[c] - s) + (R ? R[r * ldr + c] : 0.f);
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
  hipStream_t st = (hipStream_t)stream;
  if (F <= 32) hipLaunchKernelGGL((mstcn_layer_kernel<32, false>), grid, dim3(256), 0, st, X, Wd, bd, W1, b1, Y, T, F, dilation, causal, nullptr, nullptr);
  else hipLaunchKernelGGL((mstcn_layer_kernel<64, false>), grid, dim3(256), 0, st, X, Wd, bd, W1, b1, Y, T, F, dilation, causal, nullptr, nullptr);
  return check_launch("mstcn_layer");
}

extern "C" int svk_mstcn_layer_train(const float* X, const float* Wd, const float* bd, const float* W1, const float* b1,
                                     const float* mask, float* Y, float* H, int T, int F, int dilation, int causal,
                                     void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !Wd || !bd || !W1 || !b1 || !mask || !Y || !H || X == Y) {
    set_error("svk_mstcn_layer_train: bad args (F=%d must be <= 64, X != Y)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  dim3 grid((T + TT - 1) / TT);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 32) hipLaunchKernelGGL((mstcn_layer_kernel<32, true>), grid, dim3(256), 0, st, X, Wd, bd, W1, b1, Y, T, F, dilation, causal, mask, H);
  else hipLaunchKernelGGL((mstcn_layer_kernel<64, true>), grid, dim3(256), 0, st, X, Wd, bd, W1, b1, Y, T, F, dilation, causal, mask, H);
  return check_launch("mstcn_layer_train");
}

extern "C" int svk_mstcn_layer_bwd(const float* X, const float* H, const float* mask, const float* dY, const float* Wd,
                                   const float* W1, float* dPre, float* dX, float* dWd, float* dbd, float* dW1,
                                   float* db1, int T, int F, int dilation, int causal, void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !H || !mask || !dY || !Wd || !W1 || !dPre || !dX || !dWd ||
      !dbd || !dW1 || !db1 || dX == dY) {
    set_error("svk_mstcn_layer_bwd: bad args (F=%d must be <= 64, dX != dY)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  dim3 grid((T + TT - 1) / TT);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 32) {
    hipLaunchKernelGGL((mstcn_bwd_a<32>), grid, dim3(256), 0, st, X, H, mask, dY, W1, dPre, dWd, dbd, dW1, db1, T, F, dilation, causal);
    hipLaunchKernelGGL((mstcn_bwd_b<32>), grid, dim3(256), 0, st, dY, dPre, Wd, dX, T, F, dilation, causal);
  } else {
    hipLaunchKernelGGL((mstcn_bwd_a<64>), grid, dim3(256), 0, st, X, H, mask, dY, W1, dPre, dWd, dbd, dW1, db1, T, F, dilation, causal);
    hipLaunchKernelGGL((mstcn_bwd_b<64>), grid, dim3(256), 0, st, dY, dPre, Wd, dX, T, F, dilation, causal);
  }
  return check_launch("mstcn_layer_bwd");
}

extern "C" int svk_softmax_rows_bwd(const float* P, long ldp, const float* dP, long lddp, const float* R, long ldr,
                                    float* dX, long lddx, int M, int C, void* stream) {
  if (M < 0 || C <= 0 || !P || !dP || !dX || ldp < C || lddp < C || lddx < C || (R && ldr < C)) {
    set_error("svk_softmax_rows_bwd: bad args"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  hipLaunchKernelGGL(softmax_rows_bwd_kernel, dim3((M + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, ldp, dP,
                     lddp, R, ldr, dX, lddx, M, C);
  return check_launch("softmax_rows_bwd");
}
