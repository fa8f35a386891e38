// Training-step kernels (train_evp.py:473-515): normalisation / activation backward, batch-norm in
// train mode, bilinear-resize adjoint, phase losses, stochastic-depth / Dropout2d masks, SGD.
// Activations and their gradients are T (bf16 or f32); statistics, parameter grads and optimizer
// state are f32.
#include "svk_common.h"

namespace svk {

// ---- LayerNorm backward ---------------------------------------------------------------------
// dX = rstd * (g*dY - mean(g*dY) - xhat * mean(g*dY*xhat)) (+ dR);  dgamma += sum dY*xhat,
// dbeta += sum dY (f32 atomics, one partial per lane per block).  One wave per row, lanes over C.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ X, long ldx, const T* __restrict__ dY,
                                                            long ldy, const float* __restrict__ g, const T* __restrict__ dR,
                                                            long ldr, T* __restrict__ dX, long lddx,
                                                            float* __restrict__ dg, float* __restrict__ db, int M, int C,
                                                            float eps) {
  constexpr int PER = 8;     // C <= 512
  const int lane = threadIdx.x & 63;
  float pg[PER], pb[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  for (long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (long)gridDim.x * 4) {
    const T* x = X + row * ldx;
    const T* dy = dY + row * ldy;
    float xv[PER], gy[PER], dyv[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      xv[i] = c < C ? to_f(x[c]) : 0.f;
      dyv[i] = c < C ? to_f(dy[c]) : 0.f;
      gy[i] = c < C ? dyv[i] * g[c] : 0.f;
      s += xv[i];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) { const int c = lane + 64 * i; const float d = c < C ? xv[i] - mean : 0.f; q += d * d; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float xh = (xv[i] - mean) * rstd;
      xv[i] = xh;
      s1 += gy[i];
      s2 += gy[i] * xh;
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c >= C) continue;
      float v = rstd * (gy[i] - s1 - xv[i] * s2);
      if (dR) v += to_f(dR[row * ldr + c]);
      dX[row * lddx + c] = from_f<T>(v);
      pg[i] += dyv[i] * xv[i];
      pb[i] += dyv[i];
    }
  }
  if (dg) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = lane + 64 * i;
      if (c < C) { atomicAdd(dg + c, pg[i]); atomicAdd(db + c, pb[i]); }
    }
  }
}

// Vectorized LayerNorm backward: LPR lanes per row, 16-byte chunks (C % 8 == 0, C <= 512), grid-stride
// over rows; the affine gradients are reduced in registers over the rows a lane group visits, then
// across the wave's row groups by shuffles, then one f32 atomic per channel per wave.
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v) {
  T t[8];
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(t) = *reinterpret_cast<const uint4*>(p);
  } else {
    reinterpret_cast<uint4*>(t)[0] = reinterpret_cast<const uint4*>(p)[0];
    reinterpret_cast<uint4*>(t)[1] = reinterpret_cast<const uint4*>(p)[1];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = to_f(t[e]);
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* v) {
  T t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = from_f<T>(v[e]);
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(t);
  } else {
    reinterpret_cast<uint4*>(p)[0] = reinterpret_cast<const uint4*>(t)[0];
    reinterpret_cast<uint4*>(p)[1] = reinterpret_cast<const uint4*>(t)[1];
  }
}

template <typename T, int LPR, bool AFFINE>
__global__ __launch_bounds__(256) void layernorm_bwd_vec(const T* __restrict__ X, long ldx, const T* __restrict__ dY,
                                                         long ldy, const float* __restrict__ g,
                                                         const T* __restrict__ dR, long ldr, T* __restrict__ dX,
                                                         long lddx, float* __restrict__ dg, float* __restrict__ db,
                                                         int M, int C, float eps) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR, rg = lane / LPR;
  const int nch = C >> 3;
  const bool has = sub < nch;
  const int c0 = sub * 8;
  float gv[8], pg[8], pb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { gv[e] = has ? g[c0 + e] : 0.f; pg[e] = 0.f; pb[e] = 0.f; }
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long r0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW; r0 < M; r0 += stride) {
    const long row = r0 + rg;
    const bool ok = has && row < M;
    float x[8], dy[8];
    if (ok) { ld8(X + row * ldx + c0, x); ld8(dY + row * ldy + c0, dy); }
    else {
#pragma unroll
      for (int e = 0; e < 8; ++e) { x[e] = 0.f; dy[e] = 0.f; }
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += x[e];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / C;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = ok ? x[e] - mean : 0.f; q += d * d; }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q / C + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[e] = (x[e] - mean) * rstd;
      const float gy = dy[e] * gv[e];
      s1 += gy;
      s2 += gy * x[e];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
    s1 /= C;
    s2 /= C;
    if (ok) {
      float out[8];
      if (dR) ld8(dR + row * ldr + c0, out);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] += rstd * (dy[e] * gv[e] - s1 - x[e] * s2);
      st8(dX + row * lddx + c0, out);
      if constexpr (AFFINE) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { pg[e] += dy[e] * x[e]; pb[e] += dy[e]; }
      }
    }
  }
  if constexpr (AFFINE) {
    // reduce over the wave's row groups, then over the block's 4 waves in LDS: one atomic per channel
    // per block (the grid is capped at 256 blocks for the affine variant)
    __shared__ float red[2][4][512];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) { pg[e] += __shfl_xor(pg[e], o, 64); pb[e] += __shfl_xor(pb[e], o, 64); }
    }
    if (rg == 0 && has) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { red[0][w][c0 + e] = pg[e]; red[1][w][c0 + e] = pb[e]; }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      atomicAdd(dg + c, red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]);
      atomicAdd(db + c, red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c]);
    }
  }
}

// ---- activation backward: dX = dY * act'(U) (+ dR) --------------------------------------------
template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ U, const T* __restrict__ dY, const T* __restrict__ dR,
                               T* __restrict__ dX, long n, int act) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float u = to_f(U[i]);
  float d;
  if (act == SVK_ACT_GELU) {
    const float cdf = 0.5f * (1.0f + erff(u * 0.70710678118654752f));
    const float pdf = 0.3989422804014327f * expf(-0.5f * u * u);
    d = cdf + u * pdf;
  } else if (act == SVK_ACT_RELU) {
    d = u > 0.f ? 1.f : 0.f;
  } else if (act == SVK_ACT_TANH) {
    const float t = tanhf(u);
    d = 1.f - t * t;
  } else {
    d = 1.f;
  }
  float v = to_f(dY[i]) * d;
  if (dR) v += to_f(dR[i]);
  dX[i] = from_f<T>(v);
}

// ---- column statistics: sum and sum of squares over M rows (BN batch statistics) --------------
// Deterministic two-phase reduction (round 5).  Phase 1: block (bx, cy) sums rows bx*4 + rl, stride
// nblk*4, of 64 columns and writes its partial to ws[bx][c] (and ws[nblk + bx][c] for the squares); phase 2
// sums the nblk partials of a column in block order and adds the total to the output.  No atomics: the
// batch statistics, hence every BN + ReLU gate of the train forward, are bit-reproducible run to run.
// (The former per-block atomicAdd made the last bit of the batch mean depend on the arrival order of the
// blocks; a pre-ReLU value within that rounding of 0 then flipped its gate between runs, which is what moved
// head.linear_fuse.conv.weight's gradient by 1.6 % in the intermittent round-4 test failure.)
__host__ __device__ inline int stats_blocks(int M) { return M <= 0 ? 1 : (M + 63) / 64 < 1024 ? (M + 63) / 64 : 1024; }

template <typename T>
__global__ __launch_bounds__(256) void colstats_part_kernel(const T* __restrict__ X, long ldx, int M, int C,
                                                            float* __restrict__ ws, int want_sq) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int nblk = gridDim.x;
  float s = 0.f, q = 0.f;
  if (c < C)
    for (long r = (long)blockIdx.x * 4 + rl; r < M; r += (long)nblk * 4) {
      const float v = to_f(X[r * ldx + c]);
      s += v;
      q += v * v;
    }
  __shared__ float ss[4][64], sqq[4][64];
  ss[rl][threadIdx.x & 63] = s;
  sqq[rl][threadIdx.x & 63] = q;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int t = threadIdx.x & 63;
    ws[(long)blockIdx.x * C + c] = (ss[0][t] + ss[1][t]) + (ss[2][t] + ss[3][t]);
    if (want_sq) ws[(long)(nblk + blockIdx.x) * C + c] = (sqq[0][t] + sqq[1][t]) + (sqq[2][t] + sqq[3][t]);
  }
}

// out0[c] += sum_b ws[b][c], out1[c] += sum_b ws[nblk + b][c]; tot (optional) receives the two totals as well
// ([2][C]).  Block = 16 columns x 16 lanes; lane l owns partials l, l + 16, ... and keeps four accumulators
// (partial index / 16 mod 4) so four loads are in flight, then the 16 x 4 lane sums meet in LDS in a fixed
// tree order: the result does not depend on scheduling.  (Round 5 first had 64 columns x 4 lanes, one
// accumulator: 256 dependent adds per lane at nblk = 1024, 37 us a launch in the train step.)
constexpr int kFinCols = 16, kFinLanes = 16;
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ ws, int nblk, int C,
                                                           float* __restrict__ out0, float* __restrict__ out1,
                                                           float* __restrict__ tot) {
  const int t = threadIdx.x % kFinCols, l = threadIdx.x / kFinCols;
  const int c = blockIdx.x * kFinCols + t;
  const bool two = out1 || tot;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int i = l;
    for (; i + 3 * kFinLanes < nblk; i += 4 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += ws[(long)(i + u * kFinLanes) * C + c];
      if (two)
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] += ws[(long)(nblk + i + u * kFinLanes) * C + c];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (i + u * kFinLanes < nblk) {
        a[u] += ws[(long)(i + u * kFinLanes) * C + c];
        if (two) b[u] += ws[(long)(nblk + i + u * kFinLanes) * C + c];
      }
  }
  __shared__ float sa[kFinLanes][kFinCols], sb[kFinLanes][kFinCols];
  sa[l][t] = (a[0] + a[1]) + (a[2] + a[3]);
  sb[l][t] = (b[0] + b[1]) + (b[2] + b[3]);
  __syncthreads();
#pragma unroll
  for (int h = kFinLanes / 2; h >= 1; h >>= 1) {
    if (l < h) {
      sa[l][t] += sa[l + h][t];
      sb[l][t] += sb[l + h][t];
    }
    __syncthreads();
  }
  if (l == 0 && c < C) {
    const float x = sa[0][t], y = sb[0][t];
    if (out0) out0[c] += x;
    if (out1) out1[c] += y;
    if (tot) { tot[c] = x; tot[C + c] = y; }
  }
}

// ---- BN train-mode apply: Y = act((X - mean) * rstd * g + b), mean/var from the sums -------------
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ X, const float* __restrict__ sum, const float* __restrict__ sq,
                                const float* __restrict__ g, const float* __restrict__ b, T* __restrict__ Y, long n,
                                int C, int M, float eps, int act) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const float mean = sum[c] / M;
  const float var = fmaxf(sq[c] / M - mean * mean, 0.f);
  const float v = (to_f(X[i]) - mean) * rsqrtf(var + eps) * g[c] + b[c];
  Y[i] = from_f<T>(apply_act(v, act));
}

// BN train-mode backward (with an optional ReLU after the BN, recomputed from X):
// dxhat = dy' * g, dx = rstd/M * (M*dxhat - sum(dxhat) - xhat*sum(dxhat*xhat)).
// Phase 1 writes per-block partials of sdy = sum dy' and sdyx = sum dy'*xhat (same row split as colstats),
// colsum_final_kernel sums them in block order into tot [2][C] and adds them to dbeta / dgamma (which are
// exactly those sums), and the apply kernel reads tot — the gradient buffers may hold earlier contributions.
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_part_kernel(const T* __restrict__ X, const T* __restrict__ dY,
                                                          const float* __restrict__ sum, const float* __restrict__ sq,
                                                          const float* __restrict__ g, const float* __restrict__ b,
                                                          int M, int C, float eps, int relu, float* __restrict__ ws) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int nblk = gridDim.x;
  float a1 = 0.f, a2 = 0.f;
  if (c < C) {
    const float mean = sum[c] / M;
    const float rstd = rsqrtf(fmaxf(sq[c] / M - mean * mean, 0.f) + eps);
    for (long r = (long)blockIdx.x * 4 + rl; r < M; r += (long)nblk * 4) {
      const float xh = (to_f(X[r * C + c]) - mean) * rstd;
      float d = to_f(dY[r * C + c]);
      if (relu && xh * g[c] + b[c] <= 0.f) d = 0.f;
      a1 += d;
      a2 += d * xh;
    }
  }
  __shared__ float s1[4][64], s2[4][64];
  s1[rl][threadIdx.x & 63] = a1;
  s2[rl][threadIdx.x & 63] = a2;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int t = threadIdx.x & 63;
    ws[(long)blockIdx.x * C + c] = (s1[0][t] + s1[1][t]) + (s1[2][t] + s1[3][t]);
    ws[(long)(nblk + blockIdx.x) * C + c] = (s2[0][t] + s2[1][t]) + (s2[2][t] + s2[3][t]);
  }
}

template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ X, const T* __restrict__ dY, const float* __restrict__ sum,
                                    const float* __restrict__ sq, const float* __restrict__ g,
                                    const float* __restrict__ b, const float* __restrict__ tot, T* __restrict__ dX,
                                    long n, int C, int M, float eps, int relu) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)(i % C);
  const float mean = sum[c] / M;
  const float rstd = rsqrtf(fmaxf(sq[c] / M - mean * mean, 0.f) + eps);
  const float xh = (to_f(X[i]) - mean) * rstd;
  float d = to_f(dY[i]);
  if (relu && xh * g[c] + b[c] <= 0.f) d = 0.f;
  const float v = g[c] * rstd / M * (M * d - tot[c] - xh * tot[C + c]);
  dX[i] = from_f<T>(v);
}

// ---- bilinear resize adjoint (align_corners=False): dX[b, src, c] += w * dY[b, dst, c] (f32 atomics)
__device__ __forceinline__ void src_index_b(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = (float)in / (float)out;
  float s = scale * (dst + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = s - i0;
  l0 = 1.f - l1;
}

template <typename T>
__global__ void resize_bwd_kernel(const T* __restrict__ dY, long ldy, float* __restrict__ dX, int B, int H, int W,
                                  int C, int OH, int OW) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * OH * OW * C) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int ox = (int)(pix % OW);
  const long t = pix / OW;
  const int oy = (int)(t % OH);
  const int b = (int)(t / OH);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  src_index_b(oy, H, OH, y0, y1, ly0, ly1);
  src_index_b(ox, W, OW, x0, x1, lx0, lx1);
  const float g = to_f(dY[((long)b * OH * OW + (long)oy * OW + ox) * ldy + c]);
  float* base = dX + (long)b * H * W * C + c;
  atomicAdd(base + ((long)y0 * W + x0) * C, g * ly0 * lx0);
  atomicAdd(base + ((long)y0 * W + x1) * C, g * ly0 * lx1);
  atomicAdd(base + ((long)y1 * W + x0) * C, g * ly1 * lx0);
  atomicAdd(base + ((long)y1 * W + x1) * C, g * ly1 * lx1);
}

// ---- broadcast row-mean adjoint: dY[b*R + r, c] = dF[b, c] * scale ---------------------------
template <typename T>
__global__ void bcast_rows_kernel(const float* __restrict__ dF, const float* __restrict__ mask, float scale,
                                  T* __restrict__ dY, int B, int R, int C) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * R * C) return;
  const int c = (int)(i % C);
  const long b = i / ((long)R * C);
  float v = dF[b * C + c] * scale;
  if (mask) v *= mask[b * C + c];
  dY[i] = from_f<T>(v);
}

__global__ void mul_f32_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a[i] * b[i];
}

// running_mean = (1 - mom) * running_mean + mom * mean; running_var likewise with the unbiased variance
// (torch.nn.BatchNorm2d train-mode buffer update).
__global__ void bn_running_kernel(const float* __restrict__ sum, const float* __restrict__ sq, int M, int C,
                                  float mom, float* __restrict__ rm, float* __restrict__ rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = sum[c] / M;
  const float var = fmaxf(sq[c] / M - mean * mean, 0.f);
  rm[c] = (1.f - mom) * rm[c] + mom * mean;
  rv[c] = (1.f - mom) * rv[c] + mom * var * ((float)M / (float)max(M - 1, 1));
}

// Batched parameter packing: every descriptor is a 4-D strided gather from the f32 master copy into
// a packed (compute-dtype) layout; source indices at or past `lim` read as zero (channel padding).
// One launch refreshes every packed view of the trainable weights after an optimizer step.
struct PackDesc {
  long src, dst;     // element offsets
  int n[4];          // packed shape
  long s[4];         // source stride of each packed dim
  int lim[4];        // source extent of each packed dim
  long start;        // first packed element of this descriptor in the launch's linear index space
};

template <typename T>
__global__ void pack_params_kernel(const PackDesc* __restrict__ d, int nd, long total, const float* __restrict__ src,
                                   T* __restrict__ dst) {
  // one binary search per block (its first index), then each thread steps forward over the few descriptors
  // the block spans; per-descriptor index math in 32 bits (every packed tensor has < 2^31 elements)
  __shared__ int s_first;
  const long blk0 = (long)blockIdx.x * blockDim.x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = nd - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (d[mid].start <= blk0) lo = mid; else hi = mid - 1;
    }
    s_first = lo;
  }
  __syncthreads();
  const long i = blk0 + threadIdx.x;
  if (i >= total) return;
  int lo = s_first;
  while (lo + 1 < nd && d[lo + 1].start <= i) ++lo;
  const PackDesc& e = d[lo];
  int r = (int)(i - e.start);
  if (r >= e.n[0] * e.n[1] * e.n[2] * e.n[3]) return;          // alignment gap between descriptors
  long off = e.src;
  bool ok = true;
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    const int idx = r % e.n[k];
    r /= e.n[k];
    ok = ok && idx < e.lim[k];
    off += (long)idx * e.s[k];
  }
  dst[e.dst + (i - e.start)] = from_f<T>(ok ? src[off] : 0.f);
}

// The same gather, 8 consecutive packed elements per thread: every descriptor starts at a multiple of 8 of the
// linear index space (and of the packed buffer), so a thread's 8 elements share one descriptor; the 4-D index
// is decomposed once and stepped, and the 8 values leave as one 16-byte store (two for f32).  Elements past a
// tensor's end up to its 8-aligned slot end are written as zeros (the packed buffer's alignment padding).
template <typename T>
__global__ void pack_params8_kernel(const PackDesc* __restrict__ d, int nd, long total, const float* __restrict__ src,
                                    T* __restrict__ dst) {
  __shared__ int s_first;
  const long blk0 = (long)blockIdx.x * blockDim.x * 8;
  if (threadIdx.x == 0) {
    int lo = 0, hi = nd - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (d[mid].start <= blk0) lo = mid; else hi = mid - 1;
    }
    s_first = lo;
  }
  __syncthreads();
  const long i0 = blk0 + (long)threadIdx.x * 8;
  if (i0 >= total) return;
  int lo = s_first;
  while (lo + 1 < nd && d[lo + 1].start <= i0) ++lo;
  const PackDesc& e = d[lo];
  const int numel = e.n[0] * e.n[1] * e.n[2] * e.n[3];
  const int r0 = (int)(i0 - e.start);
  if (r0 >= numel) return;
  int idx[4];
  {
    int r = r0;
#pragma unroll
    for (int k = 3; k >= 0; --k) { idx[k] = r % e.n[k]; r /= e.n[k]; }
  }
  T v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float x = 0.f;
    if (r0 + q < numel) {
      const bool ok = idx[0] < e.lim[0] && idx[1] < e.lim[1] && idx[2] < e.lim[2] && idx[3] < e.lim[3];
      if (ok) x = src[e.src + idx[0] * e.s[0] + idx[1] * e.s[1] + idx[2] * e.s[2] + idx[3] * e.s[3]];
#pragma unroll
      for (int k = 3; k >= 0; --k) {             // step the index: innermost first, with carry
        if (++idx[k] < e.n[k]) break;
        idx[k] = 0;
      }
    }
    v[q] = from_f<T>(x);
  }
  T* out = dst + e.dst + r0;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(out) = *reinterpret_cast<const uint4*>(v);
  } else {
    reinterpret_cast<uint4*>(out)[0] = *reinterpret_cast<const uint4*>(v);
    reinterpret_cast<uint4*>(out)[1] = *reinterpret_cast<const uint4*>(v + 4);
  }
}

// ---- transposed 2-D packs: one workgroup per 64 x 64 tile of a row-major [N, K] f32 master ----------
struct PackTile {
  long src, dst;     // element offsets of the master matrix / the packed [K, N] view
  int K, N, n0, k0;  // master shape, tile origin
};

template <typename T>
__global__ __launch_bounds__(256) void pack_transpose_kernel(const PackTile* __restrict__ tl, const float* __restrict__ src,
                                                             T* __restrict__ dst) {
  __shared__ float tile[64][65];
  const PackTile t = tl[blockIdx.x];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // master rows n0 + r, columns k0 + tx: 256 B per wave-row, coalesced
#pragma unroll 4
  for (int r = ty; r < 64; r += 4) {
    const int n = t.n0 + r, k = t.k0 + tx;
    tile[r][tx] = (n < t.N && k < t.K) ? src[t.src + (long)n * t.K + k] : 0.f;
  }
  __syncthreads();
  // packed rows k0 + r, columns n0 + tx
#pragma unroll 4
  for (int r = ty; r < 64; r += 4) {
    const int k = t.k0 + r, n = t.n0 + tx;
    if (k < t.K && n < t.N) dst[t.dst + (long)k * t.N + n] = from_f<T>(tile[tx][r]);
  }
}

// ---- per-row scale (stochastic depth / Dropout2d masks): Y[r, c] = X[r, c] * s[r / rows_per] ---
template <typename T>
__global__ void row_scale_kernel(const T* __restrict__ X, const float* __restrict__ s, T* __restrict__ Y, long n,
                                 int C, int rows_per) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Y[i] = from_f<T>(to_f(X[i]) * s[(i / C) / rows_per]);
}

// Counter-based Bernoulli keep-mask scaled by 1/keep (mask values 0 or 1/keep), seeded per call.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__global__ void keep_mask_kernel(float* __restrict__ out, long n, float keep, uint32_t seed,
                                 const long long* __restrict__ counter) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // the optional device counter (the trainer's step count) makes replays of a captured graph draw
  // fresh masks
  if (counter) seed = hash32(seed ^ hash32((uint32_t)*counter * 0x85EBCA6BU));
  const float u = (hash32((uint32_t)i * 0x9E3779B9U ^ hash32(seed)) >> 8) * (1.0f / 16777216.0f);
  out[i] = u < keep ? 1.0f / keep : 0.f;
}

// nm masks of n floats each in one launch (mask m: keep[m], seed[m]); element (m, e) is the value
// keep_mask_kernel gives element e of a mask with that keep / seed, bit for bit
__global__ void keep_mask_multi_kernel(float* __restrict__ out, long n, int nm, const float* __restrict__ keeps,
                                       const uint32_t* __restrict__ seeds, const long long* __restrict__ counter) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * nm) return;
  const int m = (int)(i / n);
  const long e = i - (long)m * n;
  uint32_t seed = seeds[m];
  if (counter) seed = hash32(seed ^ hash32((uint32_t)*counter * 0x85EBCA6BU));
  const float keep = keeps[m];
  const float u = (hash32((uint32_t)e * 0x9E3779B9U ^ hash32(seed)) >> 8) * (1.0f / 16777216.0f);
  out[i] = u < keep ? 1.0f / keep : 0.f;
}

// ---- phase losses: CrossEntropy(sum) + SmoothL1(sum) and their gradients (train_evp.py:390-391, 500-509)
__global__ void phase_loss_kernel(const float* __restrict__ logits, const float* __restrict__ ant,
                                  const long* __restrict__ labels, const float* __restrict__ ant_t, int B, int K,
                                  float* __restrict__ loss, float* __restrict__ dlogits, float* __restrict__ dant) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* z = logits + (long)b * K;
  float m = -INFINITY;
  for (int k = 0; k < K; ++k) m = fmaxf(m, z[k]);
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += expf(z[k] - m);
  const long y = labels[b];
  atomicAdd(loss, logf(s) + m - z[y]);
  for (int k = 0; k < K; ++k) dlogits[(long)b * K + k] = expf(z[k] - m) / s - (k == y ? 1.f : 0.f);
  float l1 = 0.f;
  for (int k = 0; k < K; ++k) {
    const float d = ant[(long)b * K + k] - ant_t[(long)b * K + k];
    const float ad = fabsf(d);
    l1 += ad < 1.f ? 0.5f * d * d : ad - 0.5f;
    dant[(long)b * K + k] = ad < 1.f ? d : (d > 0.f ? 1.f : -1.f);
  }
  atomicAdd(loss + 1, l1);
}

// ---- SGD with momentum / dampening / weight decay / nesterov (torch.optim.SGD semantics) -------
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ gr, float* __restrict__ buf, long n,
                           float lr, float momentum, float dampening, float wd, int nesterov, int first) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d = gr[i] + wd * p[i];
  if (momentum != 0.f) {
    const float bv = first ? d : momentum * buf[i] + (1.f - dampening) * d;
    buf[i] = bv;
    d = nesterov ? d + momentum * bv : bv;
  }
  p[i] -= lr * d;
}

// ---- unpatchify: [B*PH*PW, s*s*C] patch rows -> NHWC [B, PH*s, PW*s, C] (+ optional accumulate) ---
template <typename T>
__global__ void unpatchify_kernel(const T* __restrict__ P, T* __restrict__ Y, int B, int PH, int PW, int s, int C,
                                  int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)B * PH * PW * s * s * C;
  if (i >= n) return;
  const int c = (int)(i % C);
  long t = i / C;
  const int j = (int)(t % s); t /= s;
  const int ii = (int)(t % s); t /= s;
  const int px = (int)(t % PW); t /= PW;
  const int py = (int)(t % PH);
  const long b = t / PH;
  const long dst = ((b * PH * s + (long)py * s + ii) * ((long)PW * s) + (long)px * s + j) * C + c;
  const float v = to_f(P[i]);
  Y[dst] = from_f<T>(accumulate ? to_f(Y[dst]) + v : v);
}

// 8 channels per thread (C % 8 == 0, 16-byte aligned maps): one 16-byte load of P, one 16-byte
// read-modify-write of Y; consecutive threads walk a patch row's contiguous s*C run of a pixel row
template <typename T>
__global__ void unpatchify8_kernel(const T* __restrict__ P, T* __restrict__ Y, long n8, int PH, int PW, int s, int C8,
                                   int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int c8 = (int)(i % C8);
  long t = i / C8;
  const int j = (int)(t % s); t /= s;
  const int ii = (int)(t % s); t /= s;
  const int px = (int)(t % PW); t /= PW;
  const int py = (int)(t % PH);
  const long b = t / PH;
  const long dst = (((b * PH * s + (long)py * s + ii) * ((long)PW * s) + (long)px * s + j) * C8 + c8) * 8;
  uint4 pv = reinterpret_cast<const uint4*>(P)[i];
  if (accumulate) {
    const uint4 yv = *reinterpret_cast<const uint4*>(Y + dst);
    const T* pe = reinterpret_cast<const T*>(&pv);
    const T* ye = reinterpret_cast<const T*>(&yv);
    T o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f<T>(to_f(ye[e]) + to_f(pe[e]));
    pv = *reinterpret_cast<const uint4*>(o);
  }
  *reinterpret_cast<uint4*>(Y + dst) = pv;
}

// ---- col2im: conv data gradient from the per-tap products P = dY Wc^T ------------------------------
// P [B*OH*OW, k*k*Cin] (column (ky*k + kx)*Cin + ci) -> dX NHWC [B, H, W, Cin] (+ residual): each input
// pixel gathers the taps that reached it, dX[y, x] = sum over (ky, kx) with y + pad - ky = stride*oy (and
// likewise x) of P[(oy, ox), (ky, kx)].  The GEMM producing P does exactly k*k*Cin*Cout MACs per output
// pixel (a direct transposed-conv GEMM over dX pixels multiplies stride^2 - 1 of every stride^2 taps by zero).
// 8 channels per thread, 16-byte loads / stores, f32 sums.
template <typename T>
__global__ void col2im8_kernel(const T* __restrict__ P, const T* __restrict__ Rs, T* __restrict__ Y, long n8, int H,
                               int W, int C8, int OH, int OW, int k, int stride, int pad) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int c8 = (int)(i % C8);
  long t = i / C8;
  const int x = (int)(t % W); t /= W;
  const int y = (int)(t % H);
  const long b = t / H;
  float acc[8];
  if (Rs) {
    const uint4 rv = reinterpret_cast<const uint4*>(Rs)[i];
    const T* re = reinterpret_cast<const T*>(&rv);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = to_f(re[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  }
  const long ldp = (long)k * k * C8;   // P row stride in 8-element chunks
  const uint4* P4 = reinterpret_cast<const uint4*>(P);
  for (int ky = (y + pad) % stride; ky < k; ky += stride) {
    const int oy = (y + pad - ky) / stride;
    if (oy < 0) break;
    if (oy >= OH) continue;
    for (int kx = (x + pad) % stride; kx < k; kx += stride) {
      const int ox = (x + pad - kx) / stride;
      if (ox < 0) break;
      if (ox >= OW) continue;
      const uint4 pv = P4[((b * OH + oy) * OW + ox) * ldp + (long)(ky * k + kx) * C8 + c8];
      const T* pe = reinterpret_cast<const T*>(&pv);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += to_f(pe[e]);
    }
  }
  T o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = from_f<T>(acc[e]);
  reinterpret_cast<uint4*>(Y)[i] = *reinterpret_cast<const uint4*>(o);
}

inline dim3 g1(long n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace svk

using namespace svk;

template <typename T, int LPR>
static void launch_ln_bwd_vec(const T* X, long ldx, const T* dY, long ldy, const float* g, const T* dR, long ldr, T* dX,
                              long lddx, float* dg, float* db, int M, int C, float eps, hipStream_t st) {
  constexpr int RPB = 4 * (64 / LPR);
  const int blocks = (int)std::min<long>((M + RPB - 1) / RPB, dg ? 256 : 1L << 30);
  if (dg)
    hipLaunchKernelGGL((layernorm_bwd_vec<T, LPR, true>), dim3(blocks), dim3(256), 0, st, X, ldx, dY, ldy, g, dR, ldr,
                       dX, lddx, dg, db, M, C, eps);
  else
    hipLaunchKernelGGL((layernorm_bwd_vec<T, LPR, false>), dim3(blocks), dim3(256), 0, st, X, ldx, dY, ldy, g, dR, ldr,
                       dX, lddx, dg, db, M, C, eps);
}

extern "C" int svk_layernorm_bwd(int dtype, const void* X, long ldx, const void* dY, long ldy, const float* gamma,
                                 const void* dR, long ldr, void* dX, long lddx, float* dgamma, float* dbeta, int M,
                                 int C, float eps, void* stream) {
  if (M < 0 || C <= 0 || C > 512 || !X || !dY || !gamma || !dX || ((dgamma == nullptr) != (dbeta == nullptr))) {
    set_error("svk_layernorm_bwd: bad args (C <= 512)"); return SVK_EINVAL;
  }
  if (M == 0) return SVK_OK;
  {
    const uintptr_t al = (uintptr_t)X | (uintptr_t)dY | (uintptr_t)dX | (uintptr_t)dR;
    const long vw = dtype == SVK_BF16 ? 8 : 4;
    if (C % 8 == 0 && (al & 15) == 0 && ldx % vw == 0 && ldy % vw == 0 && lddx % vw == 0 && (!dR || ldr % vw == 0)) {
      hipStream_t st = (hipStream_t)stream;
      const int nch = C / 8;
      SVK_DISPATCH_DTYPE(dtype, T, {
        auto go = [&](auto lpr) {
          constexpr int L = decltype(lpr)::value;
          launch_ln_bwd_vec<T, L>((const T*)X, ldx, (const T*)dY, ldy, gamma, (const T*)dR, ldr, (T*)dX, lddx, dgamma,
                                  dbeta, M, C, eps, st);
        };
        if (nch <= 1) go(std::integral_constant<int, 1>{});
        else if (nch <= 2) go(std::integral_constant<int, 2>{});
        else if (nch <= 4) go(std::integral_constant<int, 4>{});
        else if (nch <= 8) go(std::integral_constant<int, 8>{});
        else if (nch <= 16) go(std::integral_constant<int, 16>{});
        else if (nch <= 32) go(std::integral_constant<int, 32>{});
        else go(std::integral_constant<int, 64>{});
        return check_launch("layernorm_bwd_vec");
      });
    }
  }
  const int blocks = (int)std::min<long>((M + 3) / 4, 2048);
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((layernorm_bwd_kernel<T>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const T*)X, ldx,
                       (const T*)dY, ldy, gamma, (const T*)dR, ldr, (T*)dX, lddx, dgamma, dbeta, M, C, eps);
    return check_launch("layernorm_bwd");
  });
}

extern "C" int svk_act_bwd(int dtype, const void* U, const void* dY, const void* dR, void* dX, long n, int act,
                           void* stream) {
  if (n < 0 || !U || !dY || !dX) { set_error("svk_act_bwd: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((act_bwd_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, (const T*)U, (const T*)dY,
                       (const T*)dR, (T*)dX, n, act);
    return check_launch("act_bwd");
  });
}

extern "C" long svk_stats_ws_floats(int M, int C) {
  if (M < 0 || C <= 0) return -1;
  return 2L * stats_blocks(M) * C + 2L * C;
}

extern "C" int svk_colstats(int dtype, const void* X, long ldx, int M, int C, float* sum, float* sumsq, float* ws,
                            void* stream) {
  if (M < 0 || C <= 0 || !X || !sum || !ws) { set_error("svk_colstats: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  const int nb = stats_blocks(M);
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((colstats_part_kernel<T>), dim3(nb, (C + 63) / 64), dim3(256), 0, st, (const T*)X, ldx, M, C,
                       ws, sumsq ? 1 : 0);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + kFinCols - 1) / kFinCols), dim3(256), 0, st, (const float*)ws, nb, C, sum,
                       sumsq, (float*)nullptr);
    return check_launch("colstats");
  });
}

extern "C" int svk_colstats_set(int dtype, const void* X, long ldx, int M, int C, float* sums, float* ws,
                                void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M == 0 && C > 0 && sums)   // no rows: zero sums (X and ws may be empty)
    return hipMemsetAsync(sums, 0, sizeof(float) * 2 * C, st) == hipSuccess ? SVK_OK : SVK_ELAUNCH;
  if (M < 0 || C <= 0 || !X || !sums || !ws) { set_error("svk_colstats_set: bad args"); return SVK_EINVAL; }
  const int nb = stats_blocks(M);
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((colstats_part_kernel<T>), dim3(nb, (C + 63) / 64), dim3(256), 0, st, (const T*)X, ldx, M, C,
                       ws, 1);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + kFinCols - 1) / kFinCols), dim3(256), 0, st, (const float*)ws, nb, C,
                       (float*)nullptr, (float*)nullptr, sums);
    return check_launch("colstats_set");
  });
}

extern "C" int svk_bn_apply(int dtype, const void* X, const float* sum, const float* sumsq, const float* gamma,
                            const float* beta, void* Y, int M, int C, float eps, int act, void* stream) {
  if (M < 0 || C <= 0 || !X || !sum || !sumsq || !gamma || !beta || !Y) { set_error("svk_bn_apply: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  const long n = (long)M * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((bn_apply_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, sum, sumsq, gamma,
                       beta, (T*)Y, n, C, M, eps, act);
    return check_launch("bn_apply");
  });
}

extern "C" int svk_bn_bwd(int dtype, const void* X, const void* dY, const float* sum, const float* sumsq,
                          const float* gamma, const float* beta, void* dX, float* dgamma, float* dbeta, int M, int C,
                          float eps, int relu, float* ws, void* stream) {
  if (M <= 0 || C <= 0 || !X || !dY || !sum || !sumsq || !gamma || !beta || !dX || !dgamma || !dbeta || !ws) {
    set_error("svk_bn_bwd: bad args"); return SVK_EINVAL;
  }
  const long n = (long)M * C;
  const int nb = stats_blocks(M);
  float* tot = ws + 2L * nb * C;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((bn_bwd_part_kernel<T>), dim3(nb, (C + 63) / 64), dim3(256), 0, st, (const T*)X, (const T*)dY,
                       sum, sumsq, gamma, beta, M, C, eps, relu, ws);
    // dbeta += sum dy', dgamma += sum dy'*xhat (exactly the two sums)
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + kFinCols - 1) / kFinCols), dim3(256), 0, st, (const float*)ws, nb, C, dbeta,
                       dgamma, tot);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T>), g1(n), dim3(256), 0, st, (const T*)X, (const T*)dY, sum, sumsq, gamma,
                       beta, (const float*)tot, (T*)dX, n, C, M, eps, relu);
    return check_launch("bn_bwd");
  });
}

extern "C" int svk_resize_bilinear_bwd(int dtype, const void* dY, long ldy, float* dX, int B, int H, int W, int C,
                                       int OH, int OW, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0 || !dY || !dX) { set_error("svk_resize_bilinear_bwd: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * OH * OW * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((resize_bwd_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, (const T*)dY, ldy, dX, B, H, W,
                       C, OH, OW);
    return check_launch("resize_bilinear_bwd");
  });
}

extern "C" int svk_bcast_rows(int dtype, const float* dF, const float* mask, float scale, void* dY, int B, int R, int C,
                              void* stream) {
  if (B < 0 || R <= 0 || C <= 0 || !dF || !dY) { set_error("svk_bcast_rows: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * R * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((bcast_rows_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, dF, mask, scale, (T*)dY, B, R,
                       C);
    return check_launch("bcast_rows");
  });
}

extern "C" int svk_row_scale(int dtype, const void* X, const float* s, void* Y, long M, int C, int rows_per,
                             void* stream) {
  if (M < 0 || C <= 0 || rows_per <= 0 || !X || !s || !Y) { set_error("svk_row_scale: bad args"); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  const long n = M * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((row_scale_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, (const T*)X, s, (T*)Y, n, C,
                       rows_per);
    return check_launch("row_scale");
  });
}

extern "C" int svk_keep_mask(float* out, long n, float keep, unsigned seed, const long long* counter, void* stream) {
  if (n < 0 || !out || !(keep > 0.f) || keep > 1.f) { set_error("svk_keep_mask: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipLaunchKernelGGL(keep_mask_kernel, g1(n), dim3(256), 0, (hipStream_t)stream, out, n, keep, (uint32_t)seed, counter);
  return check_launch("keep_mask");
}

extern "C" int svk_keep_mask_multi(float* out, long n, int nm, const float* keeps, const unsigned* seeds,
                                   const long long* counter, void* stream) {
  if (n < 0 || nm < 0 || (n * nm > 0 && (!out || !keeps || !seeds))) { set_error("svk_keep_mask_multi: bad args"); return SVK_EINVAL; }
  if (n * nm == 0) return SVK_OK;
  hipLaunchKernelGGL(keep_mask_multi_kernel, g1(n * nm), dim3(256), 0, (hipStream_t)stream, out, n, nm, keeps,
                     (const uint32_t*)seeds, counter);
  return check_launch("keep_mask_multi");
}

extern "C" int svk_phase_loss(const float* logits, const float* ant, const long* labels, const float* ant_t, int B,
                              int K, float* loss, float* dlogits, float* dant, void* stream) {
  if (B <= 0 || K <= 0 || !logits || !ant || !labels || !ant_t || !loss || !dlogits || !dant) {
    set_error("svk_phase_loss: bad args"); return SVK_EINVAL;
  }
  hipLaunchKernelGGL(phase_loss_kernel, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, logits, ant, labels,
                     ant_t, B, K, loss, dlogits, dant);
  return check_launch("phase_loss");
}

extern "C" int svk_sgd(float* p, const float* grad, float* buf, long n, float lr, float momentum, float dampening,
                       float wd, int nesterov, int first, void* stream) {
  if (n < 0 || !p || !grad || (momentum != 0.f && !buf)) { set_error("svk_sgd: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipLaunchKernelGGL(sgd_kernel, g1(n), dim3(256), 0, (hipStream_t)stream, p, grad, buf, n, lr, momentum, dampening,
                     wd, nesterov, first);
  return check_launch("sgd");
}

extern "C" int svk_unpatchify(int dtype, const void* P, void* Y, int B, int PH, int PW, int s, int C, int accumulate,
                              void* stream) {
  if (B < 0 || PH <= 0 || PW <= 0 || s <= 0 || C <= 0 || !P || !Y) { set_error("svk_unpatchify: bad args"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long n = (long)B * PH * PW * s * s * C;
  SVK_DISPATCH_DTYPE(dtype, T, {
    if (sizeof(T) == 2 && C % 8 == 0 && ((((uintptr_t)P) | ((uintptr_t)Y)) & 15) == 0) {
      hipLaunchKernelGGL((unpatchify8_kernel<T>), g1(n / 8), dim3(256), 0, (hipStream_t)stream, (const T*)P, (T*)Y, n / 8,
                         PH, PW, s, C / 8, accumulate);
      return check_launch("unpatchify8");
    }
    hipLaunchKernelGGL((unpatchify_kernel<T>), g1(n), dim3(256), 0, (hipStream_t)stream, (const T*)P, (T*)Y, B, PH, PW,
                       s, C, accumulate);
    return check_launch("unpatchify");
  });
}

extern "C" int svk_col2im_nhwc(int dtype, const void* P, const void* R, void* Y, int B, int H, int W, int Cin, int OH,
                               int OW, int k, int stride, int pad, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || OH <= 0 || OW <= 0 || k <= 0 || stride <= 0 || pad < 0 || !P || !Y) {
    set_error("svk_col2im_nhwc: bad args"); return SVK_EINVAL;
  }
  if ((dtype != SVK_BF16 && dtype != SVK_F16) || Cin % 8 || ((((uintptr_t)P) | ((uintptr_t)R) | ((uintptr_t)Y)) & 15)) {
    set_error("svk_col2im_nhwc: needs bf16 / f16, Cin %% 8 == 0, 16-byte aligned maps"); return SVK_EUNSUPPORTED;
  }
  if (B == 0) return SVK_OK;
  const long n8 = (long)B * H * W * (Cin / 8);
  SVK_DISPATCH_H16(dtype, T, {
    hipLaunchKernelGGL((col2im8_kernel<T>), g1(n8), dim3(256), 0, (hipStream_t)stream, (const T*)P, (const T*)R, (T*)Y,
                       n8, H, W, Cin / 8, OH, OW, k, stride, pad);
    return check_launch("col2im");
  });
}

extern "C" int svk_mul_f32(const float* a, const float* b, float* y, long n, void* stream) {
  if (n < 0 || !a || !b || !y) { set_error("svk_mul_f32: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipLaunchKernelGGL(mul_f32_kernel, g1(n), dim3(256), 0, (hipStream_t)stream, a, b, y, n);
  return check_launch("mul_f32");
}

extern "C" int svk_bn_update_running(const float* sum, const float* sumsq, int M, int C, float momentum,
                                     float* running_mean, float* running_var, void* stream) {
  if (M <= 0 || C <= 0 || !sum || !sumsq || !running_mean || !running_var) {
    set_error("svk_bn_update_running: bad args"); return SVK_EINVAL;
  }
  hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sum, sumsq, M, C,
                     momentum, running_mean, running_var);
  return check_launch("bn_update_running");
}

extern "C" int svk_pack_transpose(int dtype, const void* tiles, int ntiles, const float* src, void* dst, void* stream) {
  if (ntiles < 0 || !tiles || !src || !dst) { set_error("svk_pack_transpose: bad args"); return SVK_EINVAL; }
  if (ntiles == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((pack_transpose_kernel<T>), dim3((unsigned)ntiles), dim3(256), 0, (hipStream_t)stream,
                       (const PackTile*)tiles, src, (T*)dst);
    return check_launch("pack_transpose");
  });
}

extern "C" int svk_pack_params8(int dtype, const void* desc, int ndesc, long total, const float* src, void* dst,
                                void* stream) {
  if (ndesc <= 0 || total < 0 || total % 8 || !desc || !src || !dst || ((uintptr_t)dst & 15)) {
    set_error("svk_pack_params8: bad args (total %% 8 == 0, 16-byte aligned dst)"); return SVK_EINVAL;
  }
  if (total == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((pack_params8_kernel<T>), g1(total / 8), dim3(256), 0, (hipStream_t)stream,
                       (const PackDesc*)desc, ndesc, total, src, (T*)dst);
    return check_launch("pack_params8");
  });
}

extern "C" int svk_pack_params(int dtype, const void* desc, int ndesc, long total, const float* src, void* dst,
                               void* stream) {
  if (ndesc <= 0 || total < 0 || !desc || !src || !dst) { set_error("svk_pack_params: bad args"); return SVK_EINVAL; }
  if (total == 0) return SVK_OK;
  SVK_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((pack_params_kernel<T>), g1(total), dim3(256), 0, (hipStream_t)stream, (const PackDesc*)desc,
                       ndesc, total, src, (T*)dst);
    return check_launch("pack_params");
  });
}
