// MS-TCN DilatedResidualLayer (mstcn.py:181-214) over a time-major [T, F] f32 map (F <= 64):
//   h = relu(Wd0 x[t+o0] + Wd1 x[t+o1] + Wd2 x[t+o2] + bd);  y = x + m * (W1 h + b1)
// Causal (pad 2d, trim last 2d): taps o = (-2d, -d, 0); non-causal (pad d): (-d, 0, +d); m = 1 in eval,
// the nn.Dropout(0.5) keep mask (0 or 1/keep) in training (tecno.py:195-259).
//
// Layout of the work: a workgroup owns TT = 16 time steps (T / 16 workgroups: ~190 for a 3000-frame
// video, enough to spread over the chip; 64-step tiles left 3/4 of the CUs idle).  Lanes run over
// CHANNELS (lane = output channel in the forward / input channel in the backward), so every weight
// row is one coalesced 256-byte load per wave, reused from registers for the thread's TT*F/256 time
// rows, while the activations are LDS broadcasts (all lanes of a wave read the same row element).
// The three shifted input windows and the hidden tile sit in LDS with rows padded to F+1 floats.
//
// Weights (f32): forward WdT [3][F_in][F_out] and W1T [F_in][F_out] (transposed packs); backward
// Wd [3][F_out][F_in] and W1 [F_out][F_in] (the 1x1 conv's own layout).
//
// Backward, per layer:
//   A  dout = dy * m;  dpre = (dout W1) * [h > 0] -> dPre;  the tile's partial weight gradients
//      dW1 = dout^T h, dWd[j] = dpre^T x[t + o_j] (4 F x F) and db1 / dbd, written to a per-tile slab
//      (no atomics in the hot loop);
//   R  slab reduction over tiles into dWd ([F_out][F_in][3], the nn.Conv1d layout), dbd, dW1, db1;
//   B  dx[t] = dy[t] + sum_j Wd[j]^T dpre[t - o_j]  (the transposed dilated conv).
#include "svk_common.h"

namespace svk {

constexpr int TT = 16;           // time steps per workgroup
constexpr int NTH = 256;

__device__ __forceinline__ void tap_offsets(int causal, int dil, int* off) {
  if (causal) { off[0] = -2 * dil; off[1] = -dil; off[2] = 0; }
  else { off[0] = -dil; off[1] = 0; off[2] = dil; }
}

// lanes over channels: FMAX lanes per row group, RP row groups, RT rows per thread
template <int FMAX>
struct Map {
  static constexpr int RP = NTH / FMAX, RT = TT / RP;
};

// Ragged multi-video batches (trans_SV_output.py:251-291 / tecno.py:80-91 walk the test videos one by
// one): the videos' maps are concatenated time-major and one launch covers every video's tiles.  Tile
// record {first row of the tile's video, that video's length, tile start inside the video, 0}; taps
// never cross a video boundary (out-of-video rows read zero, exactly the per-video zero padding).
// tiles == nullptr: one video of length T, tile = blockIdx.x.
template <int FMAX, bool TRAIN>
__global__ __launch_bounds__(NTH) void mstcn_layer_kernel(const float* __restrict__ X, const float* __restrict__ WdT,
                                                          const float* __restrict__ bd, const float* __restrict__ W1T,
                                                          const float* __restrict__ b1, float* __restrict__ Y, int T,
                                                          int F, int dil, int causal, const float* __restrict__ mask,
                                                          float* __restrict__ Hout, const int4* __restrict__ tiles) {
  // rows padded to a multiple of 4 floats + 4: 16-byte broadcast reads of 4 input channels
  constexpr int LD = FMAX + 4, RP = Map<FMAX>::RP, RT = Map<FMAX>::RT;
  __shared__ __attribute__((aligned(16))) float xs[3][TT][LD];
  __shared__ __attribute__((aligned(16))) float hs[TT][LD];
  int t0 = blockIdx.x * TT;
  if (tiles) {
    const int4 tl = tiles[blockIdx.x];
    X += (long)tl.x * F;
    Y += (long)tl.x * F;
    T = tl.y;
    t0 = tl.z;
  }
  int off[3];
  tap_offsets(causal, dil, off);
  for (int e = threadIdx.x; e < 3 * TT * F; e += NTH) {
    const int j = e / (TT * F);
    const int r = e - j * TT * F;
    const int tl = r / F, c = r - tl * F;
    const int t = t0 + tl + off[j];
    xs[j][tl][c] = (t >= 0 && t < T && t0 + tl < T) ? X[(long)t * F + c] : 0.f;
  }
  __syncthreads();
  const int fo = threadIdx.x % FMAX, rg = threadIdx.x / FMAX;
  const bool act = fo < F;
  const int F4 = F & ~3;
  float acc[RT];
#pragma unroll
  for (int k = 0; k < RT; ++k) acc[k] = act ? bd[fo] : 0.f;
  if (act) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float* w = WdT + (long)j * F * F + fo;
      int ci = 0;
      for (; ci < F4; ci += 4) {
        const float w0 = w[(long)ci * F], w1 = w[(long)(ci + 1) * F], w2 = w[(long)(ci + 2) * F], w3 = w[(long)(ci + 3) * F];
#pragma unroll
        for (int k = 0; k < RT; ++k) {
          const float4 xv = *reinterpret_cast<const float4*>(&xs[j][rg + k * RP][ci]);
          acc[k] += w0 * xv.x;
          acc[k] += w1 * xv.y;
          acc[k] += w2 * xv.z;
          acc[k] += w3 * xv.w;
        }
      }
      for (; ci < F; ++ci) {
        const float wv = w[(long)ci * F];
#pragma unroll
        for (int k = 0; k < RT; ++k) acc[k] += wv * xs[j][rg + k * RP][ci];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    const int tl = rg + k * RP;
    const float h = acc[k] > 0.f ? acc[k] : 0.f;
    if (act) {
      hs[tl][fo] = h;
      if (TRAIN && t0 + tl < T) Hout[(long)(t0 + tl) * F + fo] = h;
    }
  }
  __syncthreads();
  if (!act) return;
#pragma unroll
  for (int k = 0; k < RT; ++k) acc[k] = b1[fo];
  {
    int ci = 0;
    for (; ci < F4; ci += 4) {
      const float w0 = W1T[(long)ci * F + fo], w1 = W1T[(long)(ci + 1) * F + fo], w2 = W1T[(long)(ci + 2) * F + fo],
                  w3 = W1T[(long)(ci + 3) * F + fo];
#pragma unroll
      for (int k = 0; k < RT; ++k) {
        const float4 hv = *reinterpret_cast<const float4*>(&hs[rg + k * RP][ci]);
        acc[k] += w0 * hv.x;
        acc[k] += w1 * hv.y;
        acc[k] += w2 * hv.z;
        acc[k] += w3 * hv.w;
      }
    }
    for (; ci < F; ++ci) {
      const float wv = W1T[(long)ci * F + fo];
#pragma unroll
      for (int k = 0; k < RT; ++k) acc[k] += wv * hs[rg + k * RP][ci];
    }
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    const int tl = rg + k * RP, t = t0 + tl;
    if (t < T) {
      float y = acc[k];
      if (TRAIN) y *= mask[(long)t * F + fo];
      Y[(long)t * F + fo] = xs[causal ? 2 : 1][tl][fo] + y;
    }
  }
}

// slab per tile: [dW1 | dWd0 | dWd1 | dWd2] (each F x F, [f_out][f_in]) then db1 [F], dbd [F]
__host__ __device__ constexpr long slab_floats(int F) { return 4L * F * F + 2L * F; }

template <int FMAX>
__global__ __launch_bounds__(NTH) void mstcn_bwd_a(const float* __restrict__ X, const float* __restrict__ H,
                                                   const float* __restrict__ mask, const float* __restrict__ dY,
                                                   const float* __restrict__ W1, float* __restrict__ dPre,
                                                   float* __restrict__ part, int T, int F, int dil, int causal) {
  constexpr int LD = FMAX + 1, RP = Map<FMAX>::RP, RT = Map<FMAX>::RT, QF = FMAX / RP;
  __shared__ float xs[3][TT][LD];          // x[t + o_j]
  __shared__ float hs[TT][LD];             // h
  __shared__ float ds[TT][LD];             // dout = dy * m
  __shared__ float ps[TT][LD];             // dpre
  const int t0 = blockIdx.x * TT;
  int off[3];
  tap_offsets(causal, dil, off);
  for (int e = threadIdx.x; e < TT * F; e += NTH) {
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
  const int c = threadIdx.x % FMAX, rg = threadIdx.x / FMAX;
  const bool act = c < F;
  {                                        // dh[t][c] = sum_fo dout[t][fo] W1[fo][c]
    float acc[RT];
#pragma unroll
    for (int k = 0; k < RT; ++k) acc[k] = 0.f;
    if (act) {
      for (int fo = 0; fo < F; ++fo) {
        const float wv = W1[(long)fo * F + c];
#pragma unroll
        for (int k = 0; k < RT; ++k) acc[k] += wv * ds[rg + k * RP][fo];
      }
#pragma unroll
      for (int k = 0; k < RT; ++k) {
        const int tl = rg + k * RP;
        const float p = hs[tl][c] > 0.f ? acc[k] : 0.f;
        ps[tl][c] = p;
        if (t0 + tl < T) dPre[(long)(t0 + tl) * F + c] = p;
      }
    }
  }
  __syncthreads();
  // partial weight gradients of this tile: thread (c, rg) owns f_out = rg + q * RP, q < QF
  float a1[QF], a0[QF], am[QF], ap[QF];
#pragma unroll
  for (int q = 0; q < QF; ++q) a1[q] = a0[q] = am[q] = ap[q] = 0.f;
  const int nt = min(TT, T - t0);
  for (int k = 0; k < nt; ++k) {
    const float hv = hs[k][c], x0 = xs[0][k][c], x1 = xs[1][k][c], x2 = xs[2][k][c];
#pragma unroll
    for (int q = 0; q < QF; ++q) {
      const int fo = rg + q * RP;
      const float d = ds[k][fo], p = ps[k][fo];
      a1[q] += d * hv;
      a0[q] += p * x0;
      am[q] += p * x1;
      ap[q] += p * x2;
    }
  }
  float* sl = part + (long)blockIdx.x * slab_floats(F);
  const long FF = (long)F * F;
  if (act) {
#pragma unroll
    for (int q = 0; q < QF; ++q) {
      const int fo = rg + q * RP;
      if (fo < F) {
        const long e = (long)fo * F + c;
        sl[e] = a1[q];
        sl[FF + e] = a0[q];
        sl[2 * FF + e] = am[q];
        sl[3 * FF + e] = ap[q];
      }
    }
  }
  if (threadIdx.x < F) {
    const int fo = threadIdx.x;
    float a = 0.f, b = 0.f;
    for (int k = 0; k < nt; ++k) { a += ds[k][fo]; b += ps[k][fo]; }
    sl[4 * FF + fo] = a;
    sl[4 * FF + F + fo] = b;
  }
}

// Sum the per-tile slabs (tile chunks of RCH per thread, one f32 atomic per chunk) into the gradients.
constexpr int RCH = 32;
__global__ __launch_bounds__(NTH) void mstcn_bwd_reduce(const float* __restrict__ part, int nblk, int F,
                                                        float* __restrict__ dWd, float* __restrict__ dbd,
                                                        float* __restrict__ dW1, float* __restrict__ db1) {
  const long E = slab_floats(F), FF = (long)F * F;
  const long e = (long)blockIdx.x * NTH + threadIdx.x;
  if (e >= E) return;
  const int b0 = blockIdx.y * RCH, b1 = min(nblk, b0 + RCH);
  float s = 0.f;
  for (int b = b0; b < b1; ++b) s += part[(long)b * E + e];
  if (e < FF) atomicAdd(dW1 + e, s);
  else if (e < 4 * FF) {
    const long m = e / FF - 1, r = e - (m + 1) * FF;       // r = fo * F + ci
    atomicAdd(dWd + r * 3 + m, s);                          // nn.Conv1d layout [F_out][F_in][3]
  } else if (e < 4 * FF + F) atomicAdd(db1 + (e - 4 * FF), s);
  else atomicAdd(dbd + (e - 4 * FF - F), s);
}

template <int FMAX>
__global__ __launch_bounds__(NTH) void mstcn_bwd_b(const float* __restrict__ dY, const float* __restrict__ dPre,
                                                   const float* __restrict__ Wd, float* __restrict__ dX, int T, int F,
                                                   int dil, int causal) {
  constexpr int LD = FMAX + 1, RP = Map<FMAX>::RP, RT = Map<FMAX>::RT;
  __shared__ float ps[3][TT][LD];          // dpre[t - o_j]
  const int t0 = blockIdx.x * TT;
  int off[3];
  tap_offsets(causal, dil, off);
  for (int e = threadIdx.x; e < 3 * TT * F; e += NTH) {
    const int j = e / (TT * F);
    const int r = e - j * TT * F;
    const int tl = r / F, c = r - tl * F;
    const int ts = t0 + tl - off[j];
    ps[j][tl][c] = (ts >= 0 && ts < T && t0 + tl < T) ? dPre[(long)ts * F + c] : 0.f;
  }
  __syncthreads();
  const int c = threadIdx.x % FMAX, rg = threadIdx.x / FMAX;
  if (c >= F) return;
  float acc[RT];
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    const int t = t0 + rg + k * RP;
    acc[k] = t < T ? dY[(long)t * F + c] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float* w = Wd + (long)j * F * F + c;             // Wd[j][fo][c]
    for (int fo = 0; fo < F; ++fo) {
      const float wv = w[(long)fo * F];
#pragma unroll
      for (int k = 0; k < RT; ++k) acc[k] += wv * ps[j][rg + k * RP][fo];
    }
  }
#pragma unroll
  for (int k = 0; k < RT; ++k) {
    const int t = t0 + rg + k * RP;
    if (t < T) dX[(long)t * F + c] = acc[k];
  }
}

// softmax over C classes per row: backward dx = p * (dp - sum_c p dp) (+ r)
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

template <bool TRAIN>
static int launch_layer(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                        const float* mask, float* Y, float* H, int T, int F, int dil, int causal, hipStream_t st,
                        const int4* tiles = nullptr, int ntiles = 0) {
  dim3 grid(tiles ? ntiles : (T + TT - 1) / TT);
  if (F <= 32)
    hipLaunchKernelGGL((mstcn_layer_kernel<32, TRAIN>), grid, dim3(NTH), 0, st, X, WdT, bd, W1T, b1, Y, T, F, dil, causal,
                       mask, H, tiles);
  else
    hipLaunchKernelGGL((mstcn_layer_kernel<64, TRAIN>), grid, dim3(NTH), 0, st, X, WdT, bd, W1T, b1, Y, T, F, dil, causal,
                       mask, H, tiles);
  return check_launch(TRAIN ? "mstcn_layer_train" : "mstcn_layer");
}

}  // namespace svk

using namespace svk;

extern "C" int svk_mstcn_layer(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                               float* Y, int T, int F, int dilation, int causal, void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !WdT || !bd || !W1T || !b1 || !Y || X == Y) {
    set_error("svk_mstcn_layer: bad args (F=%d must be <= 64, X != Y)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  return launch_layer<false>(X, WdT, bd, W1T, b1, nullptr, Y, nullptr, T, F, dilation, causal, (hipStream_t)stream);
}

extern "C" int svk_mstcn_tile_size() { return TT; }

extern "C" int svk_mstcn_layer_ragged(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                                      float* Y, const int* tiles, int ntiles, int F, int dilation, int causal,
                                      void* stream) {
  if (ntiles < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !WdT || !bd || !W1T || !b1 || !Y || X == Y ||
      (ntiles > 0 && (!tiles || ((uintptr_t)tiles & 15)))) {
    set_error("svk_mstcn_layer_ragged: bad args (F=%d must be <= 64, X != Y, 16-byte aligned tile table)", F);
    return SVK_EINVAL;
  }
  if (ntiles == 0) return SVK_OK;
  return launch_layer<false>(X, WdT, bd, W1T, b1, nullptr, Y, nullptr, 0, F, dilation, causal, (hipStream_t)stream,
                             reinterpret_cast<const int4*>(tiles), ntiles);
}

extern "C" int svk_mstcn_layer_train(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                                     const float* mask, float* Y, float* H, int T, int F, int dilation, int causal,
                                     void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !WdT || !bd || !W1T || !b1 || !mask || !Y || !H || X == Y) {
    set_error("svk_mstcn_layer_train: bad args (F=%d must be <= 64, X != Y)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  return launch_layer<true>(X, WdT, bd, W1T, b1, mask, Y, H, T, F, dilation, causal, (hipStream_t)stream);
}

extern "C" long svk_mstcn_bwd_workspace(int T, int F) {
  if (T <= 0 || F <= 0) return 0;
  return (long)((T + TT - 1) / TT) * slab_floats(F) * (long)sizeof(float);
}

extern "C" int svk_mstcn_layer_bwd(const float* X, const float* H, const float* mask, const float* dY, const float* Wd,
                                   const float* W1, float* dPre, float* dX, float* dWd, float* dbd, float* dW1,
                                   float* db1, float* ws, int T, int F, int dilation, int causal, void* stream) {
  if (T < 0 || F <= 0 || F > 64 || dilation <= 0 || !X || !H || !mask || !dY || !Wd || !W1 || !dPre || !dX || !dWd ||
      !dbd || !dW1 || !db1 || !ws || dX == dY) {
    set_error("svk_mstcn_layer_bwd: bad args (F=%d must be <= 64, dX != dY, ws required)", F); return SVK_EINVAL;
  }
  if (T == 0) return SVK_OK;
  const int nblk = (T + TT - 1) / TT;
  dim3 grid(nblk);
  hipStream_t st = (hipStream_t)stream;
  if (F <= 32) hipLaunchKernelGGL((mstcn_bwd_a<32>), grid, dim3(NTH), 0, st, X, H, mask, dY, W1, dPre, ws, T, F, dilation, causal);
  else hipLaunchKernelGGL((mstcn_bwd_a<64>), grid, dim3(NTH), 0, st, X, H, mask, dY, W1, dPre, ws, T, F, dilation, causal);
  const long E = slab_floats(F);
  hipLaunchKernelGGL(mstcn_bwd_reduce, dim3((unsigned)((E + NTH - 1) / NTH), (unsigned)((nblk + RCH - 1) / RCH)),
                     dim3(NTH), 0, st, ws, nblk, F, dWd, dbd, dW1, db1);
  if (F <= 32) hipLaunchKernelGGL((mstcn_bwd_b<32>), grid, dim3(NTH), 0, st, dY, dPre, Wd, dX, T, F, dilation, causal);
  else hipLaunchKernelGGL((mstcn_bwd_b<64>), grid, dim3(NTH), 0, st, dY, dPre, Wd, dX, T, F, dilation, causal);
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
