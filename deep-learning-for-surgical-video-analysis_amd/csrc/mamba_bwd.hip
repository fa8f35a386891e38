// Backward of the CausalMambaModel block kernels (mamba.hip) for tecno.py's training loop
// (tecno.py:195-259: model.train(), loss.backward(), clip_grad_norm_, AdamW).
//
// Selective scan, per video b, channel d, state n (rows r = b*T + t):
//   delta = softplus(s),  s = bdt[d] + Wdt[d, :] . dt_low[r, :]      a_t = exp(delta_t A[d, n])
//   h_t = a_t h_{t-1} + delta_t B_t[n] u_t                            yss_t = sum_n C_t[n] h_t + D[d] u_t
//   out_t = yss_t * silu(z_t)
// Given dout:  dz = dout yss silu'(z),  g_t = dout silu(z) (= d yss),  dD += g u,  du += g D, and the
// reverse-time recurrence of the state gradient
//   gh_t = C_t[n] g_t + a_{t+1} gh_{t+1}
// with, per step, d delta_t += sum_n gh_t (A a_t h_{t-1} + B_t[n] u_t), dA[d, n] += gh_t delta_t a_t h_{t-1},
// dB_t[n] += sum_d gh_t delta_t u_t, dC_t[n] += sum_d g_t h_t, du_t += sum_n gh_t delta_t B_t[n];
// ds = d delta * sigmoid(s) = d delta * (1 - exp(-delta)) is written out and the dt projection's
// gradients (d dt_low = ds Wdt, dWdt = ds^T dt_low, dbdt = colsum ds) are GEMMs on the host side.
//
// One workgroup = 4 waves = 4 * 64/N channels x N states (lane = (channel, state)), sequential in time:
// pass 1 runs the recurrence forward and checkpoints h at every 16-step chunk start; pass 2 walks the
// chunks backwards, recomputes the chunk's 16 states into registers from its checkpoint, runs the
// reverse recurrence, and reduces the per-lane terms through LDS: over the states of a channel (d delta,
// du) and over the workgroup's channels (dB, dC: one f32 atomic per (row, state) per workgroup into
// the zeroed x_proj-output gradient).  The dt_low | B | C rows of a chunk are staged in LDS as in the
// forward.
//
// Causal depthwise conv + SiLU backward: dpre = dy silu'(pre) (pre recomputed), dx[t] = sum_k W[d, k]
// dpre[t + K - 1 - k] (same video), dW / dbias reduced per 64-channel x 256-row tile in registers and
// LDS, one atomic per weight per tile.
#include "svk_common.h"

namespace svk {

constexpr int MBB_TC = 16;     // time steps per backward chunk (8: 416k vs 453-471k frames/s tecno_train)
constexpr int MBB_RMAX = 16;

__device__ __forceinline__ float softplus_bwd20(float s) { return s <= 20.f ? log1pf(__expf(s)) : s; }

// Staging of one chunk of rows (shared by the segment passes): the dt_low | B | C rows into LDS, and per
// (channel, step) delta = softplus(s), u and — mode >= 1 — g = dout * silu(z) (the gradient of yss);
// mode 2 also writes dz and accumulates the D-skip gradient.
template <int NS>
struct ScanBwdSmem {
  static constexpr int TC = MBB_TC, CPW = 64 / NS, CPB = 4 * CPW, XW = MBB_RMAX + 2 * NS + 1;
  float xd[TC][XW];
  float dl[CPB][TC + 1], uu[CPB][TC + 1], gy[CPB][TC + 1];
};

template <int NS>
__device__ __forceinline__ void scan_bwd_stage(ScanBwdSmem<NS>& sm, int t0, int tn, int mode, const float* XD, long ldxd,
                                               const float* U, const float* Z, long ldz, const float* dOut,
                                               const float* Yss, float* dZ, long lddz, long row0, int W, int R, int Di,
                                               int sc, int dd, const float* wdt, float bd, float& dDacc) {
  constexpr int TC = MBB_TC, CPB = ScanBwdSmem<NS>::CPB;
  __syncthreads();                         // earlier readers of the chunk buffers are done
  for (int e = threadIdx.x; e < tn * W; e += 256) {
    const int r = e / W, c = e - r * W;
    sm.xd[r][c] = XD[(row0 + t0 + r) * ldxd + c];
  }
  __syncthreads();
  for (int tl = threadIdx.x / CPB; tl < TC; tl += 256 / CPB) {
    float dv = 0.f, uv = 0.f, g = 0.f;
    if (tl < tn && dd < Di) {
      const long row = row0 + t0 + tl;
      float s = bd;
#pragma unroll
      for (int r = 0; r < MBB_RMAX; ++r)
        if (r < R) s += wdt[r] * sm.xd[tl][r];
      dv = softplus_bwd20(s);
      uv = U[row * Di + dd];
      if (mode >= 1) {
        const float zv = Z[row * ldz + dd], go = dOut[row * Di + dd];
        const float sg = 1.f / (1.f + __expf(-zv));
        g = go * zv * sg;                                                 // d yss = dout * silu(z)
        if (mode == 2) {
          dZ[row * lddz + dd] = go * Yss[row * Di + dd] * sg * (1.f + zv * (1.f - sg));
          dDacc += g * uv;
        }
      }
    }
    sm.dl[sc][tl] = dv;
    sm.uu[sc][tl] = uv;
    sm.gy[sc][tl] = g;
  }
  __syncthreads();
}

// Time is split into segments of seg_len steps (a multiple of the 16-step chunk), one workgroup per
// (channel group, segment, video), so a single video's backward spreads over the chip:
//   pass S (mamba_scan_bwd_seg): per segment, the forward recurrence from a zero state gives the local
//     end state E and the decay product P = prod a = exp(A sum delta); the reverse recurrence from a zero
//     carry gives the local carry-out M = a_first gh_first.  Stored per (video, segment, channel, state);
//   main pass: the segment's true start state H_k = sum_{j<k} (prod_{j<i<k} P_i) E_j and its true carry-in
//     G_k = M_{k+1} + P_{k+1} G_{k+1} (both linear recurrences over the segment summaries, folded by every
//     workgroup in a short loop), then the exact per-segment backward below.
template <int NS>
__global__ __launch_bounds__(256) void mamba_scan_bwd_seg(
    const float* __restrict__ U, const float* __restrict__ XD, long ldxd, const float* __restrict__ Z, long ldz,
    const float* __restrict__ Wdt, const float* __restrict__ bdt, const float* __restrict__ A,
    const float* __restrict__ dOut, float* __restrict__ SE, float* __restrict__ SP, float* __restrict__ SM, int T,
    int Di, int R, int seg_len) {
  using SM_ = ScanBwdSmem<NS>;
  constexpr int TC = MBB_TC, CPW = SM_::CPW, CPB = SM_::CPB;
  __shared__ SM_ sm;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cl = lane / NS, n = lane - cl * NS;
  const int cw = wave * CPW + cl;
  const int c0 = blockIdx.x * CPB, d = c0 + cw;
  const int k = blockIdx.y, nseg = gridDim.y, b = blockIdx.z;
  const long row0 = (long)b * T;
  const float a_ = d < Di ? A[(long)d * NS + n] : 0.f;
  const int W = R + 2 * NS;
  const int sc = threadIdx.x % CPB, dd = c0 + sc;
  float wdt[MBB_RMAX];
#pragma unroll
  for (int r = 0; r < MBB_RMAX; ++r) wdt[r] = (r < R && dd < Di) ? Wdt[(long)dd * R + r] : 0.f;
  const float bd = dd < Di ? bdt[dd] : 0.f;
  float unused = 0.f;
  const int ts = k * seg_len, te = min(T, ts + seg_len);
  float h = 0.f, ssum = 0.f;
  for (int t0 = ts; t0 < te; t0 += TC) {
    const int tn = min(TC, te - t0);
    scan_bwd_stage<NS>(sm, t0, tn, 0, XD, ldxd, U, Z, ldz, dOut, nullptr, nullptr, 0, row0, W, R, Di, sc, dd, wdt, bd,
                       unused);
    for (int tl = 0; tl < tn; ++tl) {
      const float dv = sm.dl[cw][tl];
      h = __expf(dv * a_) * h + dv * sm.xd[tl][R + n] * sm.uu[cw][tl];
      ssum += dv;
    }
  }
  float carry = 0.f;
  const int nch = (te - ts + TC - 1) / TC;
  for (int c = nch - 1; c >= 0; --c) {
    const int t0 = ts + c * TC, tn = min(TC, te - t0);
    scan_bwd_stage<NS>(sm, t0, tn, 1, XD, ldxd, U, Z, ldz, dOut, nullptr, nullptr, 0, row0, W, R, Di, sc, dd, wdt, bd,
                       unused);
    for (int tl = tn - 1; tl >= 0; --tl) {
      const float dv = sm.dl[cw][tl];
      carry = __expf(dv * a_) * (sm.xd[tl][R + NS + n] * sm.gy[cw][tl] + carry);
    }
  }
  if (d < Di) {
    const long o = (((long)b * nseg + k) * Di + d) * NS + n;
    SE[o] = h;
    SP[o] = __expf(a_ * ssum);
    SM[o] = carry;
  }
}

template <int NS>
__global__ __launch_bounds__(256) void mamba_scan_bwd_kernel(
    const float* __restrict__ U, const float* __restrict__ XD, long ldxd, const float* __restrict__ Z, long ldz,
    const float* __restrict__ Wdt, const float* __restrict__ bdt, const float* __restrict__ A,
    const float* __restrict__ Dp, const float* __restrict__ Yss, const float* __restrict__ dOut,
    float* __restrict__ dU, float* __restrict__ dZ, long lddz, float* __restrict__ dS, float* __restrict__ dXD,
    long lddxd, float* __restrict__ dA, float* __restrict__ dD, float* __restrict__ HCK, const float* __restrict__ SE,
    const float* __restrict__ SP, const float* __restrict__ SMv, int T, int Di, int R, int seg_len) {
  using SM_ = ScanBwdSmem<NS>;
  constexpr int TC = MBB_TC, CPW = SM_::CPW, CPB = SM_::CPB;
  __shared__ SM_ sm;
  __shared__ float P1[4][TC][65], P2[4][TC][65], Q1[4][TC][65], Q2[4][TC][65];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cl = lane / NS, n = lane - cl * NS;
  const int cw = wave * CPW + cl;
  const int c0 = blockIdx.x * CPB;
  const int d = c0 + cw;
  const int k = blockIdx.y, nseg = gridDim.y, b = blockIdx.z;
  const long row0 = (long)b * T;
  const float a_ = d < Di ? A[(long)d * NS + n] : 0.f;
  const int W = R + 2 * NS;
  const int nchunk = (T + TC - 1) / TC;
  const int ts = k * seg_len, te = min(T, ts + seg_len);
  const int cs = ts / TC, ce = (te + TC - 1) / TC;       // this segment's chunks
  const int sc = threadIdx.x % CPB, dd = c0 + sc;
  float wdt[MBB_RMAX];
#pragma unroll
  for (int r = 0; r < MBB_RMAX; ++r) wdt[r] = (r < R && dd < Di) ? Wdt[(long)dd * R + r] : 0.f;
  const float bd = dd < Di ? bdt[dd] : 0.f;
  float dDacc = 0.f;

  // the segment's true start state and carry-in from the segment summaries
  float h = 0.f, carry = 0.f;
  if (nseg > 1 && d < Di) {
    const long base = (long)b * nseg * Di * NS + (long)d * NS + n, step = (long)Di * NS;
    for (int j = 0; j < k; ++j) h = SP[base + j * step] * h + SE[base + j * step];
    for (int j = nseg - 1; j > k; --j) carry = SMv[base + j * step] + SP[base + j * step] * carry;
  }

  // pass 1: forward recurrence over the segment, h checkpoint at each chunk start
  for (int c = cs; c < ce; ++c) {
    const int t0 = c * TC, tn = min(TC, te - t0);
    if (d < Di) HCK[(((long)b * nchunk + c) * Di + d) * NS + n] = h;
    scan_bwd_stage<NS>(sm, t0, tn, 0, XD, ldxd, U, Z, ldz, dOut, Yss, dZ, lddz, row0, W, R, Di, sc, dd, wdt, bd, dDacc);
    for (int tl = 0; tl < tn; ++tl) {
      const float dv = sm.dl[cw][tl];
      h = __expf(dv * a_) * h + dv * sm.xd[tl][R + n] * sm.uu[cw][tl];
    }
  }
  __threadfence_block();

  // pass 2: the segment's chunks backwards
  float dAacc = 0.f;
  for (int c = ce - 1; c >= cs; --c) {
    const int t0 = c * TC, tn = min(TC, te - t0);
    const float hstart = d < Di ? HCK[(((long)b * nchunk + c) * Di + d) * NS + n] : 0.f;
    scan_bwd_stage<NS>(sm, t0, tn, 2, XD, ldxd, U, Z, ldz, dOut, Yss, dZ, lddz, row0, W, R, Di, sc, dd, wdt, bd, dDacc);
    float hh[TC];
    float hc = hstart;
#pragma unroll
    for (int tl = 0; tl < TC; ++tl) {
      if (tl < tn) {
        const float dv = sm.dl[cw][tl];
        hc = __expf(dv * a_) * hc + dv * sm.xd[tl][R + n] * sm.uu[cw][tl];
      }
      hh[tl] = hc;
    }
#pragma unroll
    for (int tl = TC - 1; tl >= 0; --tl) {
      if (tl < tn) {
        const float dv = sm.dl[cw][tl], uv = sm.uu[cw][tl], g = sm.gy[cw][tl];
        const float Bn = sm.xd[tl][R + n], Cn = sm.xd[tl][R + NS + n];
        const float at = __expf(dv * a_);
        const float hp = tl > 0 ? hh[tl - 1] : hstart;
        const float gh = Cn * g + carry;
        P1[wave][tl][lane] = gh * (a_ * at * hp + Bn * uv);
        P2[wave][tl][lane] = gh * dv * Bn;
        Q1[wave][tl][lane] = gh * dv * uv;
        Q2[wave][tl][lane] = g * hh[tl];
        dAacc += gh * dv * at * hp;
        carry = at * gh;
      }
    }
    __syncthreads();
    // per (channel, t): d delta and du summed over the channel's states
    for (int e = threadIdx.x; e < CPB * TC; e += 256) {
      const int cw2 = e % CPB, tl = e / CPB;
      const int d2 = c0 + cw2;
      if (tl >= tn || d2 >= Di) continue;
      const int w2 = cw2 / CPW, cl2 = cw2 - w2 * CPW;
      float sd = 0.f, su = 0.f;
#pragma unroll 8
      for (int q = 0; q < NS; ++q) {
        sd += P1[w2][tl][cl2 * NS + q];
        su += P2[w2][tl][cl2 * NS + q];
      }
      const long row = row0 + t0 + tl;
      const float dv = sm.dl[cw2][tl];
      dS[row * Di + d2] = sd * (1.f - __expf(-dv));                       // sigmoid(s) = 1 - exp(-softplus(s))
      dU[row * Di + d2] = su + sm.gy[cw2][tl] * Dp[d2];
    }
    // per (t, state): dB and dC summed over the workgroup's channels
    for (int e = threadIdx.x; e < TC * NS; e += 256) {
      const int tl = e / NS, q = e - tl * NS;
      if (tl >= tn) continue;
      float sb = 0.f, scc = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 4; ++w2)
#pragma unroll
        for (int cl2 = 0; cl2 < CPW; ++cl2) {
          if (c0 + w2 * CPW + cl2 < Di) {
            sb += Q1[w2][tl][cl2 * NS + q];
            scc += Q2[w2][tl][cl2 * NS + q];
          }
        }
      const long row = row0 + t0 + tl;
      atomicAdd(dXD + row * lddxd + R + q, sb);
      atomicAdd(dXD + row * lddxd + R + NS + q, scc);
    }
  }
  if (d < Di) atomicAdd(dA + (long)d * NS + n, dAacc);
  // dD: every staging thread owns one channel; reduce the threads of the same channel through LDS
  __syncthreads();
  float* red = &P1[0][0][0];
  red[threadIdx.x] = dDacc;
  __syncthreads();
  if (threadIdx.x < CPB && c0 + threadIdx.x < Di) {
    float s = 0.f;
    for (int i = threadIdx.x; i < 256; i += CPB) s += red[i];
    atomicAdd(dD + c0 + threadIdx.x, s);
  }
}

// ---- causal depthwise conv + SiLU backward ------------------------------------------------------
// tile = 64 channels x 256 rows (4 row groups of 64); thread (channel c, group g) walks its 64 rows
__global__ __launch_bounds__(256) void mamba_conv_silu_bwd_w(const float* __restrict__ X, long ldx,
                                                             const float* __restrict__ Wc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ dY, float* __restrict__ dPre,
                                                             float* __restrict__ dW, float* __restrict__ db, int T,
                                                             long rows, int Di, int K) {
  __shared__ float red[4][64][9];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int d = blockIdx.x * 64 + c;
  const long r0 = (long)blockIdx.y * 256 + g * 64;
  float w[8], acc[8], accb = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) { w[k] = (k < K && d < Di) ? Wc[(long)d * K + k] : 0.f; acc[k] = 0.f; }
  const float bv = (bias && d < Di) ? bias[d] : 0.f;
  if (d < Di) {
    for (long r = r0; r < min(r0 + 64, rows); ++r) {
      const int t = (int)(r % T);
      float xv[8];
      float pre = bv;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int dt = K - 1 - k;
        xv[k] = (k < K && t >= dt) ? X[(r - dt) * ldx + d] : 0.f;
        pre += w[k] * xv[k];
      }
      const float sg = 1.f / (1.f + __expf(-pre));
      const float dp = dY[r * Di + d] * sg * (1.f + pre * (1.f - sg));
      dPre[r * Di + d] = dp;
      accb += dp;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += dp * xv[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[g][c][k] = acc[k];
  red[g][c][8] = accb;
  __syncthreads();
  if (g == 0 && d < Di) {
    for (int k = 0; k <= K; ++k) {
      const int kk = k == K ? 8 : k;
      const float s = red[0][c][kk] + red[1][c][kk] + red[2][c][kk] + red[3][c][kk];
      if (k < K) atomicAdd(dW + (long)d * K + k, s);
      else if (db) atomicAdd(db + d, s);
    }
  }
}

__global__ __launch_bounds__(256) void mamba_conv_silu_bwd_x(const float* __restrict__ dPre,
                                                             const float* __restrict__ Wc, float* __restrict__ dX,
                                                             long lddx, int T, long total, int Di, int K) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % Di);
  const long r = i / Di;
  const int t = (int)(r % T);
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    const int dt = K - 1 - k;            // x[t] feeds output t + dt through tap k
    if (t + dt < T) s += Wc[(long)d * K + k] * dPre[(r + dt) * Di + d];
  }
  dX[r * lddx + d] = s;
}

}  // namespace svk

using namespace svk;

// segment length for the backward: enough (channel group, segment, video) workgroups to fill the chip
static int scan_bwd_seg_len(int B, int T, int Di, int N) {
  const int groups = B * ((Di + 4 * (64 / N) - 1) / (4 * (64 / N)));
  int nseg = std::max(1, std::min(512 / std::max(groups, 1), (T + 63) / 64));
  int seg = (T + nseg - 1) / nseg;
  return (seg + MBB_TC - 1) / MBB_TC * MBB_TC;
}

extern "C" long svk_mamba_scan_bwd_workspace(int B, int T, int Di, int N) {
  if (B <= 0 || T <= 0 || Di <= 0 || N <= 0) return 0;
  const int seg = scan_bwd_seg_len(B, T, Di, N), nseg = (T + seg - 1) / seg;
  const long hck = (long)B * ((T + MBB_TC - 1) / MBB_TC) * Di * N;
  const long sums = nseg > 1 ? 3L * B * nseg * Di * N : 0;
  return (hck + sums) * (long)sizeof(float);
}

extern "C" int svk_mamba_scan_bwd(const float* U, const float* XD, long ldxd, const float* Z, long ldz,
                                  const float* Wdt, const float* bdt, const float* A, const float* Dp,
                                  const float* Yss, const float* dOut, float* dU, float* dZ, long lddz, float* dS,
                                  float* dXD, long lddxd, float* dA, float* dD, int B, int T, int Di, int N, int R,
                                  float* ws, void* stream) {
  if (B < 0 || T < 0 || Di <= 0 || R <= 0 || R > MBB_RMAX || (N != 16 && N != 32 && N != 64) || ldxd < R + 2 * N ||
      ldz < Di || lddz < Di || lddxd < R + 2 * N || !U || !XD || !Z || !Wdt || !bdt || !A || !Dp || !Yss || !dOut ||
      !dU || !dZ || !dS || !dXD || !dA || !dD || !ws) {
    set_error("svk_mamba_scan_bwd: bad args (Di=%d N=%d R=%d)", Di, N, R);
    return SVK_EINVAL;
  }
  if ((long)B * T == 0) return SVK_OK;
  const int cpb = 4 * (64 / N);
  const int seg = scan_bwd_seg_len(B, T, Di, N), nseg = (T + seg - 1) / seg;
  dim3 grid((Di + cpb - 1) / cpb, nseg, B);
  hipStream_t s = (hipStream_t)stream;
  float* hck = ws;
  const long nh = (long)B * ((T + MBB_TC - 1) / MBB_TC) * Di * N;
  float *SE = ws + nh, *SP = SE + (long)B * nseg * Di * N, *SMv = SP + (long)B * nseg * Di * N;
#define SVK_MAMBA_BWD(NS)                                                                                       \
  do {                                                                                                          \
    if (nseg > 1)                                                                                               \
      hipLaunchKernelGGL((mamba_scan_bwd_seg<NS>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt, A, dOut, \
                         SE, SP, SMv, T, Di, R, seg);                                                           \
    hipLaunchKernelGGL((mamba_scan_bwd_kernel<NS>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt, A, Dp,  \
                       Yss, dOut, dU, dZ, lddz, dS, dXD, lddxd, dA, dD, hck, SE, SP, SMv, T, Di, R, seg);        \
  } while (0)
  if (N == 64) SVK_MAMBA_BWD(64);
  else if (N == 32) SVK_MAMBA_BWD(32);
  else SVK_MAMBA_BWD(16);
#undef SVK_MAMBA_BWD
  return check_launch("mamba_scan_bwd");
}

extern "C" int svk_mamba_conv_silu_bwd(const float* X, long ldx, const float* W, const float* bias, const float* dY,
                                       float* dPre, float* dX, long lddx, float* dW, float* db, int B, int T, int Di,
                                       int K, void* stream) {
  if (B < 0 || T < 0 || Di <= 0 || K <= 0 || K > 8 || ldx < Di || lddx < Di || !X || !W || !dY || !dPre || !dX ||
      !dW) {
    set_error("svk_mamba_conv_silu_bwd: bad args (Di=%d K=%d)", Di, K);
    return SVK_EINVAL;
  }
  const long rows = (long)B * T;
  if (rows == 0) return SVK_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mamba_conv_silu_bwd_w, dim3((unsigned)((Di + 63) / 64), (unsigned)((rows + 255) / 256)),
                     dim3(256), 0, s, X, ldx, W, bias, dY, dPre, dW, db, T, rows, Di, K);
  const long total = rows * Di;
  hipLaunchKernelGGL(mamba_conv_silu_bwd_x, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, dPre, W, dX, lddx,
                     T, total, Di, K);
  return check_launch("mamba_conv_silu_bwd");
}
