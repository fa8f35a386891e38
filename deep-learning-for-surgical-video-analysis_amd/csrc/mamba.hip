// Mamba (selective state-space) block kernels for CausalMambaModel (mstcn.py:282-343), which stacks
// mamba_ssm's `Mamba` module (v1, mamba_simple.py; the reference imports it at mstcn.py:9 and builds
// it with d_model = f_maps, d_state 64, d_conv 4, expand 2, mstcn.py:316-322).  Time-major f32
// layout: one video = T consecutive rows; B videos = B*T rows.
//
//   xz  = in_proj(x)                     GEMM (svk_gemm), [BT, 2*Di]; x-half = cols [0, Di), z-half = [Di, 2Di)
//   xc  = silu(causal depthwise conv_K(x-half) + conv_b)          svk_mamba_conv_silu
//   xdb = x_proj(xc)                     GEMM, [BT, R + 2N]  (dt_low | B | C)
//   y   = (scan(xc, softplus(dt_proj(dt_low) + dt_b), A, B, C) + D*xc) * silu(z)   svk_mamba_scan
//   out = x + out_proj(y)                GEMM with the residual fused (CausalMambaModel: x = x + blk(x))
//
// The scan is the published selective-scan recurrence (selective_scan_ref):
//   h_t[n] = exp(delta_t * A[d, n]) * h_{t-1}[n] + delta_t * B_t[n] * u_t ;  y_t = sum_n C_t[n] h_t[n]
// It is sequential in t and parallel over (video, channel d, state n): one 64-lane wave carries
// 64/N channels x N states in registers.  To fill the chip with one video (Di = 128 channels = 32
// workgroups) time is also cut into segments scanned concurrently in two passes (end state + delta sum
// per segment, then a rerun from the folded initial state: h_init = sum over earlier segments of
// exp(A * sum delta) products x end states).  Per 32-step chunk the workgroup stages the (shared across
// channels) dt_low|B|C rows in LDS with coalesced loads, computes delta and u for its channels once,
// runs the recurrence writing C_t[n] h_t[n] into a per-wave LDS tile (rows padded to 65 floats),
// then each lane reduces one time step's row over n (conflict-free: row stride 65) and applies the
// D skip and the silu(z) gate.
#include "svk_common.h"

namespace svk {

constexpr int MB_TC = 16;      // time steps per chunk (LDS ~29 KB at d_state 64: 5 workgroups per CU; sweep: 32 steps (57 KB, 2 per CU) 5.69 M, 16: 6.41 M, 8: 5.66 M frames/s ragged)
constexpr int MB_RMAX = 16;    // dt_rank <= 16 (d_model <= 256)

__global__ __launch_bounds__(256) void mamba_conv_silu_kernel(const float* __restrict__ X, long ldx,
                                                              const float* __restrict__ W,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ Y, int T, long total, int Di,
                                                              int K, const int* __restrict__ tpos) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % Di);
  const long r = i / Di;                 // global row b*T + t
  const int t = tpos ? tpos[r] : (int)(r % T);   // ragged batch: the row's time index inside its video
  float acc = bias ? bias[d] : 0.f;
  for (int k = 0; k < K; ++k) {
    const int dt = K - 1 - k;            // tap k reads x[t - (K-1) + k] (pad K-1, keep first T)
    if (t >= dt) acc += W[d * K + k] * X[(r - dt) * ldx + d];
  }
  Y[r * Di + d] = acc / (1.f + __expf(-acc));
}

__device__ __forceinline__ float softplus20(float s) { return s <= 20.f ? log1pf(__expf(s)) : s; }

// Segmented scan: time is cut into S segments of `seg` steps (blockIdx.z).  OUT = false (pass 1): run
// the recurrence from h = 0 over the segment and store the end state HS[b, z, d, n] and the segment's
// delta sum DS[b, z, d] (its decay is exp(A * sum delta)).  OUT = true (pass 2): fold the earlier
// segments' (decay, end state) pairs into the initial state, rerun the segment and write y.  With one
// segment pass 2 alone is the plain sequential scan.
// Ragged batches (segs != nullptr, gridDim.z == 1): blockIdx.y indexes a table of (video, segment)
// records {first row of the video, its length T_v, segment index z, index of the video's first record};
// a video's records are consecutive, so its segment states HS / DS sit at records sbase .. sbase + S_v - 1.
template <int NS, bool OUT>
__global__ __launch_bounds__(256) void mamba_scan_kernel(const float* __restrict__ U, const float* __restrict__ XD,
                                                         long ldxd, const float* __restrict__ Z, long ldz,
                                                         const float* __restrict__ Wdt, const float* __restrict__ bdt,
                                                         const float* __restrict__ A, const float* __restrict__ Dp,
                                                         float* __restrict__ Y, float* __restrict__ HS,
                                                         float* __restrict__ DS, int T, int Di, int R, int seg,
                                                         float* __restrict__ Yss, const int4* __restrict__ segs) {
  constexpr int CPW = 64 / NS;           // channels per wave
  constexpr int CPB = 4 * CPW;           // channels per workgroup
  constexpr int XW = MB_RMAX + 2 * NS + 1;
  __shared__ float xd[MB_TC][XW];        // dt_low | B | C rows of the chunk
  __shared__ float P[OUT ? 4 : 1][MB_TC][65];   // C_t[n] * h_t[n] per wave
  __shared__ float dl[CPB][MB_TC + 1];   // delta per (channel, t)
  __shared__ float uu[CPB][MB_TC + 1];   // u = xc per (channel, t)

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cl = lane / NS, n = lane - cl * NS;
  const int cw = wave * CPW + cl;        // channel slot within the workgroup
  const int c0 = blockIdx.x * CPB;
  const int d = c0 + cw;
  long row0;
  int z, sbase;
  if (segs) {
    const int4 e = segs[blockIdx.y];
    row0 = e.x;
    T = e.y;
    z = e.z;
    sbase = e.w;
  } else {
    z = blockIdx.z;
    row0 = (long)blockIdx.y * T;
    sbase = blockIdx.y * gridDim.z;
  }
  const float a = d < Di ? A[(long)d * NS + n] : 0.f;
  const int W = R + 2 * NS;
  const int tbeg = z * seg, tend = min(T, tbeg + seg);
  float h = 0.f, dsum = 0.f;
  if (OUT && d < Di) {
    for (int zz = 0; zz < z; ++zz) {
      const long sidx = ((long)sbase + zz) * Di + d;
      h = __expf(a * DS[sidx]) * h + HS[sidx * NS + n];
    }
  }
  // delta/u staging: thread -> fixed channel (256 % CPB == 0), dt_proj row and bias kept in registers
  const int sc = threadIdx.x % CPB, dd = c0 + sc;
  float wdt[MB_RMAX];
#pragma unroll
  for (int r = 0; r < MB_RMAX; ++r) wdt[r] = (r < R && dd < Di) ? Wdt[(long)dd * R + r] : 0.f;
  const float bd = dd < Di ? bdt[dd] : 0.f;
  // the next chunk's dt_low|B|C rows and u values are loaded into registers while the current chunk scans
  constexpr int XR = (MB_TC * (MB_RMAX + 2 * NS) + 255) / 256;
  constexpr int UR = (CPB * MB_TC + 255) / 256;
  float xreg[XR], ureg[UR];
  auto load_chunk = [&](int t0) {
    const int tn = min(MB_TC, tend - t0);
#pragma unroll
    for (int k = 0; k < XR; ++k) {
      const int e = threadIdx.x + k * 256;
      const int r = e / W, c = e - r * W;
      xreg[k] = e < tn * W ? XD[(row0 + t0 + r) * ldxd + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < UR; ++k) {
      const int tl = (threadIdx.x + k * 256) / CPB;
      ureg[k] = (tl < tn && dd < Di) ? U[(row0 + t0 + tl) * Di + dd] : 0.f;
    }
  };
  if (tbeg < tend) load_chunk(tbeg);

  for (int t0 = tbeg; t0 < tend; t0 += MB_TC) {
    const int tn = min(MB_TC, tend - t0);
    __syncthreads();                     // previous chunk's readers of xd / dl / uu are done
#pragma unroll
    for (int k = 0; k < XR; ++k) {
      const int e = threadIdx.x + k * 256;
      const int r = e / W, c = e - r * W;
      if (e < tn * W) xd[r][c] = xreg[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < UR; ++k) {
      const int tl = (threadIdx.x + k * 256) / CPB;
      if (tl < MB_TC) {
        float dv = 0.f;
        if (tl < tn && dd < Di) {
          float s = bd;
#pragma unroll
          for (int r = 0; r < MB_RMAX; ++r)
            if (r < R) s += wdt[r] * xd[tl][r];
          dv = softplus20(s);
        }
        dl[sc][tl] = dv;
        uu[sc][tl] = ureg[k];
      }
    }
    __syncthreads();
    if (t0 + MB_TC < tend) load_chunk(t0 + MB_TC);
    if (OUT) {
#pragma unroll 8
      for (int tl = 0; tl < tn; ++tl) {
        const float dv = dl[cw][tl];
        h = __expf(dv * a) * h + dv * xd[tl][R + n] * uu[cw][tl];
        P[OUT ? wave : 0][tl][lane] = h * xd[tl][R + NS + n];
      }
      __syncthreads();
      if (lane < tn) {
        const long row = row0 + t0 + lane;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
          const int d2 = c0 + wave * CPW + c;
          if (d2 >= Di) break;
          float s = 0.f;
#pragma unroll 16
          for (int k = 0; k < NS; ++k) s += P[OUT ? wave : 0][lane][c * NS + k];
          const float zv = Z[row * ldz + d2];
          const float ys = s + uu[wave * CPW + c][lane] * Dp[d2];
          Y[row * Di + d2] = ys * (zv / (1.f + __expf(-zv)));
          if (Yss) Yss[row * Di + d2] = ys;        // training: the pre-gate output for the z-gate backward
        }
      }
    } else {
#pragma unroll 8
      for (int tl = 0; tl < tn; ++tl) {
        const float dv = dl[cw][tl];
        h = __expf(dv * a) * h + dv * xd[tl][R + n] * uu[cw][tl];
        dsum += dv;
      }
    }
  }
  if (!OUT && d < Di) {
    const long sidx = ((long)sbase + z) * Di + d;
    HS[sidx * NS + n] = h;
    if (n == 0) DS[sidx] = dsum;
  }
}

}  // namespace svk

using namespace svk;

extern "C" int svk_mamba_conv_silu(const float* X, long ldx, const float* W, const float* bias, float* Y, int B,
                                   int T, int Di, int K, void* stream) {
  if (B < 0 || T < 0 || Di <= 0 || K <= 0 || K > 8 || ldx < Di || !X || !W || !Y) {
    set_error("svk_mamba_conv_silu: bad args (B=%d T=%d Di=%d K=%d ldx=%ld)", B, T, Di, K, ldx);
    return SVK_EINVAL;
  }
  const long total = (long)B * T * Di;
  if (total == 0) return SVK_OK;
  hipLaunchKernelGGL(mamba_conv_silu_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, W, bias, Y, T, total, Di, K, nullptr);
  return check_launch("mamba_conv_silu");
}

extern "C" int svk_mamba_conv_silu_ragged(const float* X, long ldx, const float* W, const float* bias, float* Y,
                                          const int* tpos, long rows, int Di, int K, void* stream) {
  if (rows < 0 || Di <= 0 || K <= 0 || K > 8 || ldx < Di || !X || !W || !Y || (rows > 0 && !tpos)) {
    set_error("svk_mamba_conv_silu_ragged: bad args (rows=%ld Di=%d K=%d ldx=%ld)", rows, Di, K, ldx);
    return SVK_EINVAL;
  }
  const long total = rows * Di;
  if (total == 0) return SVK_OK;
  hipLaunchKernelGGL(mamba_conv_silu_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, W, bias, Y, 1, total, Di, K, tpos);
  return check_launch("mamba_conv_silu_ragged");
}

static int mamba_scan_launch(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                             const float* bdt, const float* A, const float* Dp, float* Y, int B, int T, int Di,
                             int N, int R, int seg_len, float* ws, float* Yss, void* stream) {
  if (B < 0 || T < 0 || Di <= 0 || R <= 0 || R > MB_RMAX || (N != 16 && N != 32 && N != 64) ||
      ldxd < R + 2 * N || ldz < Di || !U || !XD || !Z || !Wdt || !bdt || !A || !Dp || !Y || seg_len <= 0 ||
      (seg_len < T && (seg_len % MB_TC != 0 || !ws))) {
    set_error("svk_mamba_scan: bad args (Di=%d N=%d must be 16/32/64, R=%d must be 1..%d, ldxd=%ld, seg_len=%d "
              "must be >= T or a multiple of %d with a workspace)", Di, N, R, MB_RMAX, ldxd, seg_len, MB_TC);
    return SVK_EINVAL;
  }
  if ((long)B * T == 0) return SVK_OK;
  const int S = seg_len >= T ? 1 : (T + seg_len - 1) / seg_len;
  const int seg = S == 1 ? T : seg_len;
  const int cpb = 4 * (64 / N);
  dim3 grid((Di + cpb - 1) / cpb, B, S);
  hipStream_t s = (hipStream_t)stream;
  float* HS = ws;
  float* DS = ws ? ws + (long)B * S * Di * N : nullptr;
#define SVK_MAMBA_LAUNCH(NS)                                                                                   \
  do {                                                                                                          \
    if (S > 1)                                                                                                  \
      hipLaunchKernelGGL((mamba_scan_kernel<NS, false>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt,  \
                         A, Dp, Y, HS, DS, T, Di, R, seg, nullptr, nullptr);                                    \
    hipLaunchKernelGGL((mamba_scan_kernel<NS, true>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt, A, \
                       Dp, Y, HS, DS, T, Di, R, seg, Yss, nullptr);                                             \
  } while (0)
  if (N == 64) SVK_MAMBA_LAUNCH(64);
  else if (N == 32) SVK_MAMBA_LAUNCH(32);
  else SVK_MAMBA_LAUNCH(16);
#undef SVK_MAMBA_LAUNCH
  return check_launch("mamba_scan");
}

extern "C" int svk_mamba_scan(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                              const float* bdt, const float* A, const float* Dp, float* Y, int B, int T, int Di,
                              int N, int R, int seg_len, float* ws, void* stream) {
  return mamba_scan_launch(U, XD, ldxd, Z, ldz, Wdt, bdt, A, Dp, Y, B, T, Di, N, R, seg_len, ws, nullptr, stream);
}

extern "C" int svk_mamba_scan_train(const float* U, const float* XD, long ldxd, const float* Z, long ldz,
                                    const float* Wdt, const float* bdt, const float* A, const float* Dp, float* Y,
                                    float* Yss, int B, int T, int Di, int N, int R, int seg_len, float* ws,
                                    void* stream) {
  if (!Yss) { set_error("svk_mamba_scan_train: Yss is required"); return SVK_EINVAL; }
  return mamba_scan_launch(U, XD, ldxd, Z, ldz, Wdt, bdt, A, Dp, Y, B, T, Di, N, R, seg_len, ws, Yss, stream);
}

extern "C" int svk_mamba_scan_ragged(const float* U, const float* XD, long ldxd, const float* Z, long ldz,
                                     const float* Wdt, const float* bdt, const float* A, const float* Dp, float* Y,
                                     const int* segs, int nseg, int Di, int N, int R, int seg_len, float* ws,
                                     void* stream) {
  if (nseg < 0 || Di <= 0 || R <= 0 || R > MB_RMAX || (N != 16 && N != 32 && N != 64) || ldxd < R + 2 * N ||
      ldz < Di || !U || !XD || !Z || !Wdt || !bdt || !A || !Dp || !Y || seg_len <= 0 || seg_len % MB_TC != 0 ||
      (nseg > 0 && (!segs || !ws || ((uintptr_t)segs & 15)))) {
    set_error("svk_mamba_scan_ragged: bad args (Di=%d N=%d R=%d ldxd=%ld seg_len=%d must be a multiple of %d; "
              "segs 16-byte aligned, workspace required)", Di, N, R, ldxd, seg_len, MB_TC);
    return SVK_EINVAL;
  }
  if (nseg == 0) return SVK_OK;
  const int cpb = 4 * (64 / N);
  dim3 grid((Di + cpb - 1) / cpb, nseg, 1);
  hipStream_t s = (hipStream_t)stream;
  float* HS = ws;
  float* DS = ws + (long)nseg * Di * N;
  const int4* sg = reinterpret_cast<const int4*>(segs);
#define SVK_MAMBA_RLAUNCH(NS)                                                                                  \
  do {                                                                                                          \
    hipLaunchKernelGGL((mamba_scan_kernel<NS, false>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt, A, \
                       Dp, Y, HS, DS, 0, Di, R, seg_len, nullptr, sg);                                          \
    hipLaunchKernelGGL((mamba_scan_kernel<NS, true>), grid, dim3(256), 0, s, U, XD, ldxd, Z, ldz, Wdt, bdt, A,  \
                       Dp, Y, HS, DS, 0, Di, R, seg_len, nullptr, sg);                                          \
  } while (0)
  if (N == 64) SVK_MAMBA_RLAUNCH(64);
  else if (N == 32) SVK_MAMBA_RLAUNCH(32);
  else SVK_MAMBA_RLAUNCH(16);
#undef SVK_MAMBA_RLAUNCH
  return check_launch("mamba_scan_ragged");
}

extern "C" long svk_mamba_scan_ragged_workspace(int nseg, int Di, int N) {
  if (nseg <= 0 || Di <= 0 || N <= 0) return 0;
  return (long)nseg * Di * (N + 1) * (long)sizeof(float);
}

extern "C" long svk_mamba_scan_workspace(int B, int T, int Di, int N, int seg_len) {
  if (B <= 0 || T <= 0 || Di <= 0 || N <= 0 || seg_len <= 0 || seg_len >= T) return 0;
  const long S = (T + seg_len - 1) / seg_len;
  return (long)B * S * Di * (N + 1) * (long)sizeof(float);
}
