// Relaxed-boundary phase-recognition metrics (eval_and_vis.py:35-161, the Cholec80 Evaluate.m rules):
// integer counts per video, one workgroup per video, so the host forms the reference's float64 ratios
// from exact integers.
//
//   diff = pred - gt;  for every maximal run [s, e) of one ground-truth phase p, t = min(tol, e - s):
//   diff values in the run's first t frames ("head") and last t frames ("tail") are forgiven (set to 0)
//   when they match the phase's rule:  p in {3, 4}: head -1, tail +1/+2;  p in {5, 6}: head -1/-2,
//   tail +1/+2;  otherwise head -1, tail +1 (decisions on the ORIGINAL diff; head and tail may overlap).
//   Per phase: TP = #(union of gt==p, pred==p with forgiven diff 0), |union|, #pred==p, #gt==p;
//   total = #(forgiven diff == 0).
//
// Run boundaries come from two block-wide scans over per-thread chunks (last run start at or before
// each frame: inclusive max-scan; first run end at or after: suffix min-scan), counts from LDS atomics.
#include "svk_common.h"

namespace svk {

constexpr int MT = 1024;          // threads per video
constexpr int MP_MAX = 16;        // phases

__device__ __forceinline__ bool head_forgiven(int p, long long d) {
  if (p == 5 || p == 6) return d == -1 || d == -2;
  return d == -1;
}
__device__ __forceinline__ bool tail_forgiven(int p, long long d) {
  if (p >= 3 && p <= 6) return d == 1 || d == 2;
  return d == 1;
}

__global__ __launch_bounds__(MT) void phase_metrics_kernel(const long long* __restrict__ gt,
                                                           const long long* __restrict__ pred,
                                                           const long long* __restrict__ offs, int P, int tol,
                                                           long long* __restrict__ out) {
  __shared__ int sc[MT];
  __shared__ unsigned long long cnt[1 + 4 * MP_MAX];
  const int v = blockIdx.x, tid = threadIdx.x;
  const long long o0 = offs[v];
  const int T = (int)(offs[v + 1] - o0);
  const long long* g = gt + o0;
  const long long* q = pred + o0;
  for (int i = tid; i < 1 + 4 * P; i += MT) cnt[i] = 0;
  const int ch = (T + MT - 1) / MT;
  const int c0 = min(T, tid * ch), c1 = min(T, c0 + ch);
  // run starts: inclusive max-scan of "last start in my chunk"
  int last = -1;
  for (int i = c0; i < c1; ++i)
    if (i == 0 || g[i] != g[i - 1]) last = i;
  sc[tid] = last;
  __syncthreads();
  for (int o = 1; o < MT; o <<= 1) {
    const int x = tid >= o ? sc[tid - o] : -1;
    __syncthreads();
    sc[tid] = max(sc[tid], x);
    __syncthreads();
  }
  const int start_carry = tid > 0 ? sc[tid - 1] : -1;
  __syncthreads();
  // run ends (exclusive): suffix min-scan of "first end in my chunk"
  int first = 0x7fffffff;
  for (int i = c1 - 1; i >= c0; --i)
    if (i == T - 1 || g[i] != g[i + 1]) first = i + 1;
  sc[tid] = first;
  __syncthreads();
  for (int o = 1; o < MT; o <<= 1) {
    const int x = tid + o < MT ? sc[tid + o] : 0x7fffffff;
    __syncthreads();
    sc[tid] = min(sc[tid], x);
    __syncthreads();
  }
  const int end_carry = tid + 1 < MT ? sc[tid + 1] : 0x7fffffff;
  // per frame: forgiven diff, counts (per-thread total, LDS atomics per phase)
  auto is_end = [&](int j) { return j == T - 1 || g[j] != g[j + 1]; };
  unsigned long long tot = 0;
  int s = start_carry, e_next = 0;
  for (int i = c0; i < c1; ++i) {
    if (i == 0 || g[i] != g[i - 1]) s = i;
    if (i == c0 || i == s) {               // entering a run: find its end (inside the chunk or after it)
      int j = i;
      while (j < c1 && !is_end(j)) ++j;
      e_next = j < c1 ? j + 1 : end_carry;
    }
    const int e = e_next;
    const int p = (int)g[i];
    const long long d = q[i] - g[i];
    const int t = min(tol, e - s);
    bool fz = d == 0;
    if (!fz && p >= 0 && p < P) {
      if (i - s < t && head_forgiven(p, d)) fz = true;
      if (e - i <= t && tail_forgiven(p, d)) fz = true;
    }
    tot += fz;
    const int pp = (int)q[i];
    if (p >= 0 && p < P) {
      atomicAdd(&cnt[1 + 4 * p + 1], 1ull);                 // union (gt side)
      atomicAdd(&cnt[1 + 4 * p + 3], 1ull);                 // gt count
      if (fz) atomicAdd(&cnt[1 + 4 * p + 0], 1ull);         // TP
    }
    if (pp >= 0 && pp < P) {
      atomicAdd(&cnt[1 + 4 * pp + 2], 1ull);                // pred count
      if (pp != p) {                                        // union (pred side, not already counted)
        atomicAdd(&cnt[1 + 4 * pp + 1], 1ull);
        if (fz) atomicAdd(&cnt[1 + 4 * pp + 0], 1ull);
      }
    }
  }
  atomicAdd(&cnt[0], tot);
  __syncthreads();
  for (int i = tid; i < 1 + 4 * P; i += MT) out[(long)v * (2 + 4 * P) + 1 + i] = (long long)cnt[i];
  if (tid == 0) out[(long)v * (2 + 4 * P)] = T;
}

}  // namespace svk

using namespace svk;

extern "C" int svk_phase_metrics(const long long* gt, const long long* pred, const long long* offsets, int V, int P,
                                 int tolerance, long long* counts, void* stream) {
  if (V < 0 || P <= 0 || P > MP_MAX || tolerance < 0 || !gt || !pred || !offsets || !counts) {
    set_error("svk_phase_metrics: bad args (P=%d <= %d)", P, MP_MAX);
    return SVK_EINVAL;
  }
  if (V == 0) return SVK_OK;
  hipLaunchKernelGGL(phase_metrics_kernel, dim3(V), dim3(MT), 0, (hipStream_t)stream, gt, pred, offsets, P, tolerance,
                     counts);
  return check_launch("phase_metrics");
}
