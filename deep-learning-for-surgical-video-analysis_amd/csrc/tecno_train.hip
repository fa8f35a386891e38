// Temporal-model training step pieces (tecno.py:195-259): the per-stage phase loss and its gradient,
// the global gradient norm of clip_grad_norm_ and torch.optim.AdamW — each one launch, every scalar
// that changes between steps (step count, learning rate) read from device memory so the whole step
// replays from a HIP graph.
#include "svk_common.h"

namespace svk {

constexpr int NORM_PARTS = 256;   // fixed partial-sum count of the gradient norm (deterministic, no atomics)

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// One workgroup: pass 1 sums the class weights of the labels (CrossEntropyLoss(weight) 'mean' divides by
// it), pass 2 walks every (stage, frame) row: weighted NLL over the P phase logits, SmoothL1 (beta 1,
// 'mean' over T x P) over the P anticipation outputs, and writes the gradient of
//   loss = (1/S) sum_s CE_s + (1/S) sum_s SmoothL1_s        (tecno.py:237-254)
// loss[0] = clc term, loss[1] = anticipation term, loss[2] = correct argmax count of the last stage.
__global__ __launch_bounds__(1024) void tecno_loss_kernel(const float* __restrict__ Z, long ld, long sstride, int S,
                                                          int T, int P, const long* __restrict__ labels,
                                                          const float* __restrict__ ant, const float* __restrict__ cw,
                                                          float* __restrict__ loss, float* __restrict__ dZ) {
  __shared__ float red[16];
  float wsum = 0.f;
  for (int t = threadIdx.x; t < T; t += blockDim.x) wsum += cw ? cw[labels[t]] : 1.f;
  const float W = block_sum(wsum, red);
  const float gce = 1.f / (W * S), gl1 = 1.f / ((float)T * P * S);
  float ce = 0.f, l1 = 0.f, corr = 0.f;
  for (long r = threadIdx.x; r < (long)S * T; r += blockDim.x) {
    const int s = (int)(r / T), t = (int)(r - (long)s * T);
    const float* z = Z + s * sstride + (long)t * ld;
    float* dz = dZ + s * sstride + (long)t * ld;
    const long y = labels[t];
    float m = -INFINITY;
    int am = 0;
    for (int k = 0; k < P; ++k) {
      if (z[k] > m) { m = z[k]; am = k; }
    }
    float se = 0.f;
    for (int k = 0; k < P; ++k) se += expf(z[k] - m);
    const float wy = cw ? cw[y] : 1.f;
    ce += wy * (logf(se) + m - z[y]);
    if (s == S - 1 && am == y) corr += 1.f;
    const float inv = 1.f / se;
    for (int k = 0; k < P; ++k) dz[k] = wy * gce * (expf(z[k] - m) * inv - (k == y ? 1.f : 0.f));
    for (int k = 0; k < P; ++k) {
      const float d = z[P + k] - ant[(long)t * P + k];
      const float ad = fabsf(d);
      l1 += ad < 1.f ? 0.5f * d * d : ad - 0.5f;
      dz[P + k] = gl1 * (ad < 1.f ? d : (d > 0.f ? 1.f : -1.f));
    }
  }
  ce = block_sum(ce, red);
  l1 = block_sum(l1, red);
  corr = block_sum(corr, red);
  if (threadIdx.x == 0) {
    loss[0] = ce / (W * S);
    loss[1] = l1 / ((float)T * P * S);
    loss[2] = corr;
  }
}

// Partial sums of squares (NORM_PARTS blocks, grid-stride); block 0 also advances the optimizer's
// device step counter (read by adamw_kernel, which runs after this kernel on the stream).
__global__ __launch_bounds__(256) void grad_sqnorm_kernel(const float* __restrict__ g, long n,
                                                          float* __restrict__ part, long long* __restrict__ step) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += g[i] * g[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    if (blockIdx.x == 0 && step) step[0] += 1;
  }
}

// clip_grad_norm_(max_norm) then torch.optim.AdamW (decoupled weight decay, bias-corrected moments):
//   g *= min(max_norm / (||g|| + 1e-6), 1);  p *= 1 - lr wd;  m += (1 - b1)(g - m);
//   v = b2 v + (1 - b2) g^2;  p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// The clipped gradient is written back (clip_grad_norm_ scales .grad in place).
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, long n, const float* __restrict__ part,
                                                    float max_norm, const float* __restrict__ lr_p, float b1, float b2,
                                                    float eps, float wd, const long long* __restrict__ step) {
  __shared__ float coef_s;
  if (threadIdx.x < 64) {
    float s = 0.f;
    if (part)
      for (int i = threadIdx.x; i < NORM_PARTS; i += 64) s += part[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) coef_s = part && max_norm > 0.f ? fminf(max_norm / (sqrtf(s) + 1e-6f), 1.f) : 1.f;
  }
  __syncthreads();
  const float coef = coef_s, lr = lr_p[0];
  const double t = (double)step[0];
  const float bc1 = (float)(1.0 - pow((double)b1, t)), bc2s = (float)sqrt(1.0 - pow((double)b2, t));
  const float step_size = lr / bc1, decay = 1.f - lr * wd;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * coef;
    g[i] = gi;
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] * decay - step_size * mi / (sqrtf(vi) / bc2s + eps);
  }
}

__global__ void neg_exp_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = -expf(x[i]);
}

}  // namespace svk

using namespace svk;

extern "C" int svk_neg_exp(const float* X, float* Y, long n, void* stream) {
  if (n < 0 || !X || !Y) { set_error("svk_neg_exp: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  hipLaunchKernelGGL(neg_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, X, Y, n);
  return check_launch("neg_exp");
}

extern "C" int svk_tecno_loss(const float* logits, long ld, long sstride, int S, int T, int P, const long* labels,
                              const float* ant_targets, const float* class_w, float* loss, float* dlogits,
                              void* stream) {
  if (S <= 0 || T <= 0 || P <= 0 || ld < 2 * P || sstride < (long)T * ld || !logits || !labels || !ant_targets ||
      !loss || !dlogits) {
    set_error("svk_tecno_loss: bad args (S=%d T=%d P=%d)", S, T, P);
    return SVK_EINVAL;
  }
  hipLaunchKernelGGL(tecno_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, logits, ld, sstride, S, T, P,
                     labels, ant_targets, class_w, loss, dlogits);
  return check_launch("tecno_loss");
}

extern "C" int svk_norm_parts(void) { return NORM_PARTS; }

extern "C" int svk_grad_sqnorm(const float* g, long n, float* partials, long long* step, void* stream) {
  if (n < 0 || !g || !partials) { set_error("svk_grad_sqnorm: bad args"); return SVK_EINVAL; }
  hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(NORM_PARTS), dim3(256), 0, (hipStream_t)stream, g, n, partials, step);
  return check_launch("grad_sqnorm");
}

extern "C" int svk_adamw(float* p, float* g, float* m, float* v, long n, const float* partials, float max_norm,
                         const float* lr, float beta1, float beta2, float eps, float weight_decay,
                         const long long* step, void* stream) {
  if (n < 0 || !p || !g || !m || !v || !lr || !step) { set_error("svk_adamw: bad args"); return SVK_EINVAL; }
  if (n == 0) return SVK_OK;
  const long blocks = std::min<long>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, partials,
                     max_norm, lr, beta1, beta2, eps, weight_decay, step);
  return check_launch("adamw");
}
