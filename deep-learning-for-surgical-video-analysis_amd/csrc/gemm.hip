// MFMA GEMM with fused epilogue, and implicit-GEMM NHWC Conv2d, for gfx950.
//
//   C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]
//
// Both operands are K-contiguous (activations [M, K] token-major, nn.Linear weights
// [N, K]), which is exactly the MFMA operand layout: lane l of a 16x16x32 bf16 MFMA
// holds 8 consecutive k of row (l & 15), so every fragment read is one 16-byte LDS
// read and every global load is a 16-byte vector.
//
// Tile: BM x BN x 32, 256 threads = 4 waves arranged 2 x 2, each wave owning a
// (BM/2) x (BN/2) sub-tile of 16x16 MFMA blocks.  LDS is double-buffered; the next
// K-tile is fetched into registers while the MFMAs of the current one run (one
// __syncthreads per K-step).
//
// dtype f32 uses v_mfma_f32_16x16x4_f32 (exact f32 products, the parity path): the
// 8 k a lane holds for one 32-deep K-step are consumed by 8 MFMAs, MFMA s using
// element s of every lane group — a permutation of the k order inside the step,
// which leaves the dot product mathematically unchanged.
//
// ASRC = 1 turns the A loader into an im2col gather from an NHWC map (implicit-GEMM
// convolution, weights packed [Cout][kh][kw][Cin] so that k = (i*kw + j)*Cin + ci).
#include "svk_common.h"

namespace svk {

constexpr int BK = 32;
constexpr int NTHREADS = 256;

struct GemmArgs {
  const void* A; long lda;
  const void* W; long ldw;
  const float* bias;
  const void* R; long ldr;
  void* C; long ldc;
  int M, N, K, act;
  // implicit-GEMM conv geometry (ASRC == 1)
  int H, Wd, Cin, OH, OW, kw, stride, pad;
};

template <typename T> struct Chunk { T v[8]; };

template <typename T>
__device__ __forceinline__ void load_vec8(const T* p, Chunk<T>& c) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(c.v) = *reinterpret_cast<const uint4*>(p);
  } else {
    reinterpret_cast<uint4*>(c.v)[0] = reinterpret_cast<const uint4*>(p)[0];
    reinterpret_cast<uint4*>(c.v)[1] = reinterpret_cast<const uint4*>(p)[1];
  }
}
template <typename T>
__device__ __forceinline__ void zero8(Chunk<T>& c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c.v[j] = from_f<T>(0.f);
}
template <typename T>
__device__ __forceinline__ void store_lds8(T* dst, const Chunk<T>& c) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(c.v);
  } else {
    reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(c.v)[0];
    reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(c.v)[1];
  }
}

// Dense row loader: 8 elements of row `row` starting at column k (zero outside [0,rows)x[0,K)).
template <typename T, bool VEC>
__device__ __forceinline__ void load_dense(const T* base, long ld, int row, int rows, int k, int K, Chunk<T>& c) {
  if (row >= rows) { zero8(c); return; }
  const T* p = base + (long)row * ld + k;
  if (VEC && k + 8 <= K) { load_vec8(p, c); return; }
#pragma unroll
  for (int j = 0; j < 8; ++j) c.v[j] = (k + j < K) ? p[j] : from_f<T>(0.f);
}

struct ConvRow { long base; int iy0, ix0; bool valid; };

template <typename T, bool VEC>
__device__ __forceinline__ void load_im2col(const T* X, const GemmArgs& p, const ConvRow& r, int k, Chunk<T>& c) {
  if (!r.valid) { zero8(c); return; }
  if (VEC) {  // Cin % 8 == 0: the 8 k of a chunk share one tap
    if (k >= p.K) { zero8(c); return; }
    int tap = k / p.Cin, ci = k - tap * p.Cin;
    int i = tap / p.kw, j = tap - i * p.kw;
    int iy = r.iy0 + i, ix = r.ix0 + j;
    if (iy < 0 || iy >= p.H || ix < 0 || ix >= p.Wd) { zero8(c); return; }
    load_vec8(X + r.base + ((long)iy * p.Wd + ix) * p.Cin + ci, c);
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    int kk = k + e;
    T v = from_f<T>(0.f);
    if (kk < p.K) {
      int tap = kk / p.Cin, ci = kk - tap * p.Cin;
      int i = tap / p.kw, j = tap - i * p.kw;
      int iy = r.iy0 + i, ix = r.ix0 + j;
      if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.Wd) v = X[r.base + ((long)iy * p.Wd + ix) * p.Cin + ci];
    }
    c.v[e] = v;
  }
}

template <typename T>
__device__ __forceinline__ void mfma_step(const Chunk<T>& a, const Chunk<T>& b, f32x4& acc) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 av = *reinterpret_cast<const bf16x8*>(a.v);
    bf16x8 bv = *reinterpret_cast<const bf16x8*>(b.v);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[s], b.v[s], acc, 0, 0, 0);
  }
}

template <typename T, int BM, int BN, bool VEC, int ASRC>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(GemmArgs p) {
  constexpr int PADK = 16 / sizeof(T);
  constexpr int LDK = BK + PADK;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM * (BK / 8) / NTHREADS;   // A chunks per thread
  constexpr int BCH = BN * (BK / 8) / NTHREADS;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) T sA[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) T sB[2][BN][LDK];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const T* A = static_cast<const T*>(p.A);
  const T* Wt = static_cast<const T*>(p.W);

  // Each thread loads chunk (row = tid/4 + 64*i, kc = tid%4) of the A and B tiles.
  const int lrow = tid >> 2, lk = (tid & 3) * 8;
  ConvRow crow[ACH];
  if constexpr (ASRC == 1) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int m = m0 + lrow + 64 * i;
      crow[i].valid = m < p.M;
      int mm = crow[i].valid ? m : 0;
      int hw = p.OH * p.OW;
      int b = mm / hw, rem = mm - b * hw;
      int oy = rem / p.OW, ox = rem - oy * p.OW;
      crow[i].base = (long)b * p.H * p.Wd * p.Cin;
      crow[i].iy0 = oy * p.stride - p.pad;
      crow[i].ix0 = ox * p.stride - p.pad;
    }
  }

  Chunk<T> ra[ACH], rb[BCH];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      if constexpr (ASRC == 1) load_im2col<T, VEC>(A, p, crow[i], k0 + lk, ra[i]);
      else load_dense<T, VEC>(A, p.lda, m0 + lrow + 64 * i, p.M, k0 + lk, p.K, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) load_dense<T, VEC>(Wt, p.ldw, n0 + lrow + 64 * i, p.N, k0 + lk, p.K, rb[i]);
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) store_lds8(&sA[buf][lrow + 64 * i][lk], ra[i]);
#pragma unroll
    for (int i = 0; i < BCH; ++i) store_lds8(&sB[buf][lrow + 64 * i][lk], rb[i]);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  fetch(0);
  stash(0);
  __syncthreads();

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) fetch((kt + 1) * BK);
    Chunk<T> fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const Chunk<T>*>(&sA[buf][wm * WM + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const Chunk<T>*>(&sB[buf][wn * WN + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma_step<T>(fa[i], fb[j], acc[i][j]);
    if (kt + 1 < nk) stash(buf ^ 1);
    __syncthreads();
  }

  // Epilogue: C/D map of the 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r.
  T* C = static_cast<T*>(p.C);
  const T* R = static_cast<const T*>(p.R);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + fr;
    if (n >= p.N) continue;
    const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.M) continue;
        float v = apply_act(acc[i][j][r] + bn, p.act);
        if (R) v += to_f(R[(long)m * p.ldr + n]);
        C[(long)m * p.ldc + n] = from_f<T>(v);
      }
    }
  }
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

template <typename T, int ASRC>
static int launch_gemm(const GemmArgs& a, bool vec, hipStream_t st) {
  const int M = a.M, N = a.N;
  auto go = [&](auto bm_c, auto bn_c) {
    constexpr int BM = decltype(bm_c)::value, BN = decltype(bn_c)::value;
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
    if (vec) hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, ASRC>), grid, dim3(NTHREADS), 0, st, a);
    else hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, ASRC>), grid, dim3(NTHREADS), 0, st, a);
  };
  using I64 = std::integral_constant<int, 64>;
  using I128 = std::integral_constant<int, 128>;
  if (N <= 64) {
    if ((long)((M + 127) / 128) >= 512) go(I128{}, I64{}); else go(I64{}, I64{});
  } else {
    long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128);
    if (tiles128 >= 512) go(I128{}, I128{}); else go(I64{}, I64{});
  }
  return check_launch("gemm");
}

}  // namespace svk

using namespace svk;

extern "C" int svk_gemm(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
                        const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act, void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !A || !W || !C) { set_error("svk_gemm: bad args M=%d N=%d K=%d", M, N, K); return SVK_EINVAL; }
  if (M == 0) return SVK_OK;
  if (lda < K || ldw < K || ldc < N || (R && ldr < N)) { set_error("svk_gemm: leading dims too small"); return SVK_EINVAL; }
  GemmArgs a{};
  a.A = A; a.lda = lda; a.W = W; a.ldw = ldw; a.bias = bias; a.R = R; a.ldr = ldr; a.C = C; a.ldc = ldc;
  a.M = M; a.N = N; a.K = K; a.act = act;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    const long vecw = 16 / (long)sizeof(T);
    bool vec = aligned16(A) && aligned16(W) && (lda % vecw == 0) && (ldw % vecw == 0);
    return launch_gemm<T, 0>(a, vec, st);
  });
}

extern "C" int svk_conv2d_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* Wt,
                               const float* bias, const void* R, void* Y, int Cout, int k, int stride, int pad,
                               int act, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || k <= 0 || stride <= 0 || pad < 0 || !X || !Wt || !Y) {
    set_error("svk_conv2d_nhwc: bad args"); return SVK_EINVAL;
  }
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) { set_error("svk_conv2d_nhwc: empty output"); return SVK_EINVAL; }
  if (B == 0) return SVK_OK;
  const long M = (long)B * OH * OW;
  if (M > 0x7fffffffL) { set_error("svk_conv2d_nhwc: too many output pixels"); return SVK_EUNSUPPORTED; }
  GemmArgs a{};
  a.A = X; a.lda = 0; a.W = Wt; a.ldw = (long)k * k * Cin; a.bias = bias; a.R = R; a.ldr = Cout; a.C = Y; a.ldc = Cout;
  a.M = (int)M; a.N = Cout; a.K = k * k * Cin; a.act = act;
  a.H = H; a.Wd = W; a.Cin = Cin; a.OH = OH; a.OW = OW; a.kw = k; a.stride = stride; a.pad = pad;
  hipStream_t st = (hipStream_t)stream;
  SVK_DISPATCH_DTYPE(dtype, T, {
    bool vec = aligned16(X) && aligned16(Wt) && (Cin % 8 == 0);
    return launch_gemm<T, 1>(a, vec, st);
  });
}
