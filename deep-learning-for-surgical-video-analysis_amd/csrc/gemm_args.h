// Argument block of the GEMM / implicit-GEMM conv kernels (gemm.hip, gemm_pk.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>

namespace svk {

struct GemmArgs {
  const void* A; long lda;
  const void* W; long ldw;
  const float* bias;
  const void* R; long ldr;
  void* C; long ldc;
  int M, N, K, act;
  int vec_out;          // C (and R) rows 16-byte aligned with whole chunks -> vector epilogue
  // implicit-GEMM conv geometry.  ASRC == 1 (forward im2col): source map H x Wd x Cin, GEMM rows
  // are the OH x OW output pixels.  ASRC == 2 (data gradient, transposed-conv gather): source map
  // is dY (H x Wd x Cin = OHy x OWy x Cout), GEMM rows are the OH x OW input pixels of the conv.
  int H, Wd, Cin, OH, OW, kw, stride, pad;
  int sshift;           // log2(stride) (ASRC == 2)
  const float* rscale;  // optional per-row scale of act(A W^T + bias) before the residual add
  int rdiv;             //   rscale index = m / rdiv (stochastic depth: rdiv = tokens per frame)
  const void* U; long ldu; int uact;   // optional activation backward: v *= act'(U[m, n]) (same dtype as C)
  // out_mode 1: C (and R) are an NHWC map [B, uH, uW, uC] and GEMM row m = (b, py, px) of the
  // (uH/us) x (uW/us) patch grid, column n = (i, j, ci): the adjoint of a k = s patchify conv.
  int out_mode, uH, uW, us, uC;
  // split-K (gemm_pk_conv_splitk): raw f32 partial sums of ksplit K parts -> slab [ksplit][M][N]
  int ksplit; float* slab;
};

// gemm_pk.hip: persistent LDS-DMA bf16 / f16 GEMM / implicit-GEMM conv (asrc 1) for the plain-epilogue
// case; returns 0 when it launched, 1 when the arguments are not eligible (caller falls back to gemm_kernel).
// T = __bf16 or _Float16 (instantiated in gemm_pk.hip).
template <typename T> int gemm_pk_try(const GemmArgs& a, hipStream_t st, int asrc);
template <typename T> int gemm_pk_conv_splitk(const GemmArgs& a, hipStream_t st);
// Row-tile height of the split-K patchify convs for N <= 128 (SVK_SPLITK_BM = 64 / 128): each unit reads its W
// slice once per row tile, so at N = 64 a 64-row tile moves as many W bytes (from L2) as A bytes (from HBM)
inline int splitk_bm() {
  static const int bm = getenv("SVK_SPLITK_BM") ? atoi(getenv("SVK_SPLITK_BM")) : 64;
  return bm == 128 ? 128 : 64;
}
// gemm_pp.hip: 256 x 256 ping-pong persistent GEMM, dense A, plain epilogue; variant 0 / 1 = first / deep DMA
// schedule; returns 1 when not eligible.
template <typename T> int gemm_pp_try(const GemmArgs& a, hipStream_t st, int variant);
// gemm_wt.hip: wide-tile (one 256-thread workgroup per CU, 2 x 2 waves of 128-row sub-tiles) persistent GEMM,
// dense A, plain epilogue; cfg 0 / 1 / 2 = 256 x 256 / 256 x 160 / 256 x 128 tiles; returns 1 when not eligible.
template <typename T> int gemm_wt_try(const GemmArgs& a, hipStream_t st, int cfg);


// wgrad_pk.hip: dW (+ db) += dY^T X (16-bit operands, LDS-DMA slabs + ds_read_b64_tr_b16 fragments),
// batched over Z = (Z / nzi, Z % nzi) element offsets; returns 1 when not eligible (caller: wgrad_kernel).
template <typename T>
int wgrad_pk_try(const void* dY, long ldy, long sa_o, long sa_i, const void* X, long ldx, long sx_o, long sx_i,
                 float* dW, long lddw, long sw_o, long sw_i, float* db, int Z, int nzi, int M, int N, int K,
                 hipStream_t st);
template <typename T>
int wgrad_pk_conv_try(const void* X, int B, int H, int W, int Cin, const void* dY, int Cout, int k, int stride, int pad,
                      int OH, int OW, float* dW, float* db, hipStream_t st);

}  // namespace svk
