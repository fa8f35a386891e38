// Library GEMM backend: hipBLASLt for the plain-epilogue token GEMMs where the hand-written kernels measure
// slower (mix_transformer_evp.py:60-67 fc1 / fc2 and :81-90 kv of stages 3-4, segformer_head.py:74-80 the
// linear_fuse; profiles/r04/pk_cfg_sweep_pp.txt).  Host code only: one hipBLASLt handle per process, a plan
// (matmul descriptor, layouts, heuristic algorithm) per shape, the bias pointer set per call.
//
// Row-major C [M, N] = A [M, K] · Wᵀ (W = nn.Linear's [N, K]) is the column-major product Cᵀ [N, M] =
// op(W) · Aᵀ with op = transpose: hipBLASLt m = N, n = M, k = K; bias (f32) per hipBLASLt row = per output
// column; the residual R rides as beta · C with D = the output (epilogue: act(AB + R + bias) — so R is only
// taken with act == none, matching gemm_kernel's act(AB + bias) + R; ReLU without R).  No workspace: the
// call must stay capturable into a HIP graph on its first use.
#include "svk_common.h"
#include "gemm_args.h"
#include <hipblaslt/hipblaslt.h>
#include <map>
#include <mutex>
#include <tuple>

namespace svk {

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};

using Key = std::tuple<int, int, int, int, long, long, long, long, int, int, int>;

struct State {
  std::mutex mu;
  hipblasLtHandle_t h = nullptr;
  bool init_failed = false;
  std::map<Key, Plan> plans;
};

State& state() {
  static State* s = new State();   // never destroyed: plans may be used by graphs replayed at exit
  return *s;
}

}  // namespace

// 0 = launched; 1 = not eligible / no algorithm (the caller launches a hand-written kernel)
int libgemm_try(const GemmArgs& a, hipStream_t st, int dtype) {
  if (a.U || a.rscale || a.out_mode || a.ksplit) return 1;
  if (a.act != SVK_ACT_NONE && a.act != SVK_ACT_RELU) return 1;
  if (a.act != SVK_ACT_NONE && a.R) return 1;
  const hipDataType dt = dtype == SVK_F16 ? HIP_R_16F : HIP_R_16BF;
  State& S = state();
  std::lock_guard<std::mutex> lock(S.mu);
  if (S.init_failed) return 1;
  if (!S.h && hipblasLtCreate(&S.h) != HIPBLAS_STATUS_SUCCESS) { S.init_failed = true; return 1; }
  const int epi = a.act == SVK_ACT_RELU ? (a.bias ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_RELU)
                                        : (a.bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT);
  const Key key{dtype, a.M, a.N, a.K, a.lda, a.ldw, a.ldc, a.R ? a.ldr : -1L, epi, a.R != nullptr, 0};
  auto it = S.plans.find(key);
  if (it == S.plans.end()) {
    Plan p;
    bool good = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
    const hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    const uint32_t e = (uint32_t)epi;
    const int32_t bt = HIP_R_32F;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT)) == 0;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN)) == 0;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)) == 0;
    if (a.bias) good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) == 0;
    // A operand (hipBLASLt's): W as column-major [K, N], ld = ldw; B operand: A as column-major [K, M], ld = lda
    good = good && hipblasLtMatrixLayoutCreate(&p.la, dt, a.K, a.N, a.ldw) == 0;
    good = good && hipblasLtMatrixLayoutCreate(&p.lb, dt, a.K, a.M, a.lda) == 0;
    good = good && hipblasLtMatrixLayoutCreate(&p.lc, dt, a.N, a.M, a.R ? a.ldr : a.ldc) == 0;
    good = good && hipblasLtMatrixLayoutCreate(&p.ld, dt, a.N, a.M, a.ldc) == 0;
    if (good) {
      hipblasLtMatmulPreference_t pref = nullptr;
      uint64_t ws = 0;
      hipblasLtMatmulHeuristicResult_t res[1];
      int n = 0;
      if (hipblasLtMatmulPreferenceCreate(&pref) == 0 &&
          hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)) == 0 &&
          hipblasLtMatmulAlgoGetHeuristic(S.h, p.desc, p.la, p.lb, p.lc, p.ld, pref, 1, res, &n) == 0 && n > 0 &&
          res[0].state == HIPBLAS_STATUS_SUCCESS && res[0].workspaceSize == 0) {
        p.algo = res[0].algo;
        p.ok = true;
      }
      if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    }
    it = S.plans.emplace(key, p).first;
  }
  Plan& p = it->second;
  if (!p.ok) return 1;
  if (a.bias && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a.bias, sizeof(a.bias)) != 0)
    return 1;
  const float alpha = 1.f, beta = a.R ? 1.f : 0.f;
  const void* cptr = a.R ? a.R : a.C;
  if (hipblasLtMatmul(S.h, p.desc, &alpha, a.W, p.la, a.A, p.lb, &beta, cptr, p.lc, a.C, p.ld, &p.algo, nullptr, 0, st) !=
      HIPBLAS_STATUS_SUCCESS)
    return 1;
  set_last_kernel("hipblaslt");
  return 0;
}

}  // namespace svk
