// Plain bf16-operand GEMMs through hipBLASLt: the weight-gradient and input-gradient
// contractions of the backward pass (dW_lin, dH, dW_ih, dW_hh, dX), which carry no fused
// epilogue.  The fused forward GEMMs (input projection + bias, Linear + bias + tanh) stay on
// the hand-written MFMA kernel (gemm_bb.hip).
//
// Semantics are those of dl4ss_gemm_bf16_batched (row-major C[M,N] = op(A) op(B) + beta C,
// A stored M x K or K x M (transA), B stored K x N or N x K (transB), bf16 operands, fp32
// C and accumulation).  hipBLASLt is column-major, so the call computes the transposed
// product C^T = op(B)^T op(A)^T on the same memory.  One hipBLASLt handle per device
// (std::call_once); the heuristic's first algorithm is cached per problem (mutex-guarded),
// so a step's repeated shapes pay the query once.  The workspace is the caller's.
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

namespace {

struct LtKey {
  int ta, tb, M, N, K, batch, beta0;
  long long lda, ldb, ldc, sa, sb, sc, ws;
  bool operator<(const LtKey& o) const {
    return std::tie(ta, tb, M, N, K, batch, beta0, lda, ldb, ldc, sa, sb, sc, ws) <
           std::tie(o.ta, o.tb, o.M, o.N, o.K, o.batch, o.beta0, o.lda, o.ldb, o.ldc, o.sa, o.sb, o.sc, o.ws);
  }
};

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};

constexpr int MAX_DEV = 16;
hipblasLtHandle_t g_handle[MAX_DEV] = {};
std::once_flag g_once[MAX_DEV];
std::mutex g_mu;
std::map<std::pair<int, LtKey>, LtPlan> g_plans;

hipblasLtMatrixLayout_t layout(hipDataType t, uint64_t rows, uint64_t cols, int64_t ld, int batch, int64_t stride) {
  hipblasLtMatrixLayout_t l = nullptr;
  if (hipblasLtMatrixLayoutCreate(&l, t, rows, cols, ld) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  if (batch > 1) {
    int32_t b = batch;
    hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b));
    hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride, sizeof(stride));
  }
  return l;
}

constexpr int LT_CANDIDATES = 16;

bool tune_enabled() {
  const char* e = std::getenv("DL4SS_LT_TUNE");
  return !(e && std::strcmp(e, "0") == 0);
}

// time each candidate (2 warm runs, then 5 timed) and return the index of the fastest;
// C (extent c_elems floats) is restored afterwards
int pick_fastest(hipblasLtHandle_t h, const LtPlan& p, const hipblasLtMatmulHeuristicResult_t* res, int nres,
                 const void* A, const void* B, float* C, size_t c_elems, float beta, void* ws, long long ws_bytes,
                 hipStream_t st) {
  float* save = nullptr;
  if (hipMalloc(&save, c_elems * sizeof(float)) != hipSuccess) return 0;
  (void)hipMemcpyAsync(save, C, c_elems * sizeof(float), hipMemcpyDeviceToDevice, st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const float alpha = 1.0f;
  int best = 0;
  float best_ms = 1e30f;
  for (int i = 0; i < nres; ++i) {
    if ((long long)res[i].workspaceSize > ws_bytes) continue;
    bool ok = true;
    for (int r = 0; r < 2 && ok; ++r)
      ok = hipblasLtMatmul(h, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo, ws,
                           res[i].workspaceSize, st) == HIPBLAS_STATUS_SUCCESS;
    if (!ok) continue;
    (void)hipEventRecord(e0, st);
    for (int r = 0; r < 5; ++r)
      hipblasLtMatmul(h, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &res[i].algo, ws,
                      res[i].workspaceSize, st);
    (void)hipEventRecord(e1, st);
    float ms = 0.0f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
    if (std::getenv("DL4SS_LT_VERBOSE"))
      fprintf(stderr, "[lt] cand %d ws %zu: %.2f us\n", i, (size_t)res[i].workspaceSize, ms * 1000.0f / 5);
    if (ms < best_ms) {
      best_ms = ms;
      best = i;
    }
  }
  (void)hipMemcpyAsync(C, save, c_elems * sizeof(float), hipMemcpyDeviceToDevice, st);
  (void)hipStreamSynchronize(st);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(save);
  return best;
}

}  // namespace

DL4SS_API int dl4ss_gemm_bf16_lt(int transA, int transB, int M, int N, int K, const void* A, long long lda,
                                 const void* B, long long ldb, float* C, long long ldc, float beta, int batch,
                                 long long strideA, long long strideB, long long strideC, void* workspace,
                                 long long ws_bytes, void* stream) {
  DL4SS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && A && B && C && batch >= 1 && ws_bytes >= 0);
  DL4SS_REQUIRE(ws_bytes == 0 || workspace);
  if (M == 0 || N == 0) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return (int)hipErrorInvalidDevice;
  std::call_once(g_once[dev], [dev] { hipblasLtCreate(&g_handle[dev]); });
  if (!g_handle[dev]) return (int)hipErrorNotInitialized;
  const LtKey key{transA, transB, M, N, K, batch, beta == 0.0f, lda, ldb, ldc, strideA, strideB, strideC, ws_bytes};
  LtPlan plan;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find({dev, key});
    if (it != g_plans.end()) {
      plan = it->second;
    } else {
      // column-major view: first operand op(B)^T (N x K), second op(A)^T (K x M), C^T (N x M)
      const hipblasOperation_t opx = transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      const hipblasOperation_t opy = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      if (hipblasLtMatmulDescCreate(&plan.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
        return (int)hipErrorInvalidValue;
      hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opx, sizeof(opx));
      hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opy, sizeof(opy));
      plan.la = transB ? layout(HIP_R_16BF, K, N, ldb, batch, strideB) : layout(HIP_R_16BF, N, K, ldb, batch, strideB);
      plan.lb = transA ? layout(HIP_R_16BF, M, K, lda, batch, strideA) : layout(HIP_R_16BF, K, M, lda, batch, strideA);
      plan.lc = layout(HIP_R_32F, N, M, ldc, batch, strideC);
      if (!plan.la || !plan.lb || !plan.lc) return (int)hipErrorInvalidValue;
      hipblasLtMatmulPreference_t pref = nullptr;
      hipblasLtMatmulPreferenceCreate(&pref);
      uint64_t wsmax = (uint64_t)ws_bytes;
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax, sizeof(wsmax));
      hipblasLtMatmulHeuristicResult_t res[LT_CANDIDATES];
      int nres = 0;
      const int want = tune_enabled() ? LT_CANDIDATES : 1;
      const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic(g_handle[dev], plan.desc, plan.la, plan.lb, plan.lc,
                                                                 plan.lc, pref, want, res, &nres);
      hipblasLtMatmulPreferenceDestroy(pref);
      if (hs != HIPBLAS_STATUS_SUCCESS || nres < 1) return (int)hipErrorNotSupported;
      int pick = 0;
      if (nres > 1) {
        const size_t c_elems = (size_t)(batch - 1) * (size_t)strideC + (size_t)(M - 1) * (size_t)ldc + (size_t)N;
        pick = pick_fastest(g_handle[dev], plan, res, nres, A, B, C, c_elems, beta, workspace, ws_bytes,
                            as_stream(stream));
        if (std::getenv("DL4SS_LT_VERBOSE"))
          fprintf(stderr, "[lt] ta %d tb %d M %d N %d K %d batch %d beta %g: %d candidates, pick %d\n", transA,
                  transB, M, N, K, batch, beta, nres, pick);
      }
      plan.algo = res[pick].algo;
      plan.ws = res[pick].workspaceSize;
      g_plans[{dev, key}] = plan;
    }
  }
  const float alpha = 1.0f;
  const hipblasStatus_t s = hipblasLtMatmul(g_handle[dev], plan.desc, &alpha, B, plan.la, A, plan.lb, &beta, C,
                                            plan.lc, C, plan.lc, &plan.algo, workspace, plan.ws, as_stream(stream));
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : (int)hipErrorLaunchFailure;
}
