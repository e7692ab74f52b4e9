// hipBLASLt as a yardstick for the hand-written GEMMs (host code only).  OFF by default since r04: every product of
// the step runs on the hand-written gfx950 kernels of gemm.hip; MAPFED_GEMM_LIB=1 (or mf_gemm_lib_enable) routes
// the products below to hipBLASLt for A/B runs against the vendor library (tests/diagnostics/gemm_bench.py also
// times torch.mm, i.e. hipBLASLt, beside every tile).
//
// The hand-written kernels (gemm.hip) carry every fused epilogue of the path (residual add, QuickGELU and its
// derivative at the reference's fp16 rounding points).  Three products have no epilogue beyond a bias and
// run faster in the vendor library on their c4 shapes (tests/diagnostics/gemm_bench.py, graph-replayed,
// profiles/r03_v2_gemm_vs_hipblaslt.txt):
//   vision in-projection  6368 x 2304 x 768,  EPI_BIAS: 877 against 743 TFLOP/s;
//   vision c_fc dX        6368 x 768 x 3072,  plain:    853 against 728;
//   text c_fc dX          2926 x 512 x 2048,  plain:    427 against 349.
// hipBLASLt's bias epilogue adds the bias to the fp32 accumulator and rounds once to fp16, the reference's
// rounding point for Linear (fp16(acc + bias)).  On MI355X its results are bit-identical to the hand-written
// kernels' on every routed shape (tests/test_kernels_gpu.py::test_gemm_lib_route), so the route changes the
// step's time only (same-box A/B +1.8 %), not a single value.
//
// Row-major C[M,N] = A[M,K] B[N,K]^T is the column-major D = op(B) op(A) with D = C^T (N x M, ld = ldc):
// matrix "A" of the call is our B (K x N column-major, ld = ldb, transposed), matrix "B" is our A (K x M,
// ld = lda, not transposed), m = N, n = M.
//
// The algorithm is the heuristic's first answer for the shape, cached per shape; the workspace is the
// caller's (mf_gemm_lib_init), so nothing is allocated inside a captured graph.
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "mf_common.h"

namespace {

enum { LIB_EPI_NONE = 0, LIB_EPI_BIAS = 1 };  // gemm.hip's EPI_NONE / EPI_BIAS

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

struct LibState {
  std::mutex mu;
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  int enabled = 0;
  std::map<std::tuple<int, int, int, int64_t, int64_t, int64_t, int>, Plan> plans;
};

LibState& state() {
  static LibState s;
  return s;
}

}  // namespace

// Register the workspace (device memory the caller keeps alive) and create the handle.  Idempotent.
extern "C" int mf_gemm_lib_init(void* workspace, int64_t bytes) {
  LibState& s = state();
  std::lock_guard<std::mutex> lk(s.mu);
  if (!s.handle && hipblasLtCreate(&s.handle) != HIPBLAS_STATUS_SUCCESS)
    return mf_set_error("mf_gemm_lib_init: hipblasLtCreate failed", -1);
  s.ws = workspace;
  s.ws_bytes = workspace ? (size_t)bytes : 0;
  const char* env = getenv("MAPFED_GEMM_LIB");  // A/B knob: 1 routes the products below to hipBLASLt
  s.enabled = env && atoi(env) != 0;
  return 0;
}

// Runtime switch (tests compare the hand-written kernels against themselves bit for bit).
extern "C" int mf_gemm_lib_enable(int on) {
  state().enabled = on != 0;
  return 0;
}

// Which products go to the library when enabled (the heuristic tile path of mf_gemm_nt asks this).
extern "C" int mf_gemm_lib_wants(int M, int N, int K, int epilogue) {
  LibState& s = state();
  if (!s.handle || !s.enabled) return 0;
  if (epilogue == LIB_EPI_BIAS) return M >= 4096 && N == 2304 && K == 768;  // vision in-projection
  if (epilogue == LIB_EPI_NONE)
    return (M >= 4096 && N == 768 && K == 3072) || (M >= 2048 && M < 4096 && N == 512 && K == 2048);  // c_fc dX
  return 0;
}

extern "C" int mf_gemm_lib(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                           int K, const void* bias, int epilogue, void* stream) {
  LibState& s = state();
  if (!s.handle) return mf_set_error("mf_gemm_lib: call mf_gemm_lib_init first", -1);
  if (epilogue != LIB_EPI_NONE && epilogue != LIB_EPI_BIAS) return mf_set_error("mf_gemm_lib: epilogue", -1);
  if (epilogue == LIB_EPI_BIAS && !bias) return mf_set_error("mf_gemm_lib: bias epilogue needs bias", -1);
  if (M <= 0 || N <= 0) return 0;
  std::lock_guard<std::mutex> lk(s.mu);  // the plan's bias pointer is set per call
  Plan* p;
  {
    auto key = std::make_tuple(M, N, K, lda, ldb, ldc, epilogue);
    p = &s.plans[key];
    if (!p->ok) {
      bool good = hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
      const hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
      good = good && hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA)) ==
                         HIPBLAS_STATUS_SUCCESS;
      good = good && hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB)) ==
                         HIPBLAS_STATUS_SUCCESS;
      if (epilogue == LIB_EPI_BIAS) {
        const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
        const hipDataType bt = HIP_R_16F;
        good = good && hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) ==
                           HIPBLAS_STATUS_SUCCESS;
        good = good && hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt,
                                                       sizeof(bt)) == HIPBLAS_STATUS_SUCCESS;
      }
      good = good && hipblasLtMatrixLayoutCreate(&p->la, HIP_R_16F, K, N, ldb) == HIPBLAS_STATUS_SUCCESS;
      good = good && hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_16F, K, M, lda) == HIPBLAS_STATUS_SUCCESS;
      good = good && hipblasLtMatrixLayoutCreate(&p->lc, HIP_R_16F, N, M, ldc) == HIPBLAS_STATUS_SUCCESS;
      hipblasLtMatmulPreference_t pref = nullptr;
      good = good && hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
      // workspace-free algorithms only: the vision and text towers' products run on two streams at once and a
      // shared workspace would let two concurrent launches overwrite each other's partial sums
      const uint64_t wsb = 0;
      good = good && hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                           sizeof(wsb)) == HIPBLAS_STATUS_SUCCESS;
      hipblasLtMatmulHeuristicResult_t res[1];
      int n = 0;
      good = good && hipblasLtMatmulAlgoGetHeuristic(s.handle, p->desc, p->la, p->lb, p->lc, p->lc, pref, 1, res,
                                                     &n) == HIPBLAS_STATUS_SUCCESS && n > 0;
      if (pref) hipblasLtMatmulPreferenceDestroy(pref);
      if (!good) {
        s.plans.erase(key);
        return mf_set_error("mf_gemm_lib: no hipBLASLt algorithm for this product", -1);
      }
      p->algo = res[0].algo;
      p->ws = 0;
      p->ok = true;
    }
  }
  if (epilogue == LIB_EPI_BIAS &&
      hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
          HIPBLAS_STATUS_SUCCESS)
    return mf_set_error("mf_gemm_lib: bias pointer", -1);
  const float alpha = 1.0f, beta = 0.0f;
  const hipblasStatus_t st = hipblasLtMatmul(s.handle, p->desc, &alpha, B, p->la, A, p->lb, &beta, C, p->lc, C, p->lc,
                                             &p->algo, s.ws, p->ws, (hipStream_t)stream);
  if (st != HIPBLAS_STATUS_SUCCESS) return mf_set_error("mf_gemm_lib: hipblasLtMatmul failed", -1);
  return 0;
}
