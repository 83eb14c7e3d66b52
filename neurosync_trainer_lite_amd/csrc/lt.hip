// Plain bf16 GEMMs on hipBLASLt (NSTL_GEMM_LT, default on): nstl_gemm calls with
// no fused epilogue beyond a bias -- the step's forward out-projection / FFN
// linear2 / cross-attention q GEMMs and the input-gradient GEMMs handed to the
// next LayerNorm backward -- run on the library's tuned gfx950 kernels (256x256x64
// tiles on four waves, stream-K), measured 8-25 % faster than the ring kernel on
// those shapes (tools/bench_torch_mm.py).  Every GEMM with a
// fused epilogue (ReLU-dropout with keep bits, RoPE, dReLU with column sums,
// grouped weight gradients with norm partials, fp8) stays on the hand-written
// kernels.  No device code here: host-side descriptor and algorithm caches.
//
// Mapping: nstl_gemm computes row-major C[M][N] = alpha sum_r A(i,r) B(j,r) (+ bias[j])
// (+ beta C).  hipBLASLt is column-major, so it computes C^T (N x M, ld = ldc) =
// B_math (N x K) * A_math^T (K x M): its "A" is our B (K-major rows [N][K] seen
// column-major as K x N, transposed; or [K][N] rows seen as N x K, not
// transposed) and its "B" is our A (rows [M][K] seen as K x M).  Our bias over
// columns j is its bias over rows of D.
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <tuple>

#include "../../include/nstl.h"
#include "status.h"

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

typedef std::tuple<int, int, int, int, int64_t, int64_t, int64_t, int, int, int, int> LtKey;

constexpr size_t LT_WS = 64ull << 20;  // workspace offered to the heuristics (stream-K partials)

struct LtState {
  std::mutex mu;
  std::map<int, hipblasLtHandle_t> handles;
  std::map<LtKey, LtPlan> plans;
  std::map<std::pair<int, hipStream_t>, void*> ws;
};
LtState& state() {
  static LtState* s = new LtState();  // never destroyed: handles outlive static teardown order
  return *s;
}

int lt_enabled() {
  static const int v = [] {
    const char* e = getenv("NSTL_GEMM_LT");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return v;
}

bool eligible(const nstl_gemm_args* a) {
  // bf16 output only: with f32 output and beta = 1 (the accumulating input
  // gradients) the library measured 2-5 % slower than the ring kernel
  if (a->dtype != NSTL_BF16 || a->c_dtype != NSTL_BF16) return false;
  if (a->epilogue != NSTL_EPI_NONE && a->epilogue != NSTL_EPI_BIAS) return false;
  if (a->split_k > 1 || a->colsum_part || a->relu_mask || a->a_scale || a->b_scale || a->sq_part) return false;
  if (!a->a_kmajor) return false;  // the weight-gradient layouts stay on the grouped ring kernel
  if (a->beta != 0.f) return false;
  // the sizes the ring kernel takes (>= 32 of its 256^2 tiles): smaller ones keep their kernels
  const int64_t tiles = (int64_t)((a->M + 255) / 256) * ((a->N + 255) / 256);
  if (tiles < 32 || a->K % 64 != 0) return false;
  if (a->lda % 8 || a->ldb % 8 || a->ldc % 8) return false;
  if (((uintptr_t)a->A | (uintptr_t)a->B | (uintptr_t)a->C) % 16) return false;
  return true;
}

// hipBLASLt is an accelerator here, never a dependency of a result: any failure
// of the library leaves the call to the hand-written kernels (one warning).
void lt_warn(const char* what, int status) {
  static bool once = false;
  if (!once) {
    once = true;
    fprintf(stderr, "[nstl] hipBLASLt: %s failed (%d); plain GEMMs stay on the hand-written kernels\n", what, status);
  }
}
#define LT_TRY(x)                     \
  do {                                \
    hipblasStatus_t s_ = (x);         \
    if (s_ != HIPBLAS_STATUS_SUCCESS) { \
      lt_warn(#x, (int)s_);           \
      return false;                   \
    }                                 \
  } while (0)

// false: no plan (the caller's kernels run the GEMM)
bool make_plan(hipblasLtHandle_t h, const nstl_gemm_args* a, LtPlan& pl) {
  const hipDataType ct = a->c_dtype == NSTL_F32 ? HIP_R_32F : HIP_R_16BF;
  LT_TRY(hipblasLtMatmulDescCreate(&pl.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = a->b_kmajor ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  LT_TRY(hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_TRY(hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (a->epilogue == NSTL_EPI_BIAS && a->bias) {
    const uint32_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_32F;
    LT_TRY(hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    LT_TRY(hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    const void* bp = a->bias;
    LT_TRY(hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
  }
  // its A = our B: K x N (transposed, K-major rows [N][K]) or N x K (rows [K][N])
  if (a->b_kmajor) LT_TRY(hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, a->K, a->N, a->ldb));
  else LT_TRY(hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, a->N, a->K, a->ldb));
  LT_TRY(hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, a->K, a->M, a->lda));  // its B = our A^T
  LT_TRY(hipblasLtMatrixLayoutCreate(&pl.lc, ct, a->N, a->M, a->ldc));          // D = C^T
  hipblasLtMatmulPreference_t pref;
  LT_TRY(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = LT_WS;
  LT_TRY(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(h, pl.desc, pl.la, pl.lb, pl.lc, pl.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) return false;
  pl.algo = res[0].algo;
  pl.ws = res[0].workspaceSize;
  pl.ok = true;
  return true;
}

}  // namespace

namespace nstl {
// Runs `a` on hipBLASLt when it is a plain bf16 GEMM that the library handles;
// *handled = 0 leaves it to the caller's kernels (also whenever the library fails).
int lt_gemm(const nstl_gemm_args* a, hipStream_t st, int* handled) {
  *handled = 0;
  if (!lt_enabled() || !eligible(a)) return 0;
  LtState& S = state();
  std::lock_guard<std::mutex> lk(S.mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  auto hit = S.handles.find(dev);
  if (hit == S.handles.end()) {
    hipblasLtHandle_t h = nullptr;
    const hipblasStatus_t hs = hipblasLtCreate(&h);
    if (hs != HIPBLAS_STATUS_SUCCESS) {
      lt_warn("hipblasLtCreate", (int)hs);
      h = nullptr;
    }
    hit = S.handles.emplace(dev, h).first;  // nullptr: unavailable on this device
  }
  if (hit->second == nullptr) return 0;
  const LtKey key{dev, a->M, a->N, a->K, a->lda, a->ldb, a->ldc, a->b_kmajor, a->c_dtype,
                  a->epilogue == NSTL_EPI_BIAS && a->bias ? 1 : 0, a->beta != 0.f ? 1 : 0};
  auto pit = S.plans.find(key);
  if (pit == S.plans.end()) {
    LtPlan pl;
    if (!make_plan(hit->second, a, pl)) pl.ok = false;
    pit = S.plans.emplace(key, pl).first;
  }
  LtPlan& pl = pit->second;
  if (!pl.ok) return 0;
  void*& ws = S.ws[{dev, st}];
  if (pl.ws > 0 && ws == nullptr && hipMalloc(&ws, LT_WS) != hipSuccess) {
    ws = nullptr;
    lt_warn("workspace allocation", (int)hipErrorOutOfMemory);
    return 0;
  }
  if (a->epilogue == NSTL_EPI_BIAS && a->bias) {
    const void* bp = a->bias;
    const hipblasStatus_t hs =
        hipblasLtMatmulDescSetAttribute(pl.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
    if (hs != HIPBLAS_STATUS_SUCCESS) {
      lt_warn("bias pointer", (int)hs);
      return 0;
    }
  }
  const float alpha = a->alpha, beta = a->beta;
  const hipblasStatus_t hs = hipblasLtMatmul(hit->second, pl.desc, &alpha, a->B, pl.la, a->A, pl.lb, &beta, a->C,
                                             pl.lc, a->C, pl.lc, &pl.algo, pl.ws > 0 ? ws : nullptr, pl.ws, st);
  if (hs != HIPBLAS_STATUS_SUCCESS) {  // nothing was launched: the caller's kernels run it
    lt_warn("hipblasLtMatmul", (int)hs);
    return 0;
  }
  nstl::count(NSTL_K_GEMM_LT);
  *handled = 1;
  return 0;
}
}  // namespace nstl
