// hipBLASLt for plain bf16 GEMMs (library GEMMs; the hand-written kernels keep the fused and mixed-type rest):
// the encoder's in-place-residual MLP2 / projection and its QKV projection, and the mask decoder's token-side
// products (M = prompts x 7 tokens).
//
// The encoder's MLP2 and attention projection are x += A W^T + b on the fp32 residual stream x (hf:modeling_sam.py
// SamVisionLayer: hidden_states = residual + mlp(...) / + attn(...)): a plain GEMM with a bias epilogue and beta = 1
// into an fp32 D. hipBLASLt's stream-K kernels run it faster than the 8-phase kernel, whose 384 tiles leave
// half of a second wave idle at MLP2 (same-operand yardstick, scripts/micro/blaslt_epi.cpp,
// profiles/r05/blaslt_yardstick.log: MLP2 180.4 -> 143.6 us, projection 67.3 -> 60.6 us).
//
// - Column-major view: D^T [N x M] = op(W) x A^T (A stored K x M); op(W) = W^T stored K x N (b_mode 0, TRANSA = T)
//   or W stored N x K (b_mode 1, k-major weights, TRANSA = N); bias per D^T row = output feature.
// - Algorithm: the heuristic's first candidate for the shape, planned once per (device, shape, layout, epilogue).
//   The plan is deterministic for one library build and device, so eager, graph-captured and multi-process runs
//   take the same kernel and the same bits (run-to-run bit-identical, checked in tests/test_gpu_gemm.py).
// - Workspace: owned by the caller (octsam_gemm_set_workspace; the Python side hands over a torch buffer), so the
//   library still allocates nothing. Without one the native kernels run.
// - Handles and plans are made on the first eligible call (the step's eager pass precedes every graph capture).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "../../include/octsam.h"

namespace octsam {
void set_error(const char* fmt, ...);
}

namespace {
struct Plan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
};
// (M, N, K, lda, ldb, ldc, ldr, b_mode, fp32 D, bias, act, C kind: 0 none / 1 = D / 2 separate R)
typedef std::tuple<int, int, int, long long, long long, long long, long long, int, int, int, int, int> Key;
struct Dev {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  std::map<Key, Plan> plans;
};
std::mutex g_mu;
std::map<int, Dev> g_devs;

int c_kind(const octsam_gemm_args* a) {
  if (a->R && a->R != a->C) return 2;
  return (a->R && a->R == a->C) || a->beta != 0.0f ? 1 : 0;
}

bool make_plan(Dev& d, const octsam_gemm_args* a, Plan& p) {
  const hipDataType et = HIP_R_16BF, dt = a->c_f32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const hipblasOperation_t ta = a->b_mode == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const bool relu = a->act == OCTSAM_ACT_RELU;
  const hipblasLtEpilogue_t epi = a->bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                                          : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (a->bias) {
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a->bias, sizeof(a->bias));
  }
  const bool lw = (a->b_mode == 0 ? hipblasLtMatrixLayoutCreate(&p.la, et, a->K, a->N, a->ldb)
                                  : hipblasLtMatrixLayoutCreate(&p.la, et, a->N, a->K, a->ldb)) == HIPBLAS_STATUS_SUCCESS;
  const long long ldcc = c_kind(a) == 2 ? a->ldr : a->ldc;
  if (!lw || hipblasLtMatrixLayoutCreate(&p.lb, et, a->K, a->M, a->lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, dt, a->N, a->M, ldcc) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.ld, dt, a->N, a->M, a->ldc) != HIPBLAS_STATUS_SUCCESS)
    return false;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t wsz = d.ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(d.h, p.desc, p.la, p.lb, p.lc, p.ld, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].workspaceSize > d.ws_bytes) return false;
  p.algo = res[0].algo;
  return true;
}

bool aligned(const void* q) { return ((uintptr_t)q & 15) == 0; }
}  // namespace

int g_blaslt_enabled = 1;  // octsam_gemm_set_fast_path bit 65536 turns it off (A/B)
int g_blaslt_qkv = 1;      // bit 131072 turns the QKV kind off (A/B)
int g_blaslt_tok = 1;      // bit 262144 turns the token-side kind off (A/B)

// Eligible: bf16 operands (the caller is octsam_gemm, not _f16), one batch, a_mode 0, no row map / pre-activation
// copy / broadcast addends / split-K / column sums, alpha 1, 16-B aligned pointers, leading dimensions % 8, and
//   x += A W^T (+ bias) with x fp32 and the residual IS the output (in place), b_mode 0, M >= 8192, N >= 256,
//   K >= 512: the encoder's MLP2 and projection; or
//   a bf16 D = A W^T + bias, no residual, b_mode 0, M >= 8192, 2048 <= N <= 4096, K <= 1024: the encoder's QKV
//   (same-process step A/B 16.28 -> 15.92 ms pipelined, 18.16 -> 17.99 sequential, profiles/r05/blaslt_step_ab.log);
//   or, at 1024 <= M < 8192 (the decoder's token side, P x 7 rows): b_mode 0 / 1, fp32 or bf16 D, bias, ReLU,
//   beta * D accumulation, or a separate same-type residual (graph-timed yardstick, M = 1176: 7.5 -> 4.2 us at
//   N = K = 256, 21.6 -> 7.5 us at K = 2048, profiles/r05/blaslt_yardstick_token.log).
// (MLP1 has the GELU: native. The decoder's plain 16-bit image-side products measured slower in the step.)
bool blaslt_eligible(const octsam_gemm_args* a) {
  if (!(g_blaslt_enabled && a->batch == 1 && a->a_mode == 0 && (a->b_mode == 0 || a->b_mode == 1) && !a->row_map &&
        !a->C_pre && !a->A2 && !a->B2 && !a->a_blk && !a->b_blk && !a->r_blk && !a->k_total && !a->a_colsum &&
        !a->b_colsum && a->alpha == 1.0f && aligned(a->A) && aligned(a->B) && aligned(a->C) &&
        (!a->R || aligned(a->R)) && (!a->bias || aligned(a->bias)) && a->lda % 8 == 0 && a->ldb % 8 == 0 &&
        a->ldc % 8 == 0 && (!a->R || a->ldr % 8 == 0) && a->lda >= a->K && a->ldc >= a->N))
    return false;
  if (a->M >= 8192) {
    if (a->b_mode != 0 || a->act != 0 || a->beta != 0.0f || a->lda != a->K || a->ldb != a->K || a->ldc != a->N)
      return false;
    if (!a->c_f32) return g_blaslt_qkv && a->R == nullptr && a->bias && a->N >= 2048 && a->N <= 4096 && a->K <= 1024;
    return a->r_f32 && a->R == a->C && a->ldr == a->ldc && a->N >= 256 && a->K >= 512;
  }
  if (!g_blaslt_tok || a->M < 1024 || (a->act != 0 && a->act != OCTSAM_ACT_RELU)) return false;
  if (a->b_mode == 0 ? a->ldb < a->K : a->ldb < a->N) return false;
  if (a->R) {
    // D = A W^T + b + R: hipBLASLt adds beta * C before the epilogue's activation, the native order adds R after
    // it, so only without an activation; R in D's type
    if (a->act != 0 || a->beta != 0.0f || a->r_f32 != a->c_f32 || a->ldr < a->N) return false;
    if (a->R == a->C && a->ldr != a->ldc) return false;
  }
  if (!a->R && a->beta != 0.0f && a->act != 0) return false;  // (native: act then beta * C? keep it native)
  return true;
}

// 1: ran, 0: not taken (no workspace, no plan: the caller runs the native kernels), -1: error (set)
int blaslt_gemm(const octsam_gemm_args* a, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  Dev& d = g_devs[dev];
  if (!d.ws) return 0;
  if (!d.h && hipblasLtCreate(&d.h) != HIPBLAS_STATUS_SUCCESS) {
    d.h = nullptr;
    return 0;
  }
  const int ck = c_kind(a);
  const Key key(a->M, a->N, a->K, a->lda, a->ldb, a->ldc, ck == 2 ? a->ldr : 0, a->b_mode, a->c_f32 ? 1 : 0,
                a->bias ? 1 : 0, a->act, ck);
  auto it = d.plans.find(key);
  if (it == d.plans.end()) {
    Plan p;
    p.ok = make_plan(d, a, p);
    it = d.plans.emplace(key, p).first;
  }
  Plan& p = it->second;
  if (!p.ok) return 0;
  if (a->bias) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a->bias, sizeof(a->bias));
  // C: none (beta 0), D itself (the in-place residual: beta 1; or beta * D), or the separate residual (beta 1)
  const float alpha = 1.0f;
  const float beta = ck == 0 ? 0.0f : (a->R ? 1.0f : a->beta);
  const void* C = ck == 2 ? a->R : a->C;
  const hipblasStatus_t st = hipblasLtMatmul(d.h, p.desc, &alpha, a->B, p.la, a->A, p.lb, &beta, C, p.lc, a->C, p.ld,
                                             &p.algo, d.ws, d.ws_bytes, s);
  if (st != HIPBLAS_STATUS_SUCCESS) {
    octsam::set_error("octsam_gemm: hipblasLtMatmul failed (%d) M=%d N=%d K=%d", (int)st, a->M, a->N, a->K);
    return -1;
  }
  return 1;
}

extern "C" int octsam_gemm_set_workspace(void* ws, int64_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    octsam::set_error("octsam_gemm_set_workspace: no device");
    return 1;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  Dev& d = g_devs[dev];
  if (d.ws && (ws != d.ws || (size_t)bytes != d.ws_bytes)) {
    // plans were made against the old size: drop them (the handle stays)
    for (auto& kv : d.plans) {
      Plan& p = kv.second;
      if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
      if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
      if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
      if (p.lc) hipblasLtMatrixLayoutDestroy(p.lc);
      if (p.ld) hipblasLtMatrixLayoutDestroy(p.ld);
    }
    d.plans.clear();
  }
  d.ws = bytes > 0 ? ws : nullptr;
  d.ws_bytes = bytes > 0 ? (size_t)bytes : 0;
  return 0;
}
