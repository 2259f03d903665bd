// hipBLASLt for the encoder's plain GEMMs: the in-place-residual MLP2 / projection and the QKV projection (library
// GEMMs; the hand-written kernels keep the rest).
//
// The encoder's MLP2 and attention projection are x += A W^T + b on the fp32 residual stream x (hf:modeling_sam.py
// SamVisionLayer: hidden_states = residual + mlp(...) / + attn(...)): a plain GEMM with a bias epilogue and beta = 1
// into an fp32 D. hipBLASLt's stream-K kernels run it faster than the 8-phase kernel, whose 384 tiles leave
// half of a second wave idle at MLP2 (same-operand yardstick, scripts/micro/blaslt_epi.cpp,
// profiles/r05/blaslt_yardstick.log: MLP2 180.4 -> 143.6 us, projection 67.3 -> 60.6 us).
//
// - Column-major view: D^T [N x M] = op_T(W^T stored K x N) x A^T (stored K x M); bias per D^T row = output feature.
// - Algorithm: the heuristic's first candidate for the shape, planned once per (device, shape, types). The plan is
//   deterministic for one library build and device, so eager, graph-captured and multi-process runs take the same
//   kernel and the same bits (run-to-run bit-identical, checked in tests/test_gpu_gemm.py).
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
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
};
struct Dev {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // (M, N, K, f16 operands, bias, 16-bit D)
  std::map<std::tuple<int, int, int, int, int, int>, Plan> plans;
};
std::mutex g_mu;
std::map<int, Dev> g_devs;

bool make_plan(Dev& d, const octsam_gemm_args* a, bool f16, Plan& p) {
  const hipDataType et = f16 ? HIP_R_16F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  const hipblasLtEpilogue_t epi = a->bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (a->bias) {
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a->bias, sizeof(a->bias));
  }
  if (hipblasLtMatrixLayoutCreate(&p.la, et, a->K, a->N, a->K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, et, a->K, a->M, a->K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, a->c_f32 ? HIP_R_32F : et, a->N, a->M, a->N) != HIPBLAS_STATUS_SUCCESS)
    return false;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t wsz = d.ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(d.h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].workspaceSize > d.ws_bytes) return false;
  p.algo = res[0].algo;
  return true;
}
}  // namespace

int g_blaslt_enabled = 1;  // octsam_gemm_set_fast_path bit 65536 turns it off (A/B)
int g_blaslt_qkv = 1;      // bit 131072 turns the QKV kind off (A/B)

// Eligible, with K-contiguous dense operands, one batch, no activation / scaling / row map, M >= 8192 (the encoder's
// token rows), either
//   x += A W^T (+ bias) with x fp32 and the residual IS the output (in place), N >= 256, K >= 512: MLP2, projection;
//   or a 16-bit D = A W^T + bias, no residual, 2048 <= N <= 4096, K <= 1024: the QKV projection (same-process step
//   A/B 16.28 -> 15.92 ms pipelined, 18.16 -> 17.99 sequential, profiles/r05/blaslt_step_ab.log).
// (MLP1 has the GELU: native. The decoder's plain 16-bit image-side products measured slower in the step.)
bool blaslt_eligible(const octsam_gemm_args* a) {
  if (!(g_blaslt_enabled && a->batch == 1 && a->a_mode == 0 && a->b_mode == 0 && !a->row_map && !a->C_pre &&
        !a->A2 && !a->B2 && !a->a_blk && !a->b_blk && !a->r_blk && !a->k_total && !a->a_colsum && !a->b_colsum &&
        a->act == 0 && a->alpha == 1.0f && a->beta == 0.0f && a->lda == a->K && a->ldb == a->K && a->ldc == a->N &&
        a->M >= 8192))
    return false;
  if (!a->c_f32) return g_blaslt_qkv && a->R == nullptr && a->bias && a->N >= 2048 && a->N <= 4096 && a->K <= 1024;
  return a->r_f32 && a->R == a->C && a->ldr == a->ldc && a->N >= 256 && a->K >= 512;
}

// 1: ran, 0: not taken (no workspace, no plan: the caller runs the native kernels), -1: error (set)
int blaslt_gemm(const octsam_gemm_args* a, hipStream_t s, bool f16) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  Dev& d = g_devs[dev];
  if (!d.ws) return 0;
  if (!d.h && hipblasLtCreate(&d.h) != HIPBLAS_STATUS_SUCCESS) {
    d.h = nullptr;
    return 0;
  }
  const auto key = std::make_tuple(a->M, a->N, a->K, f16 ? 1 : 0, a->bias ? 1 : 0, a->c_f32 ? 0 : 1);
  auto it = d.plans.find(key);
  if (it == d.plans.end()) {
    Plan p;
    p.ok = make_plan(d, a, f16, p);
    it = d.plans.emplace(key, p).first;
  }
  Plan& p = it->second;
  if (!p.ok) return 0;
  if (a->bias) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a->bias, sizeof(a->bias));
  const float alpha = 1.0f, beta = a->c_f32 ? 1.0f : 0.0f;  // (fp32: the in-place residual)
  const hipblasStatus_t st = hipblasLtMatmul(d.h, p.desc, &alpha, a->B, p.la, a->A, p.lb, &beta, a->C, p.lc, a->C,
                                             p.lc, &p.algo, d.ws, d.ws_bytes, s);
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
    }
    d.plans.clear();
  }
  d.ws = bytes > 0 ? ws : nullptr;
  d.ws_bytes = bytes > 0 ? (size_t)bytes : 0;
  return 0;
}
