// hipBLASLt on the encoder's GEMMs with this step's epilogues (diagnostic yardstick, not product code): MLP2 and
// the projection as D = A W^T + bias + D in place (fp32 D, beta = 1), QKV / MLP1 as bf16 D = A W^T + bias; every
// heuristic candidate timed with hipEvents (median of 20 after 5 warm; min over 3 rounds interleaved with
// octsam_gemm's), its bits checked run to run and against octsam_gemm on the same operands (max |diff| / max |ref|).
// build: hipcc --offload-arch=gfx950 -O2 blaslt_epi.cpp -o blaslt_epi -lhipblaslt -L../../dilabhelmholtzoct_amd
//        -loctsam_hip -Wl,-rpath,$PWD/../../dilabhelmholtzoct_amd
#include <hip/hip_runtime.h>
#include <hip/hip_bfloat16.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/octsam.h"

#define CK(x)                                                                 \
  do {                                                                        \
    auto e_ = (x);                                                            \
    if ((int)e_ != 0) {                                                       \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)e_); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void fill_bf16(uint16_t* p, long long n, unsigned seed, float scale) {
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)(i * 2654435761u) ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    float v = ((h & 0xffff) / 65535.0f - 0.5f) * scale;
    unsigned u = __float_as_uint(v);
    p[i] = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
}
__global__ void fill_f32(float* p, long long n, unsigned seed, float scale) {
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)(i * 2246822519u) ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = ((h & 0xffff) / 65535.0f - 0.5f) * scale;
  }
}

struct Shape {
  const char* name;
  int M, N, K;
  bool f32_inplace;  // fp32 D += A W^T + bias; else bf16 D = A W^T + bias
  int gelu = 0;      // 1: bf16 D = GELU(A W^T + bias) (hipBLASLt's GELU epilogue against octsam's exact-erf GELU)
};

int main() {
  hipblasLtHandle_t lt;
  CK(hipblasLtCreate(&lt));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t ws_bytes = 64 << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  Shape shapes[] = {{"fc2", 32768, 768, 3072, true}, {"qkv", 32768, 2304, 768, false},
                    {"proj", 32768, 768, 768, true}, {"fc1_bias_only", 32768, 3072, 768, false},
                    {"dec_256x512", 688128, 256, 512, false}, {"dec_256x256", 688128, 256, 256, false},
                    {"dec_128x256", 688128, 128, 256, false}, {"dec_384x256", 688128, 384, 256, false},
                    {"fc1_gelu", 32768, 3072, 768, false, 1},
                    {"tok_256x256", 1176, 256, 256, false}, {"tok_2048x256", 1176, 2048, 256, false},
                    {"tok_256x2048", 1176, 256, 2048, false}};
  const char* only = std::getenv("SHAPES");
  for (const Shape& s : shapes) {
    if (only) {  // SHAPES: comma list of name prefixes
      bool hit = false;
      for (const char* t = only; *t;) {
        const char* e = std::strchr(t, ',');
        const size_t n = e ? (size_t)(e - t) : std::strlen(t);
        if (n && std::strncmp(s.name, t, n) == 0) hit = true;
        t += n + (e ? 1 : 0);
      }
      if (!hit) continue;
    }
    const long long nA = (long long)s.M * s.K, nW = (long long)s.N * s.K, nD = (long long)s.M * s.N;
    uint16_t *A, *W;
    float* bias;
    void *D, *D0, *Dref;
    const size_t es = s.f32_inplace ? 4 : 2;
    CK(hipMalloc(&A, nA * 2));
    CK(hipMalloc(&W, nW * 2));
    CK(hipMalloc(&bias, s.N * 4));
    CK(hipMalloc(&D, nD * es));
    CK(hipMalloc(&D0, nD * es));
    CK(hipMalloc(&Dref, nD * es));
    fill_bf16<<<2048, 256, 0, st>>>(A, nA, 1, 2.0f);
    fill_bf16<<<2048, 256, 0, st>>>(W, nW, 2, 2.0f / std::sqrt((float)s.K));
    fill_f32<<<64, 256, 0, st>>>(bias, s.N, 3, 1.0f);
    if (s.f32_inplace) fill_f32<<<2048, 256, 0, st>>>((float*)D0, nD, 4, 2.0f);
    CK(hipStreamSynchronize(st));

    // col-major view: D^T [N x M] = op_T(W^T stored K x N) * (A^T stored K x M)
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtEpilogue_t epi = s.gelu ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    hipDataType bt = HIP_R_32F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    hipblasLtMatrixLayout_t la, lb, lc;
    const hipDataType dt = s.f32_inplace ? HIP_R_32F : HIP_R_16BF;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, s.K, s.N, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, s.K, s.M, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lc, dt, s.N, s.M, s.N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsz = ws_bytes;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    hipblasLtMatmulHeuristicResult_t res[16];
    int nres = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(lt, desc, la, lb, lc, lc, pref, 16, res, &nres));
    const float alpha = 1.0f, beta = s.f32_inplace ? 1.0f : 0.0f;

    // octsam_gemm reference on the same operands
    octsam_gemm_args g;
    std::memset(&g, 0, sizeof(g));
    g.A = A; g.B = W; g.C = Dref; g.bias = bias; g.R = s.f32_inplace ? Dref : nullptr;
    g.M = s.M; g.N = s.N; g.K = s.K; g.batch = 1;
    g.lda = s.K; g.ldb = s.K; g.ldc = s.N; g.ldr = s.N;
    g.alpha = 1.0f; g.beta = 0.0f; g.c_f32 = s.f32_inplace; g.r_f32 = s.f32_inplace;
    g.act = s.gelu ? OCTSAM_ACT_GELU : 0;
    auto run_ours = [&]() {
      if (s.f32_inplace) CK(hipMemcpyAsync(Dref, D0, nD * es, hipMemcpyDeviceToDevice, st));
      CK(octsam_gemm(&g, st));
    };
    const bool graph_mode = std::getenv("GRAPH") != nullptr;
    auto time_graph = [&](auto&& fn) {
      hipGraph_t gr;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < 50; ++i) fn();
      CK(hipStreamEndCapture(st, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      float best = 1e30f;
      for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms * 1e3f / 50);
      }
      hipGraphExecDestroy(ge);
      hipGraphDestroy(gr);
      return best;
    };
    auto time_it = [&](auto&& fn, bool reset) {
      if (graph_mode) return time_graph(fn);
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      std::vector<float> t;
      for (int it = 0; it < 25; ++it) {
        if (reset && s.f32_inplace) CK(hipMemcpyAsync(D, D0, nD * es, hipMemcpyDeviceToDevice, st));
        CK(hipEventRecord(e0, st));
        fn();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 5) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      hipEventDestroy(e0);
      hipEventDestroy(e1);
      return t[t.size() / 2];
    };
    float ours = 1e30f;  // (min over rounds interleaved with the candidates: no clock-ramp bias)
    run_ours();
    CK(hipStreamSynchronize(st));
    std::vector<float> ref(nD);
    {
      std::vector<uint16_t> tmp;
      if (s.f32_inplace) {
        CK(hipMemcpy(ref.data(), Dref, nD * 4, hipMemcpyDeviceToHost));
      } else {
        tmp.resize(nD);
        CK(hipMemcpy(tmp.data(), Dref, nD * 2, hipMemcpyDeviceToHost));
        for (long long i = 0; i < nD; ++i) { unsigned u = (unsigned)tmp[i] << 16; std::memcpy(&ref[i], &u, 4); }
      }
    }
    std::vector<float> cand(nres, 1e30f);
    for (int round = 0; round < 3; ++round) {
      ours = std::min(ours, time_it([&]() { CK(octsam_gemm(&g, st)); }, false));
      for (int r = 0; r < nres; ++r)
        cand[r] = std::min(cand[r], time_it([&]() {
          CK(hipblasLtMatmul(lt, desc, &alpha, W, la, A, lb, &beta, D, lc, D, lc, &res[r].algo, ws, ws_bytes, st));
        }, true));
    }
    std::printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"octsam_us\": %.1f, \"candidates\": %d}\n", s.name,
                s.M, s.N, s.K, ours, nres);
    for (int r = 0; r < nres; ++r) {
      auto run = [&]() {
        CK(hipblasLtMatmul(lt, desc, &alpha, W, la, A, lb, &beta, D, lc, D, lc, &res[r].algo, ws, ws_bytes, st));
      };
      float us = cand[r];
      // bits run to run, and against octsam_gemm
      std::vector<uint8_t> b1(nD * es), b2(nD * es);
      for (int k = 0; k < 2; ++k) {
        if (s.f32_inplace) CK(hipMemcpyAsync(D, D0, nD * es, hipMemcpyDeviceToDevice, st));
        run();
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(k ? b2.data() : b1.data(), D, nD * es, hipMemcpyDeviceToHost));
      }
      double md = 0, mr = 0;
      for (long long i = 0; i < nD; ++i) {
        float v;
        if (s.f32_inplace) std::memcpy(&v, b1.data() + 4 * i, 4);
        else { unsigned u = (unsigned)(*(uint16_t*)(b1.data() + 2 * i)) << 16; std::memcpy(&v, &u, 4); }
        md = std::max(md, (double)std::fabs(v - ref[i]));
        mr = std::max(mr, (double)std::fabs(ref[i]));
      }
      std::printf("  {\"algo\": %d, \"us\": %.1f, \"deterministic\": %s, \"rel_vs_octsam\": %.2e}\n", r, us,
                  b1 == b2 ? "true" : "false", md / mr);
    }
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(desc);
    hipFree(A); hipFree(W); hipFree(bias); hipFree(D); hipFree(D0); hipFree(Dref);
  }
  hipFree(ws);
  hipblasLtDestroy(lt);
  return 0;
}
