// Shared helpers for the octsam HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace octsam {

// Thread-local error message, exposed through octsam_last_error().
void set_error(const char* fmt, ...);

}  // namespace octsam

#define OCTSAM_CHECK_ARG(cond, ...)                 \
  do {                                              \
    if (!(cond)) {                                  \
      octsam::set_error(__VA_ARGS__);               \
      return 1;                                     \
    }                                               \
  } while (0)

#define OCTSAM_LAUNCH_CHECK(name)                                                   \
  do {                                                                              \
    hipError_t e_ = hipGetLastError();                                              \
    if (e_ != hipSuccess) {                                                         \
      octsam::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));      \
      return (int)e_;                                                               \
    }                                                                               \
  } while (0)

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
// Branch-free erf (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7) for epilogues whose output is bf16:
// libm erff branches per value range, which diverges inside a wave and serialises a GEMM epilogue.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-ax * ax);
  return copysignf(y, x);
}
// GELU on the same A&S erf, rearranged so that a pair of values runs on packed f32 arithmetic: with
// z = |x|/sqrt2, t = 1/(1 + p z), q = P(t) t exp(-x^2/2) (so erf(z) = 1 - q), GELU(x) = max(x, 0) - |x q / 2|
// (x >= 0: x - x q/2; x < 0: x q/2). The 1/2 is folded into P's coefficients (exact). gelu_fast and
// gelu_fast2 run the same operation sequence (packed FMA/MUL round like their scalar forms), so every GEMM
// epilogue — scalar or pairwise — gives bit-identical outputs.
namespace gelu_c {
constexpr float P = 0.3275911f * 0.70710678118654752f, A1 = 0.5f * 0.254829592f, A2 = 0.5f * -0.284496736f,
                A3 = 0.5f * 1.421413741f, A4 = 0.5f * -1.453152027f, A5 = 0.5f * 1.061405429f,
                E = -0.5f * 1.4426950408889634f;  // exp(-x^2/2) = exp2(E x^2)
}
typedef float fx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float gelu_fast(float x) {
  using namespace gelu_c;
  const float t = __builtin_amdgcn_rcpf(fmaf(P, fabsf(x), 1.0f));
  float pp = fmaf(t, A5, A4);
  pp = fmaf(pp, t, A3);
  pp = fmaf(pp, t, A2);
  pp = fmaf(pp, t, A1);
  const float u = pp * t, w = (x * E) * x;
  const float h = (u * __builtin_amdgcn_exp2f(w)) * x;
  return fmaxf(x, 0.0f) - fabsf(h);
}
__device__ __forceinline__ fx2 gelu_fast2(fx2 x) {
  using namespace gelu_c;
  const fx2 t = {__builtin_amdgcn_rcpf(fmaf(P, fabsf(x[0]), 1.0f)), __builtin_amdgcn_rcpf(fmaf(P, fabsf(x[1]), 1.0f))};
  const fx2 a5 = {A5, A5}, a4 = {A4, A4}, a3 = {A3, A3}, a2 = {A2, A2}, a1 = {A1, A1}, e2 = {E, E};
  fx2 pp = __builtin_elementwise_fma(t, a5, a4);
  pp = __builtin_elementwise_fma(pp, t, a3);
  pp = __builtin_elementwise_fma(pp, t, a2);
  pp = __builtin_elementwise_fma(pp, t, a1);
  const fx2 u = pp * t, w = (x * e2) * x;
  const fx2 ex = {__builtin_amdgcn_exp2f(w[0]), __builtin_amdgcn_exp2f(w[1])};
  const fx2 h = (u * ex) * x;
  return (fx2){fmaxf(x[0], 0.0f) - fabsf(h[0]), fmaxf(x[1], 0.0f) - fabsf(h[1])};
}
__device__ __forceinline__ float gelu_fast_grad(float x) {
  return 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  // d/dx [0.5 x (1 + erf(x/sqrt2))] = 0.5 (1 + erf(x/sqrt2)) + x * exp(-x^2/2) / sqrt(2 pi)
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) +
         x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
