// Fused Adam over a flat fp32 parameter buffer (torch.optim.Adam, foreach/single-tensor math:
// lerp first moment, addcmul second moment, bias-corrected addcdiv; L2 weight decay added to the
// gradient), optionally refreshing a bf16 copy of the parameters for the next forward.
// Replaces Adam(model.mask_decoder.parameters(), lr, weight_decay).step()
// (ref:octsam/models/training_utils.py:31,68).
#include <algorithm>
#include "common.h"
#include "../../include/octsam.h"

namespace {
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float omb1, float beta2, float omb2, float eps,
                            float wd, float step_size, float bc2_sqrt, bf16* __restrict__ pb) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float pv = p[i];
  float gv = g[i];
  if (wd != 0.0f) gv = gv + wd * pv;
  float mv = m[i];
  mv = mv + omb1 * (gv - mv);  // torch.lerp(m, g, 1-beta1), weight < 0.5 branch
  float vv = v[i] * beta2 + omb2 * gv * gv;  // mul_(beta2).addcmul_(g, g, value=1-beta2)
  float denom = sqrtf(vv) / bc2_sqrt + eps;
  pv = pv + (-step_size) * (mv / denom);
  p[i] = pv;
  m[i] = mv;
  v[i] = vv;
  if (pb) pb[i] = (bf16)pv;
}

template <typename E>
__global__ void cast16_kernel(const float* __restrict__ x, E* __restrict__ y, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (E)x[i];
}
// 8 elements per thread: two 16-B loads, one 16-B store (n % 8 == 0, 16-B aligned x and y; host-checked)
template <typename E>
__global__ __launch_bounds__(256) void cast16x8_kernel(const float4* __restrict__ x, uint4* __restrict__ y, long long n8) {
  typedef E e8 __attribute__((ext_vector_type(8)));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const float4 a = x[2 * i], b = x[2 * i + 1];
    const e8 o = {(E)a.x, (E)a.y, (E)a.z, (E)a.w, (E)b.x, (E)b.y, (E)b.z, (E)b.w};
    y[i] = __builtin_bit_cast(uint4, o);
  }
}
template <typename E>
void launch_cast(const float* x, void* y, long long n, hipStream_t s) {
  if (n % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    const long long n8 = n / 8;
    const long long blocks = std::min<long long>((n8 + 255) / 256, 256LL * 16);
    hipLaunchKernelGGL(cast16x8_kernel<E>, dim3((unsigned)blocks), dim3(256), 0, s, (const float4*)x, (uint4*)y, n8);
  } else {
    hipLaunchKernelGGL(cast16_kernel<E>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, (E*)y, n);
  }
}
}  // namespace

extern "C" int octsam_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double beta1,
                           double beta2, float eps, float weight_decay, float step_size, float bias_correction2_sqrt,
                           void* params_bf16, void* stream) {
  OCTSAM_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && n > 0, "octsam_adam: bad args");
  // 1 - beta in double, then rounded: the scalars torch.optim.Adam hands its fp32 kernels
  const float omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, params, grads,
                     exp_avg, exp_avg_sq, n, omb1, (float)beta2, omb2, eps, weight_decay, step_size,
                     bias_correction2_sqrt, (bf16*)params_bf16);
  OCTSAM_LAUNCH_CHECK("octsam_adam");
  return 0;
}

extern "C" int octsam_cast_bf16(const float* x, void* y, int64_t n, void* stream) {
  OCTSAM_CHECK_ARG(x && y && n > 0, "octsam_cast_bf16: bad args");
  launch_cast<bf16>(x, y, n, (hipStream_t)stream);
  OCTSAM_LAUNCH_CHECK("octsam_cast_bf16");
  return 0;
}

extern "C" int octsam_cast_f16(const float* x, void* y, int64_t n, void* stream) {
  OCTSAM_CHECK_ARG(x && y && n > 0, "octsam_cast_f16: bad args");
  launch_cast<_Float16>(x, y, n, (hipStream_t)stream);
  OCTSAM_LAUNCH_CHECK("octsam_cast_f16");
  return 0;
}
