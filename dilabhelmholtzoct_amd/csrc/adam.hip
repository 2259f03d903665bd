// Fused Adam over a flat fp32 parameter buffer (torch.optim.Adam, foreach/single-tensor math:
// lerp first moment, addcmul second moment, bias-corrected addcdiv; L2 weight decay added to the
// gradient), optionally refreshing a bf16 copy of the parameters for the next forward.
// Replaces Adam(model.mask_decoder.parameters(), lr, weight_decay).step()
// (ref:octsam/models/training_utils.py:31,68).
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
  hipLaunchKernelGGL(cast16_kernel<bf16>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16*)y, n);
  OCTSAM_LAUNCH_CHECK("octsam_cast_bf16");
  return 0;
}

extern "C" int octsam_cast_f16(const float* x, void* y, int64_t n, void* stream) {
  OCTSAM_CHECK_ARG(x && y && n > 0, "octsam_cast_f16: bad args");
  hipLaunchKernelGGL(cast16_kernel<_Float16>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     x, (_Float16*)y, n);
  OCTSAM_LAUNCH_CHECK("octsam_cast_f16");
  return 0;
}
