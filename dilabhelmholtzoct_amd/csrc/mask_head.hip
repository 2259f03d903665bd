// Mask prediction head of SamMaskDecoder: masks = hyper_in @ upscaled_embedding
// (hf:modeling_sam.py:523-542), forward and backward.
//
// The upscaled embedding is produced by two ConvTranspose2d(k2,s2) GEMMs whose outputs are kept in
// "blocked" order: row = (((((y1*64+x1)*2+dy1)*2+dx1)*2+dy2)*2+dx2) with 32 channels, i.e. output pixel
// y = 4*y1 + 2*dy1 + dy2, x = 4*x1 + 2*dx1 + dx2 of the 256x256 mask. No pixel shuffle is ever
// materialised; these kernels translate the index while reading/writing.
#include "common.h"
#include "../../include/octsam.h"

namespace {

__device__ __forceinline__ int blocked_to_pixel(int b) {
  int dx2 = b & 1, dy2 = (b >> 1) & 1, dx1 = (b >> 2) & 1, dy1 = (b >> 3) & 1, x1 = (b >> 4) & 63, y1 = (b >> 10) & 63;
  int y = 4 * y1 + 2 * dy1 + dy2, x = 4 * x1 + 2 * dx1 + dx2;
  return y * 256 + x;
}

// up2 bf16 [P, 65536, 32]; hyper fp32 [P, ntok, 32]; masks fp32 [P, ntok, 65536] (row-major 256x256)
__global__ __launch_bounds__(256) void mask_dot_fwd_kernel(const bf16* __restrict__ up2, const float* __restrict__ hyper,
                                                           int ntok, float* __restrict__ masks) {
  const int p = blockIdx.y;
  __shared__ float sh[4][32];
  for (int e = threadIdx.x; e < ntok * 32; e += 256) sh[e / 32][e % 32] = hyper[(long long)p * ntok * 32 + e];
  __syncthreads();
  const int b = blockIdx.x * 256 + threadIdx.x;
  const bf16* row = up2 + ((long long)p * 65536 + b) * 32;
  float u[32];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bf16x8 v = *(const bf16x8*)(row + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) u[8 * c + e] = (float)v[e];
  }
  const int pix = blocked_to_pixel(b);
  for (int t = 0; t < ntok; ++t) {
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < 32; ++c) acc += sh[t][c] * u[c];
    masks[((long long)p * ntok + t) * 65536 + pix] = acc;
  }
}

// d_up2pre bf16 [P,65536,32] = (sum_t dmask[t,pix] * hyper[t]) * gelu'(up2pre)
// part fp32 [gridDim.x=256, P, ntok, 32]: per-block partial of d_hyper = sum_pix dmask * up2
template <int NT>
__global__ __launch_bounds__(256) void mask_dot_bwd_kernel(const bf16* __restrict__ up2, const bf16* __restrict__ up2pre,
                                                           const float* __restrict__ hyper,
                                                           const float* __restrict__ dmask, bf16* __restrict__ dup2pre,
                                                           float* __restrict__ part) {
  const int p = blockIdx.y;
  constexpr int ntok = NT;
  __shared__ float sh[NT][32];
  __shared__ float red[4][NT][32];
  for (int e = threadIdx.x; e < ntok * 32; e += 256) sh[e / 32][e % 32] = hyper[(long long)p * ntok * 32 + e];
  __syncthreads();
  const int b = blockIdx.x * 256 + threadIdx.x;
  const long long ro = ((long long)p * 65536 + b) * 32;
  const int pix = blocked_to_pixel(b);
  float dm[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dm[t] = dmask[((long long)p * ntok + t) * 65536 + pix];
  float hacc[NT][32];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bf16x8 u = *(const bf16x8*)(up2 + ro + 8 * c);
    bf16x8 pre = *(const bf16x8*)(up2pre + ro + 8 * c);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int ch = 8 * c + e;
      float g = 0.0f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        g += dm[t] * sh[t][ch];
        hacc[t][ch] = dm[t] * (float)u[e];
      }
      o[e] = (bf16)(g * gelu_erf_grad((float)pre[e]));
    }
    *(bf16x8*)(dup2pre + ro + 8 * c) = o;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ch = 0; ch < 32; ++ch) {
      float s = wave_sum(hacc[t][ch]);
      if (lane == 0) red[wave][t][ch] = s;
    }
  __syncthreads();
  for (int e = threadIdx.x; e < ntok * 32; e += 256) {
    int t = e / 32, ch = e % 32;
    part[(((long long)blockIdx.x * gridDim.y + p) * ntok + t) * 32 + ch] =
        red[0][t][ch] + red[1][t][ch] + red[2][t][ch] + red[3][t][ch];
  }
}

}  // namespace

extern "C" int octsam_mask_dot_fwd(const void* up2, const float* hyper, int32_t P, int32_t ntok, float* masks,
                                   void* stream) {
  OCTSAM_CHECK_ARG(up2 && hyper && masks && P > 0 && ntok >= 1 && ntok <= 4, "octsam_mask_dot_fwd: bad args");
  hipLaunchKernelGGL(mask_dot_fwd_kernel, dim3(65536 / 256, P), dim3(256), 0, (hipStream_t)stream, (const bf16*)up2,
                     hyper, ntok, masks);
  OCTSAM_LAUNCH_CHECK("octsam_mask_dot_fwd");
  return 0;
}

/* partials: fp32 [256, P, ntok, 32] (reduce over the 256 blocks with octsam_splitk_reduce) */
extern "C" int octsam_mask_dot_bwd(const void* up2, const void* up2pre, const float* hyper, int32_t P, int32_t ntok,
                                   const float* dmask, void* dup2pre, float* partials, void* stream) {
  OCTSAM_CHECK_ARG(up2 && up2pre && hyper && dmask && dup2pre && partials && P > 0 && ntok >= 1 && ntok <= 4,
                   "octsam_mask_dot_bwd: bad args");
  dim3 grid(65536 / 256, P);
  hipStream_t s = (hipStream_t)stream;
  if (ntok == 1)
    hipLaunchKernelGGL(mask_dot_bwd_kernel<1>, grid, dim3(256), 0, s, (const bf16*)up2, (const bf16*)up2pre, hyper, dmask,
                       (bf16*)dup2pre, partials);
  else if (ntok == 3)
    hipLaunchKernelGGL(mask_dot_bwd_kernel<3>, grid, dim3(256), 0, s, (const bf16*)up2, (const bf16*)up2pre, hyper, dmask,
                       (bf16*)dup2pre, partials);
  else if (ntok == 4)
    hipLaunchKernelGGL(mask_dot_bwd_kernel<4>, grid, dim3(256), 0, s, (const bf16*)up2, (const bf16*)up2pre, hyper, dmask,
                       (bf16*)dup2pre, partials);
  else {
    octsam::set_error("octsam_mask_dot_bwd: ntok must be 1, 3 or 4");
    return 1;
  }
  OCTSAM_LAUNCH_CHECK("octsam_mask_dot_bwd");
  return 0;
}
