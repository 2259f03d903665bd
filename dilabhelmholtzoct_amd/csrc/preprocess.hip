// SamProcessor image path on the GPU: PIL-exact bilinear resize (8-bit fixed
// point, two separable passes with uint8 rounding between them), rescale 1/255 + normalize as a per-channel
// lookup table, zero pad to the model's square input, fp32 planar [B, 3, out_h, out_w].
//
// Replaces hf:image_processing_pil_sam.py:227-263 (resize -> rescale -> normalize -> pad) whose resize is
// Pillow's ImagingResample (BILINEAR, 8 bpc): per output column / row a window [min, min + cnt) of source
// pixels with int32 weights of 22 fractional bits; each pass adds 1 << 21, shifts right by 22 and clamps
// to [0, 255]. The horizontal pass runs first (Pillow's order) and its uint8 result feeds the vertical pass;
// the integer arithmetic is recomputed per output pixel, so the result is the same bytes Pillow produces.
// Weight tables are built on the host in double precision (dilabhelmholtzoct_amd/preprocess.py).
//
// Layout: one workgroup per (output row, image). The <= KMAX source rows the row's vertical window needs
// are staged in LDS as bytes (HWC, 3 channels), then each thread finishes 4 consecutive output columns and
// writes a float4 per channel plane (full 64-B runs per 4 lanes, coalesced). HBM-bound on the fp32 writes:
// 12.6 MB per 1024^2 image vs 0.76 MB of uint8 input.
#include "common.h"
#include "../../include/octsam.h"

namespace {

constexpr int KMAX = 16; // max taps per pass (bilinear: 3 when upscaling, 2*ceil(scale)+1 when reducing)

__device__ __forceinline__ int clip8(int v) { return min(max(v >> 22, 0), 255); }

__global__ __launch_bounds__(256) void sam_preprocess_kernel(const uint8_t* __restrict__ img, int H, int W,
                                                             long long img_stride, const int* __restrict__ xtab,
                                                             int kx, const int* __restrict__ ytab, int ky, int rh,
                                                             int rw, const float* __restrict__ lut,
                                                             float* __restrict__ out, int out_h, int out_w) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rows[];
  const int y = blockIdx.x, b = blockIdx.y;
  const long long plane = (long long)out_h * out_w;
  float* o = out + (long long)b * 3 * plane + (long long)y * out_w;
  if (y >= rh) {  // bottom padding
    for (int x = threadIdx.x * 4; x < out_w; x += blockDim.x * 4)
#pragma unroll
      for (int c = 0; c < 3; ++c) *(float4*)(o + c * plane + x) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int* yt = ytab + y * (2 + ky);
  const int ymin = yt[0], ycnt = yt[1];
  // stage source rows ymin .. ymin + ycnt - 1 (contiguous in HWC) as 32-bit words when aligned
  const uint8_t* src = img + (long long)b * img_stride + (long long)ymin * W * 3;
  const int nbytes = ycnt * W * 3;
  if ((((uintptr_t)src) & 3) == 0 && (nbytes & 3) == 0) {
    for (int i = threadIdx.x; i < nbytes / 4; i += blockDim.x) ((uint32_t*)rows)[i] = ((const uint32_t*)src)[i];
  } else {
    for (int i = threadIdx.x; i < nbytes; i += blockDim.x) rows[i] = src[i];
  }
  __syncthreads();
  for (int x0 = threadIdx.x * 4; x0 < out_w; x0 += blockDim.x * 4) {
    float r[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = x0 + e;
      if (x >= rw) {  // right padding
#pragma unroll
        for (int c = 0; c < 3; ++c) r[c][e] = 0.0f;
        continue;
      }
      const int* xt = xtab + x * (2 + kx);
      const int xmin = xt[0], xcnt = xt[1];
      int acc[3] = {1 << 21, 1 << 21, 1 << 21};
      for (int j = 0; j < ycnt; ++j) {
        const uint8_t* row = rows + (j * W + xmin) * 3;
        const int wyj = yt[2 + j];
        int h[3] = {1 << 21, 1 << 21, 1 << 21};
        for (int i = 0; i < xcnt; ++i) {
          const int w = xt[2 + i];
#pragma unroll
          for (int c = 0; c < 3; ++c) h[c] += (int)row[i * 3 + c] * w;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += clip8(h[c]) * wyj;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) r[c][e] = lut[c * 256 + clip8(acc[c])];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) *(float4*)(o + c * plane + x0) = make_float4(r[c][0], r[c][1], r[c][2], r[c][3]);
  }
}

}  // namespace

extern "C" int octsam_sam_preprocess(const uint8_t* images, int32_t B, int32_t H, int32_t W, int64_t img_stride,
                                     const int32_t* xtab, int32_t kx, const int32_t* ytab, int32_t ky, int32_t rh,
                                     int32_t rw, const float* lut, float* out, int32_t out_h, int32_t out_w,
                                     void* stream) {
  OCTSAM_CHECK_ARG(images && xtab && ytab && lut && out && B > 0 && H > 0 && W > 0,
                   "octsam_sam_preprocess: bad args");
  OCTSAM_CHECK_ARG(kx >= 1 && kx <= KMAX && ky >= 1 && ky <= KMAX,
                   "octsam_sam_preprocess: taps per pass must be in [1, %d] (got %d, %d)", KMAX, kx, ky);
  OCTSAM_CHECK_ARG(rh >= 1 && rh <= out_h && rw >= 1 && rw <= out_w && out_w % 4 == 0,
                   "octsam_sam_preprocess: resized %dx%d must fit the %dx%d output (width %% 4 == 0)", rh, rw,
                   out_h, out_w);
  OCTSAM_CHECK_ARG(((uintptr_t)out & 15) == 0 && img_stride >= (int64_t)H * W * 3,
                   "octsam_sam_preprocess: output must be 16-B aligned, image stride >= H*W*3");
  const int smem = ky * W * 3;
  OCTSAM_CHECK_ARG(smem <= 65536, "octsam_sam_preprocess: %d source rows of width %d exceed 64 KiB of LDS", ky, W);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sam_preprocess_kernel, dim3(out_h, B), dim3(256), (smem + 15) & ~15, s, images, H, W,
                     (long long)img_stride, xtab, kx, ytab, ky, rh, rw, lut, out, out_h, out_w);
  OCTSAM_LAUNCH_CHECK("octsam_sam_preprocess");
  return 0;
}
