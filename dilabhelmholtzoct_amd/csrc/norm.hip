// LayerNorm over the last dimension (one wave per row), forward and backward.
//
// Covers nn.LayerNorm of SamVisionLayer (hf:modeling_sam.py:954-972, eps 1e-6), the channels-first
// SamLayerNorm of the neck and of the mask-decoder upscaling (:975-992, :519-521; applied per pixel on
// NHWC data), and the decoder LayerNorms (:306-348; layer_norm_final_attn eps 1e-5, :363).
// Forward options: input fp32/bf16; output bf16 and/or fp32; fused GELU (upscale LN -> GELU);
// row gather (window_partition with zero padding: output row r reads input row src_rows[r], or
// writes zeros when src_rows[r] < 0); mean/rstd saved for backward.
// Backward: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w (optionally through the
// fused GELU); per-block dw/db partials reduced deterministically by octsam_splitk_reduce.
#include "common.h"
#include "../../include/octsam.h"

namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i) { return (float)p[i]; }

template <int PL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, int x_f32, const int* __restrict__ src_rows,
                                                     long long rows, const float* __restrict__ w,
                                                     const float* __restrict__ b, float eps, void* __restrict__ y,
                                                     int y_f32, void* __restrict__ y2, int act,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int D = PL * 64;
  const int lane = threadIdx.x & 63;
  long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  long long src = src_rows ? (long long)src_rows[row] : row;
  float v[PL];
  if (src < 0) {
#pragma unroll
    for (int i = 0; i < PL; ++i) v[i] = 0.0f;
  } else if (x_f32) {
    const float* xr = (const float*)x + src * D;
#pragma unroll
    for (int i = 0; i < PL; ++i) v[i] = xr[i * 64 + lane];
  } else {
    const bf16* xr = (const bf16*)x + src * D;
#pragma unroll
    for (int i = 0; i < PL; ++i) v[i] = (float)xr[i * 64 + lane];
  }
  float out[PL];
  if (src < 0) {
    // window padding: HF pads AFTER layer_norm1, so padded tokens are exact zeros
#pragma unroll
    for (int i = 0; i < PL; ++i) out[i] = 0.0f;
    if (mean_out) { if (lane == 0) { mean_out[row] = 0.0f; rstd_out[row] = 0.0f; } }
  } else {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < PL; ++i) s += v[i];
    const float mean = wave_sum(s) * (1.0f / D);
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < PL; ++i) { float d = v[i] - mean; q += d * d; }
    const float var = wave_sum(q) * (1.0f / D);
    const float rstd = rsqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      int c = i * 64 + lane;
      float o = (v[i] - mean) * rstd * w[c] + b[c];
      if (act == OCTSAM_ACT_GELU) o = gelu_erf(o);
      else if (act == OCTSAM_ACT_RELU) o = fmaxf(o, 0.0f);
      out[i] = o;
    }
    if (mean_out && lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
  }
  if (y_f32) {
    float* yr = (float*)y + row * D;
#pragma unroll
    for (int i = 0; i < PL; ++i) yr[i * 64 + lane] = out[i];
  } else {
    bf16* yr = (bf16*)y + row * D;
#pragma unroll
    for (int i = 0; i < PL; ++i) yr[i * 64 + lane] = (bf16)out[i];
  }
  if (y2) {  // secondary fp32 copy (residual stream)
    float* yr = (float*)y2 + row * D;
#pragma unroll
    for (int i = 0; i < PL; ++i) yr[i * 64 + lane] = out[i];
  }
}

// Backward. grid-stride over rows; each block keeps dw/db partials for its rows.
template <int PL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ dy, int dy_f32, const void* __restrict__ x,
                                                     int x_f32, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ w,
                                                     const float* __restrict__ b, int act, long long rows,
                                                     void* __restrict__ dx, int dx_f32, float beta,
                                                     bf16* __restrict__ dx2, float* __restrict__ dw_part,
                                                     float* __restrict__ db_part) {
  constexpr int D = PL * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dwa[PL], dba[PL];
#pragma unroll
  for (int i = 0; i < PL; ++i) { dwa[i] = 0.0f; dba[i] = 0.0f; }
  for (long long row = (long long)blockIdx.x * 4 + wave; row < rows; row += (long long)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[PL], g[PL];
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      int c = i * 64 + lane;
      float xv = x_f32 ? ((const float*)x)[row * D + c] : (float)((const bf16*)x)[row * D + c];
      float gy = dy_f32 ? ((const float*)dy)[row * D + c] : (float)((const bf16*)dy)[row * D + c];
      xh[i] = (xv - mu) * rs;
      if (act == OCTSAM_ACT_GELU) {
        float pre = xh[i] * w[c] + b[c];
        gy *= gelu_erf_grad(pre);
      } else if (act == OCTSAM_ACT_RELU) {
        float pre = xh[i] * w[c] + b[c];
        gy = pre > 0.0f ? gy : 0.0f;
      }
      dwa[i] += gy * xh[i];
      dba[i] += gy;
      g[i] = gy * w[c];
    }
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int i = 0; i < PL; ++i) { s1 += g[i]; s2 += g[i] * xh[i]; }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      int c = i * 64 + lane;
      float d = rs * (g[i] - s1 - xh[i] * s2);
      if (dx_f32) {
        float* p = (float*)dx + row * D + c;
        d = (beta != 0.0f ? beta * *p : 0.0f) + d;
        *p = d;
      } else {
        bf16* p = (bf16*)dx + row * D + c;
        d = (beta != 0.0f ? beta * (float)*p : 0.0f) + d;
        *p = (bf16)d;
      }
      if (dx2) dx2[row * D + c] = (bf16)d;
    }
  }
  // block-level reduction of dw/db partials over the 4 waves through LDS
  __shared__ float red[4][D];
#pragma unroll
  for (int i = 0; i < PL; ++i) red[wave][i * 64 + lane] = dwa[i];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) dw_part[(long long)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PL; ++i) red[wave][i * 64 + lane] = dba[i];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) db_part[(long long)blockIdx.x * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

template <int PL>
int fwd_launch(const void* x, int x_f32, const int* src_rows, long long rows, const float* w, const float* b, float eps,
               void* y, int y_f32, void* y2, int act, float* mean, float* rstd, hipStream_t s) {
  unsigned blocks = (unsigned)((rows + 3) / 4);
  hipLaunchKernelGGL(ln_fwd_kernel<PL>, dim3(blocks), dim3(256), 0, s, x, x_f32, src_rows, rows, w, b, eps, y, y_f32,
                     y2, act, mean, rstd);
  OCTSAM_LAUNCH_CHECK("octsam_layernorm_fwd");
  return 0;
}

template <int PL>
int bwd_launch(const void* dy, int dy_f32, const void* x, int x_f32, const float* mean, const float* rstd,
               const float* w, const float* b, int act, long long rows, void* dx, int dx_f32, float beta,
               bf16* dx2, float* dw_part, float* db_part, int nblocks, hipStream_t s) {
  hipLaunchKernelGGL(ln_bwd_kernel<PL>, dim3(nblocks), dim3(256), 0, s, dy, dy_f32, x, x_f32, mean, rstd, w, b, act,
                     rows, dx, dx_f32, beta, dx2, dw_part, db_part);
  OCTSAM_LAUNCH_CHECK("octsam_layernorm_bwd");
  return 0;
}

}  // namespace

extern "C" int octsam_layernorm_fwd(const void* x, int32_t x_f32, const int32_t* src_rows, int64_t rows, int32_t D,
                                    const float* w, const float* b, float eps, void* y, int32_t y_f32, float* y2_f32,
                                    int32_t act, float* mean, float* rstd, void* stream) {
  OCTSAM_CHECK_ARG(x && w && b && y && rows > 0, "octsam_layernorm_fwd: bad args");
  OCTSAM_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "octsam_layernorm_fwd: mean/rstd both or neither");
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 64: return fwd_launch<1>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 256: return fwd_launch<4>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 768: return fwd_launch<12>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 1024: return fwd_launch<16>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 1280: return fwd_launch<20>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    default: octsam::set_error("octsam_layernorm_fwd: unsupported D=%d", D); return 1;
  }
}

extern "C" int octsam_layernorm_bwd(const void* dy, int32_t dy_f32, const void* x, int32_t x_f32, const float* mean,
                                    const float* rstd, const float* w, const float* b, int32_t act, int64_t rows,
                                    int32_t D, void* dx, int32_t dx_f32, float beta, void* dx2_bf16, float* dw_part,
                                    float* db_part, int32_t nblocks, void* stream) {
  OCTSAM_CHECK_ARG(dy && x && mean && rstd && w && b && dx && dw_part && db_part && rows > 0 && nblocks > 0,
                   "octsam_layernorm_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 64: return bwd_launch<1>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    case 256: return bwd_launch<4>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    case 768: return bwd_launch<12>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    default: octsam::set_error("octsam_layernorm_bwd: unsupported D=%d", D); return 1;
  }
}
