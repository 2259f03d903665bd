// Small element-wise / reduction / embedding kernels of the step.
//   octsam_axpby        out = alpha*a + beta*b[i % b_period]   (residual adds, dense-prompt broadcast
//                       image_embeddings + dense_prompt_embeddings, hf:modeling_sam.py:499)
//   octsam_colsum       per-block column partials of a [rows, cols] matrix (bias gradients)
//   octsam_prompt_tokens SamPromptEncoder._embed_boxes/_embed_points + token concat of SamMaskDecoder
//                       (hf:modeling_sam.py:613-656, :489-496)
//   octsam_image_pe     SamModel.get_image_wide_positional_embeddings (hf:modeling_sam.py:1128-1139),
//                       written [64*64, 256] channels-last
#include "common.h"
#include "../../include/octsam.h"

namespace {

__global__ void axpby_kernel(const void* __restrict__ a, int a_f32, const void* __restrict__ b, int b_f32,
                             long long b_period, float alpha, float beta, void* __restrict__ out, int out_f32,
                             float* __restrict__ out2, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float va = a ? (a_f32 ? ((const float*)a)[i] : (float)((const bf16*)a)[i]) : 0.0f;
  float vb = 0.0f;
  if (b) {
    long long j = b_period > 0 ? i % b_period : i;
    vb = b_f32 ? ((const float*)b)[j] : (float)((const bf16*)b)[j];
  }
  float v = alpha * va + beta * vb;
  if (out_f32) ((float*)out)[i] = v;
  else ((bf16*)out)[i] = (bf16)v;
  if (out2) out2[i] = v;
}

__global__ __launch_bounds__(256) void colsum_kernel(const void* __restrict__ x, int x_f32, long long rows, int cols,
                                                     float* __restrict__ part) {
  // block b sums rows b, b+nb, ... for columns c = tid, tid+256, ...
  for (int c = threadIdx.x; c < cols; c += 256) {
    float s = 0.0f;
    for (long long r = blockIdx.x; r < rows; r += gridDim.x)
      s += x_f32 ? ((const float*)x)[r * cols + c] : (float)((const bf16*)x)[r * cols + c];
    part[(long long)blockIdx.x * cols + c] = s;
  }
}

// Vectorised column sums: thread = (row lane, 8-column group); 16/32-byte loads; LDS combine.
template <bool F32>
__global__ __launch_bounds__(256) void colsum8_kernel(const void* __restrict__ x, long long rows, int cols,
                                                      float* __restrict__ part) {
  const int G = cols >> 3;
  const int lanes = 256 / G;
  const int g = threadIdx.x % G, lane = threadIdx.x / G;
  __shared__ float red[2048];
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
  if (lane < lanes) {
    for (long long r = (long long)blockIdx.x * lanes + lane; r < rows; r += (long long)gridDim.x * lanes) {
      if (F32) {
        const float4* p = (const float4*)((const float*)x + r * cols + g * 8);
        float4 a = p[0], b = p[1];
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      } else {
        bf16x8 v = *(const bf16x8*)((const bf16*)x + r * cols + g * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      }
    }
  }
  for (int l = 0; l < lanes; ++l) {
    if (lane == l) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[g * 8 + e] = (l == 0 ? 0.0f : red[g * 8 + e]) + acc[e];
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < cols; c += 256) part[(long long)blockIdx.x * cols + c] = red[c];
}

// dx = dy * (y > 0)  (ReLU backward from the saved ReLU output)
__global__ void relu_bwd_kernel(const float* __restrict__ dy, const bf16* __restrict__ y, long long ldy, int cols,
                                bf16* __restrict__ dx, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long r = i / cols, c = i % cols;
  float g = (float)y[r * ldy + c] > 0.0f ? dy[i] : 0.0f;
  dx[i] = (bf16)g;
}

// out[g][i] = sum_{j<nper} in[(g*nper + j)*n + i]  (sum over the prompts of one image, fixed order)
__global__ void group_sum_kernel(const bf16* __restrict__ in, long long ld_in, int cols, int nper, long long rows_per,
                                 bf16* __restrict__ out, long long total) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  long long per = rows_per * cols;
  long long g = e / per, rem = e % per, r = rem / cols, c = rem % cols;
  float s = 0.0f;
  for (int j = 0; j < nper; ++j) s += (float)in[((g * nper + j) * rows_per + r) * ld_in + c];
  out[e] = (bf16)s;
}
// 8 columns per thread (16-B loads and stores), 32-bit index math: cols, ld_in % 8 == 0, 16-B aligned
__global__ __launch_bounds__(256) void group_sum8_kernel(const bf16* __restrict__ in, int ld_in, int c8, int nper,
                                                         int rows_per, bf16* __restrict__ out, int total8) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total8) return;
  const int row = e / c8, c = (e - row * c8) * 8;  // output row = g * rows_per + r
  const int g = row / rows_per, r = row - g * rows_per;
  const bf16* src = in + ((long long)g * nper * rows_per + r) * ld_in + c;
  const long long step = (long long)rows_per * ld_in;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // 8 loads in flight per thread (the sum stays in j order: same bits as one load at a time); the group count is
  // small (few waves per CU), so each thread needs its own memory-level parallelism
  int j = 0;
  for (; j + 8 <= nper; j += 8) {
    bf16x8 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *(const bf16x8*)(src + (j + u) * step);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += (float)v[u][k];
  }
  for (; j < nper; ++j) {
    const bf16x8 v = *(const bf16x8*)(src + j * step);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += (float)v[k];
  }
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = (bf16)s[k];
  *(bf16x8*)(out + (long long)row * c8 * 8 + c) = o;
}

__device__ __forceinline__ void pe256(float cx, float cy, const float* __restrict__ G, float* __restrict__ out, int t) {
  // coordinates in [0,1]: 2c-1, @ G [2,128], * 2pi, [sin, cos]
  float x = 2.0f * cx - 1.0f, y = 2.0f * cy - 1.0f;
  for (int j = t; j < 128; j += 64) {
    float v = x * G[j] + y * G[128 + j];
    v = 6.283185307179586f * v;
    out[j] = sinf(v);
    out[128 + j] = cosf(v);
  }
}

// One wave per prompt. tokens: [P, 5 + nsparse, 256] fp32.
__global__ void prompt_tokens_kernel(const float* __restrict__ boxes, const float* __restrict__ points,
                                     const int* __restrict__ labels, int P, int npts, const float* __restrict__ G,
                                     const float* __restrict__ point_embed, const float* __restrict__ not_a_point,
                                     const float* __restrict__ out_tokens, float input_size, float* __restrict__ tokens) {
  const int p = blockIdx.x, t = threadIdx.x;
  const int nsparse = (points ? (boxes ? npts : npts + 1) : 0) + (boxes ? 2 : 0);
  const int ntok = 5 + nsparse;
  float* tok = tokens + (long long)p * ntok * 256;
  for (int i = t; i < 5 * 256; i += 64) tok[i] = out_tokens[i];
  int slot = 5;
  if (points) {
    for (int k = 0; k < npts; ++k, ++slot) {
      float* o = tok + slot * 256;
      int lab = labels ? labels[p * npts + k] : 1;
      float px = points[(p * npts + k) * 2 + 0] + 0.5f, py = points[(p * npts + k) * 2 + 1] + 0.5f;
      pe256(px / input_size, py / input_size, G, o, t);
      __syncthreads();
      for (int j = t; j < 256; j += 64) {
        float v = o[j];
        if (lab == -1) v = not_a_point[j];
        if (lab == -10) v = 0.0f;
        if (lab == 0) v += point_embed[0 * 256 + j];
        if (lab == 1) v += point_embed[1 * 256 + j];
        o[j] = v;
      }
    }
    if (!boxes) {  // pad point (0,0) with label -1 -> not_a_point_embed
      float* o = tok + slot * 256;
      for (int j = t; j < 256; j += 64) o[j] = not_a_point[j];
      ++slot;
    }
  }
  if (boxes) {
    const float* bx = boxes + p * 4;
    for (int c = 0; c < 2; ++c, ++slot) {
      float* o = tok + slot * 256;
      pe256((bx[2 * c] + 0.5f) / input_size, (bx[2 * c + 1] + 0.5f) / input_size, G, o, t);
      __syncthreads();
      for (int j = t; j < 256; j += 64) o[j] += point_embed[(2 + c) * 256 + j];
    }
  }
}

__global__ void image_pe_kernel(const float* __restrict__ G, int size, float* __restrict__ out) {
  const int pix = blockIdx.x, t = threadIdx.x;
  const int y = pix / size, x = pix % size;
  pe256(((float)x + 0.5f) / size, ((float)y + 0.5f) / size, G, out + (long long)pix * 256, t);
}

// SamMaskEmbedding.forward (hf:modeling_sam.py:569-592), the dense prompt of input_masks: conv 2x2/s2 (1 -> 4) ->
// LayerNorm2d(4) -> GELU -> conv 2x2/s2 (4 -> 16) -> LayerNorm2d(16) -> GELU -> conv 1x1 (16 -> 256). One thread per
// output pixel of the 64 x 64 grid: its 4 x 4 input patch gives the 2 x 2 first-stage pixels, the second stage and
// the 1x1 projection stay in registers; the weights are in LDS. masks fp32 [B, 256, 256] -> out fp32 [B, 4096, 256]
// (pixel-major: the decoder's image-embedding layout). Packed weights wp (fp32): conv1 w [4][4] (o, ky*2+kx), b [4],
// ln1 w [4], b [4], conv2 w [16][16] (o, c*4 + dy*2 + dx), b [16], ln2 w [16], b [16], conv3 w [256][16], b [256].
constexpr int ME_W = 16 + 4 + 4 + 4 + 256 + 16 + 16 + 16 + 4096 + 256;
__device__ __forceinline__ float me_gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__global__ __launch_bounds__(256) void mask_embed_kernel(const float* __restrict__ masks, const float* __restrict__ wp,
                                                         float eps, float* __restrict__ out) {
  __shared__ float w[ME_W];
  for (int i = threadIdx.x; i < ME_W; i += 256) w[i] = wp[i];
  __syncthreads();
  const float *w1 = w, *b1 = w + 16, *g1 = w + 20, *be1 = w + 24, *w2 = w + 28, *b2 = w + 284, *g2 = w + 300,
              *be2 = w + 316, *w3 = w + 332, *b3 = w + 332 + 4096;
  const int b = blockIdx.y, pix = blockIdx.x * 256 + threadIdx.x;  // 16 blocks x 256 = 4096 pixels
  const int Y = pix >> 6, X = pix & 63;
  const float* m = masks + (long long)b * 65536;
  float h1[4][4];  // [2x2 first-stage pixel][channel]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int y = 4 * Y + 2 * (q >> 1), x = 4 * X + 2 * (q & 1);
    const float in[4] = {m[y * 256 + x], m[y * 256 + x + 1], m[(y + 1) * 256 + x], m[(y + 1) * 256 + x + 1]};
    float v[4], mu = 0.0f;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      v[o] = b1[o] + w1[o * 4 + 0] * in[0] + w1[o * 4 + 1] * in[1] + w1[o * 4 + 2] * in[2] + w1[o * 4 + 3] * in[3];
      mu += v[o];
    }
    mu *= 0.25f;
    float var = 0.0f;
#pragma unroll
    for (int o = 0; o < 4; ++o) var += (v[o] - mu) * (v[o] - mu);
    const float rs = 1.0f / sqrtf(var * 0.25f + eps);
#pragma unroll
    for (int o = 0; o < 4; ++o) h1[q][o] = me_gelu((v[o] - mu) * rs * g1[o] + be1[o]);
  }
  float h2[16], mu = 0.0f;
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float a = b2[o];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) a += w2[o * 16 + c * 4 + q] * h1[q][c];
    h2[o] = a;
    mu += a;
  }
  mu *= 1.0f / 16.0f;
  float var = 0.0f;
#pragma unroll
  for (int o = 0; o < 16; ++o) var += (h2[o] - mu) * (h2[o] - mu);
  const float rs = 1.0f / sqrtf(var * (1.0f / 16.0f) + eps);
#pragma unroll
  for (int o = 0; o < 16; ++o) h2[o] = me_gelu((h2[o] - mu) * rs * g2[o] + be2[o]);
  float* o = out + ((long long)b * 4096 + pix) * 256;
  for (int j = 0; j < 256; j += 4) {
    float4 r;
    float* rp = (float*)&r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float a = b3[j + e];
#pragma unroll
      for (int c = 0; c < 16; ++c) a += w3[(j + e) * 16 + c] * h2[c];
      rp[e] = a;
    }
    *(float4*)(o + j) = r;
  }
}

}  // namespace

extern "C" int octsam_mask_embed(const float* masks, int32_t B, const float* packed_weights, float eps, float* out,
                                 void* stream) {
  OCTSAM_CHECK_ARG(masks && packed_weights && out && B > 0 && B <= 65535, "octsam_mask_embed: bad args");
  OCTSAM_CHECK_ARG(((uintptr_t)out & 15) == 0, "octsam_mask_embed: out must be 16-B aligned");
  hipLaunchKernelGGL(mask_embed_kernel, dim3(16, B), dim3(256), 0, (hipStream_t)stream, masks, packed_weights, eps, out);
  OCTSAM_LAUNCH_CHECK("octsam_mask_embed");
  return 0;
}

extern "C" int octsam_axpby(const void* a, int32_t a_f32, const void* b, int32_t b_f32, int64_t b_period, float alpha,
                            float beta, void* out, int32_t out_f32, float* out2_f32, int64_t n, void* stream) {
  OCTSAM_CHECK_ARG(out && n > 0, "octsam_axpby: bad args");
  unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(axpby_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, a_f32, b, b_f32, b_period, alpha,
                     beta, out, out_f32, out2_f32, n);
  OCTSAM_LAUNCH_CHECK("octsam_axpby");
  return 0;
}

extern "C" int octsam_colsum(const void* x, int32_t x_f32, int64_t rows, int32_t cols, float* part, int32_t nblocks,
                             void* stream) {
  OCTSAM_CHECK_ARG(x && part && rows > 0 && cols > 0 && nblocks > 0, "octsam_colsum: bad args");
  if (cols % 8 == 0 && cols <= 2048) {
    if (x_f32)
      hipLaunchKernelGGL(colsum8_kernel<true>, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, x, rows, cols, part);
    else
      hipLaunchKernelGGL(colsum8_kernel<false>, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, x, rows, cols, part);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, x, x_f32, rows, cols, part);
  }
  OCTSAM_LAUNCH_CHECK("octsam_colsum");
  return 0;
}

extern "C" int octsam_prompt_tokens(const float* boxes, const float* points, const int32_t* labels, int32_t P,
                                    int32_t points_per_prompt, const float* pos_gauss, const float* point_embed,
                                    const float* not_a_point, const float* out_tokens, float input_size,
                                    float* tokens, void* stream) {
  OCTSAM_CHECK_ARG(P > 0 && pos_gauss && point_embed && not_a_point && out_tokens && tokens,
                   "octsam_prompt_tokens: bad args");
  OCTSAM_CHECK_ARG(boxes || points, "octsam_prompt_tokens: need boxes or points");
  hipLaunchKernelGGL(prompt_tokens_kernel, dim3(P), dim3(64), 0, (hipStream_t)stream, boxes, points, labels, P,
                     points_per_prompt, pos_gauss, point_embed, not_a_point, out_tokens, input_size, tokens);
  OCTSAM_LAUNCH_CHECK("octsam_prompt_tokens");
  return 0;
}

extern "C" int octsam_image_pe(const float* pos_gauss, int32_t size, float* out, void* stream) {
  OCTSAM_CHECK_ARG(pos_gauss && out && size > 0, "octsam_image_pe: bad args");
  hipLaunchKernelGGL(image_pe_kernel, dim3(size * size), dim3(64), 0, (hipStream_t)stream, pos_gauss, size, out);
  OCTSAM_LAUNCH_CHECK("octsam_image_pe");
  return 0;
}

extern "C" int octsam_relu_bwd(const float* dy, const void* y, int64_t ldy, int32_t cols, void* dx, int64_t n,
                               void* stream) {
  OCTSAM_CHECK_ARG(dy && y && dx && cols > 0 && n > 0 && n % cols == 0, "octsam_relu_bwd: bad args");
  hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy,
                     (const bf16*)y, ldy, cols, (bf16*)dx, n);
  OCTSAM_LAUNCH_CHECK("octsam_relu_bwd");
  return 0;
}

extern "C" int octsam_group_sum(const void* in, int64_t ld_in, int32_t cols, int32_t groups, int32_t nper,
                                int64_t rows_per, void* out, void* stream) {
  OCTSAM_CHECK_ARG(in && out && cols > 0 && groups > 0 && nper > 0 && rows_per > 0, "octsam_group_sum: bad args");
  long long total = (long long)groups * rows_per * cols;
  if (cols % 8 == 0 && ld_in % 8 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
      total / 8 < (1LL << 31) && groups * rows_per < (1LL << 31)) {
    const int total8 = (int)(total / 8);
    hipLaunchKernelGGL(group_sum8_kernel, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)in, (int)ld_in, cols / 8, nper, (int)rows_per, (bf16*)out, total8);
    OCTSAM_LAUNCH_CHECK("octsam_group_sum");
    return 0;
  }
  hipLaunchKernelGGL(group_sum_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)in, ld_in, cols, nper, rows_per, (bf16*)out, total);
  OCTSAM_LAUNCH_CHECK("octsam_group_sum");
  return 0;
}

// Patch-embedding operand (SamPatchEmbeddings, hf:modeling_sam.py Conv2d(3, D, 16, stride 16)): pixel_values
// fp32 [B, 3, 1024, 1024] -> bf16 [B * 4096, 768], row = (b, patch row, patch col), k = (c, ky, kx) -- the
// conv as a plain NT GEMM on the 8-phase kernel. One thread per 8 consecutive pixels of an image row:
// 32-B coalesced reads, one 16-B store.
namespace {
template <typename E>
__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ px, E* __restrict__ out, long long n8) {
  typedef E E8 __attribute__((ext_vector_type(8)));
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const int x8 = (int)(i & 127), y = (int)((i >> 7) & 1023);
  const long long bc = i >> 17;  // b * 3 + c
  const int c = (int)(bc % 3);
  const long long b = bc / 3;
  const float4 a0 = *(const float4*)(px + i * 8), a1 = *(const float4*)(px + i * 8 + 4);
  E8 v;
  v[0] = (E)a0.x; v[1] = (E)a0.y; v[2] = (E)a0.z; v[3] = (E)a0.w;
  v[4] = (E)a1.x; v[5] = (E)a1.y; v[6] = (E)a1.z; v[7] = (E)a1.w;
  const long long row = b * 4096 + (y >> 4) * 64 + (x8 >> 1);
  *(E8*)(out + row * 768 + c * 256 + (y & 15) * 16 + (x8 & 1) * 8) = v;
}
}  // namespace

static int patchify(const float* px, int32_t B, void* out, bool f16, void* stream) {
  OCTSAM_CHECK_ARG(px && out && B > 0 && ((uintptr_t)px & 15) == 0 && ((uintptr_t)out & 15) == 0,
                   "octsam_patchify: bad args (16-B aligned operands required)");
  const long long n8 = (long long)B * 3 * 1024 * 128;
  const dim3 grid((unsigned)((n8 + 255) / 256));
  if (f16)
    hipLaunchKernelGGL(patchify_kernel<_Float16>, grid, dim3(256), 0, (hipStream_t)stream, px, (_Float16*)out, n8);
  else
    hipLaunchKernelGGL(patchify_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, px, (bf16*)out, n8);
  OCTSAM_LAUNCH_CHECK("octsam_patchify");
  return 0;
}

extern "C" int octsam_patchify_bf16(const float* px, int32_t B, void* out, void* stream) {
  return patchify(px, B, out, false, stream);
}
extern "C" int octsam_patchify_f16(const float* px, int32_t B, void* out, void* stream) {
  return patchify(px, B, out, true, stream);
}
