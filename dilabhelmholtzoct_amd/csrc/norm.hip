// LayerNorm over the last dimension, forward and backward.
//
// Covers nn.LayerNorm of SamVisionLayer (hf:modeling_sam.py:954-972, eps 1e-6), the channels-first
// SamLayerNorm of the neck and of the mask-decoder upscaling (:975-992, :519-521; applied per pixel on
// NHWC data), and the decoder LayerNorms (:306-348; layer_norm_final_attn eps 1e-5, :363).
// Forward options: input fp32/bf16; output bf16 and/or fp32; fused GELU (upscale LN -> GELU);
// row gather (window_partition with zero padding: output row r reads input row src_rows[r], or
// writes zeros when src_rows[r] < 0); mean/rstd saved for backward.
// Backward: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w (optionally through the
// fused GELU); per-block dw/db partials reduced deterministically by octsam_splitk_reduce.
//
// Layout: a row is owned by a group of G lanes (G = 8 for D = 64, 32 for D = 256, 64 otherwise), so a
// wave holds 64/G rows; lane j of a group owns NCH chunks of CW consecutive columns at CW*j + G*CW*c
// (16-B bf16 / 32-B fp32 vector accesses, whole cache lines per wave instruction). Grid-stride over
// row groups; the statistics reduce with xor-shuffles inside the group.
#include "common.h"
#include "../../include/octsam.h"

namespace {

template <int D>
struct LnGeo;
template <> struct LnGeo<64> { static constexpr int G = 8, CW = 8, NCH = 1; };
template <> struct LnGeo<256> { static constexpr int G = 32, CW = 8, NCH = 1; };
template <> struct LnGeo<768> { static constexpr int G = 64, CW = 4, NCH = 3; };
template <> struct LnGeo<1024> { static constexpr int G = 64, CW = 8, NCH = 2; };
template <> struct LnGeo<1280> { static constexpr int G = 64, CW = 4, NCH = 5; };

template <int CW>
__device__ __forceinline__ void ldv(const void* base, long long idx, bool f32, float* v) {
  if (f32) {
    const float* p = (const float*)base + idx;
    if constexpr (CW == 8) {
      const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const float4 a = *(const float4*)p;
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    }
  } else {
    const bf16* p = (const bf16*)base + idx;
    if constexpr (CW == 8) {
      const u32x4 a = *(const u32x4*)p;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = __builtin_bit_cast(float, a[e] << 16);
        v[2 * e + 1] = __builtin_bit_cast(float, a[e] & 0xffff0000u);
      }
    } else {
      const uint2 a = *(const uint2*)p;
      v[0] = __builtin_bit_cast(float, a.x << 16);
      v[1] = __builtin_bit_cast(float, a.x & 0xffff0000u);
      v[2] = __builtin_bit_cast(float, a.y << 16);
      v[3] = __builtin_bit_cast(float, a.y & 0xffff0000u);
    }
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16x2 w;
  w[0] = (bf16)a;
  w[1] = (bf16)b;
  return __builtin_bit_cast(uint32_t, w);
}

__device__ __forceinline__ uint32_t pack2h(float a, float b) {  // IEEE half pair (the fp16 encoder)
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  h2 w;
  w[0] = (_Float16)a;
  w[1] = (_Float16)b;
  return __builtin_bit_cast(uint32_t, w);
}

// ty: 1 = fp32, 2 = fp16, otherwise bf16
template <int CW>
__device__ __forceinline__ void stv(void* base, long long idx, int ty, const float* v) {
  if (ty == 1) {
    float* p = (float*)base + idx;
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    if constexpr (CW == 8) *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    bf16* p = (bf16*)base + idx;
    auto pk = [&](float a, float b) { return ty == 2 ? pack2h(a, b) : pack2(a, b); };
    if constexpr (CW == 8) {
      u32x4 a;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = pk(v[2 * e], v[2 * e + 1]);
      *(u32x4*)p = a;
    } else {
      *(uint2*)p = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
    }
  }
}

// Cross-lane sums without LDS round trips: DPP within a row of 16 lanes, v_permlane16/32_swap across rows.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// x + (x of lane ^ 16) / (x of lane ^ 32): the swap of x with itself leaves each lane {lower, upper} of its pair
__device__ __forceinline__ float add_xor16(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (uint32_t)r[0]) + __builtin_bit_cast(float, (uint32_t)r[1]);
}
__device__ __forceinline__ float add_xor32(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (uint32_t)r[0]) + __builtin_bit_cast(float, (uint32_t)r[1]);
}

// sum over each aligned group of G lanes, in every lane of the group (fixed order: deterministic)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (G >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  if constexpr (G >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  if constexpr (G >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: the other quad of the 8 (all hold quad sums)
  if constexpr (G >= 16) v += dpp_mov<0x140>(v); // row_mirror: the other 8 of the row (all hold 8-lane sums)
  if constexpr (G >= 32) v = add_xor16(v);
  if constexpr (G >= 64) v = add_xor32(v);
  return v;
}

// v + (v of lane ^ O) for a single lane distance O >= 8 (lane positions matter: per-column partials)
template <int O>
__device__ __forceinline__ float add_lane_xor(float v) {
  static_assert(O == 8 || O == 16 || O == 32, "lane distance 8, 16 or 32");
  if constexpr (O == 8) return v + dpp_mov<0x128>(v);  // row_ror:8 = lane ^ 8 within the row
  else if constexpr (O == 16) return add_xor16(v);
  else return add_xor32(v);
}

template <int D>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, int x_f32, const int* __restrict__ src_rows,
                                                     long long rows, const float* __restrict__ w,
                                                     const float* __restrict__ b, float eps, void* __restrict__ y,
                                                     int y_f32, float* __restrict__ y2, int act,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  using Geo = LnGeo<D>;
  constexpr int G = Geo::G, CW = Geo::CW, NCH = Geo::NCH, RPW = 64 / G, PL = CW * NCH;
  const int lane = threadIdx.x & 63, j = lane % G;
  float wv[PL], bv[PL];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    ldv<CW>(w, CW * j + G * CW * c, true, wv + c * CW);
    ldv<CW>(b, CW * j + G * CW * c, true, bv + c * CW);
  }
  const long long nwaves = (long long)gridDim.x * 4;
  for (long long rg = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); rg * RPW < rows; rg += nwaves) {
    const long long row = rg * RPW + lane / G;
    const bool live = row < rows;
    const long long src = !live ? -1 : (src_rows ? (long long)src_rows[row] : row);
    float v[PL];
    if (src >= 0) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) ldv<CW>(x, src * D + CW * j + G * CW * c, x_f32, v + c * CW);
    } else {
#pragma unroll
      for (int e = 0; e < PL; ++e) v[e] = 0.0f;
    }
    float s = 0.0f;
#pragma unroll
    for (int e = 0; e < PL; ++e) s += v[e];
    const float mean = group_sum<G>(s) * (1.0f / D);
    float q = 0.0f;
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      const float d = v[e] - mean;
      q += d * d;
    }
    const float rstd = rsqrtf(group_sum<G>(q) * (1.0f / D) + eps);
    if (!live) continue;
    float out[PL];
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      float o = (v[e] - mean) * rstd * wv[e] + bv[e];
      if (act == OCTSAM_ACT_GELU) o = gelu_fast(o);
      else if (act == OCTSAM_ACT_RELU) o = fmaxf(o, 0.0f);
      // window padding: HF pads AFTER layer_norm1, so padded tokens are exact zeros
      out[e] = src >= 0 ? o : 0.0f;
    }
    if (mean_out && j == 0) {
      mean_out[row] = src >= 0 ? mean : 0.0f;
      rstd_out[row] = src >= 0 ? rstd : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      stv<CW>(y, row * D + CW * j + G * CW * c, y_f32, out + c * CW);
      if (y2) stv<CW>(y2, row * D + CW * j + G * CW * c, 1, out + c * CW);  // fp32 residual-stream copy
    }
  }
}

// Backward. Grid-stride over row groups; each block writes one dw/db partial row (fixed order).
template <int D>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ dy, int dy_f32, const void* __restrict__ x,
                                                     int x_f32, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ w,
                                                     const float* __restrict__ b, int act, long long rows,
                                                     void* __restrict__ dx, int dx_f32, float beta,
                                                     bf16* __restrict__ dx2, float* __restrict__ dw_part,
                                                     float* __restrict__ db_part) {
  using Geo = LnGeo<D>;
  constexpr int G = Geo::G, CW = Geo::CW, NCH = Geo::NCH, RPW = 64 / G, PL = CW * NCH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane % G;
  float wv[PL], bv[PL], dwa[PL], dba[PL];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    ldv<CW>(w, CW * j + G * CW * c, true, wv + c * CW);
    ldv<CW>(b, CW * j + G * CW * c, true, bv + c * CW);
  }
#pragma unroll
  for (int e = 0; e < PL; ++e) { dwa[e] = 0.0f; dba[e] = 0.0f; }
  const long long nwaves = (long long)gridDim.x * 4;
  for (long long rg = (long long)blockIdx.x * 4 + wave; rg * RPW < rows; rg += nwaves) {
    const long long row = rg * RPW + lane / G;
    const bool live = row < rows;
    const long long rr = live ? row : rows - 1;  // dead lanes compute on a valid row, contribute nothing
    const float mu = mean[rr], rs = rstd[rr];
    float xh[PL], g[PL];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      ldv<CW>(x, rr * D + CW * j + G * CW * c, x_f32, xh + c * CW);
      ldv<CW>(dy, rr * D + CW * j + G * CW * c, dy_f32, g + c * CW);
    }
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      xh[e] = (xh[e] - mu) * rs;
      float gy = live ? g[e] : 0.0f;
      if (act == OCTSAM_ACT_GELU) gy *= gelu_fast_grad(xh[e] * wv[e] + bv[e]);
      else if (act == OCTSAM_ACT_RELU) gy = xh[e] * wv[e] + bv[e] > 0.0f ? gy : 0.0f;
      dwa[e] += gy * xh[e];
      dba[e] += gy;
      g[e] = gy * wv[e];
      s1 += g[e];
      s2 += g[e] * xh[e];
    }
    s1 = group_sum<G>(s1) * (1.0f / D);
    s2 = group_sum<G>(s2) * (1.0f / D);
    if (!live) continue;
    float d[PL];
#pragma unroll
    for (int e = 0; e < PL; ++e) d[e] = rs * (g[e] - s1 - xh[e] * s2);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const long long idx = row * D + CW * j + G * CW * c;
      if (beta != 0.0f) {
        float old[CW];
        ldv<CW>(dx, idx, dx_f32, old);
#pragma unroll
        for (int e = 0; e < CW; ++e) d[c * CW + e] += beta * old[e];
      }
      stv<CW>(dx, idx, dx_f32, d + c * CW);
      if (dx2) stv<CW>(dx2, idx, false, d + c * CW);
    }
  }
  // rows of one wave that share columns: fold the RPW groups, then the 4 waves through LDS
#pragma unroll
  for (int e = 0; e < PL; ++e) {
    if constexpr (G <= 8) {
      dwa[e] = add_lane_xor<8>(dwa[e]);
      dba[e] = add_lane_xor<8>(dba[e]);
    }
    if constexpr (G <= 16) {
      dwa[e] = add_lane_xor<16>(dwa[e]);
      dba[e] = add_lane_xor<16>(dba[e]);
    }
    if constexpr (G <= 32) {
      dwa[e] = add_lane_xor<32>(dwa[e]);
      dba[e] = add_lane_xor<32>(dba[e]);
    }
  }
  __shared__ float red[2][4][D];
  if (lane < G) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < CW; ++e) {
        red[0][wave][CW * j + G * CW * c + e] = dwa[c * CW + e];
        red[1][wave][CW * j + G * CW * c + e] = dba[c * CW + e];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    dw_part[(long long)blockIdx.x * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    db_part[(long long)blockIdx.x * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

template <int D>
int fwd_launch(const void* x, int x_f32, const int* src_rows, long long rows, const float* w, const float* b, float eps,
               void* y, int y_f32, float* y2, int act, float* mean, float* rstd, hipStream_t s) {
  constexpr int RPB = 4 * (64 / LnGeo<D>::G);  // rows per block per grid-stride step
  const long long need = (rows + RPB - 1) / RPB;
  const unsigned blocks = (unsigned)(need < 8192 ? need : 8192);
  hipLaunchKernelGGL(ln_fwd_kernel<D>, dim3(blocks), dim3(256), 0, s, x, x_f32, src_rows, rows, w, b, eps, y, y_f32,
                     y2, act, mean, rstd);
  OCTSAM_LAUNCH_CHECK("octsam_layernorm_fwd");
  return 0;
}

template <int D>
int bwd_launch(const void* dy, int dy_f32, const void* x, int x_f32, const float* mean, const float* rstd,
               const float* w, const float* b, int act, long long rows, void* dx, int dx_f32, float beta,
               bf16* dx2, float* dw_part, float* db_part, int nblocks, hipStream_t s) {
  hipLaunchKernelGGL(ln_bwd_kernel<D>, dim3(nblocks), dim3(256), 0, s, dy, dy_f32, x, x_f32, mean, rstd, w, b, act,
                     rows, dx, dx_f32, beta, dx2, dw_part, db_part);
  OCTSAM_LAUNCH_CHECK("octsam_layernorm_bwd");
  return 0;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int octsam_layernorm_fwd(const void* x, int32_t x_f32, const int32_t* src_rows, int64_t rows, int32_t D,
                                    const float* w, const float* b, float eps, void* y, int32_t y_f32, float* y2_f32,
                                    int32_t act, float* mean, float* rstd, void* stream) {
  OCTSAM_CHECK_ARG(x && w && b && y && rows > 0, "octsam_layernorm_fwd: bad args");
  OCTSAM_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "octsam_layernorm_fwd: mean/rstd both or neither");
  OCTSAM_CHECK_ARG(aligned16(x) && aligned16(y) && aligned16(w) && aligned16(b) && (!y2_f32 || aligned16(y2_f32)),
                   "octsam_layernorm_fwd: x, y, y2, w, b must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 64: return fwd_launch<64>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 256: return fwd_launch<256>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 768: return fwd_launch<768>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 1024: return fwd_launch<1024>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    case 1280: return fwd_launch<1280>(x, x_f32, src_rows, rows, w, b, eps, y, y_f32, y2_f32, act, mean, rstd, s);
    default: octsam::set_error("octsam_layernorm_fwd: unsupported D=%d", D); return 1;
  }
}

extern "C" int octsam_layernorm_bwd(const void* dy, int32_t dy_f32, const void* x, int32_t x_f32, const float* mean,
                                    const float* rstd, const float* w, const float* b, int32_t act, int64_t rows,
                                    int32_t D, void* dx, int32_t dx_f32, float beta, void* dx2_bf16, float* dw_part,
                                    float* db_part, int32_t nblocks, void* stream) {
  OCTSAM_CHECK_ARG(dy && x && mean && rstd && w && b && dx && dw_part && db_part && rows > 0 && nblocks > 0,
                   "octsam_layernorm_bwd: bad args");
  OCTSAM_CHECK_ARG(aligned16(dy) && aligned16(x) && aligned16(dx) && aligned16(w) && aligned16(b) &&
                       (!dx2_bf16 || aligned16(dx2_bf16)),
                   "octsam_layernorm_bwd: dy, x, dx, dx2, w, b must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  switch (D) {
    case 64: return bwd_launch<64>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    case 256: return bwd_launch<256>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    case 768: return bwd_launch<768>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    case 1024: return bwd_launch<1024>(dy, dy_f32, x, x_f32, mean, rstd, w, b, act, rows, dx, dx_f32, beta, (bf16*)dx2_bf16, dw_part, db_part, nblocks, s);
    default: octsam::set_error("octsam_layernorm_bwd: unsupported D=%d", D); return 1;
  }
}
