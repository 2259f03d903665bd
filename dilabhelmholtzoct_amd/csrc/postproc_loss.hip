// Mask post-processing, DiceCE loss and the dense parts of the topological loss, forward/backward.
//
//   postproc : F.interpolate(256->1024, bilinear, align_corners=False), crop to reshaped_input_sizes,
//              F.interpolate(-> original_sizes) (ref:octsam/models/training_utils.py:57-59), fused:
//              each output pixel evaluates the 4 stage-1 samples it needs straight from the low-res
//              mask with torch's upsample_bilinear2d index/lambda arithmetic (area_pixel_compute_*).
//              Backward is the transposed composite operator, applied as two gather passes with
//              host-built CSR weight tables (no atomics, deterministic).
//   dice/ce  : monai 1.3.0 DiceCELoss(sigmoid=True) (training_utils.py:32,62), restated:
//              dice = mean_{b,n} 1 - (2*sum(p t) + 1e-5)/(sum t + sum p + 1e-5), p = sigmoid(x)
//              ce   = nn.CrossEntropyLoss over the PROMPT dim with probability targets,
//                     mean_{b,h,w} sum_n t_n (lse_n(x) - x_n)
//   topo     : sigmoid + F.interpolate(->50x50, bilinear, align_corners=True) of the selected pred maps
//              and of the gt maps (ref:octsam/models/topological_loss.py:33-46), and the scatter of
//              the diagram-value gradients back through that downsample and the sigmoid.
#include "common.h"
#include "../../include/octsam.h"

namespace {

struct Lin {
  int i0, i1;
  float l0, l1;
};

// torch upsample_bilinear2d source index (align_corners=False), scale = (float)in / out
__device__ __forceinline__ Lin lin_acf(int dst, int in, float scale) {
  float r = scale * ((float)dst + 0.5f) - 0.5f;
  if (r < 0.0f) r = 0.0f;
  int i0 = (int)r;
  int off = (i0 < in - 1) ? 1 : 0;
  float l1 = r - (float)i0;
  return {i0, i0 + off, 1.0f - l1, l1};
}
// align_corners=True, scale = (float)(in-1)/(out-1)
__device__ __forceinline__ Lin lin_act(int dst, int in, float scale) {
  float r = scale * (float)dst;
  int i0 = (int)r;
  int off = (i0 < in - 1) ? 1 : 0;
  float l1 = r - (float)i0;
  return {i0, i0 + off, 1.0f - l1, l1};
}

struct PP {
  int S;          // low-res side (256)
  int mid;        // stage-1 side (1024)
  int ch, cw;     // crop (reshaped_input_sizes)
  int oh, ow;     // original_sizes
  float s1, s2h, s2w;
};

__device__ __forceinline__ float stage1(const float* __restrict__ x, const PP& pp, int r, int c) {
  Lin a = lin_acf(r, pp.S, pp.s1), b = lin_acf(c, pp.S, pp.s1);
  const float* r0 = x + a.i0 * pp.S;
  const float* r1 = x + a.i1 * pp.S;
  return a.l0 * (b.l0 * r0[b.i0] + b.l1 * r0[b.i1]) + a.l1 * (b.l0 * r1[b.i0] + b.l1 * r1[b.i1]);
}

// out[m][i][j] and Dice partials: part[m][blk][3] = (sum p*t, sum t, sum p)
__global__ __launch_bounds__(256) void postproc_fwd_kernel(const float* __restrict__ low, PP pp,
                                                           float* __restrict__ out, const uint8_t* __restrict__ gt,
                                                           float* __restrict__ part) {
  const int m = blockIdx.y;
  const float* x = low + (long long)m * pp.S * pp.S;
  const long long npix = (long long)pp.oh * pp.ow;
  float si = 0.0f, st = 0.0f, sp = 0.0f;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < npix; e += (long long)gridDim.x * 256) {
    int i = (int)(e / pp.ow), j = (int)(e % pp.ow);
    Lin h = lin_acf(i, pp.ch, pp.s2h), w = lin_acf(j, pp.cw, pp.s2w);
    float v00 = stage1(x, pp, h.i0, w.i0), v01 = stage1(x, pp, h.i0, w.i1);
    float v10 = stage1(x, pp, h.i1, w.i0), v11 = stage1(x, pp, h.i1, w.i1);
    float v = h.l0 * (w.l0 * v00 + w.l1 * v01) + h.l1 * (w.l0 * v10 + w.l1 * v11);
    out[(long long)m * npix + e] = v;
    if (gt) {
      float t = (float)gt[(long long)m * npix + e];
      float p = 1.0f / (1.0f + __expf(-v));
      si += p * t;
      st += t;
      sp += p;
    }
  }
  if (!gt) return;
  __shared__ float red[3][4];
  si = wave_sum(si); st = wave_sum(st); sp = wave_sum(sp);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][wave] = si; red[1][wave] = st; red[2][wave] = sp; }
  __syncthreads();
  if (threadIdx.x < 3) {
    float s = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    part[((long long)m * gridDim.x + blockIdx.x) * 3 + threadIdx.x] = s;
  }
}

// per-map dice sums -> dice loss per map, and the per-map gradient coefficients
// coef[m] = (c1, c2): d(mean dice)/dx = (c1 * t + c2) * p (1 - p)
__global__ void dice_reduce_kernel(const float* __restrict__ part, int M, int nblk, double smooth_nr, double smooth_dr,
                                   double inv_count, double* __restrict__ dice_map, float* __restrict__ coef) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  double I = 0, G = 0, Ps = 0;
  for (int b = 0; b < nblk; ++b) {
    I += part[((long long)m * nblk + b) * 3 + 0];
    G += part[((long long)m * nblk + b) * 3 + 1];
    Ps += part[((long long)m * nblk + b) * 3 + 2];
  }
  double num = 2.0 * I + smooth_nr, den = G + Ps + smooth_dr;
  dice_map[m] = 1.0 - num / den;
  coef[2 * m + 0] = (float)(-2.0 / den * inv_count);
  coef[2 * m + 1] = (float)(num / (den * den) * inv_count);
}

// per (b, pixel): CE over the N prompt channels + Dice gradient. dmask = w_dice*ddice + w_ce*dce.
// ce_part[blk] (double) = sum over the block's pixels of sum_n t_n (lse - x_n)
__global__ __launch_bounds__(256) void dicece_bwd_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                         const float* __restrict__ coef, int B, int N, long long HW,
                                                         float w_dice, float w_ce, float inv_bhw,
                                                         float* __restrict__ dx, double* __restrict__ ce_part) {
  const long long total = (long long)B * HW;
  double ce = 0.0;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int b = (int)(e / HW);
    const long long pix = e % HW;
    const float* xb = x + (long long)b * N * HW + pix;
    const uint8_t* tb = gt + (long long)b * N * HW + pix;
    float mx = -INFINITY;
    for (int n = 0; n < N; ++n) mx = fmaxf(mx, xb[n * HW]);
    float se = 0.0f, tsum = 0.0f, tx = 0.0f;
    for (int n = 0; n < N; ++n) {
      float xv = xb[n * HW];
      float t = (float)tb[n * HW];
      se += __expf(xv - mx);
      tsum += t;
      tx += t * xv;
    }
    const float lse = mx + __logf(se);
    ce += (double)(lse * tsum - tx);
    float* db = dx + (long long)b * N * HW + pix;
    for (int n = 0; n < N; ++n) {
      float xv = xb[n * HW];
      float t = (float)tb[n * HW];
      float sm = __expf(xv - lse);
      float p = 1.0f / (1.0f + __expf(-xv));
      const float* cf = coef + 2 * (b * N + n);
      float gd = (cf[0] * t + cf[1]) * p * (1.0f - p);
      float gc = (sm * tsum - t) * inv_bhw;
      db[n * HW] = w_dice * gd + w_ce * gc;
    }
  }
  __shared__ double red[4];
  ce = wave_sum_d(ce);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ce;
  __syncthreads();
  if (threadIdx.x == 0) ce_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// loss[0] = mean dice, loss[1] = ce, loss[2] = w_dice*dice + w_ce*ce
__global__ void loss_finalize_kernel(const double* __restrict__ dice_map, int M, const double* __restrict__ ce_part,
                                     int nblk, double inv_bhw, double w_dice, double w_ce, double* __restrict__ loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double d = 0.0, c = 0.0;
  for (int m = 0; m < M; ++m) d += dice_map[m];
  for (int b = 0; b < nblk; ++b) c += ce_part[b];
  d /= M;
  c *= inv_bhw;
  loss[0] = d;
  loss[1] = c;
  loss[2] = w_dice * d + w_ce * c;
}

// Backward of the composite post-processing operator: dlow[m] = Wy^T dout[m] Wx.
// Row pass: tmp[m][i][b] = sum_{(j,w) in colcsr[b]} w * dout[m][i][j]
__global__ __launch_bounds__(256) void pp_bwd_rows_kernel(const float* __restrict__ dout, int oh, int ow, int S,
                                                          const int* __restrict__ cptr, const int* __restrict__ cidx,
                                                          const float* __restrict__ cw, float* __restrict__ tmp) {
  const int m = blockIdx.y;
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)oh * S) return;
  const int i = (int)(e / S), b = (int)(e % S);
  const float* row = dout + ((long long)m * oh + i) * ow;
  float acc = 0.0f;
  for (int k = cptr[b]; k < cptr[b + 1]; ++k) acc += cw[k] * row[cidx[k]];
  tmp[((long long)m * oh + i) * S + b] = acc;
}
// Column pass: dlow[m][a][b] = sum_{(i,w) in rowcsr[a]} w * tmp[m][i][b]
__global__ __launch_bounds__(256) void pp_bwd_cols_kernel(const float* __restrict__ tmp, int oh, int S,
                                                          const int* __restrict__ rptr, const int* __restrict__ ridx,
                                                          const float* __restrict__ rw, float* __restrict__ dlow) {
  const int m = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S * S) return;
  const int a = e / S, b = e % S;
  float acc = 0.0f;
  for (int k = rptr[a]; k < rptr[a + 1]; ++k) acc += rw[k] * tmp[((long long)m * oh + ridx[k]) * S + b];
  dlow[(long long)m * S * S + e] = acc;
}

// topo forward: pred50[k] = interp_ac(sigmoid(masks[map_idx[k]])), gt50[k] = interp_ac(gt[map_idx[k]])
__global__ __launch_bounds__(256) void topo_down_kernel(const float* __restrict__ masks, const uint8_t* __restrict__ gt,
                                                        const int* __restrict__ map_idx, int ih, int iw, int oh, int ow,
                                                        float sh, float sw, int sig, float* __restrict__ pred,
                                                        float* __restrict__ gto) {
  const int k = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= oh * ow) return;
  const int i = e / ow, j = e % ow;
  const long long mo = (long long)map_idx[k] * ih * iw;
  Lin a = lin_act(i, ih, sh), b = lin_act(j, iw, sw);
  auto sg = [&](int r, int c) {
    float x = masks[mo + (long long)r * iw + c];
    return sig ? 1.0f / (1.0f + __expf(-x)) : x;
  };
  auto gv = [&](int r, int c) { return (float)gt[mo + (long long)r * iw + c]; };
  pred[(long long)k * oh * ow + e] =
      a.l0 * (b.l0 * sg(a.i0, b.i0) + b.l1 * sg(a.i0, b.i1)) + a.l1 * (b.l0 * sg(a.i1, b.i0) + b.l1 * sg(a.i1, b.i1));
  if (gto)
    gto[(long long)k * oh * ow + e] =
        a.l0 * (b.l0 * gv(a.i0, b.i0) + b.l1 * gv(a.i0, b.i1)) + a.l1 * (b.l0 * gv(a.i1, b.i0) + b.l1 * gv(a.i1, b.i1));
}

// topo backward: dmask[map_idx[k]] += d(interp_ac o sigmoid)^T dpred[k]
__global__ __launch_bounds__(256) void topo_bwd_kernel(const float* __restrict__ masks, const int* __restrict__ map_idx,
                                                       int ih, int iw, int oh, int ow, float sh, float sw, int sig,
                                                       const float* __restrict__ dpred, float scale,
                                                       float* __restrict__ dmask) {
  const int k = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= oh * ow) return;
  const float g = dpred[(long long)k * oh * ow + e] * scale;
  if (g == 0.0f) return;
  const int i = e / ow, j = e % ow;
  const long long mo = (long long)map_idx[k] * ih * iw;
  Lin a = lin_act(i, ih, sh), b = lin_act(j, iw, sw);
  auto add = [&](int r, int c, float w) {
    long long idx = mo + (long long)r * iw + c;
    float d = 1.0f;
    if (sig) {
      float s = 1.0f / (1.0f + __expf(-masks[idx]));
      d = s * (1.0f - s);
    }
    atomicAdd(dmask + idx, g * w * d);
  };
  add(a.i0, b.i0, a.l0 * b.l0);
  add(a.i0, b.i1, a.l0 * b.l1);
  add(a.i1, b.i0, a.l1 * b.l0);
  add(a.i1, b.i1, a.l1 * b.l1);
}

}  // namespace

extern "C" int octsam_postproc_fwd(const float* lowres, int32_t M, int32_t S, int32_t mid, int32_t crop_h,
                                   int32_t crop_w, int32_t out_h, int32_t out_w, float* out, const uint8_t* gt,
                                   float* dice_part, int32_t nblk, void* stream) {
  OCTSAM_CHECK_ARG(lowres && out && M > 0 && S > 0 && mid > 0 && crop_h > 0 && crop_w > 0 && out_h > 0 && out_w > 0 &&
                       crop_h <= mid && crop_w <= mid && nblk > 0,
                   "octsam_postproc_fwd: bad args");
  OCTSAM_CHECK_ARG(!gt || dice_part, "octsam_postproc_fwd: gt needs dice_part");
  PP pp{S, mid, crop_h, crop_w, out_h, out_w, (float)S / (float)mid, (float)crop_h / (float)out_h,
        (float)crop_w / (float)out_w};
  hipLaunchKernelGGL(postproc_fwd_kernel, dim3(nblk, M), dim3(256), 0, (hipStream_t)stream, lowres, pp, out, gt,
                     dice_part);
  OCTSAM_LAUNCH_CHECK("octsam_postproc_fwd");
  return 0;
}

extern "C" int octsam_dice_reduce(const float* dice_part, int32_t M, int32_t nblk, double* dice_map, float* coef,
                                  void* stream) {
  OCTSAM_CHECK_ARG(dice_part && dice_map && coef && M > 0 && nblk > 0, "octsam_dice_reduce: bad args");
  hipLaunchKernelGGL(dice_reduce_kernel, dim3((M + 127) / 128), dim3(128), 0, (hipStream_t)stream, dice_part, M, nblk,
                     1e-5, 1e-5, 1.0 / M, dice_map, coef);
  OCTSAM_LAUNCH_CHECK("octsam_dice_reduce");
  return 0;
}

extern "C" int octsam_dicece_bwd(const float* masks, const uint8_t* gt, const float* coef, int32_t B, int32_t N,
                                 int64_t HW, float w_dice, float w_ce, float* dmask, double* ce_part, int32_t nblk,
                                 void* stream) {
  OCTSAM_CHECK_ARG(masks && gt && coef && dmask && ce_part && B > 0 && N > 0 && HW > 0 && nblk > 0,
                   "octsam_dicece_bwd: bad args");
  hipLaunchKernelGGL(dicece_bwd_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, masks, gt, coef, B, N, HW, w_dice,
                     w_ce, (float)(1.0 / ((double)B * HW)), dmask, ce_part);
  OCTSAM_LAUNCH_CHECK("octsam_dicece_bwd");
  return 0;
}

extern "C" int octsam_loss_finalize(const double* dice_map, int32_t M, const double* ce_part, int32_t nblk, int32_t B,
                                    int64_t HW, double w_dice, double w_ce, double* loss, void* stream) {
  OCTSAM_CHECK_ARG(dice_map && ce_part && loss && M > 0 && nblk > 0, "octsam_loss_finalize: bad args");
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dice_map, M, ce_part, nblk,
                     1.0 / ((double)B * HW), w_dice, w_ce, loss);
  OCTSAM_LAUNCH_CHECK("octsam_loss_finalize");
  return 0;
}

extern "C" int octsam_postproc_bwd(const float* dout, int32_t M, int32_t S, int32_t out_h, int32_t out_w,
                                   const int32_t* col_ptr, const int32_t* col_idx, const float* col_w,
                                   const int32_t* row_ptr, const int32_t* row_idx, const float* row_w, float* tmp,
                                   float* dlowres, void* stream) {
  OCTSAM_CHECK_ARG(dout && col_ptr && col_idx && col_w && row_ptr && row_idx && row_w && tmp && dlowres && M > 0,
                   "octsam_postproc_bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pp_bwd_rows_kernel, dim3((unsigned)(((long long)out_h * S + 255) / 256), M), dim3(256), 0, s, dout,
                     out_h, out_w, S, col_ptr, col_idx, col_w, tmp);
  OCTSAM_LAUNCH_CHECK("octsam_postproc_bwd");
  hipLaunchKernelGGL(pp_bwd_cols_kernel, dim3((S * S + 255) / 256, M), dim3(256), 0, s, tmp, out_h, S, row_ptr, row_idx,
                     row_w, dlowres);
  OCTSAM_LAUNCH_CHECK("octsam_postproc_bwd");
  return 0;
}

extern "C" int octsam_topo_down(const float* masks, const uint8_t* gt, const int32_t* map_idx, int32_t K, int32_t in_h,
                                int32_t in_w, int32_t out_h, int32_t out_w, int32_t apply_sigmoid, float* pred,
                                float* gt_out, void* stream) {
  OCTSAM_CHECK_ARG(masks && map_idx && pred && K >= 0 && in_h > 1 && in_w > 1 && out_h > 1 && out_w > 1,
                   "octsam_topo_down: bad args");
  OCTSAM_CHECK_ARG(!gt_out || gt, "octsam_topo_down: gt_out needs gt");
  if (K == 0) return 0;
  float sh = (float)(in_h - 1) / (float)(out_h - 1), sw = (float)(in_w - 1) / (float)(out_w - 1);
  hipLaunchKernelGGL(topo_down_kernel, dim3((out_h * out_w + 255) / 256, K), dim3(256), 0, (hipStream_t)stream, masks,
                     gt, map_idx, in_h, in_w, out_h, out_w, sh, sw, apply_sigmoid, pred, gt_out);
  OCTSAM_LAUNCH_CHECK("octsam_topo_down");
  return 0;
}

extern "C" int octsam_topo_bwd(const float* masks, const int32_t* map_idx, int32_t K, int32_t in_h, int32_t in_w,
                               int32_t out_h, int32_t out_w, int32_t apply_sigmoid, const float* dpred, float scale,
                               float* dmask, void* stream) {
  OCTSAM_CHECK_ARG(masks && map_idx && dpred && dmask && K >= 0, "octsam_topo_bwd: bad args");
  if (K == 0) return 0;
  float sh = (float)(in_h - 1) / (float)(out_h - 1), sw = (float)(in_w - 1) / (float)(out_w - 1);
  hipLaunchKernelGGL(topo_bwd_kernel, dim3((out_h * out_w + 255) / 256, K), dim3(256), 0, (hipStream_t)stream, masks,
                     map_idx, in_h, in_w, out_h, out_w, sh, sw, apply_sigmoid, dpred, scale, dmask);
  OCTSAM_LAUNCH_CHECK("octsam_topo_bwd");
  return 0;
}
