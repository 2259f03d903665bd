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
#include <cstdlib>
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

// out[m][i][j] and Dice partials: part[m][blk][3] = (sum p*t, sum t, sum p), blk = group of 4 output rows.
// One workgroup per (map, 4 output rows): the contiguous range of low-res rows those rows need (<= 8, host-
// checked) is staged in LDS with coalesced float4 loads, every one of the 16 taps
// of an output pixel is an LDS read (the global gather version was address-bound), and each column's
// stage-2 / stage-1 coordinates are computed once for the 4 rows.
constexpr int PP_ROWS = 4, PP_LRMAX = 16;
__global__ __launch_bounds__(256) void postproc_fwd_kernel(const float* __restrict__ low, PP pp,
                                                           float* __restrict__ out, const uint8_t* __restrict__ gt,
                                                           float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float rows[PP_LRMAX][256];
  __shared__ float red[3][4];
  const int m = blockIdx.y, i0 = blockIdx.x * PP_ROWS, tid = threadIdx.x;
  const int nr = min(PP_ROWS, pp.oh - i0);
  const float* x = low + (long long)m * pp.S * pp.S;
  // low-res row range of the group: rows are monotone in i, so the first row's lowest and the last row's
  // highest source bound it; only those rows are staged (staging all PP_LRMAX rows read ~5x the low-res bytes:
  // 382 MB fetched per launch against 87 MB compulsory, profiles/r03/traffic_kernels_r03r.txt)
  const int lo = lin_acf(lin_acf(i0, pp.ch, pp.s2h).i0, pp.S, pp.s1).i0;
  const int hi = lin_acf(lin_acf(i0 + nr - 1, pp.ch, pp.s2h).i1, pp.S, pp.s1).i1;
  const int nlr = min(hi - lo + 1, PP_LRMAX);
  for (int e = tid; e < nlr * 64; e += 256) {
    const int r = e >> 6, c4 = (e & 63) * 4;
    if (c4 < pp.S) *(float4*)&rows[r][c4] = *(const float4*)(x + (long long)(lo + r) * pp.S + c4);
  }
  __syncthreads();
  float si = 0.0f, st = 0.0f, sp = 0.0f;
  Lin hs[PP_ROWS], a0s[PP_ROWS], a1s[PP_ROWS];  // row coordinates, once per row
#pragma unroll
  for (int r = 0; r < PP_ROWS; ++r) {
    hs[r] = lin_acf(min(i0 + r, pp.oh - 1), pp.ch, pp.s2h);
    a0s[r] = lin_acf(hs[r].i0, pp.S, pp.s1);
    a1s[r] = lin_acf(hs[r].i1, pp.S, pp.s1);
  }
  for (int j = tid; j < pp.ow; j += 256) {
    const Lin w = lin_acf(j, pp.cw, pp.s2w);
    const Lin b0 = lin_acf(w.i0, pp.S, pp.s1), b1 = lin_acf(w.i1, pp.S, pp.s1);
#pragma unroll
    for (int r = 0; r < PP_ROWS; ++r) {
      if (r >= nr) break;
      const int i = i0 + r;
      const Lin h = hs[r], a0 = a0s[r], a1 = a1s[r];
      auto st1 = [&](const Lin& a, const Lin& bb) {
        const float* ra = rows[a.i0 - lo];
        const float* rb = rows[a.i1 - lo];
        return a.l0 * (bb.l0 * ra[bb.i0] + bb.l1 * ra[bb.i1]) + a.l1 * (bb.l0 * rb[bb.i0] + bb.l1 * rb[bb.i1]);
      };
      const float v00 = st1(a0, b0), v01 = st1(a0, b1), v10 = st1(a1, b0), v11 = st1(a1, b1);
      const float v = h.l0 * (w.l0 * v00 + w.l1 * v01) + h.l1 * (w.l0 * v10 + w.l1 * v11);
      const long long o = ((long long)m * pp.oh + i) * pp.ow + j;
      out[o] = v;
      if (gt) {
        const float t = (float)gt[o];
        const float pr = 1.0f / (1.0f + __expf(-v));
        si += pr * t;
        st += t;
        sp += pr;
      }
    }
  }
  if (!gt) return;
  si = wave_sum(si); st = wave_sum(st); sp = wave_sum(sp);
  const int wave = tid >> 6, lane = tid & 63;
  if (lane == 0) { red[0][wave] = si; red[1][wave] = st; red[2][wave] = sp; }
  __syncthreads();
  if (tid < 3)
    part[((long long)m * gridDim.x + blockIdx.x) * 3 + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

// Dice partial sums of already post-processed masks (the drop-in DiceCELoss on [B, N, H, W] logits):
// part[m][blk][3] = (sum p*t, sum t, sum p) over the blk-th contiguous chunk of map m, float4 loads.
__global__ __launch_bounds__(256) void dice_partials_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                            long long HW, long long chunk, float* __restrict__ part) {
  __shared__ float red[3][4];
  const int m = blockIdx.y, tid = threadIdx.x;
  const long long lo = (long long)blockIdx.x * chunk, hi = min(HW, lo + chunk);
  const float* xm = x + (long long)m * HW;
  const uint8_t* tm = gt + (long long)m * HW;
  float si = 0.0f, st = 0.0f, sp = 0.0f;
  for (long long e = lo + tid; e < hi; e += 256) {
    const float t = (float)tm[e];
    const float pr = 1.0f / (1.0f + __expf(-xm[e]));
    si += pr * t;
    st += t;
    sp += pr;
  }
  si = wave_sum(si); st = wave_sum(st); sp = wave_sum(sp);
  const int wave = tid >> 6, lane = tid & 63;
  if (lane == 0) { red[0][wave] = si; red[1][wave] = st; red[2][wave] = sp; }
  __syncthreads();
  if (tid < 3)
    part[((long long)m * gridDim.x + blockIdx.x) * 3 + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

// Per-map binary confusion counts of (x > 0) == (sigmoid(x) > 0.5) vs gt (evaluate_metrics,
// ref:octsam/models/training_utils.py:126-156): counts[m] += (tp, fp, fn, tn), integer atomics (exact,
// order-independent). One workgroup per (chunk, map), 16-B loads of 4 logits + 4 gt bytes per lane.
__global__ __launch_bounds__(256) void confusion_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                        long long HW, long long chunk,
                                                        unsigned long long* __restrict__ counts) {
  __shared__ unsigned red[4][4];
  const int m = blockIdx.y, tid = threadIdx.x;
  const long long lo = (long long)blockIdx.x * chunk, hi = min(HW, lo + chunk);
  const float* xm = x + (long long)m * HW;
  const uint8_t* tm = gt + (long long)m * HW;
  unsigned tp = 0, fp = 0, fn = 0, tn = 0;
  for (long long e = lo + tid; e < hi; e += 256) {
    const bool p = xm[e] > 0.0f, t = tm[e] != 0;
    tp += p & t;
    fp += p & !t;
    fn += !p & t;
    tn += !p & !t;
  }
  unsigned v[4] = {tp, fp, fn, tn};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  }
  if ((tid & 63) == 0)
    for (int k = 0; k < 4; ++k) red[k][tid >> 6] = v[k];
  __syncthreads();
  if (tid < 4)
    atomicAdd(counts + 4 * m + tid,
              (unsigned long long)(red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3]));
}

// dicece_bwd_kernel with four consecutive pixels per thread (HW % 4 == 0, N <= NR): 16-B logit loads and stores,
// 4-B target loads (the scalar form's 1-B loads move a quarter of the bytes per wave instruction). The same
// per-element arithmetic in the same order (dmask agrees with the scalar form to the last bits the compiler's FMA
// contraction moves): 200 -> 124 us at B = 8, N = 21, 496 x 512 (scripts/dicece_ab.py, profiles/r03/dicece_ab.log).
template <int NR>
__global__ __launch_bounds__(256) void dicece_bwd4_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                          const float* __restrict__ coef, int B, int N, int HW,
                                                          float w_dice, float w_ce, float inv_bhw,
                                                          float* __restrict__ dx, double* __restrict__ ce_part) {
  const int q4 = HW >> 2, total = B * q4;  // host-checked: B * HW < 2^31
  double ce = 0.0;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int b = e / q4, pix = (e - b * q4) * 4;
    const long long o0 = (long long)b * N * HW + pix;
    const float* cfb = coef + 2 * b * N;
    float4 xv[NR];
    uint32_t tv[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (n < N) {
        xv[n] = *(const float4*)(x + o0 + (long long)n * HW);
        tv[n] = *(const uint32_t*)(gt + o0 + (long long)n * HW);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < NR; ++n)
        if (n < N) mx = fmaxf(mx, ((const float*)&xv[n])[k]);
      float se = 0.0f, tsum = 0.0f, tx = 0.0f;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          const float xk = ((const float*)&xv[n])[k], tk = (float)((tv[n] >> (8 * k)) & 0xFF);
          se += __expf(xk - mx);
          tsum += tk;
          tx += tk * xk;
        }
      }
      const float lse = mx + __logf(se);
      ce += (double)(lse * tsum - tx);
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          const float xk = ((const float*)&xv[n])[k], tk = (float)((tv[n] >> (8 * k)) & 0xFF);
          const float sm = __expf(xk - lse);
          const float p = 1.0f / (1.0f + __expf(-xk));
          const float gd = (cfb[2 * n] * tk + cfb[2 * n + 1]) * p * (1.0f - p);
          const float gc = (sm * tsum - tk) * inv_bhw;
          ((float*)&xv[n])[k] = w_dice * gd + w_ce * gc;  // the logit is dead: its register takes d
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NR; ++n)
      if (n < N) *(float4*)(dx + o0 + (long long)n * HW) = xv[n];
  }
  __shared__ double red[4];
  ce = wave_sum_d(ce);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ce;
  __syncthreads();
  if (threadIdx.x == 0) ce_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// A/B: OCTSAM_DICECE_SCALAR=1 in the environment keeps the scalar kernel
bool dicece_vec_enabled() {
  static const bool on = [] {
    const char* v = getenv("OCTSAM_DICECE_SCALAR");
    return !(v && v[0] == '1');
  }();
  return on;
}

// per-map dice sums -> dice loss per map, and the per-map gradient coefficients
// coef[m] = (c1, c2): d(mean dice)/dx = (c1 * t + c2) * p (1 - p)
__global__ __launch_bounds__(256) void dice_reduce_kernel(const float* __restrict__ part, int M, int nblk,
                                                          double smooth_nr, double smooth_dr, double inv_count,
                                                          double* __restrict__ dice_map, float* __restrict__ coef) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  double I = 0, G = 0, Ps = 0;
  for (int b = lane; b < nblk; b += 64) {
    I += part[((long long)m * nblk + b) * 3 + 0];
    G += part[((long long)m * nblk + b) * 3 + 1];
    Ps += part[((long long)m * nblk + b) * 3 + 2];
  }
  I = wave_sum_d(I);
  G = wave_sum_d(G);
  Ps = wave_sum_d(Ps);
  if (lane) return;
  double num = 2.0 * I + smooth_nr, den = G + Ps + smooth_dr;
  dice_map[m] = 1.0 - num / den;
  coef[2 * m + 0] = (float)(-2.0 / den * inv_count);
  coef[2 * m + 1] = (float)(num / (den * den) * inv_count);
}

// per (b, pixel): CE over the N prompt channels + Dice gradient. dmask = w_dice*ddice + w_ce*dce.
// ce_part[blk] (double) = sum over the block's pixels of sum_n t_n (lse - x_n). NR > 0: the pixel's N <= NR
// logits and targets are read once into registers (NR = 0: three strided passes, any N).
template <int NR>
__global__ __launch_bounds__(256) void dicece_bwd_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                         const float* __restrict__ coef, int B, int N, int HW,
                                                         float w_dice, float w_ce, float inv_bhw,
                                                         float* __restrict__ dx, double* __restrict__ ce_part) {
  const int total = B * HW;  // host-checked < 2^31
  double ce = 0.0;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int b = e / HW, pix = e - b * HW;
    const float* xb = x + (long long)b * N * HW + pix;
    const uint8_t* tb = gt + (long long)b * N * HW + pix;
    float* db = dx + (long long)b * N * HW + pix;
    const float* cfb = coef + 2 * b * N;
    if constexpr (NR > 0) {
      float xv[NR], tv[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        xv[n] = n < N ? xb[(long long)n * HW] : -INFINITY;
        tv[n] = n < N ? (float)tb[(long long)n * HW] : 0.0f;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < NR; ++n) mx = fmaxf(mx, xv[n]);
      float se = 0.0f, tsum = 0.0f, tx = 0.0f;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          se += __expf(xv[n] - mx);
          tsum += tv[n];
          tx += tv[n] * xv[n];
        }
      }
      const float lse = mx + __logf(se);
      ce += (double)(lse * tsum - tx);
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          const float sm = __expf(xv[n] - lse);
          const float p = 1.0f / (1.0f + __expf(-xv[n]));
          const float gd = (cfb[2 * n] * tv[n] + cfb[2 * n + 1]) * p * (1.0f - p);
          const float gc = (sm * tsum - tv[n]) * inv_bhw;
          db[(long long)n * HW] = w_dice * gd + w_ce * gc;
        }
      }
    } else {
      float mx = -INFINITY;
      for (int n = 0; n < N; ++n) mx = fmaxf(mx, xb[(long long)n * HW]);
      float se = 0.0f, tsum = 0.0f, tx = 0.0f;
      for (int n = 0; n < N; ++n) {
        const float xv = xb[(long long)n * HW], t = (float)tb[(long long)n * HW];
        se += __expf(xv - mx);
        tsum += t;
        tx += t * xv;
      }
      const float lse = mx + __logf(se);
      ce += (double)(lse * tsum - tx);
      for (int n = 0; n < N; ++n) {
        const float xv = xb[(long long)n * HW], t = (float)tb[(long long)n * HW];
        const float sm = __expf(xv - lse);
        const float p = 1.0f / (1.0f + __expf(-xv));
        const float gd = (cfb[2 * n] * t + cfb[2 * n + 1]) * p * (1.0f - p);
        const float gc = (sm * tsum - t) * inv_bhw;
        db[(long long)n * HW] = w_dice * gd + w_ce * gc;
      }
    }
  }
  __shared__ double red[4];
  ce = wave_sum_d(ce);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ce;
  __syncthreads();
  if (threadIdx.x == 0) ce_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// loss[0] = mean dice, loss[1] = ce, loss[2] = w_dice*dice + w_ce*ce; one 256-thread block, strided sums then
// a fixed reduction tree (deterministic)
__global__ __launch_bounds__(256) void loss_finalize_kernel(const double* __restrict__ dice_map, int M,
                                                            const double* __restrict__ ce_part, int nblk,
                                                            double inv_bhw, double w_dice, double w_ce,
                                                            double* __restrict__ loss) {
  __shared__ double red[2][4];
  double d = 0.0, c = 0.0;
  for (int m = threadIdx.x; m < M; m += 256) d += dice_map[m];
  for (int b = threadIdx.x; b < nblk; b += 256) c += ce_part[b];
  d = wave_sum_d(d);
  c = wave_sum_d(c);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = d;
    red[1][wave] = c;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  d = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / M;
  c = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) * inv_bhw;
  loss[0] = d;
  loss[1] = c;
  loss[2] = w_dice * d + w_ce * c;
}

// Backward of the composite post-processing operator: dlow[m] = Wy^T dout[m] Wx.
// Row pass: tmp[m][i][b] = sum_{(j,w) in colcsr[b]} w * dout[m][i][j]; 4 rows of dout per workgroup staged
// in LDS by coalesced loads (ow <= 1024, host-checked), thread b walks column b's taps once for all 4 rows.
__global__ __launch_bounds__(256) void pp_bwd_rows_kernel(const float* __restrict__ dout, int oh, int ow, int S,
                                                          const int* __restrict__ cptr, const int* __restrict__ cidx,
                                                          const float* __restrict__ cw, float* __restrict__ tmp) {
  __shared__ float rows[4][1024];
  const int m = blockIdx.y, i0 = blockIdx.x * 4, tid = threadIdx.x;
  const int nr = min(4, oh - i0);
  for (int e = tid; e < nr * ow; e += 256) {
    const int r = e / ow, j = e - r * ow;
    rows[r][j] = dout[((long long)m * oh + i0 + r) * ow + j];
  }
  __syncthreads();
  for (int b = tid; b < S; b += 256) {
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int k = cptr[b]; k < cptr[b + 1]; ++k) {
      const int j = cidx[k];
      const float wv = cw[k];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += wv * rows[r][j];
    }
    for (int r = 0; r < nr; ++r) tmp[((long long)m * oh + i0 + r) * S + b] = acc[r];
  }
}
// Column pass: dlow[m][a][b] = sum_{(i,w) in rowcsr[a]} w * tmp[m][i][b]
__global__ __launch_bounds__(256) void pp_bwd_cols_kernel(const float* __restrict__ tmp, int oh, int S,
                                                          const int* __restrict__ rptr, const int* __restrict__ ridx,
                                                          const float* __restrict__ rw, float* __restrict__ dlow) {
  const int m = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S * S) return;
  const int a = e / S, b = e % S;
  const int k0 = rptr[a], k1 = rptr[a + 1];
  const float* src = tmp + (long long)m * oh * S + b;
  // the first CT taps' loads issued together (a row's taps: about 8 at the step's 256 -> 1024 -> 496 resampling), then
  // summed in tap order as the plain loop does (bit-identical); any further taps by the plain loop
  constexpr int CT = 12;
  float v[CT], wv[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const bool on = k0 + t < k1;
    wv[t] = on ? rw[k0 + t] : 0.0f;
    v[t] = on ? src[(long long)ridx[k0 + t] * S] : 0.0f;
  }
  float acc = 0.0f;
#pragma unroll
  for (int t = 0; t < CT; ++t)
    if (k0 + t < k1) acc += wv[t] * v[t];
  for (int k = k0 + CT; k < k1; ++k) acc += rw[k] * src[(long long)ridx[k] * S];
  dlow[(long long)m * S * S + e] = acc;
}

// DiceCE backward fused with the post-processing adjoint's row pass (the 170 MB d-mask write + read of the two-kernel
// form): one workgroup per (image b, output row i) computes d(DiceCE)/d mask for the row's pixels of all N prompts
// (dicece_bwd_kernel's per-pixel arithmetic: the CE couples the N prompts at a pixel, so one workgroup holds all of
// them) into LDS, adds the row's CE partial, and runs the row pass tmp[m][i][c] = sum_{(j,w) in colcsr[c]} w d[m][j]
// for every map m = b N + n with keep[m] < 0 (thread c: one output column, its taps walked once for all N maps).
// A map with keep[m] = k >= 0 (the topological loss's maps: their topo gradient joins later) gets its d-mask row
// written to dkeep[k] instead; octsam_topo_bwd_compact and octsam_pp_bwd_rows_maps finish it.
template <int NR>
__global__ __launch_bounds__(128) void dicece_pp_rows_kernel(const float* __restrict__ x, const uint8_t* __restrict__ gt,
                                                             const float* __restrict__ coef, int N, int H, int W,
                                                             float w_dice, float w_ce, float inv_bhw, int S,
                                                             const int* __restrict__ cptr, const int* __restrict__ cidx,
                                                             const float* __restrict__ cw, const int* __restrict__ keep,
                                                             float* __restrict__ dkeep, float* __restrict__ tmp,
                                                             double* __restrict__ ce_part) {
  // 128 threads x 4 consecutive pixels (16-B logit loads, 4-B target loads: dicece_bwd4_kernel's access pattern)
  extern __shared__ float dm[];  // [N][W]
  const int i = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const long long HW = (long long)H * W;
  const long long row0 = (long long)b * N * HW + (long long)i * W;  // (b, n = 0, i, 0)
  const float* cfb = coef + 2 * b * N;
  int kp[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) kp[n] = (n < N && keep) ? keep[b * N + n] : -1;
  double ce = 0.0;
  for (int j0 = 4 * tid; j0 < W; j0 += 4 * 128) {
    float4 xv[NR];
    uint32_t tv[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (n < N) {
        xv[n] = *(const float4*)(x + row0 + n * HW + j0);
        tv[n] = *(const uint32_t*)(gt + row0 + n * HW + j0);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < NR; ++n)
        if (n < N) mx = fmaxf(mx, ((const float*)&xv[n])[k]);
      float se = 0.0f, tsum = 0.0f, tx = 0.0f;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          const float xk = ((const float*)&xv[n])[k], tk = (float)((tv[n] >> (8 * k)) & 0xFF);
          se += __expf(xk - mx);
          tsum += tk;
          tx += tk * xk;
        }
      }
      const float lse = mx + __logf(se);
      ce += (double)(lse * tsum - tx);
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        if (n < N) {
          const float xk = ((const float*)&xv[n])[k], tk = (float)((tv[n] >> (8 * k)) & 0xFF);
          const float sm = __expf(xk - lse);
          const float p = 1.0f / (1.0f + __expf(-xk));
          const float gd = (cfb[2 * n] * tk + cfb[2 * n + 1]) * p * (1.0f - p);
          const float gc = (sm * tsum - tk) * inv_bhw;
          ((float*)&xv[n])[k] = w_dice * gd + w_ce * gc;  // the logit is dead: its register takes d
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (n < N) {
        if (kp[n] >= 0) *(float4*)(dkeep + (long long)kp[n] * HW + (long long)i * W + j0) = xv[n];
        else *(float4*)(dm + n * W + j0) = xv[n];
      }
    }
  }
  __syncthreads();
  for (int c = tid; c < S; c += 128) {
    float acc[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[n] = 0.0f;
    for (int e = cptr[c]; e < cptr[c + 1]; ++e) {
      const int j = cidx[e];
      const float wv = cw[e];
#pragma unroll
      for (int n = 0; n < NR; ++n)
        if (n < N) acc[n] += wv * dm[n * W + j];
    }
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (n < N && kp[n] < 0) tmp[((long long)(b * N + n) * H + i) * S + c] = acc[n];
    }
  }
  __shared__ double red[2];
  ce = wave_sum_d(ce);
  if ((tid & 63) == 0) red[tid >> 6] = ce;
  __syncthreads();
  if (tid == 0) ce_part[(long long)b * H + i] = red[0] + red[1];
}

// the row pass for maps given in compact storage: dout[k] (k < K) -> tmp[map_idx[k]] (pp_bwd_rows_kernel's order)
__global__ __launch_bounds__(256) void pp_bwd_rows_maps_kernel(const float* __restrict__ dout, const int* __restrict__ map_idx,
                                                               int oh, int ow, int S, const int* __restrict__ cptr,
                                                               const int* __restrict__ cidx, const float* __restrict__ cw,
                                                               float* __restrict__ tmp) {
  __shared__ float rows[4][1024];
  const int k = blockIdx.y, i0 = blockIdx.x * 4, tid = threadIdx.x;
  const int m = map_idx[k];
  const int nr = min(4, oh - i0);
  for (int e = tid; e < nr * ow; e += 256) {
    const int r = e / ow, j = e - r * ow;
    rows[r][j] = dout[((long long)k * oh + i0 + r) * ow + j];
  }
  __syncthreads();
  for (int b = tid; b < S; b += 256) {
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int e = cptr[b]; e < cptr[b + 1]; ++e) {
      const int j = cidx[e];
      const float wv = cw[e];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += wv * rows[r][j];
    }
    for (int r = 0; r < nr; ++r) tmp[((long long)m * oh + i0 + r) * S + b] = acc[r];
  }
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
// compact: dmask holds the K maps themselves ([K, ih, iw]; masks are still read at map_idx[k])
__global__ __launch_bounds__(256) void topo_bwd_kernel(const float* __restrict__ masks, const int* __restrict__ map_idx,
                                                       int ih, int iw, int oh, int ow, float sh, float sw, int sig,
                                                       const float* __restrict__ dpred, float scale,
                                                       float* __restrict__ dmask, int compact) {
  const int k = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= oh * ow) return;
  const float g = dpred[(long long)k * oh * ow + e] * scale;
  if (g == 0.0f) return;
  const int i = e / ow, j = e % ow;
  const long long mo = (long long)map_idx[k] * ih * iw;
  const long long md = compact ? (long long)k * ih * iw : mo;
  Lin a = lin_act(i, ih, sh), b = lin_act(j, iw, sw);
  auto add = [&](int r, int c, float w) {
    const long long off = (long long)r * iw + c;
    float d = 1.0f;
    if (sig) {
      float s = 1.0f / (1.0f + __expf(-masks[mo + off]));
      d = s * (1.0f - s);
    }
    atomicAdd(dmask + md + off, g * w * d);
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
  OCTSAM_CHECK_ARG((long long)out_h * out_w < (1 << 24), "octsam_postproc_fwd: output too large (%d x %d)", out_h,
                   out_w);
  PP pp{S, mid, crop_h, crop_w, out_h, out_w, (float)S / (float)mid, (float)crop_h / (float)out_h,
        (float)crop_w / (float)out_w};
  const int ngrp = (out_h + PP_ROWS - 1) / PP_ROWS;
  OCTSAM_CHECK_ARG(S <= 256 && S % 4 == 0 && ((uintptr_t)lowres & 15) == 0 && (!gt || nblk == ngrp),
                   "octsam_postproc_fwd: needs S <= 256, S %% 4 == 0, 16-B aligned lowres and nblk == ceil(out_h/4)");
  // the low-res rows of 4 consecutive output rows must fit the LDS range (PP_LRMAX): originals down to
  // ~1/12 of the crop
  OCTSAM_CHECK_ARG((double)PP_ROWS * crop_h / out_h * S / mid + 4.0 <= PP_LRMAX,
                   "octsam_postproc_fwd: output rows too coarse for the staged low-res range");
  hipLaunchKernelGGL(postproc_fwd_kernel, dim3(ngrp, M), dim3(256), 0, (hipStream_t)stream, lowres, pp, out, gt,
                     dice_part);
  OCTSAM_LAUNCH_CHECK("octsam_postproc_fwd");
  return 0;
}

extern "C" int octsam_dice_partials(const float* masks, const uint8_t* gt, int32_t M, int64_t HW, float* dice_part,
                                    int32_t nblk, void* stream) {
  OCTSAM_CHECK_ARG(masks && gt && dice_part && M > 0 && HW > 0 && nblk > 0 && M <= 65535,
                   "octsam_dice_partials: bad args");
  const long long chunk = (HW + nblk - 1) / nblk;
  hipLaunchKernelGGL(dice_partials_kernel, dim3(nblk, M), dim3(256), 0, (hipStream_t)stream, masks, gt, (long long)HW,
                     chunk, dice_part);
  OCTSAM_LAUNCH_CHECK("octsam_dice_partials");
  return 0;
}

extern "C" int octsam_confusion(const float* masks, const uint8_t* gt, int32_t M, int64_t HW, uint64_t* counts,
                                void* stream) {
  OCTSAM_CHECK_ARG(masks && gt && counts && M >= 0 && HW > 0 && M <= 65535, "octsam_confusion: bad args");
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(counts, 0, (size_t)M * 4 * sizeof(uint64_t), s);
  if (e != hipSuccess) {
    octsam::set_error("octsam_confusion: memset failed: %s", hipGetErrorString(e));
    return (int)e;
  }
  const long long nb = (HW + 4095) / 4096;
  const int nblk = (int)(nb < 64 ? nb : 64);
  const long long chunk = (HW + nblk - 1) / nblk;
  hipLaunchKernelGGL(confusion_kernel, dim3(nblk, M), dim3(256), 0, s, masks, gt, (long long)HW, chunk,
                     (unsigned long long*)counts);
  OCTSAM_LAUNCH_CHECK("octsam_confusion");
  return 0;
}

extern "C" int octsam_dice_reduce(const float* dice_part, int32_t M, int32_t nblk, double* dice_map, float* coef,
                                  void* stream) {
  OCTSAM_CHECK_ARG(dice_part && dice_map && coef && M > 0 && nblk > 0, "octsam_dice_reduce: bad args");
  hipLaunchKernelGGL(dice_reduce_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, dice_part, M, nblk,
                     1e-5, 1e-5, 1.0 / M, dice_map, coef);
  OCTSAM_LAUNCH_CHECK("octsam_dice_reduce");
  return 0;
}

extern "C" int octsam_dicece_bwd(const float* masks, const uint8_t* gt, const float* coef, int32_t B, int32_t N,
                                 int64_t HW, float w_dice, float w_ce, float* dmask, double* ce_part, int32_t nblk,
                                 void* stream) {
  OCTSAM_CHECK_ARG(masks && gt && coef && dmask && ce_part && B > 0 && N > 0 && HW > 0 && nblk > 0,
                   "octsam_dicece_bwd: bad args");
  OCTSAM_CHECK_ARG((long long)B * HW < (1LL << 31), "octsam_dicece_bwd: B*HW too large");
  const float inv = (float)(1.0 / ((double)B * HW));
  hipStream_t s = (hipStream_t)stream;
  const bool vec = dicece_vec_enabled() && HW % 4 == 0 && ((uintptr_t)masks & 15) == 0 && ((uintptr_t)dmask & 15) == 0 &&
                   ((uintptr_t)gt & 3) == 0;
  if (vec && N <= 24)
    hipLaunchKernelGGL(dicece_bwd4_kernel<24>, dim3(nblk), dim3(256), 0, s, masks, gt, coef, B, N, (int)HW, w_dice,
                       w_ce, inv, dmask, ce_part);
  else if (N <= 32)
    hipLaunchKernelGGL(dicece_bwd_kernel<32>, dim3(nblk), dim3(256), 0, s, masks, gt, coef, B, N, (int)HW, w_dice, w_ce,
                       inv, dmask, ce_part);
  else
    hipLaunchKernelGGL(dicece_bwd_kernel<0>, dim3(nblk), dim3(256), 0, s, masks, gt, coef, B, N, (int)HW, w_dice, w_ce,
                       inv, dmask, ce_part);
  OCTSAM_LAUNCH_CHECK("octsam_dicece_bwd");
  return 0;
}

extern "C" int octsam_loss_finalize(const double* dice_map, int32_t M, const double* ce_part, int32_t nblk, int32_t B,
                                    int64_t HW, double w_dice, double w_ce, double* loss, void* stream) {
  OCTSAM_CHECK_ARG(dice_map && ce_part && loss && M > 0 && nblk > 0, "octsam_loss_finalize: bad args");
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, dice_map, M, ce_part, nblk,
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
  OCTSAM_CHECK_ARG(out_w <= 1024, "octsam_postproc_bwd: out_w must be <= 1024");
  hipLaunchKernelGGL(pp_bwd_rows_kernel, dim3((unsigned)((out_h + 3) / 4), M), dim3(256), 0, s, dout, out_h, out_w, S,
                     col_ptr, col_idx, col_w, tmp);
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
                     map_idx, in_h, in_w, out_h, out_w, sh, sw, apply_sigmoid, dpred, scale, dmask, 0);
  OCTSAM_LAUNCH_CHECK("octsam_topo_bwd");
  return 0;
}

extern "C" int octsam_topo_bwd_compact(const float* masks, const int32_t* map_idx, int32_t K, int32_t in_h,
                                       int32_t in_w, int32_t out_h, int32_t out_w, int32_t apply_sigmoid,
                                       const float* dpred, float scale, float* dmask_k, void* stream) {
  OCTSAM_CHECK_ARG(masks && map_idx && dpred && dmask_k && K >= 0, "octsam_topo_bwd_compact: bad args");
  if (K == 0) return 0;
  float sh = (float)(in_h - 1) / (float)(out_h - 1), sw = (float)(in_w - 1) / (float)(out_w - 1);
  hipLaunchKernelGGL(topo_bwd_kernel, dim3((out_h * out_w + 255) / 256, K), dim3(256), 0, (hipStream_t)stream, masks,
                     map_idx, in_h, in_w, out_h, out_w, sh, sw, apply_sigmoid, dpred, scale, dmask_k, 1);
  OCTSAM_LAUNCH_CHECK("octsam_topo_bwd_compact");
  return 0;
}

extern "C" int octsam_dicece_pp_rows(const float* masks, const uint8_t* gt, const float* coef, int32_t B, int32_t N,
                                     int32_t H, int32_t W, float w_dice, float w_ce, int32_t S, const int32_t* col_ptr,
                                     const int32_t* col_idx, const float* col_w, const int32_t* keep, float* dkeep,
                                     float* tmp, double* ce_part, void* stream) {
  OCTSAM_CHECK_ARG(masks && gt && coef && col_ptr && col_idx && col_w && tmp && ce_part && B > 0 && N > 0 && H > 0 &&
                       W > 0 && S > 0 && (!keep || dkeep) && B <= 65535,
                   "octsam_dicece_pp_rows: bad args");
  OCTSAM_CHECK_ARG(N <= 32 && (size_t)N * W * 4 <= 160 * 1024 && (long long)B * H * W < (1LL << 31) && W % 4 == 0 &&
                       ((uintptr_t)masks & 15) == 0 && ((uintptr_t)gt & 3) == 0 && (!dkeep || ((uintptr_t)dkeep & 15) == 0),
                   "octsam_dicece_pp_rows: needs N <= 32 prompts, N * W * 4 <= 160 KB, W %% 4 == 0 and 16-B aligned "
                   "masks / dkeep (N=%d, W=%d)", N, W);
  const float inv = (float)(1.0 / ((double)B * H * W));
  const size_t lds = (size_t)N * W * 4;
  hipStream_t s = (hipStream_t)stream;
  if (N <= 24) {
    static size_t attr = 0;
    if (lds > 65536 && lds > attr) {
      (void)hipFuncSetAttribute((const void*)dicece_pp_rows_kernel<24>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr = lds;
    }
    hipLaunchKernelGGL(dicece_pp_rows_kernel<24>, dim3(H, B), dim3(128), lds, s, masks, gt, coef, N, H, W, w_dice, w_ce,
                       inv, S, col_ptr, col_idx, col_w, keep, dkeep, tmp, ce_part);
  } else {
    static size_t attr = 0;
    if (lds > 65536 && lds > attr) {
      (void)hipFuncSetAttribute((const void*)dicece_pp_rows_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr = lds;
    }
    hipLaunchKernelGGL(dicece_pp_rows_kernel<32>, dim3(H, B), dim3(128), lds, s, masks, gt, coef, N, H, W, w_dice, w_ce,
                       inv, S, col_ptr, col_idx, col_w, keep, dkeep, tmp, ce_part);
  }
  OCTSAM_LAUNCH_CHECK("octsam_dicece_pp_rows");
  return 0;
}

extern "C" int octsam_pp_bwd_rows_maps(const float* dout_k, const int32_t* map_idx, int32_t K, int32_t S, int32_t out_h,
                                       int32_t out_w, const int32_t* col_ptr, const int32_t* col_idx, const float* col_w,
                                       float* tmp, void* stream) {
  OCTSAM_CHECK_ARG(dout_k && map_idx && col_ptr && col_idx && col_w && tmp && K >= 0 && out_w <= 1024 && K <= 65535,
                   "octsam_pp_bwd_rows_maps: bad args");
  if (K == 0) return 0;
  hipLaunchKernelGGL(pp_bwd_rows_maps_kernel, dim3((unsigned)((out_h + 3) / 4), K), dim3(256), 0, (hipStream_t)stream,
                     dout_k, map_idx, out_h, out_w, S, col_ptr, col_idx, col_w, tmp);
  OCTSAM_LAUNCH_CHECK("octsam_pp_bwd_rows_maps");
  return 0;
}

extern "C" int octsam_pp_bwd_cols(const float* tmp, int32_t M, int32_t S, int32_t out_h, const int32_t* row_ptr,
                                  const int32_t* row_idx, const float* row_w, float* dlowres, void* stream) {
  OCTSAM_CHECK_ARG(tmp && row_ptr && row_idx && row_w && dlowres && M > 0 && M <= 65535, "octsam_pp_bwd_cols: bad args");
  hipLaunchKernelGGL(pp_bwd_cols_kernel, dim3((S * S + 255) / 256, M), dim3(256), 0, (hipStream_t)stream, tmp, out_h, S,
                     row_ptr, row_idx, row_w, dlowres);
  OCTSAM_LAUNCH_CHECK("octsam_pp_bwd_cols");
  return 0;
}
