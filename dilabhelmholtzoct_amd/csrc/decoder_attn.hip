// Attention cores of SamTwoWayTransformer (hf:modeling_sam.py:195-405), forward and backward.
// The q/k/v/out projections are octsam_gemm calls; these kernels do softmax(q k^T * scale) v.
//
//   tok   : token self-attention, T<=8 tokens, 8 heads x 32 (SamTwoWayAttentionBlock.self_attn)
//   t2i   : tokens -> image, Tq<=8 queries, L=4096 keys, 8 heads x 16 (cross_attn_token_to_image,
//           final_attn_token_to_image). K/V may be per image (layer 0: keys = image embedding +
//           dense prompt, shared by the image's prompts, repeat_interleave at :499-501) - kv_rep.
//   i2t   : image -> tokens, L=4096 queries, Tk<=8 keys, 8 heads x 16 (cross_attn_image_to_token).
//           Q may be per image (q_rep).
// Token-side tensors are fp32, image-side tensors bf16 with an explicit row stride, so the kernels
// read straight out of concatenated projection buffers. Backward recomputes probabilities
// (t2i from the saved log-sum-exp, i2t and tok from scratch). Reductions over the 4096 image rows
// are done in fixed order (per-block partials + octsam_splitk_reduce): deterministic.
#include "common.h"
#include "../../include/octsam.h"

namespace {

constexpr int MAXT = 8;

// ---------------------------------------------------------------------------------------- tok
// q,k,v fp32 [P, T, 256]; out bf16 [P, T, 256]; probs fp32 [P, 8, T, T]
__global__ __launch_bounds__(256) void tok_attn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, int T, bf16* __restrict__ out,
                                                           float* __restrict__ probs) {
  const int p = blockIdx.x;
  __shared__ float sp[8][MAXT][MAXT];
  const float scale = 0.17677669529663687f;  // 32^-0.5
  const float* qp = q + (long long)p * T * 256;
  const float* kp = k + (long long)p * T * 256;
  const float* vp = v + (long long)p * T * 256;
  for (int hi = threadIdx.x; hi < 8 * T; hi += 256) {
    int h = hi / T, i = hi % T;
    float s[MAXT];
    float mx = -INFINITY;
    for (int j = 0; j < T; ++j) {
      float acc = 0.0f;
      for (int d = 0; d < 32; ++d) acc += qp[i * 256 + h * 32 + d] * kp[j * 256 + h * 32 + d];
      s[j] = acc * scale;
      mx = fmaxf(mx, s[j]);
    }
    float sum = 0.0f;
    for (int j = 0; j < T; ++j) { s[j] = __expf(s[j] - mx); sum += s[j]; }
    for (int j = 0; j < T; ++j) {
      float pr = s[j] / sum;
      sp[h][i][j] = pr;
      probs[(((long long)p * 8 + h) * T + i) * T + j] = pr;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * 256; e += 256) {
    int i = e / 256, c = e % 256, h = c / 32;
    float acc = 0.0f;
    for (int j = 0; j < T; ++j) acc += sp[h][i][j] * vp[j * 256 + c];
    out[(long long)p * T * 256 + e] = (bf16)acc;
  }
}

// dout fp32 [P,T,256] -> dq, dk, dv bf16 [P,T,256]
__global__ __launch_bounds__(256) void tok_attn_bwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, const float* __restrict__ probs,
                                                           const float* __restrict__ dout, int T,
                                                           bf16* __restrict__ dq, bf16* __restrict__ dk,
                                                           bf16* __restrict__ dv) {
  const int p = blockIdx.x;
  __shared__ float sP[8][MAXT][MAXT];
  __shared__ float sdS[8][MAXT][MAXT];
  const float scale = 0.17677669529663687f;
  const long long base = (long long)p * T * 256;
  for (int e = threadIdx.x; e < 8 * T * T; e += 256) {
    int h = e / (T * T), i = (e / T) % T, j = e % T;
    sP[h][i][j] = probs[(((long long)p * 8 + h) * T + i) * T + j];
  }
  __syncthreads();
  for (int hi = threadIdx.x; hi < 8 * T; hi += 256) {
    int h = hi / T, i = hi % T;
    float dp[MAXT];
    float dsum = 0.0f;
    for (int j = 0; j < T; ++j) {
      float acc = 0.0f;
      for (int d = 0; d < 32; ++d) acc += dout[base + i * 256 + h * 32 + d] * v[base + j * 256 + h * 32 + d];
      dp[j] = acc;
      dsum += sP[h][i][j] * acc;
    }
    for (int j = 0; j < T; ++j) sdS[h][i][j] = sP[h][i][j] * (dp[j] - dsum);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * 256; e += 256) {
    int i = e / 256, c = e % 256, h = c / 32;
    float aq = 0.0f, ak = 0.0f, av = 0.0f;
    for (int j = 0; j < T; ++j) {
      aq += sdS[h][i][j] * k[base + j * 256 + c];
      ak += sdS[h][j][i] * q[base + j * 256 + c];
      av += sP[h][j][i] * dout[base + j * 256 + c];
    }
    dq[base + e] = (bf16)(aq * scale);
    dk[base + e] = (bf16)(ak * scale);
    dv[base + e] = (bf16)av;
  }
}

// ---------------------------------------------------------------------------------------- t2i
// XCD-aware (prompt, head) decode: the 8 heads of a prompt share one XCD (same K/V rows in L2).
__device__ __forceinline__ void t2i_decode(int id, int& p, int& h) {
  p = (id & 7) + 8 * (id >> 6);
  h = (id >> 3) & 7;
}

// q fp32 [P,Tq,128]; k,v bf16 rows (kv block b = p / kv_rep) [*, L, ldkv]; out bf16 [P,Tq,128]; lse [P,8,Tq]
__global__ __launch_bounds__(MAXT * 64) void t2i_fwd_kernel(const float* __restrict__ q, const bf16* __restrict__ k,
                                                            const bf16* __restrict__ v, long long ldkv, int kv_rep,
                                                            int P, int Tq, int L, bf16* __restrict__ out,
                                                            float* __restrict__ lse) {
  int p, h;
  t2i_decode(blockIdx.x, p, h);
  if (p >= P) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= Tq) return;
  const long long kvb = (long long)(p / kv_rep) * L;
  float qr[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) qr[d] = q[((long long)p * Tq + wave) * 128 + h * 16 + d] * 0.25f;
  float m = -INFINITY, l = 0.0f, o[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = 0.0f;
  for (int key = lane; key < L; key += 64) {
    const bf16* kr = k + (kvb + key) * ldkv + h * 16;
    const bf16* vr = v + (kvb + key) * ldkv + h * 16;
    bf16x8 k0 = *(const bf16x8*)kr, k1 = *(const bf16x8*)(kr + 8);
    float s = 0.0f;
#pragma unroll
    for (int d = 0; d < 8; ++d) s += qr[d] * (float)k0[d] + qr[8 + d] * (float)k1[d];
    float mn = fmaxf(m, s);
    float a = __expf(m - mn), e = __expf(s - mn);
    bf16x8 v0 = *(const bf16x8*)vr, v1 = *(const bf16x8*)(vr + 8);
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      o[d] = o[d] * a + e * (float)v0[d];
      o[8 + d] = o[8 + d] * a + e * (float)v1[d];
    }
    l = l * a + e;
    m = mn;
  }
  const float M = wave_max(m);
  const float f = (m == -INFINITY) ? 0.0f : __expf(m - M);
  l = wave_sum(l * f);
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = wave_sum(o[d] * f);
  if (lane < 16) {
    float val = 0.0f;
#pragma unroll
    for (int d = 0; d < 16; ++d) val = (lane == d) ? o[d] : val;
    out[((long long)p * Tq + wave) * 128 + h * 16 + lane] = (bf16)(val / l);
  }
  if (lane == 0) lse[((long long)p * 8 + h) * Tq + wave] = M + __logf(l);
}

// Backward: one block per (prompt, head), 256 threads; keys in chunks of 256 (one per thread).
// dq bf16 [P,Tq,128]; dk, dv bf16 per prompt [P, L, lddkv] (head slice h*16)
__global__ __launch_bounds__(256) void t2i_bwd_kernel(const float* __restrict__ q, const bf16* __restrict__ k,
                                                      const bf16* __restrict__ v, long long ldkv, int kv_rep, int P,
                                                      int Tq, int L, const bf16* __restrict__ out,
                                                      const float* __restrict__ dout, const float* __restrict__ lse,
                                                      bf16* __restrict__ dq, bf16* __restrict__ dk,
                                                      bf16* __restrict__ dv, long long lddkv) {
  int p, h;
  t2i_decode(blockIdx.x, p, h);
  if (p >= P) return;
  __shared__ float sq[MAXT][16], sdo[MAXT][16], sD[MAXT], sL[MAXT];
  __shared__ float sds[256][MAXT + 1];
  __shared__ float skf[256][17];
  __shared__ float red[2][MAXT * 16];
  const int tid = threadIdx.x;
  for (int e = tid; e < Tq * 16; e += 256) {
    int i = e / 16, d = e % 16;
    sq[i][d] = q[((long long)p * Tq + i) * 128 + h * 16 + d] * 0.25f;
    sdo[i][d] = dout[((long long)p * Tq + i) * 128 + h * 16 + d];
  }
  if (tid < Tq) {
    float acc = 0.0f;
    for (int d = 0; d < 16; ++d)
      acc += dout[((long long)p * Tq + tid) * 128 + h * 16 + d] * (float)out[((long long)p * Tq + tid) * 128 + h * 16 + d];
    sD[tid] = acc;
    sL[tid] = lse[((long long)p * 8 + h) * Tq + tid];
  }
  __syncthreads();
  const long long kvb = (long long)(p / kv_rep) * L;
  // phase-2 owner: (i, d, half) -> sums 128 of the chunk's 256 keys
  const int oi = (tid >> 1) / 16, od = (tid >> 1) % 16, ohalf = tid & 1;
  float dq_acc = 0.0f;
  for (int c0 = 0; c0 < L; c0 += 256) {
    const int key = c0 + tid;
    if (key < L) {
      const bf16* kr = k + (kvb + key) * ldkv + h * 16;
      const bf16* vr = v + (kvb + key) * ldkv + h * 16;
      float kf[16], vf[16];
      bf16x8 k0 = *(const bf16x8*)kr, k1 = *(const bf16x8*)(kr + 8);
      bf16x8 v0 = *(const bf16x8*)vr, v1 = *(const bf16x8*)(vr + 8);
#pragma unroll
      for (int d = 0; d < 8; ++d) { kf[d] = (float)k0[d]; kf[8 + d] = (float)k1[d]; vf[d] = (float)v0[d]; vf[8 + d] = (float)v1[d]; }
      float dka[16], dva[16];
#pragma unroll
      for (int d = 0; d < 16; ++d) { dka[d] = 0.0f; dva[d] = 0.0f; skf[tid][d] = kf[d]; }
#pragma unroll
      for (int i = 0; i < MAXT; ++i) {
        float ds = 0.0f;
        if (i < Tq) {
          float s = 0.0f, dp = 0.0f;
#pragma unroll
          for (int d = 0; d < 16; ++d) { s += sq[i][d] * kf[d]; dp += sdo[i][d] * vf[d]; }
          float pr = __expf(s - sL[i]);
          ds = pr * (dp - sD[i]);
#pragma unroll
          for (int d = 0; d < 16; ++d) {
            dva[d] += pr * sdo[i][d];
            dka[d] += ds * sq[i][d];
          }
        }
        sds[tid][i] = ds;
      }
      bf16x8 o0, o1, w0, w1;
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        o0[d] = (bf16)dka[d]; o1[d] = (bf16)dka[8 + d];
        w0[d] = (bf16)dva[d]; w1[d] = (bf16)dva[8 + d];
      }
      bf16* dkr = dk + ((long long)p * L + key) * lddkv + h * 16;
      bf16* dvr = dv + ((long long)p * L + key) * lddkv + h * 16;
      *(bf16x8*)dkr = o0; *(bf16x8*)(dkr + 8) = o1;
      *(bf16x8*)dvr = w0; *(bf16x8*)(dvr + 8) = w1;
    } else {
#pragma unroll
      for (int i = 0; i < MAXT; ++i) sds[tid][i] = 0.0f;
#pragma unroll
      for (int d = 0; d < 16; ++d) skf[tid][d] = 0.0f;
    }
    __syncthreads();
    if (oi < Tq) {
      float a = 0.0f;
      for (int t = ohalf * 128; t < ohalf * 128 + 128; ++t) a += sds[t][oi] * skf[t][od];
      dq_acc += a;
    }
    __syncthreads();
  }
  if (oi < Tq) red[ohalf][oi * 16 + od] = dq_acc;
  __syncthreads();
  for (int e = tid; e < Tq * 16; e += 256) {
    int i = e / 16, d = e % 16;
    // ds was formed with the scaled q; d(s)/d(q) = 0.25 * k
    dq[((long long)p * Tq + i) * 128 + h * 16 + d] = (bf16)((red[0][e] + red[1][e]) * 0.25f);
  }
}

// ---------------------------------------------------------------------------------------- i2t
constexpr int I2T_ROWS = 256;  // image rows per block

// q bf16 rows (q block b = p / q_rep) [*, L, ldq]; k, v fp32 [P, Tk, 128]; out bf16 [P, L, ldo]
__global__ __launch_bounds__(256) void i2t_fwd_kernel(const bf16* __restrict__ q, long long ldq, int q_rep,
                                                      const float* __restrict__ k, const float* __restrict__ v, int Tk,
                                                      int L, bf16* __restrict__ out, long long ldo) {
  const int p = blockIdx.y;
  const int r0 = blockIdx.x * I2T_ROWS;
  __shared__ float sk[MAXT][128], sv[MAXT][128];
  for (int e = threadIdx.x; e < Tk * 128; e += 256) {
    sk[e / 128][e % 128] = k[(long long)p * Tk * 128 + e] * 0.25f;
    sv[e / 128][e % 128] = v[(long long)p * Tk * 128 + e];
  }
  __syncthreads();
  const int h = threadIdx.x & 7;
  const long long qb = (long long)(p / q_rep) * L;
  for (int r = r0 + (threadIdx.x >> 3); r < r0 + I2T_ROWS && r < L; r += 32) {
    const bf16* qr = q + (qb + r) * ldq + h * 16;
    bf16x8 a0 = *(const bf16x8*)qr, a1 = *(const bf16x8*)(qr + 8);
    float qf[16];
#pragma unroll
    for (int d = 0; d < 8; ++d) { qf[d] = (float)a0[d]; qf[8 + d] = (float)a1[d]; }
    float s[MAXT];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      if (j < Tk) {
        float acc = 0.0f;
#pragma unroll
        for (int d = 0; d < 16; ++d) acc += qf[d] * sk[j][h * 16 + d];
        s[j] = acc;
        mx = fmaxf(mx, acc);
      }
    }
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) { s[j] = __expf(s[j] - mx); sum += s[j]; }
    const float inv = 1.0f / sum;
    float o[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d] = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) {
        float pr = s[j] * inv;
#pragma unroll
        for (int d = 0; d < 16; ++d) o[d] += pr * sv[j][h * 16 + d];
      }
    bf16x8 o0, o1;
#pragma unroll
    for (int d = 0; d < 8; ++d) { o0[d] = (bf16)o[d]; o1[d] = (bf16)o[8 + d]; }
    bf16* orow = out + ((long long)p * L + r) * ldo + h * 16;
    *(bf16x8*)orow = o0;
    *(bf16x8*)(orow + 8) = o1;
  }
}

// Backward. dout bf16 [P, L, lddo]; writes dq bf16 [P, L, lddq] and per-block partials
// part[blk][P][2][Tk][128] (dk then dv), blk = blockIdx.x (L / 256 blocks per prompt).
__global__ __launch_bounds__(256) void i2t_bwd_kernel(const bf16* __restrict__ q, long long ldq, int q_rep,
                                                      const float* __restrict__ k, const float* __restrict__ v, int Tk,
                                                      int L, const bf16* __restrict__ dout, long long lddo,
                                                      bf16* __restrict__ dq, long long lddq, float* __restrict__ part,
                                                      int P) {
  const int p = blockIdx.y;
  const int r0 = blockIdx.x * I2T_ROWS;
  __shared__ float sk[MAXT][128], sv[MAXT][128];
  __shared__ float sds[32][8][MAXT], spr[32][8][MAXT];
  __shared__ float sq[32][128], sdo[32][128];
  for (int e = threadIdx.x; e < Tk * 128; e += 256) {
    sk[e / 128][e % 128] = k[(long long)p * Tk * 128 + e] * 0.25f;
    sv[e / 128][e % 128] = v[(long long)p * Tk * 128 + e];
  }
  __syncthreads();
  const int h = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const long long qb = (long long)(p / q_rep) * L;
  // phase-2 ownership: 2*Tk*128 outputs over 256 threads
  float accs[2 * MAXT * 128 / 256];
#pragma unroll
  for (int i = 0; i < 2 * MAXT * 128 / 256; ++i) accs[i] = 0.0f;
  const int nout = 2 * Tk * 128;
  for (int it = 0; it < I2T_ROWS / 32; ++it) {
    const int r = r0 + it * 32 + rl;
    const bool valid = r < L;
    float qf[16], dof[16];
    if (valid) {
      const bf16* qr = q + (qb + r) * ldq + h * 16;
      const bf16* dr = dout + ((long long)p * L + r) * lddo + h * 16;
      bf16x8 a0 = *(const bf16x8*)qr, a1 = *(const bf16x8*)(qr + 8);
      bf16x8 b0 = *(const bf16x8*)dr, b1 = *(const bf16x8*)(dr + 8);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        qf[d] = (float)a0[d]; qf[8 + d] = (float)a1[d];
        dof[d] = (float)b0[d]; dof[8 + d] = (float)b1[d];
      }
    } else {
#pragma unroll
      for (int d = 0; d < 16; ++d) { qf[d] = 0.0f; dof[d] = 0.0f; }
    }
    float s[MAXT], dp[MAXT];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) {
        float acc = 0.0f, acc2 = 0.0f;
#pragma unroll
        for (int d = 0; d < 16; ++d) { acc += qf[d] * sk[j][h * 16 + d]; acc2 += dof[d] * sv[j][h * 16 + d]; }
        s[j] = acc;
        dp[j] = acc2;
        mx = fmaxf(mx, acc);
      }
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) { s[j] = __expf(s[j] - mx); sum += s[j]; }
    const float inv = 1.0f / sum;
    float dsum = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) { s[j] *= inv; dsum += s[j] * dp[j]; }
    float dqf[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) dqf[d] = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXT; ++j)
      if (j < Tk) {
        float ds = valid ? s[j] * (dp[j] - dsum) : 0.0f;
        sds[rl][h][j] = ds;
        spr[rl][h][j] = valid ? s[j] : 0.0f;
#pragma unroll
        for (int d = 0; d < 16; ++d) dqf[d] += ds * sk[j][h * 16 + d];  // sk already * 0.25
      }
    if (valid) {
      bf16x8 o0, o1;
#pragma unroll
      for (int d = 0; d < 8; ++d) { o0[d] = (bf16)dqf[d]; o1[d] = (bf16)dqf[8 + d]; }
      bf16* dr = dq + ((long long)p * L + r) * lddq + h * 16;
      *(bf16x8*)dr = o0;
      *(bf16x8*)(dr + 8) = o1;
    }
#pragma unroll
    for (int d = 0; d < 16; ++d) { sq[rl][h * 16 + d] = qf[d]; sdo[rl][h * 16 + d] = dof[d]; }
    __syncthreads();
    // phase 2: dk[j][c] += 0.25 * sum_r ds[r][h(c)][j] * q[r][c];  dv[j][c] += sum_r p[r][h(c)][j] * dout[r][c]
#pragma unroll
    for (int i = 0; i < 2 * MAXT * 128 / 256; ++i) {
      int o = threadIdx.x + i * 256;
      if (o < nout) {
        int which = o / (Tk * 128), jc = o % (Tk * 128), j = jc / 128, c = jc % 128, hh = c / 16;
        float a = 0.0f;
        if (which == 0) {
          for (int rr = 0; rr < 32; ++rr) a += sds[rr][hh][j] * sq[rr][c];
          a *= 0.25f;
        } else {
          for (int rr = 0; rr < 32; ++rr) a += spr[rr][hh][j] * sdo[rr][c];
        }
        accs[i] += a;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2 * MAXT * 128 / 256; ++i) {
    int o = threadIdx.x + i * 256;
    if (o < nout) part[((long long)blockIdx.x * P + p) * nout + o] = accs[i];
  }
}

}  // namespace

extern "C" int octsam_dec_tok_attn_fwd(const float* q, const float* k, const float* v, int32_t P, int32_t T, void* out,
                                       float* probs, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && probs && P > 0 && T > 0 && T <= MAXT, "octsam_dec_tok_attn_fwd: bad args");
  hipLaunchKernelGGL(tok_attn_fwd_kernel, dim3(P), dim3(256), 0, (hipStream_t)stream, q, k, v, T, (bf16*)out, probs);
  OCTSAM_LAUNCH_CHECK("octsam_dec_tok_attn_fwd");
  return 0;
}

extern "C" int octsam_dec_tok_attn_bwd(const float* q, const float* k, const float* v, const float* probs,
                                       const float* dout, int32_t P, int32_t T, void* dq, void* dk, void* dv,
                                       void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && probs && dout && dq && dk && dv && P > 0 && T > 0 && T <= MAXT,
                   "octsam_dec_tok_attn_bwd: bad args");
  hipLaunchKernelGGL(tok_attn_bwd_kernel, dim3(P), dim3(256), 0, (hipStream_t)stream, q, k, v, probs, dout, T,
                     (bf16*)dq, (bf16*)dk, (bf16*)dv);
  OCTSAM_LAUNCH_CHECK("octsam_dec_tok_attn_bwd");
  return 0;
}

extern "C" int octsam_dec_t2i_fwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                  int32_t Tq, int32_t L, void* out, float* lse, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && lse && P > 0 && Tq > 0 && Tq <= MAXT && L > 0 && kv_rep > 0 && ldkv % 8 == 0,
                   "octsam_dec_t2i_fwd: bad args");
  int nblk = ((P + 7) / 8) * 64;
  hipLaunchKernelGGL(t2i_fwd_kernel, dim3(nblk), dim3(Tq * 64), 0, (hipStream_t)stream, q, (const bf16*)k,
                     (const bf16*)v, ldkv, kv_rep, P, Tq, L, (bf16*)out, lse);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_fwd");
  return 0;
}

extern "C" int octsam_dec_t2i_bwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                  int32_t Tq, int32_t L, const void* out, const float* dout, const float* lse, void* dq,
                                  void* dk, void* dv, int64_t lddkv, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && dout && lse && dq && dk && dv && P > 0 && Tq > 0 && Tq <= MAXT && L > 0 &&
                       kv_rep > 0 && ldkv % 8 == 0 && lddkv % 8 == 0,
                   "octsam_dec_t2i_bwd: bad args");
  int nblk = ((P + 7) / 8) * 64;
  hipLaunchKernelGGL(t2i_bwd_kernel, dim3(nblk), dim3(256), 0, (hipStream_t)stream, q, (const bf16*)k, (const bf16*)v,
                     ldkv, kv_rep, P, Tq, L, (const bf16*)out, dout, lse, (bf16*)dq, (bf16*)dk, (bf16*)dv, lddkv);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd");
  return 0;
}

extern "C" int octsam_dec_i2t_fwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P,
                                  int32_t Tk, int32_t L, void* out, int64_t ldo, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && P > 0 && Tk > 0 && Tk <= MAXT && L > 0 && q_rep > 0 && ldq % 8 == 0 &&
                       ldo % 8 == 0,
                   "octsam_dec_i2t_fwd: bad args");
  dim3 grid((L + I2T_ROWS - 1) / I2T_ROWS, P);
  hipLaunchKernelGGL(i2t_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)q, ldq, q_rep, k, v, Tk, L,
                     (bf16*)out, ldo);
  OCTSAM_LAUNCH_CHECK("octsam_dec_i2t_fwd");
  return 0;
}

extern "C" int64_t octsam_dec_i2t_bwd_partials(int32_t P, int32_t Tk, int32_t L) {
  return (int64_t)((L + I2T_ROWS - 1) / I2T_ROWS) * P * 2 * Tk * 128;
}

extern "C" int octsam_dec_i2t_bwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P,
                                  int32_t Tk, int32_t L, const void* dout, int64_t lddo, void* dq, int64_t lddq,
                                  float* partials, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && dout && dq && partials && P > 0 && Tk > 0 && Tk <= MAXT && L > 0 && q_rep > 0 &&
                       ldq % 8 == 0 && lddo % 8 == 0 && lddq % 8 == 0,
                   "octsam_dec_i2t_bwd: bad args");
  dim3 grid((L + I2T_ROWS - 1) / I2T_ROWS, P);
  hipLaunchKernelGGL(i2t_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16*)q, ldq, q_rep, k, v, Tk, L,
                     (const bf16*)dout, lddo, (bf16*)dq, lddq, partials, P);
  OCTSAM_LAUNCH_CHECK("octsam_dec_i2t_bwd");
  return 0;
}
