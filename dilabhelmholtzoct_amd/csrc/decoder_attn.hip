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

typedef float f32x2_t __attribute__((ext_vector_type(2)));
namespace {
// Symmetric cross-lane reductions between lane and lane ^ 16 / lane ^ 32 by v_permlane16/32_swap of x with itself
// (each lane ends with {lower, upper} of its pair) instead of a ds_bpermute round trip.
__device__ __forceinline__ f32x2_t pair16(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return {__builtin_bit_cast(float, (uint32_t)r[0]), __builtin_bit_cast(float, (uint32_t)r[1])};
}
__device__ __forceinline__ f32x2_t pair32(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return {__builtin_bit_cast(float, (uint32_t)r[0]), __builtin_bit_cast(float, (uint32_t)r[1])};
}
__device__ __forceinline__ float max_xor16(float x) { const f32x2_t p = pair16(x); return fmaxf(p[0], p[1]); }
__device__ __forceinline__ float max_xor32(float x) { const f32x2_t p = pair32(x); return fmaxf(p[0], p[1]); }
__device__ __forceinline__ float add_xor16(float x) { const f32x2_t p = pair16(x); return p[0] + p[1]; }
__device__ __forceinline__ float add_xor32(float x) { const f32x2_t p = pair32(x); return p[0] + p[1]; }


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
// Token -> image attention: per prompt Tq <= 8 queries x 8 heads x 16 dims against L = 4096 keys,
// flash-decoding on MFMA. A workgroup = (prompt, 512-key chunk); wave w owns the head pair (2w, 2w+1).
// The pair's 64-B slices of the K and V rows stream into a wave-private LDS ring by LDS-DMA
// (global_load_lds, 32 keys per step, 3 steps in flight). One v_mfma_f32_16x16x32_bf16 per 16 keys
// gives the scores of BOTH heads: A = the K rows (32 dims = 2 heads), B = the queries block-diagonally
// (column n < 8: query n of head 2w with the other head's dims zero; n >= 8: query n-8 of head 2w+1),
// so the transposed score tile S^T[key][n] has one (query, head) per lane column and the online softmax
// is per lane (+ two xor-shuffles for the tile max). P^T (bf16) is the B operand of O^T += V^T P^T,
// V^T read with ds_read_b64_tr_b16. The queries are split hi + lo bf16 (two MFMAs), so scores keep
// ~16 mantissa bits. Per-chunk (m, l, O) partials are merged in fixed order by t2i_combine_kernel.
// Backward recomputes P from the forward's log-sum-exp in both orientations (S^T for dQ, S for dK/dV,
// each two MFMAs) so that every product takes its operands without a register transpose.
namespace t2 {
constexpr int CHUNK = 512, STEP = 32, RING = 4;
constexpr int STEP_BYTES = 2 * STEP * 64;    // K + V: 32 rows x 64 B each
constexpr int WAVE_LDS = RING * STEP_BYTES;  // 16 KiB per wave
constexpr int SMEM = 4 * WAVE_LDS;
constexpr int PART = 16 * 16 + 16 + 16;      // fwd: O[n][d], m[n], l[n] per (prompt, chunk, pair); bwd: dQ[n][d]
constexpr float L2E = 1.4426950408889634f;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 16-B chunk swizzles: K image (row reads) chunk ^ ((r>>2)&3); V image (transposed reads) chunk ^ 2((r>>2)&1)
__device__ __forceinline__ int ksw(int r, int c) { return c ^ ((r >> 2) & 3); }
__device__ __forceinline__ int vsw(int r, int c) { return c ^ (((r >> 2) & 1) << 1); }

// rows key0 .. key0+31 of the pair's K and V slices -> ring slot: 4 LDS-DMA instructions of 1 KiB
__device__ __forceinline__ void load_step(const bf16* kb, long long ldk, const bf16* vb, long long ldv, int key0,
                                          char* slot, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * i + (lane >> 2), pc = lane & 3;
    __builtin_amdgcn_global_load_lds((const void*)(kb + (long long)(key0 + r) * ldk + 8 * ksw(r, pc)),
                                     (lds_ptr_t)(slot + 1024 * i), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vb + (long long)(key0 + r) * ldv + 8 * vsw(r, pc)),
                                     (lds_ptr_t)(slot + 2048 + 1024 * i), 16, 0, 0);
  }
}

// rows of a 16-key tile as an MFMA row operand: lane (g, c) = row 16t + c, pair dims 8g .. 8g+7
__device__ __forceinline__ bf16x8 row_op(const char* img, int t, bool vimg, int lane) {
  const int r = 16 * t + (lane & 15), g = lane >> 4;
  return *(const bf16x8*)(img + 64 * r + 16 * (vimg ? vsw(r, g) : ksw(r, g)));
}
// transposed: element q of lane (g, c) = X[16t + 4g + q][dim 16 hl + c]
__device__ __forceinline__ s16x4 tr_op(const char* img, int t, int hl, bool vimg, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = 16 * t + 4 * g + q, lc = 2 * hl + (p >> 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(img + 64 * r + 16 * (vimg ? vsw(r, lc) : ksw(r, lc)) + 8 * (p & 1)));
}
// tr_op through inline asm. hipcc puts an s_waitcnt vmcnt(0) in front of the ds_read_tr builtin whenever an LDS-DMA
// may be in flight (it cannot tell the ring slot being loaded from the one read), which drained the K / V ring -- the
// next steps' loads -- at every step. The slot read here is never a DMA target while it is read (each loop's
// lgkmcnt(0) before it reissues a slot), so only the read itself is waited for: tr_wait before the values are used.
#ifndef DEC_TR_ASM
#define DEC_TR_ASM 1  // 0: the builtin (A/B builds)
#endif
__device__ __forceinline__ s16x4 tr_op_a(const char* img, int t, int hl, bool vimg, int lane) {
  if constexpr (!DEC_TR_ASM) return tr_op(img, t, hl, vimg, lane);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = 16 * t + 4 * g + q, lc = 2 * hl + (p >> 1);
  const char* a = img + 64 * r + 16 * (vimg ? vsw(r, lc) : ksw(r, lc)) + 8 * (p & 1);
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_ptr_t)(char*)a));
  return v;
}
__device__ __forceinline__ void tr_wait(s16x4& a, s16x4& b) {
  if constexpr (DEC_TR_ASM) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void tr_wait(s16x4& a, s16x4& b, s16x4& c, s16x4& d) {
  if constexpr (DEC_TR_ASM) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// Block-diagonal token operand (x fp32 [P, Tq, 128]): lane (g, c), element j = pair dim 8g + j of column
// n = c (n < 8: token n of head 2hp; n >= 8: token n-8 of head 2hp+1); zero off the diagonal / n >= Tq.
__device__ __forceinline__ void tok_op(const float* x, int p, int Tq, int hp, float scale, int lane, bf16x8& hi,
                                       bf16x8& lo) {
  const int g = lane >> 4, c = lane & 15, qi = c & 7;
  const bool on = (g >> 1) == (c >> 3) && qi < Tq;
  const float* src = x + ((long long)p * Tq + (on ? qi : 0)) * 128 + hp * 32 + 8 * g;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = on ? src[j] * scale : 0.0f;
    hi[j] = (bf16)v;
    lo[j] = (bf16)(v - (float)hi[j]);
  }
}

// 16x16x16 operand "X_h^T": lane (g, c), element j = x[token n = 4g+j (head 2hp+hl: n in [8hl, 8hl+8))][16h + c]
__device__ __forceinline__ s16x4 tokT_op(const float* x, int p, int Tq, int hp, int hl, float scale, int lane) {
  const int g = lane >> 4, c = lane & 15;
  s16x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 4 * g + j, qi = n & 7;
    const bool on = (n >> 3) == hl && qi < Tq;
    const float v = on ? x[((long long)p * Tq + qi) * 128 + (2 * hp + hl) * 16 + c] * scale : 0.0f;
    r[j] = __builtin_bit_cast(short, (bf16)v);
  }
  return r;
}
// tokT_op split hi + lo (x * scale = hi + lo to ~16 mantissa bits)
__device__ __forceinline__ void tokT_split(const float* x, int p, int Tq, int hp, int hl, float scale, int lane,
                                           s16x4& hi, s16x4& lo) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 4 * g + j, qi = n & 7;
    const bool on = (n >> 3) == hl && qi < Tq;
    const float v = on ? x[((long long)p * Tq + qi) * 128 + (2 * hp + hl) * 16 + c] * scale : 0.0f;
    const bf16 h = (bf16)v;
    hi[j] = __builtin_bit_cast(short, h);
    lo[j] = __builtin_bit_cast(short, (bf16)(v - (float)h));
  }
}

__device__ __forceinline__ s16x4 pack4(const f32x4& a) {
  s16x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __builtin_bit_cast(short, (bf16)a[i]);
  return r;
}
// a = hi + lo to ~16 mantissa bits, both as bf16 MFMA operands
__device__ __forceinline__ void split4(const f32x4& a, s16x4& hi, s16x4& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16 h = (bf16)a[i];
    hi[i] = __builtin_bit_cast(short, h);
    lo[i] = __builtin_bit_cast(short, (bf16)(a[i] - (float)h));
  }
}
__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(s16x4 a, s16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// s_waitcnt vmcnt(n) for a wave-uniform n in {0, 4, ..., 60}
__device__ __forceinline__ void wait_vm(int n) {
#define T2_W(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
  switch (n) {
    T2_W(0) T2_W(4) T2_W(8) T2_W(12) T2_W(16) T2_W(20) T2_W(24) T2_W(28) T2_W(32) T2_W(36) T2_W(40) T2_W(44)
    T2_W(48) T2_W(52) T2_W(56) default: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
  }
#undef T2_W
}
// wait_vm with the loop's steady-state count tested first (one compare instead of the switch's branch tree)
template <int FAST> __device__ __forceinline__ void wait_vm_f(int n) {
  if (n == FAST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FAST) : "memory");
  else wait_vm(n);
}
}  // namespace t2

// q fp32 [P,Tq,128]; k, v bf16 rows [(p / kv_rep) * L + key] * ldkv; part fp32 [P][nchunk][4][PART];
// sbias (or null): fp32 [P][L] added to every head's and token's logits of key (hf SamAttention's
// attention_similarity mask, natural-log units)
__global__ __launch_bounds__(256) void t2i_fwd_kernel(const float* __restrict__ q, const bf16* __restrict__ k,
                                                      const bf16* __restrict__ v, long long ldkv, int kv_rep, int Tq,
                                                      int L, int nchunk, float* __restrict__ part,
                                                      const float* __restrict__ sbias) {
  using namespace t2;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6;
  const int p = blockIdx.x / nchunk, chunk = blockIdx.x - p * nchunk;
  const int key0 = chunk * CHUNK;
  const int nstep = min(CHUNK, L - key0) / STEP;
  char* ring = tsm + hp * WAVE_LDS;
  const long long kvb = (long long)(p / kv_rep) * L;
  const bf16* kb = k + kvb * ldkv + hp * 32;
  const bf16* vb = v + kvb * ldkv + hp * 32;
  bf16x8 qhi, qlo;
  tok_op(q, p, Tq, hp, 0.25f * L2E, lane, qhi, qlo);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the loop's counted waits see only the ring's loads
  for (int s = 0; s < RING - 1 && s < nstep; ++s) load_step(kb, ldkv, vb, ldkv, key0 + s * STEP, ring + s * STEP_BYTES, lane);
  f32x4 o0 = (f32x4)0.0f, o1 = (f32x4)0.0f;
  float m = -INFINITY, l = 0.0f;
  for (int s = 0; s < nstep; ++s) {
    if (s + RING - 1 < nstep) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's previous reads are done
      load_step(kb, ldkv, vb, ldkv, key0 + (s + RING - 1) * STEP, ring + ((s + RING - 1) % RING) * STEP_BYTES, lane);
    }
    wait_vm_f<4 * (RING - 1)>(4 * min(RING - 1, nstep - 1 - s));
    const char* slot = ring + (s % RING) * STEP_BYTES;
    f32x4 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x8 kf = row_op(slot, t, false, lane);
      st[t] = mfma32(kf, qhi, (f32x4)0.0f);
      st[t] = mfma32(kf, qlo, st[t]);
    }
    if (sbias) {  // S^T[key 16t + 4g + i][token c] += bias[key] (log2 units like the scores)
      const float* bp = sbias + (long long)p * L + key0 + s * STEP + 4 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x4 bv = *(const f32x4*)(bp + 16 * t);
#pragma unroll
        for (int i = 0; i < 4; ++i) st[t][i] = fmaf(bv[i], L2E, st[t][i]);
      }
    }
    float mx = fmaxf(fmaxf(fmaxf(st[0][0], st[0][1]), fmaxf(st[0][2], st[0][3])),
                     fmaxf(fmaxf(st[1][0], st[1][1]), fmaxf(st[1][2], st[1][3])));
    mx = max_xor16(mx);
    mx = max_xor32(mx);
    const float mn = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    f32x4 e0, e1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      e0[i] = __builtin_amdgcn_exp2f(st[0][i] - mn);
      e1[i] = __builtin_amdgcn_exp2f(st[1][i] - mn);
    }
    l = fmaf(l, alpha, (e0[0] + e0[1]) + (e0[2] + e0[3]) + (e1[0] + e1[1]) + (e1[2] + e1[3]));
    o0 *= alpha;
    o1 *= alpha;
    // P split hi + lo as well: O feeds the backward's delta = dO . O = sum_k P_k dP_k, which must match the
    // backward's fp32 P to the cancellation in dP - delta (a bf16 P leaves O's error at 2^-9 of the deviations of
    // V from their P-weighted mean, which dQ = sum_k dS_k K_k then scales by |mean K| / spread of K)
    s16x4 h0, l0, h1, l1;
    split4(e0, h0, l0);
    split4(e1, h1, l1);
    const bf16x8 pf = cat8(h0, h1), pfl = cat8(l0, l1);
    const char* vimg = slot + 2048;
    s16x4 a0 = tr_op_a(vimg, 0, 0, true, lane), a1 = tr_op_a(vimg, 1, 0, true, lane);
    s16x4 a2 = tr_op_a(vimg, 0, 1, true, lane), a3 = tr_op_a(vimg, 1, 1, true, lane);
    tr_wait(a0, a1, a2, a3);
    const bf16x8 vt0 = cat8(a0, a1), vt1 = cat8(a2, a3);
    o0 = mfma32(vt0, pf, o0);
    o0 = mfma32(vt0, pfl, o0);
    o1 = mfma32(vt1, pf, o1);
    o1 = mfma32(vt1, pfl, o1);
  }
  l = add_xor16(l);
  l = add_xor32(l);
  float* w = part + (((long long)p * nchunk + chunk) * 4 + hp) * PART;
  const int c = lane & 15;
  *(f32x4*)(w + c * 16 + 4 * (lane >> 4)) = c < 8 ? o0 : o1;  // O^T[d = 4g+i][n = c] -> O[n][d]
  if (lane < 16) {
    w[256 + lane] = m;
    w[272 + lane] = l;
  }
}

// merge the chunk partials in chunk order: out bf16 [P,Tq,128], lse fp32 [P,8,Tq] (natural log)
__global__ void t2i_combine_kernel(const float* __restrict__ part, int nchunk, int Tq, bf16* __restrict__ out,
                                   float* __restrict__ lse, float* __restrict__ out_f32) {
  using namespace t2;
  const int p = blockIdx.x, t = threadIdx.x;
  const int d = t & 15, hq = t >> 4, h = hq / Tq, qi = hq - h * Tq;
  const int n = (h & 1) * 8 + qi;
  const float* w = part + ((long long)p * nchunk * 4 + (h >> 1)) * PART;
  float M = -INFINITY;
  for (int c = 0; c < nchunk; ++c) M = fmaxf(M, w[(long long)c * 4 * PART + 256 + n]);
  float Ls = 0.0f, O = 0.0f;
  for (int c = 0; c < nchunk; ++c) {
    const float* wc = w + (long long)c * 4 * PART;
    const float e = __builtin_amdgcn_exp2f(wc[256 + n] - M);
    Ls = fmaf(e, wc[272 + n], Ls);
    O = fmaf(e, wc[n * 16 + d], O);
  }
  out[((long long)p * Tq + qi) * 128 + h * 16 + d] = (bf16)(O / Ls);
  if (out_f32) out_f32[((long long)p * Tq + qi) * 128 + h * 16 + d] = O / Ls;  // (the backward's dO . O)
  if (d == 0) lse[((long long)p * 8 + h) * Tq + qi] = (M + __log2f(Ls)) / L2E;
}

// Backward. dout fp32 [P,Tq,128], out bf16 (forward output), lse [P,8,Tq]; writes per-prompt dk, dv bf16
// [P*L, lddkv] (head slice 16h) and dQ partials part[P][nchunk][4][256] (reduced by t2i_dq_kernel).
__global__ __launch_bounds__(256) void t2i_bwd_kernel(const float* __restrict__ q, const bf16* __restrict__ k,
                                                      const bf16* __restrict__ v, long long ldkv, int kv_rep, int Tq,
                                                      int L, int nchunk, const bf16* __restrict__ out,
                                                      const float* __restrict__ dout, const float* __restrict__ lse,
                                                      bf16* __restrict__ dk, bf16* __restrict__ dv, long long lddkv,
                                                      float* __restrict__ part, const float* __restrict__ out_f32) {
  using namespace t2;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int p = blockIdx.x / nchunk, chunk = blockIdx.x - p * nchunk;
  const int key0 = chunk * CHUNK;
  const int nstep = min(CHUNK, L - key0) / STEP;
  char* ring = tsm + hp * WAVE_LDS;
  const long long kvb = (long long)(p / kv_rep) * L;
  const bf16* kb = k + kvb * ldkv + hp * 32;
  const bf16* vb = v + kvb * ldkv + hp * 32;
  bf16x8 qhi, qlo, dop, dlo;
  tok_op(q, p, Tq, hp, 0.25f * L2E, lane, qhi, qlo);
  tok_op(dout, p, Tq, hp, 1.0f, lane, dop, dlo);
  s16x4 adO[2], aQ[2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    adO[hl] = tokT_op(dout, p, Tq, hp, hl, 1.0f, lane);
    aQ[hl] = tokT_op(q, p, Tq, hp, hl, 0.25f, lane);
  }
  // row constants of token n (log2-domain lse; delta = dO . O): column n = c (S^T) and rows n = 4g+i (S)
  auto tok_consts = [&](int n, float& l2, float& del) {
    const int qi = n & 7, h = 2 * hp + (n >> 3);
    if (qi >= Tq) {
      l2 = INFINITY;
      del = 0.0f;
      return;
    }
    l2 = lse[((long long)p * 8 + h) * Tq + qi] * L2E;
    const float* a = dout + ((long long)p * Tq + qi) * 128 + h * 16;
    float s = 0.0f;
    if (out_f32) {  // delta = dO . O with the forward's unrounded O (= sum_k P_k dP_k exactly, up to fp32)
      const float* b = out_f32 + ((long long)p * Tq + qi) * 128 + h * 16;
#pragma unroll
      for (int d = 0; d < 16; ++d) s = fmaf(a[d], b[d], s);
    } else {
      const bf16* b = out + ((long long)p * Tq + qi) * 128 + h * 16;
#pragma unroll
      for (int d = 0; d < 16; ++d) s = fmaf(a[d], (float)b[d], s);
    }
    del = s;
  };
  float lc2, dc;
  tok_consts(c, lc2, dc);
  float lr2[4], dr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) tok_consts(4 * g + i, lr2[i], dr[i]);
  f32x4 dq0 = (f32x4)0.0f, dq1 = (f32x4)0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the loop's counted waits see only the ring and its stores
  for (int s = 0; s < RING - 1 && s < nstep; ++s) load_step(kb, ldkv, vb, ldkv, key0 + s * STEP, ring + s * STEP_BYTES, lane);
  for (int s = 0; s < nstep; ++s) {
    if (s + RING - 1 < nstep) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      load_step(kb, ldkv, vb, ldkv, key0 + (s + RING - 1) * STEP, ring + ((s + RING - 1) % RING) * STEP_BYTES, lane);
    }
    // LDS-DMA loads and global stores share vmcnt; issued after step s's loads: the loads of steps
    // s+1 .. s+3 and the 8 stores of each of the steps max(0, s-3) .. s-1
    wait_vm_f<12 * (RING - 1)>(4 * min(RING - 1, nstep - 1 - s) + 8 * min(RING - 1, s));
    const char* slot = ring + (s % RING) * STEP_BYTES;
    const char* vimg = slot + 2048;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x8 kf = row_op(slot, t, false, lane), vf = row_op(vimg, t, true, lane);
      f32x4 sT = mfma32(kf, qhi, (f32x4)0.0f);
      sT = mfma32(kf, qlo, sT);                     // S^T[key 4g+i][n c]
      // dP = V . dO with dO split hi + lo too: dP - delta cancels to the softmax gradient's size, so dP needs the
      // same ~16 mantissa bits as the scores (a bf16 dO alone gave the q_proj gradient of the final token->image
      // attention 9 % error against fp32 autograd, 50x the bf16-operand floor; scripts/grad_diag.py)
      f32x4 dpT = mfma32(vf, dop, (f32x4)0.0f);
      dpT = mfma32(vf, dlo, dpT);
      f32x4 sS = mfma32(qhi, kf, (f32x4)0.0f);
      sS = mfma32(qlo, kf, sS);                     // S[n 4g+i][key c]
      f32x4 dpS = mfma32(dop, vf, (f32x4)0.0f);
      dpS = mfma32(dlo, vf, dpS);
      f32x4 dsT, pS, dsS;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dsT[i] = __builtin_amdgcn_exp2f(sT[i] - lc2) * (dpT[i] - dc);
        pS[i] = __builtin_amdgcn_exp2f(sS[i] - lr2[i]);
        dsS[i] = pS[i] * (dpS[i] - dr[i]);
      }
      const s16x4 pSb = pack4(pS), dsSb = pack4(dsS);
      s16x4 dsTb, dsTl;
      split4(dsT, dsTb, dsTl);
      const long long row = ((long long)p * L + key0 + s * STEP + 16 * t + c) * lddkv + 32 * hp + 4 * g;
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        const f32x4 dvt = mfma16(adO[hl], pSb, (f32x4)0.0f);  // dV^T[d 4g+i][key c]
        const f32x4 dkt = mfma16(aQ[hl], dsSb, (f32x4)0.0f);  // dK^T[d 4g+i][key c]
        *(s16x4*)(dv + row + 16 * hl) = pack4(dvt);
        *(s16x4*)(dk + row + 16 * hl) = pack4(dkt);
      }
      // dQ = dS . K summed over 4096 keys whose dS sum to zero: dS split hi + lo (bf16 dS alone leaves the sum's
      // rounding noise at the size of the result)
      s16x4 k0 = tr_op_a(slot, t, 0, false, lane), k1 = tr_op_a(slot, t, 1, false, lane);
      tr_wait(k0, k1);
      dq0 = mfma16(dsTb, k0, dq0);  // dQ[n 4g+i][d c] (head 2hp)
      dq0 = mfma16(dsTl, k0, dq0);
      dq1 = mfma16(dsTb, k1, dq1);  // (head 2hp+1)
      dq1 = mfma16(dsTl, k1, dq1);
    }
  }
  float* w = part + (((long long)p * nchunk + chunk) * 4 + hp) * 256;
  const f32x4 dqs = g < 2 ? dq0 : dq1;  // rows n < 8 belong to head 2hp, n >= 8 to head 2hp+1
#pragma unroll
  for (int i = 0; i < 4; ++i) w[(4 * g + i) * 16 + c] = dqs[i];
}

// Backward of the shared-K/V form (kv_rep > 1: layer 0's keys are the image embedding, shared by the image's kv_rep
// prompts, hf modeling_sam.py:499-501 repeat_interleave) with the prompt sum of dK / dV fused in: a workgroup =
// (image, 64-key chunk), wave = head pair; the chunk's K / V slices are staged in LDS once and the workgroup walks the
// image's prompts in order, accumulating dK^T / dV^T of its 64 keys in fp32 registers over the prompts (the per-prompt
// arithmetic of t2i_bwd_kernel), and stores them once per image -- the per-prompt [P*L, 2*CI] gradients and their
// prompt-sum pass never touch HBM. The next prompt's token operands load while the current prompt computes; its row
// statistics (log2 lse, dO . O) come precomputed from t2i_rowstats_kernel. dQ partials as in t2i_bwd_kernel.
namespace t2s {
constexpr int SCH = 64;                          // keys per workgroup chunk (2 steps)
constexpr int WAVE_LDS = 2 * t2::STEP_BYTES;     // 8 KiB per wave
constexpr int SMEM = 4 * WAVE_LDS;
}  // namespace t2s

// st fp32 [P][8][Tq][2] = (lse * log2(e), dO . O) per (prompt, head, token) (the bwd kernels' row constants)
__global__ void t2i_rowstats_kernel(const float* __restrict__ dout, const bf16* __restrict__ out,
                                    const float* __restrict__ lse, int Tq, float* __restrict__ st,
                                    const float* __restrict__ out_f32) {
  const int p = blockIdx.x, t = threadIdx.x;
  if (t >= 8 * Tq) return;
  const int h = t / Tq, qi = t - h * Tq;
  const float* a = dout + ((long long)p * Tq + qi) * 128 + h * 16;
  float s = 0.0f;
  if (out_f32) {  // the forward's unrounded O (t2i_bwd_kernel's tok_consts)
    const float* b = out_f32 + ((long long)p * Tq + qi) * 128 + h * 16;
#pragma unroll
    for (int d = 0; d < 16; ++d) s = fmaf(a[d], b[d], s);
  } else {
    const bf16* b = out + ((long long)p * Tq + qi) * 128 + h * 16;
#pragma unroll
    for (int d = 0; d < 16; ++d) s = fmaf(a[d], (float)b[d], s);
  }
  float* w = st + (((long long)p * 8 + h) * Tq + qi) * 2;
  w[0] = lse[((long long)p * 8 + h) * Tq + qi] * t2::L2E;
  w[1] = s;
}

__global__ __launch_bounds__(256) void t2i_bwd_sum_kernel(const float* __restrict__ q, const bf16* __restrict__ k,
                                                          const bf16* __restrict__ v, long long ldkv, int kv_rep,
                                                          int Tq, int L, int nchunk, const float* __restrict__ dout,
                                                          const float* __restrict__ st, bf16* __restrict__ dk,
                                                          bf16* __restrict__ dv, long long lddkv,
                                                          float* __restrict__ part) {
  using namespace t2;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int img = blockIdx.x / nchunk, chunk = blockIdx.x - img * nchunk;
  const int key0 = chunk * t2s::SCH;
  char* ring = tsm + hp * t2s::WAVE_LDS;
  const long long kvb = (long long)img * L;
  const bf16* kb = k + kvb * ldkv + hp * 32;
  const bf16* vb = v + kvb * ldkv + hp * 32;
  load_step(kb, ldkv, vb, ldkv, key0, ring, lane);
  load_step(kb, ldkv, vb, ldkv, key0 + STEP, ring + STEP_BYTES, lane);
  // token operands of one prompt, loaded raw (fp32) so the next prompt's loads overlap this prompt's products
  struct Raw {
    float qv[8], dv8[8], dT[2][4], qT[2][4], cs[2], rs[4][2];
  };
  auto load_raw = [&](int p, Raw& r) {
    const int qi = c & 7;
    const bool on = (g >> 1) == (c >> 3) && qi < Tq;
    const float* qs = q + ((long long)p * Tq + (on ? qi : 0)) * 128 + hp * 32 + 8 * g;
    const float* ds = dout + ((long long)p * Tq + (on ? qi : 0)) * 128 + hp * 32 + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r.qv[j] = on ? qs[j] : 0.0f;
      r.dv8[j] = on ? ds[j] : 0.0f;
    }
#pragma unroll
    for (int hl = 0; hl < 2; ++hl)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 4 * g + j, qj = n & 7;
        const bool o2 = (n >> 3) == hl && qj < Tq;
        const long long e = ((long long)p * Tq + (o2 ? qj : 0)) * 128 + (2 * hp + hl) * 16 + c;
        r.dT[hl][j] = o2 ? dout[e] : 0.0f;
        r.qT[hl][j] = o2 ? q[e] : 0.0f;
      }
    auto cst = [&](int n, float* o) {
      const int qn = n & 7, h = 2 * hp + (n >> 3);
      if (qn >= Tq) {
        o[0] = INFINITY;
        o[1] = 0.0f;
        return;
      }
      const float* w = st + (((long long)p * 8 + h) * Tq + qn) * 2;
      o[0] = w[0];
      o[1] = w[1];
    };
    cst(c, r.cs);
#pragma unroll
    for (int i = 0; i < 4; ++i) cst(4 * g + i, r.rs[i]);
  };
  f32x4 adk[2][2][2], adv[2][2][2];  // [step][16-key half][head of the pair]
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) adk[s2][t][hl] = adv[s2][t][hl] = (f32x4)0.0f;
  Raw cur, nxt;
  load_raw(img * kv_rep, cur);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the chunk's K / V slices (and the first prompt's operands)
  __builtin_amdgcn_wave_barrier();
  for (int pi = 0; pi < kv_rep; ++pi) {
    const int p = img * kv_rep + pi;
    if (pi + 1 < kv_rep) load_raw(p + 1, nxt);
    bf16x8 qhi, qlo, dop, dlo;
    const float qs = 0.25f * L2E;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v8 = cur.qv[j] * qs;
      qhi[j] = (bf16)v8;
      qlo[j] = (bf16)(v8 - (float)qhi[j]);
      dop[j] = (bf16)cur.dv8[j];
      dlo[j] = (bf16)(cur.dv8[j] - (float)dop[j]);
    }
    s16x4 adO[2], aQ[2];
#pragma unroll
    for (int hl = 0; hl < 2; ++hl)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        adO[hl][j] = __builtin_bit_cast(short, (bf16)cur.dT[hl][j]);
        aQ[hl][j] = __builtin_bit_cast(short, (bf16)(cur.qT[hl][j] * 0.25f));
      }
    const float lc2 = cur.cs[0], dc = cur.cs[1];
    f32x4 dq0 = (f32x4)0.0f, dq1 = (f32x4)0.0f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const char* slot = ring + s2 * STEP_BYTES;
      const char* vimg = slot + 2048;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8 kf = row_op(slot, t, false, lane), vf = row_op(vimg, t, true, lane);
        f32x4 sT = mfma32(kf, qhi, (f32x4)0.0f);
        sT = mfma32(kf, qlo, sT);
        f32x4 dpT = mfma32(vf, dop, (f32x4)0.0f);  // (dO hi + lo: t2i_bwd_kernel)
        dpT = mfma32(vf, dlo, dpT);
        f32x4 sS = mfma32(qhi, kf, (f32x4)0.0f);
        sS = mfma32(qlo, kf, sS);
        f32x4 dpS = mfma32(dop, vf, (f32x4)0.0f);
        dpS = mfma32(dlo, vf, dpS);
        f32x4 dsT, pS, dsS;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dsT[i] = __builtin_amdgcn_exp2f(sT[i] - lc2) * (dpT[i] - dc);
          pS[i] = __builtin_amdgcn_exp2f(sS[i] - cur.rs[i][0]);
          dsS[i] = pS[i] * (dpS[i] - cur.rs[i][1]);
        }
        const s16x4 pSb = pack4(pS), dsSb = pack4(dsS);
        s16x4 dsTb, dsTl;  // (dS hi + lo: t2i_bwd_kernel)
        split4(dsT, dsTb, dsTl);
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
          adv[s2][t][hl] = mfma16(adO[hl], pSb, adv[s2][t][hl]);
          adk[s2][t][hl] = mfma16(aQ[hl], dsSb, adk[s2][t][hl]);
        }
        s16x4 k0 = tr_op_a(slot, t, 0, false, lane), k1 = tr_op_a(slot, t, 1, false, lane);
        tr_wait(k0, k1);
        dq0 = mfma16(dsTb, k0, dq0);
        dq0 = mfma16(dsTl, k0, dq0);
        dq1 = mfma16(dsTb, k1, dq1);
        dq1 = mfma16(dsTl, k1, dq1);
      }
    }
    float* w = part + (((long long)p * nchunk + chunk) * 4 + hp) * 256;
    const f32x4 dqs = g < 2 ? dq0 : dq1;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[(4 * g + i) * 16 + c] = dqs[i];
    if (pi + 1 < kv_rep) cur = nxt;
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const long long row = (kvb + key0 + s2 * STEP + 16 * t + c) * lddkv + 32 * hp + 4 * g;
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        *(s16x4*)(dv + row + 16 * hl) = pack4(adv[s2][t][hl]);
        *(s16x4*)(dk + row + 16 * hl) = pack4(adk[s2][t][hl]);
      }
    }
}

// dq bf16 [P,Tq,128] = 0.25 * sum over chunks (in order) of the dQ partials
__global__ void t2i_dq_kernel(const float* __restrict__ part, int nchunk, int Tq, bf16* __restrict__ dq) {
  const int p = blockIdx.x, t = threadIdx.x;
  const int d = t & 15, hq = t >> 4, h = hq / Tq, qi = hq - h * Tq;
  const int n = (h & 1) * 8 + qi;
  const float* w = part + ((long long)p * nchunk * 4 + (h >> 1)) * 256 + n * 16 + d;
  float s = 0.0f;
  for (int c = 0; c < nchunk; ++c) s += w[(long long)c * 4 * 256];
  dq[((long long)p * Tq + qi) * 128 + h * 16 + d] = (bf16)(0.25f * s);
}

// ---------------------------------------------------------------------------------------- i2t
// Image -> token attention: L = 4096 image-row queries x Tk <= 8 token keys, 8 heads x 16. The t2i
// scheme with the roles swapped: a workgroup = (prompt, 512-row chunk), one wave per head pair; the token
// keys/values are constant block-diagonal operands, the image rows the streamed ones. The score tile is
// taken transposed, S^T[token n][row r] (softmax over a head's 8 token slots: in-lane + one xor-16
// shuffle), and O^T = V^T P^T. Backward also forms S[r][n] (two more MFMAs) for dK^T = Q^T dS and
// dV^T = dO^T P, whose Q^T / dO^T operands are ds_read_b64_tr_b16 reads of the rows staged by LDS-DMA;
// the per-row softmax statistics move from the S^T to the S layout by ds_bpermute. dK / dV partials per
// (chunk, prompt) are reduced in fixed order by octsam_splitk_reduce.
namespace i2 {
constexpr int CHUNK = 512;
}

// q bf16 rows [(p / q_rep) * L + r] * ldq; k, v fp32 [P, Tk, 128]; out bf16 [P*L, ldo]
__global__ __launch_bounds__(256) void i2t_fwd_kernel(const bf16* __restrict__ q, long long ldq, int q_rep,
                                                      const float* __restrict__ k, const float* __restrict__ v, int Tk,
                                                      int L, int nchunk, bf16* __restrict__ out, long long ldo) {
  using namespace t2;
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int p = blockIdx.x / nchunk, chunk = blockIdx.x - p * nchunk;
  const int r0 = chunk * i2::CHUNK;
  const int ntile = min(i2::CHUNK, L - r0) / 16;
  bf16x8 khi, klo;
  tok_op(k, p, Tk, hp, 0.25f * L2E, lane, khi, klo);  // [n = c][pair dim 8g+j]
  s16x4 av[2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) av[hl] = tokT_op(v, p, Tk, hp, hl, 1.0f, lane);  // V_h^T [d = c][n = 4g+j]
  bool nv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) nv[i] = ((4 * g + i) & 7) < Tk;
  const bf16* qb = q + ((long long)(p / q_rep) * L + r0) * ldq + hp * 32 + 8 * g;
  bf16* ob = out + ((long long)p * L + r0) * ldo + hp * 32 + 4 * g;
  bf16x8 qf = *(const bf16x8*)(qb + (long long)c * ldq);
  for (int t = 0; t < ntile; ++t) {
    bf16x8 qn = qf;
    if (t + 1 < ntile) qn = *(const bf16x8*)(qb + (long long)(16 * (t + 1) + c) * ldq);
    f32x4 s = mfma32(khi, qf, (f32x4)0.0f);
    s = mfma32(klo, qf, s);  // S^T[n 4g+i][r c]
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) mx = nv[i] ? fmaxf(mx, s[i]) : mx;
    mx = max_xor16(mx);
    f32x4 e;
    float sum = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      e[i] = nv[i] ? __builtin_amdgcn_exp2f(s[i] - mx) : 0.0f;
      sum += e[i];
    }
    sum = add_xor16(sum);
    e *= 1.0f / sum;
    const s16x4 pb = pack4(e);
#pragma unroll
    for (int hl = 0; hl < 2; ++hl)
      *(s16x4*)(ob + (long long)(16 * t + c) * ldo + 16 * hl) = pack4(mfma16(av[hl], pb, (f32x4)0.0f));
    qf = qn;
  }
}

// Backward. dout bf16 [P*L, lddo]; writes dq bf16 [P*L, lddq] and partials fp32 [nchunk][P][2][Tk][128]
// (dk; dv).
__global__ __launch_bounds__(256) void i2t_bwd_kernel(const bf16* __restrict__ q, long long ldq, int q_rep,
                                                      const float* __restrict__ k, const float* __restrict__ v, int Tk,
                                                      int L, int nchunk, const bf16* __restrict__ dout, long long lddo,
                                                      bf16* __restrict__ dq, long long lddq, float* __restrict__ part,
                                                      int P) {
  using namespace t2;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int p = blockIdx.x / nchunk, chunk = blockIdx.x - p * nchunk;
  const int r0 = chunk * i2::CHUNK;
  const int nstep = min(i2::CHUNK, L - r0) / STEP;
  char* ring = tsm + hp * WAVE_LDS;
  bf16x8 khi, klo, vop, vlo;
  tok_op(k, p, Tk, hp, 0.25f * L2E, lane, khi, klo);
  tok_op(v, p, Tk, hp, 1.0f, lane, vop, vlo);
  s16x4 ak[2], akl[2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    tokT_split(k, p, Tk, hp, hl, 0.25f, lane, ak[hl], akl[hl]);  // K_h^T / 4 [d = c][n = 4g+j]
  }
  bool nv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) nv[i] = ((4 * g + i) & 7) < Tk;
  const bool cv = (c & 7) < Tk;
  const bf16* qb = q + (long long)(p / q_rep) * L * ldq + hp * 32;
  const bf16* db = dout + (long long)p * L * lddo + hp * 32;
  f32x4 dka[2], dva[2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) dka[hl] = dva[hl] = (f32x4)0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int s = 0; s < RING - 1 && s < nstep; ++s) load_step(qb, ldq, db, lddo, r0 + s * STEP, ring + s * STEP_BYTES, lane);
  for (int s = 0; s < nstep; ++s) {
    if (s + RING - 1 < nstep) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      load_step(qb, ldq, db, lddo, r0 + (s + RING - 1) * STEP, ring + ((s + RING - 1) % RING) * STEP_BYTES, lane);
    }
    // loads of steps s+1 .. s+3 and the 4 dq stores of each of the steps max(0, s-3) .. s-1 follow step s's loads
    wait_vm_f<8 * (RING - 1)>(4 * min(RING - 1, nstep - 1 - s) + 4 * min(RING - 1, s));
    const char* slot = ring + (s % RING) * STEP_BYTES;
    const char* dimg = slot + 2048;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x8 qf = row_op(slot, t, false, lane), df = row_op(dimg, t, true, lane);
      // transposed orientation [n 4g+i][r c]: softmax statistics and dQ
      f32x4 sT = mfma32(khi, qf, (f32x4)0.0f);
      sT = mfma32(klo, qf, sT);
      // dP with V hi + lo, dQ = dS K with dS and K hi + lo: dP - delta and the sum over the <= 8 tokens (whose dS sum
      // to zero) cancel, so both carry ~16 mantissa bits (as in t2i_bwd_kernel)
      f32x4 dpT = mfma32(vop, df, (f32x4)0.0f);
      dpT = mfma32(vlo, df, dpT);
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = nv[i] ? fmaxf(mx, sT[i]) : mx;
      mx = max_xor16(mx);
      f32x4 pT;
      float sum = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pT[i] = nv[i] ? __builtin_amdgcn_exp2f(sT[i] - mx) : 0.0f;
        sum += pT[i];
      }
      sum = add_xor16(sum);
      const float inv = 1.0f / sum;
      float del = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pT[i] *= inv;
        del = fmaf(pT[i], dpT[i], del);
      }
      del = add_xor16(del);
      f32x4 dsT;
#pragma unroll
      for (int i = 0; i < 4; ++i) dsT[i] = pT[i] * (dpT[i] - del);
      s16x4 dsTb, dsTl;
      split4(dsT, dsTb, dsTl);
      bf16* dqr = dq + ((long long)p * L + r0 + s * STEP + 16 * t + c) * lddq + hp * 32 + 4 * g;
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        f32x4 a = mfma16(akl[hl], dsTb, (f32x4)0.0f);
        a = mfma16(ak[hl], dsTl, a);
        *(s16x4*)(dqr + 16 * hl) = pack4(mfma16(ak[hl], dsTb, a));
      }
      // untransposed [r 4g+i][n c] for dK / dV; row statistics from lane 32 h + r (h = head of column c)
      f32x4 sS = mfma32(qf, khi, (f32x4)0.0f);
      sS = mfma32(qf, klo, sS);
      f32x4 dpS = mfma32(df, vop, (f32x4)0.0f);
      dpS = mfma32(df, vlo, dpS);
      f32x4 pS, dsS;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int src = 32 * (c >> 3) + 4 * g + i;
        const float Mi = __shfl(mx, src, 64), Ii = __shfl(inv, src, 64), Di = __shfl(del, src, 64);
        pS[i] = cv ? __builtin_amdgcn_exp2f(sS[i] - Mi) * Ii : 0.0f;
        dsS[i] = pS[i] * (dpS[i] - Di);
      }
      const s16x4 pSb = pack4(pS), dsSb = pack4(dsS);
      s16x4 q0 = tr_op_a(slot, t, 0, false, lane), q1 = tr_op_a(slot, t, 1, false, lane);
      s16x4 o0 = tr_op_a(dimg, t, 0, true, lane), o1 = tr_op_a(dimg, t, 1, true, lane);
      tr_wait(q0, q1, o0, o1);
      dka[0] = mfma16(q0, dsSb, dka[0]);  // dK^T[d 4g+i][n c] (x4)
      dva[0] = mfma16(o0, pSb, dva[0]);   // dV^T[d 4g+i][n c]
      dka[1] = mfma16(q1, dsSb, dka[1]);
      dva[1] = mfma16(o1, pSb, dva[1]);
    }
  }
  if (cv) {
    const int hl = c >> 3, j = c & 7, h = 2 * hp + hl;
    float* w = part + (((long long)chunk * P + p) * 2) * Tk * 128 + j * 128 + h * 16 + 4 * g;
    *(f32x4*)w = (hl ? dka[1] : dka[0]) * 0.25f;
    *(f32x4*)(w + Tk * 128) = hl ? dva[1] : dva[0];
  }
}

// Backward of the shared-query form (q_rep > 1: the first block's image-side queries are the image embedding, shared
// by the image's q_rep prompts) with the prompt sum of dQ fused in: a workgroup = (image, 64-row chunk), wave = head
// pair; the chunk's query rows are staged once, each prompt's dO rows stream through a two-prompt LDS ring (the next
// prompt's rows and token operands load while the current prompt computes), dQ of the chunk accumulates over the
// prompts in fp32 registers and is stored once per image -- the per-prompt [P*L, CI] dQ and its prompt-sum pass never
// touch HBM. dK / dV partials per (chunk, prompt) as in i2t_bwd_kernel.
namespace i2s {
constexpr int SCH = 64;                                  // rows per workgroup chunk (2 steps)
constexpr int Q_BYTES = 2 * 2048, D_BYTES = 2 * 2048;    // query rows / one prompt's dO rows, 2 steps of 32 rows
constexpr int WAVE_LDS = Q_BYTES + 2 * D_BYTES;          // 12 KiB per wave
constexpr int SMEM = 4 * WAVE_LDS;
}  // namespace i2s

// 32 rows (r0 ..) of a head pair's 64-B slices -> a 2 KiB image (vimg: the V-image swizzle, else the K-image one)
__device__ __forceinline__ void load_rows32(const bf16* b, long long ld, int r0, char* dst, bool vimg, int lane) {
  using namespace t2;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * i + (lane >> 2), pc = lane & 3;
    __builtin_amdgcn_global_load_lds((const void*)(b + (long long)(r0 + r) * ld + 8 * (vimg ? vsw(r, pc) : ksw(r, pc))),
                                     (lds_ptr_t)(dst + 1024 * i), 16, 0, 0);
  }
}

__global__ __launch_bounds__(256) void i2t_bwd_sum_kernel(const bf16* __restrict__ q, long long ldq, int q_rep,
                                                          const float* __restrict__ k, const float* __restrict__ v,
                                                          int Tk, int L, int nchunk, const bf16* __restrict__ dout,
                                                          long long lddo, bf16* __restrict__ dq, long long lddq,
                                                          float* __restrict__ part, int P) {
  using namespace t2;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  const int lane = threadIdx.x & 63, hp = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int img = blockIdx.x / nchunk, chunk = blockIdx.x - img * nchunk;
  const int r0 = chunk * i2s::SCH;
  char* qimg = tsm + hp * i2s::WAVE_LDS;
  char* dring = qimg + i2s::Q_BYTES;
  const bf16* qb = q + (long long)img * L * ldq + hp * 32;
  const int p0 = img * q_rep;
  auto dbase = [&](int p) { return dout + (long long)p * L * lddo + hp * 32; };
  load_rows32(qb, ldq, r0, qimg, false, lane);
  load_rows32(qb, ldq, r0 + STEP, qimg + 2048, false, lane);
  load_rows32(dbase(p0), lddo, r0, dring, true, lane);
  load_rows32(dbase(p0), lddo, r0 + STEP, dring + 2048, true, lane);
  // token operands of one prompt, raw fp32 (tok_op / tokT_op's elements), so the next prompt's loads overlap
  struct Raw {
    float kv[8], vv[8], kT[2][4];
  };
  auto load_raw = [&](int p, Raw& r) {
    const int qi = c & 7;
    const bool on = (g >> 1) == (c >> 3) && qi < Tk;
    const float* ks = k + ((long long)p * Tk + (on ? qi : 0)) * 128 + hp * 32 + 8 * g;
    const float* vs = v + ((long long)p * Tk + (on ? qi : 0)) * 128 + hp * 32 + 8 * g;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r.kv[j] = on ? ks[j] : 0.0f;
      r.vv[j] = on ? vs[j] : 0.0f;
    }
#pragma unroll
    for (int hl = 0; hl < 2; ++hl)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 4 * g + j, qj = n & 7;
        const bool o2 = (n >> 3) == hl && qj < Tk;
        r.kT[hl][j] = o2 ? k[((long long)p * Tk + qj) * 128 + (2 * hp + hl) * 16 + c] : 0.0f;
      }
  };
  bool nv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) nv[i] = ((4 * g + i) & 7) < Tk;
  const bool cv = (c & 7) < Tk;
  f32x4 adq[2][2][2];  // [step][16-row half][head of the pair]
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) adq[s2][t][hl] = (f32x4)0.0f;
  Raw cur, nxt;
  load_raw(p0, cur);
  for (int pi = 0; pi < q_rep; ++pi) {
    const int p = p0 + pi;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // this prompt's rows (and operands) landed
    __builtin_amdgcn_wave_barrier();
    if (pi + 1 < q_rep) {  // the next prompt's dO rows into the other buffer (read two iterations ago), its operands
      char* nb = dring + ((pi + 1) & 1) * i2s::D_BYTES;
      load_rows32(dbase(p + 1), lddo, r0, nb, true, lane);
      load_rows32(dbase(p + 1), lddo, r0 + STEP, nb + 2048, true, lane);
      load_raw(p + 1, nxt);
    }
    bf16x8 khi, klo, vop, vlo;
    const float ks = 0.25f * L2E;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = cur.kv[j] * ks;
      khi[j] = (bf16)x;
      klo[j] = (bf16)(x - (float)khi[j]);
      vop[j] = (bf16)cur.vv[j];
      vlo[j] = (bf16)(cur.vv[j] - (float)vop[j]);
    }
    s16x4 ak[2], akl[2];
#pragma unroll
    for (int hl = 0; hl < 2; ++hl)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = cur.kT[hl][j] * 0.25f;
        const bf16 hi = (bf16)x;
        ak[hl][j] = __builtin_bit_cast(short, hi);
        akl[hl][j] = __builtin_bit_cast(short, (bf16)(x - (float)hi));
      }
    f32x4 dka[2], dva[2];
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) dka[hl] = dva[hl] = (f32x4)0.0f;
    const char* dcur = dring + (pi & 1) * i2s::D_BYTES;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const char* slot = qimg + s2 * 2048;
      const char* dimg = dcur + s2 * 2048;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8 qf = row_op(slot, t, false, lane), df = row_op(dimg, t, true, lane);
        f32x4 sT = mfma32(khi, qf, (f32x4)0.0f);
        sT = mfma32(klo, qf, sT);
        f32x4 dpT = mfma32(vop, df, (f32x4)0.0f);  // (V, dS and K hi + lo: i2t_bwd_kernel)
        dpT = mfma32(vlo, df, dpT);
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = nv[i] ? fmaxf(mx, sT[i]) : mx;
        mx = max_xor16(mx);
        f32x4 pT;
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pT[i] = nv[i] ? __builtin_amdgcn_exp2f(sT[i] - mx) : 0.0f;
          sum += pT[i];
        }
        sum = add_xor16(sum);
        const float inv = 1.0f / sum;
        float del = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pT[i] *= inv;
          del = fmaf(pT[i], dpT[i], del);
        }
        del = add_xor16(del);
        f32x4 dsT;
#pragma unroll
        for (int i = 0; i < 4; ++i) dsT[i] = pT[i] * (dpT[i] - del);
        s16x4 dsTb, dsTl;
        split4(dsT, dsTb, dsTl);
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
          adq[s2][t][hl] = mfma16(akl[hl], dsTb, adq[s2][t][hl]);
          adq[s2][t][hl] = mfma16(ak[hl], dsTl, adq[s2][t][hl]);
          adq[s2][t][hl] = mfma16(ak[hl], dsTb, adq[s2][t][hl]);
        }
        f32x4 sS = mfma32(qf, khi, (f32x4)0.0f);
        sS = mfma32(qf, klo, sS);
        f32x4 dpS = mfma32(df, vop, (f32x4)0.0f);
        dpS = mfma32(df, vlo, dpS);
        f32x4 pS, dsS;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int src = 32 * (c >> 3) + 4 * g + i;
          const float Mi = __shfl(mx, src, 64), Ii = __shfl(inv, src, 64), Di = __shfl(del, src, 64);
          pS[i] = cv ? __builtin_amdgcn_exp2f(sS[i] - Mi) * Ii : 0.0f;
          dsS[i] = pS[i] * (dpS[i] - Di);
        }
        const s16x4 pSb = pack4(pS), dsSb = pack4(dsS);
        s16x4 q0 = tr_op_a(slot, t, 0, false, lane), q1 = tr_op_a(slot, t, 1, false, lane);
        s16x4 o0 = tr_op_a(dimg, t, 0, true, lane), o1 = tr_op_a(dimg, t, 1, true, lane);
        tr_wait(q0, q1, o0, o1);
        dka[0] = mfma16(q0, dsSb, dka[0]);
        dva[0] = mfma16(o0, pSb, dva[0]);
        dka[1] = mfma16(q1, dsSb, dka[1]);
        dva[1] = mfma16(o1, pSb, dva[1]);
      }
    }
    if (cv) {
      const int hl = c >> 3, j = c & 7, h = 2 * hp + hl;
      float* w = part + (((long long)chunk * P + p) * 2) * Tk * 128 + j * 128 + h * 16 + 4 * g;
      *(f32x4*)w = (hl ? dka[1] : dka[0]) * 0.25f;
      *(f32x4*)(w + Tk * 128) = hl ? dva[1] : dva[0];
    }
    if (pi + 1 < q_rep) cur = nxt;
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16* dqr = dq + ((long long)img * L + r0 + s2 * STEP + 16 * t + c) * lddq + hp * 32 + 4 * g;
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) *(s16x4*)(dqr + 16 * hl) = pack4(adq[s2][t][hl]);
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

static int t2i_nchunk(int L) { return (L + t2::CHUNK - 1) / t2::CHUNK; }

extern "C" int64_t octsam_dec_t2i_workspace(int32_t P, int32_t L) {
  return (int64_t)P * t2i_nchunk(L) * 4 * t2::PART;
}

static void t2i_smem_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)t2i_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, t2::SMEM);
    (void)hipFuncSetAttribute((const void*)t2i_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, t2::SMEM);
    done = true;
  }
}

// out_f32 (optional, fp32 [P, Tq, 128]): the unrounded O as well, for the backward's delta = dO . O
extern "C" int octsam_dec_t2i_fwd2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                   int32_t Tq, int32_t L, const float* score_bias, void* out, float* out_f32, float* lse,
                                   float* workspace, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && lse && workspace && P > 0 && Tq > 0 && Tq <= MAXT && L > 0 && L % 32 == 0 &&
                       kv_rep > 0 && P % kv_rep == 0 && ldkv % 8 == 0 && (uintptr_t)k % 16 == 0 &&
                       (uintptr_t)v % 16 == 0 && (uintptr_t)score_bias % 16 == 0,
                   "octsam_dec_t2i_fwd: bad args");
  t2i_smem_attr();
  const int nch = t2i_nchunk(L);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(t2i_fwd_kernel, dim3(P * nch), dim3(256), t2::SMEM, s, q, (const bf16*)k, (const bf16*)v, ldkv,
                     kv_rep, Tq, L, nch, workspace, score_bias);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_fwd");
  hipLaunchKernelGGL(t2i_combine_kernel, dim3(P), dim3(8 * Tq * 16), 0, s, workspace, nch, Tq, (bf16*)out, lse,
                     out_f32);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_fwd");
  return 0;
}

extern "C" int octsam_dec_t2i_fwd_bias(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep,
                                       int32_t P, int32_t Tq, int32_t L, const float* score_bias, void* out, float* lse,
                                       float* workspace, void* stream) {
  return octsam_dec_t2i_fwd2(q, k, v, ldkv, kv_rep, P, Tq, L, score_bias, out, nullptr, lse, workspace, stream);
}

extern "C" int octsam_dec_t2i_fwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                  int32_t Tq, int32_t L, void* out, float* lse, float* workspace, void* stream) {
  return octsam_dec_t2i_fwd_bias(q, k, v, ldkv, kv_rep, P, Tq, L, nullptr, out, lse, workspace, stream);
}

// out_f32: the forward's fp32 O (octsam_dec_t2i_fwd2) for delta, or null (delta from the bf16 out)
extern "C" int octsam_dec_t2i_bwd2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                   int32_t Tq, int32_t L, const void* out, const float* out_f32, const float* dout,
                                   const float* lse, void* dq, void* dk, void* dv, int64_t lddkv, float* workspace,
                                   void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && dout && lse && dq && dk && dv && workspace && P > 0 && Tq > 0 &&
                       Tq <= MAXT && L > 0 && L % 32 == 0 && kv_rep > 0 && P % kv_rep == 0 && ldkv % 8 == 0 &&
                       lddkv % 4 == 0 && (uintptr_t)k % 16 == 0 && (uintptr_t)v % 16 == 0 &&
                       (uintptr_t)dk % 8 == 0 && (uintptr_t)dv % 8 == 0,
                   "octsam_dec_t2i_bwd: bad args");
  t2i_smem_attr();
  const int nch = t2i_nchunk(L);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(t2i_bwd_kernel, dim3(P * nch), dim3(256), t2::SMEM, s, q, (const bf16*)k, (const bf16*)v, ldkv,
                     kv_rep, Tq, L, nch, (const bf16*)out, dout, lse, (bf16*)dk, (bf16*)dv, lddkv, workspace, out_f32);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd");
  hipLaunchKernelGGL(t2i_dq_kernel, dim3(P), dim3(8 * Tq * 16), 0, s, workspace, nch, Tq, (bf16*)dq);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd");
  return 0;
}

extern "C" int octsam_dec_t2i_bwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                                  int32_t Tq, int32_t L, const void* out, const float* dout, const float* lse, void* dq,
                                  void* dk, void* dv, int64_t lddkv, float* workspace, void* stream) {
  return octsam_dec_t2i_bwd2(q, k, v, ldkv, kv_rep, P, Tq, L, out, nullptr, dout, lse, dq, dk, dv, lddkv, workspace,
                             stream);
}

// the shared-K/V backward with the prompt sum fused in (t2i_bwd_sum_kernel): dk / dv are the IMAGE rows
// [(P / kv_rep) * L, lddkv]; workspace: octsam_dec_t2i_bwd_sum_workspace(P, Tq, L) floats
extern "C" int64_t octsam_dec_t2i_bwd_sum_workspace(int32_t P, int32_t Tq, int32_t L) {
  return (int64_t)P * (L / t2s::SCH) * 4 * 256 + (int64_t)P * 8 * Tq * 2;
}

extern "C" int octsam_dec_t2i_bwd_sum2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep,
                                       int32_t P, int32_t Tq, int32_t L, const void* out, const float* out_f32,
                                       const float* dout, const float* lse, void* dq, void* dk, void* dv, int64_t lddkv,
                                       float* workspace, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && dout && lse && dq && dk && dv && workspace && P > 0 && Tq > 0 &&
                       Tq <= MAXT && L > 0 && L % t2s::SCH == 0 && kv_rep > 0 && P % kv_rep == 0 && ldkv % 8 == 0 &&
                       lddkv % 4 == 0 && (uintptr_t)k % 16 == 0 && (uintptr_t)v % 16 == 0 &&
                       (uintptr_t)dk % 8 == 0 && (uintptr_t)dv % 8 == 0,
                   "octsam_dec_t2i_bwd_sum: bad args");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)t2i_bwd_sum_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, t2s::SMEM);
    attr = true;
  }
  const int nch = L / t2s::SCH, nimg = P / kv_rep;
  float* part = workspace;
  float* st = workspace + (int64_t)P * nch * 4 * 256;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(t2i_rowstats_kernel, dim3(P), dim3(64), 0, s, dout, (const bf16*)out, lse, Tq, st, out_f32);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd_sum");
  hipLaunchKernelGGL(t2i_bwd_sum_kernel, dim3(nimg * nch), dim3(256), t2s::SMEM, s, q, (const bf16*)k, (const bf16*)v,
                     ldkv, kv_rep, Tq, L, nch, dout, st, (bf16*)dk, (bf16*)dv, lddkv, part);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd_sum");
  hipLaunchKernelGGL(t2i_dq_kernel, dim3(P), dim3(8 * Tq * 16), 0, s, part, nch, Tq, (bf16*)dq);
  OCTSAM_LAUNCH_CHECK("octsam_dec_t2i_bwd_sum");
  return 0;
}

extern "C" int octsam_dec_t2i_bwd_sum(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep,
                                      int32_t P, int32_t Tq, int32_t L, const void* out, const float* dout,
                                      const float* lse, void* dq, void* dk, void* dv, int64_t lddkv, float* workspace,
                                      void* stream) {
  return octsam_dec_t2i_bwd_sum2(q, k, v, ldkv, kv_rep, P, Tq, L, out, nullptr, dout, lse, dq, dk, dv, lddkv, workspace,
                                 stream);
}

static int i2t_nchunk(int L) { return (L + i2::CHUNK - 1) / i2::CHUNK; }

extern "C" int octsam_dec_i2t_fwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P,
                                  int32_t Tk, int32_t L, void* out, int64_t ldo, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && out && P > 0 && Tk > 0 && Tk <= MAXT && L > 0 && L % 16 == 0 && q_rep > 0 &&
                       P % q_rep == 0 && ldq % 8 == 0 && ldo % 4 == 0 && (uintptr_t)q % 16 == 0 &&
                       (uintptr_t)out % 8 == 0,
                   "octsam_dec_i2t_fwd: bad args");
  const int nch = i2t_nchunk(L);
  hipLaunchKernelGGL(i2t_fwd_kernel, dim3(P * nch), dim3(256), 0, (hipStream_t)stream, (const bf16*)q, ldq, q_rep, k, v,
                     Tk, L, nch, (bf16*)out, ldo);
  OCTSAM_LAUNCH_CHECK("octsam_dec_i2t_fwd");
  return 0;
}

extern "C" int64_t octsam_dec_i2t_bwd_partials(int32_t P, int32_t Tk, int32_t L) {
  return (int64_t)i2t_nchunk(L) * P * 2 * Tk * 128;
}

extern "C" int octsam_dec_i2t_bwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P,
                                  int32_t Tk, int32_t L, const void* dout, int64_t lddo, void* dq, int64_t lddq,
                                  float* partials, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && dout && dq && partials && P > 0 && Tk > 0 && Tk <= MAXT && L > 0 && L % 32 == 0 &&
                       q_rep > 0 && P % q_rep == 0 && ldq % 8 == 0 && lddo % 8 == 0 && lddq % 4 == 0 &&
                       (uintptr_t)q % 16 == 0 && (uintptr_t)dout % 16 == 0 && (uintptr_t)dq % 8 == 0,
                   "octsam_dec_i2t_bwd: bad args");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)i2t_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, t2::SMEM);
    attr = true;
  }
  const int nch = i2t_nchunk(L);
  hipLaunchKernelGGL(i2t_bwd_kernel, dim3(P * nch), dim3(256), t2::SMEM, (hipStream_t)stream, (const bf16*)q, ldq,
                     q_rep, k, v, Tk, L, nch, (const bf16*)dout, lddo, (bf16*)dq, lddq, partials, P);
  OCTSAM_LAUNCH_CHECK("octsam_dec_i2t_bwd");
  return 0;
}

// the shared-query backward with the prompt sum of dQ fused in (i2t_bwd_sum_kernel): dq holds the IMAGE rows
// [(P / q_rep) * L, lddq]; dK / dV partials: octsam_dec_i2t_bwd_sum_partials(P, Tk, L) floats, reduced by the caller
extern "C" int64_t octsam_dec_i2t_bwd_sum_partials(int32_t P, int32_t Tk, int32_t L) {
  return (int64_t)(L / i2s::SCH) * P * 2 * Tk * 128;
}

extern "C" int octsam_dec_i2t_bwd_sum(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v,
                                      int32_t P, int32_t Tk, int32_t L, const void* dout, int64_t lddo, void* dq,
                                      int64_t lddq, float* partials, void* stream) {
  OCTSAM_CHECK_ARG(q && k && v && dout && dq && partials && P > 0 && Tk > 0 && Tk <= MAXT && L > 0 &&
                       L % i2s::SCH == 0 && q_rep > 0 && P % q_rep == 0 && ldq % 8 == 0 && lddo % 8 == 0 &&
                       lddq % 4 == 0 && (uintptr_t)q % 16 == 0 && (uintptr_t)dout % 16 == 0 && (uintptr_t)dq % 8 == 0,
                   "octsam_dec_i2t_bwd_sum: bad args");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)i2t_bwd_sum_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, i2s::SMEM);
    attr = true;
  }
  const int nch = L / i2s::SCH, nimg = P / q_rep;
  hipLaunchKernelGGL(i2t_bwd_sum_kernel, dim3(nimg * nch), dim3(256), i2s::SMEM, (hipStream_t)stream, (const bf16*)q,
                     ldq, q_rep, k, v, Tk, L, nch, (const bf16*)dout, lddo, (bf16*)dq, lddq, partials, P);
  OCTSAM_LAUNCH_CHECK("octsam_dec_i2t_bwd_sum");
  return 0;
}
