// MFMA e16 GEMM for gfx950 with fused epilogues and implicit-GEMM operand loaders.
//
//   C[b][m][n] = epi( alpha * sum_k A[b][m][k] * B[b][n][k] )          (fp32 accumulate)
//
// A operand modes (template AM):
//   0  row-major  A[m*lda + k]                     (Linear input, K contiguous)
//   1  transposed A[k*lda + m]                     (dY^T for weight gradients)
//   2  patch16    A from fp32 NCHW pixels          (SamPatchEmbeddings conv 16x16/s16 as im2col,
//                                                   hf modeling_sam.py:116-129)
//   3  conv3x3    A from e16 NHWC 64x64 map, k = (ky*3+kx)*C + c, zero padding 1
//                                                  (SamVisionNeck.conv2, modeling_sam.py:985-992)
//   4  row-major plus a row-periodic addend A2[(m % a2_rows)*lda + k]   (keys + key_pe,
//                                                  SamTwoWayAttentionBlock, modeling_sam.py:327-343)
// B operand modes (template BMODE):
//   0  B[n*ldb + k]   (nn.Linear weight [out,in])
//   1  B[k*ldb + n]   (weight used transposed, activations for dW)
//   2  like 1 plus B2[(k % b2_rows)*ldb + n]       (dW of a product whose input was keys + key_pe)
//
// Epilogue (runtime): v = alpha*acc (+ beta*C_old) (+ bias[n]) -> act -> (+ residual) ; optional
// pre-activation store; optional output row remap (window unpartition: drop padded tokens).
//
// Tiling: 128x128x64 block tile, 4 waves (2x2), each wave 64x64 via 2x2 v_mfma_f32_32x32x16_bf16.
// LDS image [row][64] e16 with the 16-byte chunk index XOR-swizzled by ((row>>1)&7) so that the
// ds_read_b128 lane groups of the 32x32x16 fragment reads are conflict-free.
// Register-staged double buffer, one barrier per K-step; XCD-aware block remap so that the tiles
// of one A row-panel run on one XCD (shared L2).
#include "common.h"
#include <cstdio>
#include <cstdlib>
#include "../../include/octsam.h"

// 16-bit operand type of this build: bf16 (octsam_gemm) or IEEE half (built again with OCTSAM_GEMM_F16:
// octsam_gemm_f16, the fp16 encoder of BASELINE configs[4]). The two MFMA shapes and the epilogue's
// 16-bit <-> fp32 conversions are the only type-dependent operations; data movement is byte-agnostic.
#ifdef OCTSAM_GEMM_F16
typedef _Float16 e16;
typedef _Float16 e16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 e16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 e16x2 __attribute__((ext_vector_type(2)));
#define OCTSAM_GEMM_ENTRY octsam_gemm_f16
#else
typedef bf16 e16;
typedef bf16x8 e16x8;
typedef bf16x4 e16x4;
typedef bf16x2 e16x2;
#define OCTSAM_GEMM_ENTRY octsam_gemm
#endif

namespace {
__device__ __forceinline__ f32x16 mma32(e16x8 a, e16x8 b, f32x16 c, int, int, int) {
#ifdef OCTSAM_GEMM_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}
__device__ __forceinline__ f32x4 mma16(e16x8 a, e16x8 b, f32x4 c, int, int, int) {
#ifdef OCTSAM_GEMM_F16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}
// low / high 16-bit element of a packed pair as fp32
__device__ __forceinline__ float lo16f(uint32_t r) {
#ifdef OCTSAM_GEMM_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(r & 0xffffu));
#else
  return __builtin_bit_cast(float, r << 16);
#endif
}
__device__ __forceinline__ float hi16f(uint32_t r) {
#ifdef OCTSAM_GEMM_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(r >> 16));
#else
  return __builtin_bit_cast(float, r & 0xffff0000u);
#endif
}
}  // namespace

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;

struct GemmK {
  const void* A;
  const void* B;
  void* C;
  const float* bias;
  const void* R;
  void* Cpre;
  const int* row_map;
  const void* A2;
  const void* B2;
  int a2_rows, b2_rows;
  int a_blk, a_rep, b_blk, b_rep, r_blk, r_rep;
  int M, N, K;
  long long lda, ldb, ldc, ldr;
  long long sA, sB, sC, sR;
  float alpha, beta;
  int act;
  int c_f32, r_f32, pre_f32;
  int conv_c;  // channels for conv3x3 mode
  int tiles_m, tiles_n;
  int k_total;  // split-K over k-major operands: rows >= k_total (counted from batch 0) read as zero
  int fast_epi;  // 8-phase kernels: lean epilogue kind (0 = general; else 1 + FE bits, see epilogue_fast)
  int c_rows;    // rows of C (and R) when a row map scatters the output (fast epilogue range)
  float* a_cs;   // k-major operands: per-batch column sums of A [batch][M] / B [batch][N] (or null)
  float* b_cs;
  int rgroup;    // broadcast-residual tile order (rgroup_tm); 0 = plain order
  int res_lds;   // gemm8 in-place fp32 residual kind: residual through LDS (ph8::epilogue_res_lds)
};

// repeat_interleave row remap: logical row -> stored row = (row / (blk*rep)) * blk + row % blk
__device__ __forceinline__ long long remap(int row, int blk, int rep) {
  return blk > 0 ? (long long)(row / (blk * rep)) * blk + row % blk : (long long)row;
}

// Row-tile order for a row-remapped broadcast residual (r_blk % 256 == 0, rgroup set): the 256-row tiles that
// read the same residual rows (same row % r_blk inside one r_blk * r_rep group — the decoder's per-prompt tiles at
// one positional block) get consecutive logical ids, so the tiles in flight on an XCD share one residual block in
// L2 instead of re-fetching the whole period per prompt.
__device__ __forceinline__ int rgroup_tm(const GemmK& p, int tm) {
  if (!p.rgroup) return tm;
  const int nb = p.r_blk >> 8, gsz = nb * p.r_rep;
  const int g = tm / gsz, j = tm - g * gsz;
  return g * gsz + (j % p.r_rep) * nb + j / p.r_rep;
}

__device__ __forceinline__ int lds_idx(int r, int c) {  // e16 element index in a [rows][64] image
  return r * BK + ((c ^ ((r >> 1) & 7)) << 3);
}

__device__ __forceinline__ e16x8 cvt8(const float4 a, const float4 b) {
  e16x8 r;
  r[0] = (e16)a.x; r[1] = (e16)a.y; r[2] = (e16)a.z; r[3] = (e16)a.w;
  r[4] = (e16)b.x; r[5] = (e16)b.y; r[6] = (e16)b.z; r[7] = (e16)b.w;
  return r;
}

// Stage: each thread holds R/32 chunks of 8 e16 for the operand tile (R rows x 64 k).
template <int MODE, int R = 128>
struct Loader {
  static constexpr int NC = R / 32;  // chunks per thread
  static constexpr int RC = R / 8;   // 8-row chunks per k row (transposed modes)
  e16x8 v[NC];

  __device__ __forceinline__ void load(const GemmK& p, const void* base, const void* add, int period,
                                       long long ld, int rows, int row0, int k0, int tid, int blk, int rep,
                                       int kcap) {
    if constexpr (MODE == 4) {
      const e16* src = (const e16*)base;
      const e16* ad = (const e16*)add;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int r = ci >> 3, c = ci & 7;
        int gr = row0 + r, gk = k0 + c * 8;
        if (gr < rows && gk < p.K) {
          e16x8 x = *(const e16x8*)(src + remap(gr, blk, rep) * ld + gk);
          e16x8 y = *(const e16x8*)(ad + (long long)(gr % period) * ld + gk);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = (e16)((float)x[e] + (float)y[e]);
          v[i] = x;
        } else {
          v[i] = (e16x8)(e16)0.0f;
        }
      }
    } else if constexpr (MODE == 5) {  // B mode 2: transposed plus k-periodic addend
      const e16* src = (const e16*)base;
      const e16* ad = (const e16*)add;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int k = ci / RC, rc = ci % RC;
        int gr = row0 + rc * 8, gk = k0 + k;
        if (gr < rows && gk < p.K) {
          e16x8 x = *(const e16x8*)(src + remap(gk, blk, rep) * ld + gr);
          e16x8 y = *(const e16x8*)(ad + (long long)(gk % period) * ld + gr);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = (e16)((float)x[e] + (float)y[e]);
          v[i] = x;
        } else {
          v[i] = (e16x8)(e16)0.0f;
        }
      }
    } else if constexpr (MODE == 0) {
      const e16* src = (const e16*)base;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int r = ci >> 3, c = ci & 7;
        int gr = row0 + r, gk = k0 + c * 8;
        if (gr < rows && gk < p.K)
          v[i] = *(const e16x8*)(src + remap(gr, blk, rep) * ld + gk);
        else
          v[i] = (e16x8)(e16)0.0f;
      }
    } else if constexpr (MODE == 1) {
      const e16* src = (const e16*)base;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int k = ci / RC, rc = ci % RC;
        int gr = row0 + rc * 8, gk = k0 + k;
        if (gr < rows && gk < kcap)
          v[i] = *(const e16x8*)(src + remap(gk, blk, rep) * ld + gr);
        else
          v[i] = (e16x8)(e16)0.0f;
      }
    } else if constexpr (MODE == 2) {
      const float* px = (const float*)base;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int r = ci >> 3, c = ci & 7;
        int gr = row0 + r, gk = k0 + c * 8;
        if (gr < rows && gk < p.K) {
          int b = gr >> 12, ph = (gr >> 6) & 63, pw = gr & 63;
          int ch = gk >> 8, kh = (gk >> 4) & 15, kw = gk & 15;
          const float* s = px + (((long long)(b * 3 + ch) * 1024 + ph * 16 + kh) * 1024 + pw * 16 + kw);
          float4 a0 = *(const float4*)s;
          float4 a1 = *(const float4*)(s + 4);
          v[i] = cvt8(a0, a1);
        } else {
          v[i] = (e16x8)(e16)0.0f;
        }
      }
    } else {  // MODE 3: conv3x3 over NHWC 64x64 e16
      const e16* src = (const e16*)base;
      const int C = p.conv_c;
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int r = ci >> 3, c = ci & 7;
        int gr = row0 + r, gk = k0 + c * 8;
        e16x8 val = (e16x8)(e16)0.0f;
        if (gr < rows && gk < p.K) {
          int b = gr >> 12, y = (gr >> 6) & 63, x = gr & 63;
          int tap = gk / C, ch = gk - tap * C;
          int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
          if (yy >= 0 && yy < 64 && xx >= 0 && xx < 64)
            val = *(const e16x8*)(src + (((long long)b * 64 + yy) * 64 + xx) * C + ch);
        }
        v[i] = val;
      }
    }
  }

  __device__ __forceinline__ void store(e16* lds, int tid) {
    if constexpr (MODE == 1 || MODE == 5) {
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int k = ci / RC, rc = ci % RC;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          int r = rc * 8 + e;
          lds[lds_idx(r, k >> 3) + (k & 7)] = v[i][e];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        int ci = tid + i * NTHR;
        int r = ci >> 3, c = ci & 7;
        *(e16x8*)(lds + lds_idx(r, c)) = v[i];
      }
    }
  }
};

// T = 128 (block tile 128x128, wave 64x64) or 64 (block 64x64, wave 32x32: small problems, 4x the blocks)
template <int AM, int BMODE, int T = 128>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(GemmK p) {
  constexpr int MB = T / 64;  // 32x32 MFMA blocks per wave and dimension
  __shared__ __attribute__((aligned(16))) e16 smem[2 * (T + T) * BK];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the linear block id.
  const int nwg = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    int xcd = bid & 7, loc = bid >> 3;
    int q = nwg >> 3, rr = nwg & 7;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int row0 = tm * T, col0 = tn * T;
  const int bz = blockIdx.y;

  const char* Ab = (const char*)p.A;
  const char* Bb = (const char*)p.B;
  const void* Abase = (AM == 2) ? (const void*)(Ab + bz * p.sA * 4) : (const void*)(Ab + bz * p.sA * 2);
  const void* Bbase = (const void*)(Bb + bz * p.sB * 2);

  Loader<AM, T> la;
  Loader<BMODE, T> lb;
  f32x16 acc[MB][MB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < MB; ++j) acc[i][j] = (f32x16)0.0f;
  // split-K over k-major operands (k_total): rows past k_total (counted from batch 0) read as zero
  const int kcap = p.k_total > 0 ? min(p.K, p.k_total - bz * p.K) : p.K;

  const int nk = (p.K + BK - 1) / BK;
  la.load(p, Abase, p.A2, p.a2_rows, p.lda, p.M, row0, 0, tid, p.a_blk, p.a_rep, kcap);
  lb.load(p, Bbase, p.B2, p.b2_rows, p.ldb, p.N, col0, 0, tid, p.b_blk, p.b_rep, kcap);
  la.store(smem, tid);
  lb.store(smem + T * BK, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    e16* sa = smem + (kt & 1) * (T + T) * BK;
    e16* sb = sa + T * BK;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(p, Abase, p.A2, p.a2_rows, p.lda, p.M, row0, (kt + 1) * BK, tid, p.a_blk, p.a_rep, kcap);
      lb.load(p, Bbase, p.B2, p.b2_rows, p.ldb, p.N, col0, (kt + 1) * BK, tid, p.b_blk, p.b_rep, kcap);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = kk * 2 + (lane >> 5);
      e16x8 af[MB], bfr[MB];
#pragma unroll
      for (int i = 0; i < MB; ++i) af[i] = *(const e16x8*)(sa + lds_idx(wm * (T / 2) + i * 32 + (lane & 31), ch));
#pragma unroll
      for (int j = 0; j < MB; ++j) bfr[j] = *(const e16x8*)(sb + lds_idx(wn * (T / 2) + j * 32 + (lane & 31), ch));
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
          acc[i][j] = mma32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      e16* na = smem + ((kt + 1) & 1) * (T + T) * BK;
      la.store(na, tid);
      lb.store(na + T * BK, tid);
    }
    __syncthreads();
  }

  // Epilogue.
  char* Cb = (char*)p.C + bz * p.sC * (p.c_f32 ? 4 : 2);
  const char* Rb = p.R ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    const int n = col0 + wn * (T / 2) + j * 32 + (lane & 31);
    if (n >= p.N) continue;
    const float bv = p.bias ? p.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = row0 + wm * (T / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        int om = m;
        if (p.row_map) {
          om = p.row_map[m];
          if (om < 0) continue;
        }
        const long long ci = (long long)om * p.ldc + n;
        float v = acc[i][j][r] * p.alpha;
        if (p.beta != 0.0f) v += p.beta * (p.c_f32 ? ((float*)Cb)[ci] : (float)((e16*)Cb)[ci]);
        v += bv;
        if (Pb) {
          if (p.pre_f32) ((float*)Pb)[ci] = v;
          else ((e16*)Pb)[ci] = (e16)v;
        }
        if (p.act == OCTSAM_ACT_RELU) v = fmaxf(v, 0.0f);
        else if (p.act == OCTSAM_ACT_GELU) v = gelu_erf(v);
        if (Rb) {
          const long long ri = remap(om, p.r_blk, p.r_rep) * p.ldr + n;
          v += p.r_f32 ? ((const float*)Rb)[ri] : (float)((const e16*)Rb)[ri];
        }
        if (p.c_f32) ((float*)Cb)[ci] = v;
        else ((e16*)Cb)[ci] = (e16)v;
      }
    }
  }
}

// Small problems with K <= 256 (the decoder's token-side products: M = prompts x 7 rows, N, K = 128-256): the
// 64x64-tile kernel above chains one global load latency per 64-deep K-step (load, LDS store, barrier, MFMAs).
// Here every K-step's operand chunks are loaded into registers at once (at most 4 stages x 2 operands x 2 chunks
// of 16 B per thread), stored into a 4-stage LDS image, one barrier, then all MFMAs: one load latency per tile.
// Same LDS image, fragments, MFMA order (the K-steps in sequence) and epilogue as gemm_kernel<AM, BMODE, 64>, so the
// results are bit-identical to it.
template <int AM, int BMODE>
__global__ __launch_bounds__(NTHR, 2) void gemm_small_kernel(GemmK p) {
  constexpr int T = 64, NS = 4;
  __shared__ __attribute__((aligned(16))) e16 smem[NS * (T + T) * BK];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    int xcd = bid & 7, loc = bid >> 3;
    int q = nwg >> 3, rr = nwg & 7;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int row0 = tm * T, col0 = tn * T;
  const int bz = blockIdx.y;
  const void* Abase = (const void*)((const char*)p.A + bz * p.sA * 2);
  const void* Bbase = (const void*)((const char*)p.B + bz * p.sB * 2);
  const int kcap = p.k_total > 0 ? min(p.K, p.k_total - bz * p.K) : p.K;
  const int nk = (p.K + BK - 1) / BK;  // <= NS (host-checked)
  Loader<AM, T> la[NS];
  Loader<BMODE, T> lb[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < nk) {
      la[s].load(p, Abase, p.A2, p.a2_rows, p.lda, p.M, row0, s * BK, tid, p.a_blk, p.a_rep, kcap);
      lb[s].load(p, Bbase, p.B2, p.b2_rows, p.ldb, p.N, col0, s * BK, tid, p.b_blk, p.b_rep, kcap);
    }
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < nk) {
      la[s].store(smem + s * (T + T) * BK, tid);
      lb[s].store(smem + s * (T + T) * BK + T * BK, tid);
    }
  __syncthreads();
  f32x16 acc = (f32x16)0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s >= nk) break;
    const e16* sa = smem + s * (T + T) * BK;
    const e16* sb = sa + T * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = kk * 2 + (lane >> 5);
      const e16x8 af = *(const e16x8*)(sa + lds_idx(wm * (T / 2) + (lane & 31), ch));
      const e16x8 bfr = *(const e16x8*)(sb + lds_idx(wn * (T / 2) + (lane & 31), ch));
      acc = mma32(af, bfr, acc, 0, 0, 0);
    }
  }
  char* Cb = (char*)p.C + bz * p.sC * (p.c_f32 ? 4 : 2);
  const char* Rb = p.R ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
  const int n = col0 + wn * (T / 2) + (lane & 31);
  if (n >= p.N) return;
  const float bv = p.bias ? p.bias[n] : 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = row0 + wm * (T / 2) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m >= p.M) continue;
    int om = m;
    if (p.row_map) {
      om = p.row_map[m];
      if (om < 0) continue;
    }
    const long long ci = (long long)om * p.ldc + n;
    float v = acc[r] * p.alpha;
    if (p.beta != 0.0f) v += p.beta * (p.c_f32 ? ((float*)Cb)[ci] : (float)((e16*)Cb)[ci]);
    v += bv;
    if (Pb) {
      if (p.pre_f32) ((float*)Pb)[ci] = v;
      else ((e16*)Pb)[ci] = (e16)v;
    }
    if (p.act == OCTSAM_ACT_RELU) v = fmaxf(v, 0.0f);
    else if (p.act == OCTSAM_ACT_GELU) v = gelu_erf(v);
    if (Rb) {
      const long long ri = remap(om, p.r_blk, p.r_rep) * p.ldr + n;
      v += p.r_f32 ? ((const float*)Rb)[ri] : (float)((const e16*)Rb)[ri];
    }
    if (p.c_f32) ((float*)Cb)[ci] = v;
    else ((e16*)Cb)[ci] = (e16)v;
  }
}

template <int AM, int BMODE>
int launch_small(const GemmK& k0, int batch, hipStream_t s) {
  GemmK k = k0;
  k.tiles_m = (k.M + 63) / 64;
  k.tiles_n = (k.N + 63) / 64;
  dim3 grid(k.tiles_m * k.tiles_n, batch);
  hipLaunchKernelGGL((gemm_small_kernel<AM, BMODE>), grid, dim3(NTHR), 0, s, k);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

template <int AM, int BMODE, int T = 128>
int launch(const GemmK& k0, int batch, hipStream_t s) {
  GemmK k = k0;
  k.tiles_m = (k.M + T - 1) / T;
  k.tiles_n = (k.N + T - 1) / T;
  dim3 grid(k.tiles_m * k.tiles_n, batch);
  hipLaunchKernelGGL((gemm_kernel<AM, BMODE, T>), grid, dim3(NTHR), 0, s, k);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}


// ------------------------------------------------------------------------------------------------
// Fast path for C = A . B^T with both operands K-contiguous (a_mode 0, b_mode 0), K % BK == 0.
// Persistent: one 512-thread workgroup per CU walks its XCD's contiguous range of tiles (L2 reuse of the
// A row panel and of B). Operands stream global -> LDS by global_load_lds_dwordx4 (no VGPR staging) into
// an NS-stage ring, NS-1 stages in flight behind a counted vmcnt and a raw s_barrier; the ring runs
// across tile boundaries so the next tile's loads overlap the current epilogue. The XOR chunk swizzle of
// the LDS image (conflict-free ds_read_b128 fragment reads) is applied on the per-lane SOURCE address.
// 8 waves = 4 (M) x 2 (N); wave tile 64 x BN/2 of v_mfma_f32_32x32x16_bf16. Rows beyond M / N are
// clamped to a valid row (their results are never stored).
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// raw s_barrier with compiler fences: the intrinsic alone does not stop LDS reads / LDS-DMA issue
// from being moved across it
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BK>
__device__ __forceinline__ int sw_off(int r, int c) {  // byte offset of 16-B chunk c of row r
  if constexpr (BK == 64) return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
  else return r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
}

template <int BK>
__device__ __forceinline__ void glds_tile(const e16* __restrict__ src, long long ld, int rows, int row0, int k0,
                                          char* lds, int nrows_tile, int wave, int lane) {
  constexpr int CPR = BK / 8;          // 16-B chunks per row
  constexpr int RPI = 64 / CPR;        // rows per wave-instruction (1 KiB)
  const int ninst = nrows_tile / RPI;
  for (int j = wave; j < ninst; j += 8) {
    const int rr = lane / CPR, slot = lane % CPR;
    const int r = j * RPI + rr;
    // inverse swizzle: LDS slot `slot` of row r holds logical chunk c
    int c;
    if constexpr (BK == 64) c = slot ^ ((r >> 1) & 7);
    else c = slot ^ ((r >> 2) & 3);
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const e16* g = src + (long long)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_ptr_t)(lds + j * 1024), 16, 0, 0);
  }
}

// k-major operand (the operand stored [K][X], X = M or N contiguous: dY^T / X^T of weight gradients,
// a weight used as W rather than W^T). LDS image: per 128-column half a [64 k-rows][128] tile with 256-B
// rows and chunk swizzle f(r) = ((r&3)<<2) | ((r>>2)&3); fragments come out of ds_read_b64_tr_b16
// (gfx950 LDS transpose read), conflict-free on this image. X % 8 == 0 and ld % 8 == 0 (host-checked);
// columns past X are clamped to the last chunk (their results are never stored).
__device__ __forceinline__ int km_off(int r, int ch) { return r * 256 + ((ch ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4); }

__device__ uint4 g_zero16[4];  // 16 zero bytes: LDS-DMA source of k rows past the end of a K tail

template <int TX>
__device__ __forceinline__ void glds_tile_km(const e16* __restrict__ src, long long ld, int xdim, int x0, int k0,
                                             char* lds, int wave, int lane, int kmax = 0x7fffffff) {
  constexpr int NINST = TX / 8;  // 64 rows * TX * 2 B / 1 KiB
#pragma unroll
  for (int j = wave; j < NINST; j += 8) {
    const int h = j >> 4, r = ((j & 15) << 2) + (lane >> 4), slot = lane & 15;
    const int ch = slot ^ (((r & 3) << 2) | ((r >> 2) & 3));
    int col = x0 + h * 128 + ch * 8;
    col = col < xdim ? col : xdim - 8;
    const e16* g = k0 + r < kmax ? src + (long long)(k0 + r) * ld + col : (const e16*)g_zero16;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_ptr_t)(lds + h * 16384 + (j & 15) * 1024), 16, 0, 0);
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 32x32x16 MFMA operand (8 consecutive k of row xb + (lane & 31), k from kb + 8*(lane>>5)) from a k-major image
__device__ __forceinline__ e16x8 frag_km(const char* img, int xb, int kb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int x = xb + 16 * (g & 1);
  const int h = x >> 7, c0 = (x & 127) >> 3;
  const int r0 = kb + 8 * (g >> 1) + q;
  const char* base = img + h * 16384 + 8 * (pp & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + km_off(r0, c0 + (pp >> 1))));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + km_off(r0 + 4, c0 + (pp >> 1))));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(e16x8, v);
}

// s + the sum of an MFMA operand fragment's 8 elements (4 v_dot2 with ones: exact products, fp32 sums). A
// k-major fragment holds 8 consecutive k of one row, so summing it over a tile's K-steps gives that row's
// column sum of the operand (a bias gradient) from registers the MFMAs already loaded.
__device__ __forceinline__ float frag_sum(e16x8 v, float s) {
  const e16x2 one = {(e16)1.0f, (e16)1.0f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const e16x2 pr = {v[2 * q], v[2 * q + 1]};
#ifdef OCTSAM_GEMM_F16
    s = __builtin_amdgcn_fdot2(pr, one, s, false);
#else
    s = __builtin_amdgcn_fdot2_f32_bf16(pr, one, s, false);
#endif
  }
  return s;
}

// Fast epilogue: adjacent lanes trade one value with a DPP quad swap so each lane owns two adjacent
// columns of one row (even lane: row m, cols n,n+1; odd lane: row m+1, cols n-1,n) and writes them with one
// 4-B (e16x2) or 8-B (float2) store. Loads are hoisted ahead of the stores so a store never waits on an
// earlier store's completion (vmcnt counts both): bias + row map first, then a e16 residual for the whole
// wave tile; an fp32 residual or a beta*C read is loaded per 32-column group (one wait per group).
// Requires N, ldc (and ldr) even and 4/8-B aligned C / R / C_pre (checked on the host).
__device__ __forceinline__ float2 ld_pair(const void* base, long long idx, bool f32) {
  if (f32) return *(const float2*)((const float*)base + idx);
  const uint32_t r = *(const uint32_t*)((const e16*)base + idx);
  return make_float2(lo16f(r), hi16f(r));
}
__device__ __forceinline__ void st_pair(void* base, long long idx, bool f32, float lo, float hi) {
  if (f32) {
    *(float2*)((float*)base + idx) = make_float2(lo, hi);
  } else {
    e16x2 w;
    w[0] = (e16)lo;
    w[1] = (e16)hi;
    *(e16x2*)((e16*)base + idx) = w;
  }
}
__device__ __forceinline__ float dpp_swap1(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

template <int NI, int NJ, bool LATE>
__device__ __forceinline__ void epilogue_fast(const GemmK& p, f32x16 (&acc)[NI][NJ], int bz, int row0, int col0,
                                              int lane) {
  const int esz_c = p.c_f32 ? 4 : 2;
  char* Cb = (char*)p.C + bz * p.sC * esz_c;
  const char* Rb = p.R ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
  const bool odd = lane & 1;
  const int ncol = lane & 31;
  float bv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = col0 + j * 32 + ncol;
    bv[j] = (p.bias && n < p.N) ? p.bias[n] : 0.0f;
  }
  int om[NI][8];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int r0 = 2 * t;
      const int m = row0 + i * 32 + (r0 & 3) + 8 * (r0 >> 2) + 4 * (lane >> 5) + (odd ? 1 : 0);
      om[i][t] = m < p.M ? (p.row_map ? p.row_map[m] : m) : -1;
    }
  uint32_t rv[LATE ? 1 : NI][LATE ? 1 : NJ][8];
  if (!LATE && Rb) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = col0 + j * 32 + (ncol & ~1);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int o = om[i][t];
          rv[LATE ? 0 : i][LATE ? 0 : j][t] = (o >= 0 && c < p.N)
                            ? *(const uint32_t*)((const e16*)Rb + remap(o, p.r_blk, p.r_rep) * p.ldr + c) : 0u;
        }
      }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = col0 + j * 32 + (ncol & ~1);
    float2 lr[LATE ? NI : 1][8], lc[LATE ? NI : 1][8];
    if constexpr (LATE) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int o = om[i][t];
          const bool ok = o >= 0 && c < p.N;
          lr[i][t] = (Rb && ok) ? ld_pair(Rb, remap(o, p.r_blk, p.r_rep) * p.ldr + c, p.r_f32) : make_float2(0.f, 0.f);
          lc[i][t] = (p.beta != 0.0f && ok) ? ld_pair(Cb, (long long)o * p.ldc + c, p.c_f32) : make_float2(0.f, 0.f);
        }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        float v0 = acc[i][j][2 * t] * p.alpha;
        float v1 = acc[i][j][2 * t + 1] * p.alpha;
        // pair layout first, so the beta*C / residual reads use the stored pair order. Every DPP runs
        // unconditionally in all lanes (a DPP under a divergent select would read inactive lanes).
        const float send = odd ? v0 : v1;
        const float recv = dpp_swap1(send);
        const float bsw = dpp_swap1(bv[j]);
        float lo = odd ? recv : v0, hi = odd ? v1 : recv;
        const float b_lo = odd ? bsw : bv[j];
        const float b_hi = odd ? bv[j] : bsw;
        if constexpr (LATE) {
          lo += p.beta * lc[i][t].x;
          hi += p.beta * lc[i][t].y;
        }
        lo += b_lo;
        hi += b_hi;
        const int o = om[i][t];
        const bool ok = o >= 0 && c < p.N;
        const long long ci = (long long)o * p.ldc + c;
        if (Pb && ok) st_pair(Pb, ci, p.pre_f32, lo, hi);
        if (p.act == OCTSAM_ACT_RELU) {
          lo = fmaxf(lo, 0.0f);
          hi = fmaxf(hi, 0.0f);
        } else if (p.act == OCTSAM_ACT_GELU) {
          lo = gelu_erf(lo);
          hi = gelu_erf(hi);
        }
        if (Rb) {
          if constexpr (LATE) {
            lo += lr[i][t].x;
            hi += lr[i][t].y;
          } else {
            const uint32_t r = rv[LATE ? 0 : i][LATE ? 0 : j][t];
            lo += lo16f(r);
            hi += hi16f(r);
          }
        }
        if (ok) st_pair(Cb, ci, p.c_f32, lo, hi);
      }
  }
}

template <int BN_, int BK, int NS, bool LATE, bool AKM, bool BKM>
__global__ __launch_bounds__(512, 2) void gemm_glds_kernel(GemmK p, int batch) {
  static_assert(!(AKM || BKM) || BK == 64, "k-major operands use BK = 64");
  constexpr int BM_ = 256;
  constexpr int A_BYTES = BM_ * BK * 2, B_BYTES = BN_ * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int NJ = BN_ / 64;  // 32-wide fragments per wave in N (wave tile 64 x BN/2)
  constexpr int CPR = BK / 8, RPI = 64 / CPR;
  constexpr int GL_PER_WAVE = (BM_ / RPI + BN_ / RPI) / 8;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int per_batch = p.tiles_m * p.tiles_n;
  const int ntiles = per_batch * batch;
  const int nxcd_wg = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int tper = (ntiles + 7) >> 3;
  const int tbeg = xcd * tper, tend = min(ntiles, tbeg + tper);
  const int first = tbeg + loc;
  const int mycnt = first < tend ? (tend - first + nxcd_wg - 1) / nxcd_wg : 0;
  const int nk = (p.K + BK - 1) / BK;  // (K % BK != 0 only with a k_total tail: zero-filled rows)
  const int total = mycnt * nk;
  if (total == 0) return;

  auto tile_of = [&](int i, int& bz, int& row0, int& col0) {
    int t = first + i * nxcd_wg;
    bz = t / per_batch;
    int r = t - bz * per_batch;
    int tm = r / p.tiles_n, tn = r - tm * p.tiles_n;
    row0 = tm * BM_;
    col0 = tn * BN_;
  };
  auto issue = [&](int g) {
    int i = g / nk, kt = g - i * nk;
    int bz, r0, c0;
    tile_of(i, bz, r0, c0);
    char* st = gsm + (g % NS) * STAGE;
    const int kmax = p.k_total > 0 ? p.k_total - bz * p.K : 0x7fffffff;
    if constexpr (AKM) glds_tile_km<BM_>((const e16*)p.A + bz * p.sA, p.lda, p.M, r0, kt * BK, st, wave, lane, kmax);
    else glds_tile<BK>((const e16*)p.A + bz * p.sA, p.lda, p.M, r0, kt * BK, st, BM_, wave, lane);
    if constexpr (BKM) glds_tile_km<BN_>((const e16*)p.B + bz * p.sB, p.ldb, p.N, c0, kt * BK, st + A_BYTES, wave, lane, kmax);
    else glds_tile<BK>((const e16*)p.B + bz * p.sB, p.ldb, p.N, c0, kt * BK, st + A_BYTES, BN_, wave, lane);
  };

  f32x16 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x16)0.0f;
  // fused column sums (k-major operands), one fragment per wave so no wave carries much more VALU than the
  // others: on the tiles of column 0 wave (wm, wn) sums A fragment i = wn (rows wm*64 + wn*32 ..), on the tiles
  // of row 0 waves wm < NJ sum B fragment j = wm (columns wn*BN/2 + wm*32 ..): every element once per batch
  float csa = 0.0f, csb = 0.0f;
  bool cs_a = false, cs_b = false;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) issue(s);
  for (int g = 0; g < total; ++g) {
    if constexpr (AKM || BKM) {
      if (g % nk == 0) {
        int bz, r0, c0;
        tile_of(g / nk, bz, r0, c0);
        cs_a = AKM && p.a_cs != nullptr && c0 == 0;
        cs_b = BKM && p.b_cs != nullptr && wm < NJ && r0 == 0;
      }
    }
    // wait for stage g: leave the younger (NS-2) stages in flight
    const int ahead = min(NS - 2, total - 1 - g);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL_PER_WAVE) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL_PER_WAVE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    if (g + NS - 1 < total) issue(g + NS - 1);
    const char* sa = gsm + (g % NS) * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ch = kk * 2 + (lane >> 5);
      e16x8 af[2], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (AKM) af[i] = frag_km(sa, wm * 64 + i * 32, kk * 16, lane);
        else af[i] = *(const e16x8*)(sa + sw_off<BK>(wm * 64 + i * 32 + (lane & 31), ch));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (BKM) bfr[j] = frag_km(sb, wn * (BN_ / 2) + j * 32, kk * 16, lane);
        else bfr[j] = *(const e16x8*)(sb + sw_off<BK>(wn * (BN_ / 2) + j * 32 + (lane & 31), ch));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = mma32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if constexpr (AKM) {
        if (cs_a) csa = frag_sum(wn ? af[1] : af[0], csa);
      }
      if constexpr (BKM) {
        if (cs_b) {
          e16x8 f = bfr[0];
#pragma unroll
          for (int j = 1; j < NJ; ++j) f = wm == j ? bfr[j] : f;
          csb = frag_sum(f, csb);
        }
      }
    }
    if (g % nk == nk - 1) {
      int bz, r0, c0;
      tile_of(g / nk, bz, r0, c0);
      if constexpr (AKM) {
        if (cs_a) {  // lanes l and l + 32 hold the two k halves of row (l & 31)
          const float v = csa + __shfl_xor(csa, 32, 64);
          const int m = r0 + wm * 64 + wn * 32 + lane;
          if (lane < 32 && m < p.M) p.a_cs[(long long)bz * p.M + m] = v;
          csa = 0.0f;
        }
      }
      if constexpr (BKM) {
        if (cs_b) {
          const float v = csb + __shfl_xor(csb, 32, 64);
          const int n = c0 + wn * (BN_ / 2) + wm * 32 + lane;
          if (lane < 32 && n < p.N) p.b_cs[(long long)bz * p.N + n] = v;
          csb = 0.0f;
        }
      }
      epilogue_fast<2, NJ, LATE>(p, acc, bz, r0 + wm * 64, c0 + wn * (BN_ / 2), lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x16)0.0f;
    }
  }
}

template <int BN_, int BK, int NS, bool LATE, bool AKM, bool BKM>
int launch_glds_t(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  constexpr int STAGE = (256 + BN_) * BK * 2;
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = (a->N + BN_ - 1) / BN_;
  static int n_cu = 0;
  if (!n_cu) {
    (void)hipFuncSetAttribute((const void*)gemm_glds_kernel<BN_, BK, NS, LATE, AKM, BKM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        NS * STAGE);
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
  }
  const int ntiles = g.tiles_m * g.tiles_n * a->batch;
  int grid = ((n_cu + 7) / 8) * 8;
  while (grid > 8 && grid / 2 >= ntiles) grid /= 2;
  hipLaunchKernelGGL((gemm_glds_kernel<BN_, BK, NS, LATE, AKM, BKM>), dim3(grid), dim3(512), NS * STAGE, s, g, a->batch);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

template <int BN_, int BK, int NS, bool AKM = false, bool BKM = false>
int launch_glds(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  // fp32 residual / beta*C epilogue: the 256x128 tile (the 256x256 one would spill)
  if ((a->R && a->r_f32) || a->beta != 0.0f) return launch_glds_t<128, 64, 3, true, AKM, BKM>(k0, a, s);
  return launch_glds_t<BN_, BK, NS, false, AKM, BKM>(k0, a, s);
}

// ------------------------------------------------------------------------------------------------
// 8-phase NT GEMM (a_mode 0, b_mode 0, K % 64 == 0): 256x256 tile, BK = 64, 8 waves as 2 (M) x 4 (N),
// wave tile 128 x 64 of v_mfma_f32_16x16x32_bf16, one tile per workgroup (XCD-contiguous tile order).
// Two LDS buffers (K-tiles alternate); each buffer is split into regions by the phase that reads them:
// A-lo / A-hi = rows 0-63 / 64-127 of each wave-row block, B-n0 / B-n1 = cols 0-31 / 32-63 of each
// wave-column block. A K-tile is four phases, one 64x32 quadrant of the wave tile x K = 64 (16 MFMAs)
// each: Q(0,0) reads A-lo + B-n0, Q(0,1) B-n1, Q(1,0) A-hi, Q(1,1) nothing. A region is reloaded by
// global_load_lds two phases after its last read and read ~6 phases after its load is issued; counted
// vmcnt before the first barrier of the phase preceding the read, raw s_barrier, and the two wave rows
// run one barrier apart so one row's MFMAs overlap the other's LDS reads.
namespace ph8 {
constexpr int BUF = 65536;  // A [256][64] + B [256][64] e16
constexpr int BIAS_MAX_LDS = 8192;  // fp32 bias entries the persistent kernel keeps in LDS (32 KiB)

// region 0 A-lo, 1 A-hi, 2 B-n0, 3 B-n1: 128 rows x 128 B = 16 instructions of 8 rows, 2 per wave
__device__ __forceinline__ void load_region(const GemmK& p, const e16* A, const e16* B, int region, int row0,
                                            int col0, int k0, char* buf, int wave, int lane) {
  const bool isA = region < 2;
  const e16* src = isA ? A : B;
  const long long ld = isA ? p.lda : p.ldb;
  const int lim = isA ? p.M : p.N, g0 = isA ? row0 : col0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = wave * 2 + u;
    const int rbase = isA ? (j >> 3) * 128 + (region & 1) * 64 + (j & 7) * 8
                          : (j >> 2) * 64 + (region & 1) * 32 + (j & 3) * 8;
    const int r = rbase + (lane >> 3), slot = lane & 7;
    const int c = slot ^ ((r >> 1) & 7);
    int gr = g0 + r;
    gr = gr < lim ? gr : lim - 1;
    const e16* g = src + (long long)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_ptr_t)(buf + (isA ? 0 : 32768) + rbase * 128), 16, 0, 0);
  }
}

// Tile-invariant part of load_region's addresses: byte offset (r * ld + c * 8) * 2 of each lane's 16-B
// chunk for region / issue u. A full tile (no clamped rows) then needs one uniform base per operand and
// K-step (SGPRs) and one add per issue, instead of a 64-bit multiply-add per lane and issue.
struct LdPlan {
  uint32_t off[4][2];
};
__device__ __forceinline__ LdPlan make_plan(const GemmK& p, int wave, int lane) {
  LdPlan pl;
#pragma unroll
  for (int region = 0; region < 4; ++region)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool isA = region < 2;
      const int j = wave * 2 + u;
      const int rbase = isA ? (j >> 3) * 128 + (region & 1) * 64 + (j & 7) * 8
                            : (j >> 2) * 64 + (region & 1) * 32 + (j & 3) * 8;
      const int r = rbase + (lane >> 3), slot = lane & 7;
      const int c = slot ^ ((r >> 1) & 7);
      pl.off[region][u] = (uint32_t)((r * (isA ? p.lda : p.ldb) + c * 8) * 2);
    }
  return pl;
}
// Buffer-descriptor form (persistent kernel): the descriptor starts at the tile's first row and ends at the
// operand's last row, so rows past M (N) read as zero through the hardware range check (no clamp, no
// per-lane 64-bit address); voffset = the tile-invariant plan offset, soffset = the K-step's byte offset.
// Requires rows_left * ld * 2 < 2^31 (host-checked).
__device__ __forceinline__ void load_region_buf(const GemmK& p, const e16* A, const e16* B, int row0, int col0, int kt,
                                                int region, const LdPlan& pl, char* buf, int wave) {
  const bool isA = region < 2;
  const e16* base = isA ? A + (long long)row0 * p.lda : B + (long long)col0 * p.ldb;
  const long long ld = isA ? p.lda : p.ldb;
  const int bytes = (int)((long long)((isA ? p.M - row0 : p.N - col0)) * ld * 2);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = wave * 2 + u;
    const int rbase = isA ? (j >> 3) * 128 + (region & 1) * 64 + (j & 7) * 8
                          : (j >> 2) * 64 + (region & 1) * 32 + (j & 3) * 8;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(buf + (isA ? 0 : 32768) + rbase * 128), 16,
                                             pl.off[region][u], (uint32_t)(kt * 128), 0, 0);
  }
}

__device__ __forceinline__ e16x8 frag(const char* img, int row, int kc) {
  return *(const e16x8*)(img + sw_off<64>(row, kc));
}

// lane: col n = lane & 15, rows 4*(lane>>4) + i. Pairs (i, i+1) of adjacent lanes are merged by a DPP
// swap as in epilogue_fast: even lane -> row r (cols n, n+1), odd lane -> row r+1 (cols n-1, n).
template <bool LATE>
__device__ __forceinline__ void epilogue16(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0, int col0, int lane) {
  const int esz_c = p.c_f32 ? 4 : 2;
  char* Cb = (char*)p.C + bz * p.sC * esz_c;
  const char* Rb = p.R ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
  const bool odd = lane & 1;
  float bv[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = col0 + ni * 16 + (lane & 15);
    bv[ni] = (p.bias && n < p.N) ? p.bias[n] : 0.0f;
  }
  int om[8][2];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int m = row0 + mi * 16 + 4 * (lane >> 4) + 2 * t + (odd ? 1 : 0);
      om[mi][t] = m < p.M ? (p.row_map ? p.row_map[m] : m) : -1;
    }
  uint32_t rv[LATE ? 1 : 8][LATE ? 1 : 4][2];
  if (!LATE && Rb) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int c = col0 + ni * 16 + ((lane & 15) & ~1);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int o = om[mi][t];
          rv[LATE ? 0 : mi][LATE ? 0 : ni][t] =
              (o >= 0 && c < p.N) ? *(const uint32_t*)((const e16*)Rb + remap(o, p.r_blk, p.r_rep) * p.ldr + c) : 0u;
        }
      }
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int c = col0 + ni * 16 + ((lane & 15) & ~1);
    float2 lr[LATE ? 8 : 1][2], lc[LATE ? 8 : 1][2];
    if constexpr (LATE) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int o = om[mi][t];
          const bool ok = o >= 0 && c < p.N;
          lr[mi][t] = (Rb && ok) ? ld_pair(Rb, remap(o, p.r_blk, p.r_rep) * p.ldr + c, p.r_f32) : make_float2(0.f, 0.f);
          lc[mi][t] = (p.beta != 0.0f && ok) ? ld_pair(Cb, (long long)o * p.ldc + c, p.c_f32) : make_float2(0.f, 0.f);
        }
    }
    const float bsw = dpp_swap1(bv[ni]);
    const float b_lo = odd ? bsw : bv[ni], b_hi = odd ? bv[ni] : bsw;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float v0 = acc[mi][ni][2 * t] * p.alpha, v1 = acc[mi][ni][2 * t + 1] * p.alpha;
        const float send = odd ? v0 : v1;
        const float recv = dpp_swap1(send);
        float lo = odd ? recv : v0, hi = odd ? v1 : recv;
        if constexpr (LATE) {
          lo += p.beta * lc[mi][t].x;
          hi += p.beta * lc[mi][t].y;
        }
        lo += b_lo;
        hi += b_hi;
        const int o = om[mi][t];
        const bool ok = o >= 0 && c < p.N;
        const long long ci = (long long)o * p.ldc + c;
        if (Pb && ok) st_pair(Pb, ci, p.pre_f32, lo, hi);
        if (p.act == OCTSAM_ACT_RELU) {
          lo = fmaxf(lo, 0.0f);
          hi = fmaxf(hi, 0.0f);
        } else if (p.act == OCTSAM_ACT_GELU) {
          lo = gelu_erf(lo);
          hi = gelu_erf(hi);
        }
        if (Rb) {
          if constexpr (LATE) {
            lo += lr[mi][t].x;
            hi += lr[mi][t].y;
          } else {
            const uint32_t r = rv[LATE ? 0 : mi][LATE ? 0 : ni][t];
            lo += lo16f(r);
            hi += hi16f(r);
          }
        }
        if (ok) st_pair(Cb, ci, p.c_f32, lo, hi);
      }
  }
}

// LDS-staged epilogue: the fp32 tile goes through LDS in two 128-row passes ([128][256+4] fp32,
// padded against bank conflicts) and every lane then finishes 8 consecutive columns of one row with
// 16-B vector loads (bias, residual, beta*C) and 16-B (e16) / 2x16-B (fp32) stores: full cache lines
// instead of the MFMA layout's 32-B row segments. Requires N, ldc (ldr) % 8 == 0 and 16-B aligned
// C / C_pre / R (host-checked).
constexpr int EPI_LD = 260;
constexpr int EPI_BYTES = 128 * EPI_LD * 4;

__device__ __forceinline__ void load8(const void* base, long long idx, bool f32, float (&v)[8]) {
  if (f32) {
    const float4 a = *(const float4*)((const float*)base + idx), b = *(const float4*)((const float*)base + idx + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const e16x8 a = *(const e16x8*)((const e16*)base + idx);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)a[e];
  }
}
__device__ __forceinline__ void store8(void* base, long long idx, bool f32, const float (&v)[8]) {
  if (f32) {
    *(float4*)((float*)base + idx) = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)((float*)base + idx + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    e16x8 a;
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = (e16)v[e];
    *(e16x8*)((e16*)base + idx) = a;
  }
}

__device__ __forceinline__ void epilogue_lds(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0, int col0, int wr,
                                             int wc, int wave, int lane, char* smem) {
  float* st = (float*)smem;
  char* Cb = (char*)p.C + bz * p.sC * (p.c_f32 ? 4 : 2);
  const char* Rb = p.R ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
  const int c8 = (lane & 31) * 8;
  const int n0 = col0 + c8;
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.0f;
  if (p.bias && n0 < p.N) {
    const float4 a = *(const float4*)(p.bias + n0), b = *(const float4*)(p.bias + n0 + 4);
    bv[0] = a.x; bv[1] = a.y; bv[2] = a.z; bv[3] = a.w; bv[4] = b.x; bv[5] = b.y; bv[6] = b.z; bv[7] = b.w;
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    raw_barrier();  // LDS free (main loop done / previous pass read)
    if (wr == pass) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            st[(mi * 16 + 4 * (lane >> 4) + i) * EPI_LD + wc * 64 + ni * 16 + (lane & 15)] = acc[mi][ni][i];
    }
    raw_barrier();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int rr = it * 16 + wave * 2 + (lane >> 5);
      const int m = row0 + pass * 128 + rr;
      if (m >= p.M || n0 >= p.N) continue;
      const int om = p.row_map ? p.row_map[m] : m;
      if (om < 0) continue;
      const float4 a = *(const float4*)(st + rr * EPI_LD + c8), b = *(const float4*)(st + rr * EPI_LD + c8 + 4);
      float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const long long ci = (long long)om * p.ldc + n0;
      float old[8], res[8];
      if (p.beta != 0.0f) load8(Cb, ci, p.c_f32, old);
      if (Rb) load8(Rb, remap(om, p.r_blk, p.r_rep) * p.ldr + n0, p.r_f32, res);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] *= p.alpha;
        if (p.beta != 0.0f) v[e] += p.beta * old[e];
        v[e] += bv[e];
      }
      if (Pb) store8(Pb, ci, p.pre_f32, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (p.act == OCTSAM_ACT_RELU) v[e] = fmaxf(v[e], 0.0f);
        else if (p.act == OCTSAM_ACT_GELU) v[e] = gelu_erf(v[e]);
        if (Rb) v[e] += res[e];
      }
      store8(Cb, ci, p.c_f32, v);
    }
  }
}

// Register epilogue for the operand-swapped MFMA: acc[mi][ni] holds the 16x16 block transposed, so lane
// (q = lane>>4, r = lane&15) owns output row m = 16*mi + r and the 4 consecutive columns 16*ni + 4q .. +3.
// One v_permlane16_swap per value between blocks (2p, 2p+1) gives every lane 8 consecutive columns of its
// row, starting at 32p + 16*(q&1) + 8*(q>>1): 16-B e16 (32-B fp32) stores, 64-B row runs per
// instruction, no LDS round trip and no barrier (the next tile's loads can be in flight). Every input the
// stores depend on (row map, bias, residual, beta*C) is loaded before the first store, so no load waits
// behind a store (vmcnt counts both). Requires N, ldc (ldr) % 8 == 0 and 16-B aligned C / C_pre / R / bias.
template <int ACT>
__device__ __forceinline__ float act_apply(float v) {
  if constexpr (ACT == OCTSAM_ACT_RELU) return fmaxf(v, 0.0f);
  else if constexpr (ACT == OCTSAM_ACT_GELU) return gelu_fast(v);
  else return v;
}

// MI0 / NMI: the row blocks mi in [MI0, MI0 + NMI) this call finishes (the persistent kernel runs two
// halves of 4 so the epilogue's temporaries fit beside the live prefetch state)
// BIAS_LDS: the bias comes from lds_bias (indexed by output column) and the epilogue issues no global
// loads at all: no residual, no row map (the host routes those elsewhere)
template <int ACT, int MI0 = 0, int NMI = 8, bool BIAS_LDS = false>
__device__ __forceinline__ void epilogue_reg(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0, int col0,
                                             int lane, const float* lds_bias = nullptr) {
  char* Cb = (char*)p.C + bz * p.sC * (p.c_f32 ? 4 : 2);
  const char* Rb = (!BIAS_LDS && p.R) ? (const char*)p.R + bz * p.sR * (p.r_f32 ? 4 : 2) : nullptr;
  char* Pb = p.Cpre ? (char*)p.Cpre + bz * p.sC * (p.pre_f32 ? 4 : 2) : nullptr;
  const int q = lane >> 4;
  const int cofs = 16 * (q & 1) + 8 * (q >> 1);
  // permute first (all lanes active), then everything is per-lane elementwise on 8 consecutive columns
  float v[NMI][2][8];
#pragma unroll
  for (int j = 0; j < NMI; ++j)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      // (bit-cast the whole vector first: hipcc 7.2 drops all but element 0 of a per-element
      // __builtin_bit_cast(uint32_t, f32x4[i]) feeding this builtin)
      const u32x4 x = __builtin_bit_cast(u32x4, acc[MI0 + j][2 * pr]);
      const u32x4 y = __builtin_bit_cast(u32x4, acc[MI0 + j][2 * pr + 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t xi = x[i], yi = y[i];
        const auto r = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
        v[j][pr][i] = __builtin_bit_cast(float, (uint32_t)r[0]);
        v[j][pr][4 + i] = __builtin_bit_cast(float, (uint32_t)r[1]);
      }
    }
  int om[NMI];
#pragma unroll
  for (int j = 0; j < NMI; ++j) {
    const int m = row0 + 16 * (MI0 + j) + (lane & 15);
    om[j] = m < p.M ? ((!BIAS_LDS && p.row_map) ? p.row_map[m] : m) : -1;
  }
  float bv[2][8];
  if constexpr (BIAS_LDS) {
    // read through inline asm: hipcc would put a vmcnt(0) (the in-flight LDS-DMA prefetch) in front of an
    // ordinary LDS load here; the bias region is never a DMA target, so only lgkmcnt matters
    if (p.bias) {
      f32x4 t[2][2];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int n = min(col0 + 32 * pr + cofs, BIAS_MAX_LDS - 8);  // columns >= N are never stored
        const uint32_t ad = (uint32_t)(uintptr_t)(lds_ptr_t)(lds_bias + n);
        asm volatile("ds_read_b128 %0, %1" : "=v"(t[pr][0]) : "v"(ad));
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(t[pr][1]) : "v"(ad));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bv[pr][e] = t[pr][0][e];
          bv[pr][4 + e] = t[pr][1][e];
        }
    } else {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[pr][e] = 0.0f;
    }
  }
#pragma unroll
  for (int pr = 0; pr < 2 && !BIAS_LDS; ++pr) {
    const int n = col0 + 32 * pr + cofs;
    if (p.bias && n < p.N) {
      const float* bsrc = p.bias;
      const float4 a = *(const float4*)(bsrc + n), b = *(const float4*)(bsrc + n + 4);
      bv[pr][0] = a.x; bv[pr][1] = a.y; bv[pr][2] = a.z; bv[pr][3] = a.w;
      bv[pr][4] = b.x; bv[pr][5] = b.y; bv[pr][6] = b.z; bv[pr][7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[pr][e] = 0.0f;
    }
  }
#pragma unroll
  for (int j = 0; j < NMI; ++j)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][pr][e] = v[j][pr][e] * p.alpha + bv[pr][e];
  // (beta != 0 is routed to the other kernels by the host)
  auto finish = [&](int j, int pr, const float (&res)[8]) {
    const int n = col0 + 32 * pr + cofs;
    const bool ok = om[j] >= 0 && n < p.N;
    const long long ci = (long long)om[j] * p.ldc + n;
    if (Pb && ok) store8(Pb, ci, p.pre_f32, v[j][pr]);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[j][pr][e] = act_apply<ACT>(v[j][pr][e]) + res[e];
    if (ok) store8(Cb, ci, p.c_f32, v[j][pr]);
  };
  if (Rb && !p.r_f32) {
    u32x4 raw[NMI][2];
#pragma unroll
    for (int j = 0; j < NMI; ++j)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int n = col0 + 32 * pr + cofs;
        raw[j][pr] = (om[j] >= 0 && n < p.N)
                         ? *(const u32x4*)((const e16*)Rb + remap(om[j], p.r_blk, p.r_rep) * p.ldr + n)
                         : (u32x4)0u;
      }
#pragma unroll
    for (int j = 0; j < NMI; ++j)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        float res[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          res[2 * e] = lo16f(raw[j][pr][e]);
          res[2 * e + 1] = hi16f(raw[j][pr][e]);
        }
        finish(j, pr, res);
      }
  } else if (Rb) {  // fp32 residual: groups of 4 row blocks (register budget)
#pragma unroll
    for (int h = 0; h < NMI / 4; ++h) {
      float4 raw[4][2][2];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int j = 4 * h + jj, n = col0 + 32 * pr + cofs;
          if (om[j] >= 0 && n < p.N) {
            const float* s = (const float*)Rb + remap(om[j], p.r_blk, p.r_rep) * p.ldr + n;
            raw[jj][pr][0] = *(const float4*)s;
            raw[jj][pr][1] = *(const float4*)(s + 4);
          } else {
            raw[jj][pr][0] = raw[jj][pr][1] = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const float res[8] = {raw[jj][pr][0].x, raw[jj][pr][0].y, raw[jj][pr][0].z, raw[jj][pr][0].w,
                                raw[jj][pr][1].x, raw[jj][pr][1].y, raw[jj][pr][1].z, raw[jj][pr][1].w};
          finish(4 * h + jj, pr, res);
        }
    }
  } else {
    const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NMI; ++j)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) finish(j, pr, zero);
  }
}

// Lean register epilogue (no C_pre, N % 8 == 0): C and the residual go through buffer descriptors, so every
// store is one voffset add + buffer_store_dwordx4 and the hardware range check takes the row bounds — rows
// past M are dropped (stores) / read as zero (residual); columns past N (a ragged last column tile) are
// masked per lane.
//   FE bits (FE = 1 + bits): 1 fp32 C (else e16), 2 residual of C's type (ldr, stride_r), 4 row map (output
//   row row_map[m], -1 = dropped; the descriptors then span the whole C / R, row m's offset is
//   row_map[m] * ld, a dropped row gets an offset past the range), 8 residual row remap (r_blk, r_rep:
//   residual row = remap(m), a broadcast addend such as the decoder's per-prompt positional projection).
// BIAS_LDS: bias read from LDS (persistent kernel), else from global. Host guarantees (fast_epi) that every
// byte offset fits 31 bits: M * ld * esize without a row map, c_rows * ld * esize with one.
template <int ACT, int FE, bool BIAS_LDS, int MI0 = 0, int NMI = 8>
__device__ __forceinline__ void epilogue_fast(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0, int col0,
                                              int lane, const float* lds_bias = nullptr) {
  constexpr bool CF32 = ((FE - 1) & 1) != 0, RES = ((FE - 1) & 2) != 0, RMAP = ((FE - 1) & 4) != 0;
  constexpr bool RREMAP = ((FE - 1) & 8) != 0;
  constexpr bool RF32 = CF32 || ((FE - 1) & 16) != 0;  // bit 16: an fp32 residual under an e16 C
  constexpr int ES = CF32 ? 4 : 2, RS = RF32 ? 4 : 2;
  const int q = lane >> 4;
  const int cofs = 16 * (q & 1) + 8 * (q >> 1);
  // descriptor origin / extent and each lane's row offsets (bytes)
  const long long c_origin = RMAP ? bz * p.sC + col0 : bz * p.sC + (long long)row0 * p.ldc + col0;
  const long long r_origin = (RMAP || RREMAP) ? bz * p.sR + col0 : bz * p.sR + (long long)row0 * p.ldr + col0;
  const int rows_left = max(0, p.M - row0);
  const int c_bytes = RMAP ? p.c_rows * (int)p.ldc * ES : rows_left * (int)p.ldc * ES;
  // (a remapped residual has r_blk * ceil(M / (r_blk * r_rep)) stored rows: remap(m) < that for m < M)
  const int r_rows = RREMAP ? p.r_blk * ((p.M - 1) / (p.r_blk * p.r_rep) + 1) : 0;
  const int r_bytes = RMAP ? p.c_rows * (int)p.ldr * RS : RREMAP ? r_rows * (int)p.ldr * RS : rows_left * (int)p.ldr * RS;
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc((void*)((char*)p.C + c_origin * ES), (short)0, c_bytes, 0x00020000);
  uint32_t crow[NMI], rrow[NMI];
#pragma unroll
  for (int j = 0; j < NMI; ++j) {
    const int rl = 16 * (MI0 + j) + (lane & 15);  // row within the wave tile
    if constexpr (RMAP) {
      const int m = row0 + rl;
      const int om = m < p.M ? p.row_map[m] : -1;
      crow[j] = om >= 0 ? (uint32_t)(om * (int)p.ldc * ES) : 0x80000000u;
      rrow[j] = om >= 0 ? (uint32_t)(om * (int)p.ldr * RS) : 0x80000000u;
    } else {
      crow[j] = (uint32_t)(rl * (int)p.ldc * ES);
      rrow[j] = RREMAP ? (uint32_t)((int)remap(row0 + rl, p.r_blk, p.r_rep) * (int)p.ldr * RS)
                       : (uint32_t)(rl * (int)p.ldr * RS);
      if (RREMAP && row0 + rl >= p.M) rrow[j] = 0x80000000u;
    }
  }
  bool colok[2];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) colok[pr] = col0 + 32 * pr + cofs < p.N;
  float v[NMI][2][8];
#pragma unroll
  for (int j = 0; j < NMI; ++j)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const u32x4 x = __builtin_bit_cast(u32x4, acc[MI0 + j][2 * pr]);
      const u32x4 y = __builtin_bit_cast(u32x4, acc[MI0 + j][2 * pr + 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t xi = x[i], yi = y[i];
        const auto r = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
        v[j][pr][i] = __builtin_bit_cast(float, (uint32_t)r[0]);
        v[j][pr][4 + i] = __builtin_bit_cast(float, (uint32_t)r[1]);
      }
    }
  float bv[2][8];
  if (p.bias) {
    f32x4 t[2][2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int n = colok[pr] ? col0 + 32 * pr + cofs : 0;  // (columns past N: any in-range bias, never stored)
      if constexpr (BIAS_LDS) {
        // inline asm: hipcc would put a vmcnt(0) (the in-flight LDS-DMA prefetch) in front of an ordinary
        // LDS load; the bias region is never a DMA target
        const uint32_t ad = (uint32_t)(uintptr_t)(lds_ptr_t)(lds_bias + n);
        asm volatile("ds_read_b128 %0, %1" : "=v"(t[pr][0]) : "v"(ad));
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(t[pr][1]) : "v"(ad));
      } else {
        t[pr][0] = *(const f32x4*)(p.bias + n);
        t[pr][1] = *(const f32x4*)(p.bias + n + 4);
      }
    }
    if constexpr (BIAS_LDS) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bv[pr][e] = t[pr][0][e];
        bv[pr][4 + e] = t[pr][1][e];
      }
  } else {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[pr][e] = 0.0f;
  }
  const uint32_t cl = (uint32_t)(cofs * ES);
  float res[RES ? NMI : 1][2][8];
  if constexpr (RES) {
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc((void*)((char*)p.R + r_origin * RS), (short)0, r_bytes, 0x00020000);
#pragma unroll
    for (int j = 0; j < NMI; ++j)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        // (columns past N read as zero: their offset is sent past the range like the stores')
        const uint32_t o = colok[pr] ? rrow[j] + (uint32_t)(cofs * RS) + (uint32_t)(32 * pr * RS) : 0x80000000u;
        if constexpr (RF32) {
          const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, o, 0, 0));
          const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, o + 16, 0, 0));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            res[j][pr][e] = a[e];
            res[j][pr][4 + e] = b[e];
          }
        } else {
          const u32x4 w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, o, 0, 0));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            res[j][pr][2 * e] = lo16f(w[e]);
            res[j][pr][2 * e + 1] = hi16f(w[e]);
          }
        }
      }
  }
#pragma unroll
  for (int j = 0; j < NMI; ++j)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float o8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = act_apply<ACT>(v[j][pr][e] * p.alpha + bv[pr][e]);
        if constexpr (RES) t += res[j][pr][e];
        o8[e] = t;
      }
      // a column chunk past N is sent past the descriptor's range (dropped) instead of branching
      const uint32_t o = colok[pr] ? crow[j] + cl + (uint32_t)(32 * pr * ES) : 0x80000000u;
      if constexpr (CF32) {
        const f32x4 a = {o8[0], o8[1], o8[2], o8[3]}, b = {o8[4], o8[5], o8[6], o8[7]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rc, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), rc, o + 16, 0, 0);
      } else {
        e16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (e16)o8[e];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), rc, o, 0, 0);
      }
    }
}
// LDS-staged fp32 residual for the in-place fp32 residual kind (FE 4: the encoder's MLP2 writing the fp32 residual
// stream, C == R): the residual of a wave's 128 x 64 tile comes in four quarters (row blocks 2q, 2q+1: 32 rows x 64
// fp32 columns = 8 KiB) by LDS-DMA into a wave-private region, so no VGPR holds an in-flight residual and a quarter's
// load runs under the previous quarter's arithmetic and stores (the register form waits for each half's loads with
// the previous half's stores ahead of them in the counter). 16-B chunk c of row r sits at position c ^ (r & 15): the
// 16 rows a ds_read_b128 lane group reads at one chunk column land on 16 distinct chunk slots.
__device__ __forceinline__ void res_dma_q(const GemmK& p, int bz, int row0w, int col0w, int q, char* region, int lane) {
  const int r0 = row0w + 32 * q;
  const long long origin = (long long)bz * p.sR + (long long)r0 * p.ldr + col0w;
  const int rows_left = max(0, p.M - r0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const float*)p.R + origin), (short)0, rows_left * (int)p.ldr * 4, 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 4 * i + (lane >> 4), c = (lane & 15) ^ (r & 15);
    // (a chunk past N reads as zero: its offset is sent past the range; its columns are never stored)
    const uint32_t vo = col0w + 4 * c < p.N ? (uint32_t)((r * (int)p.ldr + 4 * c) * 4) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(region + i * 1024), 16, vo, 0, 0, 0);
  }
}

template <int ACT, int Q>
__device__ __forceinline__ void res_quarter(const GemmK& p, f32x4 (&acc)[8][4], const __amdgpu_buffer_rsrc_t& rc,
                                            int row0w, int col0w, const float (&bv)[2][8], const char* region, int lane) {
  const int q4 = lane >> 4;
  const int cofs = 16 * (q4 & 1) + 8 * (q4 >> 1);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int mi = 2 * Q + j;
    const int rl = 16 * j + (lane & 15);  // row within the quarter
    float v[2][8];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const u32x4 x = __builtin_bit_cast(u32x4, acc[mi][2 * pr]);
      const u32x4 y = __builtin_bit_cast(u32x4, acc[mi][2 * pr + 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t xi = x[i], yi = y[i];
        const auto r = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
        v[pr][i] = __builtin_bit_cast(float, (uint32_t)r[0]);
        v[pr][4 + i] = __builtin_bit_cast(float, (uint32_t)r[1]);
      }
    }
    // residual rows from LDS by inline asm: hipcc puts a vmcnt(0) (the next quarter's LDS-DMA in flight) in front of
    // an ordinary LDS load; this quarter's DMA was retired by the caller's counted wait
    f32x4 ra[2], rb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c0 = 8 * pr + (cofs >> 2);
      const uint32_t base = (uint32_t)(uintptr_t)(lds_ptr_t)(region + rl * 256);
      const uint32_t aa = base + (uint32_t)((c0 ^ (rl & 15)) << 4), ab = base + (uint32_t)(((c0 + 1) ^ (rl & 15)) << 4);
      asm volatile("ds_read_b128 %0, %1" : "=v"(ra[pr]) : "v"(aa));
      asm volatile("ds_read_b128 %0, %1" : "=v"(rb[pr]) : "v"(ab));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra[0]), "+v"(rb[0]), "+v"(ra[1]), "+v"(rb[1])::"memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const f32x4 a = ra[pr], b = rb[pr];
      float o8[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o8[e] = act_apply<ACT>(v[pr][e] * p.alpha + bv[pr][e]) + a[e];
        o8[4 + e] = act_apply<ACT>(v[pr][4 + e] * p.alpha + bv[pr][4 + e]) + b[e];
      }
      const uint32_t o = col0w + 32 * pr + cofs < p.N
                             ? (uint32_t)((((Q * 32 + rl) * (int)p.ldc) + 32 * pr + cofs) * 4)
                             : 0x80000000u;
      const f32x4 oa = {o8[0], o8[1], o8[2], o8[3]}, ob = {o8[4], o8[5], o8[6], o8[7]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, oa), rc, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ob), rc, o + 16, 0, 0);
    }
  }
}

// the four quarters: Q0 already in flight in bufX (issued during the last K-step), Q1 -> bufY, Q2 -> bufX, Q3 -> bufY,
// each issued as soon as its region's previous quarter has been read; counted waits (each quarter's 8 stores and the
// next quarter's 8 DMA ops may stay in flight)
template <int ACT>
__device__ __forceinline__ void epilogue_res_lds(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0w, int col0w,
                                                 int lane, char* bufX, char* bufY) {
  const int q4 = lane >> 4;
  const int cofs = 16 * (q4 & 1) + 8 * (q4 >> 1);
  f32x4 bt[2][2];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const int n = col0w + 32 * pr + cofs;
    const bool ok = p.bias && n < p.N;
    bt[pr][0] = ok ? *(const f32x4*)(p.bias + n) : (f32x4)0.0f;
    bt[pr][1] = ok ? *(const f32x4*)(p.bias + n + 4) : (f32x4)0.0f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Q0 and the bias
  // (the bias consumed here, before any LDS-DMA is issued: hipcc waits vmcnt(0) at the first use of an ordinary load's
  //  result while an LDS-DMA is in flight)
  asm volatile("" : "+v"(bt[0][0]), "+v"(bt[0][1]), "+v"(bt[1][0]), "+v"(bt[1][1]));
  float bv[2][8];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bv[pr][e] = bt[pr][0][e];
      bv[pr][4 + e] = bt[pr][1][e];
    }
  const long long c_origin = (long long)bz * p.sC + (long long)row0w * p.ldc + col0w;
  const int rows_left = max(0, p.M - row0w);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)((float*)p.C + c_origin), (short)0,
                                                                      rows_left * (int)p.ldc * 4, 0x00020000);
  res_dma_q(p, bz, row0w, col0w, 1, bufY, lane);
  res_quarter<ACT, 0>(p, acc, rc, row0w, col0w, bv, bufX, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // Q0 read before its region is refilled
  res_dma_q(p, bz, row0w, col0w, 2, bufX, lane);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // Q1 (Q0's stores and Q2's DMA may stay in flight)
  res_quarter<ACT, 1>(p, acc, rc, row0w, col0w, bv, bufY, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  res_dma_q(p, bz, row0w, col0w, 3, bufY, lane);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // Q2
  res_quarter<ACT, 2>(p, acc, rc, row0w, col0w, bv, bufX, lane);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // Q3 (Q2's stores may stay in flight)
  res_quarter<ACT, 3>(p, acc, rc, row0w, col0w, bv, bufY, lane);
}
}  // namespace ph8

// TR (register epilogue): operands swapped, the accumulator holds each 16x16 block transposed
#define PH8_MFMA_QUAD(MH, NH, BF)                                                                       \
  __builtin_amdgcn_s_setprio(1);                                                                        \
  _Pragma("unroll") for (int kb = 0; kb < 2; ++kb)                                                     \
  _Pragma("unroll") for (int mi = 0; mi < 4; ++mi)                                                     \
  _Pragma("unroll") for (int ni = 0; ni < 2; ++ni)                                                     \
    acc[(MH) * 4 + mi][(NH) * 2 + ni] =                                                                 \
        TR ? mma16(BF[ni][kb], af[mi][kb], acc[(MH) * 4 + mi][(NH) * 2 + ni], 0, 0, 0) \
           : mma16(af[mi][kb], BF[ni][kb], acc[(MH) * 4 + mi][(NH) * 2 + ni], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);
// first K-step of a tile: the kb = 0 MFMAs take an inline-constant zero accumulator (no per-tile zeroing of
// the 128 accumulator registers)
#define PH8_MFMA_QUAD_Z(MH, NH, BF)                                                                     \
  __builtin_amdgcn_s_setprio(1);                                                                        \
  _Pragma("unroll") for (int kb = 0; kb < 2; ++kb)                                                     \
  _Pragma("unroll") for (int mi = 0; mi < 4; ++mi)                                                     \
  _Pragma("unroll") for (int ni = 0; ni < 2; ++ni)                                                     \
    acc[(MH) * 4 + mi][(NH) * 2 + ni] =                                                                 \
        TR ? mma16(BF[ni][kb], af[mi][kb], kb == 0 ? (f32x4)0.0f : acc[(MH) * 4 + mi][(NH) * 2 + ni], 0, 0, 0) \
           : mma16(af[mi][kb], BF[ni][kb], kb == 0 ? (f32x4)0.0f : acc[(MH) * 4 + mi][(NH) * 2 + ni], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);
#define PH8_MFMA_QUAD_F(MH, NH, BF, FIRST) \
  if (FIRST) {                             \
    PH8_MFMA_QUAD_Z(MH, NH, BF)            \
  } else {                                 \
    PH8_MFMA_QUAD(MH, NH, BF)              \
  }

// EPI < 0: LDS-staged epilogue; EPI >= 0: register epilogue with activation EPI (operand-swapped MFMA).
// FE: 0 = general register epilogue, else the lean buffer epilogue of that kind (epilogue_fast; needs
// N % 256 == 0; one epilogue per instantiation keeps the register allocation spill-free)
// DBG 3 (diagnostics, octsam_gemm_debug_stamps): per workgroup s_memtime at entry, after the main loop and after
// the epilogue's stores have completed, plus the hardware ids (XCC, CU) -- how long each phase takes in the real
// kernel and how aligned the workgroups' epilogues are across the chip.
constexpr int STAMP_WG = 8192;
__device__ long long g_stamps[STAMP_WG * 4];

template <int DBG, int EPI, int FE = 0>
__global__ __launch_bounds__(512, 2) void gemm8_kernel(GemmK p) {
  constexpr bool TR = EPI >= 0;
  // the in-place fp32 residual kind stages its residual through LDS (ph8::epilogue_res_lds; p.res_lds, fast path
  // bit 4096 turns it off for A/B)
  constexpr bool RES_LDS = TR && FE == 4 && DBG == 0;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  long long st0 = 0, st1 = 0;
  if constexpr (DBG == 3) st0 = __builtin_amdgcn_s_memtime();
  const int wr = wave >> 2, wc = wave & 3;
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int per_batch = p.tiles_m * p.tiles_n;
  const int bz = bid / per_batch, rem = bid - bz * per_batch;
  const int tm = rem / p.tiles_n, tn = rem - tm * p.tiles_n;
  const int row0 = tm * 256, col0 = tn * 256;
  const e16* A = (const e16*)p.A + bz * p.sA;
  const e16* B = (const e16*)p.B + bz * p.sB;
  const int nk = p.K / 64;

  f32x4 acc[8][4];  // written by the first K-step's zero-accumulator MFMAs
  if (DBG == 2 || p.K < 64) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)0.0f;
  }
  e16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = wr * 128 + (lane & 15), brow = wc * 64 + (lane & 15), kq = lane >> 4;

  // prologue: K-tile 0 (A-lo, B-n0 | B-n1 | A-hi), K-tile 1 (A-lo, B-n0 | B-n1)
  ph8::load_region(p, A, B, 0, row0, col0, 0, gsm, wave, lane);
  ph8::load_region(p, A, B, 2, row0, col0, 0, gsm, wave, lane);
  ph8::load_region(p, A, B, 3, row0, col0, 0, gsm, wave, lane);
  ph8::load_region(p, A, B, 1, row0, col0, 0, gsm, wave, lane);
  if (nk > 1) {
    ph8::load_region(p, A, B, 0, row0, col0, 64, gsm + ph8::BUF, wave, lane);
    ph8::load_region(p, A, B, 2, row0, col0, 64, gsm + ph8::BUF, wave, lane);
    ph8::load_region(p, A, B, 3, row0, col0, 64, gsm + ph8::BUF, wave, lane);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();

  for (int t = 0; t < (DBG == 2 ? 0 : nk); ++t) {
    char* cur = gsm + (t & 1) * ph8::BUF;
    char* nxt = gsm + ((t + 1) & 1) * ph8::BUF;
    const char* ca = cur;
    const char* cb = cur + 32768;
    const bool h1 = t + 1 < nk, h2 = t + 2 < nk;
    // ---- phase 0: Q(0,0) — A-lo, B-n0
    if (h1) ph8::load_region(p, A, B, 1, row0, col0, (t + 1) * 64, nxt, wave, lane);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + mi * 16, kb * 4 + kq);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b0[ni][kb] = ph8::frag(cb, brow + ni * 16, kb * 4 + kq);
    }
    if (h1) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // retire B-n1(t)
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(0, 0, b0, t == 0)
    raw_barrier();
    // ---- phase 1: Q(0,1) — B-n1
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b1[ni][kb] = ph8::frag(cb, brow + 32 + ni * 16, kb * 4 + kq);
    if (h1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // retire A-hi(t)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (RES_LDS)  // last K-step: the first residual quarter into the buffer no K-tile needs any more
      if (!h1 && p.res_lds) ph8::res_dma_q(p, bz, row0 + wr * 128, col0 + wc * 64, 0, nxt + wave * 8192, lane);
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(0, 1, b1, t == 0)
    raw_barrier();
    // ---- phase 2: Q(1,0) — A-hi; restage A-lo, B-n0 of K-tile t+2
    if (h2) {
      ph8::load_region(p, A, B, 0, row0, col0, (t + 2) * 64, cur, wave, lane);
      ph8::load_region(p, A, B, 2, row0, col0, (t + 2) * 64, cur, wave, lane);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + 64 + mi * 16, kb * 4 + kq);
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(1, 0, b0, t == 0)
    raw_barrier();
    // ---- phase 3: Q(1,1); restage B-n1 of K-tile t+2; retire A-lo, B-n0 of K-tile t+1
    if (h2) ph8::load_region(p, A, B, 3, row0, col0, (t + 2) * 64, cur, wave, lane);
    if (h2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (h1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    raw_barrier();
    PH8_MFMA_QUAD_F(1, 1, b1, t == 0)
    raw_barrier();
  }
  if (wr == 0) raw_barrier();  // balance the stagger
  if (DBG == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DBG == 3) st1 = __builtin_amdgcn_s_memtime();
  if (DBG == 1) {
    float x = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) x += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (x == 12345.f) ((float*)p.C)[0] = x;
    return;
  }
  if constexpr (RES_LDS) {
    if (p.res_lds) {  // (buffer nk & 1 holds residual quarter 0 since the last K-step; nk + 1 is free now)
      ph8::epilogue_res_lds<EPI>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane, gsm + (nk & 1) * ph8::BUF + wave * 8192,
                                 gsm + ((nk + 1) & 1) * ph8::BUF + wave * 8192);
      return;
    }
  }
  if constexpr (TR) {
    if constexpr (FE == 1) {
      ph8::epilogue_fast<EPI, FE, false>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
    } else if constexpr (FE > 1) {  // halves: the residual / fp32 temporaries fit beside the accumulator
      ph8::epilogue_fast<EPI, FE, false, 0, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
      ph8::epilogue_fast<EPI, FE, false, 4, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
    } else {
      ph8::epilogue_reg<EPI>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
    }
  } else {
    ph8::epilogue_lds(p, acc, bz, row0, col0, wr, wc, wave, lane, gsm);
  }
  if constexpr (DBG == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const long long st2 = __builtin_amdgcn_s_memtime();
    if (tid == 0 && blockIdx.x < STAMP_WG) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
      long long* d = g_stamps + 4 * blockIdx.x;
      d[0] = st0;
      d[1] = st1;
      d[2] = st2;
      d[3] = ((long long)xcc << 32) | hw;
    }
  }
}

template <int DBG, int EPI, int FE = 0>
int launch_gemm8_fe(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = (a->N + 255) / 256;
  constexpr int LDS = EPI < 0 ? ph8::EPI_BYTES : 2 * ph8::BUF;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8_kernel<DBG, EPI, FE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS);
    attr = true;
  }
  const long long nwg = (long long)g.tiles_m * g.tiles_n * a->batch;
  hipLaunchKernelGGL((gemm8_kernel<DBG, EPI, FE>), dim3((unsigned)nwg), dim3(512), LDS, s, g);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

// ------------------------------------------------------------------------------------------------
// 256x192 variant of the 8-phase kernel for GEMMs whose 256-column tiles quantise badly on the chip (MLP2 /
// proj at M = 32768, N = 768: 384 tiles = 1.5 waves of 256 CUs -> 512 tiles of 3/4 the work = 2 full waves).
// Same phases, barriers and stagger; each wave owns 128 x 48 (3 column blocks of 16): Q(., 0) covers blocks
// 0-1 (B-n0, 32 columns), Q(., 1) block 2 (B-n1, 16 columns). B-n1 is 64 rows per K-tile, one LDS-DMA op per
// wave (A-lo, A-hi, B-n0 two each), so the counted waits are 9 / 7 / 8 in steady state (see launch notes).
namespace ph8 {
constexpr int BUF192 = 32768 + 192 * 128;  // A [256][64] + B [192][64] e16

__device__ __forceinline__ void load_region192(const GemmK& p, const e16* A, const e16* B, int region, int row0,
                                               int col0, int k0, char* buf, int wave, int lane) {
  if (region < 2) {
    load_region(p, A, B, region, row0, col0, k0, buf, wave, lane);
    return;
  }
  const int nops = region == 2 ? 2 : 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u >= nops) break;
    int rbase;
    if (region == 2) {
      const int j = wave * 2 + u;  // 16 groups of 8 rows: columns 0..31 of each wave column
      rbase = (j >> 2) * 48 + (j & 3) * 8;
    } else {
      const int j = wave;  // 8 groups: columns 32..47 of each wave column
      rbase = (j >> 1) * 48 + 32 + (j & 1) * 8;
    }
    const int r = rbase + (lane >> 3), slot = lane & 7;
    const int c = slot ^ ((r >> 1) & 7);
    int gr = col0 + r;
    gr = gr < p.N ? gr : p.N - 1;
    const e16* g = B + (long long)gr * p.ldb + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_ptr_t)(buf + 32768 + rbase * 128), 16, 0, 0);
  }
}

// lean epilogue of a 128 x 48 wave tile: columns 0..31 (blocks 0, 1) as in epilogue_fast (permlane16_swap
// to 8 consecutive columns per lane), columns 32..47 (block 2) straight from the transposed block: 4
// consecutive columns per lane. FE as in epilogue_fast (kinds 1: e16 C, 4: fp32 C + in-place fp32 residual).
template <int ACT, int FE, int MI0, int NMI>
__device__ __forceinline__ void epilogue_n192(const GemmK& p, f32x4 (&acc)[8][3], int bz, int row0, int col0,
                                              int lane) {
  constexpr bool CF32 = FE == 4, RES = FE == 4;
  static_assert(FE == 1 || FE == 4, "n192 epilogue kinds: 1 (e16 C), 4 (fp32 C + fp32 residual)");
  constexpr int ES = CF32 ? 4 : 2;
  const int q = lane >> 4;
  const int cofs = 16 * (q & 1) + 8 * (q >> 1);
  const int rows_left = max(0, p.M - row0);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((char*)p.C + (bz * p.sC + (long long)row0 * p.ldc + col0) * ES), (short)0,
      rows_left * (int)p.ldc * ES, 0x00020000);
  __amdgpu_buffer_rsrc_t rr = rc;
  if constexpr (RES)
    rr = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)p.R + (bz * p.sR + (long long)row0 * p.ldr + col0) * ES),
                                           (short)0, rows_left * (int)p.ldr * ES, 0x00020000);
  // bias: 8 columns (pair part) + 4 columns (block 2) per lane
  float bp[8], bt[4];
  if (p.bias) {
    const f32x4 x0 = *(const f32x4*)(p.bias + col0 + cofs), x1 = *(const f32x4*)(p.bias + col0 + cofs + 4);
    const f32x4 x2 = *(const f32x4*)(p.bias + col0 + 32 + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bp[e] = x0[e];
      bp[4 + e] = x1[e];
      bt[e] = x2[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) bp[e] = 0.0f;
#pragma unroll
    for (int e = 0; e < 4; ++e) bt[e] = 0.0f;
  }
#pragma unroll
  for (int jj = 0; jj < NMI; ++jj) {
    const int j = MI0 + jj;
    const uint32_t rowoff = (uint32_t)((16 * j + (lane & 15)) * (int)p.ldc * ES);
    const uint32_t rowoff_r = (uint32_t)((16 * j + (lane & 15)) * (int)p.ldr * ES);
    // blocks 0, 1 -> 8 consecutive columns
    float v[8];
    {
      const u32x4 x = __builtin_bit_cast(u32x4, acc[j][0]);
      const u32x4 y = __builtin_bit_cast(u32x4, acc[j][1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t xi = x[i], yi = y[i];
        const auto r = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
        v[i] = __builtin_bit_cast(float, (uint32_t)r[0]);
        v[4 + i] = __builtin_bit_cast(float, (uint32_t)r[1]);
      }
    }
    float w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = acc[j][2][i];
    const uint32_t op = rowoff + (uint32_t)(cofs * ES), ot = rowoff + (uint32_t)((32 + 4 * q) * ES);
    const uint32_t opr = rowoff_r + (uint32_t)(cofs * ES), otr = rowoff_r + (uint32_t)((32 + 4 * q) * ES);
    float rp[8], rt[4];
    if constexpr (RES) {
      const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, opr, 0, 0));
      const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, opr + 16, 0, 0));
      const f32x4 c = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, otr, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rp[e] = a[e];
        rp[4 + e] = b[e];
        rt[e] = c[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = act_apply<ACT>(v[e] * p.alpha + bp[e]);
      if constexpr (RES) v[e] += rp[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      w[e] = act_apply<ACT>(w[e] * p.alpha + bt[e]);
      if constexpr (RES) w[e] += rt[e];
    }
    if constexpr (CF32) {
      const f32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]}, c = {w[0], w[1], w[2], w[3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rc, op, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), rc, op + 16, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, c), rc, ot, 0, 0);
    } else {
      e16x8 h;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = (e16)v[e];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), rc, op, 0, 0);
      e16x4 t4;
#pragma unroll
      for (int e = 0; e < 4; ++e) t4[e] = (e16)w[e];
      typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, t4), rc, ot, 0, 0);
    }
  }
}
}  // namespace ph8

// ------------------------------------------------------------------------------------------------
// Ping-pong 8-wave kernel (gemm8w): the same 256x256x64 tile, wave tiles (2 M x 4 N waves of 128 x 64), LDS
// images and epilogues as gemm8, but each K-step of a wave is TWO segments between barriers instead of eight:
//   L(t): the wave's 24 fragments of K-step t (8 A row blocks, 4 B column blocks, 2 k-halves; ds_read_b128 by
//         inline asm into registers) plus its share of the LDS-DMA for later stages;
//   C(t): all 64 of its 16x16x32 MFMAs of K-step t (1024 MFMA cycles, no LDS access).
// The two wave rows run one segment apart (waves w and w+4 share a SIMD), so every segment pairs one wave's
// matrix cluster with its SIMD partner's loads; gemm8's phases were 16 MFMAs (256 cycles) per barrier.
// Stage t lives in buffer t & 1 ([A 256 x 64 | B 256 x 64] e16, 64 KiB); A rows 0-127 are read only by wave row
// 0 (segment 2t), rows 128-255 only by wave row 1 (segment 2t+1), B by both, so each region is refilled as soon
// as its last reader has passed a barrier, with the DMA split evenly over the loading waves:
//   wave row 0 in L(t) (segment 2t):     B(t+1)                    -> landed at the end of its C(t): vmcnt(0)
//   wave row 1 in L(t) (segment 2t+1):   A-hi(t+1), A-lo(t+2)      -> A-hi(t+1) landed at the end of its C(t)
//                                                                     (vmcnt 4), A-lo(t+1) (issued in L(t-1))
//                                                                     at the end of L(t) (vmcnt 8)
//   prologue (all waves): stage 0 and A-lo(1).
// Operands through buffer descriptors (rows past M / N read as zero); each 1 KiB DMA piece is 8 rows x 128 B, its
// lane part of the offset depends only on the piece's parity (the chunk swizzle (r >> 1) & 7 of sw_off<64>).
namespace pp8 {
__device__ __forceinline__ void rd(e16x8& d, const char* base, int off) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"((uint32_t)(uintptr_t)(lds_ptr_t)(base + off)));
}

// The ping-pong main loop over K-steps [kb0, kb0 + n) of one 256x256 tile (n >= 1): acc = sum over those K-steps
// (the first K-step's MFMAs start from zero). Stage t of the loop lives in buffer t & 1. Every wave enters and leaves
// with the same barrier count (wave row 1 takes one extra at the start and skips the last); on return wave row 0 is
// one segment ahead (its epilogue overlaps wave row 1's last MFMA cluster) and every LDS read of the loop is done.
// SKIP (diagnostics, wrong results): bit 1 no DMA after the prologue, bit 2 no fragment reads, bit 4 no MFMAs;
// bit 8: the DMA pieces are issued in the wave's MFMA segment (one after every 4 MFMAs) instead of its load segment;
// bit 16: the load segment issues its DMA share before its fragment reads
// NB: 16-column blocks per wave (4: the 256x256 tile; 3: 256x192, B 192 rows x 64 k per stage, 2 * NB DMA pieces per
// wave of row 0 per K-step instead of 8; every wait count is unchanged, wave row 0 waits for all of its pieces)
template <bool ZACC = true, int SKIP = 0, int NB = 4>  // ZACC: the first K-step's MFMAs start from zero (else from acc: zeroed)
__device__ __forceinline__ void mainloop(const GemmK& p, const e16* A, const e16* B, int row0, int col0, int kb0, int n,
                                         f32x4 (&acc)[8][NB], char* gsm, int wave, int lane) {
  static_assert(NB == 3 || NB == 4, "gemm8w: 256- or 192-column tiles");
  const int wr = wave >> 2, wc = wave & 3;
  const int lda2 = (int)p.lda * 2, ldb2 = (int)p.ldb * 2;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (long long)row0 * p.lda), (short)0, (p.M - row0) * lda2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B + (long long)col0 * p.ldb), (short)0, (p.N - col0) * ldb2, 0x00020000);
  uint32_t va[2], vb[2];  // lane part of a DMA piece's offset (by the piece's parity: the chunk swizzle of sw_off<64>)
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int r = e * 8 + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    va[e] = (uint32_t)(r * lda2 + c * 16);
    vb[e] = (uint32_t)(r * ldb2 + c * 16);
  }
  // piece j (8 rows) of A rows [h*128, h*128+128) / of B, loop stage t (K-step kb0 + t) into buffer t & 1
  auto dma_a = [&](int h, int j, int t) {
    char* dst = gsm + (t & 1) * ph8::BUF + (h * 128 + j * 8) * 128;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)dst, 16, va[j & 1],
                                             (h * 128 + (j & ~1) * 8) * lda2 + (kb0 + t) * 128, 0, 0);
  };
  auto dma_b = [&](int j, int t) {
    char* dst = gsm + (t & 1) * ph8::BUF + 32768 + j * 8 * 128;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)dst, 16, vb[j & 1],
                                             (j & ~1) * 8 * ldb2 + (kb0 + t) * 128, 0, 0);
  };
  e16x8 af[8][2], bf[NB][2];
  const int arow = wr * 128 + (lane & 15), brow = wc * 16 * NB + (lane & 15), kq = lane >> 4;

  // prologue: stage 0 (A-lo 2, A-hi 2, B NB pieces per wave) and A-lo(1) (2 per wave)
#pragma unroll
  for (int i = 0; i < 2; ++i) dma_a(0, wave * 2 + i, 0);
#pragma unroll
  for (int i = 0; i < 2; ++i) dma_a(1, wave * 2 + i, 0);
#pragma unroll
  for (int i = 0; i < NB; ++i) dma_b(wave * NB + i, 0);
  if (n > 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i) dma_a(0, wave * 2 + i, 1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();  // wave row 1 runs one segment behind

  for (int t = 0; t < n; ++t) {
    const char* cur = gsm + (t & 1) * ph8::BUF;
    // ---- L(t): the fragments of K-step t, then the DMA share, whose issue (~60+ cycles a piece) then overlaps the
    // reads' latency instead of delaying them (qkv 120.6 -> 117.9 us, MLP2 (bf16 out) 134.7 -> 128.9,
    // profiles/r06/gemm8w_rdfirst_ab.log; SKIP bit 16: the DMA share first, the first form, for A/B)
    constexpr bool DMA_IN_C = (SKIP & 8) != 0, READS_FIRST = (SKIP & 16) == 0;
    auto issue_dma = [&]() {
    if ((SKIP & 1) || DMA_IN_C) {
    } else if (wr == 0) {
      if (t + 1 < n) {
#pragma unroll
        for (int i = 0; i < 2 * NB; ++i) dma_b(wc * 2 * NB + i, t + 1);
      }
    } else {
      if (t + 1 < n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dma_a(1, wc * 4 + i, t + 1);
      }
      if (t + 2 < n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dma_a(0, wc * 4 + i, t + 2);
      }
    }
    };
    if (!READS_FIRST) issue_dma();
#pragma unroll
    for (int kb = 0; kb < 2 && !(SKIP & 2); ++kb) {
#pragma unroll
      for (int ni = 0; ni < NB; ++ni) rd(bf[ni][kb], cur + 32768, sw_off<64>(brow + ni * 16, kb * 4 + kq));
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rd(af[mi][kb], cur, sw_off<64>(arow + mi * 16, kb * 4 + kq));
    }
    if (READS_FIRST) issue_dma();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (wr == 1 && DMA_IN_C) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A-lo(t+1), issued in C(t-1)
    } else if (wr == 1) {  // A-lo(t+1), issued in L(t-1), before wave row 0 reads it in the next segment
      if (t + 2 < n) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (t + 1 < n) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    // ---- C(t): the wave's 64 MFMAs
    if constexpr ((SKIP & 4) != 0) {
      if (t == 0)
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni) acc[mi][ni] = __builtin_bit_cast(f32x4, af[mi][0]) + __builtin_bit_cast(f32x4, bf[ni][1]);
    } else if (!DMA_IN_C && ZACC && t == 0) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc[mi][ni] = mma16(bf[ni][kb], af[mi][kb], kb == 0 ? (f32x4)0.0f : acc[mi][ni], 0, 0, 0);
    } else if (DMA_IN_C) {
      // the wave's DMA share, one piece after every 4 MFMAs (sched_group_barrier: 4 MFMA, 1 VMEM)
      const bool z = ZACC && t == 0;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc[mi][ni] = mma16(bf[ni][kb], af[mi][kb], (z && kb == 0) ? (f32x4)0.0f : acc[mi][ni], 0, 0, 0);
          const int q = kb * 8 + mi;
          if (q < 8) {
            if (wr == 0) {
              if (t + 1 < n && q < 2 * NB) dma_b(wc * 2 * NB + q, t + 1);
            } else if (q < 4) {
              if (t + 1 < n) dma_a(1, wc * 4 + q, t + 1);
            } else {
              if (t + 2 < n) dma_a(0, wc * 4 + q - 4, t + 2);
            }
          }
        }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni) acc[mi][ni] = mma16(bf[ni][kb], af[mi][kb], acc[mi][ni], 0, 0, 0);
    }
    if (wr == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // B(t+1)
      raw_barrier();
    } else {
      if (t + 2 < n) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A-hi(t+1)
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (t + 1 < n) raw_barrier();
    }
  }
}

// the tile's epilogue (the lean kinds of epilogue_fast; the in-place fp32 residual through LDS, ph8::epilogue_res_lds,
// in the LDS the main loop no longer reads)
template <int EPI, int FE>
__device__ __forceinline__ void epilogue(const GemmK& p, f32x4 (&acc)[8][4], int bz, int row0w, int col0w, char* gsm,
                                         int wave, int lane) {
  if constexpr (FE == 4) {
    if (p.res_lds) {
      char* bx = gsm + wave * 8192;
      ph8::res_dma_q(p, bz, row0w, col0w, 0, bx, lane);
      ph8::epilogue_res_lds<EPI>(p, acc, bz, row0w, col0w, lane, bx, gsm + ph8::BUF + wave * 8192);
      return;
    }
  }
  if constexpr (FE == 1) {
    ph8::epilogue_fast<EPI, FE, false>(p, acc, bz, row0w, col0w, lane);
  } else {
    ph8::epilogue_fast<EPI, FE, false, 0, 4>(p, acc, bz, row0w, col0w, lane);
    ph8::epilogue_fast<EPI, FE, false, 4, 4>(p, acc, bz, row0w, col0w, lane);
  }
}
}  // namespace pp8

// DBG 3 (diagnostics, fast path 9): per workgroup s_memtime at entry, at the end of wave row 0's and of wave row 1's
// main loop and after the epilogue's stores (octsam_gemm_debug_stamps)
// NB = 3: 256x192 tiles (the 192-column main loop; the lean epilogue of a 128 x 48 wave tile, ph8::epilogue_n192)
template <int EPI, int FE, int DBG = 0, int NB = 4>
__global__ __launch_bounds__(512, 2) void gemm8w_kernel(GemmK p) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  long long st0 = 0;
  if constexpr (DBG == 3) st0 = __builtin_amdgcn_s_memtime();
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int per_batch = p.tiles_m * p.tiles_n;
  const int bz = bid / per_batch, rem = bid - bz * per_batch;
  const int tm = rem / p.tiles_n, tn = rem - tm * p.tiles_n;
  const int row0 = tm * 256, col0 = tn * 64 * NB;
  f32x4 acc[8][NB];
  pp8::mainloop<true, (DBG >= 16 ? DBG - 16 : 0), NB>(p, (const e16*)p.A + bz * p.sA, (const e16*)p.B + bz * p.sB, row0,
                                                       col0, 0, p.K / 64, acc, gsm, wave, lane);
  if constexpr (DBG == 3) {
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((wave & 3) == 0 && lane == 0 && blockIdx.x < STAMP_WG) g_stamps[4 * blockIdx.x + 1 + wr] = t1;
  }
  if constexpr (NB == 3) {
    static_assert(FE == 1 || FE == 4, "gemm8w 192-column tiles: epilogue kinds 1 and 4");
    if constexpr (FE == 1) {
      ph8::epilogue_n192<EPI, FE, 0, 8>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
    } else {
      ph8::epilogue_n192<EPI, FE, 0, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
      ph8::epilogue_n192<EPI, FE, 4, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
    }
  } else {
    pp8::epilogue<EPI, FE>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, gsm, wave, lane);
  }
  if constexpr (DBG == 3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const long long t2 = __builtin_amdgcn_s_memtime();
    if (tid == 0 && blockIdx.x < STAMP_WG) {
      g_stamps[4 * blockIdx.x] = st0;
      g_stamps[4 * blockIdx.x + 3] = t2;
    }
  }
}

template <int EPI, int FE, int DBG = 0, int NB = 4>
int launch_gemm8w_fe(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = NB == 4 ? (a->N + 255) / 256 : a->N / 192;  // (192: N % 192 == 0 host-checked)
  constexpr int LDS = 2 * ph8::BUF;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8w_kernel<EPI, FE, DBG, NB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS);
    attr = true;
  }
  const long long nwg = (long long)g.tiles_m * g.tiles_n * a->batch;
  hipLaunchKernelGGL((gemm8w_kernel<EPI, FE, DBG, NB>), dim3((unsigned)nwg), dim3(512), LDS, s, g);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

static int g_small_oneshot = 1;  // K <= 256 small problems on gemm_small_kernel (fast path bit 65536 turns it off)
static int g_pp_skip = 0;  // diagnostics (fast path bits 0x100000 << {0,1,2}): gemm8w main loop parts skipped
// 256x192 ping-pong tiles where they fill the chip's waves better (fast path bit 262144 turns them on): opt-in, since
// in the step they lose although they win in isolation — MLP2 163.9 -> 154.2 us, projection 63.7 -> 60.7 (QKV 121.7
// -> 123.9), but the pipelined step 16.00 -> 16.48 ms and the sequential 18.19 -> 18.27 (profiles/r06/n192w_ab.log,
// n192w_step_ab.log): the 1.5-wave 256x256 launches leave half the chip to the decoder stream in their last wave
static int g_n192w = 0;

// kinds of the ping-pong kernel (-1: not built for this kind, the caller takes gemm8)
template <int EPI>
int launch_gemm8w(const GemmK& k, const octsam_gemm_args* a, hipStream_t s, bool stamped = false) {
  if (g_pp_skip) {  // (diagnostics: the main loop without DMA / fragment reads / MFMAs; wrong results)
    if (k.fast_epi != 1) return -1;
    switch (g_pp_skip) {
      case 1: return launch_gemm8w_fe<EPI, 1, 17>(k, a, s);
      case 2: return launch_gemm8w_fe<EPI, 1, 18>(k, a, s);
      case 4: return launch_gemm8w_fe<EPI, 1, 20>(k, a, s);
      case 3: return launch_gemm8w_fe<EPI, 1, 19>(k, a, s);
      case 5: return launch_gemm8w_fe<EPI, 1, 24>(k, a, s);  // (fast path bits: 5 << 20 = DMA in the MFMA segment)
      case 6: return launch_gemm8w_fe<EPI, 1, 32>(k, a, s);  // (6 << 20: the DMA share before the fragments)
      default: return -1;
    }
  }
  if (stamped) {  // (diagnostics)
    if (k.fast_epi == 1) return launch_gemm8w_fe<EPI, 1, 3>(k, a, s);
    if (k.fast_epi == 4) return launch_gemm8w_fe<EPI, 4, 3>(k, a, s);
    return -1;
  }
  switch (k.fast_epi) {
    case 1: return launch_gemm8w_fe<EPI, 1>(k, a, s);
    case 2: return launch_gemm8w_fe<EPI, 2>(k, a, s);
    case 4: return launch_gemm8w_fe<EPI, 4>(k, a, s);
    case 8: return launch_gemm8w_fe<EPI, 8>(k, a, s);
    default: return -1;
  }
}


#define PH8_MFMA_N192(MH, NH, BF, NNI, FIRST)                                                            \
  __builtin_amdgcn_s_setprio(1);                                                                          \
  _Pragma("unroll") for (int kb = 0; kb < 2; ++kb)                                                       \
  _Pragma("unroll") for (int mi = 0; mi < 4; ++mi)                                                       \
  _Pragma("unroll") for (int ni = 0; ni < NNI; ++ni)                                                     \
    acc[(MH) * 4 + mi][(NH) * 2 + ni] = mma16(BF[ni][kb], af[mi][kb],                                     \
        (FIRST && kb == 0) ? (f32x4)0.0f : acc[(MH) * 4 + mi][(NH) * 2 + ni], 0, 0, 0);                   \
  __builtin_amdgcn_s_setprio(0);

template <int EPI, int FE>
__global__ __launch_bounds__(512, 2) void gemm8n192_kernel(GemmK p) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int per_batch = p.tiles_m * p.tiles_n;
  const int bz = bid / per_batch, rem = bid - bz * per_batch;
  const int tm = rem / p.tiles_n, tn = rem - tm * p.tiles_n;
  const int row0 = tm * 256, col0 = tn * 192;
  const e16* A = (const e16*)p.A + bz * p.sA;
  const e16* B = (const e16*)p.B + bz * p.sB;
  const int nk = p.K / 64;

  f32x4 acc[8][3];  // written by the first K-step's zero-accumulator MFMAs (K >= 64 host-checked)
  e16x8 af[4][2], b0[2][2], b1[1][2];
  const int arow = wr * 128 + (lane & 15), brow = wc * 48 + (lane & 15), kq = lane >> 4;

  // prologue: K-tile 0 (A-lo, B-n0 | B-n1 | A-hi), K-tile 1 (A-lo, B-n0 | B-n1); ops per wave 2,2,1,2 | 2,2,1
  ph8::load_region192(p, A, B, 0, row0, col0, 0, gsm, wave, lane);
  ph8::load_region192(p, A, B, 2, row0, col0, 0, gsm, wave, lane);
  ph8::load_region192(p, A, B, 3, row0, col0, 0, gsm, wave, lane);
  ph8::load_region192(p, A, B, 1, row0, col0, 0, gsm, wave, lane);
  if (nk > 1) {
    ph8::load_region192(p, A, B, 0, row0, col0, 64, gsm + ph8::BUF192, wave, lane);
    ph8::load_region192(p, A, B, 2, row0, col0, 64, gsm + ph8::BUF192, wave, lane);
    ph8::load_region192(p, A, B, 3, row0, col0, 64, gsm + ph8::BUF192, wave, lane);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A-lo, B-n0 of K-tile 0 landed
  } else {
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();

  for (int t = 0; t < nk; ++t) {
    char* cur = gsm + (t & 1) * ph8::BUF192;
    char* nxt = gsm + ((t + 1) & 1) * ph8::BUF192;
    const char* ca = cur;
    const char* cb = cur + 32768;
    const bool h1 = t + 1 < nk, h2 = t + 2 < nk;
    const bool first = t == 0;
    // ---- phase 0: Q(0,0) — A-lo, B-n0
    if (h1) ph8::load_region192(p, A, B, 1, row0, col0, (t + 1) * 64, nxt, wave, lane);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + mi * 16, kb * 4 + kq);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b0[ni][kb] = ph8::frag(cb, brow + ni * 16, kb * 4 + kq);
    }
    if (h1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // retire B-n1(t)
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (first) { PH8_MFMA_N192(0, 0, b0, 2, true) } else { PH8_MFMA_N192(0, 0, b0, 2, false) }
    raw_barrier();
    // ---- phase 1: Q(0,1) — B-n1
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) b1[0][kb] = ph8::frag(cb, brow + 32, kb * 4 + kq);
    if (h1) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // retire A-hi(t)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (first) { PH8_MFMA_N192(0, 1, b1, 1, true) } else { PH8_MFMA_N192(0, 1, b1, 1, false) }
    raw_barrier();
    // ---- phase 2: Q(1,0) — A-hi; restage A-lo, B-n0 of K-tile t+2
    if (h2) {
      ph8::load_region192(p, A, B, 0, row0, col0, (t + 2) * 64, cur, wave, lane);
      ph8::load_region192(p, A, B, 2, row0, col0, (t + 2) * 64, cur, wave, lane);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + 64 + mi * 16, kb * 4 + kq);
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (first) { PH8_MFMA_N192(1, 0, b0, 2, true) } else { PH8_MFMA_N192(1, 0, b0, 2, false) }
    raw_barrier();
    // ---- phase 3: Q(1,1); restage B-n1 of K-tile t+2; retire A-lo, B-n0 of K-tile t+1
    if (h2) ph8::load_region192(p, A, B, 3, row0, col0, (t + 2) * 64, cur, wave, lane);
    if (h2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (h1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    raw_barrier();
    if (first) { PH8_MFMA_N192(1, 1, b1, 1, true) } else { PH8_MFMA_N192(1, 1, b1, 1, false) }
    raw_barrier();
  }
  if (wr == 0) raw_barrier();  // balance the stagger
  if constexpr (FE == 1) {
    ph8::epilogue_n192<EPI, FE, 0, 8>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
  } else {
    ph8::epilogue_n192<EPI, FE, 0, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
    ph8::epilogue_n192<EPI, FE, 4, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 48, lane);
  }
}

template <int EPI, int FE>
int launch_gemm8n192(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = a->N / 192;
  constexpr int LDS = 2 * ph8::BUF192;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8n192_kernel<EPI, FE>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const long long nwg = (long long)g.tiles_m * g.tiles_n * a->batch;
  hipLaunchKernelGGL((gemm8n192_kernel<EPI, FE>), dim3((unsigned)nwg), dim3(512), LDS, s, g);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Two workgroups per CU: 256x128 tiles, 4 waves (2 M x 2 N; each wave owns 128 x 64 exactly as in gemm8_kernel, so
// the same lean epilogues apply), K-steps of 32 through a 3-stage LDS-DMA ring (24 KiB per stage, 72 KiB per
// workgroup, two workgroups per CU). Each SIMD runs one wave of each workgroup and the two workgroups keep their
// own barriers, so one's epilogue and next-tile prologue (no MFMA) overlap the other's main loop — the 256x256
// kernel holds the whole CU (128 KiB LDS, 2 x 256 VGPR per SIMD) and leaves its matrix pipes idle through every
// epilogue (QKV 27 us, MLP1 56 us of 126 / 174, profiles/r02f/gemm_variants_epilogue.log).
namespace g4 {
constexpr int KS = 32, NS = 3, A_BYTES = 256 * KS * 2, B_BYTES = 128 * KS * 2, STAGE = A_BYTES + B_BYTES;
constexpr int LDS = NS * STAGE;
constexpr int OPS = 6;  // LDS-DMA issues per wave per stage: A 16 KiB + B 8 KiB = 24 x 1 KiB over 4 waves

// [row][32] e16 images (64-B rows), 16-B chunk k stored at position k ^ swz(row). The 16x16x32 fragment read
// (lane: row lane & 15, chunk lane >> 4) meets ds_read_b128's lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...
// (MI355X_MICROARCH.md §LDS): for a fixed row & 3 each group holds four (row group, chunk) pairs, which land on
// distinct 16-B bank slots iff swz = [0, 3, 2, 1] over (row >> 2) & 3 (sw_off<32>'s (row >> 2) & 3 puts two of them
// on one slot: 2-way conflicts, SQ_LDS_BANK_CONFLICT = 1/3 of the LDS cycles, profiles/r03/gemm4x_pmc_*.txt).
__device__ __forceinline__ int swz(int r) { return (-(r >> 2)) & 3; }
// per-lane source of each of the wave's 6 issues (16 rows x 64 B per issue, [row][32] image with the 16-B chunk
// index XOR-swizzled by swz(row) applied to the source: the LDS image stays lane-linear)
struct Src {
  const e16* p[OPS];
};
__device__ __forceinline__ Src make_src(const GemmK& p, const e16* A, const e16* B, int row0, int col0, int wave,
                                        int lane) {
  Src s;
  const int rr = lane >> 2, slot = lane & 3;
#pragma unroll
  for (int u = 0; u < OPS; ++u) {
    const bool isA = u < 4;
    const int j = isA ? wave * 4 + u : wave * 2 + (u - 4);
    const int r = j * 16 + rr;
    const int c = slot ^ swz(r);
    const int lim = isA ? p.M : p.N;
    int g = (isA ? row0 : col0) + r;
    g = g < lim ? g : lim - 1;  // rows past M / N: any valid row (never stored)
    s.p[u] = (isA ? A + (long long)g * p.lda : B + (long long)g * p.ldb) + c * 8;
  }
  return s;
}
__device__ __forceinline__ void stage(const Src& s, int k0, char* buf, int wave) {
#pragma unroll
  for (int u = 0; u < OPS; ++u) {
    const bool isA = u < 4;
    const int j = isA ? wave * 4 + u : wave * 2 + (u - 4);
    __builtin_amdgcn_global_load_lds((const void*)(s.p[u] + k0), (lds_ptr_t)(buf + (isA ? 0 : A_BYTES) + j * 1024), 16,
                                     0, 0);
  }
}
__device__ __forceinline__ e16x8 frag(const char* img, int row, int kc) {
  return *(const e16x8*)(img + row * 64 + ((kc ^ swz(row)) << 4));
}
// conv3x3 (a_mode 3: NHWC 64x64 images of C channels, k = tap * C + c): the A rows of one 32-wide K-step all read
// one tap, so each issue's 16 rows are 16 shifted pixels; out-of-image pixels read a zero row (LDS-DMA cannot
// zero-fill). A is re-addressed per stage; B as in make_src.
__device__ __attribute__((aligned(16))) e16 g_zero_row[4096] = {};
struct ConvSrc {
  const e16* img;  // batch image base
  int y[4], x[4], c;  // the lane's A row per A issue, its 16-B chunk (swizzled) within the row
};
__device__ __forceinline__ ConvSrc make_conv_src(const GemmK& p, const e16* A, int row0, int wave, int lane) {
  ConvSrc s;
  const int rr = lane >> 2, slot = lane & 3;
  s.img = A + (long long)(row0 >> 12) * 4096 * p.conv_c;  // a 256-row tile stays inside one image (M % 4096 == 0)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int g = row0 + (wave * 4 + u) * 16 + rr;
    s.y[u] = (g >> 6) & 63;
    s.x[u] = g & 63;
  }
  s.c = slot;
  return s;
}
__device__ __forceinline__ void stage_conv(const GemmK& p, const ConvSrc& cs, const Src& s, int k0, char* buf,
                                           int wave, int lane) {
  const int C = p.conv_c, tap = k0 / C, ch = k0 - tap * C, dy = tap / 3 - 1, dx = tap % 3 - 1;
  const int rr = lane >> 2;
#pragma unroll
  for (int u = 0; u < OPS; ++u) {
    const bool isA = u < 4;
    const int j = isA ? wave * 4 + u : wave * 2 + (u - 4);
    const e16* src;
    if (isA) {
      const int r = j * 16 + rr;
      const int yy = cs.y[u] + dy, xx = cs.x[u] + dx;
      const int c = cs.c ^ swz(r);
      src = (yy >= 0 && yy < 64 && xx >= 0 && xx < 64) ? cs.img + ((long long)yy * 64 + xx) * C + ch + c * 8
                                                       : g_zero_row + c * 8;
    } else {
      src = s.p[u] + k0;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(buf + (isA ? 0 : A_BYTES) + j * 1024), 16, 0, 0);
  }
}
}  // namespace g4

// one K-step of the wave's 128 x 64 tile: 8 A + 4 B fragment reads, 32 operand-swapped 16x16x32 MFMAs
#define G4_STEP(CA, CB, FIRST)                                                                             \
  {                                                                                                        \
    e16x8 af[8], bf[4];                                                                                    \
    _Pragma("unroll") for (int mi = 0; mi < 8; ++mi) af[mi] = g4::frag(CA, arow + mi * 16, kq);           \
    _Pragma("unroll") for (int ni = 0; ni < 4; ++ni) bf[ni] = g4::frag(CB, brow + ni * 16, kq);           \
    __builtin_amdgcn_s_setprio(1);                                                                         \
    _Pragma("unroll") for (int mi = 0; mi < 8; ++mi)                                                       \
    _Pragma("unroll") for (int ni = 0; ni < 4; ++ni)                                                       \
      acc[mi][ni] = mma16(bf[ni], af[mi], (FIRST) ? (f32x4)0.0f : acc[mi][ni], 0, 0, 0);                  \
    __builtin_amdgcn_s_setprio(0);                                                                         \
  }

template <int EPI, int FE, bool CONV = false>
__global__ __launch_bounds__(256, 2) void gemm4w_kernel(GemmK p) {
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int bid = blockIdx.x;
  {  // XCD-contiguous logical ids: the column tiles of one 256-row A panel share an L2
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int per_batch = p.tiles_m * p.tiles_n;
  const int bz = bid / per_batch, rem = bid - bz * per_batch;
  const int tm = rem / p.tiles_n, tn = rem - tm * p.tiles_n;
  const int row0 = rgroup_tm(p, tm) * 256, col0 = tn * 128;
  const e16* A = (const e16*)p.A + bz * p.sA;
  const e16* B = (const e16*)p.B + bz * p.sB;
  const int nk = p.K / g4::KS;
  const g4::Src src = g4::make_src(p, A, B, row0, col0, wave, lane);
  g4::ConvSrc csrc{};
  if constexpr (CONV) csrc = g4::make_conv_src(p, A, row0, wave, lane);
  auto stage = [&](int k0, char* buf) {
    if constexpr (CONV) g4::stage_conv(p, csrc, src, k0, buf, wave, lane);
    else g4::stage(src, k0, buf, wave);
  };
  const int arow = wr * 128 + (lane & 15), brow = wc * 64 + (lane & 15), kq = lane >> 4;
  f32x4 acc[8][4];

  stage(0, gsm);
  if (nk > 1) stage(g4::KS, gsm + g4::STAGE);
  // K-step t: stage t resident (stage t + 1 may stay in flight), every wave past step t - 1's fragment reads ->
  // stage t + 2 refills the buffer of step t - 1
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    if (t + 2 < nk) stage((t + 2) * g4::KS, gsm + ((t + 2) % g4::NS) * g4::STAGE);
    const char* ca = gsm + (t % g4::NS) * g4::STAGE;
    const char* cb = ca + g4::A_BYTES;
    if (t == 0) G4_STEP(ca, cb, true) else G4_STEP(ca, cb, false)
  }
  if constexpr (FE == 4 && !CONV) {  // in-place fp32 residual (the encoder's projection): residual through LDS
    if (p.res_lds) {
      raw_barrier();  // every wave's reads of the ring done: 16 KiB per wave for two residual quarters
      char* bx = gsm + wave * 16384;
      ph8::res_dma_q(p, bz, row0 + wr * 128, col0 + wc * 64, 0, bx, lane);
      ph8::epilogue_res_lds<EPI>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane, bx, bx + 8192);
      return;
    }
  }
  if constexpr (FE == 1) {
    ph8::epilogue_fast<EPI, FE, false>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
  } else {
    ph8::epilogue_fast<EPI, FE, false, 0, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
    ph8::epilogue_fast<EPI, FE, false, 4, 4>(p, acc, bz, row0 + wr * 128, col0 + wc * 64, lane);
  }
}

template <int EPI, int FE, bool CONV = false>
int launch_gemm4w_fe(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s) {
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = (a->N + 127) / 128;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm4w_kernel<EPI, FE, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              g4::LDS);
    attr = true;
  }
  const long long nwg = (long long)g.tiles_m * g.tiles_n * a->batch;
  hipLaunchKernelGGL((gemm4w_kernel<EPI, FE, CONV>), dim3((unsigned)nwg), dim3(256), g4::LDS, s, g);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}

// the lean kinds of the encoder's GEMMs (QKV / MLP1: e16 C; projections: fp32 C + in-place fp32 residual, with
// or without the window row map) on the two-workgroup kernel: fast path 0 (default) when g_gemm4w, K % 32 == 0
static int g_gemm4w = 1;

// the row-remapped broadcast-addend kind (11) on the two-workgroup kernel when N is not a multiple of 256: the
// decoder's [K | Q' | V] projection of the per-prompt keys (M = P*4096, N = 384, K = 256) fills 256x128 tiles
// exactly where 256x256 tiles waste a third; 320 -> 284 us, 270 with the rgroup_tm order (scripts/gemm_res_ab.py,
// profiles/r03/gemm_res_ab.log;
// the N = 256 shapes and the plain e16 residual kind 3 measured equal or slower there and stay on the 8-phase
// kernels); and the fp32 row-remapped kind (12: the patch embedding's periodic positional addend onto the fp32
// encoder stream, M = B*4096, N = K = 768), which the 8-phase kernels only run through the general register
// epilogue; fast path bit 1024 turns both off (A/B)
static int g_gemm4w_res = 1;
static int g_rgroup = 1;  // rgroup_tm ordering (fast path bit 2048 turns it off: A/B)
static int g_res_lds = 1;  // gemm8 fp32 residual kind through LDS (fast path bit 4096 turns it off: A/B)
static int g_gemm8w = 1;   // ping-pong kernel (gemm8w) for the shapes gemm8 takes (fast path bit 8192 turns it off: A/B)
static int g_gemm8w4 = 0;  // ... and for those gemm4w takes (fast path bit 16384 turns it on: A/B)
template <int EPI>
int launch_gemm4w(const GemmK& k, const octsam_gemm_args* a, hipStream_t s) {
  switch (k.fast_epi) {
    case 1: return launch_gemm4w_fe<EPI, 1>(k, a, s);
    case 2: return launch_gemm4w_fe<EPI, 2>(k, a, s);
    case 3: return launch_gemm4w_fe<EPI, 3>(k, a, s);
    case 4: return launch_gemm4w_fe<EPI, 4>(k, a, s);
    case 8: return launch_gemm4w_fe<EPI, 8>(k, a, s);
    case 11: return launch_gemm4w_fe<EPI, 11>(k, a, s);
    case 12: return launch_gemm4w_fe<EPI, 12>(k, a, s);
    default: return -1;
  }
}

// 256x192 tiles when they fill the chip's waves better than 256x256 ones (3/4 of the work per tile);
// 256x192 tiles are opt-in (fast path 24): standalone they fill the chip's waves better for N = 768 / 2304, but
// under the encoder lookahead (decoder kernels share the chip, quantisation stops mattering) the 256x256 tiles'
// fewer epilogues win, 17.77 -> 17.43 ms/step (scripts/step_ab2.py, profiles/r02g/n192_ab.log)
static int g_n192 = 0;
inline int device_cus() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
  }
  return n_cu;
}
inline bool prefer_n192(const octsam_gemm_args* a, int n_cu) {
  if (a->N % 192 != 0 || a->K < 64) return false;
  const long long tm = (a->M + 255) / 256;
  const long long t256 = tm * ((a->N + 255) / 256) * a->batch, t192 = tm * (a->N / 192) * a->batch;
  const double w256 = (double)((t256 + n_cu - 1) / n_cu), w192 = 0.75 * (double)((t192 + n_cu - 1) / n_cu);
  return w192 < w256 - 0.2;
}

template <int DBG, int EPI>
int launch_gemm8(const GemmK& k, const octsam_gemm_args* a, hipStream_t s) {
  if constexpr (EPI >= 0 && DBG == 3) {  // stamps: the lean epilogue kinds of the encoder
    switch (k.fast_epi) {
      case 1: return launch_gemm8_fe<DBG, EPI, 1>(k, a, s);
      case 4: return launch_gemm8_fe<DBG, EPI, 4>(k, a, s);
      default: break;
    }
  }
  if constexpr (EPI >= 0 && DBG == 0) {
    static int n_cu = 0;
    if (!n_cu) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
      if (n_cu <= 0) n_cu = 256;
    }
    if (g_n192 && (k.fast_epi == 1 || k.fast_epi == 4) && a->row_map == nullptr &&
        (a->R == nullptr || a->r_blk == 0) && prefer_n192(a, n_cu)) {
      if (k.fast_epi == 1) return launch_gemm8n192<EPI, 1>(k, a, s);
      return launch_gemm8n192<EPI, 4>(k, a, s);
    }
    switch (k.fast_epi) {  // the kinds the encoder and decoder use
      case 1: return launch_gemm8_fe<DBG, EPI, 1>(k, a, s);    // e16 C
      case 2: return launch_gemm8_fe<DBG, EPI, 2>(k, a, s);    // fp32 C
      case 3: return launch_gemm8_fe<DBG, EPI, 3>(k, a, s);    // e16 C + e16 residual
      case 4: return launch_gemm8_fe<DBG, EPI, 4>(k, a, s);    // fp32 C + fp32 residual
      case 8: return launch_gemm8_fe<DBG, EPI, 8>(k, a, s);    // fp32 C + fp32 residual, row map
      case 11: return launch_gemm8_fe<DBG, EPI, 11>(k, a, s);  // e16 C + broadcast e16 residual
      // e16 C + broadcast fp32 residual (one tile per workgroup: the persistent kernel, whose epilogue loads drain
      // the next tile's prefetch, took 467.8 vs 198.3 us on the decoder's M = 688 128, N = 256, K = 128 call)
      case 27: return launch_gemm8_fe<DBG, EPI, 27>(k, a, s);
      default: break;
    }
  }
  if (DBG == 0 && std::getenv("OCTSAM_GEMM_TRACE"))  // diagnostics: which calls take the general epilogue
    fprintf(stderr, "[gemm8 general epilogue] M=%d N=%d K=%d batch=%d act=%d fast_epi=%d c_f32=%d R=%d r_f32=%d r_blk=%d "
                    "C_pre=%d row_map=%d ldc=%lld ldr=%lld C%%16=%d beta=%g\n", a->M, a->N, a->K, a->batch, a->act,
            k.fast_epi, a->c_f32, a->R != nullptr, a->r_f32, a->r_blk, a->C_pre != nullptr, a->row_map != nullptr,
            (long long)a->ldc, (long long)a->ldr, (int)((uintptr_t)a->C & 15), a->beta);
  return launch_gemm8_fe<DBG, EPI, 0>(k, a, s);
}

// ------------------------------------------------------------------------------------------------
// Persistent 8-phase kernel: one workgroup per CU walks its tiles (XCD-contiguous ranges) as ONE flat
// sequence of K-steps g = tile * nk + kt, so the two-deep LDS-DMA prefetch runs straight across tile
// boundaries: the next tile's first K-tiles are in flight while the register epilogue of the finished tile
// computes and stores. The only cost of a boundary is the first K-step after it, whose counted waits must
// also cover the epilogue's stores (vmcnt counts both); for full tiles without a row map the store count is
// exact and the waits are relaxed by it, so the stores drain under that step's MFMAs.
namespace ph8 {
struct Cursor {  // the K-step a prefetch targets: tile i (this workgroup's i-th), K-tile kt
  const e16* A;
  const e16* B;
  int row0, col0, i, kt;
};
__device__ __forceinline__ Cursor tile_cursor(const GemmK& p, int i, int first, int stride, int per_batch) {
  const int t = first + i * stride;
  const int bz = t / per_batch, rem = t - bz * per_batch;
  const int tm = rem / p.tiles_n, tn = rem - tm * p.tiles_n;
  Cursor c;
  c.A = (const e16*)p.A + bz * p.sA;
  c.B = (const e16*)p.B + bz * p.sB;
  c.row0 = rgroup_tm(p, tm) * 256;
  c.col0 = tn * 256;
  c.i = i;
  c.kt = 0;
  return c;
}
// counted vmcnt wait; relax: the ST_PER_EPI stores of the previous tile's epilogue were issued after the
// operation this wait retires, so they are added to the count (they drain under the MFMAs instead)
constexpr int ST_PER_EPI = 16;
template <int BASE>
__device__ __forceinline__ void vm_wait(bool relax) {
  if (relax) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE + ST_PER_EPI) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BASE) : "memory");
}
constexpr int BIAS_MAX = BIAS_MAX_LDS;
}  // namespace ph8

// Persistent variant for bias / activation epilogues (no residual, no row map): the bias vector lives in LDS
// (copied once per workgroup before the first prefetch), so the epilogue issues no vector-memory loads and
// the compiler never drains the in-flight prefetch of the next tile; only stores follow it, and for a full
// e16 tile (exactly ST_PER_EPI store instructions per wave) the first waits of the next tile count them
// (relaxed) rather than waiting for them.
template <int EPI, int FE>
__global__ __launch_bounds__(512, 2) void gemm8p_kernel(GemmK p, int batch, int dbg) {
  constexpr bool TR = true;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int per_batch = p.tiles_m * p.tiles_n;
  const int ntiles = per_batch * batch;
  const int stride = gridDim.x >> 3;  // workgroups per XCD (grid is a multiple of 8)
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int tper = (ntiles + 7) >> 3;
  const int tbeg = xcd * tper, tend = min(ntiles, tbeg + tper);
  const int first = tbeg + loc;
  const int mycnt = first < tend ? (tend - first + stride - 1) / stride : 0;
  const int nk = p.K / 64;
  const int G = mycnt * nk;
  if (G == 0) return;
  float* lbias = (float*)(gsm + 2 * ph8::BUF);
  if (p.bias) {  // whole bias vector -> LDS (N <= BIAS_MAX, N % 8 == 0: host-checked)
    for (int i = tid * 4; i < p.N; i += 512 * 4) *(float4*)(lbias + i) = *(const float4*)(p.bias + i);
  }
  // only e16-output epilogues without a pre-activation copy have the exact store count the relaxed waits
  // assume; everything else waits for its stores (conservative)
  // relaxed waits are opt-in (fast path 13): measured slower on the encoder shapes — the next tile's loads
  // then queue behind the stores instead of after them
  const bool relax_ok = !p.c_f32 && p.Cpre == nullptr && (dbg & 1) && !(dbg & 4);
  GemmK pe = p;          // the epilogue's view (diagnostics: 4 = no stores, 8 = every tile stores to tile 0)
  if (dbg & 4) pe.M = 0;

  f32x4 acc[8][4];  // written by each tile's first K-step (zero-accumulator MFMAs); K >= 64 host-checked
  e16x8 af[4][2], b0[2][2], b1[2][2];
  const int arow = wr * 128 + (lane & 15), brow = wc * 64 + (lane & 15), kq = lane >> 4;

  // prefetch cursors: c1 -> step g+1, c2 -> step g+2 (advanced once per step; divisions once per tile)
  ph8::Cursor cc = ph8::tile_cursor(p, 0, first, stride, per_batch);
  auto advance = [&](ph8::Cursor c) {
    if (++c.kt == nk) c = ph8::tile_cursor(p, c.i + 1, first, stride, per_batch);
    return c;
  };
  const ph8::LdPlan plan = ph8::make_plan(p, wave, lane);
  auto issue = [&](const ph8::Cursor& c, int region, char* buf) {
    ph8::load_region_buf(p, c.A, c.B, c.row0, c.col0, c.kt, region, plan, buf, wave);
  };
  ph8::Cursor c1 = advance(cc);
  ph8::Cursor c2 = advance(c1);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // bias copy done before the DMA count starts
  issue(cc, 0, gsm);
  issue(cc, 2, gsm);
  issue(cc, 3, gsm);
  issue(cc, 1, gsm);
  if (G > 1) {
    issue(c1, 0, gsm + ph8::BUF);
    issue(c1, 2, gsm + ph8::BUF);
    issue(c1, 3, gsm + ph8::BUF);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  raw_barrier();
  if (wr == 1) raw_barrier();

  // since: K-steps since the last epilogue (1: every wait of this step has the stores above the operation it
  // retires; 2: only phase 0's does); relax: the last epilogue issued exactly ST_PER_EPI stores
  int since = 3;
  bool relax_epi = false;
  for (int g = 0; g < G; ++g) {
    char* cur = gsm + (g & 1) * ph8::BUF;
    char* nxt = gsm + ((g + 1) & 1) * ph8::BUF;
    const char* ca = cur;
    const char* cb = cur + 32768;
    const bool h1 = g + 1 < G, h2 = g + 2 < G;
    const bool rx1 = relax_epi && since == 1, rx0 = relax_epi && since <= 2;
    const bool first_k = cc.kt == 0;
    // ---- phase 0: Q(0,0) — A-lo, B-n0
    if (h1) issue(c1, 1, nxt);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + mi * 16, kb * 4 + kq);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b0[ni][kb] = ph8::frag(cb, brow + ni * 16, kb * 4 + kq);
    }
    if (h1) ph8::vm_wait<10>(rx0);  // retire B-n1(g)
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(0, 0, b0, first_k)
    raw_barrier();
    // ---- phase 1: Q(0,1) — B-n1
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) b1[ni][kb] = ph8::frag(cb, brow + 32 + ni * 16, kb * 4 + kq);
    if (h1) ph8::vm_wait<8>(rx1);  // retire A-hi(g)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(0, 1, b1, first_k)
    raw_barrier();
    // ---- phase 2: Q(1,0) — A-hi; restage A-lo, B-n0 of step g+2
    if (h2) {
      issue(c2, 0, cur);
      issue(c2, 2, cur);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][kb] = ph8::frag(ca, arow + 64 + mi * 16, kb * 4 + kq);
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PH8_MFMA_QUAD_F(1, 0, b0, first_k)
    raw_barrier();
    // ---- phase 3: Q(1,1); restage B-n1 of step g+2; retire A-lo, B-n0 of step g+1
    if (h2) issue(c2, 3, cur);
    if (h2) ph8::vm_wait<10>(rx1);
    else if (h1) ph8::vm_wait<4>(rx1);
    raw_barrier();
    PH8_MFMA_QUAD_F(1, 1, b1, first_k)
    raw_barrier();
    ++since;
    if (++cc.kt == nk) {  // last K-step of tile cc.i: epilogue while steps g+1, g+2 load
      const int ebz = (dbg & 8) ? 0 : (first + cc.i * stride) / per_batch;
      const int er0 = ((dbg & 8) ? 0 : cc.row0) + wr * 128, ec0 = ((dbg & 8) ? 0 : cc.col0) + wc * 64;
      if constexpr (FE == 11) {  // residual kind: quarters (the loaded residual must fit too)
        ph8::epilogue_fast<EPI, FE, true, 0, 2>(pe, acc, ebz, er0, ec0, lane, lbias);
        ph8::epilogue_fast<EPI, FE, true, 2, 2>(pe, acc, ebz, er0, ec0, lane, lbias);
        ph8::epilogue_fast<EPI, FE, true, 4, 2>(pe, acc, ebz, er0, ec0, lane, lbias);
        ph8::epilogue_fast<EPI, FE, true, 6, 2>(pe, acc, ebz, er0, ec0, lane, lbias);
      } else if constexpr (FE != 0) {
        ph8::epilogue_fast<EPI, FE, true, 0, 4>(pe, acc, ebz, er0, ec0, lane, lbias);
        ph8::epilogue_fast<EPI, FE, true, 4, 4>(pe, acc, ebz, er0, ec0, lane, lbias);
      } else {
        ph8::epilogue_reg<EPI, 0, 4, true>(pe, acc, ebz, er0, ec0, lane, lbias);
        ph8::epilogue_reg<EPI, 4, 4, true>(pe, acc, ebz, er0, ec0, lane, lbias);
      }
      relax_epi = relax_ok && cc.row0 + 256 <= p.M && cc.col0 + 256 <= p.N;
      since = 1;
      cc = c1;  // (c1 is tile cc.i + 1 at K-tile 0 here)
    }
    c1 = c2;
    c2 = advance(c2);
  }
  if (wr == 0) raw_barrier();  // balance the stagger
}

template <int EPI, int FE>
int launch_gemm8p_fe(const GemmK& k0, const octsam_gemm_args* a, hipStream_t s, int dbg) {
  GemmK g = k0;
  g.tiles_m = (a->M + 255) / 256;
  g.tiles_n = (a->N + 255) / 256;
  constexpr int LDS = 2 * ph8::BUF + ph8::BIAS_MAX * 4;
  static int n_cu = 0;
  if (!n_cu) {
    (void)hipFuncSetAttribute((const void*)gemm8p_kernel<EPI, FE>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
  }
  const long long ntiles = (long long)g.tiles_m * g.tiles_n * a->batch;
  long long grid = ((n_cu + 7) / 8) * 8;
  while (grid > 8 && grid / 2 >= ntiles) grid /= 2;
  if (dbg & 2) grid = (ntiles + 7) / 8 * 8;  // diagnostics: one tile per workgroup
  hipLaunchKernelGGL((gemm8p_kernel<EPI, FE>), dim3((unsigned)grid), dim3(512), LDS, s, g, a->batch, dbg);
  OCTSAM_LAUNCH_CHECK("octsam_gemm");
  return 0;
}
template <int EPI>
int launch_gemm8p(const GemmK& k, const octsam_gemm_args* a, hipStream_t s, int dbg) {
  if (k.fast_epi == 1) return launch_gemm8p_fe<EPI, 1>(k, a, s, dbg);
  if constexpr (EPI == 0) {  // decoder image-side projections: e16 C + e16 (broadcast) residual, K <= 512
    if (k.fast_epi == 11) return launch_gemm8p_fe<EPI, 11>(k, a, s, dbg);
  }
  // (fp32 output + GELU would spill in this kernel: general epilogue)
  if constexpr (EPI != OCTSAM_ACT_GELU)
    if (k.fast_epi == 2) return launch_gemm8p_fe<EPI, 2>(k, a, s, dbg);
  return launch_gemm8p_fe<EPI, 0>(k, a, s, dbg);
}

// Deterministic split reduction: out[i] = sum_s part[s*n + i] (+ beta*out[i]).
__global__ void splitk_reduce_kernel(const float* part, float* out, long long n, int splits, float beta) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  for (int j = 0; j < splits; ++j) s += part[j * n + i];
  out[i] = (beta != 0.0f ? beta * out[i] : 0.0f) + s;
}

// Vectorised variant: 64 float4 columns x 4 split lanes per block, fixed-order LDS combine.
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float4* __restrict__ part, float4* __restrict__ out,
                                                             long long n4, int splits, float beta) {
  __shared__ float4 red[4][64];
  const int c = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
#pragma unroll 4
    for (int j = lane; j < splits; j += 4) {
      float4 v = part[(long long)j * n4 + i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[lane][c] = s;
  __syncthreads();
  if (lane == 0 && i < n4) {
    float4 r = red[0][c];
#pragma unroll
    for (int l = 1; l < 4; ++l) { r.x += red[l][c].x; r.y += red[l][c].y; r.z += red[l][c].z; r.w += red[l][c].w; }
    if (beta != 0.0f) {
      float4 o = out[i];
      r.x += beta * o.x; r.y += beta * o.y; r.z += beta * o.z; r.w += beta * o.w;
    }
    out[i] = r;
  }
}

// 16 float4 columns x 16 split lanes per block, fixed-order combine (deterministic).
__global__ __launch_bounds__(256) void splitk_reduce16_kernel(const float4* __restrict__ part, float4* __restrict__ out,
                                                              long long n4, int splits, float beta) {
  __shared__ float4 red[16][16];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const long long i = (long long)blockIdx.x * 16 + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
#pragma unroll 4
    for (int j = sl; j < splits; j += 16) {
      const float4 v = part[(long long)j * n4 + i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && i < n4) {
    float4 r = red[0][c];
#pragma unroll
    for (int l = 1; l < 16; ++l) { r.x += red[l][c].x; r.y += red[l][c].y; r.z += red[l][c].z; r.w += red[l][c].w; }
    if (beta != 0.0f) {
      const float4 o = out[i];
      r.x += beta * o.x; r.y += beta * o.y; r.z += beta * o.z; r.w += beta * o.w;
    }
    out[i] = r;
  }
}

}  // namespace


// launch options and the last path taken are shared by the bf16 and fp16 builds of this file (the bf16
// build owns them; the fp16 build reaches them through these hidden accessors), so
// octsam_gemm_set_fast_path / octsam_gemm_last_path cover both entry points
namespace __attribute__((visibility("hidden"))) octsam_gemm_state {
int& use_glds();
int& small_path();
int& last_path();
#ifndef OCTSAM_GEMM_F16
int& use_glds() { static int v = 1; return v; }
int& small_path() { static int v = 1; return v; }
int& last_path() { static thread_local int v = 0; return v; }
#endif
}  // namespace octsam_gemm_state
#define g_use_glds (octsam_gemm_state::use_glds())
#define g_small (octsam_gemm_state::small_path())
#define t_last_path (octsam_gemm_state::last_path())
#ifndef OCTSAM_GEMM_F16
// enable: 0 = generic kernels only; 1 = default; 2..10 = fast-path variants (diagnostics); bit 8 (256)
// disables the small-problem 64x64 path
extern "C" void octsam_gemm_set_fast_path(int32_t enable) {
  g_small = (enable & 256) ? 0 : 1;
  g_gemm4w = (enable & 512) ? 0 : 1;
  g_gemm4w_res = (enable & 1024) ? 0 : 1;
  g_rgroup = (enable & 2048) ? 0 : 1;
  g_res_lds = (enable & 4096) ? 0 : 1;
  g_gemm8w = (enable & 8192) ? 0 : 1;
  g_gemm8w4 = (enable & 16384) ? 1 : 0;
  g_pp_skip = (enable >> 20) & 7;
  g_small_oneshot = (enable & 65536) ? 0 : 1;
  g_n192w = (enable & 262144) ? 1 : 0;
  g_use_glds = enable & 255;
  g_n192 = g_use_glds == 24 ? 1 : 0;
}
extern "C" int32_t octsam_gemm_last_path(void) { return t_last_path; }
extern "C" int octsam_gemm_debug_stamps(int64_t* host, int32_t n_wg) {
  OCTSAM_CHECK_ARG(host && n_wg > 0 && n_wg <= STAMP_WG, "octsam_gemm_debug_stamps: bad args");
  const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n_wg * 4 * sizeof(long long));
  OCTSAM_CHECK_ARG(e == hipSuccess, "octsam_gemm_debug_stamps: %s", hipGetErrorString(e));
  return 0;
}
#endif

extern "C" int OCTSAM_GEMM_ENTRY(const octsam_gemm_args* a, void* stream) {
  OCTSAM_CHECK_ARG(a != nullptr, "octsam_gemm: null args");
  OCTSAM_CHECK_ARG(a->M > 0 && a->N > 0 && a->K > 0 && a->batch > 0, "octsam_gemm: bad sizes M=%d N=%d K=%d batch=%d",
                   a->M, a->N, a->K, a->batch);
  OCTSAM_CHECK_ARG(a->A && a->B && a->C, "octsam_gemm: null operand");
  OCTSAM_CHECK_ARG(a->a_mode >= 0 && a->a_mode <= 4 && a->b_mode >= 0 && a->b_mode <= 2, "octsam_gemm: bad mode");
  // K-contiguous operand loads move 8 consecutive k at a time; transposed loads move one k per chunk
  if (a->a_mode != 1 || a->b_mode == 0)
    OCTSAM_CHECK_ARG(a->K % 8 == 0, "octsam_gemm: K=%d must be a multiple of 8", a->K);
  OCTSAM_CHECK_ARG(a->a_blk == 0 || a->a_mode == 0 || a->a_mode == 4, "octsam_gemm: a_blk needs a_mode 0/4");
  OCTSAM_CHECK_ARG(a->b_blk == 0 || a->b_mode >= 1, "octsam_gemm: b_blk needs b_mode 1/2");
  if (a->a_mode == 1) OCTSAM_CHECK_ARG(a->M % 8 == 0 && a->lda % 8 == 0, "octsam_gemm: transposed A needs M%%8==0");
  if (a->a_mode == 0 || a->a_mode == 4) OCTSAM_CHECK_ARG(a->lda % 8 == 0, "octsam_gemm: lda must be a multiple of 8");
  if (a->a_mode == 4) OCTSAM_CHECK_ARG(a->A2 && a->a2_rows > 0, "octsam_gemm: a_mode 4 needs A2 and a2_rows");
  if (a->b_mode == 2) OCTSAM_CHECK_ARG(a->B2 && a->b2_rows > 0, "octsam_gemm: b_mode 2 needs B2 and b2_rows");
  if (a->b_mode >= 1) OCTSAM_CHECK_ARG(a->N % 8 == 0 && a->ldb % 8 == 0, "octsam_gemm: transposed B needs N%%8==0");
  if (a->b_mode == 0) OCTSAM_CHECK_ARG(a->ldb % 8 == 0, "octsam_gemm: ldb must be a multiple of 8");
  if (a->a_mode == 2) OCTSAM_CHECK_ARG(a->K == 768 && a->M % 4096 == 0, "octsam_gemm: patch16 mode needs K=768, M=B*4096");
  if (a->a_mode == 3)
    OCTSAM_CHECK_ARG(a->conv_c % 8 == 0 && a->K == 9 * a->conv_c && a->M % 4096 == 0,
                     "octsam_gemm: conv3x3 mode needs K=9*C, C%%8==0, M=B*4096");
  GemmK k;
  k.A2 = a->A2; k.B2 = a->B2; k.a2_rows = a->a2_rows; k.b2_rows = a->b2_rows;
  k.a_blk = a->a_blk; k.a_rep = a->a_rep > 0 ? a->a_rep : 1;
  k.b_blk = a->b_blk; k.b_rep = a->b_rep > 0 ? a->b_rep : 1;
  k.r_blk = a->r_blk; k.r_rep = a->r_rep > 0 ? a->r_rep : 1;
  k.A = a->A; k.B = a->B; k.C = a->C; k.bias = a->bias; k.R = a->R; k.Cpre = a->C_pre; k.row_map = a->row_map;
  k.M = a->M; k.N = a->N; k.K = a->K;
  k.lda = a->lda; k.ldb = a->ldb; k.ldc = a->ldc; k.ldr = a->ldr;
  k.sA = a->stride_a; k.sB = a->stride_b; k.sC = a->stride_c; k.sR = a->stride_r;
  k.alpha = a->alpha; k.beta = a->beta; k.act = a->act;
  k.c_f32 = a->c_f32; k.r_f32 = a->r_f32; k.pre_f32 = a->pre_f32; k.conv_c = a->conv_c;
  k.k_total = a->k_total;
  // broadcast-residual tile order: whole 256-row tiles per residual period, whole groups of tiles
  k.rgroup = (g_rgroup && a->R && a->r_blk > 0 && (a->r_blk & 255) == 0 && k.r_rep > 1 && a->row_map == nullptr &&
              ((a->M + 255) / 256) % ((a->r_blk >> 8) * k.r_rep) == 0)
                 ? 1
                 : 0;
  k.a_cs = a->a_colsum;
  k.b_cs = a->b_colsum;
  k.res_lds = g_res_lds;
  const bool want_cs = a->a_colsum != nullptr || a->b_colsum != nullptr;
  OCTSAM_CHECK_ARG(!want_cs || (a->a_mode == 1 && a->b_mode == 1), "octsam_gemm: a_colsum / b_colsum need a_mode = b_mode = 1");
  {  // lean epilogue kind (epilogue_fast): no C_pre; a residual must have C's type, no broadcast (r_blk)
    const int es = a->c_f32 ? 4 : 2;
    // (an fp32 residual under an e16 C: the broadcast kind only -- the decoder's first block adds the fp32 image
    //  embedding to its per-prompt keys)
    const bool r_mixed = a->R && a->r_f32 && !a->c_f32 && a->r_blk > 0 && a->row_map == nullptr;
    const bool res_ok = a->R == nullptr || ((a->r_f32 == a->c_f32 || r_mixed) && (a->r_blk == 0 || a->row_map == nullptr) &&
                                            (a->ldr & 7) == 0 && ((uintptr_t)a->R & 15) == 0);
    const long long rows = a->row_map ? (long long)a->c_rows : (long long)a->M;
    const bool range_ok = rows > 0 && rows * a->ldc * es < (1LL << 31) &&
                          (a->R == nullptr || rows * a->ldr * (a->r_f32 ? 4 : 2) < (1LL << 31));
    k.fast_epi = (a->C_pre == nullptr && (a->ldc & 7) == 0 && ((uintptr_t)a->C & 15) == 0 && res_ok && range_ok)
                     ? 1 + (a->c_f32 ? 1 : 0) + (a->R ? 2 : 0) + (a->row_map ? 4 : 0) +
                           (a->R && a->r_blk > 0 ? 8 : 0) + (r_mixed ? 16 : 0)
                     : 0;
    k.c_rows = a->c_rows;
    if (g_use_glds == 18) k.fast_epi = 0;  // diagnostics / parity: the general register epilogue
  }
  OCTSAM_CHECK_ARG(a->k_total == 0 || (a->a_mode == 1 && a->b_mode == 1 && a->k_total <= (long long)a->K * a->batch &&
                                       a->k_total > (long long)a->K * (a->batch - 1)),
                   "octsam_gemm: k_total needs a_mode = b_mode = 1 and (batch-1)*K < k_total <= batch*K");
  k.tiles_m = (a->M + BM - 1) / BM;
  k.tiles_n = (a->N + BN - 1) / BN;
  hipStream_t s = (hipStream_t)stream;
  const int am = a->a_mode, bm = a->b_mode;
  const bool fast_epi = (a->N & 1) == 0 && (a->ldc & 1) == 0 && ((uintptr_t)a->C & 7) == 0 &&
                        (!a->C_pre || ((uintptr_t)a->C_pre & 7) == 0) &&
                        (!a->R || ((a->ldr & 1) == 0 && ((uintptr_t)a->R & 7) == 0));
  // Small problems (token-side decoder GEMMs: M ~ P*7 rows, split-K weight gradients): a 256-row tile
  // leaves most CUs idle, so the register-staged kernel with 64x64 tiles takes them.
  {
    const long long t64 = (long long)((a->M + 63) / 64) * ((a->N + 63) / 64) * a->batch;
    const long long t256 = (long long)((a->M + 255) / 256) * ((a->N + 255) / 256) * a->batch;
    if (am <= 1 && bm <= 1 && a->a_blk == 0 && a->b_blk == 0 && t256 < 96 && t64 <= 4096 && g_small && !want_cs) {
      t_last_path = 3;
      // (one-shot when its 64 KiB-LDS workgroups fit one wave of the chip at two per CU: N = 2048 measured slower,
      //  13.2 vs 10.2 us, scripts/tok_gemm_ab.py)
      if (a->K <= 256 && g_small_oneshot && t64 <= 512) {
        if (am == 0 && bm == 0) return launch_small<0, 0>(k, a->batch, s);
        if (am == 0 && bm == 1) return launch_small<0, 1>(k, a->batch, s);
        if (am == 1 && bm == 0) return launch_small<1, 0>(k, a->batch, s);
        return launch_small<1, 1>(k, a->batch, s);
      }
      if (am == 0 && bm == 0) return launch<0, 0, 64>(k, a->batch, s);
      if (am == 0 && bm == 1) return launch<0, 1, 64>(k, a->batch, s);
      if (am == 1 && bm == 0) return launch<1, 0, 64>(k, a->batch, s);
      return launch<1, 1, 64>(k, a->batch, s);
    }
  }
  // persistent LDS-DMA kernel: K-contiguous (mode 0) or k-major (mode 1, transposed-read) operands
  const bool ok_a = (a->lda & 7) == 0 && (am == 0 || (am == 1 && (a->M & 7) == 0 && a->M >= 8));
  const bool ok_b = (a->ldb & 7) == 0 && (bm == 0 || (bm == 1 && (a->N & 7) == 0 && a->N >= 8));
  const long long tiles = (long long)((a->M + 255) / 256) * ((a->N + 127) / 128) * a->batch;
  const bool k_ok = a->K % 64 == 0 || (a->k_total > 0 && a->K % 8 == 0);  // km operands: zero-filled tail
  if (g_use_glds && ok_a && ok_b && k_ok && a->a_blk == 0 && a->b_blk == 0 && fast_epi &&
      (a->M >= 1024 || tiles >= 64 || a->k_total > 0) && ((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->B & 15) == 0 &&
      (a->batch == 1 || ((a->stride_a & 7) == 0 && (a->stride_b & 7) == 0))) {
    t_last_path = 1;
    // transposed-read operands need more address registers: the 256x128 tile (no spills)
    if (am == 1 && bm == 1) return launch_glds<128, 64, 3, true, true>(k, a, s);
    if (am == 1) return launch_glds<128, 64, 3, true, false>(k, a, s);
    if (bm == 1) return launch_glds<128, 64, 3, false, true>(k, a, s);
    if (g_use_glds == 2) return launch_glds<128, 64, 3>(k, a, s);
    if (g_use_glds == 3) return launch_glds<256, 32, 4>(k, a, s);
    if (a->N <= 64) return launch_glds<64, 64, 3>(k, a, s);  // narrow outputs (ConvT 64-channel GEMMs)
    // 8-phase kernel with the LDS-staged epilogue: 16-B aligned rows for every epilogue operand
    const bool a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; }(a->C);
    const bool epi8 = (a->N & 7) == 0 && (a->ldc & 7) == 0 && a16 && ((uintptr_t)a->bias & 15) == 0 &&
                      ((uintptr_t)a->C_pre & 15) == 0 && ((uintptr_t)a->R & 15) == 0 &&
                      (!a->R || (a->ldr & 7) == 0) && (a->batch == 1 || ((a->stride_c & 7) == 0 &&
                                                                          (!a->R || (a->stride_r & 7) == 0)));
    if (epi8 && g_use_glds != 5 && a->beta == 0.0f) {
      t_last_path = 2;
      if (g_use_glds == 6) return launch_gemm8<1, 0>(k, a, s);
      if (g_use_glds == 7) return launch_gemm8<2, 0>(k, a, s);
      if (g_use_glds == 8) return launch_gemm8<0, -1>(k, a, s);
      if (g_use_glds == 9 && g_gemm8w && am == 0 && bm == 0 && a->K % 64 == 0 && a->K >= 128 &&
          (long long)a->M * a->lda * 2 < (1LL << 31) && (long long)a->N * a->ldb * 2 < (1LL << 31) &&
          (a->act == 0 || a->act == OCTSAM_ACT_GELU)) {  // stamped ping-pong kernel (diagnostics)
        const int r = a->act == OCTSAM_ACT_GELU ? launch_gemm8w<OCTSAM_ACT_GELU>(k, a, s, true)
                                                : launch_gemm8w<0>(k, a, s, true);
        if (r >= 0) return r;
      }
      if (g_use_glds == 9) {  // stamped one-tile-per-workgroup kernel (diagnostics)
        if (a->act == OCTSAM_ACT_GELU) return launch_gemm8<3, OCTSAM_ACT_GELU>(k, a, s);
        return launch_gemm8<3, 0>(k, a, s);
      }
      // persistent variant: bias / activation epilogues (no residual or row map loads in the epilogue);
      // fast path 11 forces the one-tile-per-workgroup kernel (A/B diagnostics)
      // (an e16 residual is allowed at small K: its loads drain the next tile's prefetch, which is the whole
      // next tile there anyway, and the tile's load latency still overlaps the epilogue)
      // two workgroups per CU (gemm4w_kernel): the lean kinds without a broadcast residual, K % 32 == 0
      // (measured, scripts/gemm_ab.py, profiles/r03/gemm_ab.log: faster for N, K <= 1024 — proj 76 -> 69 us,
      // decoder ConvT1 178 -> 173 us — and slower for the wide / deep ones: QKV 129 -> 140, MLP1 179 -> 194, MLP2
      // 184 -> 195 us, where the 8-phase interleave of one 256x256 workgroup keeps the matrix pipes busier)
      const bool w_ok = (g_use_glds == 1 || g_use_glds == 9) && am == 0 && bm == 0 && a->K % 64 == 0 && a->K >= 128 &&
                        (k.fast_epi == 1 || k.fast_epi == 2 || k.fast_epi == 4 || k.fast_epi == 8) &&
                        (a->act == 0 || a->act == OCTSAM_ACT_GELU) && (long long)a->M * a->lda * 2 < (1LL << 31) &&
                        (long long)a->N * a->ldb * 2 < (1LL << 31);
      if (w_ok && g_gemm8w4) {
        t_last_path = 2;
        const int r = a->act == OCTSAM_ACT_GELU ? launch_gemm8w<OCTSAM_ACT_GELU>(k, a, s) : launch_gemm8w<0>(k, a, s);
        if (r >= 0) return r;
      }
      // (opt-in) 256x192 ping-pong tiles where 256-column tiles quantise badly (N = 768: 384 tiles = 1.5 waves of 256
      // CUs, as 512 tiles of 3/4 the work = 2 full waves; QKV's N = 2304: 4.5 -> 6 x 3/4): MLP2, the projection, QKV
      if (w_ok && g_gemm8w && g_n192w && g_use_glds == 1 && (k.fast_epi == 1 || k.fast_epi == 4) &&
          a->row_map == nullptr && prefer_n192(a, device_cus())) {
        t_last_path = 2;
        if (a->act == OCTSAM_ACT_GELU)
          return k.fast_epi == 1 ? launch_gemm8w_fe<OCTSAM_ACT_GELU, 1, 0, 3>(k, a, s)
                                 : launch_gemm8w_fe<OCTSAM_ACT_GELU, 4, 0, 3>(k, a, s);
        return k.fast_epi == 1 ? launch_gemm8w_fe<0, 1, 0, 3>(k, a, s) : launch_gemm8w_fe<0, 4, 0, 3>(k, a, s);
      }
      if (g_gemm4w && g_use_glds == 1 && a->K % 32 == 0 && a->K >= 64 && a->K <= 1024 && a->N <= 1024 &&
          a->batch == 1 && am == 0 && bm == 0 &&
          a->M >= 4096 &&
          (k.fast_epi == 1 || k.fast_epi == 2 || k.fast_epi == 4 || k.fast_epi == 8 ||
           (g_gemm4w_res && k.fast_epi == 11 && a->K <= 512 && a->N % 256 != 0) ||
           (g_gemm4w_res && k.fast_epi == 12)) &&
          (a->act == 0 || a->act == OCTSAM_ACT_GELU) && (long long)a->M * a->lda * 2 < (1LL << 40)) {
        t_last_path = 2;
        if (a->act == OCTSAM_ACT_GELU) return launch_gemm4w<OCTSAM_ACT_GELU>(k, a, s);
        return launch_gemm4w<0>(k, a, s);
      }
      const bool res_small_k =
          a->R != nullptr && k.fast_epi == 11 && a->K <= 512 && a->act == 0;  // (kind 3 measured slower)
      // bias / activation kinds (encoder QKV, MLP1) run one tile per workgroup by default: under the encoder
      // lookahead (train.FusedTrainStep pipeline) the decoder's kernels share the chip, and hardware-scheduled
      // workgroups fill the CUs they leave while a fixed persistent grid waits for all of them (same-process
      // A/B: 18.2 -> 17.7 ms/step); fast path 23 (and the 12..17 diagnostics) keep them persistent
      const bool persist_bias = g_use_glds == 23 || (g_use_glds >= 12 && g_use_glds <= 17);
      const bool persist = ((a->R == nullptr && persist_bias) || res_small_k) && a->row_map == nullptr &&
                           a->N <= ph8::BIAS_MAX && g_use_glds != 11 && g_use_glds != 20 &&
                           (long long)a->M * a->lda * 2 < (1LL << 31) && (long long)a->N * a->ldb * 2 < (1LL << 31);
      if (persist) {
        // fast paths 12..15: persistent-kernel diagnostics (bit 0: relaxed waits after full-tile epilogues,
        // bit 1: one tile per workgroup)
        // (16: no epilogue stores, 17: every tile stores to tile 0)
        const int dbg = g_use_glds >= 12 && g_use_glds <= 15 ? g_use_glds - 12
                        : g_use_glds == 16 ? 4 : g_use_glds == 17 ? 8 : 0;
        if (a->act == OCTSAM_ACT_RELU) return launch_gemm8p<OCTSAM_ACT_RELU>(k, a, s, dbg);
        if (a->act == OCTSAM_ACT_GELU) return launch_gemm8p<OCTSAM_ACT_GELU>(k, a, s, dbg);
        return launch_gemm8p<0>(k, a, s, dbg);
      }
      if (w_ok && g_gemm8w) {
        const int r = a->act == OCTSAM_ACT_GELU ? launch_gemm8w<OCTSAM_ACT_GELU>(k, a, s) : launch_gemm8w<0>(k, a, s);
        if (r >= 0) return r;
      }
      if (a->act == OCTSAM_ACT_RELU) return launch_gemm8<0, OCTSAM_ACT_RELU>(k, a, s);
      if (a->act == OCTSAM_ACT_GELU) return launch_gemm8<0, OCTSAM_ACT_GELU>(k, a, s);
      return launch_gemm8<0, 0>(k, a, s);
    }
    return launch_glds<256, 64, 2>(k, a, s);
  }
  OCTSAM_CHECK_ARG(!want_cs, "octsam_gemm: a_colsum / b_colsum need the LDS-DMA k-major path (16-B aligned operands, "
                             "K %% 64 == 0 or a k_total tail, enough tiles)");
  t_last_path = 0;
  OCTSAM_CHECK_ARG(a->k_total == 0 || (am == 1 && bm == 1), "octsam_gemm: k_total needs a_mode = b_mode = 1");
  if (am == 0 && bm == 0) return launch<0, 0>(k, a->batch, s);
  if (am == 0 && bm == 1) return launch<0, 1>(k, a->batch, s);
  if (am == 1 && bm == 0) return launch<1, 0>(k, a->batch, s);
  if (am == 1 && bm == 1) return launch<1, 1>(k, a->batch, s);
  if (am == 2 && bm == 0) return launch<2, 0>(k, a->batch, s);
  // conv3x3 on the two-workgroup kernel (the neck: M = B*4096, N = C = 256, K = 9C; fp32 C, no activation)
  if (am == 3 && bm == 0 && g_gemm4w_res && g_use_glds == 1 && a->conv_c % 32 == 0 && a->conv_c <= 4096 &&
      a->batch == 1 && a->act == 0 && (k.fast_epi == 1 || k.fast_epi == 2) && ((uintptr_t)a->A & 15) == 0 &&
      (a->ldb & 7) == 0 && ((uintptr_t)a->B & 15) == 0) {
    t_last_path = 2;
    if (k.fast_epi == 1) return launch_gemm4w_fe<0, 1, true>(k, a, s);
    return launch_gemm4w_fe<0, 2, true>(k, a, s);
  }
  if (am == 3 && bm == 0) return launch<3, 0>(k, a->batch, s);
  if (am == 4 && bm == 0) return launch<4, 0>(k, a->batch, s);
  if (am == 1 && bm == 2) return launch<1, 5>(k, a->batch, s);
  octsam::set_error("octsam_gemm: unsupported mode combination a=%d b=%d", am, bm);
  return 1;
}

#ifndef OCTSAM_GEMM_F16
extern "C" int octsam_splitk_reduce(const float* partials, float* out, int64_t n, int32_t splits, float beta,
                                    void* stream) {
  OCTSAM_CHECK_ARG(partials && out && n > 0 && splits > 0, "octsam_splitk_reduce: bad args");
  if (n % 4 == 0 && ((uintptr_t)partials & 15) == 0 && ((uintptr_t)out & 15) == 0 && splits >= 32 && n / 4 <= 16384) {
    // few columns, many splits: 16 float4 columns x 16 split lanes per block
    long long n4 = n / 4;
    hipLaunchKernelGGL(splitk_reduce16_kernel, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)partials, (float4*)out, n4, splits, beta);
    OCTSAM_LAUNCH_CHECK("octsam_splitk_reduce");
    return 0;
  }
  if (n % 4 == 0 && ((uintptr_t)partials & 15) == 0 && ((uintptr_t)out & 15) == 0 && splits >= 4) {
    long long n4 = n / 4;
    hipLaunchKernelGGL(splitk_reduce4_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)partials, (float4*)out, n4, splits, beta);
    OCTSAM_LAUNCH_CHECK("octsam_splitk_reduce");
    return 0;
  }
  long long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, partials, out,
                     n, splits, beta);
  OCTSAM_LAUNCH_CHECK("octsam_splitk_reduce");
  return 0;
}
#endif  // OCTSAM_GEMM_F16
