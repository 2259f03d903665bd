// SAM ViT attention with decomposed relative-position bias, fused (flash-style), forward only.
//
// Replaces SamVisionAttention / SamVisionSdpaAttention.forward (hf:modeling_sam.py:803-882) together
// with get_rel_pos / get_decomposed_rel_pos (:729-801). The [B*h, T, T] bias tensor that HF
// materialises (805 MB per image for a global vit-b layer) is never formed:
//
//   s[q,k] = (q/8)·k + rel_h[q, kh] + rel_w[q, kw],   rel_h[q,kh] = q·Rh[qh-kh+S-1], rel_w likewise
//
// (rel-pos resize is an identity for SAM: 2*max(q,k)-1 == table length).
//
// Layout/mapping (one wave = 32 queries, all MFMAs v_mfma_f32_32x32x16_bf16):
//   S^T = K · Q^T  : A = K rows from LDS (XOR-swizzled), B = Q^T fragments kept in registers
//                    -> every lane owns ONE query (col) and 16 keys (rows) per 32x32 tile
//   O^T = V^T · P^T: A = V^T from LDS (padded rows, ds_read_b64), B = P^T taken straight from the
//                    S^T accumulator registers (bf16-packed, k order permuted to match)
//   so softmax statistics, the rel-pos terms and the O rescale are all per-lane (plus one
//   lane^32 exchange) and nothing crosses lanes through LDS in the main loop.
// rel_h / rel_w tables for the wave's queries are themselves MFMA products P^T = R · Q^T staged
// once through LDS.
//
// Global layers (S=64, T=4096): 4 waves (128 queries = 2 image rows) per workgroup, 64-key tiles
// (= one key image row, so rel_h is one scalar per lane per tile and rel_w is a fixed register set),
// register-staged double-buffered K/V tiles.
// Windowed layers (S=14, T=196): 7 waves (224 queries) per (window, head), the whole window's K/V
// (padded to 256 keys, masked) resident in LDS.
#include "common.h"
#include "../../include/octsam.h"

namespace {

constexpr float kScale = 0.125f;  // 64^-0.5, exact in bf16

__device__ __forceinline__ int ksw(int r, int c) {  // K image [rows][64] bf16, 16-B chunk swizzle
  return r * 64 + ((c ^ ((r >> 1) & 7)) << 3);
}

__device__ __forceinline__ bf16x8 scale8(bf16x8 v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)((float)v[i] * kScale);
  return v;
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[base + j];
  return r;
}

// Row index (within a 32x32 tile) held in accumulator register r by lane half h.
__device__ __forceinline__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// P^T = R_ext · Qs^T for the wave's 32 queries; writes 8 * P^T (undo the 1/8 in Qs) to
// prel[j * 33 + ql] for j in [0, 32*NJT) (rows >= 2S-1 are zero).
template <int NJT>
__device__ __forceinline__ void relpos_table(const float* __restrict__ R, int nrows, const bf16x8 (&qf)[4],
                                             float* prel, int lane) {
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int t = 0; t < NJT; ++t) {
    f32x16 acc = (f32x16)0.0f;
    const int j = t * 32 + l32;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a;
      if (j < nrows) {
        const float* rp = R + j * 64 + 16 * s + 8 * h;
        float4 x0 = *(const float4*)rp, x1 = *(const float4*)(rp + 4);
        a[0] = (bf16)x0.x; a[1] = (bf16)x0.y; a[2] = (bf16)x0.z; a[3] = (bf16)x0.w;
        a[4] = (bf16)x1.x; a[5] = (bf16)x1.y; a[6] = (bf16)x1.z; a[7] = (bf16)x1.w;
      } else {
        a = (bf16x8)(bf16)0.0f;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) prel[(t * 32 + acc_row(r, h)) * 33 + l32] = acc[r] * 8.0f;
  }
}

// ------------------------------------------------------------------------------------ global
constexpr int G_NW = 4, G_THR = G_NW * 64;
constexpr int VT_LD = 68;  // V^T row stride (bf16): 64 keys + 4 pad -> conflict-free ds_read_b64

struct GSmem {
  bf16 k[2][64 * 64];
  bf16 vt[2][64 * VT_LD];
  float prel[G_NW][128 * 33];
};

__global__ __launch_bounds__(G_THR) void vit_attn_global_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                const float* __restrict__ Rh,
                                                                const float* __restrict__ Rw, int heads) {
  constexpr int S = 64, T = 4096;
  __shared__ __attribute__((aligned(16))) GSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int head = blockIdx.y, seq = blockIdx.z;
  const int D = heads * 64, ld = 3 * D;
  const bf16* base = qkv + (long long)seq * T * ld;
  const int q = blockIdx.x * (G_NW * 32) + wave * 32 + l32;
  const int qh = q >> 6, qw = q & 63;

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = scale8(*(const bf16x8*)(base + (long long)q * ld + head * 64 + 16 * s + 8 * h));

  // rel_w: fixed for the whole key loop (key tile = one key image row, kw = row index in tile)
  float* prel = sm.prel[wave];
  relpos_table<4>(Rw, 2 * S - 1, qf, prel, lane);
  __syncthreads();
  float relw[2][16];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int kw = 32 * t2 + acc_row(r, h);
      relw[t2][r] = prel[(qw - kw + S - 1) * 33 + l32];
    }
  __syncthreads();
  relpos_table<4>(Rh, 2 * S - 1, qf, prel, lane);  // rel_h read per tile below

  // K/V tile staging: 64 keys x 64 d, 512 16-B chunks of each, 2 per thread.
  const bf16* kbase = base + D + head * 64;
  const bf16* vbase = base + 2 * D + head * 64;
  bf16x8 kreg[2], vreg[2];
  auto gload = [&](int tile) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int ci = tid + i * G_THR;
      int key = ci >> 3, c = ci & 7;
      long long off = (long long)(tile * 64 + key) * ld + c * 8;
      kreg[i] = *(const bf16x8*)(kbase + off);
      vreg[i] = *(const bf16x8*)(vbase + off);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int ci = tid + i * G_THR;
      int key = ci >> 3, c = ci & 7;
      *(bf16x8*)(sm.k[buf] + ksw(key, c)) = kreg[i];
      bf16* vt = sm.vt[buf];
#pragma unroll
      for (int e = 0; e < 8; ++e) vt[(c * 8 + e) * VT_LD + key] = vreg[i][e];
    }
  };

  f32x16 acc_o[2];
  acc_o[0] = (f32x16)0.0f;
  acc_o[1] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;

  gload(0);
  lstore(0);
  __syncthreads();
  constexpr int NT = T / 64;
  for (int tile = 0; tile < NT; ++tile) {
    const int buf = tile & 1;
    if (tile + 1 < NT) gload(tile + 1);
    const bf16* sk = sm.k[buf];
    const bf16* svt = sm.vt[buf];
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      sacc[t2] = (f32x16)0.0f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 a = *(const bf16x8*)(sk + ksw(t2 * 32 + l32, 2 * s + h));
        sacc[t2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], sacc[t2], 0, 0, 0);
      }
    }
    // tile = key image row kh
    const float relh = prel[(qh - tile + S - 1) * 33 + l32];
    float mx = -INFINITY;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = sacc[t2][r] + relw[t2][r] + relh;
        sacc[t2][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __expf(m_run - m_new);
    m_run = m_new;
    float ls = 0.0f;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __expf(sacc[t2][r] - m_new);
        sacc[t2][r] = p;
        ls += p;
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int td = 0; td < 2; ++td)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc_o[td][r] *= alpha;
    // O^T += V^T · P^T over the 64 keys (4 k-steps of 16)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf = pack8(sacc[ks >> 1], 8 * (ks & 1));
#pragma unroll
      for (int td = 0; td < 2; ++td) {
        const bf16* row = svt + (td * 32 + l32) * VT_LD + 16 * ks + 4 * h;
        bf16x4 lo = *(const bf16x4*)row;
        bf16x4 hi = *(const bf16x4*)(row + 8);
        bf16x8 vf;
        vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
        vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
        acc_o[td] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, acc_o[td], 0, 0, 0);
      }
    }
    if (tile + 1 < NT) lstore(buf ^ 1);
    __syncthreads();
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  bf16* orow = out + ((long long)seq * T + q) * D + head * 64;
#pragma unroll
  for (int td = 0; td < 2; ++td)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)(acc_o[td][4 * g + e] * inv);
      *(bf16x4*)(orow + td * 32 + 8 * g + 4 * h) = o;
    }
}

// ------------------------------------------------------------------------------------ global, v2
// 8 waves (256 queries = 4 image rows) per workgroup, two waves per SIMD so one wave's softmax overlaps
// the other's MFMAs. K and V tiles (64 keys x 64 d) stream global -> LDS with global_load_lds into a
// 3-deep ring (one instruction per wave per operand per tile, counted vmcnt + raw barrier). K keeps the
// ds_read_b128 swizzle; V stays row-major and is read transposed with ds_read_b64_tr_b16 (its image
// swaps 64-B halves on rows 2,3 mod 4 so the transposed reads are conflict-free). rel_w lives in
// registers; rel_h as a [64 kh][32 q] fp32 table per wave. Softmax in base 2 (one FMA + exp per score).
namespace g2 {
constexpr int NW = 8, THR = NW * 64, NBUF = 3;
constexpr int RELH_BYTES = NW * 64 * 32 * 4;       // 64 KiB
constexpr int TILE_BYTES = 2 * 64 * 128;            // K + V, 16 KiB
constexpr int SMEM = RELH_BYTES + NBUF * TILE_BYTES;  // 112 KiB
constexpr int SCR_LD = 33;                          // rel_w scratch [96][33] per wave (overlaps the above)
constexpr float L2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int vsw(int r, int c) { return r * 128 + ((c ^ (((r >> 1) & 1) << 2)) << 4); }
__device__ __forceinline__ int ksw_b(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}



// 32 table rows j0 .. j0+31 of P^T = R · Qs^T (times 8: undo the 1/8 folded into Qs), rows >= nrows zero.
__device__ __forceinline__ f32x16 rel_block(const float* __restrict__ R, int j0, int nrows, const bf16x8 (&qf)[4],
                                            int lane) {
  const int h = lane >> 5, j = j0 + (lane & 31);
  f32x16 acc = (f32x16)0.0f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 a;
    if (j >= 0 && j < nrows) {
      const float* rp = R + j * 64 + 16 * s + 8 * h;
      float4 x0 = *(const float4*)rp, x1 = *(const float4*)(rp + 4);
      a[0] = (bf16)x0.x; a[1] = (bf16)x0.y; a[2] = (bf16)x0.z; a[3] = (bf16)x0.w;
      a[4] = (bf16)x1.x; a[5] = (bf16)x1.y; a[6] = (bf16)x1.z; a[7] = (bf16)x1.w;
    } else {
      a = (bf16x8)(bf16)0.0f;
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], acc, 0, 0, 0);
  }
  return acc * 8.0f;
}

// K and V tile `tile` -> ring slot: 8 instructions of 1 KiB (8 rows x 128 B) per operand, one per wave
__device__ __forceinline__ void load_tile(const bf16* kbase, const bf16* vbase, int ld, int tile, char* slot,
                                          int wave, int lane) {
  const int r = wave * 8 + (lane >> 3), sl = lane & 7;
  const long long row = (long long)(tile * 64 + r) * ld;
  const int ck = sl ^ ((r >> 1) & 7), cv = sl ^ (((r >> 1) & 1) << 2);
  __builtin_amdgcn_global_load_lds((const void*)(kbase + row + ck * 8), (lds_ptr_t)(slot + wave * 1024), 16, 0, 0);
  __builtin_amdgcn_global_load_lds((const void*)(vbase + row + cv * 8), (lds_ptr_t)(slot + 8192 + wave * 1024), 16,
                                   0, 0);
}
}  // namespace g2

__global__ __launch_bounds__(g2::THR, 2) void vit_attn_global2_kernel(const bf16* __restrict__ qkv,
                                                                      bf16* __restrict__ out,
                                                                      const float* __restrict__ Rh,
                                                                      const float* __restrict__ Rw, int heads) {
  using namespace g2;
  constexpr int S = 64, T = 4096, NT = T / 64;
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int head = blockIdx.y, seq = blockIdx.z;
  const int D = heads * 64, ld = 3 * D;
  const bf16* base = qkv + (long long)seq * T * ld;
  const int q = blockIdx.x * (NW * 32) + wave * 32 + l32;
  const int qh = q >> 6, qw = q & 63, qw0 = qw - l32;
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);  // static priority: the SIMD's two waves drift apart

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = scale8(*(const bf16x8*)(base + (long long)q * ld + head * 64 + 16 * s + 8 * h));

  // rel_w (registers): rows j = qw - kw + 63 in [qw0, qw0 + 95) of the table, staged through scratch
  float* scr = (float*)gsm + wave * (96 * SCR_LD);
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 t = rel_block(Rw, qw0 + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) scr[(32 * b + acc_row(r, h)) * SCR_LD + l32] = t[r];
  }
  __syncthreads();
  // rel_w in natural units, as the initial accumulator of the S^T chain (free: the MFMA's C operand)
  f32x16 relw[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; ++r) relw[t2][r] = scr[(l32 - (32 * t2 + acc_row(r, h)) + 63) * SCR_LD + l32];
  __syncthreads();
  // rel_h table [kh][q]: row j = qh - kh + 63 -> block rows i = j - qh = 63 - kh
  float* relh = (float*)gsm + wave * (64 * 32);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const f32x16 t = rel_block(Rh, qh + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) relh[(63 - (32 * b + acc_row(r, h))) * 32 + l32] = t[r] * L2E;
  }
  __syncthreads();

  const bf16* kbase = base + D + head * 64;
  const bf16* vbase = base + 2 * D + head * 64;
  char* ring = gsm + RELH_BYTES;
  load_tile(kbase, vbase, ld, 0, ring, wave, lane);
  load_tile(kbase, vbase, ld, 1, ring + TILE_BYTES, wave, lane);

  f32x16 acc_o[2];
  acc_o[0] = (f32x16)0.0f;
  acc_o[1] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;  // base-2 running max / sum
  // tr-read lane geometry (V^T operand): group g = lane >> 4, lane 4qq + pp of the group
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;

  for (int tile = 0; tile < NT; ++tile) {
    if (tile + 1 < NT) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    if (tile + 2 < NT) load_tile(kbase, vbase, ld, tile + 2, ring + ((tile + 2) % NBUF) * TILE_BYTES, wave, lane);
    const char* sk = ring + (tile % NBUF) * TILE_BYTES;
    const char* sv = sk + 8192;
    // S^T + rel_w (natural units): the chain starts from the rel_w registers
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 a = *(const bf16x8*)(sk + ksw_b(t2 * 32 + l32, 2 * s + h));
        sacc[t2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], s == 0 ? relw[t2] : sacc[t2], 0, 0, 0);
      }
    }
    // tile = key image row kh: rel_h is one constant per lane (log2 units), so max and exponent take it
    // once per tile: p = exp2(L2E * s + (rh - m)), one FMA + one exp per score
    const float rh = relh[tile * 32 + l32];
    // (no inline-asm v_max3 here: hipcc's hazard recognizer does not see an asm statement read the MFMA
    // result registers, and an early read made the row max -- and the rounding -- nondeterministic)
    float mx = -INFINITY;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = fmaxf(mx, fmaxf(sacc[t2][r], sacc[t2][r + 1]));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, fmaf(mx, L2E, rh));
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    const float c = rh - m_new;
    float ls = 0.0f;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(sacc[t2][r], L2E, c));
        sacc[t2][r] = pv;
        ls += pv;
      }
    l_run = fmaf(l_run, alpha, ls);
    if (__builtin_amdgcn_ballot_w64(alpha != 1.0f)) {
#pragma unroll
      for (int td = 0; td < 2; ++td) acc_o[td] *= alpha;
    }
    // O^T += V^T · P^T: P^T k-slot j of lane half hh is key 16ks + 8(j>>2) + 4hh + (j&3)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 pf = pack8(sacc[ks >> 1], 8 * (ks & 1));
#pragma unroll
      for (int td = 0; td < 2; ++td) {
        const int r0 = 16 * ks + 4 * (g >> 1) + qq;
        const int ch = 4 * td + 2 * (g & 1) + (pp >> 1);
        const char* a0 = sv + vsw(r0, ch) + 8 * (pp & 1);
        const char* a1 = sv + vsw(r0 + 8, ch) + 8 * (pp & 1);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc_o[td] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v8), pf, acc_o[td], 0, 0, 0);
      }
    }
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  bf16* orow = out + ((long long)seq * T + q) * D + head * 64;
#pragma unroll
  for (int td = 0; td < 2; ++td)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)(acc_o[td][4 * gg + e] * inv);
      *(bf16x4*)(orow + td * 32 + 8 * gg + 4 * h) = o;
    }
}

// ------------------------------------------------------------------------------------ window
constexpr int W_NW = 7, W_THR = W_NW * 64;
constexpr int W_KEYS = 256;
constexpr int WVT_LD = W_KEYS + 4;

struct WSmem {
  bf16 k[W_KEYS * 64];
  bf16 vt[64 * WVT_LD];
  float prel[W_NW][2][32 * 33];
};

__global__ __launch_bounds__(W_THR) void vit_attn_window_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                const float* __restrict__ Rh,
                                                                const float* __restrict__ Rw, int heads) {
  constexpr int S = 14, T = 196;
  __shared__ __attribute__((aligned(16))) WSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int head = blockIdx.y, win = blockIdx.x;
  const int D = heads * 64, ld = 3 * D;
  const bf16* base = qkv + (long long)win * T * ld;

  // stage the whole window's K (row-major, swizzled) and V^T; keys >= 196 zero
  for (int ci = tid; ci < W_KEYS * 8; ci += W_THR) {
    int key = ci >> 3, c = ci & 7;
    bf16x8 kv = (bf16x8)(bf16)0.0f, vv = (bf16x8)(bf16)0.0f;
    if (key < T) {
      kv = *(const bf16x8*)(base + (long long)key * ld + D + head * 64 + c * 8);
      vv = *(const bf16x8*)(base + (long long)key * ld + 2 * D + head * 64 + c * 8);
    }
    *(bf16x8*)(sm.k + ksw(key, c)) = kv;
#pragma unroll
    for (int e = 0; e < 8; ++e) sm.vt[(c * 8 + e) * WVT_LD + key] = vv[e];
  }

  const int q = wave * 32 + l32;
  const bool qvalid = q < T;
  const int qh = qvalid ? q / S : 0, qw = qvalid ? q % S : 0;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = qvalid ? scale8(*(const bf16x8*)(base + (long long)q * ld + head * 64 + 16 * s + 8 * h))
                   : (bf16x8)(bf16)0.0f;
  relpos_table<1>(Rw, 2 * S - 1, qf, sm.prel[wave][0], lane);
  relpos_table<1>(Rh, 2 * S - 1, qf, sm.prel[wave][1], lane);
  __syncthreads();
  float relw[S], relh[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    relw[i] = sm.prel[wave][0][(qw - i + S - 1) * 33 + l32];
    relh[i] = sm.prel[wave][1][(qh - i + S - 1) * 33 + l32];
  }

  f32x16 acc_o[2];
  acc_o[0] = (f32x16)0.0f;
  acc_o[1] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;
#pragma unroll
  for (int tile = 0; tile < W_KEYS / 64; ++tile) {
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      sacc[t2] = (f32x16)0.0f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 a = *(const bf16x8*)(sm.k + ksw(tile * 64 + t2 * 32 + l32, 2 * s + h));
        sacc[t2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], sacc[t2], 0, 0, 0);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // key index for lane half 0 and 1 (compile-time), selected by h
        constexpr int dummy = 0;
        (void)dummy;
        const int k0 = tile * 64 + t2 * 32 + acc_row(r, 0);
        const int k1 = k0 + 4;
        float b0 = (k0 < T) ? relh[(k0 < T ? k0 : 0) / S] + relw[(k0 < T ? k0 : 0) % S] : -INFINITY;
        float b1 = (k1 < T) ? relh[(k1 < T ? k1 : 0) / S] + relw[(k1 < T ? k1 : 0) % S] : -INFINITY;
        float v = sacc[t2][r] + (h ? b1 : b0);
        sacc[t2][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __expf(m_run - m_new);
    m_run = m_new;
    float ls = 0.0f;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __expf(sacc[t2][r] - m_new);
        sacc[t2][r] = p;
        ls += p;
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int td = 0; td < 2; ++td)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc_o[td][r] *= alpha;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf = pack8(sacc[ks >> 1], 8 * (ks & 1));
#pragma unroll
      for (int td = 0; td < 2; ++td) {
        const bf16* row = sm.vt + (td * 32 + l32) * WVT_LD + tile * 64 + 16 * ks + 4 * h;
        bf16x4 lo = *(const bf16x4*)row;
        bf16x4 hi = *(const bf16x4*)(row + 8);
        bf16x8 vf;
        vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
        vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
        acc_o[td] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, acc_o[td], 0, 0, 0);
      }
    }
  }
  if (!qvalid) return;
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  bf16* orow = out + ((long long)win * T + q) * D + head * 64;
#pragma unroll
  for (int td = 0; td < 2; ++td)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)(acc_o[td][4 * g + e] * inv);
      *(bf16x4*)(orow + td * 32 + 8 * g + 4 * h) = o;
    }
}

// ------------------------------------------------------------------------------------ window, v2
// Same mapping as vit_attn_window_kernel (7 waves x 32 queries, the window's 196 keys padded to 256 and
// masked, rel_w / rel_h from MFMA tables), with 64 KiB of LDS instead of 124 so that two workgroups share a
// CU: K keeps the swizzled row image; V stays row-major (LDS image of global2's tr-read swizzle) and is
// read transposed with ds_read_b64_tr_b16; the per-wave rel-pos tables are staged one after the other
// through a scratch that overlays the V image before V is written. Key blocks that hold only padding
// (keys 224..255: the second half of the last 64-key tile) are skipped.
namespace w2 {
constexpr int NW = 7, THR = NW * 64, KEYS = 256;
constexpr int K_BYTES = KEYS * 128, V_BYTES = KEYS * 128;
constexpr int SMEM = K_BYTES + V_BYTES;  // 64 KiB
static_assert(NW * 32 * 33 * 4 <= V_BYTES, "rel-pos scratch must fit in the V image");
}  // namespace w2

__global__ __launch_bounds__(w2::THR, 2) void vit_attn_window2_kernel(const bf16* __restrict__ qkv,
                                                                      bf16* __restrict__ out,
                                                                      const float* __restrict__ Rh,
                                                                      const float* __restrict__ Rw, int heads) {
  using namespace g2;
  constexpr int S = 14, T = 196;
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  char* kimg = wsm;
  char* vimg = wsm + w2::K_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int head = blockIdx.y, win = blockIdx.x;
  const int D = heads * 64, ld = 3 * D;
  const bf16* base = qkv + (long long)win * T * ld;

  // K rows (swizzled [256][64] image; keys >= 196 zero)
  for (int ci = tid; ci < w2::KEYS * 8; ci += w2::THR) {
    const int key = ci >> 3, c = ci & 7;
    bf16x8 kv = (bf16x8)(bf16)0.0f;
    if (key < T) kv = *(const bf16x8*)(base + (long long)key * ld + D + head * 64 + c * 8);
    *(bf16x8*)(kimg + 2 * ksw(key, c)) = kv;
  }
  const int q = wave * 32 + l32;
  const bool qvalid = q < T;
  const int qh = qvalid ? q / S : 0, qw = qvalid ? q % S : 0;
  bf16x8 qf[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4)
    qf[s4] = qvalid ? scale8(*(const bf16x8*)(base + (long long)q * ld + head * 64 + 16 * s4 + 8 * h))
                    : (bf16x8)(bf16)0.0f;
  // rel_w then rel_h through this wave's scratch (inside the V image; LDS ops of one wave run in order)
  float* scr = (float*)vimg + wave * (32 * 33);
  float relw[S], relh[S];
  relpos_table<1>(Rw, 2 * S - 1, qf, scr, lane);
#pragma unroll
  for (int i = 0; i < S; ++i) relw[i] = scr[(qw - i + S - 1) * 33 + l32];
  relpos_table<1>(Rh, 2 * S - 1, qf, scr, lane);
#pragma unroll
  for (int i = 0; i < S; ++i) relh[i] = scr[(qh - i + S - 1) * 33 + l32];
  __syncthreads();  // every wave is done with its scratch: the V image may be written
  for (int ci = tid; ci < w2::KEYS * 8; ci += w2::THR) {
    const int key = ci >> 3, c = ci & 7;
    bf16x8 vv = (bf16x8)(bf16)0.0f;
    if (key < T) vv = *(const bf16x8*)(base + (long long)key * ld + 2 * D + head * 64 + c * 8);
    *(bf16x8*)(vimg + vsw(key, c)) = vv;
  }
  __syncthreads();

  f32x16 acc_o[2];
  acc_o[0] = (f32x16)0.0f;
  acc_o[1] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
  for (int tile = 0; tile < w2::KEYS / 64; ++tile) {
    constexpr int dummy = 0;
    (void)dummy;
    const int nb = tile == 3 ? 1 : 2;  // 32-key blocks holding a real key (keys < 224)
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      sacc[t2] = (f32x16)0.0f;
      if (t2 < nb) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          bf16x8 a = *(const bf16x8*)(kimg + 2 * ksw(tile * 64 + t2 * 32 + l32, 2 * s4 + h));
          sacc[t2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s4], sacc[t2], 0, 0, 0);
        }
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k0 = tile * 64 + t2 * 32 + acc_row(r, 0);
        const int k1 = k0 + 4;
        float b0 = (k0 < T) ? relh[(k0 < T ? k0 : 0) / S] + relw[(k0 < T ? k0 : 0) % S] : -INFINITY;
        float b1 = (k1 < T) ? relh[(k1 < T ? k1 : 0) / S] + relw[(k1 < T ? k1 : 0) % S] : -INFINITY;
        float v = sacc[t2][r] + (h ? b1 : b0);
        sacc[t2][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __expf(m_run - m_new);
    m_run = m_new;
    float ls = 0.0f;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float pv = __expf(sacc[t2][r] - m_new);
        sacc[t2][r] = pv;
        ls += pv;
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int td = 0; td < 2; ++td) acc_o[td] *= alpha;
    // O^T += V^T P^T over the tile's real 16-key steps (the last tile: keys 192..207 only)
    const char* sv = vimg + tile * 64 * 128;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (tile == 3 && ks > 0) break;
      const bf16x8 pf = pack8(sacc[ks >> 1], 8 * (ks & 1));
#pragma unroll
      for (int td = 0; td < 2; ++td) {
        const int r0 = 16 * ks + 4 * (g >> 1) + qq;
        const int ch = 4 * td + 2 * (g & 1) + (pp >> 1);
        const char* a0 = sv + vsw(r0, ch) + 8 * (pp & 1);
        const char* a1 = sv + vsw(r0 + 8, ch) + 8 * (pp & 1);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc_o[td] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v8), pf, acc_o[td], 0, 0, 0);
      }
    }
  }
  if (!qvalid) return;
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / l_tot;
  bf16* orow = out + ((long long)win * T + q) * D + head * 64;
#pragma unroll
  for (int td = 0; td < 2; ++td)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)(acc_o[td][4 * gg + e] * inv);
      *(bf16x4*)(orow + td * 32 + 8 * gg + 4 * h) = o;
    }
}

}  // namespace

static int g_attn_v2 = 1;
extern "C" void octsam_attention_set_variant(int32_t v) { g_attn_v2 = v; }

extern "C" int octsam_vit_attention(const void* qkv, void* out, const float* rel_pos_h, const float* rel_pos_w,
                                    int32_t nseq, int32_t side, int32_t heads, int32_t head_dim, void* stream) {
  OCTSAM_CHECK_ARG(qkv && out && rel_pos_h && rel_pos_w && nseq > 0 && heads > 0,
                   "octsam_vit_attention: bad args");
  OCTSAM_CHECK_ARG(head_dim == 64, "octsam_vit_attention: head_dim must be 64 (got %d)", head_dim);
  hipStream_t s = (hipStream_t)stream;
  if (side == 64 && g_attn_v2) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)vit_attn_global2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                g2::SMEM);
      attr = true;
    }
    dim3 grid(4096 / (g2::NW * 32), heads, nseq);
    hipLaunchKernelGGL(vit_attn_global2_kernel, grid, dim3(g2::THR), g2::SMEM, s, (const bf16*)qkv, (bf16*)out,
                       rel_pos_h, rel_pos_w, heads);
  } else if (side == 64) {
    dim3 grid(4096 / (G_NW * 32), heads, nseq);
    hipLaunchKernelGGL(vit_attn_global_kernel, grid, dim3(G_THR), 0, s, (const bf16*)qkv, (bf16*)out, rel_pos_h,
                       rel_pos_w, heads);
  } else if (side == 14 && g_attn_v2 == 2) {  // (64 KiB variant; VGPR-bound to one workgroup per CU like v1)
    static bool wattr = false;
    if (!wattr) {
      (void)hipFuncSetAttribute((const void*)vit_attn_window2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                w2::SMEM);
      wattr = true;
    }
    dim3 grid(nseq, heads, 1);
    hipLaunchKernelGGL(vit_attn_window2_kernel, grid, dim3(w2::THR), w2::SMEM, s, (const bf16*)qkv, (bf16*)out,
                       rel_pos_h, rel_pos_w, heads);
  } else if (side == 14) {
    dim3 grid(nseq, heads, 1);
    hipLaunchKernelGGL(vit_attn_window_kernel, grid, dim3(W_THR), 0, s, (const bf16*)qkv, (bf16*)out, rel_pos_h,
                       rel_pos_w, heads);
  } else {
    octsam::set_error("octsam_vit_attention: side must be 64 (global) or 14 (window), got %d", side);
    return 1;
  }
  OCTSAM_LAUNCH_CHECK("octsam_vit_attention");
  return 0;
}
