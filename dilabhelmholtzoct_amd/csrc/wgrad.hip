// Image-side weight gradients of the mask decoder (the backward of the per-prompt image-side projections,
// hf modeling_sam.py:219-221 / 254 q,k,v_proj and out_proj on the keys, and the upscaling ConvT1 :1054):
//
//   out[o][i] (+)= sum_m dY[m][o] * X[m][i]      m over the P*4096 per-prompt image rows (688 128 at the bench)
//   db[o] = sum_m dY[m][o],  dbx[i mod I/fold] = sum_m X[m][i]            (bias gradients, optional)
//
// with O in {128, 256, 384} and I in {128, 256}: a tall reduction whose operands (O + I bf16 per row, 1280 B at
// O = 384, I = 256) are the whole cost. Each workgroup holds the WHOLE O x I output in its accumulators (8 waves as
// 2 (O) x 4 (I), up to 192 fp32 per lane) and streams one contiguous range of rows through a 4-stage LDS-DMA ring,
// so every operand byte crosses HBM once and 80-120 KB per CU stay in flight. (The split-K tile GEMM it replaces
// re-reads A per N tile and B per M tile through L2, keeps one 48 KB stage in flight and reached 1.85 TB/s,
// scripts/dw_ab.py.) Fragments come from the LDS images by ds_read_b64_tr_b16 (the operands are k-major: row m of
// dY holds the k-th element of every output row o). The per-workgroup partials (fp32 [nwg][O][I], plus the column
// sums) are summed over workgroups in a fixed order by a second launch: deterministic, independent of timing.
#include "common.h"
#include "../../include/octsam.h"

extern "C" int octsam_splitk_reduce(const float* partials, float* out, int64_t n, int32_t splits, float beta,
                                    void* stream);

namespace {
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int SROWS = 32;  // rows (k) per ring stage
constexpr int NS = 4;      // ring stages (160 KB at O = 384, I = 256)

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Stage image of a k-major operand [SROWS rows][W columns] in 8-row x 32-column subtiles of 512 B (64-B rows), laid
// out across the whole width so that subtile X of a row group sits at a constant 512 X: byte offset of 16-B chunk
// ch of row r = rowg (r >> 3) + 512 (ch >> 2) + 64 (r & 7) + 16 (ch & 3), rowg = 16 W. A fragment read (32 lanes:
// 4 rows x 2 x 16 columns) then covers 4 whole 64-B rows = all 64 banks once: conflict-free without a swizzle, and
// the second read of a fragment (rows + 4) is the first one + 256 B.
//
// One stage: 1 KiB LDS-DMA buffer loads, each two subtiles (64 columns) of one row group; instruction J of the
// W/64 per row group, wave w issues J = w, w + 8, ... (J counted across both operands: j0 = the instructions of the
// operand before this one). The buffer descriptor spans the workgroup's rows only; voffset = the lane's part (row rr
// of the group, chunk 4 st + slot: the same for every instruction), soffset = the stage's rows + 16 ld gq + 128 jp.
// Rows past the range read as zero: gfx950's raw-buffer range check covers voffset + soffset (measured,
// scripts/probe/range_probe.hip), so a workgroup's partial last stage needs no per-lane test.
__device__ __forceinline__ int stage_lane_off(long long ld, int lane) {
  const int st = lane >> 5, rr = (lane >> 2) & 7, slot = lane & 3;
  return (int)(rr * ld * 2) + 64 * st + 16 * slot;
}
template <int W, int NJ>
__device__ __forceinline__ void stage_load(const bf16* base, int bytes, long long ld, int soff, char* lds, int voff,
                                           int wave, int j0) {
  constexpr int PER_G = W / 64, NINST = 4 * PER_G, ROWG = 16 * W;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int J = wave + 8 * jj - j0;  // wave-uniform
    if (J >= 0 && J < NINST) {
      const int gq = J / PER_G, jp = J - gq * PER_G;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(lds + ROWG * gq + 1024 * jp), 16, voff,
                                               soff + (int)(16 * ld * gq) + 128 * jp, 0, 0);
    }
  }
}

// lane part of a fragment read address (32x32x16 operand: 8 consecutive k, k = kb + 8 (lane >> 5) + t, of column
// 32 X + (lane & 31)): lane 4q + p of each 16-lane group gives row 8 (g >> 1) + q, columns 4p .. 4p + 3 of its
// 16-column block (chunk 2 (g & 1) + (p >> 1)); the subtile (512 X), the k block (rowg kb / 8) and the second read
// (+256: rows + 4) are immediates
template <int W>
__device__ __forceinline__ int frag_lane_off(int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  return 16 * W * (g >> 1) + 64 * q + 16 * (2 * (g & 1) + (p >> 1)) + 8 * (p & 1);
}

__device__ __forceinline__ bf16x8 frag(const char* base, int imm) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + imm));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + imm + 256));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// s + the 8 elements of a fragment (v_dot2 with ones: exact products, fp32 sums, fixed order)
__device__ __forceinline__ float frag_sum(bf16x8 v, float s) {
  const bf16x2 one = {(bf16)1.0f, (bf16)1.0f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bf16x2 pr = {v[2 * q], v[2 * q + 1]};
    s = __builtin_amdgcn_fdot2_f32_bf16(pr, one, s, false);
  }
  return s;
}

template <int GLW>
__device__ __forceinline__ void wait_stage(int ahead) {  // leave `ahead` younger stages (GLW loads each) in flight
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GLW) : "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GLW) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// NBO x NBI 32x32 accumulator blocks per wave: O = 64 NBO (2 wave rows), I = 128 NBI (4 wave columns)
template <int NBO, int NBI>
__global__ __launch_bounds__(512, 1) void wgrad_kernel(const bf16* __restrict__ dy, long long ldy,
                                                       const bf16* __restrict__ x, long long ldx, long long M,
                                                       long long rows_per, float* __restrict__ part,
                                                       float* __restrict__ cs_a, float* __restrict__ cs_b) {
  constexpr int O = 64 * NBO, I = 128 * NBI;
  constexpr int A_BYTES = SROWS * O * 2, STAGE = SROWS * (O + I) * 2;
  constexpr int NA = O / 16, NB = I / 16, GLW = (NA + NB) / 8;  // 1 KiB loads per stage: per operand, per wave
  static_assert(NBO % 2 == 0 && (NA + NB) % 8 == 0 && NS * STAGE <= 160 * 1024, "stage ring exceeds the LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wave >> 2, wi = wave & 3;
  const long long m_beg = (long long)blockIdx.x * rows_per;
  const long long m_end = min(M, m_beg + rows_per);
  const int nst = (int)((m_end - m_beg + SROWS - 1) / SROWS);  // >= 1 (host sizes the grid)

  // instructions per wave: A covers J in [0, NA), B in [NA, NA + NB)
  constexpr int NJA = (NA + 7) / 8, NJB = (NA + NB + 7) / 8;
  int va = stage_lane_off(ldy, lane), vb = stage_lane_off(ldx, lane);
  asm volatile("" : "+v"(va), "+v"(vb));
  const bf16* a_base = dy + m_beg * ldy;
  const bf16* b_base = x + m_beg * ldx;
  const int a_bytes = (int)((m_end - m_beg) * ldy * 2), b_bytes = (int)((m_end - m_beg) * ldx * 2);
  auto issue = [&](int s) {
    char* st = smem + (s % NS) * STAGE;
    stage_load<O, NJA>(a_base, a_bytes, ldy, (int)(s * SROWS * ldy * 2), st, va, wave, 0);
    stage_load<I, NJB>(b_base, b_bytes, ldx, (int)(s * SROWS * ldx * 2), st + A_BYTES, vb, wave, NA);
  };
  // fragment bases: lane part + this wave's first subtile (A: 32 NBO wo columns, B: 32 NBI wi columns)
  int a_off = frag_lane_off<O>(lane) + 512 * NBO * wo;
  int b_off = A_BYTES + frag_lane_off<I>(lane) + 512 * NBI * wi;
  // one register each: keep the compiler from carrying the sums' terms separately (the accumulators leave few)
  asm volatile("" : "+v"(a_off), "+v"(b_off));

  f32x16 acc[NBO][NBI];
#pragma unroll
  for (int b = 0; b < NBO; ++b)
#pragma unroll
    for (int c = 0; c < NBI; ++c) acc[b][c] = (f32x16)0.0f;
  // column sums: A block b of wave row wo is summed by the wave with wi == b % 4 (into csa[b / 4]), B block c of
  // wave column wi by the wave with wo == c: every column exactly once per workgroup
  float csa[(NBO + 3) / 4], csb = 0.0f;
#pragma unroll
  for (int b = 0; b < (NBO + 3) / 4; ++b) csa[b] = 0.0f;
  const bool want_a = cs_a != nullptr, want_b = cs_b != nullptr && wo < NBI;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) issue(s);
  for (int s = 0; s < nst; ++s) {
    wait_stage<GLW>(min(NS - 2, nst - 1 - s));
    raw_barrier();
    if (s + NS - 1 < nst) issue(s + NS - 1);
    const char* sg = smem + (s % NS) * STAGE;
#pragma unroll
    for (int kk = 0; kk < SROWS / 16; ++kk) {
      bf16x8 bfr[NBI];
#pragma unroll
      for (int c = 0; c < NBI; ++c) bfr[c] = frag(sg + b_off, 32 * I * kk + 512 * c);
#pragma unroll
      for (int b = 0; b < NBO; ++b) {
        const bf16x8 af = frag(sg + a_off, 32 * O * kk + 512 * b);
#pragma unroll
        for (int c = 0; c < NBI; ++c)
          acc[b][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[c], acc[b][c], 0, 0, 0);
        if (want_a && (b & 3) == wi) csa[b >> 2] = frag_sum(af, csa[b >> 2]);
      }
      if (want_b) {
        bf16x8 f = bfr[0];
#pragma unroll
        for (int c = 1; c < NBI; ++c) f = wo == c ? bfr[c] : f;
        csb = frag_sum(f, csb);
      }
    }
  }

  // partials: element e of block (b, c) is out[o][i], o = ob + (e & 3) + 8 (e >> 2) + 4 (lane >> 5), i = ib + lane & 31
  // (buffer stores: one lane offset for every element, the element's row and block offsets are wave-uniform)
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(part + (long long)blockIdx.x * O * I), (short)0, O * I * 4, 0x00020000);
  const int p_lane = ((wo * 32 * NBO + 4 * (lane >> 5)) * I + wi * 32 * NBI + (lane & 31)) * 4;
#pragma unroll
  for (int b = 0; b < NBO; ++b)
#pragma unroll
    for (int c = 0; c < NBI; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        // (copy the element out first: a bit_cast of the vector-element lvalue reads element 0)
        const float v = acc[b][c][e];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rp, p_lane,
                                              ((32 * b + (e & 3) + 8 * (e >> 2)) * I + 32 * c) * 4, 0);
      }
  if (want_a) {
#pragma unroll
    for (int b = 0; b < NBO; ++b)
      if ((b & 3) == wi) {  // lanes l and l + 32 hold the two k halves of column (l & 31)
        const float v = csa[b >> 2] + __shfl_xor(csa[b >> 2], 32, 64);
        if (lane < 32) cs_a[(long long)blockIdx.x * O + wo * 32 * NBO + 32 * b + lane] = v;
      }
  }
  if (want_b) {
    const float v = csb + __shfl_xor(csb, 32, 64);
    if (lane < 32) cs_b[(long long)blockIdx.x * I + wi * 32 * NBI + 32 * wo + lane] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Token-side weight gradients (the P*T prompt-token rows, a few thousand: the decoder's token projections, MLPs and
// hypernetworks): out[o][i] (+)= sum_m dY[m][o] X[m][i] and db[o] = sum_m dY[m][o] in ONE launch. Workgroup = one
// 32 x 32 output tile; its NW waves split the rows into NW contiguous ranges and each streams its range through a
// wave-private 4-stage LDS-DMA ring (32 rows x 32 columns of each operand per stage, no workgroup barrier in the
// loop), one 32x32x16 MFMA per 16 rows; the NW partial tiles (and column sums) are added in fixed wave order
// through LDS. Replaces the split-K tile GEMM + its reduction + the bias column-sum kernel + its reduction.
#ifndef OCTSAM_TOK_W64
#define OCTSAM_TOK_W64 1
#endif
namespace tok {
constexpr int NST = 4;                    // ring stages per wave (4-wave workgroups: 64 KiB, two per CU)
#ifndef OCTSAM_TOK_NST8
#define OCTSAM_TOK_NST8 2
#endif
// ring stages per wave of the 8-wave form (M > 1024 rows; 4 stages = 128 KiB, one workgroup per CU; 2 = 64 KiB, two
// per CU: step 18.30 -> 18.24 ms sequential, 16.17 -> 16.14 pipelined, profiles/r06/tok_nst2_step_ab.log)
template <int NW> constexpr int nst() { return NW == 8 ? OCTSAM_TOK_NST8 : NST; }
constexpr int OPB = SROWS * 32 * 2;       // bytes of one operand per stage (2 KiB)
constexpr int STB = 2 * OPB;              // stage bytes (A then B)

// one operand's stage: two 1 KiB loads (rows 0-15, 16-31), lane -> (row group l >> 5, row (l >> 2) & 7, chunk l & 3)
__device__ __forceinline__ void tok_load(__amdgpu_buffer_rsrc_t rs, int voff, int soff, long long ld, char* lds) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(lds + 1024 * h), 16, voff, soff + (int)(32 * ld * h), 0,
                                             0);
}
}  // namespace tok

// one 32 x 32 output tile (tile = to * tiles_i + ti) of one token-side problem
template <int NW>
__device__ __forceinline__ void tok_tile(const bf16* __restrict__ dy, long long ldy, const bf16* __restrict__ x,
                                         long long ldx, long long M, int tile, int tiles_i, float* __restrict__ out,
                                         int ldo, float beta, float* __restrict__ db, char* smem) {
  using namespace tok;
  constexpr int NST = tok::nst<NW>();
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int to = tile / tiles_i, ti = tile - to * tiles_i;
  const int o0 = to * 32, i0 = ti * 32;
  // this wave's rows: [m_beg, m_end), 32-row multiples except the last range
  const long long per = ((M + NW - 1) / NW + SROWS - 1) / SROWS * SROWS;
  const long long m_beg = min(M, (long long)wave * per), m_end = min(M, m_beg + per);
  const int nst = (int)((m_end - m_beg + SROWS - 1) / SROWS);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dy + m_beg * ldy + o0), (short)0, (int)((m_end - m_beg) * ldy * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + m_beg * ldx + i0), (short)0, (int)((m_end - m_beg) * ldx * 2), 0x00020000);
  const int rr = 8 * (lane >> 5) + ((lane >> 2) & 7), slot = lane & 3;
  int va = (int)(rr * ldy * 2) + 16 * slot, vb = (int)(rr * ldx * 2) + 16 * slot;
  char* ring = smem + wave * NST * STB;
  // fragment read: 32 x 32 image (one subtile column), lane part as frag_lane_off<32>
  const int fo = frag_lane_off<32>(lane);

  f32x16 acc = (f32x16)0.0f;
  float cs = 0.0f;
  const bool want_cs = db != nullptr && ti == 0;
  auto issue = [&](int s) {
    char* st = ring + (s % NST) * STB;
    tok::tok_load(ra, va, (int)(s * SROWS * ldy * 2), ldy, st);
    tok::tok_load(rb, vb, (int)(s * SROWS * ldx * 2), ldx, st + OPB);
  };
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nst) issue(s);
  for (int s = 0; s < nst; ++s) {
    if (s + NST - 1 < nst) {
      issue(s + NST - 1);  // (its slot's reads finished in iteration s - 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NST - 1)) : "memory");
    } else {
      const int ahead = nst - 1 - s;  // 0 .. NST-2 younger stages
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const char* sg = ring + (s % NST) * STB + fo;
#pragma unroll
    for (int kk = 0; kk < SROWS / 16; ++kk) {
      const bf16x8 af = frag(sg, 1024 * kk);
      const bf16x8 bfr = frag(sg + OPB, 1024 * kk);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc, 0, 0, 0);
      if (want_cs) cs = frag_sum(af, cs);
    }
  }
  // fixed-order sum of the NW partial tiles (and column sums) through LDS (the rings are no longer read)
  __syncthreads();
  float* red = (float*)smem;  // [NW][16][64] accumulators, then [NW][32] column sums
#pragma unroll
  for (int e = 0; e < 16; ++e) red[(wave * 16 + e) * 64 + lane] = acc[e];
  if (want_cs) {
    const float v = cs + __shfl_xor(cs, 32, 64);
    if (lane < 32) red[NW * 1024 + wave * 32 + lane] = v;
  }
  __syncthreads();
  for (int idx = tid; idx < 1024; idx += NW * 64) {
    const int e = idx >> 6, l = idx & 63;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[(w * 16 + e) * 64 + l];
    const int o = o0 + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5), i = i0 + (l & 31);
    float* dst = out + (long long)o * ldo + i;
    *dst = beta != 0.0f ? v + beta * *dst : v;
  }
  if (want_cs && tid < 32) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[NW * 1024 + w * 32 + tid];
    db[o0 + tid] = v;
  }
}

// one 64 x 64 output tile of one token-side problem (O, I multiples of 64): the same row partition over the NW waves,
// stages of 32 rows, MFMA chain per 32x32 block and fixed-order wave sum as tok_tile, so every output element gets the
// same bits as from the 32 x 32 tiles, while each dy / x column block read serves 64 outputs instead of 32 (the 32 x 32
// tiles re-read the operands (O + I) / 32 times over, almost all of it past L2: 186 MB per grouped launch)
namespace tok {
constexpr int OPB64 = SROWS * 64 * 2;  // bytes of one operand per stage (4 KiB)
constexpr int STB64 = 2 * OPB64;
template <int NW> constexpr int nst64() { return 2; }
template <int NW> constexpr int lds64() {
  return NW * nst64<NW>() * STB64 > NW * (4096 + 64) * 4 ? NW * nst64<NW>() * STB64 : NW * (4096 + 64) * 4;
}
// one operand's stage, 64 columns: four 1 KiB loads (8-row groups; lane -> subtile lane >> 5, row (lane >> 2) & 7,
// chunk lane & 3: stage_lane_off), the image of stage_load's layout at W = 64
__device__ __forceinline__ void tok_load64(__amdgpu_buffer_rsrc_t rs, int voff, int soff, long long ld, char* lds) {
#pragma unroll
  for (int gq = 0; gq < 4; ++gq)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(lds + 1024 * gq), 16, voff, soff + (int)(16 * ld * gq), 0,
                                             0);
}
}  // namespace tok

template <int NW>
__device__ __forceinline__ void tok_tile64(const bf16* __restrict__ dy, long long ldy, const bf16* __restrict__ x,
                                           long long ldx, long long M, int tile, int tiles_i, float* __restrict__ out,
                                           int ldo, float beta, float* __restrict__ db, char* smem) {
  using namespace tok;
  constexpr int NST = tok::nst64<NW>();
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int to = tile / tiles_i, ti = tile - to * tiles_i;
  const int o0 = to * 64, i0 = ti * 64;
  const long long per = ((M + NW - 1) / NW + SROWS - 1) / SROWS * SROWS;
  const long long m_beg = min(M, (long long)wave * per), m_end = min(M, m_beg + per);
  const int nst = (int)((m_end - m_beg + SROWS - 1) / SROWS);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dy + m_beg * ldy + o0), (short)0, (int)((m_end - m_beg) * ldy * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + m_beg * ldx + i0), (short)0, (int)((m_end - m_beg) * ldx * 2), 0x00020000);
  const int va = stage_lane_off(ldy, lane), vb = stage_lane_off(ldx, lane);
  char* ring = smem + wave * NST * STB64;
  const int fo = frag_lane_off<64>(lane);

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16)0.0f;
  float cs[2] = {0.0f, 0.0f};
  const bool want_cs = db != nullptr && ti == 0;
  auto issue = [&](int s) {
    char* st = ring + (s % NST) * STB64;
    tok::tok_load64(ra, va, (int)(s * SROWS * ldy * 2), ldy, st);
    tok::tok_load64(rb, vb, (int)(s * SROWS * ldx * 2), ldx, st + OPB64);
  };
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nst) issue(s);
  for (int s = 0; s < nst; ++s) {
    if (s + NST - 1 < nst) {
      issue(s + NST - 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NST - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const char* sg = ring + (s % NST) * STB64 + fo;
#pragma unroll
    for (int kk = 0; kk < SROWS / 16; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = frag(sg, 2048 * kk + 512 * a);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = frag(sg + OPB64, 2048 * kk + 512 * b);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
      if (want_cs) {
#pragma unroll
        for (int a = 0; a < 2; ++a) cs[a] = frag_sum(af[a], cs[a]);
      }
    }
  }
  // fixed-order sum of the NW partial tiles (and column sums) through LDS (the rings are no longer read)
  __syncthreads();
  float* red = (float*)smem;  // [NW][4 blocks][16][64] accumulators, then [NW][64] column sums
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) red[((wave * 4 + 2 * a + b) * 16 + e) * 64 + lane] = acc[a][b][e];
  if (want_cs) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float v = cs[a] + __shfl_xor(cs[a], 32, 64);
      if (lane < 32) red[NW * 4096 + wave * 64 + 32 * a + lane] = v;
    }
  }
  __syncthreads();
  for (int idx = tid; idx < 4096; idx += NW * 64) {
    const int blk = idx >> 10, e = (idx >> 6) & 15, l = idx & 63;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[((w * 4 + blk) * 16 + e) * 64 + l];
    const int o = o0 + 32 * (blk >> 1) + (e & 3) + 8 * (e >> 2) + 4 * (l >> 5), i = i0 + 32 * (blk & 1) + (l & 31);
    float* dst = out + (long long)o * ldo + i;
    *dst = beta != 0.0f ? v + beta * *dst : v;
  }
  if (want_cs && tid < 64) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[NW * 4096 + w * 64 + tid];
    db[o0 + tid] = v;
  }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void wgrad_tok64_kernel(const bf16* __restrict__ dy, long long ldy,
                                                              const bf16* __restrict__ x, long long ldx, long long M,
                                                              int tiles_i, float* __restrict__ out, int ldo, float beta,
                                                              float* __restrict__ db) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tok_tile64<NW>(dy, ldy, x, ldx, M, blockIdx.x, tiles_i, out, ldo, beta, db, smem);
}

// 64 x 64 tiles for the larger problems (graph-replayed alone, scripts/tok_wgrad_time.py: MLP lin1's dW 12.1 -> 7.5
// us, lin2's 9.5 -> 7.4), 32 x 32 tiles while 64 x 64 ones would leave most CUs idle (a 256 x 256 dW: 4.2 vs 7.0 us)
inline bool tok_w64(int O, int I) { return OCTSAM_TOK_W64 && O % 64 == 0 && I % 64 == 0 && (O / 64) * (I / 64) >= 64; }

template <int NW>
__global__ __launch_bounds__(NW * 64) void wgrad_tok_kernel(const bf16* __restrict__ dy, long long ldy,
                                                            const bf16* __restrict__ x, long long ldx, long long M,
                                                            int tiles_i, float* __restrict__ out, int ldo, float beta,
                                                            float* __restrict__ db) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tok_tile<NW>(dy, ldy, x, ldx, M, blockIdx.x, tiles_i, out, ldo, beta, db, smem);
}

// Several independent token-side problems in one launch (the decoder backward's weight gradients, deferred and
// issued together: one launch instead of one ~18 us latency-bound launch per weight): workgroup b takes tile
// b - start[k] of problem k, start[k] <= b < start[k + 1]. Problems of one group never share an output (the host
// flushes a group before a problem that overlaps a pending one's out / db).
constexpr int TOK_GROUP_MAX = 24;
struct TokProb {
  const bf16* dy;
  const bf16* x;
  float* out;
  float* db;
  long long ldy, ldx, M;
  int tiles_i, ldo;
  float beta;
  int w64;  // 64 x 64 output tiles (tok_w64), else 32 x 32
};
struct TokGroup {
  TokProb p[TOK_GROUP_MAX];
  int start[TOK_GROUP_MAX + 1];
  int n;
};
template <int NW>
__global__ __launch_bounds__(NW * 64) void wgrad_tok_group_kernel(const TokGroup g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < g.n && g.start[k + 1] <= b) ++k;
  const TokProb& q = g.p[k];
  if (q.w64)
    tok_tile64<NW>(q.dy, q.ldy, q.x, q.ldx, q.M, b - g.start[k], q.tiles_i, q.out, q.ldo, q.beta, q.db, smem);
  else
    tok_tile<NW>(q.dy, q.ldy, q.x, q.ldx, q.M, b - g.start[k], q.tiles_i, q.out, q.ldo, q.beta, q.db, smem);
}

int n_workgroups(long long M, long long& rows_per) {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu <= 0) n_cu = 256;
  }
  rows_per = SROWS * ((M + (long long)SROWS * n_cu - 1) / ((long long)SROWS * n_cu));
  return (int)((M + rows_per - 1) / rows_per);
}

template <int NBO, int NBI>
int launch(const bf16* dy, long long ldy, const bf16* x, long long ldx, long long M, long long rows_per, int nwg,
           float* part, float* cs_a, float* cs_b, hipStream_t s) {
  constexpr int STAGE = SROWS * (64 * NBO + 128 * NBI) * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_kernel<NBO, NBI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              NS * STAGE);
    attr = true;
  }
  hipLaunchKernelGGL((wgrad_kernel<NBO, NBI>), dim3(nwg), dim3(512), NS * STAGE, s, dy, ldy, x, ldx, M, rows_per,
                     part, cs_a, cs_b);
  OCTSAM_LAUNCH_CHECK("octsam_wgrad");
  return 0;
}
}  // namespace

extern "C" int octsam_wgrad_tok(const void* dy, int64_t ldy, const void* x, int64_t ldx, int64_t M, int32_t O,
                                int32_t I, float* out, float beta, float* db, void* stream) {
  OCTSAM_CHECK_ARG(dy && x && out && M > 0 && M < (1LL << 24) && O > 0 && I > 0 && O % 32 == 0 && I % 32 == 0,
                   "octsam_wgrad_tok: M=%lld O=%d I=%d (O, I multiples of 32)", (long long)M, O, I);
  OCTSAM_CHECK_ARG(ldy >= O && ldx >= I && ldy % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)dy & 15) == 0 &&
                       ((uintptr_t)x & 15) == 0 && (long long)M * ldy * 2 < (1LL << 31) && (long long)M * ldx * 2 < (1LL << 31),
                   "octsam_wgrad_tok: ldy / ldx multiples of 8, operands 16-B aligned");
  const int tiles = (O / 32) * (I / 32);
  hipStream_t s = (hipStream_t)stream;
  if (tok_w64(O, I)) {
    const int t64 = (O / 64) * (I / 64);
    if (M > 1024) {
      constexpr int NW = 8, LDS = tok::lds64<NW>();
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)wgrad_tok64_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        attr = true;
      }
      hipLaunchKernelGGL(wgrad_tok64_kernel<NW>, dim3(t64), dim3(NW * 64), LDS, s, (const bf16*)dy, (long long)ldy,
                         (const bf16*)x, (long long)ldx, (long long)M, I / 64, out, I, beta, db);
    } else {
      constexpr int NW = 4, LDS = tok::lds64<NW>();
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)wgrad_tok64_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        attr = true;
      }
      hipLaunchKernelGGL(wgrad_tok64_kernel<NW>, dim3(t64), dim3(NW * 64), LDS, s, (const bf16*)dy, (long long)ldy,
                         (const bf16*)x, (long long)ldx, (long long)M, I / 64, out, I, beta, db);
    }
    OCTSAM_LAUNCH_CHECK("octsam_wgrad_tok");
    return 0;
  }
  if (M > 1024) {
    constexpr int NW = 8, LDS = NW * tok::nst<8>() * tok::STB;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)wgrad_tok_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      attr = true;
    }
    hipLaunchKernelGGL(wgrad_tok_kernel<NW>, dim3(tiles), dim3(NW * 64), LDS, s, (const bf16*)dy, (long long)ldy,
                       (const bf16*)x, (long long)ldx, (long long)M, I / 32, out, I, beta, db);
  } else {
    constexpr int NW = 4, LDS = NW * tok::nst<4>() * tok::STB;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)wgrad_tok_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      attr = true;
    }
    hipLaunchKernelGGL(wgrad_tok_kernel<NW>, dim3(tiles), dim3(NW * 64), LDS, s, (const bf16*)dy, (long long)ldy,
                       (const bf16*)x, (long long)ldx, (long long)M, I / 32, out, I, beta, db);
  }
  OCTSAM_LAUNCH_CHECK("octsam_wgrad_tok");
  return 0;
}

template <int NW>
void launch_tok_group(TokGroup& g, hipStream_t s) {
  for (int k = g.n + 1; k <= TOK_GROUP_MAX; ++k) g.start[k] = g.start[g.n];
  constexpr int LDS32 = NW * tok::nst<NW>() * tok::STB, LDS64 = tok::lds64<NW>();
  constexpr int LDS = LDS32 > LDS64 ? LDS32 : LDS64;
  static_assert(LDS32 >= NW * (1024 + 32) * 4, "the fixed-order reduction reuses the rings");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_tok_group_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL(wgrad_tok_group_kernel<NW>, dim3(g.start[g.n]), dim3(NW * 64), LDS, s, g);
}

extern "C" int octsam_wgrad_tok_group(int32_t n, const void* const* dy, const int64_t* ldy, const void* const* x,
                                      const int64_t* ldx, const int64_t* M, const int32_t* O, const int32_t* I,
                                      float* const* out, const float* beta, float* const* db, void* stream) {
  OCTSAM_CHECK_ARG(n > 0 && n <= TOK_GROUP_MAX && dy && ldy && x && ldx && M && O && I && out && beta && db,
                   "octsam_wgrad_tok_group: n=%d (1..%d) and every array non-null", n, TOK_GROUP_MAX);
  // two launches at most: the problems octsam_wgrad_tok runs with 8 waves (M > 1024) and with 4, so that every
  // problem keeps its single-launch partition of the rows (same bits)
  TokGroup g8, g4;
  g8.n = g4.n = 0;
  g8.start[0] = g4.start[0] = 0;
  for (int k = 0; k < n; ++k) {
    OCTSAM_CHECK_ARG(dy[k] && x[k] && out[k] && M[k] > 0 && M[k] < (1LL << 24) && O[k] > 0 && I[k] > 0 &&
                         O[k] % 32 == 0 && I[k] % 32 == 0,
                     "octsam_wgrad_tok_group: problem %d: M=%lld O=%d I=%d (O, I multiples of 32)", k,
                     (long long)M[k], O[k], I[k]);
    OCTSAM_CHECK_ARG(ldy[k] >= O[k] && ldx[k] >= I[k] && ldy[k] % 8 == 0 && ldx[k] % 8 == 0 &&
                         ((uintptr_t)dy[k] & 15) == 0 && ((uintptr_t)x[k] & 15) == 0 &&
                         (long long)M[k] * ldy[k] * 2 < (1LL << 31) && (long long)M[k] * ldx[k] * 2 < (1LL << 31),
                     "octsam_wgrad_tok_group: problem %d: ldy / ldx multiples of 8, operands 16-B aligned", k);
    TokGroup& g = M[k] > 1024 ? g8 : g4;
    const int tw = tok_w64(O[k], I[k]) ? 64 : 32;
    g.p[g.n] = TokProb{(const bf16*)dy[k], (const bf16*)x[k], out[k], db[k], (long long)ldy[k], (long long)ldx[k],
                       (long long)M[k], I[k] / tw, I[k], beta[k], tw == 64 ? 1 : 0};
    g.start[g.n + 1] = g.start[g.n] + (O[k] / tw) * (I[k] / tw);
    ++g.n;
  }
  if (g8.n) launch_tok_group<8>(g8, (hipStream_t)stream);
  OCTSAM_LAUNCH_CHECK("octsam_wgrad_tok_group");
  if (g4.n) launch_tok_group<4>(g4, (hipStream_t)stream);
  OCTSAM_LAUNCH_CHECK("octsam_wgrad_tok_group");
  return 0;
}

extern "C" int32_t octsam_wgrad_supported(int64_t M, int32_t O, int32_t I) {
  return M > 0 && (O == 128 || O == 256 || O == 384) && (I == 128 || I == 256) ? 1 : 0;
}

extern "C" int64_t octsam_wgrad_workspace(int64_t M, int32_t O, int32_t I) {
  if (!octsam_wgrad_supported(M, O, I)) return 0;
  long long rows_per;
  const int nwg = n_workgroups(M, rows_per);
  return (int64_t)nwg * ((int64_t)O * I + O + I) * 4;
}

extern "C" int octsam_wgrad(const void* dy, int64_t ldy, const void* x, int64_t ldx, int64_t M, int32_t O, int32_t I,
                            float* out, float beta, float* db, float* dbx, int32_t dbx_fold, void* workspace,
                            int64_t workspace_bytes, void* stream) {
  OCTSAM_CHECK_ARG(octsam_wgrad_supported(M, O, I), "octsam_wgrad: unsupported shape M=%lld O=%d I=%d "
                   "(O in {128, 256, 384}, I in {128, 256})", (long long)M, O, I);
  OCTSAM_CHECK_ARG(dy && x && out && workspace, "octsam_wgrad: null pointer");
  OCTSAM_CHECK_ARG(ldy >= O && ldx >= I && ldy % 8 == 0 && ldx % 8 == 0,
                   "octsam_wgrad: ldy=%lld / ldx=%lld must be >= O / I and multiples of 8", (long long)ldy,
                   (long long)ldx);
  OCTSAM_CHECK_ARG(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)workspace & 15) == 0,
                   "octsam_wgrad: operands and workspace must be 16-B aligned");
  OCTSAM_CHECK_ARG(dbx == nullptr || (dbx_fold >= 1 && I % dbx_fold == 0 && (I / dbx_fold) % 4 == 0),
                   "octsam_wgrad: dbx_fold=%d must divide I=%d into a multiple of 4 columns", dbx_fold, I);
  OCTSAM_CHECK_ARG(workspace_bytes >= octsam_wgrad_workspace(M, O, I), "octsam_wgrad: workspace too small");
  long long rows_per;
  const int nwg = n_workgroups(M, rows_per);
  float* part = (float*)workspace;
  float* cs_a = db ? part + (long long)nwg * O * I : nullptr;
  float* cs_b = dbx ? part + (long long)nwg * (O * I + O) : nullptr;
  hipStream_t s = (hipStream_t)stream;
  const bf16 *A = (const bf16*)dy, *B = (const bf16*)x;
  int rc;
  if (O == 384 && I == 256) rc = launch<6, 2>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  else if (O == 384) rc = launch<6, 1>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  else if (O == 256 && I == 256) rc = launch<4, 2>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  else if (O == 256) rc = launch<4, 1>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  else if (I == 256) rc = launch<2, 2>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  else rc = launch<2, 1>(A, ldy, B, ldx, M, rows_per, nwg, part, cs_a, cs_b, s);
  if (rc) return rc;
  if ((rc = octsam_splitk_reduce(part, out, (int64_t)O * I, nwg, beta, stream))) return rc;
  if (db && (rc = octsam_splitk_reduce(cs_a, db, O, nwg, 0.0f, stream))) return rc;
  if (dbx && (rc = octsam_splitk_reduce(cs_b, dbx, I / dbx_fold, nwg * dbx_fold, 0.0f, stream))) return rc;
  return 0;
}
