// Fused tail of SamMaskDecoder's upscaling + mask head (hf:modeling_sam.py:519-542):
//   up2 = GELU(ConvT2(up1))  (ConvTranspose2d 64 -> 32, k2 s2, as a [rows, 64] x [64, 128] product)
//   masks[p, t] = hyper[p, t] . up2                                    (mask = hyper_in @ upscaled)
// forward and backward in one kernel each, so the 32-channel 256x256 upscaled embedding (and its
// pre-activation and gradient) never touches HBM: the forward reads up1 and writes the masks; the
// backward reads up1 and d masks, recomputes the ConvT2 product, and writes d up1 plus fixed-order
// partials of d W2, d b2 and d hyper.
//
// Layout: up1 bf16 [P * 16384, 64] in the blocked order of the ConvT GEMMs (decoder.py): row =
// (p, y1, x1, dy1, dx1), up2 column n = (dy2, dx2, c) -> pixel y = 4 y1 + 2 dy1 + dy2, x = 4 x1 + 2 dx1 + dx2.
// A tile = 128 consecutive rows = (p, y1, half h of the x1 range), i.e. the mask block rows 4 y1 .. 4 y1 + 3,
// columns 128 h .. 128 h + 127. Wave w owns tile rows 32 w .. 32 w + 31 (two 16-row MFMA blocks).
// The product runs operand-swapped (A = W2 [n][k], B = up1 rows) so each lane holds one row (lane & 15)
// and 4 consecutive n per 16-column block: the channel contraction with hyper is per lane + two xor
// shuffles, and in the backward the same registers (bf16) are directly the B operand of d up1 = dpre W2^T
// (the 8 k-slots of a lane are a permutation of n, matched in the W2^T fragments). d W2 = up1^T dpre
// contracts over rows, so dpre and up1 are staged in LDS and read transposed (ds_read_b64_tr_b16).
// Persistent workgroups (fixed grid, static tile stride) -> deterministic partial sums.
#include "common.h"
#include "../../include/octsam.h"

namespace {
// The value of lane ^ 32 (lane ^ 16): v_permlane32_swap (v_permlane16_swap) of x with itself leaves every lane
// {x of the lower, x of the upper} lane of its pair; pick the partner's by the lane's own half (hi = lane bit 5
// (bit 4)). One swap and one select instead of a ds_bpermute round trip inside the VALU-bound loop.
__device__ __forceinline__ float xor32_value(float x, bool hi) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (uint32_t)(hi ? r[0] : r[1]));
}
// Sum over the 16 lanes of a row (every lane gets it): DPP quad swaps (xor 1, xor 2) then row rotations by 4 and 8
// — no LDS traffic. Fixed order, so the reduction is deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x124>(v);  // row_ror:4
  v += dpp_mov<0x128>(v);  // row_ror:8
  return v;
}
// Reduce-scatter over the 16 lanes of a row: lane c returns sum over the row's lanes of v[c] (4 DPP exchange stages
// pairing c with c ^ 8, c ^ 7, c ^ 3, c ^ 1, each lane keeping the half its bit selects). Fixed order: deterministic.
__device__ __forceinline__ float row16_reduce_scatter(const float (&v)[16], int c) {
  float a[8], b[4], d[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool hi = c & 8;
    a[k] = (hi ? v[8 + k] : v[k]) + dpp_mov<0x128>(hi ? v[k] : v[8 + k]);  // row_ror:8 (c ^ 8)
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool hi = c & 4;
    b[k] = (hi ? a[4 + k] : a[k]) + dpp_mov<0x141>(hi ? a[k] : a[4 + k]);  // row_half_mirror (c ^ 7)
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool hi = c & 2;
    d[k] = (hi ? b[2 + k] : b[k]) + dpp_mov<0x1B>(hi ? b[k] : b[2 + k]);  // quad_perm [3,2,1,0] (c ^ 3)
  }
  const bool hi = c & 1;
  return (hi ? d[1] : d[0]) + dpp_mov<0xB1>(hi ? d[0] : d[1]);  // quad_perm [1,0,3,2] (c ^ 1)
}
__device__ __forceinline__ float xor16_value(float x, bool hi) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (uint32_t)(hi ? r[0] : r[1]));
}

namespace um {
constexpr int ROWS = 128;               // up1 rows per tile
constexpr int TILES_PER_P = 16384 / ROWS;
constexpr int NWG = 512;                // persistent grid (2 workgroups per CU)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// A operand of the swapped product: lane (g, c), element j = W[n = 16 nb + c][k = 32 ks + 8 g + j] = w2[k][n]
__device__ __forceinline__ void load_wfrag(const bf16* __restrict__ w2, bf16x8 (&wf)[8][2], int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int nb = 0; nb < 8; ++nb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) wf[nb][ks][j] = w2[(32 * ks + 8 * g + j) * 128 + 16 * nb + c];
}
// B operand: lane (g, c) = up1 row (row0 + 16 rb + c), k = 32 ks + 8 g .. + 7 (one 16-B load)
__device__ __forceinline__ void load_ufrag(const bf16* __restrict__ up1, long long row0, bf16x8 (&uf)[2][2],
                                           int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) uf[rb][ks] = *(const bf16x8*)(up1 + (row0 + 16 * rb + c) * 64 + 32 * ks + 8 * g);
}
// pre^T block: acc[nb][i] = b2[n] + sum_k up1[row][k] W2[k][n], row = lane & 15 of block rb, n = 16 nb + 4 g + i
__device__ __forceinline__ void convt2(const bf16x8 (&wf)[8][2], const bf16x8 (&ub)[2], const f32x4 (&binit)[8],
                                       f32x4 (&acc)[8]) {
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) {
    acc[nb] = mfma32(wf[nb][0], ub[0], binit[nb]);
    acc[nb] = mfma32(wf[nb][1], ub[1], acc[nb]);
  }
}
// (row within tile rr, sub-pixel s = 2 dy2 + dx2) -> offset in the tile's [4][128] mask block
__device__ __forceinline__ int pix_local(int rr, int s) {
  const int x1l = rr >> 2, dy1 = (rr >> 1) & 1, dx1 = rr & 1;
  return (2 * dy1 + (s >> 1)) * 128 + 4 * x1l + 2 * dx1 + (s & 1);
}
// GELU (erf form) and its derivative on two values at once (packed f32: v_pk_fma / v_pk_mul / v_pk_add, the
// kernels are VALU-bound), one shared erf / exp evaluation (A&S 7.1.26, |err| <= 1.5e-7)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
template <bool GRAD>
__device__ __forceinline__ void gelu2(f32x2 x, f32x2& y, f32x2& dy) {
  const f32x2 u = x * 0.70710678118654752f;
  const f32x2 au = __builtin_elementwise_abs(u);
  const f32x2 den = fma2(au, (f32x2)0.3275911f, (f32x2)1.0f);
  f32x2 t;
  t.x = __builtin_amdgcn_rcpf(den.x);
  t.y = __builtin_amdgcn_rcpf(den.y);
  f32x2 p = fma2((f32x2)1.061405429f, t, (f32x2)-1.453152027f);
  p = fma2(p, t, (f32x2)1.421413741f);
  p = fma2(p, t, (f32x2)-0.284496736f);
  p = fma2(p, t, (f32x2)0.254829592f);
  const f32x2 q = (au * au) * -1.4426950408889634f;
  f32x2 e;  // exp(-x^2 / 2)
  e.x = __builtin_amdgcn_exp2f(q.x);
  e.y = __builtin_amdgcn_exp2f(q.y);
  const f32x2 r = fma2(-(p * t), e, (f32x2)1.0f);
  const f32x2 phi2 = __builtin_elementwise_copysign(r, u) + 1.0f;
  y = (x * 0.5f) * phi2;
  if constexpr (GRAD) dy = fma2(x * 0.3989422804014327f, e, phi2 * 0.5f);
}
}  // namespace um

// grid: min(NWG, tiles) persistent workgroups of 256 threads; masks fp32 [P, NS, 256, 256]
template <int NS>
__global__ __launch_bounds__(256, 3) void upmask_fwd_kernel(const bf16* __restrict__ up1, const bf16* __restrict__ w2,
                                                            const float* __restrict__ b2,
                                                            const float* __restrict__ hyper, int ntiles,
                                                            float* __restrict__ masks) {
  using namespace um;
  __shared__ __attribute__((aligned(16))) float smask[2][NS * 512];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  bf16x8 wf[8][2];
  load_wfrag(w2, wf, lane);
  f32x4 binit[8];
#pragma unroll
  for (int nb = 0; nb < 8; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) binit[nb][i] = b2[(16 * nb + 4 * g + i) & 31];
  // Every global access in the loop is unconditional (the last prefetch re-reads a valid tile) and the
  // prefetch alternates between two register sets (the loop is unrolled by two), so the compiler's vmcnt
  // bookkeeping is exact and no copy of the prefetched registers waits inside the tile that issued it.
  bf16x8 fa[2][2], fb[2][2];
  int T = blockIdx.x;
  if (T >= ntiles) return;
  load_ufrag(up1, (long long)T * ROWS + 32 * w, fa, lane);
  auto step = [&](const bf16x8 (&uf)[2][2], bf16x8 (&nx)[2][2], int T, int it) {
    const int p = T / TILES_PER_P, y1 = (T >> 1) & 63, h = T & 1;
    f32x4 hy[NS][2];
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) hy[t][hh] = *(const f32x4*)(hyper + (p * NS + t) * 32 + 16 * hh + 4 * g);
    load_ufrag(up1, (long long)min(T + (int)gridDim.x, ntiles - 1) * ROWS + 32 * w, nx, lane);
    float* sm = smask[it & 1];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      f32x4 acc[8];
      convt2(wf, uf[rb], binit, acc);
      float m[NS][4];
#pragma unroll
      for (int t = 0; t < NS; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) m[t][s] = 0.0f;
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          f32x2 u, du;
          gelu2<false>(f32x2{acc[nb][i], acc[nb][i + 1]}, u, du);
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const f32x2 pr = f32x2{hy[t][nb & 1][i], hy[t][nb & 1][i + 1]} * u;
            m[t][nb >> 1] += pr.x + pr.y;
          }
        }
      // reduce-scatter over the 4 lane groups: group g ends with the full sum of sub-pixel s = g
      const int rr = 32 * w + 16 * rb + c;
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const bool hi2 = g & 2, hi1 = g & 1;
        float a0 = hi2 ? m[t][2] : m[t][0], a1 = hi2 ? m[t][3] : m[t][1];
        const float s0 = hi2 ? m[t][0] : m[t][2], s1 = hi2 ? m[t][1] : m[t][3];
        a0 += xor32_value(s0, hi2);
        a1 += xor32_value(s1, hi2);
        float k = hi1 ? a1 : a0;
        k += xor16_value(hi1 ? a0 : a1, hi1);
        sm[t * 512 + pix_local(rr, g)] = k;
      }
    }
    __syncthreads();  // (double-buffered staging: the buffer written next was last read before this barrier)
#pragma unroll
    for (int t = 0; t < NS; ++t) {  // 2 floats per thread and mask: the [4][128] block, 512-B row runs
      const int yl = tid >> 6, x2 = (tid & 63) * 2;
      *(float2*)(masks + ((long long)(p * NS + t) * 65536 + (4 * y1 + yl) * 256 + 128 * h + x2)) =
          *(const float2*)(sm + t * 512 + yl * 128 + x2);
    }
  };
  for (int it = 0;; it += 2) {
    step(fa, fb, T, it);
    if ((T += gridDim.x) >= ntiles) break;
    step(fb, fa, T, it + 1);
    if ((T += gridDim.x) >= ntiles) break;
  }
}

// Backward tiles are 64 rows = (p, y1, quarter q of the x1 range): mask block rows 4 y1 .. 4 y1 + 3, columns
// 64 q .. 64 q + 63; wave w owns tile rows 16 w .. 16 w + 15 (one MFMA block) -- half the forward's tile,
// for registers: the ConvT2 fragments (64 VGPRs) stay resident next to the d W2 accumulators.
namespace um {
constexpr int BROWS = 64;
constexpr int BTILES_PER_P = 16384 / BROWS;
constexpr int S_UP = 0;                       // up1 tile [64][64] bf16, 16-B chunk ^ (row & 7)
constexpr int S_DP = S_UP + BROWS * 128;      // dpre tile [64][128] bf16, 16-B chunk ^ (row & 15)
constexpr int S_W2T = S_DP + BROWS * 256;     // d up1 A-operand fragments [16][64 lanes] x 16 B
constexpr int S_BIAS = S_W2T + 16 * 64 * 16;  // b2 per n [128] fp32
constexpr int S_W2 = S_BIAS + 128 * 4;        // ConvT2 A-operand fragments [16][64 lanes] x 16 B
constexpr int S_DM = S_W2 + 16 * 64 * 16;     // d masks of the tile [NS][4][64] fp32
__device__ __forceinline__ int up_off(int r, int ch) { return S_UP + r * 128 + 16 * (ch ^ (r & 7)); }
__device__ __forceinline__ int dp_off(int r, int ch) { return S_DP + r * 256 + 16 * (ch ^ (r & 15)); }
__device__ __forceinline__ int bpix_local(int rr, int s) {
  const int x1l = rr >> 2, dy1 = (rr >> 1) & 1, dx1 = rr & 1;
  return (2 * dy1 + (s >> 1)) * 64 + 4 * x1l + 2 * dx1 + (s & 1);
}
// transposed 16x16x32 operand from a row-major LDS tile: lane (g, c), element j = X[row0 + 8 g + j][16 cb + c]
template <bool DP>
__device__ __forceinline__ bf16x8 tr_op(const char* smem, int row0, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int ch = 2 * cb + (pp >> 1);
  const int r0 = row0 + 8 * g + q, r1 = r0 + 4;
  const int o0 = (DP ? dp_off(r0, ch) : up_off(r0, ch)) + 8 * (pp & 1);
  const int o1 = (DP ? dp_off(r1, ch) : up_off(r1, ch)) + 8 * (pp & 1);
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + o0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + o1));
  return cat8(a, b);
}
// B operand of one 16-row block: lane (g, c) = up1 row (row0 + c), k = 32 ks + 8 g .. + 7
__device__ __forceinline__ void load_ublk(const bf16* __restrict__ up1, long long row0, bf16x8 (&ub)[2], int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ub[ks] = *(const bf16x8*)(up1 + (row0 + c) * 64 + 32 * ks + 8 * g);
}
}  // namespace um

// LN = true: the LayerNorm2d + GELU in front of up1 (up1 = GELU(LN(x)), hf:modeling_sam.py:519-520) is
// differentiated in the same pass, so d up1 never reaches HBM: with x the ConvT1 output row (bf16 [rows][64]),
// mean / rstd its saved statistics, xh = (x - mean) rstd and y = xh w + b,
//   gy = d up1 * GELU'(y),  g = gy w,  dx = rstd (g - mean_c(g) - xh mean_c(g xh)),
//   d w_c += gy xh, d b_c += gy  (fixed-order per-workgroup partials, part_ln [grid][2][64])
// — ln_bwd_kernel's arithmetic on the fp32 d up1 instead of its bf16 copy. A row's 64 channels are the 16 of each
// of the lanes c, c + 16, c + 32, c + 48, so the two row sums take one permlane16 and one permlane32 swap; the
// per-channel d w / d b sums over a tile's rows are one DPP reduce-scatter each (two accumulators per lane).
struct LnArgs {
  const bf16* x;
  const float* mean;
  const float* rstd;
  const float* w;
  const float* b;
  float* part;
  long long ldd;  // d up1 / d x: elements between the [P * 4096, 256] rows (4 [.., 64] rows each); 256 = contiguous
};
// part_h fp32 [256][P * NS * 32] (per tile-in-prompt), part_w [grid][64][128], part_b [grid][32]
template <int NS, bool LN>
__global__ __launch_bounds__(256, 2) void upmask_bwd_kernel(const bf16* __restrict__ up1, const bf16* __restrict__ w2,
                                                            const float* __restrict__ b2,
                                                            const float* __restrict__ hyper,
                                                            const float* __restrict__ dmask, int ntiles, int P,
                                                            bf16* __restrict__ dup1, float* __restrict__ part_h,
                                                            float* __restrict__ part_w, float* __restrict__ part_b,
                                                            LnArgs ln) {
  using namespace um;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_red = (float*)(smem + S_DM + NS * 1024);  // [4 waves][NS * 32]
  float* s_ln = s_red + 4 * NS * 32;                 // LN: w [64], b [64], then [4 waves][2][64] partials
  float* scratch = part_b + gridDim.x * 32 + blockIdx.x * 256;  // sink of the idle threads' partial stores
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  // W2^T fragments for d up1 = dpre W2^T: fragment (m, kb), lane (g, c), element j = w2[k = 16 kb + c][n],
  // n = 32 m + 16 (j >> 2) + 4 g + (j & 3) -- the lane's dpre registers of blocks 2m, 2m+1 in k-slot order
  for (int e = tid; e < 16 * 64; e += 256) {
    const int f = e >> 6, l = e & 63, m = f >> 2, kb = f & 3, lg = l >> 4, lc = l & 15;
    const bf16* src = w2 + (16 * kb + lc) * 128 + 32 * m + 4 * lg;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = src[j], v[4 + j] = src[16 + j];
    *(bf16x8*)(smem + S_W2T + 16 * e) = v;
  }
  // ConvT2 A fragments (nb, ks) in fragment order (read per tile: registers go to the d W2 accumulators)
  for (int e = tid; e < 16 * 64; e += 256) {
    const int f = e >> 6, l = e & 63, nb = f >> 1, ks = f & 1, lg = l >> 4, lc = l & 15;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = w2[(32 * ks + 8 * lg + j) * 128 + 16 * nb + lc];
    *(bf16x8*)(smem + S_W2 + 16 * e) = v;
  }
  if (tid < 128) ((float*)(smem + S_BIAS))[tid] = b2[tid & 31];
  if constexpr (LN) {
    if (tid < 128) s_ln[tid] = tid < 64 ? ln.w[tid] : ln.b[tid - 64];
  }
  // d w / d b of LayerNorm channel 16 (c >> 2) + 4 g + (c & 3), summed over the rows of this lane's row group (lanes
  // 16 g .. 16 g + 15 of the wave) and every tile (one reduce-scatter per tile)
  float lnw_acc = 0.0f, lnb_acc = 0.0f;
  f32x4 dwacc[4][2];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) dwacc[kb][0] = dwacc[kb][1] = (f32x4)0.0f;
  float bacc[2][4];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int i = 0; i < 4; ++i) bacc[hh][i] = 0.0f;

  // Unconditional global accesses and alternating prefetch buffers, as in the forward.
  bf16x8 ua[2], ubb[2];
  float da_[NS], db_[NS];
  auto prefetch = [&](int Tn, bf16x8 (&nu)[2], float (&nd)[NS]) {  // up1 block + the tile's d masks
    load_ublk(up1, (long long)Tn * BROWS + 16 * w, nu, lane);      // ([NS][4][64]: one float per thread and mask)
    const int p = Tn / BTILES_PER_P, y1 = (Tn >> 2) & 63, q = Tn & 3, yl = tid >> 6, x = tid & 63;
#pragma unroll
    for (int t = 0; t < NS; ++t) nd[t] = dmask[(long long)(p * NS + t) * 65536 + (4 * y1 + yl) * 256 + 64 * q + x];
  };
  int T = blockIdx.x;
  if (T >= ntiles) return;
  prefetch(T, ua, da_);
  auto step = [&](const bf16x8 (&ub)[2], const float (&dcur)[NS], bf16x8 (&nu)[2], float (&nd)[NS], int T) {
    // LN: the lane's x (ConvT1 output) row segments and row statistics, loaded at the tile's start (consumed after
    // its ConvT2 recompute and d up1 products; a prefetch one tile ahead would not fit the registers)
    uint2 xc[LN ? 4 : 1];
    float2 sc;
    if constexpr (LN) {
      const long long orow = (long long)T * BROWS + 16 * w + c;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) xc[kb] = *(const uint2*)(ln.x + orow * 64 + 16 * kb + 4 * g);
      sc = make_float2(ln.mean[orow], ln.rstd[orow]);
    }
    const int p = T / BTILES_PER_P;
    const int rr = 16 * w + c;
    f32x4 hy[NS][2];
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) hy[t][hh] = *(const f32x4*)(hyper + (p * NS + t) * 32 + 16 * hh + 4 * g);
    prefetch(min(T + (int)gridDim.x, ntiles - 1), nu, nd);
    __syncthreads();  // (A) the previous tile's LDS readers are done
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) *(bf16x8*)(smem + up_off(rr, 4 * ks + g)) = ub[ks];
#pragma unroll
    for (int t = 0; t < NS; ++t) ((float*)(smem + S_DM + t * 1024))[tid] = dcur[t];
    f32x4 acc[8];
    {
      f32x4 binit[8];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) binit[nb] = *(const f32x4*)(smem + S_BIAS + 4 * (16 * nb + 4 * g));
      bf16x8 wf[8][2];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) wf[nb][ks] = *(const bf16x8*)(smem + S_W2 + 16 * ((2 * nb + ks) * 64 + lane));
      convt2(wf, ub, binit, acc);
    }
    __syncthreads();  // (B) d masks staged
    float dm[NS][4];
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int dy2 = 0; dy2 < 2; ++dy2) {
        const float2 v = *(const float2*)(smem + S_DM + t * 1024 + 4 * bpix_local(rr, 2 * dy2));
        dm[t][2 * dy2] = v.x;
        dm[t][2 * dy2 + 1] = v.y;
      }
    float hacc[NS][2][4];
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int i = 0; i < 4; ++i) hacc[t][hh][i] = 0.0f;
    // elementwise per pair of 16-column blocks (2m, 2m+1) = one k-step of d up1 = dpre W2^T, accumulated at once
    // (D[k][row], lane (g, c): row c, k = 16 kb + 4 g + i) so only one pair of dpre blocks is live
    f32x4 da[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) da[kb] = (f32x4)0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      s16x4 dpk[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int nb = 2 * m + hh;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          f32x2 u, du;
          gelu2<true>(f32x2{acc[nb][i], acc[nb][i + 1]}, u, du);
          f32x2 d = (f32x2)0.0f;
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const f32x2 dmv = (f32x2)dm[t][m];
            d = fma2(dmv, f32x2{hy[t][hh][i], hy[t][hh][i + 1]}, d);
            const f32x2 h2 = fma2(dmv, u, f32x2{hacc[t][hh][i], hacc[t][hh][i + 1]});
            hacc[t][hh][i] = h2.x;
            hacc[t][hh][i + 1] = h2.y;
          }
          const f32x2 dp = d * du;
          bacc[hh][i] += dp.x;
          bacc[hh][i + 1] += dp.y;
          dpk[hh][i] = __builtin_bit_cast(short, (bf16)dp.x);
          dpk[hh][i + 1] = __builtin_bit_cast(short, (bf16)dp.y);
        }
        *(s16x4*)(smem + dp_off(rr, 2 * nb + (g >> 1)) + 8 * (g & 1)) = dpk[hh];
      }
      const bf16x8 bop = cat8(dpk[0], dpk[1]);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        da[kb] = mfma32(*(const bf16x8*)(smem + S_W2T + 16 * ((4 * m + kb) * 64 + lane)), bop, da[kb]);
    }
    // d hyper of this tile: sum over the 16 rows of each lane group (the 4 waves are summed after (C))
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = hacc[t][hh][i];
          v = row16_sum(v);
          if (c == 0) s_red[w * NS * 32 + t * 32 + 16 * hh + 4 * g + i] = v;
        }
    // d x (LN) / d up1 rows, after the d hyper sums so their registers are free
    if constexpr (LN) {  // d up1 -> d x through GELU and LayerNorm2d (see LnArgs)
      const long long orow = (long long)T * BROWS + rr;
      const float mu = sc.x, rs = sc.y;
      auto xnorm = [&](int kb, int i) {
        const uint32_t pr = (i & 2) ? xc[kb].y : xc[kb].x;
        return (__builtin_bit_cast(float, (i & 1) ? (pr & 0xffff0000u) : (pr << 16)) - mu) * rs;
      };
      float gy[16], tmp[16];
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const f32x4 lw = *(const f32x4*)(s_ln + 16 * kb + 4 * g), lb = *(const f32x4*)(s_ln + 64 + 16 * kb + 4 * g);
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const f32x2 xn = {xnorm(kb, i), xnorm(kb, i + 1)};
          f32x2 u, du;
          gelu2<true>(fma2(xn, f32x2{lw[i], lw[i + 1]}, f32x2{lb[i], lb[i + 1]}), u, du);
          const f32x2 gv = f32x2{da[kb][i], da[kb][i + 1]} * du;
          gy[4 * kb + i] = gv.x;
          gy[4 * kb + i + 1] = gv.y;
          const f32x2 gw = gv * f32x2{lw[i], lw[i + 1]};
          s1 += gw.x + gw.y;
          s2 += gw.x * xn.x + gw.y * xn.y;
          tmp[4 * kb + i] = gv.x * xn.x;
          tmp[4 * kb + i + 1] = gv.y * xn.y;
        }
      }
      lnw_acc += row16_reduce_scatter(tmp, c);
      lnb_acc += row16_reduce_scatter(gy, c);
      // row sums over the 4 lanes holding the row's 64 channels (same value in all four: + is commutative)
      s1 += xor16_value(s1, g & 1);
      s2 += xor16_value(s2, g & 1);
      s1 += xor32_value(s1, g >> 1);
      s2 += xor32_value(s2, g >> 1);
      s1 *= 1.0f / 64.0f;
      s2 *= 1.0f / 64.0f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const f32x4 lw = *(const f32x4*)(s_ln + 16 * kb + 4 * g);
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)(rs * (gy[4 * kb + i] * lw[i] - s1 - xnorm(kb, i) * s2));
        *(bf16x4*)(dup1 + (orow >> 2) * ln.ldd + (orow & 3) * 64 + 16 * kb + 4 * g) = o;
      }
    } else {
      const long long orow = (long long)T * BROWS + rr;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)da[kb][i];
        *(bf16x4*)(dup1 + (orow >> 2) * ln.ldd + (orow & 3) * 64 + 16 * kb + 4 * g) = o;
      }
    }
    __syncthreads();  // (C) dpre tile and d hyper rows complete
    {
      const int j = tid < NS * 32 ? tid : 0;
      const float v = s_red[j] + s_red[NS * 32 + j] + s_red[2 * NS * 32 + j] + s_red[3 * NS * 32 + j];
      float* dst = tid < NS * 32 ? part_h + (long long)(T % BTILES_PER_P) * P * NS * 32 + p * NS * 32 + tid
                                 : scratch + tid;
      *dst = v;
    }
    // d W2 partial over the tile's 64 rows: wave w owns n blocks 2w, 2w+1; D[k][n], lane: k = 16 kb + 4 g + i, n = 16 nb + c
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bo[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bo[j] = tr_op<true>(smem, 32 * ks, 2 * w + j, lane);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const bf16x8 ao = tr_op<false>(smem, 32 * ks, kb, lane);
        dwacc[kb][0] = mfma32(ao, bo[0], dwacc[kb][0]);
        dwacc[kb][1] = mfma32(ao, bo[1], dwacc[kb][1]);
      }
    }
  };
  for (;;) {
    step(ua, da_, ubb, db_, T);
    if ((T += gridDim.x) >= ntiles) break;
    step(ubb, db_, ua, da_, T);
    if ((T += gridDim.x) >= ntiles) break;
  }

  // per-workgroup partials of d W2 and d b2
  float* pw = part_w + (long long)blockIdx.x * 8192;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) pw[(16 * kb + 4 * g + i) * 128 + 16 * (2 * w + j) + c] = dwacc[kb][j][i];
  __syncthreads();
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = bacc[hh][i];
      v = row16_sum(v);
      if (c == 0) s_red[w * 32 + 16 * hh + 4 * g + i] = v;
    }
  __syncthreads();
  if (tid < 32) part_b[blockIdx.x * 32 + tid] = s_red[tid] + s_red[32 + tid] + s_red[64 + tid] + s_red[96 + tid];
  if constexpr (LN) {  // d w / d b of the LayerNorm: rows of the wave (lanes c) by DPP, the 4 waves through LDS
    float* s_lp = s_ln + 128;  // [4][128]
    const int ch = 16 * (c >> 2) + 4 * g + (c & 3);
    s_lp[w * 128 + ch] = lnw_acc;
    s_lp[w * 128 + 64 + ch] = lnb_acc;
    __syncthreads();
    if (tid < 128)
      ln.part[(tid >> 6) * gridDim.x * 64 + blockIdx.x * 64 + (tid & 63)] =
          s_lp[tid] + s_lp[128 + tid] + s_lp[256 + tid] + s_lp[384 + tid];
  }
}

int g_fwd_grid = 768, g_bwd_grid = um::NWG;  // persistent grids (octsam_upmask_set_grid: tuning)
int upmask_grid(int ntiles, int cap) { return ntiles < cap ? ntiles : cap; }
}  // namespace

extern "C" void octsam_upmask_set_grid(int32_t fwd, int32_t bwd) {
  if (fwd > 0) g_fwd_grid = fwd;
  if (bwd > 0) g_bwd_grid = bwd < um::NWG ? bwd : um::NWG;  // (the workspace is sized for NWG partials)
}

extern "C" int octsam_splitk_reduce(const float* partials, float* out, int64_t n, int32_t splits, float beta,
                                    void* stream);

extern "C" int octsam_upmask_fwd(const void* up1, const void* w2, const float* b2, const float* hyper, int32_t P,
                                 int32_t ntok, float* masks, void* stream) {
  OCTSAM_CHECK_ARG(up1 && w2 && b2 && hyper && masks && P > 0 && (ntok == 1 || ntok == 3),
                   "octsam_upmask_fwd: bad args (ntok must be 1 or 3)");
  OCTSAM_CHECK_ARG(((uintptr_t)up1 & 15) == 0 && ((uintptr_t)hyper & 15) == 0 && ((uintptr_t)masks & 15) == 0,
                   "octsam_upmask_fwd: up1, hyper and masks must be 16-B aligned");
  const int ntiles = P * um::TILES_PER_P, grid = upmask_grid(ntiles, g_fwd_grid);
  hipStream_t s = (hipStream_t)stream;
  if (ntok == 1)
    hipLaunchKernelGGL(upmask_fwd_kernel<1>, dim3(grid), dim3(256), 0, s, (const bf16*)up1, (const bf16*)w2, b2, hyper,
                       ntiles, masks);
  else
    hipLaunchKernelGGL(upmask_fwd_kernel<3>, dim3(grid), dim3(256), 0, s, (const bf16*)up1, (const bf16*)w2, b2, hyper,
                       ntiles, masks);
  OCTSAM_LAUNCH_CHECK("octsam_upmask_fwd");
  return 0;
}

extern "C" int64_t octsam_upmask_bwd_workspace(int32_t P, int32_t ntok) {
  if (P <= 0 || ntok <= 0) return 0;
  const long long grid = upmask_grid(P * um::BTILES_PER_P, um::NWG);
  // part_h, part_w, part_b, the idle threads' sink (grid * 256), the LayerNorm partials (grid * 128)
  return (long long)um::BTILES_PER_P * P * ntok * 32 + grid * 8192 + grid * 32 + grid * 256 + grid * 128;
}

namespace {
int upmask_bwd_impl(const void* up1, const void* w2, const float* b2, const float* hyper, const float* dmask, int32_t P,
                    int32_t ntok, void* dout, float* dw2, float* db2, float* dhyper, float* workspace, const LnArgs* ln,
                    float* dlnw, float* dlnb, void* stream, long long ldd = 256) {
  const int ntiles = P * um::BTILES_PER_P, grid = upmask_grid(ntiles, g_bwd_grid);
  float* part_h = workspace;
  float* part_w = part_h + (long long)um::BTILES_PER_P * P * ntok * 32;
  float* part_b = part_w + (long long)grid * 8192;
  LnArgs la = ln ? *ln : LnArgs{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 256};
  la.ldd = ldd;
  la.part = part_b + (long long)grid * 32 + (long long)grid * 256;  // [2][grid][64]
  hipStream_t s = (hipStream_t)stream;
  const int lds = um::S_DM + ntok * 1024 + 4 * ntok * 32 * 4 + (ln ? (128 + 512) * 4 : 0);
#define UM_BWD(NS, L)                                                                                            \
  hipLaunchKernelGGL((upmask_bwd_kernel<NS, L>), dim3(grid), dim3(256), lds, s, (const bf16*)up1, (const bf16*)w2, b2, \
                     hyper, dmask, ntiles, P, (bf16*)dout, part_h, part_w, part_b, la)
  if (ntok == 1) {
    if (ln) UM_BWD(1, true); else UM_BWD(1, false);
  } else {
    if (ln) UM_BWD(3, true); else UM_BWD(3, false);
  }
#undef UM_BWD
  OCTSAM_LAUNCH_CHECK("octsam_upmask_bwd");
  int rc = octsam_splitk_reduce(part_h, dhyper, (int64_t)P * ntok * 32, um::BTILES_PER_P, 0.0f, stream);
  if (!rc) rc = octsam_splitk_reduce(part_w, dw2, 8192, grid, 0.0f, stream);
  if (!rc) rc = octsam_splitk_reduce(part_b, db2, 32, grid, 0.0f, stream);
  if (!rc && ln) rc = octsam_splitk_reduce(la.part, dlnw, 64, grid, 0.0f, stream);
  if (!rc && ln) rc = octsam_splitk_reduce(la.part + (long long)grid * 64, dlnb, 64, grid, 0.0f, stream);
  return rc;
}
}  // namespace

extern "C" int octsam_upmask_bwd(const void* up1, const void* w2, const float* b2, const float* hyper,
                                 const float* dmask, int32_t P, int32_t ntok, void* dup1, float* dw2, float* db2,
                                 float* dhyper, float* workspace, void* stream) {
  OCTSAM_CHECK_ARG(up1 && w2 && b2 && hyper && dmask && dup1 && dw2 && db2 && dhyper && workspace && P > 0 &&
                       (ntok == 1 || ntok == 3),
                   "octsam_upmask_bwd: bad args (ntok must be 1 or 3)");
  OCTSAM_CHECK_ARG(((uintptr_t)up1 & 15) == 0 && ((uintptr_t)hyper & 15) == 0 && ((uintptr_t)dmask & 15) == 0 &&
                       ((uintptr_t)dup1 & 7) == 0 && ((uintptr_t)workspace & 15) == 0,
                   "octsam_upmask_bwd: misaligned operand");
  return upmask_bwd_impl(up1, w2, b2, hyper, dmask, P, ntok, dup1, dw2, db2, dhyper, workspace, nullptr, nullptr,
                         nullptr, stream);
}

extern "C" int octsam_upmask_ln_bwd(const void* up1, const void* w2, const float* b2, const float* hyper,
                                    const float* dmask, int32_t P, int32_t ntok, const void* x, const float* mean,
                                    const float* rstd, const float* ln_w, const float* ln_b, void* dx, float* dw2,
                                    float* db2, float* dhyper, float* dln_w, float* dln_b, float* workspace,
                                    void* stream) {
  OCTSAM_CHECK_ARG(up1 && w2 && b2 && hyper && dmask && x && mean && rstd && ln_w && ln_b && dx && dw2 && db2 &&
                       dhyper && dln_w && dln_b && workspace && P > 0 && (ntok == 1 || ntok == 3),
                   "octsam_upmask_ln_bwd: bad args (ntok must be 1 or 3)");
  OCTSAM_CHECK_ARG(((uintptr_t)up1 & 15) == 0 && ((uintptr_t)hyper & 15) == 0 && ((uintptr_t)dmask & 15) == 0 &&
                       ((uintptr_t)dx & 7) == 0 && ((uintptr_t)x & 7) == 0 && ((uintptr_t)workspace & 15) == 0,
                   "octsam_upmask_ln_bwd: misaligned operand");
  const LnArgs ln{(const bf16*)x, mean, rstd, ln_w, ln_b, nullptr, 256};
  return upmask_bwd_impl(up1, w2, b2, hyper, dmask, P, ntok, dx, dw2, db2, dhyper, workspace, &ln, dln_w, dln_b,
                         stream);
}

// octsam_upmask_ln_bwd writing d x with a row stride: row r of the [P * 4096, 256] view at dx + r * ldx (ldx >= 256,
// a multiple of 4), so d x can be the left half of a wider operand (decoder.py: [d x | d keys of the final attention]
// feed ONE keys-gradient product)
extern "C" int octsam_upmask_ln_bwd_strided(const void* up1, const void* w2, const float* b2, const float* hyper,
                                            const float* dmask, int32_t P, int32_t ntok, const void* x,
                                            const float* mean, const float* rstd, const float* ln_w,
                                            const float* ln_b, void* dx, int64_t ldx, float* dw2, float* db2,
                                            float* dhyper, float* dln_w, float* dln_b, float* workspace,
                                            void* stream) {
  OCTSAM_CHECK_ARG(up1 && w2 && b2 && hyper && dmask && x && mean && rstd && ln_w && ln_b && dx && dw2 && db2 &&
                       dhyper && dln_w && dln_b && workspace && P > 0 && (ntok == 1 || ntok == 3) && ldx >= 256 &&
                       ldx % 4 == 0,
                   "octsam_upmask_ln_bwd_strided: bad args (ntok 1 or 3, ldx >= 256 and a multiple of 4)");
  OCTSAM_CHECK_ARG(((uintptr_t)up1 & 15) == 0 && ((uintptr_t)hyper & 15) == 0 && ((uintptr_t)dmask & 15) == 0 &&
                       ((uintptr_t)dx & 7) == 0 && ((uintptr_t)x & 7) == 0 && ((uintptr_t)workspace & 15) == 0,
                   "octsam_upmask_ln_bwd_strided: misaligned operand");
  const LnArgs ln{(const bf16*)x, mean, rstd, ln_w, ln_b, nullptr, 256};
  return upmask_bwd_impl(up1, w2, b2, hyper, dmask, P, ntok, dx, dw2, db2, dhyper, workspace, &ln, dln_w, dln_b,
                         stream, ldx);
}
