// SAM ViT attention with decomposed relative-position bias, fused (flash-style), forward only.
//
// Replaces SamVisionAttention / SamVisionSdpaAttention.forward (hf:modeling_sam.py:803-882) together
// with get_rel_pos / get_decomposed_rel_pos (:729-801). The [B*h, T, T] bias tensor that HF
// materialises (805 MB per image for a global vit-b layer) is never formed:
//
//   s[q,k] = scale * q.k + rel_h[q, kh] + rel_w[q, kw],   rel_h[q,kh] = q.Rh[qh-kh+S-1], rel_w likewise
//
// (rel-pos resize is an identity for SAM: 2*max(q,k)-1 == table length; scale = head_dim^-0.5).
//
// One kernel template for both layer kinds, both head sizes (64: vit-b/l, 80: vit-h) and both 16-bit
// element types (bf16; fp16 for BASELINE configs[4]):
//   * 8 waves x 32 queries per workgroup; v_mfma_f32_32x32x16_{bf16,f16} throughout.
//   * S^T = K . Q^T (operand-swapped): every lane owns ONE query (column) and 16 keys per 32x32 block, so
//     softmax statistics, the rel-pos terms and the O rescale are per lane (+ one lane^32 exchange).
//   * K / V stream global -> LDS with global_load_lds into a 3-deep ring of 64-key tiles (counted vmcnt +
//     raw barrier). The first 64 head dims: K in a ds_read_b128 XOR-swizzled image, V row-major read
//     transposed with ds_read_b64_tr_b16 (its image swaps 64-B halves on rows 2,3 mod 4: conflict-free).
//     Head dim 80 adds a 16-dim tail image of K and V per tile (32-B rows, 4-B DMA granules, every wave
//     issuing the same number of DMA ops): one more q.k step and a third 32-row O^T block whose rows
//     80..95 read a zero block.
//   * O^T = V^T . P^T takes P^T straight from the S^T accumulator registers (k order permuted to match).
//   * Softmax in base 2: p = exp2(acc * scale*log2e + bias*log2e - m).
// Global layers (side 64, T = 4096): 256 queries (4 image rows) per workgroup, 64 tiles of 64 keys (= one key
// image row each, so rel_h is one LDS scalar per lane per tile and rel_w is the MFMA accumulator init).
// Windowed layers (side 14, T = 196): two 4-wave workgroups per (window, head), keys in 16-column slots
// (224 slots, 3.5 tiles; padding masked through the rel_w accumulator init), rel_w / rel_h per lane in
// registers.
#include "common.h"
#include "../../include/octsam.h"

namespace {

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename E> struct ET;
template <> struct ET<bf16> {
  typedef bf16x8 v8;
  typedef bf16x4 v4;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct ET<f16> {
  typedef f16x8 v8;
  typedef f16x4 v4;
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

constexpr int NW = 8, THR = NW * 64, NBUF = 3;
constexpr float L2E = 1.4426950408889634f;
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float max3f(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }
// The two lane halves hold one query's statistics: v_permlane32_swap of x with itself gives every lane {x of the
// lower half, x of the upper half} (lane i and lane i ^ 32 see the same pair), so max / sum across the halves
// take one swap and one VALU op (no ds_bpermute round trip on the softmax's dependency chain)
__device__ __forceinline__ f32x2 halves(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return (f32x2){__builtin_bit_cast(float, (uint32_t)r[0]), __builtin_bit_cast(float, (uint32_t)r[1])};
}
__device__ __forceinline__ float max_halves(float x) { const f32x2 h = halves(x); return fmaxf(h[0], h[1]); }
__device__ __forceinline__ float sum_halves(float x) { const f32x2 h = halves(x); return h[0] + h[1]; }

template <int HD> struct Geo {
  static_assert(HD == 64 || HD == 80, "head_dim 64 or 80");
  static constexpr int NKS = HD / 16;         // q.k steps of 16 dims
  static constexpr int NTD = (HD + 31) / 32;  // 32-row blocks of O^T
  static constexpr bool TAIL = HD > 64;       // the 16-dim tail images
  static constexpr int K_OFF = 0, V_OFF = 8192, KT_OFF = 16384, VT_OFF = 16384 + 2048;
  static constexpr int TILE = TAIL ? 16384 + 4096 : 16384;
  static constexpr int OPS = TAIL ? 4 : 2;    // DMA ops per 8-row group per tile
};

// Row index (within a 32x32 tile) held in accumulator register r by lane half h.
__device__ __forceinline__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ int vsw(int r, int c) { return r * 128 + ((c ^ (((r >> 1) & 1) << 2)) << 4); }
__device__ __forceinline__ int ksw_b(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Workgroup id -> logical id so each XCD runs a contiguous range of logical ids: the dispatcher deals
// workgroups to the 8 XCDs round-robin by linear id, which would put the workgroups that share K/V (the query
// blocks of one (sequence, head)) on different XCDs, each fetching them into its own L2.
__device__ __forceinline__ int xcd_logical(int id, int n) {
  const int q = n >> 3, rr = n & 7, xcd = id & 7, loc = id >> 3;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
}

template <int N> __device__ __forceinline__ void wait_vm();
template <> __device__ __forceinline__ void wait_vm<0>() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
template <> __device__ __forceinline__ void wait_vm<2>() { asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); }
template <> __device__ __forceinline__ void wait_vm<4>() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
template <> __device__ __forceinline__ void wait_vm<8>() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }

template <typename E>
__device__ __forceinline__ typename ET<E>::v8 pack8(const f32x16& a, int base) {
  typename ET<E>::v8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (E)a[base + j];
  return r;
}

// Online softmax with a lazy reference (base-2 units): the running reference m moves only when a tile's
// maximum exceeds it by more than LAZY, so the O / l rescale (a wave-uniform branch) runs on a handful of tiles
// instead of almost every one. p = exp2(score - m) <= 2^LAZY then; O / l is invariant to the reference.
constexpr float LAZY = 8.0f;
template <int NTD>
__device__ __forceinline__ void lazy_rescale(float mt, float& m_run, float& l_run, f32x16 (&acc_o)[NTD]) {
  const bool grow = mt > m_run + LAZY;
  if (__builtin_amdgcn_ballot_w64(grow)) {
    const float m_new = grow ? mt : m_run;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 0 on the first tile, 1 on lanes that keep m
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int td = 0; td < NTD; ++td) acc_o[td] *= alpha;
  }
}

// 32 table rows j0 .. j0+31 of P^T = R . Q^T for the lane's query (natural units), rows outside [0, nrows)
// zero. R fp32 [nrows][HD], rounded to the element type like the q.k operands.
// Split form for prologues that issue the K/V DMA after the table rows: rel_load fetches the lane's table row
// (rows outside [0, nrows) clamped, zeroed by rel_mma), so the compiler's counted wait for it does not cover
// DMA issued later.
template <int HD> struct RelRow {
  float4 x[Geo<HD>::NKS][2];
};
template <int HD>
__device__ __forceinline__ RelRow<HD> rel_load(const float* __restrict__ R, int j0, int nrows, int lane) {
  const int h = lane >> 5, j = min(max(j0 + (lane & 31), 0), nrows - 1);
  RelRow<HD> r;
#pragma unroll
  for (int s = 0; s < Geo<HD>::NKS; ++s) {
    const float* rp = R + j * HD + 16 * s + 8 * h;
    r.x[s][0] = *(const float4*)rp;
    r.x[s][1] = *(const float4*)(rp + 4);
  }
  return r;
}
template <int HD, typename E>
__device__ __forceinline__ f32x16 rel_mma(const RelRow<HD>& rr, int j0, int nrows,
                                          const typename ET<E>::v8 (&qf)[Geo<HD>::NKS], int lane) {
  const int j = j0 + (lane & 31);
  const bool ok = j >= 0 && j < nrows;
  f32x16 acc = (f32x16)0.0f;
#pragma unroll
  for (int s = 0; s < Geo<HD>::NKS; ++s) {
    const float4 x0 = rr.x[s][0], x1 = rr.x[s][1];
    typename ET<E>::v8 a;
    a[0] = (E)x0.x; a[1] = (E)x0.y; a[2] = (E)x0.z; a[3] = (E)x0.w;
    a[4] = (E)x1.x; a[5] = (E)x1.y; a[6] = (E)x1.z; a[7] = (E)x1.w;
    if (!ok) a = (typename ET<E>::v8)(E)0.0f;
    acc = ET<E>::mma(a, qf[s], acc);
  }
  return acc;
}

template <int HD, typename E>
__device__ __forceinline__ f32x16 rel_block(const float* __restrict__ R, int j0, int nrows,
                                            const typename ET<E>::v8 (&qf)[Geo<HD>::NKS], int lane) {
  const int h = lane >> 5, j = j0 + (lane & 31);
  f32x16 acc = (f32x16)0.0f;
#pragma unroll
  for (int s = 0; s < Geo<HD>::NKS; ++s) {
    typename ET<E>::v8 a;
    if (j >= 0 && j < nrows) {
      const float* rp = R + j * HD + 16 * s + 8 * h;
      const float4 x0 = *(const float4*)rp, x1 = *(const float4*)(rp + 4);
      a[0] = (E)x0.x; a[1] = (E)x0.y; a[2] = (E)x0.z; a[3] = (E)x0.w;
      a[4] = (E)x1.x; a[5] = (E)x1.y; a[6] = (E)x1.z; a[7] = (E)x1.w;
    } else {
      a = (typename ET<E>::v8)(E)0.0f;
    }
    acc = ET<E>::mma(a, qf[s], acc);
  }
  return acc;
}

// Global layers: keys key0 .. key0+63 -> ring slot by NWV waves, every wave the same number of ops: per 8-row
// group 1 KiB (8 rows x 128 B) of each first-64-dim image, and for head dim 80 256 B (8 rows x 32 B) of each tail.
template <int HD, int NWV, typename E>
__device__ __forceinline__ void load_tile(const E* kbase, const E* vbase, int ld, int key0, char* slot, int wave,
                                          int lane) {
  using G = Geo<HD>;
#pragma unroll
  for (int i = 0; i < 8 / NWV; ++i) {  // 8-row groups of this wave
    const int grp = wave + NWV * i;
    const int r = grp * 8 + (lane >> 3), sl = lane & 7;
    const long long row = (long long)(key0 + r) * ld;
    const int ck = sl ^ ((r >> 1) & 7), cv = sl ^ (((r >> 1) & 1) << 2);
    __builtin_amdgcn_global_load_lds((const void*)(kbase + row + ck * 8), (lds_ptr_t)(slot + G::K_OFF + grp * 1024),
                                     16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(vbase + row + cv * 8), (lds_ptr_t)(slot + G::V_OFF + grp * 1024),
                                     16, 0, 0);
    if constexpr (G::TAIL) {
      __builtin_amdgcn_global_load_lds((const void*)(kbase + row + 64 + 2 * sl),
                                       (lds_ptr_t)(slot + G::KT_OFF + grp * 256), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(vbase + row + 64 + 2 * sl),
                                       (lds_ptr_t)(slot + G::VT_OFF + grp * 256), 4, 0, 0);
    }
  }
}

// Rows of one window's 196 tokens. Window-ordered input (grid == 0): row t of the window's block of the qkv
// tensor (window_partition already applied, padding rows present). Token-ordered input (grid > 0, the image's
// grid x grid tokens row-major, B images): the window's token (ty, tx) is image row (y0 + ty, x0 + tx); tokens
// past the grid (window_partition's zero padding, whose qkv row is the bias row) read `pad`, and their
// outputs are dropped (window_unpartition), so the padded rows are never formed.
template <typename E> struct WinRows {
  const E* base;
  const E* pad;
  long long img;  // first row of the window's image (token-ordered)
  int ld, grid, y0, x0;
  __device__ __forceinline__ WinRows(const E* qkv, const E* pad_, int win, int ld_, int grid_) : pad(pad_), ld(ld_), grid(grid_) {
    if (grid == 0) {
      base = qkv + (long long)win * 196 * ld;
      img = 0; y0 = 0; x0 = 0;
    } else {
      const int nw = (grid + 13) / 14, b = win / (nw * nw), r = win - b * nw * nw, wy = r / nw;
      base = qkv;
      img = (long long)b * grid * grid;
      y0 = 14 * wy;
      x0 = 14 * (r - wy * nw);
    }
  }
  __device__ __forceinline__ bool real(int t) const {
    const int ty = t / 14;
    return grid == 0 || (y0 + ty < grid && x0 + t - 14 * ty < grid);
  }
  __device__ __forceinline__ long long row(int t) const {  // token-ordered row (grid > 0) or window row
    if (grid == 0) return t;
    const int ty = t / 14;
    return img + (long long)(y0 + ty) * grid + (x0 + t - 14 * ty);
  }
  __device__ __forceinline__ const E* at(int t) const {
    if (grid == 0) return base + (long long)t * ld;
    return real(t) ? base + row(t) * ld : pad;
  }
};

// Windowed layers: key slots key0 .. key0+63 (slot = 16 kh + kw; key rows padded 14 -> 16 columns, 14 rows ->
// 16, padding slots load the window's last key, their scores are masked) -> ring slot; same per-wave ops as
// load_tile. koff / voff: the head's K / V columns within a qkv row.
template <int HD, int NWV, typename E>
__device__ __forceinline__ void load_tile_win(const WinRows<E>& wr, int koff, int voff, int key0, char* slot,
                                              int wave, int lane) {
  using G = Geo<HD>;
#pragma unroll
  for (int i = 0; i < 8 / NWV; ++i) {
    const int grp = wave + NWV * i;
    const int r = grp * 8 + (lane >> 3), sl = lane & 7;
    const int key = key0 + r;
    const E* rp = wr.at(min((key >> 4) * 14 + min(key & 15, 13), 195));
    const int ck = sl ^ ((r >> 1) & 7), cv = sl ^ (((r >> 1) & 1) << 2);
    __builtin_amdgcn_global_load_lds((const void*)(rp + koff + ck * 8), (lds_ptr_t)(slot + G::K_OFF + grp * 1024),
                                     16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(rp + voff + cv * 8), (lds_ptr_t)(slot + G::V_OFF + grp * 1024),
                                     16, 0, 0);
    if constexpr (G::TAIL) {
      __builtin_amdgcn_global_load_lds((const void*)(rp + koff + 64 + 2 * sl),
                                       (lds_ptr_t)(slot + G::KT_OFF + grp * 256), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(rp + voff + 64 + 2 * sl),
                                       (lds_ptr_t)(slot + G::VT_OFF + grp * 256), 4, 0, 0);
    }
  }
}

// S^T block t2 (keys 32 t2 .. 32 t2 + 31 of the tile) = K . Q^T + init
template <int HD, typename E>
__device__ __forceinline__ f32x16 qk_block(const char* slot, int t2, const typename ET<E>::v8 (&qf)[Geo<HD>::NKS],
                                           f32x16 init, int l32, int h) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  f32x16 acc = init;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const V8 a = *(const V8*)(slot + G::K_OFF + ksw_b(t2 * 32 + l32, 2 * s + h));
    acc = ET<E>::mma(a, qf[s], acc);
  }
  if constexpr (G::TAIL) {
    const V8 a = *(const V8*)(slot + G::KT_OFF + (t2 * 32 + l32) * 32 + 16 * h);
    acc = ET<E>::mma(a, qf[4], acc);
  }
  return acc;
}

// O^T += V^T . P^T over keys 16 ks .. 16 ks + 15 of the tile (P^T k-slot j of lane half hh is key
// 16ks + 8(j>>2) + 4hh + (j&3)); the tail block's rows 80..95 read the zero block.
template <int HD, typename E>
__device__ __forceinline__ void pv_step(const char* slot, const char* zero, int ks, const typename ET<E>::v8& pf,
                                        f32x16 (&acc_o)[Geo<HD>::NTD], int lane) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const char* sv = slot + G::V_OFF;
  const int r0 = 16 * ks + 4 * (g >> 1) + qq;
#pragma unroll
  for (int td = 0; td < 2; ++td) {
    const int ch = 4 * td + 2 * (g & 1) + (pp >> 1);
    const char* a0 = sv + vsw(r0, ch) + 8 * (pp & 1);
    const char* a1 = sv + vsw(r0 + 8, ch) + 8 * (pp & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    const s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    acc_o[td] = ET<E>::mma(__builtin_bit_cast(V8, v8), pf, acc_o[td]);
  }
  if constexpr (G::TAIL) {
    const bool z = (g & 1) != 0;  // rows 80..95 of the third block
    const char* a0 = z ? zero + 32 * qq + 8 * pp : slot + G::VT_OFF + r0 * 32 + 8 * pp;
    const char* a1 = z ? zero + 32 * qq + 8 * pp : slot + G::VT_OFF + (r0 + 8) * 32 + 8 * pp;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    const s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    acc_o[2] = ET<E>::mma(__builtin_bit_cast(V8, v8), pf, acc_o[2]);
  }
}

template <int HD, typename E>
__device__ __forceinline__ void store_out(E* orow, const f32x16 (&acc_o)[Geo<HD>::NTD], float inv, int h) {
  using V4 = typename ET<E>::v4;
#pragma unroll
  for (int td = 0; td < Geo<HD>::NTD; ++td)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      if (td * 32 + 8 * gg + 8 > HD) continue;  // compile-time: the tail block holds dims 64..79 only
      V4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (E)(acc_o[td][4 * gg + e] * inv);
      *(V4*)(orow + td * 32 + 8 * gg + 4 * h) = o;
    }
}

template <int HD, typename E>
__device__ __forceinline__ void load_q(const E* qrow, typename ET<E>::v8 (&qf)[Geo<HD>::NKS], int h) {
#pragma unroll
  for (int s = 0; s < Geo<HD>::NKS; ++s) qf[s] = *(const typename ET<E>::v8*)(qrow + 16 * s + 8 * h);
}

// ------------------------------------------------------------------------------------ global (side 64)
constexpr int G_RELH = NW * 64 * 32 * 4;  // rel_h tables [64 kh][32 q] fp32 per wave: 64 KiB
constexpr int G_SCR = 96 * 33;           // rel_w scratch [96][33] fp32 per wave (overlays tables + ring)
template <int HD> constexpr int g_smem() { return G_RELH + NBUF * Geo<HD>::TILE + 128; }

template <int HD, typename E>
__global__ __launch_bounds__(THR) void vit_attn_global_kernel(const E* __restrict__ qkv, E* __restrict__ out,
                                                                 const float* __restrict__ Rh,
                                                                 const float* __restrict__ Rw, int heads, float scale) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  constexpr int S = 64, T = 4096, NT = T / 64;
  static_assert(NW * G_SCR * 4 <= G_RELH + NBUF * G::TILE, "rel_w scratch must fit");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  // logical id = (seq, head, query block), query block fastest: the 16 blocks of a (seq, head) on one XCD
  const int lid = xcd_logical(blockIdx.x, gridDim.x);
  const int qblk = lid & 15, head = (lid >> 4) % heads, seq = (lid >> 4) / heads;
  const int D = heads * HD, ld = 3 * D;
  const E* base = qkv + (long long)seq * T * ld;
  const int q = qblk * (NW * 32) + wave * 32 + l32;
  const int qh = q >> 6, qw = q & 63, qw0 = qw - l32;
  const float c1 = scale * L2E;
  if (__builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);  // the SIMD's 2 waves drift

  V8 qf[G::NKS];
  load_q<HD, E>(base + (long long)q * ld + head * HD, qf, h);

  // rel_w (registers): rows j = qw - kw + 63 in [qw0, qw0 + 95) of the table, staged through scratch, kept as
  // the initial accumulator of the S^T chain in units of the raw q.k (divided by the scale)
  float* scr = (float*)gsm + wave * G_SCR;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 t = rel_block<HD, E>(Rw, qw0 + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) scr[(32 * b + acc_row(r, h)) * 33 + l32] = t[r];
  }
  __syncthreads();
  const float inv_scale = 1.0f / scale;
  f32x16 relw[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; ++r) relw[t2][r] = scr[(l32 - (32 * t2 + acc_row(r, h)) + 63) * 33 + l32] * inv_scale;
  __syncthreads();
  // rel_h table [kh][q] (log2 units): row j = qh - kh + 63 -> block rows i = j - qh = 63 - kh
  float* relh = (float*)gsm + wave * (64 * 32);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const f32x16 t = rel_block<HD, E>(Rh, qh + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) relh[(63 - (32 * b + acc_row(r, h))) * 32 + l32] = t[r] * L2E;
  }
  char* ring = gsm + G_RELH;
  char* zero = ring + NBUF * G::TILE;
  if (tid < 32) ((float*)zero)[tid] = 0.0f;
  __syncthreads();

  const E* kbase = base + D + head * HD;
  const E* vbase = base + 2 * D + head * HD;
  load_tile<HD, NW, E>(kbase, vbase, ld, 0, ring, wave, lane);
  load_tile<HD, NW, E>(kbase, vbase, ld, 64, ring + G::TILE, wave, lane);

  f32x16 acc_o[G::NTD];
#pragma unroll
  for (int td = 0; td < G::NTD; ++td) acc_o[td] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;  // base-2 running max / sum

  for (int tile = 0; tile < NT; ++tile) {
    if (tile + 1 < NT) wait_vm<G::OPS>();
    else wait_vm<0>();
    raw_barrier();
    if (tile + 2 < NT)
      load_tile<HD, NW, E>(kbase, vbase, ld, (tile + 2) * 64, ring + ((tile + 2) % NBUF) * G::TILE, wave, lane);
    const char* slot = ring + (tile % NBUF) * G::TILE;
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) sacc[t2] = qk_block<HD, E>(slot, t2, qf, relw[t2], l32, h);
    // tile = key image row kh: rel_h is one constant per lane (log2 units), so max and exponent take it
    // once per tile: p = exp2(c1 * acc + (rh - m)), one FMA + one exp per score
    const float rh = relh[tile * 32 + l32];
    // max: 16 three-input maxima (scores are finite: the kernel is built without NaN canonicalisation, see
    // Makefile); sum: packed adds
    float mx = sacc[0][0];
#pragma unroll
    for (int i = 1; i < 31; i += 2) mx = max3f(mx, sacc[i >> 4][i & 15], sacc[(i + 1) >> 4][(i + 1) & 15]);
    mx = fmaxf(mx, sacc[1][15]);
    mx = max_halves(mx);
    lazy_rescale<G::NTD>(fmaf(mx, c1, rh), m_run, l_run, acc_o);
    const float c = rh - m_run;
    f32x2 ls2 = {0.0f, 0.0f};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f32x2 x = {sacc[t2][r], sacc[t2][r + 1]};
        const f32x2 y = x * c1 + c;  // v_pk_fma_f32
        const f32x2 pv = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
        sacc[t2][r] = pv[0];
        sacc[t2][r + 1] = pv[1];
        ls2 += pv;  // v_pk_add_f32
      }
    l_run += ls2[0] + ls2[1];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pv_step<HD, E>(slot, zero, ks, pack8<E>(sacc[ks >> 1], 8 * (ks & 1)), acc_o, lane);
  }
  const float l_tot = sum_halves(l_run);
  store_out<HD, E>(out + ((long long)seq * T + q) * D + head * HD, acc_o, 1.0f / l_tot, h);
}

// ---------------------------------------------------------------- global, 4-wave workgroups (A/B variant 2)
// The same per-lane arithmetic as vit_attn_global_kernel (bit-identical outputs) in 4-wave workgroups of 128
// queries (two image rows) with a 2-deep K/V ring: 32 KiB of rel_h tables + 32 KiB (head_dim 80: 40) of ring per
// workgroup, so two workgroups share a CU and each SIMD runs one wave of each. The 8-wave kernel's two waves on a
// SIMD meet at the same per-tile barrier and run each phase (q.k on the matrix pipe, the exponentials on the
// VALU, P.V) at the same time; waves of independent workgroups drift apart, so one's softmax issues beside the
// other's products (PMC, profiles/r03/pmc/attn_global.summary.txt: VALU ~60 % and MFMA ~33 % busy, 40 % of wave
// time waiting).
constexpr int NW4 = 4, THR4 = NW4 * 64;
constexpr int G4_RELH = NW4 * 64 * 32 * 4;  // rel_h tables [64 kh][32 q] fp32 per wave: 32 KiB
template <int HD> constexpr int g4_smem() { return G4_RELH + 2 * Geo<HD>::TILE + 128; }
// HALF: each wave keeps the rel_h rows of 32 key rows at a time ([32 kh][32 q] fp32, 16 KiB for the workgroup; the
// second half is computed when the loop reaches key row 32), so three workgroups share a CU (the rel_w scratch then
// sets the size). Same values as the whole table: bit-identical.
template <int HD> constexpr int g4h_smem() {
  return (G4_RELH / 2 + 2 * Geo<HD>::TILE + 128) > NW4 * G_SCR * 4 ? (G4_RELH / 2 + 2 * Geo<HD>::TILE + 128)
                                                                     : NW4 * G_SCR * 4;
}
static_assert(3 * g4h_smem<64>() <= 160 * 1024, "three half-table global workgroups per CU at head_dim 64");
static_assert(2 * g4_smem<80>() <= 160 * 1024, "two 4-wave global workgroups per CU");
template <> __device__ __forceinline__ void wait_vm<16>() { asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); }

template <int HD, typename E, bool HALF = false>
__global__ __launch_bounds__(THR4, HALF ? 3 : 2) void vit_attn_global4_kernel(const E* __restrict__ qkv, E* __restrict__ out,
                                                                   const float* __restrict__ Rh,
                                                                   const float* __restrict__ Rw, int heads, float scale) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  constexpr int S = 64, T = 4096, NT = T / 64, QB = T / (NW4 * 32);  // 32 query blocks per (sequence, head)
  static_assert(NW4 * G_SCR * 4 <= G4_RELH + 2 * G::TILE, "rel_w scratch must fit");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            l32 = lane & 31;
  const int lid = xcd_logical(blockIdx.x, gridDim.x);
  const int qblk = lid % QB, head = (lid / QB) % heads, seq = (lid / QB) / heads;
  const int D = heads * HD, ld = 3 * D;
  const E* base = qkv + (long long)seq * T * ld;
  const int q = qblk * (NW4 * 32) + wave * 32 + l32;
  const int qh = q >> 6, qw = q & 63, qw0 = qw - l32;
  const float c1 = scale * L2E;

  V8 qf[G::NKS];
  load_q<HD, E>(base + (long long)q * ld + head * HD, qf, h);
  float* scr = (float*)gsm + wave * G_SCR;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 t = rel_block<HD, E>(Rw, qw0 + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) scr[(32 * b + acc_row(r, h)) * 33 + l32] = t[r];
  }
  __syncthreads();
  const float inv_scale = 1.0f / scale;
  f32x16 relw[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; ++r) relw[t2][r] = scr[(l32 - (32 * t2 + acc_row(r, h)) + 63) * 33 + l32] * inv_scale;
  __syncthreads();
  float* relh = (float*)gsm + wave * (HALF ? 32 * 32 : 64 * 32);
  if constexpr (HALF) {  // key rows 0..31 now (table block b = 1), 32..63 at tile 32
    const f32x16 t = rel_block<HD, E>(Rh, qh + 32, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) relh[(31 - acc_row(r, h)) * 32 + l32] = t[r] * L2E;
  } else {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const f32x16 t = rel_block<HD, E>(Rh, qh + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) relh[(63 - (32 * b + acc_row(r, h))) * 32 + l32] = t[r] * L2E;
    }
  }
  char* ring = gsm + (HALF ? G4_RELH / 2 : G4_RELH);
  char* zero = ring + 2 * G::TILE;
  if (tid < 32) ((float*)zero)[tid] = 0.0f;
  __syncthreads();

  const E* kbase = base + D + head * HD;
  const E* vbase = base + 2 * D + head * HD;
  load_tile<HD, NW4, E>(kbase, vbase, ld, 0, ring, wave, lane);

  f32x16 acc_o[G::NTD];
#pragma unroll
  for (int td = 0; td < G::NTD; ++td) acc_o[td] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;
  for (int tile = 0; tile < NT; ++tile) {
    // tile resident (the only load in flight); every wave is past tile - 1, whose slot takes tile + 1
    wait_vm<0>();
    raw_barrier();
    if (tile + 1 < NT) load_tile<HD, NW4, E>(kbase, vbase, ld, (tile + 1) * 64, ring + ((tile + 1) & 1) * G::TILE, wave, lane);
    const char* slot = ring + (tile & 1) * G::TILE;
    f32x16 sacc[2];
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) sacc[t2] = qk_block<HD, E>(slot, t2, qf, relw[t2], l32, h);
    if constexpr (HALF) {
      if (tile == 32) {  // key rows 32..63 (table block b = 0) over the wave's own rows 0..31 (wave-local)
        const f32x16 t = rel_block<HD, E>(Rh, qh, 2 * S - 1, qf, lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) relh[(31 - acc_row(r, h)) * 32 + l32] = t[r] * L2E;
      }
    }
    const float rh = relh[(HALF ? (tile & 31) : tile) * 32 + l32];
    float mx = sacc[0][0];
#pragma unroll
    for (int i = 1; i < 31; i += 2) mx = max3f(mx, sacc[i >> 4][i & 15], sacc[(i + 1) >> 4][(i + 1) & 15]);
    mx = fmaxf(mx, sacc[1][15]);
    mx = max_halves(mx);
    lazy_rescale<G::NTD>(fmaf(mx, c1, rh), m_run, l_run, acc_o);
    const float c = rh - m_run;
    f32x2 ls2 = {0.0f, 0.0f};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f32x2 x = {sacc[t2][r], sacc[t2][r + 1]};
        const f32x2 y = x * c1 + c;  // v_pk_fma_f32
        const f32x2 pv = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
        sacc[t2][r] = pv[0];
        sacc[t2][r + 1] = pv[1];
        ls2 += pv;  // v_pk_add_f32
      }
    l_run += ls2[0] + ls2[1];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pv_step<HD, E>(slot, zero, ks, pack8<E>(sacc[ks >> 1], 8 * (ks & 1)), acc_o, lane);
  }
  const float l_tot = sum_halves(l_run);
  store_out<HD, E>(out + ((long long)seq * T + q) * D + head * HD, acc_o, 1.0f / l_tot, h);
}

// ---------------------------------------------------------------- global, software-pipelined (A/B variant 0)
// Same arithmetic as vit_attn_global_kernel (bit-identical outputs), reordered per wave so that its own
// instruction stream keeps both pipes busy: the q.k MFMAs of tile t+1 issue while the VALU exponentiates tile t,
// and the P.V MFMAs of tile t issue while the VALU takes the maximum of tile t+1. In the plain loop every phase
// of a tile (q.k, softmax, P.V) runs on the two waves of a SIMD at the same time (they meet at the per-tile
// barrier), so the matrix pipe idles through the softmax and the VALU through the products. A 4-deep K/V ring
// (tile t+1 must be resident while tile t's V is still read), 2 tiles in flight. Measured on MI355X: bit-identical
// to the plain loop and no faster (526 vs 521 us per vit-b layer, profiles/r03/attn_pipelined_ab.log), so the plain
// loop stays the default.
constexpr int NBUF_P = 4;
template <int HD> constexpr int gp_smem() { return G_RELH + NBUF_P * Geo<HD>::TILE + 128; }
static_assert(gp_smem<80>() <= 160 * 1024, "pipelined global attention LDS");

// exp / row-sum / bf16 pack of one tile's scores (base 2: p = exp2(c1 * s + c)); returns the four P^T operands
template <typename E>
__device__ __forceinline__ void softmax_pack(f32x16 (&s)[2], float c1, float c, f32x2& ls2,
                                             typename ET<E>::v8 (&pf)[4]) {
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const f32x2 x = {s[t2][r], s[t2][r + 1]};
      const f32x2 y = x * c1 + c;  // v_pk_fma_f32
      const f32x2 pv = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
      s[t2][r] = pv[0];
      s[t2][r + 1] = pv[1];
      ls2 += pv;  // v_pk_add_f32
    }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) pf[ks] = pack8<E>(s[ks >> 1], 8 * (ks & 1));
}

// raw maximum of one tile's 32 scores per lane, then the tile maximum in base-2 units across the lane halves
__device__ __forceinline__ float tile_max(const f32x16 (&s)[2], float c1, float rh) {
  float mx = s[0][0];
#pragma unroll
  for (int i = 1; i < 31; i += 2) mx = max3f(mx, s[i >> 4][i & 15], s[(i + 1) >> 4][(i + 1) & 15]);
  mx = fmaxf(mx, s[1][15]);
  return max_halves(fmaf(mx, c1, rh));
}

template <int HD, typename E, bool MORE, bool WAIT_PART, bool LOAD>
__device__ __forceinline__ void gpipe_step(int tile, f32x16 (&s_cur)[2], f32x16 (&s_nxt)[2], float& mx_cur,
                                           float& rh_cur, float& m_run, float& l_run, f32x16 (&acc_o)[Geo<HD>::NTD],
                                           const typename ET<E>::v8 (&qf)[Geo<HD>::NKS], const f32x16 (&relw)[2],
                                           const float* relh, char* ring, const char* zero, const E* kbase,
                                           const E* vbase, int ld, float c1, int wave, int lane) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  const int h = lane >> 5, l32 = lane & 31;
  lazy_rescale<G::NTD>(mx_cur, m_run, l_run, acc_o);
  const float c = rh_cur - m_run;
  if constexpr (MORE) {
    // tile + 1 resident (vmcnt: the loads issued after it may stay in flight); every wave is past P.V(tile - 1),
    // so the slot of tile + 3 (= tile - 1's) may be restaged
    if constexpr (WAIT_PART) wait_vm<G::OPS>();
    else wait_vm<0>();
    raw_barrier();
    if constexpr (LOAD)
      load_tile<HD, NW, E>(kbase, vbase, ld, (tile + 3) * 64, ring + ((tile + 3) % NBUF_P) * G::TILE, wave, lane);
  }
  const char* slot = ring + (tile % NBUF_P) * G::TILE;
  // q.k of tile + 1 (matrix pipe) beside the exponentials of tile (VALU)
  if constexpr (MORE) {
    const char* nslot = ring + ((tile + 1) % NBUF_P) * G::TILE;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) s_nxt[t2] = qk_block<HD, E>(nslot, t2, qf, relw[t2], l32, h);
  }
  f32x2 ls2 = {0.0f, 0.0f};
  V8 pf[4];
  softmax_pack<E>(s_cur, c1, c, ls2, pf);
  l_run += ls2[0] + ls2[1];
  if constexpr (MORE) {
    // interleave: the 8 K-fragment reads, then one q.k MFMA per 10 VALU instructions of the softmax
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int i = 0; i < 8 + (G::TAIL ? 2 : 0); ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
    }
  }
  // P.V of tile (matrix pipe) beside the maximum of tile + 1 (VALU)
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) pv_step<HD, E>(slot, zero, ks, pf[ks], acc_o, lane);
  if constexpr (MORE) {
    rh_cur = relh[(tile + 1) * 32 + l32];
    mx_cur = tile_max(s_nxt, c1, rh_cur);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
    }
  }
}

template <int HD, typename E>
__global__ __launch_bounds__(THR) void vit_attn_global_pipe_kernel(const E* __restrict__ qkv, E* __restrict__ out,
                                                                  const float* __restrict__ Rh,
                                                                  const float* __restrict__ Rw, int heads, float scale) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  constexpr int S = 64, T = 4096, NT = T / 64;
  static_assert(NT % 2 == 0 && NT >= 6, "pairs of tiles, three tail pairs");
  static_assert(NW * G_SCR * 4 <= G_RELH + NBUF_P * G::TILE, "rel_w scratch must fit");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int lid = xcd_logical(blockIdx.x, gridDim.x);
  const int qblk = lid & 15, head = (lid >> 4) % heads, seq = (lid >> 4) / heads;
  const int D = heads * HD, ld = 3 * D;
  const E* base = qkv + (long long)seq * T * ld;
  const int q = qblk * (NW * 32) + wave * 32 + l32;
  const int qh = q >> 6, qw = q & 63, qw0 = qw - l32;
  const float c1 = scale * L2E;
  if (__builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);

  V8 qf[G::NKS];
  load_q<HD, E>(base + (long long)q * ld + head * HD, qf, h);
  float* scr = (float*)gsm + wave * G_SCR;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 t = rel_block<HD, E>(Rw, qw0 + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) scr[(32 * b + acc_row(r, h)) * 33 + l32] = t[r];
  }
  __syncthreads();
  const float inv_scale = 1.0f / scale;
  f32x16 relw[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
    for (int r = 0; r < 16; ++r) relw[t2][r] = scr[(l32 - (32 * t2 + acc_row(r, h)) + 63) * 33 + l32] * inv_scale;
  __syncthreads();
  float* relh = (float*)gsm + wave * (64 * 32);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const f32x16 t = rel_block<HD, E>(Rh, qh + 32 * b, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) relh[(63 - (32 * b + acc_row(r, h))) * 32 + l32] = t[r] * L2E;
  }
  char* ring = gsm + G_RELH;
  char* zero = ring + NBUF_P * G::TILE;
  if (tid < 32) ((float*)zero)[tid] = 0.0f;
  __syncthreads();

  const E* kbase = base + D + head * HD;
  const E* vbase = base + 2 * D + head * HD;
#pragma unroll
  for (int t = 0; t < 3; ++t) load_tile<HD, NW, E>(kbase, vbase, ld, t * 64, ring + t * G::TILE, wave, lane);

  f32x16 acc_o[G::NTD];
#pragma unroll
  for (int td = 0; td < G::NTD; ++td) acc_o[td] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;
  // tile 0 resident (tiles 1, 2 in flight): its scores and maximum
  wait_vm<2 * G::OPS>();
  raw_barrier();
  f32x16 sA[2], sB[2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) sA[t2] = qk_block<HD, E>(ring, t2, qf, relw[t2], l32, h);
  float rh_cur = relh[l32];
  float mx_cur = tile_max(sA, c1, rh_cur);
  // tile pairs (sA holds even tiles' scores, sB odd ones): the last three tiles stop loading / waiting
  for (int tile = 0; tile < NT - 4; tile += 2) {
    gpipe_step<HD, E, true, true, true>(tile, sA, sB, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring, zero,
                                        kbase, vbase, ld, c1, wave, lane);
    gpipe_step<HD, E, true, true, true>(tile + 1, sB, sA, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring,
                                        zero, kbase, vbase, ld, c1, wave, lane);
  }
  gpipe_step<HD, E, true, true, true>(NT - 4, sA, sB, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring, zero,
                                      kbase, vbase, ld, c1, wave, lane);
  gpipe_step<HD, E, true, true, false>(NT - 3, sB, sA, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring, zero,
                                       kbase, vbase, ld, c1, wave, lane);
  gpipe_step<HD, E, true, false, false>(NT - 2, sA, sB, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring,
                                        zero, kbase, vbase, ld, c1, wave, lane);
  gpipe_step<HD, E, false, false, false>(NT - 1, sB, sA, mx_cur, rh_cur, m_run, l_run, acc_o, qf, relw, relh, ring,
                                         zero, kbase, vbase, ld, c1, wave, lane);
  const float l_tot = sum_halves(l_run);
  store_out<HD, E>(out + ((long long)seq * T + q) * D + head * HD, acc_o, 1.0f / l_tot, h);
}

// ------------------------------------------------------------------------------------ window (side 14)
// Keys are laid out in slots 16 kh + kw (kw < 14 real; 14 key rows -> slots 0..223, 3.5 tiles). A 32-slot
// block holds key rows kh0 = 2 block and kh0 + 1, and accumulator register r of lane half h holds slot
// (r & 3) + 8 (r >> 2) + 4 h, i.e. kw = (r & 3) + 8 ((r >> 2) & 1) + 4 h and kh = kh0 + (r >> 3). So the bias
// rel_w[kw] + rel_h[kh] is an 8-entry per-lane vector (the accumulator init, -inf on the padding columns)
// plus one constant per half block: one FMA per score, no per-score table selects.
// Two workgroups of 4 waves per (window, head), queries 0..127 and 128..255 (valid < 196), so that two
// workgroups share a CU and one's prologue (Q, first tiles, rel tables) overlaps the other's key loop.
constexpr int WNW = 4, WTHR = WNW * 64;
constexpr int W_SCR = 27 * 33;  // rel-table scratch [27 = 2*14-1 rows][33] fp32 per wave, in ring slot 2 (its
                                // first tile load is issued after the tables are read)
template <int HD> constexpr int w_smem() { return NBUF * Geo<HD>::TILE + 128; }
static_assert(WNW * W_SCR * 4 <= Geo<64>::TILE, "rel-table scratch must fit in one ring slot");
static_assert(w_smem<64>() <= 160 * 1024 / 3, "three windowed workgroups per CU at head_dim 64");

template <int HD, typename E>
__global__ __launch_bounds__(WTHR, HD == 64 ? 3 : 2) void vit_attn_window_kernel(const E* __restrict__ qkv, E* __restrict__ out,
                                                              const float* __restrict__ Rh,
                                                              const float* __restrict__ Rw, int heads, float scale,
                                                              int grid, const E* __restrict__ pad) {
  using G = Geo<HD>;
  using V8 = typename ET<E>::v8;
  constexpr int S = 14, T = 196, NT = 4;  // 224 key slots in 4 tiles (the last one half used)
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  char* ring = wsm;
  float* scr = (float*)(wsm + 2 * G::TILE) + (threadIdx.x >> 6) * W_SCR;
  char* zero = wsm + NBUF * G::TILE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
  // logical id = (window, head, query half), half fastest, dealt to XCDs in contiguous ranges: the 2*heads
  // workgroups of a window read the same qkv rows through one L2
  const int lid = xcd_logical(blockIdx.x, gridDim.x);
  const int head = (lid >> 1) % heads, win = (lid >> 1) / heads, qhalf = lid & 1;
  const int D = heads * HD, ld = 3 * D;
  const WinRows<E> wr(qkv, pad, win, ld, grid);
  const int q = qhalf * (WNW * 32) + wave * 32 + l32;
  const int qc = q < T ? q : T - 1;
  const bool qvalid = q < T && wr.real(q);
  // the second workgroup's last wave (query slots 224..255) has no real query: it skips the rel tables and
  // every q.k / softmax / P.V, keeping only its share of the K/V loads and the barriers
  const bool idle = __builtin_amdgcn_readfirstlane(q - l32) >= T;
  const int qh = qc / S, qw = qc % S;
  const float c1 = scale * L2E;

  // Q and both tables' rows first, the K/V DMA after them: the waits for Q and the tables then leave the
  // DMA in flight (vmcnt retires in issue order)
  V8 qf[G::NKS];
  load_q<HD, E>(wr.at(qc) + head * HD, qf, h);
  const RelRow<HD> rw_rows = rel_load<HD>(Rw, 0, 2 * S - 1, lane);
  const RelRow<HD> rh_rows = rel_load<HD>(Rh, 0, 2 * S - 1, lane);
  const int koff = D + head * HD, voff = 2 * D + head * HD;
  load_tile_win<HD, WNW, E>(wr, koff, voff, 0, ring, wave, lane);
  load_tile_win<HD, WNW, E>(wr, koff, voff, 64, ring + G::TILE, wave, lane);

  // rel_w for this lane half's 8 kw columns (units of the raw q.k: divided by the scale) and rel_h for the 14
  // key rows (log2 units), through this wave's scratch: table row j = q - i + 13
  f32x16 init = (f32x16)0.0f;
  float relh[S];
#pragma unroll
  for (int i = 0; i < S; ++i) relh[i] = 0.0f;
  if (!idle) {
    const f32x16 t = rel_mma<HD, E>(rw_rows, 0, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (acc_row(r, h) < 2 * S - 1) scr[acc_row(r, h) * 33 + l32] = t[r];
    const float inv_scale = 1.0f / scale;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int kw = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = kw < S ? scr[(qw - (kw < S ? kw : 0) + S - 1) * 33 + l32] * inv_scale : -INFINITY;
      init[r] = v;
      init[r + 8] = v;
    }
  }
  if (!idle) {
    const f32x16 t = rel_mma<HD, E>(rh_rows, 0, 2 * S - 1, qf, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (acc_row(r, h) < 2 * S - 1) scr[acc_row(r, h) * 33 + l32] = t[r];
#pragma unroll
    for (int i = 0; i < S; ++i) relh[i] = scr[(qh - i + S - 1) * 33 + l32] * L2E;
  }
  if (tid < 32) ((float*)zero)[tid] = 0.0f;

  f32x16 acc_o[G::NTD];
#pragma unroll
  for (int td = 0; td < G::NTD; ++td) acc_o[td] = (f32x16)0.0f;
  float m_run = -INFINITY, l_run = 0.0f;
#pragma unroll
  for (int tile = 0; tile < NT; ++tile) {
    if (tile + 1 < NT) wait_vm<G::OPS * 8 / WNW>();
    else wait_vm<0>();
    raw_barrier();
    if (tile + 2 < NT)
      load_tile_win<HD, WNW, E>(wr, koff, voff, (tile + 2) * 64, ring + ((tile + 2) % NBUF) * G::TILE, wave, lane);
    if (idle) continue;  // all 32 query slots of this wave are padding: it only loads and syncs
    const char* slot = ring + (tile % NBUF) * G::TILE;
    const int nb = tile == NT - 1 ? 1 : 2;  // 32-slot blocks holding keys (slots < 224)
    f32x16 sacc[2];
    float mh[4];  // raw max per half block (registers 0-7: key row kh0, 8-15: kh0 + 1)
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      if (t2 >= nb) continue;
      sacc[t2] = qk_block<HD, E>(slot, t2, qf, init, l32, h);
      // three-input maxima (padding columns hold -inf, never NaN)
      float a = max3f(sacc[t2][0], sacc[t2][1], sacc[t2][2]), b = max3f(sacc[t2][8], sacc[t2][9], sacc[t2][10]);
      a = max3f(a, sacc[t2][3], sacc[t2][4]);
      b = max3f(b, sacc[t2][11], sacc[t2][12]);
      a = max3f(a, sacc[t2][5], sacc[t2][6]);
      b = max3f(b, sacc[t2][13], sacc[t2][14]);
      mh[2 * t2] = fmaxf(a, sacc[t2][7]);
      mh[2 * t2 + 1] = fmaxf(b, sacc[t2][15]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 2 * nb; ++k) mx = fmaxf(mx, fmaf(mh[k], c1, relh[4 * tile + k]));
    mx = max_halves(mx);
    lazy_rescale<G::NTD>(mx, m_run, l_run, acc_o);
    f32x2 ls2 = {0.0f, 0.0f};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      if (t2 >= nb) continue;
      const float c0 = relh[4 * tile + 2 * t2] - m_run, cc1 = relh[4 * tile + 2 * t2 + 1] - m_run;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float cc = r < 8 ? c0 : cc1;
        const f32x2 x = {sacc[t2][r], sacc[t2][r + 1]};
        const f32x2 y = x * c1 + (f32x2){cc, cc};  // v_pk_fma_f32
        const f32x2 pv = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
        sacc[t2][r] = pv[0];
        sacc[t2][r + 1] = pv[1];
        ls2 += pv;  // v_pk_add_f32
      }
    }
    l_run += ls2[0] + ls2[1];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks >= 2 * nb) break;
      pv_step<HD, E>(slot, zero, ks, pack8<E>(sacc[ks >> 1], 8 * (ks & 1)), acc_o, lane);
    }
  }
  if (!qvalid) return;
  const float l_tot = sum_halves(l_run);
  const long long orow = grid == 0 ? (long long)win * T + q : wr.row(q);
  store_out<HD, E>(out + orow * D + head * HD, acc_o, 1.0f / l_tot, h);
}

// global-layer kernel (octsam_attention_set_variant): 0 software-pipelined 8-wave loop, 1 plain 8-wave loop, 2 4-wave
// workgroups two per CU, 6 the same with half rel_h tables three per CU, -1 (default) 6 for head_dim 64 and 1 for
// head_dim 80 (same-box A/Bs, scripts/attn_ab.py: profiles/r03/attn_variant_ab.log vit-b 522.5 -> 498.6 us (2),
// vit-h fp16 929.6 vs 934.3 us; profiles/r03/attn_half_table_ab.log vit-b 509.6 -> 483.7 us (6); all bit-identical)
int g_attn_variant = -1;

template <int HD, typename E>
int launch(const void* qkv, void* out, const float* Rh, const float* Rw, int nseq, int side, int heads, int grid,
           const void* pad, hipStream_t s) {
  const float scale = 1.0f / sqrtf((float)HD);
  if (side == 64) {
    static_assert(4096 / (NW * 32) == 16, "16 query blocks per (sequence, head)");
    const int variant = g_attn_variant >= 0 ? g_attn_variant : (HD == 64 ? 6 : 1);
    if (variant == 1) {  // the plain loop (A/B)
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)vit_attn_global_kernel<HD, E>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, g_smem<HD>());
        attr = true;
      }
      hipLaunchKernelGGL((vit_attn_global_kernel<HD, E>), dim3(16 * heads * nseq), dim3(THR), g_smem<HD>(), s,
                         (const E*)qkv, (E*)out, Rh, Rw, heads, scale);
    } else if (variant == 6) {  // 4-wave workgroups with half rel_h tables, three per CU
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)vit_attn_global4_kernel<HD, E, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, g4h_smem<HD>());
        attr = true;
      }
      hipLaunchKernelGGL((vit_attn_global4_kernel<HD, E, true>), dim3(32 * heads * nseq), dim3(THR4), g4h_smem<HD>(), s,
                         (const E*)qkv, (E*)out, Rh, Rw, heads, scale);
    } else if (variant == 2) {  // 4-wave workgroups, two per CU
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)vit_attn_global4_kernel<HD, E>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, g4_smem<HD>());
        attr = true;
      }
      hipLaunchKernelGGL((vit_attn_global4_kernel<HD, E>), dim3(32 * heads * nseq), dim3(THR4), g4_smem<HD>(), s,
                         (const E*)qkv, (E*)out, Rh, Rw, heads, scale);
    } else {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)vit_attn_global_pipe_kernel<HD, E>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, gp_smem<HD>());
        attr = true;
      }
      hipLaunchKernelGGL((vit_attn_global_pipe_kernel<HD, E>), dim3(16 * heads * nseq), dim3(THR), gp_smem<HD>(), s,
                         (const E*)qkv, (E*)out, Rh, Rw, heads, scale);
    }
  } else {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)vit_attn_window_kernel<HD, E>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                w_smem<HD>());
      attr = true;
    }
    hipLaunchKernelGGL((vit_attn_window_kernel<HD, E>), dim3(2 * heads * nseq), dim3(WTHR), w_smem<HD>(), s,
                       (const E*)qkv, (E*)out, Rh, Rw, heads, scale, grid, (const E*)pad);
  }
  return 0;
}

}  // namespace

extern "C" int octsam_vit_attention(const void* qkv, void* out, const float* rel_pos_h, const float* rel_pos_w,
                                    int32_t nseq, int32_t side, int32_t heads, int32_t head_dim, int32_t fp16,
                                    int32_t grid, const void* pad_row, void* stream) {
  OCTSAM_CHECK_ARG(qkv && out && rel_pos_h && rel_pos_w && nseq > 0 && heads > 0 && nseq <= 65535,
                   "octsam_vit_attention: bad args");
  OCTSAM_CHECK_ARG(head_dim == 64 || head_dim == 80, "octsam_vit_attention: head_dim must be 64 or 80 (got %d)",
                   head_dim);
  OCTSAM_CHECK_ARG(side == 64 || side == 14, "octsam_vit_attention: side must be 64 (global) or 14 (window), got %d",
                   side);
  OCTSAM_CHECK_ARG(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)rel_pos_h & 15) == 0 &&
                       ((uintptr_t)rel_pos_w & 15) == 0,
                   "octsam_vit_attention: operands must be 16-B aligned");
  OCTSAM_CHECK_ARG(grid == 0 || (side == 14 && grid > 0 && grid <= 4096 && pad_row && ((uintptr_t)pad_row & 15) == 0 &&
                                  nseq % (((grid + 13) / 14) * ((grid + 13) / 14)) == 0),
                   "octsam_vit_attention: token-ordered windows need side 14, nseq = images * windows and an aligned "
                   "pad row");
  hipStream_t s = (hipStream_t)stream;
  if (head_dim == 64)
    fp16 ? launch<64, f16>(qkv, out, rel_pos_h, rel_pos_w, nseq, side, heads, grid, pad_row, s)
         : launch<64, bf16>(qkv, out, rel_pos_h, rel_pos_w, nseq, side, heads, grid, pad_row, s);
  else
    fp16 ? launch<80, f16>(qkv, out, rel_pos_h, rel_pos_w, nseq, side, heads, grid, pad_row, s)
         : launch<80, bf16>(qkv, out, rel_pos_h, rel_pos_w, nseq, side, heads, grid, pad_row, s);
  OCTSAM_LAUNCH_CHECK("octsam_vit_attention");
  return 0;
}

extern "C" void octsam_attention_set_variant(int32_t variant) { g_attn_variant = variant; }
