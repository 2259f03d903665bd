// Sublevel-set cubical persistence (H0 and H1) of small 2-D maps, one workgroup per map.
//
// Replaces torch_topological.nn.CubicalComplex(dim=2, superlevel=False) -> gudhi CubicalComplex
// .persistence() + .cofaces_of_persistence_pairs() (ref:octsam/models/topological_loss.py:55-63).
// Bit-exact target: oracle/cubical_ph.c (same total order, same coface rule, same pair order).
//
// Per map (one 512-thread workgroup, everything in LDS):
//   1. node filtration order: vertices (lower-star value, bitmap position) and pixels (value, index) in
//      one bitonic sort; nodes are renumbered by rank, so "younger" is an integer comparison.
//   2. edge (1-cell) order: (lower-star value, bitmap position) -- gudhi's is_before_in_filtration among
//      1-cells -- bitonic sort (every thread issues all its compare-exchange loads of a stage at once).
//   3. wave 0: H1 as the Alexander-dual union-find over pixels + exterior, edges in DECREASING order;
//      wave 1: H0 union-find over vertices, edges in INCREASING order. Elder rule in 64-edge chunks:
//      lanes find their edge's roots against the chunk-start forest in parallel; a wave-uniform loop
//      resolves the chunk's edges in order (two v_readlane, min/max, whole-wave relabel, lane-j select);
//      merges are logged with ballot compaction.
//   4. in parallel: positive-persistence merges -> pairs, essential H0 class + argmax (torch_topological's
//      fake destroyer), top-dimensional cofaces, pairs ranked by (persistence desc, destroyer order).
#include "common.h"
#include "../../include/octsam.h"

namespace {

#ifdef PH_PROFILE  // phase timestamps (scripts/micro/ph_timing.hip only)
__device__ unsigned long long g_ph_stamp[64];
#define PH_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_ph_stamp[k] = __builtin_readcyclecounter()
#define PH_STAMP_W(k) \
  if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) g_ph_stamp[k] = __builtin_readcyclecounter()
#else
#define PH_STAMP(k)
#define PH_STAMP_W(k)
#endif

constexpr int NTHR = 512;
constexpr int MAX_PIX = 4096;

struct Map {
  int H, W, W2, H2;
  const float* v;  // LDS pixel values
};

__device__ __forceinline__ uint32_t ord_bits(float v) {
  if (v == 0.0f) v = 0.0f;  // -0 == +0 in gudhi's comparisons
  uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}

__device__ float cell_value(const Map& m, int p) {
  int X = p % m.W2, Y = p / m.W2;
  float best = INFINITY;
  int y0 = (Y & 1) ? Y : Y - 1, y1 = (Y & 1) ? Y : Y + 1;
  int x0 = (X & 1) ? X : X - 1, x1 = (X & 1) ? X : X + 1;
  for (int YY = y0; YY <= y1; YY += 2) {
    if (YY < 0 || YY >= m.H2) continue;
    for (int XX = x0; XX <= x1; XX += 2) {
      if (XX < 0 || XX >= m.W2) continue;
      best = fminf(best, m.v[(YY >> 1) * m.W + (XX >> 1)]);
    }
  }
  return best;
}

// gudhi get_top_dimensional_coface_of_a_cell -> pixel index
__device__ int top_coface(const Map& m, int p) {
  for (int guard = 0; guard < 4; ++guard) {
    int X = p % m.W2, Y = p / m.W2;
    if ((X & 1) && (Y & 1)) return (Y >> 1) * m.W + (X >> 1);
    float v = cell_value(m, p);
    int next = -1;
    if (!(Y & 1)) {
      if (Y > 0 && cell_value(m, p - m.W2) == v) next = p - m.W2;
      else if (Y < m.H2 - 1 && cell_value(m, p + m.W2) == v) next = p + m.W2;
    }
    if (next < 0 && !(X & 1)) {
      if (X > 0 && cell_value(m, p - 1) == v) next = p - 1;
      else if (X < m.W2 - 1 && cell_value(m, p + 1) == v) next = p + 1;
    }
    if (next < 0) return -1;
    p = next;
  }
  return -1;
}

typedef uint16_t u16;

__device__ __forceinline__ int uf_find(u16* parent, int a) {
  int p = parent[a];
  while (p != a) {
    int gp = parent[p];
    parent[a] = (u16)gp;  // path halving; concurrent writers only ever store an ancestor
    a = gp;
    p = parent[a];
  }
  return a;
}

constexpr int NP2 = 8192;        // sort width (edges; vertices + pixels)
constexpr int MAXN = 4352;       // node arrays (vertices, pixels + exterior), u16
// Record capacities of the positive-persistence merges, per dimension, from the map size bound (<= 63x63):
//   H0 pairs are born at regional minima (8-connected plateaus), pairwise non-8-adjacent: <= ceil(H/2)ceil(W/2) <= 1024
//   H1 pairs die at regional maxima (4-connected plateaus), pairwise non-4-adjacent:     <= ceil(H*W/2)      <= 1985
// so no map of an accepted size can overflow (a 50x50 checkerboard has 1152 H1 pairs).
constexpr int REC0 = 1024;
constexpr int REC1 = 2048;
__device__ __forceinline__ int rec_base(int d) { return d ? REC0 : 0; }
__device__ __forceinline__ int rec_cap(int d) { return d ? REC1 : REC0; }

struct Smem {
  uint64_t keys[NP2];  // sort buffer; after the edge sort: epos u32[NP2] | merge logs u32[nv] | u32[npix]
  float vals[MAX_PIX];
  union {
    struct {
      u16 par[2][MAXN];  // union-find forests over filtration ranks: [0] vertices (H0), [1] pixels + ext (H1)
      u16 vrank[MAXN];   // vertex id -> rank
      u16 prank[MAXN];   // pixel -> rank
    } uf;
    struct {  // dimension d's records at [rec_base(d), rec_base(d) + rec_cap(d))
      uint64_t key[REC0 + REC1];  // destroyer key (value bits << 32 | position / pixel)
      int c[REC0 + REC1];         // creator: cell position, then top-coface pixel
      double pers[REC0 + REC1];   // persistence (death - birth value, in double like gudhi), computed once
    } rec;
  } u;
  u16 vinv[MAXN];  // rank -> vertex id
  u16 pinv[MAXN];  // rank -> pixel
  int nlog[2], nrec[2];
  int overflow;
  float red_v[NTHR / 64];
  int red_i[NTHR / 64];
};

// bitonic sort of NP2 64-bit keys, ascending; every thread owns NP2/2/NTHR compare-exchange pairs per
// stage and issues all their loads before any store (one LDS latency per stage, not one per pair).
// Stages whose partner distance j is below a wave's chunk (NP2 / waves keys) stay inside that chunk, so
// each wave runs them on its own chunk with only a wave-level ordering point; the workgroup barrier is
// needed only around the stages with j >= chunk (6 of the 91 at NP2 = 8192).
__device__ void sort_keys(uint64_t* keys, int tid) {
  constexpr int PP = NP2 / 2 / NTHR;
  constexpr int NWAVE = NTHR / 64, CHUNK = NP2 / NWAVE;
  const int lane = tid & 63, wave = tid >> 6;
  bool wave_phase = false;  // the previous stage ran wave-locally (a workgroup barrier is owed)
  for (int k = 2; k <= NP2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const bool local = j < CHUNK;
      if (!local && wave_phase) __syncthreads();
      uint64_t a[PP], b[PP];
      int ia[PP];
#pragma unroll
      for (int t = 0; t < PP; ++t) {
        int i;
        if (local) {  // pair q of this wave's chunk
          const int q = lane + t * 64;
          i = wave * CHUNK + (((q & ~(j - 1)) << 1) | (q & (j - 1)));
        } else {
          const int q = tid + t * NTHR;
          i = ((q & ~(j - 1)) << 1) | (q & (j - 1));
        }
        ia[t] = i;
        a[t] = keys[i];
        b[t] = keys[i | j];
      }
#pragma unroll
      for (int t = 0; t < PP; ++t) {
        const bool up = (ia[t] & k) == 0;
        const bool sw = (a[t] > b[t]) == up;
        const uint64_t lo = sw ? b[t] : a[t], hi = sw ? a[t] : b[t];
        keys[ia[t]] = lo;
        keys[ia[t] | j] = hi;
      }
      if (local) {
        // the wave's own stores are visible to its next loads (LDS keeps a wave's accesses in order); keep
        // the compiler from moving loads above them
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        wave_phase = true;
      } else {
        __syncthreads();
        wave_phase = false;
      }
    }
  }
  if (wave_phase) __syncthreads();
}

// Stable LSD radix sort (4-bit digits) of n <= NTHR * CMAX elements in LDS, ping-ponging between a and b; the
// digits are bits [shift, shift + nbits) of each element (nbits % 4 == 0). Thread t owns the contiguous chunk
// [t C, t C + C) (C = ceil(n / NTHR)) and the digit table (u16, 16 digits x NTHR threads, digit-major) is scanned in
// that order, so equal digits keep their input order: stability makes a sort by value alone over position-ordered
// input equal to the (value, position) sort of the bitonic form. Returns the buffer holding the result.
// (Replaces two 8192-wide bitonic sorts: 415k of the kernel's 1.39M cycles, scripts/micro/ph_timing.hip.)
template <typename T, int CMAX>
__device__ T* radix_sort(T* a, T* b, int n, int shift, int nbits, uint16_t* tab, int* wtot, int tid) {
  const int C = (n + NTHR - 1) / NTHR;
  const int lo = min(n, tid * C), hi = min(n, lo + C);
  const int lane = tid & 63, wave = tid >> 6;
  for (int sh = shift; sh < shift + nbits; sh += 4) {
    T v[CMAX];
    uint64_t c0 = 0, c1 = 0;  // 8-bit per-digit counters (C <= 16)
#pragma unroll
    for (int k = 0; k < CMAX; ++k) {
      if (k < C && lo + k < hi) {
        v[k] = a[lo + k];
        const int d = (int)(v[k] >> sh) & 15;
        if (d < 8) c0 += 1ull << (8 * d);
        else c1 += 1ull << (8 * (d - 8));
      }
    }
#pragma unroll
    for (int d = 0; d < 16; ++d) tab[d * NTHR + tid] = (uint16_t)(((d < 8 ? c0 >> (8 * d) : c1 >> (8 * (d - 8)))) & 0xff);
    __syncthreads();
    // exclusive scan of the 16 * NTHR counts in digit-major order: thread t takes entries [16 t, 16 t + 16)
    uint32_t e[16];
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      e[j] = run;
      run += tab[16 * tid + j];
    }
    uint32_t incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(incl, o, 64);
      if (lane >= o) incl += x;
    }
    if (lane == 63) wtot[wave] = (int)incl;
    __syncthreads();
    uint32_t base = incl - run;
    for (int w = 0; w < wave; ++w) base += (uint32_t)wtot[w];
#pragma unroll
    for (int j = 0; j < 16; ++j) tab[16 * tid + j] = (uint16_t)(base + e[j]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CMAX; ++k) {
      if (k < C && lo + k < hi) {
        const int d = (int)(v[k] >> sh) & 15;
        const int pos = tab[d * NTHR + tid];
        tab[d * NTHR + tid] = (uint16_t)(pos + 1);
        b[pos] = v[k];
      }
    }
    __syncthreads();
    T* t = a;
    a = b;
    b = t;
  }
  return a;
}

// inclusive block scan of one int per thread (tid order)
__device__ __forceinline__ int block_scan_incl(int x, int* wtot, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wtot[wave] = x;
  __syncthreads();
  for (int w = 0; w < wave; ++w) x += wtot[w];
  __syncthreads();
  return x;
}

// vertex id <-> bitmap position
__device__ __forceinline__ int vert_pos(const Map& m, int vid) { return 2 * (vid % (m.W + 1)) + m.W2 * 2 * (vid / (m.W + 1)); }
__device__ __forceinline__ int pos_vert(const Map& m, int pos) { return (pos % m.W2) / 2 + (m.W + 1) * ((pos / m.W2) / 2); }

// one pending edge J of a chunk: its current roots from the flattened root registers (lanes 2J', 2J' + 1, J' = J
// mod 32, of A for J < 32, of B above), the merge (younger root -> older root) relabelled in every lane of the
// registers still holding unresolved edges (BOTH: A and B; else the one J is in), young | old << 16 written into
// lane J of rec. J is a compile-time constant so every lane select is an immediate (v_writelane's too: lanes
// 0-63 are inline constants, which leave its scalar data operand the one constant-bus read).
template <int DIM, bool BOTH, int J>
__device__ __forceinline__ void uf_edge(int& A, int& B, int& rec) {
  constexpr int L = 2 * (J & 31);
  int& R = J < 32 ? A : B;
  const int sa = __builtin_amdgcn_readlane(R, L);
  const int sc = __builtin_amdgcn_readlane(R, L + 1);
  const int young = DIM == 0 ? max(sa, sc) : min(sa, sc);
  const int old = DIM == 0 ? min(sa, sc) : max(sa, sc);
  R = R == young ? old : R;
  if (BOTH) B = B == young ? old : B;
  int pk;
  asm("s_pack_ll_b32_b16 %0, %1, %2" : "=s"(pk) : "s"(young), "s"(old));
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(rec) : "s"(pk), "i"(J));
}
template <int DIM, bool BOTH, int J0>
__device__ __forceinline__ void uf_edges8(int& A, int& B, int& rec) {
  uf_edge<DIM, BOTH, J0 + 0>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 1>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 2>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 3>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 4>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 5>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 6>(A, B, rec);
  uf_edge<DIM, BOTH, J0 + 7>(A, B, rec);
}

// Elder-rule union-find over filtration RANKS (node id order == filtration order, so "younger" is an
// integer comparison), 64 edges per chunk: lanes find their edge's roots against the chunk-start state in
// parallel, then a wave-uniform loop resolves the 64 edges in order (readlane the two roots, min/max,
// relabel every lane's roots, keep the merge in lane j). Merges are logged with ballot compaction
// as (young rank << 13 | sorted edge index); filtering by positive persistence happens afterwards.
// dim 0: vertices, edges increasing, younger = larger rank. dim 1: Alexander dual over pixels + exterior
// (rank npix = +inf), edges decreasing, younger = smaller rank.
template <int DIM>
__device__ void uf_wave(Smem& s, const Map& m, int ne, int npix) {
  const int lane = threadIdx.x & 63;
  const uint32_t* epos = (const uint32_t*)s.keys;
  uint32_t* log = (uint32_t*)s.keys + NP2 + DIM * (m.H + 1) * (m.W + 1);  // H0 log <= nv-1, H1 log <= npix
  u16* par = s.u.uf.par[DIM];
  // pending-edge scratch (3 x 64 ints per wave) past the union-find arrays (free until the pair records)
  int* cs = (int*)((char*)&s.u + sizeof(s.u.uf)) + DIM * 192;
  int cnt = 0;
#ifdef PH_PROFILE
  unsigned long long t_find = 0, t_res = 0, t0 = __builtin_readcyclecounter();
#endif
  for (int base = 0; base < ne; base += 64) {
    const int idx = DIM == 0 ? base + lane : ne - 1 - (base + lane);
    const bool valid = base + lane < ne;
    int ru = 0, rv = 0;
    if (valid) {
      const int pos = (int)epos[idx];
      const int X = pos % m.W2, Y = pos / m.W2;
      if (DIM == 0) {
        const int pu = (X & 1) ? pos - 1 : pos - m.W2, pv = (X & 1) ? pos + 1 : pos + m.W2;
        ru = s.u.uf.vrank[pos_vert(m, pu)];
        rv = s.u.uf.vrank[pos_vert(m, pv)];
      } else {
        int a, c;
        if (X & 1) {
          const int col = X >> 1;
          a = (Y > 0) ? ((Y >> 1) - 1) * m.W + col : -1;
          c = (Y < m.H2 - 1) ? (Y >> 1) * m.W + col : -1;
        } else {
          const int row = Y >> 1;
          a = (X > 0) ? row * m.W + (X >> 1) - 1 : -1;
          c = (X < m.W2 - 1) ? row * m.W + (X >> 1) : -1;
        }
        ru = a < 0 ? npix : s.u.uf.prank[a];
        rv = c < 0 ? npix : s.u.uf.prank[c];
      }
      // both finds walk together (two independent LDS latency chains per step); path halving on the way, then
      // the edge's own nodes point straight at their roots
      const int nu = ru, nv = rv;
      int pu = par[ru], pv = par[rv];
      while (pu != ru || pv != rv) {
        const int gu = par[pu], gv = par[pv];
        if (pu != ru) par[ru] = (u16)gu;
        if (pv != rv) par[rv] = (u16)gv;
        ru = gu;
        rv = gv;
        pu = par[ru];
        pv = par[rv];
      }
      if (nu != ru) par[nu] = (u16)ru;
      if (nv != rv) par[nv] = (u16)rv;
    }
    // Only the edges whose roots differ at the chunk start can merge: relabelling maps both roots of an edge through
    // the same function, so roots that agree keep agreeing (and such an edge is not recorded). Those edges are
    // compacted in edge order through this wave's LDS scratch, their roots flattened edge-major (edge j's at lanes
    // 2j, 2j + 1 of A for j < 32, of B above; zeros past them are no-op pairs), and the wave-uniform loop resolves
    // only them, 8 at a time. Edges past the first 32 relabel B alone. (Per pending edge: 2 readlanes, scalar
    // min/max, 2-4 VALU relabel, one writelane of young | old << 16 into the edge's lane; a compare-and-select
    // record over both roots in every lane, and an s_ff1 walk over the pending mask, measured slower.)
#ifdef PH_PROFILE
    { const unsigned long long t1 = __builtin_readcyclecounter(); t_find += t1 - t0; t0 = t1; }
#endif
    const bool pend = ru != rv;  // (invalid tail lanes hold ru == rv == 0)
    const uint64_t pm = __builtin_amdgcn_ballot_w64(pend);
    const int np = __builtin_popcountll(pm);
    if (pend) {
      const int p = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0));
      cs[2 * p] = ru;
      cs[2 * p + 1] = rv;
      cs[128 + p] = idx;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int A = lane < 2 * np ? cs[lane] : 0;
    int B = lane + 64 < 2 * np ? cs[64 + lane] : 0;
    const int cidx = lane < np ? cs[128 + lane] : 0;
    int rec = 0;
    // edges past np hold zero roots (no-op merges); groups of 8 up to np, B relabelled only while it holds edges
    if (np <= 32) {
      if (np > 0) uf_edges8<DIM, false, 0>(A, B, rec);
      if (np > 8) uf_edges8<DIM, false, 8>(A, B, rec);
      if (np > 16) uf_edges8<DIM, false, 16>(A, B, rec);
      if (np > 24) uf_edges8<DIM, false, 24>(A, B, rec);
    } else {
      uf_edges8<DIM, true, 0>(A, B, rec);
      uf_edges8<DIM, true, 8>(A, B, rec);
      uf_edges8<DIM, true, 16>(A, B, rec);
      uf_edges8<DIM, true, 24>(A, B, rec);
      uf_edges8<DIM, false, 32>(A, B, rec);
      if (np > 40) uf_edges8<DIM, false, 40>(A, B, rec);
      if (np > 48) uf_edges8<DIM, false, 48>(A, B, rec);
      if (np > 56) uf_edges8<DIM, false, 56>(A, B, rec);
    }
    const int my_young = rec & 0xffff, my_old = rec >> 16;
    const bool merged = my_young != my_old;  // (lanes past np hold rec == 0)
    if (merged) par[my_young] = (u16)my_old;
    const uint64_t mask = __builtin_amdgcn_ballot_w64(merged);
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (merged) log[cnt + below] = ((uint32_t)my_young << 13) | (uint32_t)cidx;
    cnt += __builtin_popcountll(mask);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#ifdef PH_PROFILE
    { const unsigned long long t1 = __builtin_readcyclecounter(); t_res += t1 - t0; t0 = t1; }
#endif
  }
  if (lane == 0) s.nlog[DIM] = cnt;
#ifdef PH_PROFILE
  if (lane == 0 && blockIdx.x == 0) { g_ph_stamp[16 + 2 * DIM] = t_find; g_ph_stamp[17 + 2 * DIM] = t_res; }
#endif
}

__global__ __launch_bounds__(NTHR) void cubical_ph_kernel(const float* __restrict__ maps, int H, int W, int max_pairs,
                                                          int* pairs0, int* pairs1, int* essential, int* counts) {
  __shared__ Smem s;
  const int tid = threadIdx.x;
  const int map = blockIdx.x;
  const int npix = H * W, nv = (H + 1) * (W + 1);
  Map m{H, W, 2 * W + 1, 2 * H + 1, s.vals};
  const float* src = maps + (long long)map * npix;
  PH_STAMP(0);
  for (int i = tid; i < npix; i += NTHR) s.vals[i] = src[i];
  if (tid == 0) {
    s.overflow = 0;
    s.nrec[0] = s.nrec[1] = 0;
  }
  __syncthreads();
  // radix scratch: the digit table and wave totals sit in the union past the union-find arrays (the pair records
  // that share those bytes are built only after the union-find)
  uint16_t* tab = (uint16_t*)((char*)&s.u + sizeof(s.u.uf));
  int* wtot = (int*)(tab + 16 * NTHR);
  for (int i = tid; i <= npix; i += NTHR) s.u.uf.par[1][i] = (u16)i;
  for (int i = tid; i < nv; i += NTHR) s.u.uf.par[0][i] = (u16)i;
  PH_STAMP(1);
  // 1a. pixel order (value, index): stable radix sort of (ord(value) << 32 | px) over the index-ordered pixels
  uint64_t* kp = s.keys;            // [0, 32 KB)
  uint64_t* kq = s.keys + NP2 / 2;  // [32 KB, 64 KB)
  for (int i = tid; i < npix; i += NTHR) kp[i] = ((uint64_t)ord_bits(s.vals[i]) << 32) | (uint32_t)i;
  __syncthreads();
  const uint64_t* sp = radix_sort<uint64_t, MAX_PIX / NTHR>(kp, kq, npix, 32, 32, tab, wtot, tid);  // 8 passes: kp
  // pixel ranks, and DENSE value ranks (equal values, equal rank; the node and edge values are pixel values, so
  // their orders follow from these 12-bit ranks)
  uint16_t* dr = (uint16_t*)(s.keys + NP2 - MAX_PIX / 4);  // [56 KB, 64 KB): kq is dead
  {
    const int C = (npix + NTHR - 1) / NTHR, lo = min(npix, tid * C), hi = min(npix, lo + C);
    int f = 0;
    for (int i = lo; i < hi; ++i) f += (i > 0 && (sp[i] >> 32) != (sp[i - 1] >> 32)) ? 1 : 0;
    int r = block_scan_incl(f, wtot, tid) - f;  // distinct-value steps before this chunk
    for (int i = lo; i < hi; ++i) {
      r += (i > 0 && (sp[i] >> 32) != (sp[i - 1] >> 32)) ? 1 : 0;
      const int px = (int)(sp[i] & 0xffff);
      dr[px] = (uint16_t)r;
      s.pinv[i] = (u16)px;
      s.u.uf.prank[px] = (u16)i;
    }
  }
  __syncthreads();
  // 1b. vertex order (value, position): vertex ids are position-ordered, so a stable sort by the dense rank of
  //     the vertex's lower-star value (the minimum over its <= 4 pixels) gives it
  uint32_t* va = (uint32_t*)s.keys;          // [0, 17 KB)
  uint32_t* vb = (uint32_t*)s.keys + MAXN;   // [17 KB, 34 KB)
  for (int i = tid; i < nv; i += NTHR) {
    const int vy = i / (W + 1), vx = i - vy * (W + 1);
    int r = 0xffff;
    for (int py = max(vy - 1, 0); py <= min(vy, H - 1); ++py)
      for (int px = max(vx - 1, 0); px <= min(vx, W - 1); ++px) r = min(r, (int)dr[py * W + px]);
    va[i] = ((uint32_t)r << 16) | (uint32_t)i;
  }
  __syncthreads();
  const uint32_t* sv = radix_sort<uint32_t, (MAXN + NTHR - 1) / NTHR>(va, vb, nv, 16, 12, tab, wtot, tid);  // -> vb
  for (int i = tid; i < nv; i += NTHR) {
    const int vid = (int)(sv[i] & 0xffff);
    s.vinv[i] = (u16)vid;
    s.u.uf.vrank[vid] = (u16)i;
  }
  __syncthreads();
  // 2. edge (1-cell) order (value, bitmap position): the edges in raster position order (even rows: the W
  //    horizontal edges at odd X; odd rows: the W + 1 vertical edges at even X), stably sorted by the dense rank
  //    of their lower-star value -> sorted positions epos (u32 at s.keys, as the union-find reads them)
  const int nh = (H + 1) * W, nvrt = H * (W + 1), ne = nh + nvrt;
  uint32_t* ea = (uint32_t*)s.keys;        // [0, 32 KB): the input (dr, at [56 KB, 64 KB), is read meanwhile)
  uint32_t* eb = (uint32_t*)s.keys + NP2;  // [32 KB, 64 KB): 3 passes end here
  for (int i = tid; i < ne; i += NTHR) {
    const int r2 = i / (2 * W + 1), rem = i - r2 * (2 * W + 1);
    int r;
    int pos;
    if (rem < W) {  // horizontal edge: row Y = 2 r2, X = 2 rem + 1; pixels above / below in column rem
      const int Y = 2 * r2, X = 2 * rem + 1;
      pos = X + m.W2 * Y;
      r = 0xffff;
      if (r2 > 0) r = min(r, (int)dr[(r2 - 1) * W + rem]);
      if (r2 < H) r = min(r, (int)dr[r2 * W + rem]);
    } else {  // vertical edge: row Y = 2 r2 + 1, X = 2 (rem - W); pixels left / right in row r2
      const int c = rem - W, Y = 2 * r2 + 1, X = 2 * c;
      pos = X + m.W2 * Y;
      r = 0xffff;
      if (c > 0) r = min(r, (int)dr[r2 * W + c - 1]);
      if (c < W) r = min(r, (int)dr[r2 * W + c]);
    }
    ea[i] = ((uint32_t)r << 14) | (uint32_t)pos;
  }
  __syncthreads();
  const uint32_t* se = radix_sort<uint32_t, NP2 / NTHR>(ea, eb, ne, 14, 12, tab, wtot, tid);  // 3 passes: eb
  for (int i = tid; i < ne; i += NTHR) ea[i] = se[i] & 0x3fff;  // positions to [0, 32 KB); the merge logs follow
  __syncthreads();
  const int wave = tid >> 6;
  PH_STAMP(2);
  if (wave == 0) uf_wave<1>(s, m, ne, npix);
  else if (wave == 1) uf_wave<0>(s, m, ne, npix);
  if (wave == 0) PH_STAMP_W(3);
  if (wave == 1) PH_STAMP_W(4);
  __syncthreads();
  PH_STAMP(5);

  // essential H0 class (root of vertex 0's tree, oldest vertex) and argmax pixel (first maximum)
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = tid; i < npix; i += NTHR) {
    float v = s.vals[i];
    if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if ((tid & 63) == 0) { s.red_v[wave] = bv; s.red_i[wave] = bi; }
  int root_vid = 0;
  if (tid == 0) root_vid = s.vinv[uf_find(s.u.uf.par[0], s.u.uf.vrank[0])];
  __syncthreads();  // the union-find arrays are dead from here: their bytes hold the pair records
  if (tid == 0) {
    float v = s.red_v[0];
    int ii = s.red_i[0];
    for (int w = 1; w < NTHR / 64; ++w)
      if (s.red_v[w] > v || (s.red_v[w] == v && s.red_i[w] < ii)) { v = s.red_v[w]; ii = s.red_i[w]; }
    essential[2 * map] = top_coface(m, vert_pos(m, root_vid));
    essential[2 * map + 1] = ii;
  }
  // 3. keep the merges with positive persistence (death value > birth value) -> records
  const uint32_t* epos = (const uint32_t*)s.keys;
  for (int d = 0; d < 2; ++d) {
    const uint32_t* log = (const uint32_t*)s.keys + NP2 + d * nv;
    const int n = s.nlog[d];
    for (int i = tid; i < n; i += NTHR) {
      const uint32_t e = log[i];
      const int young = (int)(e >> 13), pos = (int)epos[e & 0x1fff];
      const float ev = cell_value(m, pos);
      uint64_t key;
      int cpos;
      bool keep;
      if (d == 0) {  // birth: the young vertex; death: the edge
        const int vpos = vert_pos(m, s.vinv[young]);
        keep = ev > cell_value(m, vpos);
        key = ((uint64_t)ord_bits(ev) << 32) | (uint32_t)pos;
        cpos = vpos;
      } else {       // birth: the edge; death: the young pixel
        const int px = s.pinv[young];
        const float dv = s.vals[px];
        keep = dv > ev;
        key = ((uint64_t)ord_bits(dv) << 32) | (uint32_t)px;
        cpos = pos;
      }
      if (keep) {
        const int r = atomicAdd(&s.nrec[d], 1);
        if (r < rec_cap(d)) {
          s.u.rec.key[rec_base(d) + r] = key;
          s.u.rec.c[rec_base(d) + r] = cpos;
        }
      }
    }
  }
  __syncthreads();
  // creator cells -> top-dimensional cofaces and their values; the high word of each persistence's order-preserving
  // bit image (keys are dead: the records hold what the ranking needs) decides most comparisons of the ranking
  uint32_t* phi = (uint32_t*)s.keys;
  for (int d = 0; d < 2; ++d) {
    const int n = min(s.nrec[d], rec_cap(d)), o = rec_base(d);
    for (int i = tid; i < n; i += NTHR) {
      const int c = top_coface(m, s.u.rec.c[o + i]);
      s.u.rec.c[o + i] = c;
      const double p = (double)unord_bits((uint32_t)(s.u.rec.key[o + i] >> 32)) - (double)s.vals[c];
      s.u.rec.pers[o + i] = p;
      const uint64_t b = (uint64_t)__double_as_longlong(p + 0.0);  // (-0 -> +0: equal values, equal images)
      phi[o + i] = (uint32_t)(((int64_t)b < 0 ? ~b : b | 0x8000000000000000ull) >> 32);
    }
  }
  __syncthreads();
  PH_STAMP(6);
  if (tid == 0) {
    if (s.nrec[0] > REC0) s.overflow |= 1;
    if (s.nrec[1] > REC1) s.overflow |= 2;
    counts[3 * map + 0] = min(s.nrec[0], max_pairs);
    counts[3 * map + 1] = min(s.nrec[1], max_pairs);
    counts[3 * map + 2] = (s.overflow || s.nrec[0] > max_pairs || s.nrec[1] > max_pairs) ? 1 : 0;
  }
  // 4. rank pairs: (persistence desc, destroyer key asc) -- a total order, so the output does not depend on
  //    the record order; persistence in double like gudhi
  for (int d = 0; d < 2; ++d) {
    const int n = min(s.nrec[d], rec_cap(d)), o = rec_base(d);
    int* out = d == 0 ? pairs0 : pairs1;
    for (int i = tid; i < n; i += NTHR) {
      const uint64_t ki = s.u.rec.key[o + i];
      const int ci = s.u.rec.c[o + i];
      const double pi = s.u.rec.pers[o + i];
      const uint32_t hi = phi[o + i];  // >= 2^31 (the image of a non-negative value); 0 marks past-n slots below
      int rank = 0;
      // 8 images per trip, loaded together: distinct images decide (the image order is the persistence order);
      // equal images (ties of the high word: rare but for binary maps) take the exact (persistence, key) compare on
      // a wave-uniform branch
      for (int j0 = 0; j0 < n; j0 += 8) {
        uint32_t hv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) hv[u] = j0 + u < n ? phi[o + j0 + u] : 0u;
        bool tie = false;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          rank += hv[u] > hi;
          tie |= hv[u] == hi;
        }
        if (__builtin_amdgcn_ballot_w64(tie)) {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (hv[u] == hi) {
              const double pj = s.u.rec.pers[o + j0 + u];
              rank += (pj > pi) || (pj == pi && s.u.rec.key[o + j0 + u] < ki);
            }
        }
      }
      if (rank < max_pairs) {
        const int pos = (int)(uint32_t)ki;
        const int dpix = d == 1 ? pos : top_coface(m, pos);  // H1 records hold the destroyer pixel itself
        long long o = ((long long)map * max_pairs + rank) * 2;
        out[o] = ci;
        out[o + 1] = dpix;
      }
    }
  }
  __syncthreads();
  PH_STAMP(7);
}

}  // namespace

extern "C" int octsam_cubical_ph(const float* maps, int32_t nmaps, int32_t H, int32_t W, int32_t max_pairs,
                                 int32_t* pairs0, int32_t* pairs1, int32_t* essential, int32_t* counts,
                                 void* stream) {
  OCTSAM_CHECK_ARG(maps && pairs0 && pairs1 && essential && counts, "octsam_cubical_ph: null pointer");
  OCTSAM_CHECK_ARG(nmaps >= 0 && H >= 1 && W >= 1 && max_pairs >= 1, "octsam_cubical_ph: bad sizes");
  OCTSAM_CHECK_ARG(H * W <= MAX_PIX && (H + 1) * W + H * (W + 1) <= NP2 && (H + 1) * (W + 1) + H * W <= NP2 &&
                       (2 * W + 1) * (2 * H + 1) <= 16384 && (H + 1) * (W + 1) <= MAXN,
                   "octsam_cubical_ph: map %dx%d too large (<= 63x63)", H, W);
  if (nmaps == 0) return 0;
  hipLaunchKernelGGL(cubical_ph_kernel, dim3(nmaps), dim3(NTHR), 0, (hipStream_t)stream, maps, H, W, max_pairs,
                     pairs0, pairs1, essential, counts);
  OCTSAM_LAUNCH_CHECK("octsam_cubical_ph");
  return 0;
}
