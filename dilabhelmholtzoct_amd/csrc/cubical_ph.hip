// Sublevel-set cubical persistence (H0 and H1) of small 2-D maps, one workgroup per map.
//
// Replaces torch_topological.nn.CubicalComplex(dim=2, superlevel=False) -> gudhi CubicalComplex
// .persistence() + .cofaces_of_persistence_pairs() (ref:octsam/models/topological_loss.py:55-63).
// Bit-exact target: oracle/cubical_ph.c (same total order, same coface rule, same pair order).
//
// Per map:
//   1. pixels -> LDS; edge keys (ordered value bits << 32 | bitmap position) built in parallel and
//      bitonic-sorted in LDS (gudhi's is_before_in_filtration among 1-cells).
//   2. wave 0: H1 as the Alexander-dual union-find over pixels + exterior, edges in DECREASING
//      order; wave 1: H0 union-find over vertices, edges in INCREASING order. Both run the elder
//      rule in 64-edge chunks: every lane finds the roots of its own edge against the state at the
//      chunk start (parallel, path halving), then a wave-uniform loop over the 64 edges resolves
//      the merges in order with v_readlane broadcasts and whole-wave relabelling, so each edge costs
//      a few scalar/VALU ops instead of a chain of dependent LDS round trips. The chunk's links are
//      written back to the LDS forest after the loop.
//   3. essential H0 class + argmax (torch_topological's fake destroyer), top-dimensional cofaces,
//      pairs ranked by (persistence desc, destroyer filtration order) and written out.
#include "common.h"
#include "../../include/octsam.h"

namespace {

constexpr int NTHR = 512;
constexpr int MAX_PIX = 4096;
constexpr int MAX_EDGES_POW2 = 8192;
constexpr int MAX_VERT = 4225;  // (64+1)^2
constexpr int REC_CAP = 1024;

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

__device__ __forceinline__ int uf_find(int* parent, int a) {
  int p = parent[a];
  while (p != a) {
    int gp = parent[p];
    parent[a] = gp;  // path halving; concurrent writers only ever store an ancestor
    a = gp;
    p = parent[a];
  }
  return a;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

struct Smem {
  uint64_t keys[MAX_EDGES_POW2];
  float vals[MAX_PIX];
  int vpar[MAX_VERT];
  int ppar[MAX_PIX + 1];
  uint64_t rec_key[2][REC_CAP];
  int rec_c[2][REC_CAP];
  int nrec[2];
  int overflow;
  float red_v[NTHR / 64];
  int red_i[NTHR / 64];
};

// Key of a union-find node. H1 nodes: pixels (key = value bits, pixel idx), exterior = +inf.
__device__ __forceinline__ uint64_t pix_key(const Smem& s, int W, int node, int ext) {
  return node == ext ? ~0ull : (((uint64_t)ord_bits(s.vals[node]) << 32) | (uint32_t)node);
}
// H0 nodes: vertices indexed by vertex id (vy*(W+1)+vx); key = (value bits, bitmap position).
__device__ __forceinline__ uint64_t vert_key(const Map& m, int vid) {
  int vx = vid % (m.W + 1), vy = vid / (m.W + 1);
  int pos = 2 * vx + m.W2 * (2 * vy);
  return ((uint64_t)ord_bits(cell_value(m, pos)) << 32) | (uint32_t)pos;
}

__device__ void h1_wave(Smem& s, const Map& m, int ne) {
  const int lane = threadIdx.x & 63;
  const int ext = m.H * m.W;
  int cnt = 0;
  for (int base = 0; base < ne; base += 64) {
    const int idx = ne - 1 - (base + lane);  // decreasing filtration order
    const bool valid = idx >= 0;
    uint64_t ek = valid ? s.keys[idx] : 0;
    int pos = (int)(uint32_t)ek;
    int a = ext, c = ext;
    if (valid) {
      int X = pos % m.W2, Y = pos / m.W2;
      if (X & 1) {
        int col = X >> 1;
        a = (Y > 0) ? ((Y >> 1) - 1) * m.W + col : ext;
        c = (Y < m.H2 - 1) ? (Y >> 1) * m.W + col : ext;
      } else {
        int row = Y >> 1;
        a = (X > 0) ? row * m.W + (X >> 1) - 1 : ext;
        c = (X < m.W2 - 1) ? row * m.W + (X >> 1) : ext;
      }
    }
    int ra = valid ? uf_find(s.ppar, a) : ext;
    int rc = valid ? uf_find(s.ppar, c) : ext;
    uint64_t ka = pix_key(s, m.W, ra, ext), kc = pix_key(s, m.W, rc, ext);
    int my_young = -1, my_old = -1;
    const int nvalid = min(64, ne - base);
    for (int j = 0; j < nvalid; ++j) {
      int sa = __builtin_amdgcn_readlane(ra, j);
      int sc = __builtin_amdgcn_readlane(rc, j);
      if (sa == sc) continue;
      uint64_t kka = readlane64(ka, j), kkc = readlane64(kc, j);
      int young, old;
      uint64_t kold;
      if (kka < kkc) { young = sa; old = sc; kold = kkc; } else { young = sc; old = sa; kold = kka; }
      if (ra == young) { ra = old; ka = kold; }
      if (rc == young) { rc = old; kc = kold; }
      if (lane == j) { my_young = young; my_old = old; }
      // persistence > 0 ?  death value (young pixel) > edge value
      uint64_t ekj = readlane64(ek, j);
      float dv = s.vals[young];
      float ev = unord_bits((uint32_t)(ekj >> 32));
      if (dv > ev) {
        if (lane == j) {
          if (cnt < REC_CAP) {
            s.rec_key[1][cnt] = ((uint64_t)ord_bits(dv) << 32) | (uint32_t)young;
            s.rec_c[1][cnt] = top_coface(m, pos);
          }
        }
        ++cnt;
      }
    }
    if (my_young >= 0) s.ppar[my_young] = my_old;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  if (lane == 0) {
    s.nrec[1] = min(cnt, REC_CAP);
    if (cnt > REC_CAP) s.overflow |= 2;
  }
}

__device__ void h0_wave(Smem& s, const Map& m, int ne) {
  const int lane = threadIdx.x & 63;
  int cnt = 0;
  for (int base = 0; base < ne; base += 64) {
    const int idx = base + lane;  // increasing filtration order
    const bool valid = idx < ne;
    uint64_t ek = valid ? s.keys[idx] : 0;
    int pos = (int)(uint32_t)ek;
    int u = 0, v = 0;
    if (valid) {
      int X = pos % m.W2;
      int pu, pv;
      if (X & 1) { pu = pos - 1; pv = pos + 1; } else { pu = pos - m.W2; pv = pos + m.W2; }
      u = (pu % m.W2) / 2 + (m.W + 1) * ((pu / m.W2) / 2);
      v = (pv % m.W2) / 2 + (m.W + 1) * ((pv / m.W2) / 2);
    }
    int ru = valid ? uf_find(s.vpar, u) : 0;
    int rv = valid ? uf_find(s.vpar, v) : 0;
    uint64_t ku = vert_key(m, ru), kv = vert_key(m, rv);
    int my_young = -1, my_old = -1;
    const int nvalid = min(64, ne - base);
    for (int j = 0; j < nvalid; ++j) {
      int su = __builtin_amdgcn_readlane(ru, j);
      int sv = __builtin_amdgcn_readlane(rv, j);
      if (su == sv) continue;
      uint64_t kku = readlane64(ku, j), kkv = readlane64(kv, j);
      int young, old;
      uint64_t kold, kyoung;
      if (kku > kkv) { young = su; old = sv; kold = kkv; kyoung = kku; }
      else { young = sv; old = su; kold = kku; kyoung = kkv; }
      if (ru == young) { ru = old; ku = kold; }
      if (rv == young) { rv = old; kv = kold; }
      if (lane == j) { my_young = young; my_old = old; }
      uint64_t ekj = readlane64(ek, j);
      float bv = unord_bits((uint32_t)(kyoung >> 32));
      float ev = unord_bits((uint32_t)(ekj >> 32));
      if (ev > bv) {
        if (lane == j) {
          if (cnt < REC_CAP) {
            s.rec_key[0][cnt] = ekj;
            s.rec_c[0][cnt] = top_coface(m, (int)(uint32_t)kyoung);
          }
        }
        ++cnt;
      }
    }
    if (my_young >= 0) s.vpar[my_young] = my_old;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  if (lane == 0) {
    s.nrec[0] = min(cnt, REC_CAP);
    if (cnt > REC_CAP) s.overflow |= 1;
  }
}

__global__ __launch_bounds__(NTHR) void cubical_ph_kernel(const float* __restrict__ maps, int H, int W, int max_pairs,
                                                          int* pairs0, int* pairs1, int* essential, int* counts) {
  __shared__ Smem s;
  const int tid = threadIdx.x;
  const int map = blockIdx.x;
  const int npix = H * W;
  Map m{H, W, 2 * W + 1, 2 * H + 1, s.vals};
  const float* src = maps + (long long)map * npix;
  for (int i = tid; i < npix; i += NTHR) s.vals[i] = src[i];
  const int nh = (H + 1) * W, nvrt = H * (W + 1), ne = nh + nvrt;
  int np2 = 1;
  while (np2 < ne) np2 <<= 1;
  if (tid == 0) { s.overflow = 0; }
  __syncthreads();
  for (int i = tid; i < np2; i += NTHR) {
    uint64_t k = ~0ull;
    if (i < ne) {
      int X, Y;
      if (i < nh) { Y = 2 * (i / W); X = 2 * (i % W) + 1; }
      else { int j = i - nh; Y = 2 * (j / (W + 1)) + 1; X = 2 * (j % (W + 1)); }
      int pos = X + m.W2 * Y;
      k = ((uint64_t)ord_bits(cell_value(m, pos)) << 32) | (uint32_t)pos;
    }
    s.keys[i] = k;
  }
  for (int i = tid; i < (H + 1) * (W + 1); i += NTHR) s.vpar[i] = i;
  for (int i = tid; i <= npix; i += NTHR) s.ppar[i] = i;
  __syncthreads();
  // bitonic sort ascending
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += NTHR) {
        int l = i ^ j;
        if (l > i) {
          uint64_t a = s.keys[i], b = s.keys[l];
          bool up = (i & k) == 0;
          if ((a > b) == up) { s.keys[i] = b; s.keys[l] = a; }
        }
      }
      __syncthreads();
    }
  }
  const int wave = tid >> 6;
  if (wave == 0) h1_wave(s, m, ne);
  else if (wave == 1) h0_wave(s, m, ne);
  __syncthreads();

  // essential class root (oldest vertex) and argmax pixel (first maximum) by block reduction.
  if (wave == 2 || wave == 3) {
    // nothing: handled below by all threads
  }
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
  __syncthreads();
  if (tid == 0) {
    float v = s.red_v[0];
    int ii = s.red_i[0];
    for (int w = 1; w < NTHR / 64; ++w)
      if (s.red_v[w] > v || (s.red_v[w] == v && s.red_i[w] < ii)) { v = s.red_v[w]; ii = s.red_i[w]; }
    int root = uf_find(s.vpar, 0);
    int vx = root % (W + 1), vy = root / (W + 1);
    essential[2 * map] = top_coface(m, 2 * vx + m.W2 * 2 * vy);
    essential[2 * map + 1] = ii;
    counts[3 * map + 0] = min(s.nrec[0], max_pairs);
    counts[3 * map + 1] = min(s.nrec[1], max_pairs);
    counts[3 * map + 2] = (s.overflow || s.nrec[0] > max_pairs || s.nrec[1] > max_pairs) ? 1 : 0;
  }
  // rank pairs: (persistence desc, destroyer key asc); persistence in double like gudhi
  for (int d = 0; d < 2; ++d) {
    const int n = s.nrec[d];
    int* out = d == 0 ? pairs0 : pairs1;
    for (int i = tid; i < n; i += NTHR) {
      uint64_t ki = s.rec_key[d][i];
      int ci = s.rec_c[d][i];
      double pi = (double)unord_bits((uint32_t)(ki >> 32)) - (double)s.vals[ci];
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        uint64_t kj = s.rec_key[d][j];
        double pj = (double)unord_bits((uint32_t)(kj >> 32)) - (double)s.vals[s.rec_c[d][j]];
        rank += (pj > pi) || (pj == pi && kj < ki);
      }
      if (rank < max_pairs) {
        int dpix;
        int pos = (int)(uint32_t)ki;
        if (d == 1) dpix = pos;  // H1 records store the destroyer pixel index directly
        else dpix = top_coface(m, pos);
        long long o = ((long long)map * max_pairs + rank) * 2;
        out[o] = ci;
        out[o + 1] = dpix;
      }
    }
  }
}

}  // namespace

extern "C" int octsam_cubical_ph(const float* maps, int32_t nmaps, int32_t H, int32_t W, int32_t max_pairs,
                                 int32_t* pairs0, int32_t* pairs1, int32_t* essential, int32_t* counts,
                                 void* stream) {
  OCTSAM_CHECK_ARG(maps && pairs0 && pairs1 && essential && counts, "octsam_cubical_ph: null pointer");
  OCTSAM_CHECK_ARG(nmaps >= 0 && H >= 1 && W >= 1 && max_pairs >= 1, "octsam_cubical_ph: bad sizes");
  OCTSAM_CHECK_ARG(H * W <= MAX_PIX && H <= 64 && W <= 64, "octsam_cubical_ph: map %dx%d too large (<=64x64)", H, W);
  OCTSAM_CHECK_ARG((H + 1) * W + H * (W + 1) <= MAX_EDGES_POW2, "octsam_cubical_ph: too many edges");
  if (nmaps == 0) return 0;
  hipLaunchKernelGGL(cubical_ph_kernel, dim3(nmaps), dim3(NTHR), 0, (hipStream_t)stream, maps, H, W, max_pairs,
                     pairs0, pairs1, essential, counts);
  OCTSAM_LAUNCH_CHECK("octsam_cubical_ph");
  return 0;
}
