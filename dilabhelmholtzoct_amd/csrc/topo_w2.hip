// Device half of the topological loss: exact q-Wasserstein transport between the pred and gt persistence
// diagrams of every map, the per-entry (cost sum)^(1/q), the loss and d loss / d pred-map values — all on the
// GPU, so the training step needs no host round trip between its forward and backward graphs (SURVEY.md
// §8(f)2). Replaces torch_topological.nn.WassersteinDistance(q) -> POT ot.emd2 and the loss assembly of
// ref:octsam/models/topological_loss.py:68-96.
//
// The arithmetic is that of octsam_topo_host (w2_host.cpp) operation for operation, so results are
// bit-identical to it:
//   * cost entries in fp32 (L-inf distance, distance to the diagonal, **q) widened to double; the diagonal-
//     augmented assignment reduced to a rectangular one over the smaller diagram (rows) with one zero-cost
//     "diagonal" column per row, solved in double by the same shortest-augmenting-path Hungarian method;
//   * the column scan of each augmenting step runs on the 64 lanes of one wave (one workgroup per map) and
//     its argmin takes the lowest column index among equal minima — the host loop's first strict minimum;
//   * the transport cost is summed in the host's order by one lane; per entry the costs are summed in map
//     order, rounded to float, and the gradient is scattered into the map's row in LDS with the host's
//     per-pixel addition order (creators, then destroyers): every contribution computed once by its own thread
//     into LDS, a pixel hit several times summed in that order by the thread of its first contribution; the row
//     written out by the workgroup;
//   * no FMA contraction anywhere (the host build has none).
// Bit-identity holds for q = 2 (the call site's loss_q: **2 is one fp32 multiply, the 1/q power a
// correctly rounded sqrt on both sides); other q use pow on both sides (device ocml vs host libm may
// differ in the last bit).
#include "common.h"
#include "../../include/octsam.h"

#pragma clang fp contract(off)

namespace {

constexpr int W2_THREADS = 64;  // one wave per map: the augmenting steps synchronise through LDS only

struct W2Layout {  // per-map scratch (LDS when it fits, else a global workspace slice)
  int cap;         // max diagram points per side (= max_pairs)
  size_t off_v, off_minv, off_u, off_d1, off_d2, off_dg1, off_dg2, off_p, off_way, off_used, bytes;
  __host__ __device__ explicit W2Layout(int c) : cap(c) {
    const size_t ncol = 2 * (size_t)c + 1;  // columns 0..NC with NC <= n + m <= 2 cap
    size_t o = 0;
    off_v = o;    o += ncol * 8;
    off_minv = o; o += ncol * 8;
    off_u = o;    o += ((size_t)c + 1) * 8;
    off_d1 = o;   o += (size_t)c * 8;
    off_d2 = o;   o += (size_t)c * 8;
    off_dg1 = o;  o += (size_t)c * 4;
    off_dg2 = o;  o += (size_t)c * 4;
    off_p = o;    o += ncol * 4;
    off_way = o;  o += ncol * 4;
    off_used = o; o += ncol;
    bytes = (o + 15) & ~(size_t)15;
  }
};

__device__ __forceinline__ float w2_linf(float a0, float a1, float b0, float b1) {
  return fmaxf(fabsf(a0 - b0), fabsf(a1 - b1));
}
__device__ __forceinline__ float w2_diag(float b, float d) {
  const float h = 0.5f * (b + d);
  return fmaxf(fabsf(b - h), fabsf(d - h));
}
__device__ __forceinline__ float w2_powq(float x, double q) {
  return q == 2.0 ? x * x : (float)pow((double)x, q);
}
__device__ __forceinline__ float w2_sgn(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }
__device__ __forceinline__ double w2_root(double t, double q) { return q == 2.0 ? sqrt(t) : pow(t, 1.0 / q); }
// d t^(1/q) / d t (infinite at t = 0, as the host)
__device__ __forceinline__ double w2_droot(double t, double q) {
  if (!(t > 0)) return __builtin_huge_val();
  return q == 2.0 ? 0.5 / sqrt(t) : (1.0 / q) * pow(t, 1.0 / q - 1.0);
}

// The gradient of the transport cost with respect to point i of d1 (matched to d2 point j, or the diagonal).
__device__ __forceinline__ void w2_grad_point(const float* d1, const float* d2, int i, int j, double q, float* g0,
                                              float* g1) {
  const float b = d1[2 * i], d = d1[2 * i + 1];
  if (j >= 0) {
    const float e0 = b - d2[2 * j], e1 = d - d2[2 * j + 1];
    const float M = fmaxf(fabsf(e0), fabsf(e1));
    const float coef = q == 2.0 ? 2.0f * M : (float)(q * pow((double)M, q - 1.0));
    *g0 = coef * (fabsf(e0) == M ? w2_sgn(e0) : 0.0f);
    *g1 = coef * (fabsf(e1) == M ? w2_sgn(e1) : 0.0f);
  } else {
    const float M = w2_diag(b, d);
    const float coef = q == 2.0 ? 2.0f * M : (float)(q * pow((double)M, q - 1.0));
    *g0 = coef * 0.5f * w2_sgn(b - d);
    *g1 = coef * 0.5f * w2_sgn(d - b);
  }
}

// Phase 1: one workgroup (one wave) per map k < Kn: transport cost between pred diagram k and gt diagram
// Kn + k, and the partner (d2 index or -1) of every d1 point.
__global__ void __launch_bounds__(W2_THREADS) w2_map_kernel(const int32_t* __restrict__ pairs,
                                                            const int32_t* __restrict__ cnt,
                                                            const float* __restrict__ vals, int Kn, int max_pairs,
                                                            int nvals, int feat_col, double q, double* __restrict__ costs,
                                                            int32_t* __restrict__ match, int32_t* __restrict__ status,
                                                            char* __restrict__ gscratch, int use_lds) {
  extern __shared__ __align__(16) char w2_smem[];
  const int k = blockIdx.x, lane = threadIdx.x;
  const W2Layout L(max_pairs);
  char* base = use_lds ? w2_smem : gscratch + (size_t)k * L.bytes;
  double* v = (double*)(base + L.off_v);
  double* minv = (double*)(base + L.off_minv);
  double* u = (double*)(base + L.off_u);
  float* d1 = (float*)(base + L.off_d1);
  float* d2 = (float*)(base + L.off_d2);
  float* dg1 = (float*)(base + L.off_dg1);
  float* dg2 = (float*)(base + L.off_dg2);
  int* p = (int*)(base + L.off_p);
  int* way = (int*)(base + L.off_way);
  char* used = base + L.off_used;

  const int n = cnt[k * 3 + feat_col], m = cnt[(Kn + k) * 3 + feat_col];
  int32_t* mk = match + (size_t)k * max_pairs;
  if (n > max_pairs || m > max_pairs || n < 0 || m < 0 || cnt[k * 3 + 2] || cnt[(Kn + k) * 3 + 2]) {
    if (lane == 0) {
      status[0] = 1;  // pair-buffer overflow: the loss kernel writes NaN
      costs[k] = 0.0;
    }
    for (int i = lane; i < max_pairs; i += W2_THREADS) mk[i] = -1;
    return;
  }
  const int32_t* p1 = pairs + (size_t)k * max_pairs * 2;
  const int32_t* p2 = pairs + (size_t)(Kn + k) * max_pairs * 2;
  const float* v1 = vals + (size_t)k * nvals;
  const float* v2 = vals + (size_t)(Kn + k) * nvals;
  for (int i = lane; i < n; i += W2_THREADS) {
    const float b = v1[p1[2 * i]], d = v1[p1[2 * i + 1]];
    d1[2 * i] = b;
    d1[2 * i + 1] = d;
    dg1[i] = w2_powq(w2_diag(b, d), q);
    mk[i] = -1;
  }
  for (int j = lane; j < m; j += W2_THREADS) {
    const float b = v2[p2[2 * j]], d = v2[p2[2 * j + 1]];
    d2[2 * j] = b;
    d2[2 * j + 1] = d;
    dg2[j] = w2_powq(w2_diag(b, d), q);
  }
  const bool rows_d2 = m <= n;
  const int R = rows_d2 ? m : n, Cc = rows_d2 ? n : m, NC = Cc + R;
  for (int j = lane; j <= NC; j += W2_THREADS) {
    v[j] = 0.0;
    p[j] = 0;
    way[j] = 0;
  }
  for (int i = lane; i <= R; i += W2_THREADS) u[i] = 0.0;
  __syncthreads();

  // reduced cost of row r (0-based), column c (0-based): C_ij - dg1_i - dg2_j on the point columns, 0 on the
  // diagonal columns (octsam_w2_host's A)
  auto A = [&](int r, int c) -> double {
    if (c >= Cc) return 0.0;
    const int i = rows_d2 ? c : r, j = rows_d2 ? r : c;
    const double cij = (double)w2_powq(w2_linf(d1[2 * i], d1[2 * i + 1], d2[2 * j], d2[2 * j + 1]), q);
    return cij - (double)dg1[i] - (double)dg2[j];
  };
  const double INF = __builtin_huge_val();
  for (int i = 1; i <= R; ++i) {
    for (int j = lane; j <= NC; j += W2_THREADS) {
      minv[j] = INF;
      used[j] = 0;
    }
    if (lane == 0) p[0] = i;
    int j0 = 0;
    __syncthreads();
    while (true) {
      if (lane == 0) used[j0] = 1;
      __syncthreads();
      const int i0 = p[j0];
      const double ui0 = u[i0];
      double best = INF;
      int bj = 0;
      for (int j = 1 + lane; j <= NC; j += W2_THREADS) {
        if (!used[j]) {
          const double cur = A(i0 - 1, j - 1) - ui0 - v[j];
          double mj = minv[j];
          if (cur < mj) {
            mj = cur;
            minv[j] = cur;
            way[j] = j0;
          }
          if (mj < best) {
            best = mj;
            bj = j;
          }
        }
      }
      // argmin over the wave, the lowest column among equal minima (the host's first strict minimum)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o, 64);
        const int oj = __shfl_xor(bj, o, 64);
        if (ob < best || (ob == best && oj != 0 && (bj == 0 || oj < bj))) {
          best = ob;
          bj = oj;
        }
      }
      const double delta = best;
      __syncthreads();  // every lane has read p / u / v / minv of this step
      for (int j = lane; j <= NC; j += W2_THREADS) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      j0 = bj;
      __syncthreads();
      if (p[j0] == 0) break;
    }
    if (lane == 0) {
      do {
        const int j1 = way[j0];
        p[j0] = p[j1];
        j0 = j1;
      } while (j0);
    }
    __syncthreads();
  }
  if (lane == 0) {
    double cost = 0.0;
    for (int i = 0; i < n; ++i) cost += (double)dg1[i];
    for (int j = 0; j < m; ++j) cost += (double)dg2[j];
    if (R > 0) {
      // row -> column as the host builds it (columns in increasing order), then rows in order
      for (int j = 1; j <= NC; ++j) way[j] = -1;  // reuse: row2col by row
      for (int j = 1; j <= NC; ++j)
        if (p[j] > 0) way[p[j]] = j - 1;  // rows are 1-based: way[1..R]
      for (int r = 0; r < R; ++r) {
        const int c = way[r + 1];
        if (c >= 0 && c < Cc) {
          const int i = rows_d2 ? c : r, j = rows_d2 ? r : c;
          cost += A(r, c);
          mk[i] = j;
        }
      }
    }
    costs[k] = cost;
  }
}

// Phase 2: blocks 0..Kn-1 write the gradient row of map k (d loss / d pred-map values, zero where no pair
// points); block Kn writes the loss.
__global__ void __launch_bounds__(256) w2_loss_kernel(const int32_t* __restrict__ pairs,
                                                      const int32_t* __restrict__ cnt,
                                                      const float* __restrict__ vals, int Kn, int max_pairs,
                                                      int nvals, int feat_col, double q, double lamda,
                                                      const int32_t* __restrict__ entry_maps,
                                                      const int32_t* __restrict__ entry_off,
                                                      const int32_t* __restrict__ map_entry, int n_entries,
                                                      const double* __restrict__ costs,
                                                      const int32_t* __restrict__ match,
                                                      const int32_t* __restrict__ status, int want_grad,
                                                      double* __restrict__ loss_out, float* __restrict__ dpred) {
  extern __shared__ __align__(16) char w2_smem[];
  const int k = blockIdx.x, t = threadIdx.x;
  auto entry_tot = [&](int e) -> double {  // float32(sum of the entry's costs in map order)
    double s = 0.0;
    for (int x = entry_off[e]; x < entry_off[e + 1]; ++x) s += costs[entry_maps[x]];
    return (double)(float)s;
  };
  if (k == Kn) {
    if (t == 0) {
      double total = 0.0;
      for (int e = 0; e < n_entries; ++e) total += w2_root(entry_tot(e), q);
      loss_out[0] = status[0] ? __builtin_nan("") : lamda * total / n_entries;
    }
    return;
  }
  if (!want_grad) return;
  float* out = dpred + (size_t)k * nvals;
  if (status[0]) {  // a pair-buffer overflow anywhere: the step's topological gradient is NaN, like its loss
    for (int i = t; i < nvals; i += 256) out[i] = __builtin_nanf("");
    return;
  }
  // LDS: row[nvals] (the gradient row), hits[nvals] (contributions per pixel), first[nvals] (lowest contribution
  // index o per pixel), pix[2n] / cval[2n] (each contribution's pixel and value, computed once in parallel)
  float* row = (float*)w2_smem;
  int* hits = (int*)(row + nvals);
  int* first = hits + nvals;
  int* pix = first + nvals;
  float* cval = (float*)(pix + 2 * max_pairs);
  for (int i = t; i < nvals; i += 256) {
    row[i] = 0.0f;
    hits[i] = 0;
    first[i] = 0x7fffffff;
  }
  __syncthreads();
  const int e = map_entry[k];
  const int n = e >= 0 ? min(cnt[k * 3 + feat_col], max_pairs) : 0;
  const int32_t* p1 = pairs + (size_t)k * max_pairs * 2;
  const int32_t* p2 = pairs + (size_t)(Kn + k) * max_pairs * 2;
  const float* v1 = vals + (size_t)k * nvals;
  const float* v2 = vals + (size_t)(Kn + k) * nvals;
  const int32_t* mk = match + (size_t)k * max_pairs;
  float scale = 0.0f;
  if (n > 0) scale = (float)(lamda / n_entries * w2_droot(entry_tot(e), q));
  // The host adds the 2n contributions in the order o = pass * n + i (creators, then destroyers) into a zeroed
  // row. Here every contribution is computed once (thread o), its pixel counted and the pixel's lowest o kept
  // (LDS atomics: a count and a minimum, order-independent); a pixel hit once gets 0 + c, a pixel hit several
  // times is summed in o order by the thread of its lowest o, from LDS -- the same fp32 additions, so the row is
  // bit-identical to the host's. (Round 3 / the first parallel form re-read the pair lists from global memory in
  // per-contribution serial loops: 235-246 us per launch.)
  for (int o = t; o < 2 * n; o += 256) {
    const int i = o % n, pass = o / n;
    const int px = p1[2 * i + pass];
    const int j = mk[i];
    const float d1p[2] = {v1[p1[2 * i]], v1[p1[2 * i + 1]]};
    float d2p[2] = {0.0f, 0.0f};
    if (j >= 0) {
      d2p[0] = v2[p2[2 * j]];
      d2p[1] = v2[p2[2 * j + 1]];
    }
    float g0, g1;
    w2_grad_point(d1p, d2p, 0, j >= 0 ? 0 : -1, q, &g0, &g1);
    pix[o] = px;
    cval[o] = scale * (pass == 0 ? g0 : g1);
    atomicAdd(&hits[px], 1);
    atomicMin(&first[px], o);
  }
  __syncthreads();
  for (int o = t; o < 2 * n; o += 256) {
    const int px = pix[o];
    if (first[px] != o) continue;
    if (hits[px] == 1) {
      row[px] = 0.0f + cval[o];
      continue;
    }
    // the pixel's other contributions, in o order: scanned 8 at a time (independent LDS reads in flight), stopping
    // once all hits[px] of them are summed
    float acc = 0.0f;
    const int want = hits[px];
    int got = 0;
    for (int x0 = o; x0 < 2 * n && got < want; x0 += 8) {
      int pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) pv[u] = x0 + u < 2 * n ? pix[x0 + u] : -1;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (pv[u] == px) {
          acc += cval[x0 + u];
          ++got;
        }
      }
    }
    row[px] = acc;
  }
  __syncthreads();
  for (int i = t; i < nvals; i += 256) out[i] = row[i];
}

}  // namespace

extern "C" int64_t octsam_topo_w2_workspace(int32_t Kn, int32_t max_pairs) {
  if (Kn <= 0 || max_pairs <= 0) return 0;
  const W2Layout L(max_pairs);
  const size_t head = (((size_t)Kn * 8 + (size_t)Kn * max_pairs * 4 + 16) + 255) & ~(size_t)255;
  int dev = 0, lds_max = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
  const bool lds = L.bytes <= (size_t)(lds_max > 0 ? lds_max : 65536);
  return (int64_t)(head + (lds ? 0 : (size_t)Kn * L.bytes));
}

extern "C" int octsam_topo_w2(const int32_t* pairs, const int32_t* cnt, const float* vals, int32_t Kn,
                              int32_t max_pairs, int32_t nvals, const int32_t* entry_maps, const int32_t* entry_off,
                              const int32_t* map_entry, int32_t n_entries, int32_t feat_col, double q, double lamda,
                              int32_t want_grad, void* workspace, int64_t workspace_bytes, double* loss_out,
                              float* dpred, void* stream) {
  OCTSAM_CHECK_ARG(pairs && cnt && vals && entry_maps && entry_off && map_entry && workspace && loss_out &&
                       Kn > 0 && max_pairs > 0 && nvals > 0 && n_entries > 0 && (feat_col == 0 || feat_col == 1) &&
                       (!want_grad || dpred) && q > 0,
                   "octsam_topo_w2: bad arguments (Kn=%d, max_pairs=%d, nvals=%d, n_entries=%d, feat_col=%d)", Kn,
                   max_pairs, nvals, n_entries, feat_col);
  OCTSAM_CHECK_ARG(workspace_bytes >= octsam_topo_w2_workspace(Kn, max_pairs),
                   "octsam_topo_w2: workspace of %lld bytes, need %lld", (long long)workspace_bytes,
                   (long long)octsam_topo_w2_workspace(Kn, max_pairs));
  const size_t grad_lds = (size_t)nvals * 12 + (size_t)max_pairs * 16;  // row, hits, first + pix, cval (w2_loss)
  OCTSAM_CHECK_ARG(grad_lds <= 160 * 1024, "octsam_topo_w2: nvals %d / max_pairs %d need %zu B of LDS (> 160 KB)",
                   nvals, max_pairs, grad_lds);
  hipStream_t s = (hipStream_t)stream;
  const W2Layout L(max_pairs);
  int dev = 0, lds_max = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
  const bool lds = L.bytes <= (size_t)(lds_max > 0 ? lds_max : 65536);
  char* ws = (char*)workspace;
  double* costs = (double*)ws;
  int32_t* match = (int32_t*)(ws + (size_t)Kn * 8);
  int32_t* status = (int32_t*)(ws + (size_t)Kn * 8 + (size_t)Kn * max_pairs * 4);
  char* gscratch = ws + ((((size_t)Kn * 8 + (size_t)Kn * max_pairs * 4 + 16) + 255) & ~(size_t)255);
  (void)hipMemsetAsync(status, 0, 4, s);
  if (lds) {
    static int attr_set = 0;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)w2_map_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds_max);
      attr_set = 1;
    }
  }
  w2_map_kernel<<<Kn, W2_THREADS, lds ? L.bytes : 0, s>>>(pairs, cnt, vals, Kn, max_pairs, nvals, feat_col, q, costs,
                                                           match, status, gscratch, lds ? 1 : 0);
  OCTSAM_LAUNCH_CHECK("octsam_topo_w2 (transport)");
  if (want_grad && grad_lds > 65536) {
    static size_t attr_loss = 0;
    if (grad_lds > attr_loss) {
      (void)hipFuncSetAttribute((const void*)w2_loss_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)grad_lds);
      attr_loss = grad_lds;
    }
  }
  w2_loss_kernel<<<Kn + 1, 256, want_grad ? grad_lds : 0, s>>>(
      pairs, cnt, vals, Kn, max_pairs, nvals, feat_col, q, lamda, entry_maps, entry_off, map_entry, n_entries, costs,
      match, status, want_grad, loss_out, dpred);
  OCTSAM_LAUNCH_CHECK("octsam_topo_w2 (loss)");
  return 0;
}
