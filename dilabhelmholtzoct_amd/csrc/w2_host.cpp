// Host-side exact q-Wasserstein distance between two persistence diagrams (L-inf ground metric,
// diagonal augmentation), with the gradient of the transport cost w.r.t. the first diagram.
//
// Replaces torch_topological.nn.WassersteinDistance(q) -> POT ot.emd2 (ref:octsam/models/
// topological_loss.py:78-82), which the reference also runs on the host in float64. The EMD with
// weights a = (1,..,1,m), b = (1,..,1,n) over the (n+1)x(m+1) cost matrix is solved as the
// equivalent linear assignment (integral optimal vertex), reduced to a rectangular problem over the
// smaller diagram (see octsam_w2_host), solved with the shortest-augmenting-path Hungarian method. Cost entries are formed in fp32 exactly as torch does (cdist p=inf and
// vector_norm to the diagonal, then **q) before the float64 solve.
// Gradient semantics follow torch autograd: cdist p=inf gives sign(diff) to every coordinate that
// attains the max; the diagonal distance |d-b|/2 gives (-1/2, +1/2)*sign(d-b).
// Optimal plans are not unique under ties; POT's network simplex may pick a different optimal plan
// (same cost, different subgradient): gradient parity under such ties is unpinned.
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "../../include/octsam.h"

namespace octsam {
void set_error(const char* fmt, ...);  // api.cpp: the thread-local message behind octsam_last_error()
}

namespace {

// e-maxx Hungarian for a rectangular matrix (n rows <= m cols, row-major with stride m), minimisation;
// O(n^2 m); returns assignment row -> col (0-based)
std::vector<int> hungarian(const std::vector<double>& a, int n, int m) {
  const double INF = std::numeric_limits<double>::infinity();
  const int N = m;
  std::vector<double> u(n + 1, 0.0), v(N + 1, 0.0), minv(N + 1);
  std::vector<int> p(N + 1, 0), way(N + 1, 0);
  std::vector<char> used(N + 1);
  for (int i = 1; i <= n; ++i) {
    p[0] = i;
    int j0 = 0;
    std::fill(minv.begin(), minv.end(), INF);
    std::fill(used.begin(), used.end(), 0);
    do {
      used[j0] = 1;
      int i0 = p[j0], j1 = 0;
      double delta = INF;
      for (int j = 1; j <= N; ++j)
        if (!used[j]) {
          double cur = a[(i0 - 1) * N + (j - 1)] - u[i0] - v[j];
          if (cur < minv[j]) { minv[j] = cur; way[j] = j0; }
          if (minv[j] < delta) { delta = minv[j]; j1 = j; }
        }
      for (int j = 0; j <= N; ++j)
        if (used[j]) { u[p[j]] += delta; v[j] -= delta; }
        else minv[j] -= delta;
      j0 = j1;
    } while (p[j0] != 0);
    do {
      int j1 = way[j0];
      p[j0] = p[j1];
      j0 = j1;
    } while (j0);
  }
  std::vector<int> row2col(n, -1);
  for (int j = 1; j <= N; ++j)
    if (p[j] > 0) row2col[p[j] - 1] = j - 1;
  return row2col;
}

inline float linf(float a0, float a1, float b0, float b1) { return std::fmax(std::fabs(a0 - b0), std::fabs(a1 - b1)); }
inline float diag_dist(float b, float d) {
  float h = 0.5f * (b + d);
  return std::fmax(std::fabs(b - h), std::fabs(d - h));
}
inline float powq(float x, double q) { return q == 2.0 ? x * x : (float)std::pow((double)x, q); }
inline float sgn(float x) { return (x > 0.0f) - (x < 0.0f); }

}  // namespace

extern "C" int octsam_w2_host(const float* d1_host, int32_t n, const float* d2_host, int32_t m, double q,
                              double* cost_host, float* grad_d1_host) {
  if (n < 0 || m < 0 || !cost_host || (n > 0 && (!d1_host || !grad_d1_host)) || (m > 0 && !d2_host)) {
    octsam::set_error("octsam_w2_host: bad arguments (n=%d, m=%d, null pointer for a non-empty diagram?)", n, m);
    return 1;
  }
  for (int i = 0; i < 2 * n; ++i) grad_d1_host[i] = 0.0f;
  std::vector<float> dg1(n), dg2(m);
  for (int i = 0; i < n; ++i) dg1[i] = powq(diag_dist(d1_host[2 * i], d1_host[2 * i + 1]), q);
  for (int j = 0; j < m; ++j) dg2[j] = powq(diag_dist(d2_host[2 * j], d2_host[2 * j + 1]), q);
  auto Cij = [&](int i, int j) {
    return (double)powq(linf(d1_host[2 * i], d1_host[2 * i + 1], d2_host[2 * j], d2_host[2 * j + 1]), q);
  };
  // The (n+m)^2 diagonal-augmented assignment reduces to a rectangular one over the smaller diagram:
  // cost = sum_i dg1[i] + sum_j dg2[j] + min over partial matchings of sum (C_ij - dg1[i] - dg2[j]).
  // Rows = points of the smaller diagram, columns = points of the other one plus one "diagonal" column
  // per row (reduced cost 0). O(r^2 (r + c)) instead of O((n+m)^3).
  const bool rows_are_d2 = m <= n;
  const int R = rows_are_d2 ? m : n, Cc = rows_are_d2 ? n : m;
  double cost = 0.0;
  for (int i = 0; i < n; ++i) cost += dg1[i];
  for (int j = 0; j < m; ++j) cost += dg2[j];
  std::vector<int> match_of_d1(n, -1);  // d1 point -> d2 point or -1 (diagonal)
  if (R > 0) {
    const int NC = Cc + R;
    const int N = NC;  // row stride
    std::vector<double> A((size_t)R * N, 0.0);
    for (int r = 0; r < R; ++r)
      for (int c = 0; c < NC; ++c) {
        double v = 0.0;
        if (c < Cc) {
          int i = rows_are_d2 ? c : r, j = rows_are_d2 ? r : c;
          v = Cij(i, j) - (double)dg1[i] - (double)dg2[j];
        }
        A[(size_t)r * N + c] = v;
      }
    std::vector<int> asg = hungarian(A, R, NC);
    for (int r = 0; r < R; ++r) {
      int c = asg[r];
      if (c < Cc) {
        int i = rows_are_d2 ? c : r, j = rows_are_d2 ? r : c;
        cost += A[(size_t)r * N + c];
        match_of_d1[i] = j;
      }
    }
  }
  *cost_host = cost;
  for (int i = 0; i < n; ++i) {
    const int j = match_of_d1[i];
    const float b = d1_host[2 * i], d = d1_host[2 * i + 1];
    if (j >= 0) {
      const float e0 = b - d2_host[2 * j], e1 = d - d2_host[2 * j + 1];
      const float M = std::fmax(std::fabs(e0), std::fabs(e1));
      const float coef = q == 2.0 ? 2.0f * M : (float)(q * std::pow((double)M, q - 1.0));  // (same bits)
      grad_d1_host[2 * i] = coef * (std::fabs(e0) == M ? sgn(e0) : 0.0f);
      grad_d1_host[2 * i + 1] = coef * (std::fabs(e1) == M ? sgn(e1) : 0.0f);
    } else {
      const float M = diag_dist(b, d);
      const float coef = q == 2.0 ? 2.0f * M : (float)(q * std::pow((double)M, q - 1.0));  // (same bits)
      grad_d1_host[2 * i] = coef * 0.5f * sgn(b - d);
      grad_d1_host[2 * i + 1] = coef * 0.5f * sgn(d - b);
    }
  }
  return 0;
}

// All loss entries of one step in one call (the host half of topo_loss, topological_loss.py:68-96):
// per entry e (maps entry_maps[entry_off[e] .. entry_off[e+1])), the W_q cost between the pred diagram
// (map k) and the gt diagram (map Kn + k), tot = float32(sum of the entry's costs), loss += tot^(1/q);
// d loss / d pred-map value accumulated into dpred [Kn, nvals] in the same order and precision as the
// Python path it replaces (costs summed in double, the float32 products of numpy 2's promotion rules).
extern "C" int octsam_topo_host(const int32_t* pairs, const int32_t* cnt, const float* vals, int32_t Kn,
                                int32_t max_pairs, int32_t nvals, const int32_t* entry_maps,
                                const int32_t* entry_off, int32_t n_entries, int32_t feat_col, double q,
                                double lamda, int32_t want_grad, double* loss_out, float* dpred) {
  if (!pairs || !cnt || !vals || !entry_maps || !entry_off || !loss_out || Kn <= 0 || n_entries <= 0 ||
      (want_grad && !dpred) || feat_col < 0 || feat_col > 1) {
    octsam::set_error("octsam_topo_host: bad arguments (Kn=%d, n_entries=%d, feat_col=%d, want_grad=%d)", Kn,
                      n_entries, feat_col, want_grad);
    return 1;
  }
  if (want_grad)
    for (long long i = 0; i < (long long)Kn * nvals; ++i) dpred[i] = 0.0f;
  std::vector<float> d1, d2, g;
  std::vector<double> costs;
  double total = 0.0;
  for (int e = 0; e < n_entries; ++e) {
    costs.clear();
    const int e0 = entry_off[e], e1 = entry_off[e + 1];
    std::vector<std::vector<float>> grads;
    for (int t = e0; t < e1; ++t) {
      const int k = entry_maps[t];
      if (k < 0 || k >= Kn) {
        octsam::set_error("octsam_topo_host: entry %d names map %d outside [0, %d)", e, k, Kn);
        return 1;
      }
      const int n = cnt[k * 3 + feat_col], m = cnt[(Kn + k) * 3 + feat_col];
      if (n > max_pairs || m > max_pairs || cnt[k * 3 + 2] || cnt[(Kn + k) * 3 + 2]) {
        octsam::set_error("octsam_topo_host: map %d pair buffer overflow (pred %d, gt %d pairs, max_pairs %d)", k, n,
                          m, max_pairs);
        return 1;
      }
      d1.resize(2 * (size_t)n);
      d2.resize(2 * (size_t)m);
      const int32_t* p1 = pairs + (size_t)k * max_pairs * 2;
      const int32_t* p2 = pairs + (size_t)(Kn + k) * max_pairs * 2;
      const float* v1 = vals + (size_t)k * nvals;
      const float* v2 = vals + (size_t)(Kn + k) * nvals;
      for (int i = 0; i < n; ++i) { d1[2 * i] = v1[p1[2 * i]]; d1[2 * i + 1] = v1[p1[2 * i + 1]]; }
      for (int j = 0; j < m; ++j) { d2[2 * j] = v2[p2[2 * j]]; d2[2 * j + 1] = v2[p2[2 * j + 1]]; }
      g.assign(2 * (size_t)n, 0.0f);
      double c = 0.0;
      if (octsam_w2_host(n ? d1.data() : nullptr, n, m ? d2.data() : nullptr, m, q, &c, n ? g.data() : nullptr))
        return 1;  // message set by octsam_w2_host
      costs.push_back(c);
      grads.push_back(g);
    }
    double s = 0.0;
    for (double c : costs) s += c;  // Python sum() over floats, left to right
    const double tot = (double)(float)s;
    // q = 2 (the call site): the 1/q power as a correctly rounded sqrt, as octsam_topo_w2 computes it on the device
    total += q == 2.0 ? std::sqrt(tot) : std::pow(tot, 1.0 / q);
    if (want_grad) {
      const double dd = tot > 0 ? (q == 2.0 ? 0.5 / std::sqrt(tot) : (1.0 / q) * std::pow(tot, 1.0 / q - 1.0))
                                : std::numeric_limits<double>::infinity();
      // numpy 2 (NEP 50): python-float scale * float32 gradient is computed in float32
      const float scale = (float)(lamda / n_entries * dd);
      for (int t = e0; t < e1; ++t) {
        const int k = entry_maps[t];
        const int n = cnt[k * 3 + feat_col];
        const int32_t* p1 = pairs + (size_t)k * max_pairs * 2;
        const std::vector<float>& gg = grads[t - e0];
        float* dp = dpred + (size_t)k * nvals;
        for (int i = 0; i < n; ++i) dp[p1[2 * i]] += scale * gg[2 * i];
        for (int i = 0; i < n; ++i) dp[p1[2 * i + 1]] += scale * gg[2 * i + 1];
      }
    }
  }
  *loss_out = lamda * total / n_entries;
  return 0;
}
