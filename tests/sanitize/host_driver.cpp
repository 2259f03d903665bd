// Host-code sanitizer driver (tests/test_sanitizers_cpu.py builds it with -fsanitize=address,undefined):
// exercises the product's host C++ (w2_host.cpp: octsam_w2_host, octsam_topo_host; api.cpp) and the
// oracle's C persistence on random and adversarial inputs, and checks the W_q cost against a brute-force
// assignment over the diagonal-augmented problem for tiny diagrams.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "../../include/octsam.h"

extern "C" int oracle_cubical_ph(const float* x, int H, int W, int max_pairs, int32_t* pairs0, int32_t* n0,
                                 int32_t* pairs1, int32_t* n1, int32_t* essential);

static double brute_w(const std::vector<float>& a, const std::vector<float>& b, double q) {
  const int n = (int)a.size() / 2, m = (int)b.size() / 2, N = n + m;
  auto lq = [&](float x) { return q == 2.0 ? (double)(x * x) : std::pow((double)x, q); };
  // rows: n points of a + m diagonal slots; cols: m points of b + n diagonal slots
  std::vector<double> C(N * N, 0.0);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      const bool ri = i < n, cj = j < m;
      float v = 0.0f;
      if (ri && cj) v = std::fmax(std::fabs(a[2 * i] - b[2 * j]), std::fabs(a[2 * i + 1] - b[2 * j + 1]));
      else if (ri) v = std::fabs(a[2 * i + 1] - a[2 * i]) / 2;
      else if (cj) v = std::fabs(b[2 * j + 1] - b[2 * j]) / 2;
      C[i * N + j] = (ri || cj) ? lq(v) : 0.0;
    }
  std::vector<int> perm(N);
  std::iota(perm.begin(), perm.end(), 0);
  double best = INFINITY;
  do {
    double s = 0.0;
    for (int i = 0; i < N; ++i) s += C[i * N + perm[i]];
    best = std::min(best, s);
  } while (std::next_permutation(perm.begin(), perm.end()));
  return best;
}

int main() {
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  int fails = 0;
  // W_q against brute force (ties included: values on a coarse grid)
  for (int t = 0; t < 400; ++t) {
    const int n = t % 4, m = (t / 4) % 4;
    const double q = (t % 3 == 0) ? 1.0 : 2.0;
    std::vector<float> a(2 * n), b(2 * m);
    for (auto& v : a) v = (t % 2) ? std::floor(U(rng) * 4) / 4 : U(rng);
    for (auto& v : b) v = (t % 2) ? std::floor(U(rng) * 4) / 4 : U(rng);
    for (int i = 0; i < n; ++i) if (a[2 * i] > a[2 * i + 1]) std::swap(a[2 * i], a[2 * i + 1]);
    for (int j = 0; j < m; ++j) if (b[2 * j] > b[2 * j + 1]) std::swap(b[2 * j], b[2 * j + 1]);
    double cost = -1;
    std::vector<float> g(2 * n + 1);
    if (octsam_w2_host(n ? a.data() : nullptr, n, m ? b.data() : nullptr, m, q, &cost, g.data()) != 0) {
      std::printf("w2 error: %s\n", octsam_last_error());
      ++fails;
      continue;
    }
    const double ref = brute_w(a, b, q);
    if (!(std::fabs(cost - ref) <= 1e-6 * (1.0 + std::fabs(ref)))) {
      std::printf("w2 mismatch n=%d m=%d q=%g: %.9g vs %.9g\n", n, m, q, cost, ref);
      ++fails;
    }
  }
  // larger random diagrams (no reference; the sanitizers watch the memory traffic)
  for (int t = 0; t < 20; ++t) {
    const int n = 1 + t * 17 % 300, m = 1 + t * 29 % 300;
    std::vector<float> a(2 * n), b(2 * m), g(2 * n);
    for (auto& v : a) v = U(rng);
    for (auto& v : b) v = U(rng);
    double cost;
    if (octsam_w2_host(a.data(), n, b.data(), m, 2.0, &cost, g.data()) != 0 || !std::isfinite(cost)) ++fails;
  }
  // bad arguments report through the error channel
  double c;
  if (octsam_w2_host(nullptr, 3, nullptr, 0, 2.0, &c, nullptr) == 0) ++fails;
  // persistence (oracle C) on random, tied and checkerboard 50x50 maps, then the host loss on its pairs
  const int H = 50, W = 50, MP = (H * W + 1) / 2, Kn = 3;
  std::vector<float> maps(2 * Kn * H * W);
  for (int k = 0; k < 2 * Kn; ++k)
    for (int p = 0; p < H * W; ++p) {
      const int r = p / W, cc = p % W;
      maps[k * H * W + p] = k == 0 ? U(rng) : k == 1 ? std::floor(U(rng) * 3) : k == 2 ? (float)((r + cc) & 1)
                                                                                  : std::floor(U(rng) * 2);
    }
  std::vector<int32_t> pairs(2 * Kn * MP * 2 * 2), cnt(2 * Kn * 3);
  for (int k = 0; k < 2 * Kn; ++k) {
    int32_t n0 = 0, n1 = 0, ess[2];
    std::vector<int32_t> p0(MP * 2), p1(MP * 2);
    if (oracle_cubical_ph(&maps[k * H * W], H, W, MP, p0.data(), &n0, p1.data(), &n1, ess) != 0) ++fails;
    // octsam_topo_host layout: pairs [2Kn, max_pairs, 2] per dimension column -> use H0 pairs here
    for (int i = 0; i < n0 && i < MP; ++i) {
      pairs[(k * MP + i) * 2] = p0[2 * i];
      pairs[(k * MP + i) * 2 + 1] = p0[2 * i + 1];
    }
    cnt[k * 3] = n0;
    cnt[k * 3 + 1] = 0;
    cnt[k * 3 + 2] = 0;
  }
  std::vector<int32_t> emaps = {0, 1, 2}, eoff = {0, 1, 3};
  std::vector<float> dpred(Kn * H * W);
  double loss = 0;
  if (octsam_topo_host(pairs.data(), cnt.data(), maps.data(), Kn, MP, H * W, emaps.data(), eoff.data(), 2, 0, 2.0,
                       0.5, 1, &loss, dpred.data()) != 0) {
    std::printf("topo_host error: %s\n", octsam_last_error());
    ++fails;
  }
  if (!std::isfinite(loss)) ++fails;
  std::printf("sanitizer driver: %d failures\n", fails);
  return fails ? 1 : 0;
}
