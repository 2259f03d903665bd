// Phase timing of the cubical-PH kernel (diagnostic): hipcc --offload-arch=gfx950 -O3 -DPH_PROFILE
// -I. scripts/micro/ph_timing.hip -o scripts/micro/ph_timing_probe
#include <cstdio>
#include <cstdarg>
#include <vector>
#include <cmath>
#include <random>
#include "../../dilabhelmholtzoct_amd/csrc/cubical_ph.hip"
namespace octsam { void set_error(const char* fmt, ...) { va_list a; va_start(a, fmt); vfprintf(stderr, fmt, a); va_end(a); } }
int main() {
  const int H = 50, W = 50, n = 16, mp = 1250;
  std::mt19937 rng(0);
  std::normal_distribution<float> nd;
  for (int kind = 0; kind < 2; ++kind) {
    std::vector<float> h(n * H * W);
    for (auto& v : h) v = kind == 0 ? 1.0f / (1.0f + std::exp(-3.0f * nd(rng))) : (nd(rng) > 0 ? 1.f : 0.f);
    float* d; int *p0, *p1, *e, *c;
    hipMalloc(&d, h.size() * 4); hipMalloc(&p0, n * mp * 8); hipMalloc(&p1, n * mp * 8); hipMalloc(&e, n * 8); hipMalloc(&c, n * 12);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int it = 0; it < 3; ++it) octsam_cubical_ph(d, n, H, W, mp, p0, p1, e, c, nullptr);
    hipDeviceSynchronize();
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ph_stamp), sizeof(st));
    const char* names[] = {"load+keys", "sort", "H1 wave", "H0 wave", "->sync", "cofaces", "rank+out"};
    printf("%s maps:\n", kind == 0 ? "noise" : "binary");
    unsigned long long prev[] = {st[0], st[1], st[2], st[2], st[2], st[5], st[6]};
    unsigned long long cur[] = {st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
    for (int k = 0; k < 7; ++k) printf("  %-10s %10llu cycles\n", names[k], cur[k] - prev[k]);
    printf("  total      %10llu cycles\n", st[7] - st[0]);
    for (int d = 0; d < 2; ++d) printf("  H%d find %llu resolve %llu cycles\n", d, st[16 + 2 * d], st[17 + 2 * d]);
  }
  return 0;
}
