// Cycles per edge of the union-find chunk resolve loop (cubical_ph.hip uf_wave) in instruction variants
// (diagnostic): hipcc --offload-arch=gfx950 -O3 scripts/micro/uf_resolve_probe.hip -o scripts/micro/uf_resolve_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

constexpr int CHUNKS = 256;

// V0: SALU min/max, compare-and-select recording (the kernel's loop)
__global__ void v0(const int* in, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int c = 0; c < CHUNKS; ++c) {
    int cru = in[c * 128 + lane], crv = in[c * 128 + 64 + lane];
    int my_young = -1, my_old = 0;
    for (int j0 = 0; j0 < 64; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        const int sa = __builtin_amdgcn_readlane(cru, j);
        const int sc = __builtin_amdgcn_readlane(crv, j);
        const int young = max(sa, sc), old = min(sa, sc);
        cru = cru == young ? old : cru;
        crv = crv == young ? old : crv;
        const bool rec = lane == j && sa != sc;
        my_young = rec ? young : my_young;
        my_old = rec ? old : my_old;
      }
    }
    acc += my_young * 3 + my_old;
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

// V1: recording by writelane (no per-edge compare), young == old marks "no merge"
__global__ void v1(const int* in, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int c = 0; c < CHUNKS; ++c) {
    int cru = in[c * 128 + lane], crv = in[c * 128 + 64 + lane];
    int my_young = 0, my_old = 0;
    for (int j0 = 0; j0 < 64; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        const int sa = __builtin_amdgcn_readlane(cru, j);
        const int sc = __builtin_amdgcn_readlane(crv, j);
        const int young = max(sa, sc), old = min(sa, sc);
        cru = cru == young ? old : cru;
        crv = crv == young ? old : crv;
        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(my_young) : "s"(young), "{m0}"(j));
        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(my_old) : "s"(old), "{m0}"(j));
      }
    }
    acc += (my_young != my_old ? my_young : -1) * 3 + (my_young != my_old ? my_old : 0);
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

// V2: V1 with min/max on the VALU (inline asm keeps them off the SALU)
__global__ void v2(const int* in, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int c = 0; c < CHUNKS; ++c) {
    int cru = in[c * 128 + lane], crv = in[c * 128 + 64 + lane];
    int my_young = 0, my_old = 0;
    for (int j0 = 0; j0 < 64; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        const int sa = __builtin_amdgcn_readlane(cru, j);
        const int sc = __builtin_amdgcn_readlane(crv, j);
        int vsc, young, old;
        asm volatile("v_mov_b32 %0, %1" : "=v"(vsc) : "s"(sc));
        asm volatile("v_max_i32 %0, %1, %2" : "=v"(young) : "s"(sa), "v"(vsc));
        asm volatile("v_min_i32 %0, %1, %2" : "=v"(old) : "s"(sa), "v"(vsc));
        cru = cru == young ? old : cru;
        crv = crv == young ? old : crv;
        my_young = lane == j ? young : my_young;
        my_old = lane == j ? old : my_old;
      }
    }
    acc += (my_young != my_old ? my_young : -1) * 3 + (my_young != my_old ? my_old : 0);
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

// V3: dependency-free loop body (readlane of the chunk-start roots only): the issue-rate floor
__global__ void v3(const int* in, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int c = 0; c < CHUNKS; ++c) {
    const int ru = in[c * 128 + lane], rv = in[c * 128 + 64 + lane];
    int cru = ru, crv = rv;
    int my_young = 0, my_old = 0;
    for (int j0 = 0; j0 < 64; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        const int sa = __builtin_amdgcn_readlane(ru, j);
        const int sc = __builtin_amdgcn_readlane(rv, j);
        const int young = max(sa, sc), old = min(sa, sc);
        cru = cru == young ? old : cru;
        crv = crv == young ? old : crv;
        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(my_young) : "s"(young), "{m0}"(j));
        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(my_old) : "s"(old), "{m0}"(j));
      }
    }
    acc += (my_young != my_old ? my_young : -1) * 3 + my_old + cru + crv;
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

// V4: the chunk's 2 x 64 roots flattened edge-major into two VGPRs (edge j's roots in lanes 2j, 2j+1 of A for
// j < 32, of B above), so the second half of the edges relabels one VGPR; the merge recorded by one writelane
// of (young | old << 16)
template <int HALF>
__device__ __forceinline__ void v4_edge(int j, int& A, int& B, int& rec) {
  const int l = 2 * (HALF ? j - 32 : j);
  const int sa = __builtin_amdgcn_readlane(HALF ? B : A, l);
  const int sc = __builtin_amdgcn_readlane(HALF ? B : A, l + 1);
  const int young = max(sa, sc), old = min(sa, sc);
  if (!HALF) A = A == young ? old : A;
  B = B == young ? old : B;
  const int pk = young | (old << 16);
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(rec) : "s"(pk), "{m0}"(j));
}
__global__ void v4(const int* in, int* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  int acc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int c = 0; c < CHUNKS; ++c) {
    // edge e's roots (in[c*128 + e], in[c*128 + 64 + e]) at lanes 2e, 2e + 1
    const int e = (lane >> 1);
    int A = in[c * 128 + (lane & 1) * 64 + e], B = in[c * 128 + (lane & 1) * 64 + 32 + e];
    int rec = 0;
    for (int j0 = 0; j0 < 32; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) v4_edge<0>(j0 + u, A, B, rec);
    }
    for (int j0 = 32; j0 < 64; j0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) v4_edge<1>(j0 + u, A, B, rec);
    }
    const int my_young = rec & 0xffff, my_old = rec >> 16;
    acc += (my_young != my_old ? my_young : -1) * 3 + (my_young != my_old ? my_old : 0);
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[lane] = acc;
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  int h[CHUNKS * 128];
  unsigned s = 1;
  for (int i = 0; i < CHUNKS * 128; ++i) { s = s * 1103515245u + 12345u; h[i] = (s >> 16) % 96; }
  int *d, *o; unsigned long long* cy;
  hipMalloc(&d, sizeof(h)); hipMalloc(&o, 64 * 4); hipMalloc(&cy, 8);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  void (*ks[])(const int*, int*, unsigned long long*) = {v0, v1, v2, v3, v4};
  const char* nm[] = {"V0 salu minmax + cmp record", "V1 writelane record", "V2 valu minmax", "V3 no dependency", "V4 flattened + packed record"};
  int ref[64], got[64];
  for (int k = 0; k < 5; ++k) {
    unsigned long long c = 0;
    for (int it = 0; it < 3; ++it) { ks[k]<<<1, 64>>>(d, o, cy); hipDeviceSynchronize(); }
    hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
    hipMemcpy(k == 0 ? ref : got, o, 256, hipMemcpyDeviceToHost);
    int same = 1;
    if (k > 0 && k != 3) for (int i = 0; i < 64; ++i) same &= ref[i] == got[i];
    printf("%-30s %7.1f cycles/edge  %s\n", nm[k], (double)c / (CHUNKS * 64), k == 3 ? "" : (same ? "same" : "DIFF"));
  }
  return 0;
}
