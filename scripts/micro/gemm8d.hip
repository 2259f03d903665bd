// Micro-benchmark (diagnostics): an 8-wave 256x128-tile GEMM whose register epilogue of tile i runs inside the
// main loop of tile i+1 (two accumulator sets per wave), against the library's octsam_gemm on the encoder shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm8d.hip -o gemm8d -ldl ; run from the repo root.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../dilabhelmholtzoct_amd/csrc/common.h"
#include "../../include/octsam.h"

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef float fx2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

namespace d8 {
constexpr int BM = 256, BN = 128, HK = 32;
constexpr int A_H = BM * HK * 2;    // 16 KiB: A half-stage [256][32]
constexpr int B_H = BN * HK * 2;    // 8 KiB: B half-stage [128][32]
constexpr int SLOT = A_H + B_H;     // 24 KiB
constexpr int NSLOT = 6;
constexpr int RING = NSLOT * SLOT;  // 144 KiB
constexpr int BIAS_N = 4096;
constexpr int LDS = RING + BIAS_N * 4;  // 160 KiB
constexpr int DIST = 5;                 // half-steps prefetched ahead
constexpr int OPS = 3;                  // LDS-DMA issues per wave per half-step (A 2, B 1)
constexpr int UNR = 24;                 // phases of a tile unrolled (chunk placement is static there)
__host__ __device__ constexpr int chunk_phase(int c) { return 2 + 2 * c; }  // 8 chunks: phases 2..16
__host__ __device__ constexpr int chunk_at(int ph) {
  return (ph >= 2 && ph <= 16 && (ph & 1) == 0) ? (ph - 2) / 2 : -1;
}
__host__ __device__ constexpr int stores_in_window(int ph) {  // chunk phases in [ph-4, ph]
  int n = 0;
  for (int q = ph - 4; q <= ph; ++q) n += chunk_at(q) >= 0 ? 1 : 0;
  return n;
}

struct P {
  const bf16* A;
  const bf16* B;
  bf16* C;
  const float* bias;
  int M, N, K, lda, ldb, ldc;
  int tiles_n, ntiles, tpw;
};

__device__ __forceinline__ int swz(int r) { return (-(r >> 2)) & 3; }
__device__ __forceinline__ bf16x8 frag(const char* img, int row, int kc) {
  return *(const bf16x8*)(img + row * 64 + ((kc ^ swz(row)) << 4));
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
#define W(k) \
  case k:    \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15) W(16) W(17) W(18)
    W(19) W(20) W(21) W(22) W(23)
#undef W
    default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
  }
}
template <int N>
__device__ __forceinline__ void vm_wait_c() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// a tile's operand descriptors (rows past M / N read as zero through the range check)
struct Tile {
  __amdgpu_buffer_rsrc_t ra, rb;
  int row0, col0;
};
__device__ __forceinline__ Tile make_tile(const P& p, int id) {
  Tile t;
  const int tm = id / p.tiles_n, tn = id - tm * p.tiles_n;
  t.row0 = tm * BM;
  t.col0 = tn * BN;
  t.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(p.A + (long long)t.row0 * p.lda), (short)0,
                                           (int)((long long)(p.M - t.row0) * p.lda * 2), 0x00020000);
  t.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(p.B + (long long)t.col0 * p.ldb), (short)0,
                                           (int)((long long)max(0, p.N - t.col0) * p.ldb * 2), 0x00020000);
  return t;
}
// issue the wave's 3 LDS-DMA ops of half-step s (k = 32 s) of tile t into ring slot `slot`
__device__ __forceinline__ void dma(const Tile& t, int s, char* ring, int slot, const uint32_t (&voff)[3], int wave) {
  char* base = ring + slot * SLOT;
  const uint32_t ko = (uint32_t)s * 64u;
#pragma unroll
  for (int u = 0; u < 2; ++u)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(t.ra, (lds_ptr_t)(base + (wave * 2 + u) * 1024), 16, voff[u], ko, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(t.rb, (lds_ptr_t)(base + A_H + wave * 1024), 16, voff[2], ko, 0, 0);
}

template <int ACT>
__device__ __forceinline__ void act8(float (&v)[8]) {
  if constexpr (ACT == 2) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const fx2 r = gelu_fast2((fx2){v[e], v[e + 1]});
      v[e] = r[0];
      v[e + 1] = r[1];
    }
  }
}

// chunk c = (mi, pr) of a finished 64x64 wave tile: permlane16 pairs -> 8 consecutive columns of row 16 mi + (lane &
// 15) per lane, activation, bf16, one 16-B buffer store (row range checked, columns past N dropped)
template <int ACT, int C>
__device__ __forceinline__ void epi_chunk(const P& p, const f32x4 (&acc)[4][4], const __amdgpu_buffer_rsrc_t& rc,
                                          int wr, int wc, int col0, int lane) {
  constexpr int mi = C >> 1, pr = C & 1;
  const int q = lane >> 4;
  const int cofs = 16 * (q & 1) + 8 * (q >> 1);
  float v[8];
  const u32x4 x = __builtin_bit_cast(u32x4, acc[mi][2 * pr]);
  const u32x4 y = __builtin_bit_cast(u32x4, acc[mi][2 * pr + 1]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t xi = x[i], yi = y[i];
    const auto r = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
    v[i] = __builtin_bit_cast(float, (uint32_t)r[0]);
    v[4 + i] = __builtin_bit_cast(float, (uint32_t)r[1]);
  }
  act8<ACT>(v);
  bf16x8 h;
#pragma unroll
  for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
  const int row = wr * 64 + mi * 16 + (lane & 15);
  const int col = wc * 64 + 32 * pr + cofs;
  const uint32_t o = (col0 + col < p.N) ? (uint32_t)((row * p.ldc + col) * 2) : 0x80000000u;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), rc, o, 0, 0);
}

template <int ACT>
__device__ __forceinline__ void epi_chunk_rt(const P& p, const f32x4 (&acc)[4][4], const __amdgpu_buffer_rsrc_t& rc,
                                             int wr, int wc, int col0, int lane, int c) {
  switch (c) {
    case 0: epi_chunk<ACT, 0>(p, acc, rc, wr, wc, col0, lane); break;
    case 1: epi_chunk<ACT, 1>(p, acc, rc, wr, wc, col0, lane); break;
    case 2: epi_chunk<ACT, 2>(p, acc, rc, wr, wc, col0, lane); break;
    case 3: epi_chunk<ACT, 3>(p, acc, rc, wr, wc, col0, lane); break;
    case 4: epi_chunk<ACT, 4>(p, acc, rc, wr, wc, col0, lane); break;
    case 5: epi_chunk<ACT, 5>(p, acc, rc, wr, wc, col0, lane); break;
    case 6: epi_chunk<ACT, 6>(p, acc, rc, wr, wc, col0, lane); break;
    default: epi_chunk<ACT, 7>(p, acc, rc, wr, wc, col0, lane); break;
  }
}

// MODE 0: epilogue of tile i inside tile i+1's main loop; 1: no epilogue (accumulators kept live); 2: epilogue
// at the end of each tile (not overlapped)
template <int ACT, int MODE>
__global__ __launch_bounds__(512) void gemm8d_kernel(P p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  float* lbias = (float*)(smem + RING);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave & 3, wc = wave >> 2;  // wave tile rows 64 wr, cols 64 wc; stagger group = wc
  // XCD-contiguous workgroup ids: a workgroup's tiles and its XCD neighbours' share A panels in L2
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, rr = nwg & 7, xcd = bid & 7, loc = bid >> 3;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + loc;
  }
  const int t_first = bid * p.tpw;
  const int T = min(p.tpw, p.ntiles - t_first);
  if (T <= 0) return;
  const int nk2 = p.K / HK;  // half-steps per tile
  const int G = T * nk2;
  if (p.bias)
    for (int i = tid * 4; i < p.N; i += 512 * 4) *(float4*)(lbias + i) = *(const float4*)(p.bias + i);
  uint32_t voff[3];
  {
    const int rr = lane >> 2, sl = lane & 3;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int r = (u < 2 ? (wave * 2 + u) : wave) * 16 + rr;
      const int c = sl ^ swz(r);
      voff[u] = (uint32_t)((r * (u < 2 ? p.lda : p.ldb) + c * 8) * 2);
    }
  }
  const uint32_t frag_a = (uint32_t)((wr * 64 + (lane & 15)) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4));
  const uint32_t frag_b = (uint32_t)(A_H + (wc * 64 + (lane & 15)) * 64 + (((lane >> 4) ^ swz(lane & 15)) << 4));
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // DMA cursor: next half-step sd of tile td_i, into ring slot slot_d; dma_left half-steps still to issue
  Tile td = make_tile(p, t_first);
  int td_i = 0, sd = 0, slot_d = 0, dma_left = G;
  auto dma_next = [&]() __attribute__((always_inline)) {
    dma(td, sd, ring, slot_d, voff, wave);
    slot_d = slot_d == NSLOT - 1 ? 0 : slot_d + 1;
    --dma_left;
    if (++sd == nk2) {
      sd = 0;
      if (++td_i < T) td = make_tile(p, t_first + td_i);
    }
  };
  const int pro = min(DIST, G);
  for (int i = 0; i < pro; ++i) dma_next();
  vm_wait(OPS * (pro - 1));
  raw_barrier();
  if (wc == 1) raw_barrier();  // stagger: group 1 one barrier behind

  f32x4 acc[4][4], prev[4][4];
  bf16x8 af[4], bfr[4];
  __amdgpu_buffer_rsrc_t rc_prev = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, 0, 0x00020000);
  int col0_prev = 0, img_off = 0, g = 0;
  for (int ti = 0; ti < T; ++ti) {
    const int id = t_first + ti, tm = id / p.tiles_n, tn = id - tm * p.tiles_n;
    const int row0 = tm * BM, col0 = tn * BN;
    const bool has_prev = MODE == 0 && ti > 0;
    const __amdgpu_buffer_rsrc_t rc_cur = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.C + (long long)row0 * p.ldc + col0), (short)0,
        (int)((long long)min(BM, p.M - row0) * p.ldc * 2 - (long long)col0 * 2), 0x00020000);
    // bias as the accumulator init of the first K-half (columns past N read any in-range entry; never stored)
    f32x4 binit[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = col0 + wc * 64 + ni * 16 + 4 * (lane >> 4);
      binit[ni] = p.bias ? *(const f32x4*)(lbias + min(n, p.N - 4)) : (f32x4)0.0f;
    }
    auto phase = [&](bool first, bool s4, int chunk, int st_win) __attribute__((always_inline)) {
      if (dma_left > 0) dma_next();
      const char* img = ring + img_off;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi] = *(const bf16x8*)(img + frag_a + mi * 1024);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = *(const bf16x8*)(img + frag_b + ni * 1024);
      if (chunk >= 0 && has_prev) epi_chunk_rt<ACT>(p, prev, rc_prev, wr, wc, col0_prev, lane, chunk);
      // the next half-step resident: everything issued after its DMA (later DMAs, the epilogue stores since) may
      // stay in flight
      if (dma_left > 0) {  // steady state: the DMAs of the next DIST - 1 half-steps and the stores since
        if (MODE == 2 && ti > 0 && s4) vm_wait_c<OPS * (DIST - 1) + 8>();
        else if (has_prev && st_win == 1) vm_wait_c<OPS * (DIST - 1) + 1>();
        else if (has_prev && st_win == 2) vm_wait_c<OPS * (DIST - 1) + 2>();
        else if (has_prev && st_win == 3) vm_wait_c<OPS * (DIST - 1) + 3>();
        else vm_wait_c<OPS * (DIST - 1)>();
      } else if (g + 1 < G) {
        vm_wait(OPS * (G - g - 2) + (has_prev ? st_win : 0) + ((MODE == 2 && ti > 0 && s4) ? 8 : 0));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mma16(bfr[ni], af[mi], first ? binit[ni] : acc[mi][ni]);
      __builtin_amdgcn_s_setprio(0);
      raw_barrier();
      img_off = img_off == (NSLOT - 1) * SLOT ? 0 : img_off + SLOT;
      ++g;
    };
#pragma unroll
    for (int s = 0; s < UNR; ++s) {
      if (s < nk2) phase(s == 0, s < 4, chunk_at(s), stores_in_window(s));
    }
    for (int s = UNR; s < nk2; ++s) phase(false, false, -1, 0);
    if constexpr (MODE == 1) {
      float x = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) x += acc[i][j][0];
      if (x == 12345.f) p.C[0] = (bf16)x;
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int c = 0; c < 8; ++c) epi_chunk_rt<ACT>(p, acc, rc_cur, wr, wc, col0, lane, c);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) prev[i][j] = acc[i][j];
    }
    rc_prev = rc_cur;
    col0_prev = col0;
  }
  if constexpr (MODE == 0) {
#pragma unroll
    for (int c = 0; c < 8; ++c) epi_chunk_rt<ACT>(p, prev, rc_prev, wr, wc, col0_prev, lane, c);
  }
  if (wc == 0) raw_barrier();  // balance the stagger
}
}  // namespace d8

// fp32 reference: out = A B^T + bias (+ exact GELU), one thread per output
__global__ void ref_kernel(const bf16* A, const bf16* B, const float* bias, float* out, int M, int N, int K, int act) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = i / N, n = i % N;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long long)m * K + k] * (float)B[(long long)n * K + k];
  s += bias ? bias[n] : 0.f;
  if (act == 2) s = 0.5f * s * (1.f + erff(s * 0.70710678f));
  out[i] = s;
}
__global__ void fill_kernel(bf16* x, long long n, unsigned seed, float scale) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned h = (unsigned)i * 2654435761u ^ seed;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  x[i] = (bf16)(((h & 0xffffff) / 16777216.f * 2.f - 1.f) * scale);
}
__global__ void cmp_kernel(const bf16* c, const float* r, long long n, float* err) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float d = fabsf((float)c[i] - r[i]) / (fabsf(r[i]) + 0.05f);
  atomicMax((int*)err, __float_as_int(d));
}

template <int ACT, int MODE>
float run_d8(const d8::P& p, hipStream_t s, int iters) {
  auto k = d8::gemm8d_kernel<ACT, MODE>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, d8::LDS));
  const int grid = (p.ntiles + p.tpw - 1) / p.tpw;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), d8::LDS, s, p);
  CK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(512), d8::LDS, s, p);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  void* lib = dlopen("dilabhelmholtzoct_amd/liboctsam_hip.so", RTLD_NOW);
  typedef int (*gemm_fn)(const octsam_gemm_args*, void*);
  gemm_fn og = lib ? (gemm_fn)dlsym(lib, "octsam_gemm") : nullptr;
  if (!og) fprintf(stderr, "library gemm not found (%s)\n", dlerror());
  struct Shape {
    const char* name;
    int M, N, K, act;
  } shapes[] = {{"qkv", 32768, 2304, 768, 0}, {"fc1", 32768, 3072, 768, 2}};
  const int tpw_list[] = {2, 4, 8};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (auto& sh : shapes) {
    bf16 *A, *B, *C;
    float *bias, *ref, *err;
    CK(hipMalloc(&A, (size_t)sh.M * sh.K * 2));
    CK(hipMalloc(&B, (size_t)sh.N * sh.K * 2));
    CK(hipMalloc(&C, (size_t)sh.M * sh.N * 2));
    CK(hipMalloc(&bias, sh.N * 4));
    CK(hipMalloc(&ref, (size_t)sh.M * sh.N * 4));
    CK(hipMalloc(&err, 4));
    hipLaunchKernelGGL(fill_kernel, dim3((sh.M * (long long)sh.K + 255) / 256), dim3(256), 0, s, A,
                       (long long)sh.M * sh.K, 1u, 1.0f);
    hipLaunchKernelGGL(fill_kernel, dim3((sh.N * (long long)sh.K + 255) / 256), dim3(256), 0, s, B,
                       (long long)sh.N * sh.K, 2u, 1.0f / sqrtf((float)sh.K));
    std::vector<float> hb(sh.N);
    for (int i = 0; i < sh.N; ++i) hb[i] = 0.01f * (i % 97) - 0.4f;
    CK(hipMemcpy(bias, hb.data(), sh.N * 4, hipMemcpyHostToDevice));
    const long long n = (long long)sh.M * sh.N;
    hipLaunchKernelGGL(ref_kernel, dim3((n + 255) / 256), dim3(256), 0, s, A, B, bias, ref, sh.M, sh.N, sh.K, sh.act);
    CK(hipStreamSynchronize(s));
    const double fl = 2.0 * sh.M * sh.N * sh.K;
    auto check = [&](const char* tag) {
      CK(hipMemsetAsync(err, 0, 4, s));
      hipLaunchKernelGGL(cmp_kernel, dim3((n + 255) / 256), dim3(256), 0, s, C, ref, n, err);
      float e;
      CK(hipMemcpyAsync(&e, err, 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      return e;
    };
    for (int round = 0; round < 2; ++round) {
      if (og) {
        octsam_gemm_args a = {};
        a.A = A; a.B = B; a.C = C; a.bias = bias; a.M = sh.M; a.N = sh.N; a.K = sh.K; a.batch = 1;
        a.lda = sh.K; a.ldb = sh.K; a.ldc = sh.N; a.ldr = sh.N; a.alpha = 1.f; a.beta = 0.f; a.act = sh.act;
        CK(hipMemsetAsync(C, 0, n * 2, s));
        og(&a, s);
        const float e = check("lib");
        hipEvent_t x, y;
        CK(hipEventCreate(&x));
        CK(hipEventCreate(&y));
        CK(hipEventRecord(x, s));
        for (int i = 0; i < 20; ++i) og(&a, s);
        CK(hipEventRecord(y, s));
        CK(hipEventSynchronize(y));
        float ms;
        CK(hipEventElapsedTime(&ms, x, y));
        const float us = ms * 1e3f / 20;
        printf("{\"shape\": \"%s\", \"kernel\": \"library\", \"us\": %.1f, \"tf\": %.0f, \"maxrel\": %.4f}\n", sh.name, us,
               fl / us / 1e6, e);
      }
      for (int tpw : tpw_list) {
        d8::P p{A, B, C, bias, sh.M, sh.N, sh.K, sh.K, sh.K, sh.N, (sh.N + 127) / 128, 0, tpw};
        p.ntiles = ((sh.M + 255) / 256) * p.tiles_n;
        for (int mode = 0; mode < 3; ++mode) {
          CK(hipMemsetAsync(C, 0, n * 2, s));
          float us;
          if (sh.act == 2) us = mode == 0 ? run_d8<2, 0>(p, s, 20) : mode == 1 ? run_d8<2, 1>(p, s, 20) : run_d8<2, 2>(p, s, 20);
          else us = mode == 0 ? run_d8<0, 0>(p, s, 20) : mode == 1 ? run_d8<0, 1>(p, s, 20) : run_d8<0, 2>(p, s, 20);
          const float e = mode == 1 ? -1.f : check("d8");
          printf("{\"shape\": \"%s\", \"kernel\": \"d8\", \"mode\": %d, \"tpw\": %d, \"us\": %.1f, \"tf\": %.0f, "
                 "\"maxrel\": %.4f}\n", sh.name, mode, tpw, us, fl / us / 1e6, e);
          fflush(stdout);
        }
      }
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(bias)); CK(hipFree(ref)); CK(hipFree(err));
  }
  return 0;
}
