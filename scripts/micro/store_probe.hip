// Probe: cost of writing a 256x256 bf16 tile per workgroup (1024 WGs, 512 threads) as a function of
// dynamic LDS (1 vs 2 WGs/CU) and store pattern. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(512) void store_tile(bf16* C, int N, int tiles_n, float v) {
  extern __shared__ char sm[];
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (MODE == 0) {  // 16 B per lane, 2 rows (512 B each) per wave-instruction
    for (int it = 0; it < 16; ++it) {
      int rr = it * 16 + wave * 2 + (lane >> 5);
      int c = (lane & 31) * 8;
      bf16x8 x;
      for (int e = 0; e < 8; ++e) x[e] = (bf16)(v + rr);
      *(bf16x8*)(C + (long long)(tm * 256 + rr) * N + tn * 256 + c) = x;
    }
  } else {  // 4 B per lane, MFMA-16x16-like pattern (8 rows x 32 B per instruction)
    const int wr = wave >> 2, wc = wave & 3;
    for (int mi = 0; mi < 8; ++mi)
      for (int ni = 0; ni < 4; ++ni)
        for (int t = 0; t < 2; ++t) {
          int row = tm * 256 + wr * 128 + mi * 16 + 4 * (lane >> 4) + 2 * t + (lane & 1);
          int col = tn * 256 + wc * 64 + ni * 16 + ((lane & 15) & ~1);
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
          bf16x2 x = {(bf16)v, (bf16)v};
          *(bf16x2*)(C + (long long)row * N + col) = x;
        }
  }
  if (v == 12345.f) sm[threadIdx.x] = 1;
}

int main() {
  const int M = 32768, N = 2048, tiles_n = N / 256, nwg = (M / 256) * tiles_n;
  bf16* C;
  hipMalloc(&C, (size_t)M * N * 2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode)
    for (int lds : {0, 65536, 133120}) {
      auto k = mode == 0 ? (void*)store_tile<0> : (void*)store_tile<1>;
      hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      for (int w = 0; w < 3; ++w) {
        if (mode == 0) hipLaunchKernelGGL(store_tile<0>, dim3(nwg), dim3(512), lds, 0, C, N, tiles_n, 1.0f);
        else hipLaunchKernelGGL(store_tile<1>, dim3(nwg), dim3(512), lds, 0, C, N, tiles_n, 1.0f);
      }
      hipEventRecord(a);
      for (int it = 0; it < 20; ++it) {
        if (mode == 0) hipLaunchKernelGGL(store_tile<0>, dim3(nwg), dim3(512), lds, 0, C, N, tiles_n, 1.0f);
        else hipLaunchKernelGGL(store_tile<1>, dim3(nwg), dim3(512), lds, 0, C, N, tiles_n, 1.0f);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ms /= 20;
      printf("{\"mode\": %d, \"lds\": %d, \"us\": %.1f, \"GBps\": %.0f}\n", mode, lds, ms * 1e3,
             (double)M * N * 2 / (ms * 1e-3) / 1e9);
    }
  return 0;
}
