// Probe of the LDS-DMA buffer load (16 B per lane) and ds_read_b64_tr_b16 as used by csrc/wgrad.hip: one wave
// DMAs a [8 rows][64 columns] bf16 tile (value = 256 row + column) into LDS with the wgrad stage layout (64-B rows,
// 512-B subtiles), dumps the LDS image, then every lane's transposed read at the wgrad fragment address.
// Build: hipcc --offload-arch=gfx950 -O2 tr_probe.hip -o tr_probe. Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__global__ void probe(const uint16_t* src, int ld, uint16_t* lds_dump, uint16_t* tr_out, uint16_t* g_out, int mode) {
  __shared__ __attribute__((aligned(16))) uint16_t img[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) img[i] = 0xffff;
  __syncthreads();
  const int st = lane >> 5, rr = (lane >> 2) & 7, slot = lane & 3;
  const int voff = rr * ld * 2 + 64 * st + 16 * slot;
  if (mode == 0) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 8 * ld * 2, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)img, 16, voff, 0, 0, 0);
  } else {
    __builtin_amdgcn_global_load_lds((const void*)((const char*)src + voff), (lds_ptr_t)img, 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 1024; i += 64) lds_dump[i] = img[i];
  // transposed read: lane 4q + p of each 16-lane group -> row q, columns 4p .. 4p + 3 of its 16-column block
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int off = 64 * q + 32 * (g & 1) + 8 * p + 512 * (g >> 1);  // groups 2, 3: the next subtile (columns 32..)
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)((char*)img + off));
  for (int j = 0; j < 4; ++j) tr_out[lane * 4 + j] = (uint16_t)v[j];
  // plain 8-byte read at the same address
  const uint64_t w = *(const uint64_t*)((const char*)img + off);
  for (int j = 0; j < 4; ++j) g_out[lane * 4 + j] = (uint16_t)(w >> (16 * j));
}

int main() {
  const int ld = 64;
  uint16_t h[8 * 64];
  for (int r = 0; r < 8; ++r)
    for (int c = 0; c < 64; ++c) h[r * ld + c] = (uint16_t)(256 * r + c);
  uint16_t *d, *dump, *tr, *gp;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&dump, 2048);
  hipMalloc(&tr, 512);
  hipMalloc(&gp, 512);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, ld, dump, tr, gp, mode);
    uint16_t hd[1024], ht[256], hg[256];
    hipMemcpy(hd, dump, 2048, hipMemcpyDeviceToHost);
    hipMemcpy(ht, tr, 512, hipMemcpyDeviceToHost);
    hipMemcpy(hg, gp, 512, hipMemcpyDeviceToHost);
    printf("mode %d (%s)\nLDS bytes 0..255 as (row,col): ", mode, mode ? "global_load_lds" : "buffer_load_lds");
    for (int k = 0; k < 128; ++k) printf("%d,%d ", hd[k] >> 8, hd[k] & 255);
    printf("\nLDS 512..: ");
    for (int k = 256; k < 288; ++k) printf("%d,%d ", hd[k] >> 8, hd[k] & 255);
    printf("\ntr reads (lane: 4 x (row,col)):\n");
    for (int l = 0; l < 64; ++l) {
      printf("L%02d:", l);
      for (int j = 0; j < 4; ++j) printf(" %d,%d", ht[l * 4 + j] >> 8, ht[l * 4 + j] & 255);
      printf(l % 4 == 3 ? "\n" : " |");
    }
    printf("plain reads lanes 0..7:");
    for (int l = 0; l < 8; ++l) {
      for (int j = 0; j < 4; ++j) printf(" %d,%d", hg[l * 4 + j] >> 8, hg[l * 4 + j] & 255);
      printf(" |");
    }
    printf("\n");
  }
  return 0;
}
