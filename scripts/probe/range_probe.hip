// Does the raw-buffer range check of an LDS-DMA buffer load include soffset? num_records = 4 rows of a [8][64] bf16
// tile; lanes read rows 0..7 with the row offset in voffset (A) or in soffset (B: rows 4..7 via soffset = 4 rows).
// Build: hipcc --offload-arch=gfx950 -O2 range_probe.hip -o range_probe. Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__global__ void probe(const uint16_t* src, uint16_t* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint16_t img[512];
  const int lane = threadIdx.x;
  for (int i = lane; i < 512; i += 64) img[i] = 0xffff;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 4 * 128, 0x00020000);
  // lane l: row l >> 3 (0..7), chunk l & 7 (16 B each): 1 KiB = the whole tile
  const int row = lane >> 3, ch = lane & 7;
  if (mode == 0) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)img, 16, row * 128 + ch * 16, 0, 0, 0);
  } else {
    // rows 0..3 of the tile = lanes 0..31 in voffset; the other lanes the same offsets, + soffset 4 rows
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)img, 16, (row & 3) * 128 + ch * 16, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(img + 256), 16, (row & 3) * 128 + ch * 16, 4 * 128, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 512; i += 64) out[i] = img[i];
}

int main() {
  uint16_t h[512];
  for (int i = 0; i < 512; ++i) h[i] = (uint16_t)(i / 64 + 1);  // row + 1 (never 0)
  uint16_t *d, *o;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&o, sizeof(h));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, mode);
    uint16_t r[512];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    printf("mode %d (%s): first element of rows 0..7 in LDS:", mode, mode ? "rows 4-7 via soffset" : "rows via voffset");
    for (int row = 0; row < 8; ++row) printf(" %d", (int)r[row * 64]);
    printf("   (0 = range-checked to zero, row+1 = loaded)\n");
  }
  return 0;
}
