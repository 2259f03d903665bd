// Connected components of the label maps and the per-component prompt statistics on the GPU
// (SURVEY §8(f)1, row A2): SAMDataset._components / get_bboxes_and_gt_masks / get_points_and_gt_masks
// (ref:octsam/models/training_utils.py:389-434: for v in np.unique(label), scipy.ndimage.label of
// (label == v) with the 3x3 structure, components in label order) and the gt masks of custom_collate
// (:449-458), shipped as uint8 [B, N, H, W] instead of float64.
//
// scipy numbers the components of one value in raster order of their first pixel, and np.unique visits
// values in increasing order, so the reference's component order is the order of the key
// (value << 24 | first pixel index). Here:
//   1. octsam_cc_label: block union-find over the 8-neighbourhood (each pixel unites with its W, NW, N, NE
//      neighbours of equal value; roots are hooked onto the smaller root with atomicMin, so every component
//      ends rooted at its first raster pixel): each workgroup labels a 32 x 64 tile in LDS (LDS atomics,
//      local indices are raster-monotone, so the local root is the tile's first pixel of the component) and
//      writes global parents; a second pass unites only the pixels whose neighbours lie in another tile
//      (lock-free, global atomicMin); one flatten pass then also emits the key of every root into a per-image
//      list (unordered, counted).
//   2. the host sorts each image's keys (a few dozen) -> component order;
//   3. octsam_cc_assign: scatter the rank to the root pixels, give every pixel its root's rank, and reduce
//      (xmin, xmax, ymin, ymax, pixel count) per component through LDS atomics into global atomics;
//      optional gt writer gt[b][n][p] = (rank[b][p] == n) with 16-B stores.
// Only vector-memory atomics are used. Integer work, HBM/latency-bound: 1 B in + 4 B of ranks per pixel.
#include "common.h"
#include "../../include/octsam.h"

namespace {

constexpr int CC_MAXC = 1024;  // components per image (LDS statistics table)

__device__ __forceinline__ int ld_relaxed(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int find_root(const int* P, int x) {
  int p = ld_relaxed(P + x);
  while (p != x) {
    x = p;
    p = ld_relaxed(P + x);
  }
  return x;
}

__device__ __forceinline__ void unite(int* P, int a, int b) {
  while (true) {
    a = find_root(P, a);
    b = find_root(P, b);
    if (a == b) return;
    if (a > b) {
      const int t = a;
      a = b;
      b = t;
    }
    // hook root b onto the smaller root a; if b stopped being a root meanwhile, retry from there
    const int old = atomicMin(P + b, a);
    if (old == b) return;
    b = old;
  }
}

constexpr int TH = 32, TW = 64, TPIX = TH * TW;  // label tile (2048 pixels, 8 per thread)

__device__ __forceinline__ int lds_ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

__device__ __forceinline__ int lfind(const int* lp, int x) {
  int p = lds_ld(lp + x);
  while (p != x) {
    x = p;
    p = lds_ld(lp + x);
  }
  return x;
}

__device__ __forceinline__ void lunite(int* lp, int a, int b) {
  while (true) {
    a = lfind(lp, a);
    b = lfind(lp, b);
    if (a == b) return;
    if (a > b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicMin(lp + b, a);
    if (old == b) return;
    b = old;
  }
}

// one workgroup per (32 x 64 tile, image): union-find of the tile in LDS, then parent[p] = global index of the
// pixel's tile-local root (roots point to themselves)
__global__ __launch_bounds__(256) void cc_tile_kernel(const uint8_t* __restrict__ lab, int H, int W,
                                                      int* __restrict__ parent, int* __restrict__ nroots) {
  __shared__ int lp[TPIX];
  __shared__ uint8_t lv[TPIX];
  const int b = blockIdx.y, tiles_x = (W + TW - 1) / TW;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  const int x0 = tx * TW, y0 = ty * TH;
  const long long hw = (long long)H * W;
  const uint8_t* L = lab + b * hw;
  if (blockIdx.x == 0 && threadIdx.x == 0) nroots[b] = 0;
  for (int l = threadIdx.x; l < TPIX; l += 256) {
    const int y = y0 + l / TW, x = x0 + l % TW;
    lp[l] = l;
    lv[l] = (y < H && x < W) ? L[(long long)y * W + x] : 0;
  }
  __syncthreads();
  for (int l = threadIdx.x; l < TPIX; l += 256) {
    const int ly = l / TW, lx = l % TW, y = y0 + ly, x = x0 + lx;
    if (y >= H || x >= W) continue;
    const uint8_t v = lv[l];
    if (lx > 0 && lv[l - 1] == v) lunite(lp, l, l - 1);
    if (ly > 0) {
      if (lx > 0 && lv[l - TW - 1] == v) lunite(lp, l, l - TW - 1);
      if (lv[l - TW] == v) lunite(lp, l, l - TW);
      if (lx + 1 < TW && x + 1 < W && lv[l - TW + 1] == v) lunite(lp, l, l - TW + 1);
    }
  }
  __syncthreads();
  int* P = parent + b * hw;
  for (int l = threadIdx.x; l < TPIX; l += 256) {
    const int y = y0 + l / TW, x = x0 + l % TW;
    if (y >= H || x >= W) continue;
    const int r = lfind(lp, l);
    P[(long long)y * W + x] = (y0 + r / TW) * W + x0 + r % TW;
  }
}

// the neighbour pairs that cross a tile boundary, united in the global forest
__global__ __launch_bounds__(256) void cc_border_kernel(const uint8_t* __restrict__ lab, int H, int W,
                                                        int* __restrict__ parent) {
  const int hw = H * W;
  const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= hw) return;
  const int y = i / W, x = i - y * W;
  const bool left = x > 0 && x % TW == 0, top = y > 0 && y % TH == 0, right = x % TW == TW - 1 && x + 1 < W;
  if (!left && !top && !(right && y > 0)) return;
  const uint8_t* L = lab + (long long)b * hw;
  int* P = parent + (long long)b * hw;
  const uint8_t v = L[i];
  if (left && L[i - 1] == v) unite(P, i, i - 1);
  if (y > 0) {
    if (x > 0 && (left || top) && L[i - W - 1] == v) unite(P, i, i - W - 1);
    if (top && L[i - W] == v) unite(P, i, i - W);
    if (x + 1 < W && (right || top) && L[i - W + 1] == v) unite(P, i, i - W + 1);
  }
}

__global__ __launch_bounds__(256) void cc_flatten_kernel(const uint8_t* __restrict__ lab, int hw,
                                                         int* __restrict__ parent, int* __restrict__ roots,
                                                         int max_roots, int* __restrict__ nroots) {
  const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (i >= hw) return;
  int* P = parent + (long long)b * hw;
  const int r = find_root(P, i);
  if (r == i) {
    const int slot = atomicAdd(nroots + b, 1);
    if (slot < max_roots) roots[(long long)b * max_roots + slot] = ((int)lab[(long long)b * hw + i] << 24) | i;
  } else {
    P[i] = r;  // path to the final root (only shortens other threads' walks)
  }
}

__global__ __launch_bounds__(256) void cc_scatter_kernel(const int* __restrict__ sorted_roots, int maxc,
                                                         const int* __restrict__ ncomp, int hw,
                                                         int* __restrict__ comp, int* __restrict__ stats) {
  const int n = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (n >= maxc) return;
  int* s = stats + ((long long)b * maxc + n) * 5;
  s[0] = 0x7fffffff;
  s[1] = -1;
  s[2] = 0x7fffffff;
  s[3] = -1;
  s[4] = 0;
  if (n < ncomp[b]) comp[(long long)b * hw + sorted_roots[(long long)b * maxc + n]] = n;
}

__global__ __launch_bounds__(256) void cc_rank_kernel(const int* __restrict__ parent, int H, int W, int maxc,
                                                      const int* __restrict__ ncomp, int* __restrict__ comp,
                                                      int* __restrict__ stats) {
  __shared__ int st[CC_MAXC * 5];
  const int hw = H * W, b = blockIdx.y;
  const int nc = ncomp[b];
  for (int j = threadIdx.x; j < nc; j += 256) {
    st[j * 5 + 0] = 0x7fffffff;
    st[j * 5 + 1] = -1;
    st[j * 5 + 2] = 0x7fffffff;
    st[j * 5 + 3] = -1;
    st[j * 5 + 4] = 0;
  }
  __syncthreads();
  const int* P = parent + (long long)b * hw;
  int* C = comp + (long long)b * hw;
  constexpr int PER = 8;
  const int base = blockIdx.x * 256 * PER;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int i = base + e * 256 + threadIdx.x;
    if (i >= hw) break;
    const int r = P[i];
    const int n = C[r];  // roots hold their rank (scatter pass); a root reads its own slot
    if ((unsigned)n >= (unsigned)nc) continue;  // (host contract broken: never index LDS out of range)
    if (r != i) C[i] = n;
    const int y = i / W, x = i - y * W;
    atomicMin(&st[n * 5 + 0], x);
    atomicMax(&st[n * 5 + 1], x);
    atomicMin(&st[n * 5 + 2], y);
    atomicMax(&st[n * 5 + 3], y);
    atomicAdd(&st[n * 5 + 4], 1);
  }
  __syncthreads();
  int* S = stats + (long long)b * maxc * 5;
  for (int j = threadIdx.x; j < nc; j += 256) {
    if (st[j * 5 + 4] == 0) continue;
    atomicMin(&S[j * 5 + 0], st[j * 5 + 0]);
    atomicMax(&S[j * 5 + 1], st[j * 5 + 1]);
    atomicMin(&S[j * 5 + 2], st[j * 5 + 2]);
    atomicMax(&S[j * 5 + 3], st[j * 5 + 3]);
    atomicAdd(&S[j * 5 + 4], st[j * 5 + 4]);
  }
}

// gt[b][n][p] = comp[b][p] == n, 16 pixels per thread (hw % 16 == 0: 16-B loads/stores)
__global__ __launch_bounds__(256) void cc_gt_kernel(const int* __restrict__ comp, int hw, int N,
                                                    uint8_t* __restrict__ gt) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.z, n = blockIdx.y;
  const int p0 = (int)t * 16;
  if (p0 >= hw) return;
  const int4* c4 = (const int4*)(comp + (long long)b * hw + p0);
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int4 c = c4[q];
    w[q] = (uint32_t)(c.x == n) | ((uint32_t)(c.y == n) << 8) | ((uint32_t)(c.z == n) << 16) |
           ((uint32_t)(c.w == n) << 24);
  }
  *(uint4*)(gt + ((long long)b * N + n) * hw + p0) = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace

extern "C" int octsam_cc_label(const uint8_t* labels, int32_t B, int32_t H, int32_t W, int32_t* parent,
                               int32_t* roots, int32_t max_roots, int32_t* nroots, void* stream) {
  OCTSAM_CHECK_ARG(labels && parent && roots && nroots && B > 0 && H > 0 && W > 0 && max_roots > 0,
                   "octsam_cc_label: bad args");
  OCTSAM_CHECK_ARG((long long)H * W < (1LL << 24), "octsam_cc_label: %d x %d pixels exceed 2^24", H, W);
  hipStream_t s = (hipStream_t)stream;
  const int hw = H * W;
  const dim3 grid((hw + 255) / 256, B);
  const int ntiles = ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
  hipLaunchKernelGGL(cc_tile_kernel, dim3(ntiles, B), dim3(256), 0, s, labels, H, W, parent, nroots);
  hipLaunchKernelGGL(cc_border_kernel, grid, dim3(256), 0, s, labels, H, W, parent);
  hipLaunchKernelGGL(cc_flatten_kernel, grid, dim3(256), 0, s, labels, hw, parent, roots, max_roots, nroots);
  OCTSAM_LAUNCH_CHECK("octsam_cc_label");
  return 0;
}

extern "C" int octsam_cc_assign(const int32_t* parent, int32_t B, int32_t H, int32_t W, const int32_t* sorted_roots,
                                int32_t maxc, const int32_t* ncomp, int32_t* comp, int32_t* stats, uint8_t* gt,
                                int32_t N, void* stream) {
  OCTSAM_CHECK_ARG(parent && sorted_roots && ncomp && comp && stats && B > 0 && H > 0 && W > 0,
                   "octsam_cc_assign: bad args");
  OCTSAM_CHECK_ARG(maxc >= 1 && maxc <= CC_MAXC, "octsam_cc_assign: maxc must be in [1, %d] (got %d)", CC_MAXC,
                   maxc);
  const int hw = H * W;
  OCTSAM_CHECK_ARG(!gt || (N >= 1 && hw % 16 == 0 && ((uintptr_t)gt & 15) == 0 && ((uintptr_t)comp & 15) == 0),
                   "octsam_cc_assign: gt needs N >= 1, H*W %% 16 == 0 and 16-B aligned gt / comp");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cc_scatter_kernel, dim3((maxc + 255) / 256, B), dim3(256), 0, s, sorted_roots, maxc, ncomp, hw,
                     comp, stats);
  hipLaunchKernelGGL(cc_rank_kernel, dim3((hw + 2047) / 2048, B), dim3(256), 0, s, parent, H, W, maxc, ncomp, comp,
                     stats);
  if (gt) hipLaunchKernelGGL(cc_gt_kernel, dim3((hw / 16 + 255) / 256, N, B), dim3(256), 0, s, comp, hw, N, gt);
  OCTSAM_LAUNCH_CHECK("octsam_cc_assign");
  return 0;
}
