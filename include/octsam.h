/*
 * octsam.h — C ABI of liboctsam_hip.so, the MI355X (gfx950) implementation of the
 * OCT-SAM training step hot path (philippendres/DILabHelmholtzOCT,
 * octsam/models/training_utils.py:41-69).
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer unless the name ends in `_host`.
 *   - `stream` is a hipStream_t (void* here so the header has no HIP dependency);
 *     all work is stream-ordered, nothing synchronises the device.
 *   - Return value: 0 on success, otherwise a hipError_t or 1 for an argument error;
 *     octsam_last_error() returns the thread-local message. No C++ exception crosses the ABI.
 *   - The library allocates no device memory; callers pass workspaces sized by the
 *     *_workspace_bytes() queries.
 *   - bf16 tensors are raw IEEE bfloat16 (uint16 storage).
 *
 * Each entry point names the reference interface it replaces (file:line). "hf:" paths are
 * transformers/models/sam/ (the reference pins transformers 4.36.2, environment.yml:251);
 * "ref:" paths are under the reference repository.
 */
#ifndef OCTSAM_H_
#define OCTSAM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCTSAM_ABI_VERSION 1

#define OCTSAM_ACT_NONE 0
#define OCTSAM_ACT_RELU 1
#define OCTSAM_ACT_GELU 2

/* ---------------------------------------------------------------- library */
int octsam_abi_version(void);
const char* octsam_last_error(void);

/* ---------------------------------------------------------------- GEMM
 * Replaces every nn.Linear / Conv2d(k16,s16) / Conv2d(1x1) / Conv2d(3x3) / ConvTranspose2d(k2,s2)
 * product of SamModel (hf:modeling_sam.py:128, :132-143, :231-270, :843-882, :985-992, :519-521)
 * and their weight/input gradients.
 *   C[b][m][n] = epi(alpha * sum_k A[b][m][k] * B[b][n][k])
 * a_mode: 0 = A[m*lda+k] (bf16), 1 = A[k*lda+m] (bf16), 2 = im2col 16x16/s16 of fp32 NCHW
 *         pixels [B,3,1024,1024] (K=768, k=(c,kh,kw)), 3 = im2col 3x3/pad1 of bf16 NHWC
 *         [B,64,64,conv_c] (K=9*conv_c, k=(ky,kx,c)), 4 = like 0 plus A2[(m % a2_rows)*lda+k]
 * b_mode: 0 = B[n*ldb+k] (bf16), 1 = B[k*ldb+n] (bf16), 2 = like 1 plus B2[(k % b2_rows)*ldb+n]
 * epilogue: v = alpha*acc + beta*C_old + bias[n]; C_pre = v (optional); v = act(v);
 *           v += R[m*ldr+n] (optional); C = v.  row_map (optional, int32 [M]) redirects output
 *           row m to row_map[m] (skipped when < 0) for C, C_pre and R.
 */
typedef struct octsam_gemm_args {
  const void* A;
  const void* B;
  void* C;
  const float* bias;     /* fp32 [N] or NULL */
  const void* R;         /* residual, fp32 or bf16, or NULL */
  void* C_pre;           /* pre-activation output or NULL */
  const int32_t* row_map;/* int32 [M] or NULL */
  const void* A2;        /* broadcast addend for a_mode 4 */
  const void* B2;        /* broadcast addend for b_mode 2 */
  int32_t M, N, K, batch;
  int64_t lda, ldb, ldc, ldr;
  int64_t stride_a, stride_b, stride_c, stride_r; /* batch strides in elements */
  float alpha, beta;
  int32_t act;
  int32_t a_mode, b_mode;
  int32_t c_f32, r_f32, pre_f32; /* 1 = fp32 storage, 0 = bf16 */
  int32_t conv_c;
  int32_t a2_rows, b2_rows;
} octsam_gemm_args;

int octsam_gemm(const octsam_gemm_args* args, void* stream);

/* out[i] = sum_{s<splits} partials[s*n+i] + beta*out[i]  (fp32; deterministic split-K combine) */
int octsam_splitk_reduce(const float* partials, float* out, int64_t n, int32_t splits, float beta, void* stream);

/* ---------------------------------------------------------------- cubical persistence
 * Replaces torch_topological.nn.CubicalComplex(dim=2, superlevel=False)._forward ->
 * gudhi.CubicalComplex(dimensions=x.shape, top_dimensional_cells=x.flatten()).persistence()
 * + cofaces_of_persistence_pairs() (called at ref:octsam/models/topological_loss.py:55-63).
 * maps: fp32 [nmaps, H, W] (C order). For every map the kernel writes
 *   pairs0[map][i] = (creator pixel, destroyer pixel) of finite H0 pairs, i < counts[map*3+0]
 *   pairs1[map][i] = same for H1,                                        i < counts[map*3+1]
 *   essential[map] = (creator pixel of the essential H0 class, argmax pixel)
 *   counts[map*3+2] = 1 if a pair list overflowed max_pairs (the map is then incomplete)
 * Pixel indices are C-order flat indices into the map, exactly the index space of
 * cofaces_of_persistence_pairs(). Pairs are ordered by decreasing persistence, ties by the
 * filtration order of the destroyer cell. Zero-persistence pairs are dropped (gudhi
 * min_persistence=0). Requires H*W <= 4096 and H,W >= 1.
 */
int octsam_cubical_ph(const float* maps, int32_t nmaps, int32_t H, int32_t W, int32_t max_pairs,
                      int32_t* pairs0, int32_t* pairs1, int32_t* essential, int32_t* counts, void* stream);

/* ---------------------------------------------------------------- LayerNorm
 * Replaces nn.LayerNorm / SamLayerNorm (channels_first applied per pixel of NHWC data) of
 * SamVisionLayer (hf:modeling_sam.py:954-972), SamVisionNeck (:975-992), SamTwoWayAttentionBlock
 * (:306-348), SamTwoWayTransformer (:363, eps 1e-5) and the mask-decoder upscaling (:519-521).
 * Forward: y[r] = act(LN(x[src_rows ? src_rows[r] : r])) over the last dim D in {64,256,768,1024,1280};
 * a negative src_rows[r] writes a zero row (window_partition padding, :900-922). y is bf16 or fp32
 * (y_f32); y2_f32 (optional) receives an fp32 copy; mean/rstd (optional, fp32 [rows]) are saved.
 * Backward (D in {64,256,768}): dx = beta*dx + dLN; per-block dw/db partials [nblocks, D] are written
 * to dw_part/db_part (combine with octsam_splitk_reduce). act must match the forward. */
int octsam_layernorm_fwd(const void* x, int32_t x_f32, const int32_t* src_rows, int64_t rows, int32_t D,
                         const float* w, const float* b, float eps, void* y, int32_t y_f32, float* y2_f32,
                         int32_t act, float* mean, float* rstd, void* stream);
int octsam_layernorm_bwd(const void* dy, int32_t dy_f32, const void* x, int32_t x_f32, const float* mean,
                         const float* rstd, const float* w, const float* b, int32_t act, int64_t rows, int32_t D,
                         void* dx, int32_t dx_f32, float beta, float* dw_part, float* db_part, int32_t nblocks,
                         void* stream);

/* ---------------------------------------------------------------- ViT attention
 * Replaces SamVisionAttention.forward + get_decomposed_rel_pos (hf:modeling_sam.py:729-882).
 * qkv: bf16 [nseq, side*side, 3*heads*64] (the qkv Linear output, column = part*D + head*64 + d);
 * out: bf16 [nseq, side*side, heads*64]; rel_pos_h/w: fp32 [2*side-1, 64].
 * side = 64 (global layers, nseq = batch) or 14 (windowed layers, nseq = batch * 25 windows).
 * softmax(q k^T / 8 + rel_h + rel_w) v with fp32 statistics; the T x T bias is never materialised. */
int octsam_vit_attention(const void* qkv, void* out, const float* rel_pos_h, const float* rel_pos_w, int32_t nseq,
                         int32_t side, int32_t heads, int32_t head_dim, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OCTSAM_H_ */
