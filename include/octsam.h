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

#define OCTSAM_ABI_VERSION 24

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
 * repeat_interleave remaps (hf:modeling_sam.py:499-501): when *_blk > 0 the stored row of logical
 * row i is (i / (blk*rep)) * blk + i % blk for A rows (a_mode 0/4), B k-rows (b_mode 1/2) and
 * R rows, so per-image tensors are consumed per prompt without being replicated.
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
  int32_t a_blk, a_rep, b_blk, b_rep, r_blk, r_rep;
  /* k-major A and B (a_mode = b_mode = 1) batched as split-K over one [k_total][*] operand pair:
     batch b covers rows [b*K, (b+1)*K) and rows >= k_total read as zero (0 = no tail). */
  int32_t k_total;
  /* rows of C (and R) when row_map scatters the output; lets the 256x256 kernels use their lean epilogue
     (byte offsets range-checked against c_rows * ldc); 0 = unknown (general epilogue) */
  int32_t c_rows;
  /* column sums of the k-major operands (a_mode = b_mode = 1 only; fp32, NULL = none):
     a_colsum[b*M + m] = sum_k A[b][k][m], b_colsum[b*N + n] = sum_k B[b][k][n] per batch b (split), i.e. the
     bias gradient of a weight-gradient GEMM dW = dY^T X (A = dY), fused into the pass that reads dY; combine
     the splits with octsam_splitk_reduce. */
  float* a_colsum;
  float* b_colsum;
} octsam_gemm_args;

int octsam_gemm(const octsam_gemm_args* args, void* stream);
/* the same GEMM with IEEE-half 16-bit operands (A, B, and C / C_pre / R when not fp32): the fp16 encoder of
 * BASELINE configs[4] (sam-vit-huge, fp16) */
int octsam_gemm_f16(const octsam_gemm_args* args, void* stream);
/* enable (1, default) / disable (0) the persistent LDS-DMA 256x256 fast path of octsam_gemm (A/B testing);
   bit 256 disables the small-problem tile kernel, bit 512 the two-workgroups-per-CU 256x128 kernel, bit 8192 the
   ping-pong 256x256 kernel (the 8-phase one instead), bit 65536 the one-shot small-K kernel; bit 262144 turns on the
   opt-in 256x192 ping-pong tiles. Every path is a hand-written kernel of this library (ABI 24: the hipBLASLt path of
   ABI 23 and its octsam_gemm_set_workspace are gone). */
void octsam_gemm_set_fast_path(int32_t enable);
/* which kernel the calling thread's last octsam_gemm launched: 0 generic tile kernel, 1 persistent
   global_load_lds kernel, 2 8-phase / ping-pong / two-workgroup kernels, 3 small-problem kernel. Used to
   attribute per-kernel timings. */
int32_t octsam_gemm_last_path(void);
/* diagnostics: fast path 9 runs the one-tile-per-workgroup 8-phase kernel with per-workgroup s_memtime stamps
   (entry, main loop done, epilogue stores done) and hardware ids; this copies the first n_wg workgroups' records
   (4 x int64 each: t0, t1, t2, XCC_ID << 32 | HW_ID) to host memory (synchronous) */
int octsam_gemm_debug_stamps(int64_t* host, int32_t n_wg);

/* out[i] = sum_{s<splits} partials[s*n+i] + beta*out[i]  (fp32; deterministic split-K combine) */
int octsam_splitk_reduce(const float* partials, float* out, int64_t n, int32_t splits, float beta, void* stream);

/* Image-side weight gradient of the mask decoder (replaces the per-prompt image-side projections' and the ConvT1
 * weight-gradient GEMMs of the reference's autograd backward, hf modeling_sam.py:219-221/254 k/q/v/out_proj on the
 * keys and :1054 upscale_conv1 — dW = dY^T X over the P*4096 image rows):
 *   out[o][i] = beta*out[o][i] + sum_m dy[m*ldy + o] * x[m*ldx + i]              (bf16 operands, fp32 out)
 *   db[o] = sum_m dy[m*ldy + o];  dbx[c] = sum_m sum_t x[m*ldx + t*(I/dbx_fold) + c]   (optional, overwrite)
 * O in {128, 256, 384}, I in {128, 256} (octsam_wgrad_supported); ldy, ldx multiples of 8, dy / x / workspace
 * 16-B aligned. One workgroup per CU holds the whole O x I output and streams a contiguous row range (each operand
 * byte read once); per-workgroup partials are combined in fixed order (deterministic).
 * workspace: octsam_wgrad_workspace(M, O, I) bytes. */
int32_t octsam_wgrad_supported(int64_t M, int32_t O, int32_t I);
/* The token-side form (the P*T prompt-token rows of the decoder's token projections / MLPs / hypernetworks, M < 2^24):
 *   out[o][i] = beta*out[o][i] + sum_m dy[m*ldy + o] * x[m*ldx + i];  db[o] = sum_m dy[m*ldy + o] (optional)
 * in one launch (one 32x32 output tile per workgroup, its waves splitting the rows, fixed-order combine through LDS:
 * deterministic). O, I multiples of 32; ldy, ldx multiples of 8; dy, x 16-B aligned. */
int octsam_wgrad_tok(const void* dy, int64_t ldy, const void* x, int64_t ldx, int64_t M, int32_t O, int32_t I,
                     float* out, float beta, float* db, void* stream);
/* n (1..24) independent octsam_wgrad_tok problems in ONE launch (ABI 22; host arrays of n entries each, db[k] may be
 * NULL): the decoder backward defers its token-side weight gradients and issues them together. Problems of one call
 * must not share an output (out / db); each keeps octsam_wgrad_tok's arithmetic (same bits). */
int octsam_wgrad_tok_group(int32_t n, const void* const* dy, const int64_t* ldy, const void* const* x,
                           const int64_t* ldx, const int64_t* M, const int32_t* O, const int32_t* I, float* const* out,
                           const float* beta, float* const* db, void* stream);
int64_t octsam_wgrad_workspace(int64_t M, int32_t O, int32_t I);
int octsam_wgrad(const void* dy, int64_t ldy, const void* x, int64_t ldx, int64_t M, int32_t O, int32_t I, float* out,
                 float beta, float* db, float* dbx, int32_t dbx_fold, void* workspace, int64_t workspace_bytes,
                 void* stream);

/* ---------------------------------------------------------------- cubical persistence
 * Replaces torch_topological.nn.CubicalComplex(dim=2, superlevel=False)._forward ->
 * gudhi.CubicalComplex(dimensions=x.shape, top_dimensional_cells=x.flatten()).persistence()
 * + cofaces_of_persistence_pairs() (called at ref:octsam/models/topological_loss.py:55-63).
 * maps: fp32 [nmaps, H, W] (C order). For every map the kernel writes
 *   pairs0[map][i] = (creator pixel, destroyer pixel) of finite H0 pairs, i < counts[map*3+0]
 *   pairs1[map][i] = same for H1,                                        i < counts[map*3+1]
 *   essential[map] = (creator pixel of the essential H0 class, argmax pixel)
 *   counts[map*3+2] = 1 if a pair list overflowed max_pairs (the map is then incomplete); with
 *   max_pairs >= ceil(H*W/2) no map can overflow (finite H0 pairs <= ceil(H/2)*ceil(W/2), H1 pairs
 *   <= ceil(H*W/2): births at pairwise non-adjacent regional minima / deaths at regional maxima)
 * Pixel indices are C-order flat indices into the map, exactly the index space of
 * cofaces_of_persistence_pairs(). Pairs are ordered by decreasing persistence, ties by the
 * filtration order of the destroyer cell. Zero-persistence pairs are dropped (gudhi
 * min_persistence=0). Requires H,W >= 1, H*W <= 4096 and (H+1)*(W+1) + H*W <= 8192 (up to 64x63).
 */
int octsam_cubical_ph(const float* maps, int32_t nmaps, int32_t H, int32_t W, int32_t max_pairs,
                      int32_t* pairs0, int32_t* pairs1, int32_t* essential, int32_t* counts, void* stream);

/* ---------------------------------------------------------------- LayerNorm
 * Replaces nn.LayerNorm / SamLayerNorm (channels_first applied per pixel of NHWC data) of
 * SamVisionLayer (hf:modeling_sam.py:954-972), SamVisionNeck (:975-992), SamTwoWayAttentionBlock
 * (:306-348), SamTwoWayTransformer (:363, eps 1e-5) and the mask-decoder upscaling (:519-521).
 * Forward: y[r] = act(LN(x[src_rows ? src_rows[r] : r])) over the last dim D in {64,256,768,1024,1280};
 * a negative src_rows[r] writes a zero row (window_partition padding, :900-922). y is bf16 (y_f32 = 0), fp32
 * (y_f32 = 1) or fp16 (y_f32 = 2, the fp16 encoder); y2_f32 (optional) receives an fp32 copy; mean/rstd
 * (optional, fp32 [rows]) are saved.
 * Backward (D in {64,256,768}): dx = beta*dx + dLN (dx2_bf16 optional bf16 copy); per-block dw/db partials [nblocks, D] are written
 * to dw_part/db_part (combine with octsam_splitk_reduce). act must match the forward. */
int octsam_layernorm_fwd(const void* x, int32_t x_f32, const int32_t* src_rows, int64_t rows, int32_t D,
                         const float* w, const float* b, float eps, void* y, int32_t y_f32, float* y2_f32,
                         int32_t act, float* mean, float* rstd, void* stream);
int octsam_layernorm_bwd(const void* dy, int32_t dy_f32, const void* x, int32_t x_f32, const float* mean,
                         const float* rstd, const float* w, const float* b, int32_t act, int64_t rows, int32_t D,
                         void* dx, int32_t dx_f32, float beta, void* dx2_bf16, float* dw_part, float* db_part,
                         int32_t nblocks, void* stream);

/* ---------------------------------------------------------------- ViT attention
 * Replaces SamVisionAttention.forward + get_decomposed_rel_pos (hf:modeling_sam.py:729-882).
 * qkv: [nseq, side*side, 3*heads*head_dim] 16-bit (the qkv Linear output, column = part*D + head*head_dim + d);
 * out: [nseq, side*side, heads*head_dim], same type; rel_pos_h/w: fp32 [2*side-1, head_dim].
 * side = 64 (global layers, nseq = batch) or 14 (windowed layers, nseq = batch * 25 windows);
 * head_dim = 64 (vit-b / vit-l) or 80 (vit-h); fp16 = 1: IEEE half operands, else bf16.
 * softmax(q k^T / sqrt(head_dim) + rel_h + rel_w) v with fp32 statistics; the T x T bias is never
 * materialised. 16-B aligned operands.
 * grid = 0: windowed qkv / out are window-ordered (window_partition applied, padding rows present).
 * grid > 0 (side 14 only): qkv / out are token-ordered [images * grid * grid, ...] (no window_partition),
 * nseq = images * ceil(grid/14)^2; tokens past the grid read pad_row ([3*heads*head_dim], the qkv of a zero
 * row, i.e. the qkv bias) and their outputs are not written (window_unpartition drops them). */
int octsam_vit_attention(const void* qkv, void* out, const float* rel_pos_h, const float* rel_pos_w, int32_t nseq,
                         int32_t side, int32_t heads, int32_t head_dim, int32_t fp16, int32_t grid,
                         const void* pad_row, void* stream);
/* A/B switch for the global layers' kernel (all bit-identical): -1 (default) = 2 for head_dim 64, 1 for head_dim 80;
   1 = the plain per-tile loop of 8-wave workgroups; 2 = 4-wave workgroups, two per CU (vit-b 522.5 -> 498.6 us,
   profiles/r03/attn_variant_ab.log); 0 = software-pipelined (q.k of the next key tile beside the softmax of this one:
   measured no faster, profiles/r03/attn_pipelined_ab.log) */
void octsam_attention_set_variant(int32_t variant);

/* ---------------------------------------------------------------- element-wise / reductions / prompts */
/* out[i] = alpha*a[i] + beta*b[b_period ? i % b_period : i]  (a or b may be NULL = 0); out2_f32 optional copy.
 * e.g. image_embeddings + dense_prompt_embeddings (hf:modeling_sam.py:499, b_period = 256 channels). */
int octsam_axpby(const void* a, int32_t a_f32, const void* b, int32_t b_f32, int64_t b_period, float alpha, float beta,
                 void* out, int32_t out_f32, float* out2_f32, int64_t n, void* stream);
/* per-block column sums of x [rows, cols] into part [nblocks, cols] (bias gradients; combine with
 * octsam_splitk_reduce). */
int octsam_colsum(const void* x, int32_t x_f32, int64_t rows, int32_t cols, float* part, int32_t nblocks, void* stream);
/* SamPromptEncoder._embed_boxes / _embed_points (hf:modeling_sam.py:613-656) + the token concat of
 * SamMaskDecoder.forward (:489-496): tokens [P, 5 + nsparse, 256] fp32 = [iou, mask x4, sparse...].
 * boxes fp32 [P,4] (x0,y0,x1,y1 in the 1024 frame) and/or points fp32 [P,npts,2] with int32 labels
 * [P,npts] (NULL = all 1). nsparse = 2 (boxes), npts+1 (points, pad point added), npts+2 (both). */
int octsam_prompt_tokens(const float* boxes, const float* points, const int32_t* labels, int32_t P,
                         int32_t points_per_prompt, const float* pos_gauss, const float* point_embed,
                         const float* not_a_point, const float* out_tokens, float input_size, float* tokens,
                         void* stream);
/* SamMaskEmbedding.forward (hf:modeling_sam.py:569-592: the dense prompt of SamModel's input_masks): masks fp32
 * [B, 256, 256] -> out fp32 [B, 4096, 256] (pixel-major, the decoder's image-embedding layout). packed_weights fp32:
 * conv1 w [4][4] (out, ky*2+kx), b [4], layer_norm1 w [4], b [4], conv2 w [16][16] (out, in*4 + ky*2 + kx), b [16],
 * layer_norm2 w [16], b [16], conv3 w [256][16], b [256]; eps = layer_norm_eps. Forward only (the prompt encoder is
 * frozen on the reference's training path). */
int octsam_mask_embed(const float* masks, int32_t B, const float* packed_weights, float eps, float* out, void* stream);
/* SamModel.get_image_wide_positional_embeddings (hf:modeling_sam.py:1128-1139) as [size*size, 256]. */
int octsam_image_pe(const float* pos_gauss, int32_t size, float* out, void* stream);
/* dx bf16 [n] = dy fp32 [n] * (y > 0), y bf16 rows of stride ldy with `cols` columns (ReLU backward) */
int octsam_relu_bwd(const float* dy, const void* y, int64_t ldy, int32_t cols, void* dx, int64_t n, void* stream);
/* out bf16 [groups, rows_per, cols] = sum over nper consecutive blocks of in (bf16 rows of stride ld_in):
 * sums the per-prompt gradients of a tensor that was shared by the prompts of one image
 * (the backward of repeat_interleave, hf:modeling_sam.py:499-501). */
int octsam_group_sum(const void* in, int64_t ld_in, int32_t cols, int32_t groups, int32_t nper, int64_t rows_per,
                     void* out, void* stream);
/* bf16 / fp16 copy of an fp32 buffer */
int octsam_cast_bf16(const float* x, void* y, int64_t n, void* stream);
int octsam_cast_f16(const float* x, void* y, int64_t n, void* stream);
/* Patch-embedding operand: pixel_values fp32 [B, 3, 1024, 1024] -> bf16 [B*4096, 768], row = (b, py, px),
 * k = (c, ky, kx) (= Conv2d(3, D, 16, 16) weight.reshape(D, 768) order); replaces the gathered a_mode 2. */
int octsam_patchify_bf16(const float* px, int32_t B, void* out, void* stream);
int octsam_patchify_f16(const float* px, int32_t B, void* out, void* stream);  /* IEEE half rows */

/* ---------------------------------------------------------------- label components (A2)
 * SAMDataset._components (ref:octsam/models/training_utils.py:389-434: np.unique values, scipy.ndimage.label
 * with the 3x3 structure) on the GPU. octsam_cc_label: labels uint8 [B, H, W] (H*W < 2^24) -> parent int32
 * [B*H*W] (each pixel's root = first raster pixel of its 8-connected equal-value component) and, per image,
 * the unordered root keys (value << 24 | root index) in roots [B, max_roots] with their count in nroots [B]
 * (counts beyond max_roots are counted, not stored). The host sorts the keys: that is the reference's
 * component order. octsam_cc_assign: sorted_roots [B, maxc] root indices, ncomp [B] (<= maxc <= 1024) ->
 * comp int32 [B, H, W] = component rank of every pixel, stats int32 [B, maxc, 5] = (xmin, xmax, ymin,
 * ymax, pixel count); if gt != NULL also gt uint8 [B, N, H, W] = (comp == n) (H*W % 16 == 0, 16-B
 * aligned gt and comp). */
int octsam_cc_label(const uint8_t* labels, int32_t B, int32_t H, int32_t W, int32_t* parent, int32_t* roots,
                    int32_t max_roots, int32_t* nroots, void* stream);
int octsam_cc_assign(const int32_t* parent, int32_t B, int32_t H, int32_t W, const int32_t* sorted_roots,
                     int32_t maxc, const int32_t* ncomp, int32_t* comp, int32_t* stats, uint8_t* gt, int32_t N,
                     void* stream);

/* ---------------------------------------------------------------- image processor (A3)
 * SamProcessor image path (hf:image_processing_pil_sam.py:227-263 with Pillow's BILINEAR 8-bpc
 * ImagingResample): uint8 HWC RGB images [B, H, W, 3] (image b at images + b*img_stride) -> fp32 planar
 * [B, 3, out_h, out_w]: two-pass fixed-point resize to rh x rw, then lut[c*256 + v] (= rescale 1/255 and
 * (x - mean_c) / std_c in the processor's float arithmetic), zero padding outside rh x rw.
 * xtab [rw, 2 + kx] / ytab [rh, 2 + ky] int32 rows = (first source index, taps, kx (ky) weights of 22
 * fractional bits) as built by dilabhelmholtzoct_amd/preprocess.resample_table. Bit-exact with Pillow.
 * Requires 1 <= kx, ky <= 16, out_w % 4 == 0, out 16-B aligned, ky*W*3 <= 65536. */
int octsam_sam_preprocess(const uint8_t* images, int32_t B, int32_t H, int32_t W, int64_t img_stride,
                          const int32_t* xtab, int32_t kx, const int32_t* ytab, int32_t ky, int32_t rh,
                          int32_t rw, const float* lut, float* out, int32_t out_h, int32_t out_w, void* stream);

/* ---------------------------------------------------------------- mask decoder attention cores
 * SamAttention core softmax(q k^T / sqrt(dh)) v (hf:modeling_sam.py:231-270) for the three shapes of
 * SamTwoWayTransformer; projections are octsam_gemm. T, Tq, Tk <= 8; L = 4096 image tokens.
 * tok: q,k,v fp32 [P,T,256] (8 heads x 32) -> out bf16; probs fp32 [P,8,T,T] saved for backward.
 * t2i: q fp32 [P,Tq,128] (8 heads x 16); k,v bf16 rows of [.., L, ldkv], block p/kv_rep
 *      (kv_rep = prompts per image when K/V are per image); out bf16 [P,Tq,128]; lse fp32 [P,8,Tq].
 *      backward writes dq bf16 [P,Tq,128] and per-prompt dk, dv bf16 [P, L, lddkv]. Both take a caller-owned
 *      fp32 workspace of octsam_dec_t2i_workspace(P, L) elements (per-chunk partials); L % 32 == 0,
 *      k, v 16-B aligned, ldkv % 8 == 0, lddkv % 4 == 0.
 * i2t: q bf16 rows of [.., L, ldq], block p/q_rep; k,v fp32 [P,Tk,128]; out bf16 [P, L, ldo].
 *      backward writes dq bf16 [P, L, lddq] and partials fp32 [ceil(L/512), P, 2, Tk, 128] (dk; dv),
 *      reduce with octsam_splitk_reduce; octsam_dec_i2t_bwd_partials() gives the element count. */
int octsam_dec_tok_attn_fwd(const float* q, const float* k, const float* v, int32_t P, int32_t T, void* out,
                            float* probs, void* stream);
int octsam_dec_tok_attn_bwd(const float* q, const float* k, const float* v, const float* probs, const float* dout,
                            int32_t P, int32_t T, void* dq, void* dk, void* dv, void* stream);
int64_t octsam_dec_t2i_workspace(int32_t P, int32_t L);
int octsam_dec_t2i_fwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P, int32_t Tq,
                       int32_t L, void* out, float* lse, float* workspace, void* stream);
/* octsam_dec_t2i_fwd with score_bias fp32 [P][L] (16-B aligned, or null) added to every head's and token's logits
 * of each key: SamAttention's attention_similarity mask (hf:modeling_sam.py SamTwoWayAttentionBlock, the PerSAM
 * hook), forward only. */
int octsam_dec_t2i_fwd_bias(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                            int32_t Tq, int32_t L, const float* score_bias, void* out, float* lse, float* workspace,
                            void* stream);
int octsam_dec_t2i_bwd(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P, int32_t Tq,
                       int32_t L, const void* out, const float* dout, const float* lse, void* dq, void* dk, void* dv,
                       int64_t lddkv, float* workspace, void* stream);
/* octsam_dec_t2i_bwd for shared K / V (kv_rep prompts per image, the first two-way block) with the prompt sum fused
 * in: dk / dv are the IMAGE rows [(P / kv_rep) * L, lddkv] (bf16) = sum over the image's prompts of the per-prompt
 * gradients, accumulated in fp32 (replaces octsam_dec_t2i_bwd's per-prompt [P * L] rows + octsam_group_sum).
 * L % 64 == 0; fp32 workspace of octsam_dec_t2i_bwd_sum_workspace(P, Tq, L) elements (ABI 20). */
int64_t octsam_dec_t2i_bwd_sum_workspace(int32_t P, int32_t Tq, int32_t L);
int octsam_dec_t2i_bwd_sum(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                           int32_t Tq, int32_t L, const void* out, const float* dout, const float* lse, void* dq,
                           void* dk, void* dv, int64_t lddkv, float* workspace, void* stream);
/* The same three with the forward's unrounded O (ABI 21): octsam_dec_t2i_fwd2 also writes out_f32 fp32 [P,Tq,128]
 * (or null: = octsam_dec_t2i_fwd_bias); the backward variants take it for the row constant delta = dO . O (null: from
 * the bf16 out). The training step uses these: the backward's dP - delta cancels to the size of the softmax gradient,
 * and a bf16 O leaves delta's rounding at that size. All t2i backward variants split dO and dS into bf16 hi + lo. */
int octsam_dec_t2i_fwd2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                        int32_t Tq, int32_t L, const float* score_bias, void* out, float* out_f32, float* lse,
                        float* workspace, void* stream);
int octsam_dec_t2i_bwd2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                        int32_t Tq, int32_t L, const void* out, const float* out_f32, const float* dout,
                        const float* lse, void* dq, void* dk, void* dv, int64_t lddkv, float* workspace, void* stream);
int octsam_dec_t2i_bwd_sum2(const float* q, const void* k, const void* v, int64_t ldkv, int32_t kv_rep, int32_t P,
                            int32_t Tq, int32_t L, const void* out, const float* out_f32, const float* dout,
                            const float* lse, void* dq, void* dk, void* dv, int64_t lddkv, float* workspace,
                            void* stream);
int octsam_dec_i2t_fwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P, int32_t Tk,
                       int32_t L, void* out, int64_t ldo, void* stream);
int64_t octsam_dec_i2t_bwd_partials(int32_t P, int32_t Tk, int32_t L);
/* octsam_dec_i2t_bwd for queries shared by q_rep prompts per image (the first two-way block's image-side queries)
 * with the prompt sum of dQ fused in: dq holds the IMAGE rows [(P / q_rep) * L, lddq] = the sum over the image's
 * prompts, accumulated in fp32 (replaces the per-prompt [P * L] rows + octsam_group_sum). L % 64 == 0; dK / dV
 * partials as octsam_dec_i2t_bwd's, octsam_dec_i2t_bwd_sum_partials(P, Tk, L) elements (ABI 20). */
int64_t octsam_dec_i2t_bwd_sum_partials(int32_t P, int32_t Tk, int32_t L);
int octsam_dec_i2t_bwd_sum(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P,
                           int32_t Tk, int32_t L, const void* dout, int64_t lddo, void* dq, int64_t lddq,
                           float* partials, void* stream);
int octsam_dec_i2t_bwd(const void* q, int64_t ldq, int32_t q_rep, const float* k, const float* v, int32_t P, int32_t Tk,
                       int32_t L, const void* dout, int64_t lddo, void* dq, int64_t lddq, float* partials,
                       void* stream);

/* Fused upscaling tail + mask head (hf:modeling_sam.py:519-542: the second ConvTranspose2d, its GELU
 * and masks = hyper_in @ upscaled_embedding; replaces an octsam_gemm (conv2) + a separate mask product in the
 * training step): the 32-channel 256x256 upscaled embedding is never stored.
 * up1 bf16 [P*16384, 64] (LN+GELU output of the first ConvTranspose2d, blocked row order as above);
 * w2 bf16 [64, 128] = ConvT2 weight [in][(dy2, dx2, c)]; b2 fp32 [32]; hyper fp32 [P, ntok, 32];
 * ntok = 1 or 3; masks fp32 [P, ntok, 256, 256].
 * Backward recomputes the ConvT2 product and writes d up1 (bf16 [P*16384, 64]) and, overwriting,
 * d w2 fp32 [64, 128], d b2 fp32 [32], d hyper fp32 [P, ntok, 32] (fixed-order reductions).
 * workspace: octsam_upmask_bwd_workspace(P, ntok) floats, 16-B aligned. */
int octsam_upmask_fwd(const void* up1, const void* w2, const float* b2, const float* hyper, int32_t P, int32_t ntok,
                      float* masks, void* stream);
int64_t octsam_upmask_bwd_workspace(int32_t P, int32_t ntok);
/* tuning: persistent grid sizes of the two kernels (defaults 768 / 512; the backward is capped at 512) */
void octsam_upmask_set_grid(int32_t fwd, int32_t bwd);
int octsam_upmask_bwd(const void* up1, const void* w2, const float* b2, const float* hyper, const float* dmask,
                      int32_t P, int32_t ntok, void* dup1, float* dw2, float* db2, float* dhyper, float* workspace,
                      void* stream);
/* octsam_upmask_bwd with the LayerNorm2d(eps) + GELU in front of up1 (up1 = GELU(LN(x)), hf:modeling_sam.py:519-520)
 * differentiated in the same pass (replaces octsam_upmask_bwd + octsam_layernorm_bwd(act = GELU) over the 64-channel
 * rows: d up1 is never stored): x bf16 [P*16384, 64] the ConvT1 output, mean / rstd fp32 [P*16384] its LayerNorm
 * statistics (octsam_layernorm_fwd), ln_w / ln_b fp32 [64]; writes dx bf16 [P*16384, 64] and, overwriting, d w2, d b2,
 * d hyper, d ln_w, d ln_b fp32 (fixed-order reductions). Same workspace as octsam_upmask_bwd. */
int octsam_upmask_ln_bwd(const void* up1, const void* w2, const float* b2, const float* hyper, const float* dmask,
                         int32_t P, int32_t ntok, const void* x, const float* mean, const float* rstd, const float* ln_w,
                         const float* ln_b, void* dx, float* dw2, float* db2, float* dhyper, float* dln_w, float* dln_b,
                         float* workspace, void* stream);
/* octsam_upmask_ln_bwd with d x written at a row stride (row r of the [P * 4096, 256] view at dx + r * ldx, ldx >= 256,
 * a multiple of 4), so d x can be the left half of a wider operand (ABI 20) */
int octsam_upmask_ln_bwd_strided(const void* up1, const void* w2, const float* b2, const float* hyper,
                                 const float* dmask, int32_t P, int32_t ntok, const void* x, const float* mean,
                                 const float* rstd, const float* ln_w, const float* ln_b, void* dx, int64_t ldx,
                                 float* dw2, float* db2, float* dhyper, float* dln_w, float* dln_b, float* workspace,
                                 void* stream);

/* ---------------------------------------------------------------- post-processing + losses
 * octsam_postproc_fwd: ref:octsam/models/training_utils.py:57-59 — lowres fp32 [M,S,S] -> bilinear to
 *   mid x mid (align_corners=False) -> crop [:crop_h,:crop_w] -> bilinear to out_h x out_w, fused,
 *   torch upsample_bilinear2d index arithmetic. With gt (uint8 [M,out_h,out_w], binary) it also writes
 *   the Dice partial sums dice_part fp32 [M, nblk, 3] = (sum sigmoid(x)*t, sum t, sum sigmoid(x)).
 * octsam_dice_partials: the same partial sums for masks that are already post-processed (fp32 [M, HW],
 *   gt uint8 [M, HW]) -> dice_part [M, nblk, 3] (the drop-in DiceCELoss; M <= 65535).
 * octsam_confusion: per-map binary confusion counts (evaluate_metrics, ref:octsam/models/training_utils.py:
 *   126-156): counts uint64 [M, 4] = (tp, fp, fn, tn) of (masks > 0, i.e. sigmoid > 0.5) vs gt (overwritten).
 * octsam_dice_reduce: monai DiceLoss(sigmoid=True) per map (smooth 1e-5): dice_map double [M] and the
 *   gradient coefficients coef fp32 [M,2].
 * octsam_dicece_bwd: CrossEntropyLoss over the prompt dim N with probability targets + the Dice
 *   gradient: dmask fp32 [B,N,HW] = w_dice*dDice + w_ce*dCE; ce_part double [nblk].
 * octsam_loss_finalize: loss double [3] = (dice, ce, w_dice*dice + w_ce*ce).
 * octsam_postproc_bwd: dlowres = composite^T dout with CSR weight tables (cols: for each low-res
 *   column the (output column, weight) list; rows: likewise); tmp fp32 [M, out_h, S]. */
int octsam_postproc_fwd(const float* lowres, int32_t M, int32_t S, int32_t mid, int32_t crop_h, int32_t crop_w,
                        int32_t out_h, int32_t out_w, float* out, const uint8_t* gt, float* dice_part, int32_t nblk,
                        void* stream);
int octsam_dice_partials(const float* masks, const uint8_t* gt, int32_t M, int64_t HW, float* dice_part, int32_t nblk,
                         void* stream);
int octsam_confusion(const float* masks, const uint8_t* gt, int32_t M, int64_t HW, uint64_t* counts, void* stream);
int octsam_dice_reduce(const float* dice_part, int32_t M, int32_t nblk, double* dice_map, float* coef, void* stream);
int octsam_dicece_bwd(const float* masks, const uint8_t* gt, const float* coef, int32_t B, int32_t N, int64_t HW,
                      float w_dice, float w_ce, float* dmask, double* ce_part, int32_t nblk, void* stream);
int octsam_loss_finalize(const double* dice_map, int32_t M, const double* ce_part, int32_t nblk, int32_t B, int64_t HW,
                         double w_dice, double w_ce, double* loss, void* stream);
int octsam_postproc_bwd(const float* dout, int32_t M, int32_t S, int32_t out_h, int32_t out_w, const int32_t* col_ptr,
                        const int32_t* col_idx, const float* col_w, const int32_t* row_ptr, const int32_t* row_idx,
                        const float* row_w, float* tmp, float* dlowres, void* stream);
/* The DiceCE backward fused with the post-processing adjoint's row pass (ABI 19; the d-mask round trip of
 * octsam_dicece_bwd + octsam_postproc_bwd): one workgroup per (image, output row) forms d(DiceCE)/d mask for all N
 * prompts of the row (octsam_dicece_bwd's arithmetic) and writes tmp[m] rows (octsam_postproc_bwd's row pass) for
 * every map m = b * N + n with keep[m] < 0; keep[m] = k >= 0 writes the d-mask row to dkeep [K, H, W] instead (maps
 * whose topological gradient is added later: octsam_topo_bwd_compact, then octsam_pp_bwd_rows_maps into tmp).
 * ce_part double [B * H]; octsam_loss_finalize with nblk = B * H. keep may be NULL (every map). N <= 32.
 * octsam_pp_bwd_cols: the column pass of octsam_postproc_bwd on its own (tmp fp32 [M, out_h, S] -> dlowres). */
int octsam_dicece_pp_rows(const float* masks, const uint8_t* gt, const float* coef, int32_t B, int32_t N, int32_t H,
                          int32_t W, float w_dice, float w_ce, int32_t S, const int32_t* col_ptr, const int32_t* col_idx,
                          const float* col_w, const int32_t* keep, float* dkeep, float* tmp, double* ce_part,
                          void* stream);
int octsam_pp_bwd_rows_maps(const float* dout_k, const int32_t* map_idx, int32_t K, int32_t S, int32_t out_h,
                            int32_t out_w, const int32_t* col_ptr, const int32_t* col_idx, const float* col_w, float* tmp,
                            void* stream);
int octsam_pp_bwd_cols(const float* tmp, int32_t M, int32_t S, int32_t out_h, const int32_t* row_ptr,
                       const int32_t* row_idx, const float* row_w, float* dlowres, void* stream);

/* ---------------------------------------------------------------- topological loss (dense parts)
 * ref:octsam/models/topological_loss.py:33-46: pred = interp(f(masks[map_idx[k]]), out_h x out_w,
 * bilinear, align_corners=True) with f = sigmoid (training_utils.py:64) when apply_sigmoid, else identity;
 * gt_out likewise from uint8 gt; octsam_topo_bwd adds scale * d(interp o f)^T dpred into dmask.
 * Persistence: octsam_cubical_ph; Wasserstein: octsam_topo_w2 (device) or octsam_w2_host. */
int octsam_topo_down(const float* masks, const uint8_t* gt, const int32_t* map_idx, int32_t K, int32_t in_h,
                     int32_t in_w, int32_t out_h, int32_t out_w, int32_t apply_sigmoid, float* pred, float* gt_out,
                     void* stream);
int octsam_topo_bwd(const float* masks, const int32_t* map_idx, int32_t K, int32_t in_h, int32_t in_w, int32_t out_h,
                    int32_t out_w, int32_t apply_sigmoid, const float* dpred, float scale, float* dmask, void* stream);
/* octsam_topo_bwd into compact storage (ABI 19): dmask_k [K, in_h, in_w] holds the K maps themselves. */
int octsam_topo_bwd_compact(const float* masks, const int32_t* map_idx, int32_t K, int32_t in_h, int32_t in_w,
                            int32_t out_h, int32_t out_w, int32_t apply_sigmoid, const float* dpred, float scale,
                            float* dmask_k, void* stream);
/* HOST function (all pointers host): exact q-Wasserstein transport cost (before the 1/q power)
 * between diagrams d1 [n,2] and d2 [m,2] with L-inf ground metric and diagonal augmentation
 * (torch_topological WassersteinDistance -> POT ot.emd2, ref:octsam/models/topological_loss.py:78-82),
 * and d cost / d d1 [n,2]. */
int octsam_w2_host(const float* d1_host, int32_t n, const float* d2_host, int32_t m, double q, double* cost_host,
                   float* grad_d1_host);
/* The whole host half of topo_loss for one step: pairs [2Kn, max_pairs, 2] / cnt [2Kn, 3] / vals [2Kn, nvals]
 * as produced by octsam_cubical_ph on the Kn pred maps then the Kn gt maps; loss entries given as map lists
 * (entry_maps, CSR offsets entry_off [n_entries + 1]); feat_col 0 = H0, 1 = H1. Writes lamda * mean over
 * entries of (sum of the entry's W_q costs)^(1/q) and, if want_grad, d loss / d pred values dpred [Kn, nvals]
 * (topological_loss.py:68-96). Returns nonzero on bad arguments or a pair-buffer overflow. */
int octsam_topo_host(const int32_t* pairs, const int32_t* cnt, const float* vals, int32_t Kn, int32_t max_pairs,
                     int32_t nvals, const int32_t* entry_maps, const int32_t* entry_off, int32_t n_entries,
                     int32_t feat_col, double q, double lamda, int32_t want_grad, double* loss_out, float* dpred);

/* The same loss and gradient on the DEVICE: no host round trip between the step's forward
 * and backward. Inputs as octsam_topo_host (device pointers) plus map_entry [Kn] = the entry holding map k
 * (-1 = none). Writes loss_out[0] (NaN if a pair count exceeds max_pairs) and, if want_grad, dpred [Kn, nvals]
 * (every row written). Per map one wave solves the diagonal-augmented assignment with the host's
 * shortest-augmenting-path Hungarian method (lowest column on ties), so loss and gradient are bit-identical to
 * octsam_topo_host at q = 2. workspace: octsam_topo_w2_workspace(Kn, max_pairs) bytes.
 * Replaces torch_topological WassersteinDistance -> POT ot.emd2 + ref:octsam/models/topological_loss.py:68-96. */
int64_t octsam_topo_w2_workspace(int32_t Kn, int32_t max_pairs);
int octsam_topo_w2(const int32_t* pairs, const int32_t* cnt, const float* vals, int32_t Kn, int32_t max_pairs,
                   int32_t nvals, const int32_t* entry_maps, const int32_t* entry_off, const int32_t* map_entry,
                   int32_t n_entries, int32_t feat_col, double q, double lamda, int32_t want_grad, void* workspace,
                   int64_t workspace_bytes, double* loss_out, float* dpred, void* stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.Adam step over a flat fp32 buffer (ref:octsam/models/training_utils.py:31,68):
 * step_size = lr / (1 - beta1^t), bias_correction2_sqrt = sqrt(1 - beta2^t) computed by the caller;
 * params_bf16 (optional) receives the updated parameters in bf16. beta1/beta2 are double so that 1 - beta
 * is rounded to fp32 from the double difference, as torch forms it. */
int octsam_adam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, double beta1,
                double beta2, float eps, float weight_decay, float step_size, float bias_correction2_sqrt,
                void* params_bf16, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OCTSAM_H_ */
