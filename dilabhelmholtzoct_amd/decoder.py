"""SamMaskDecoder forward + backward on liboctsam_hip.so (hf:modeling_sam.py:273-543).

The decoder is the only trainable part of the step (ref:octsam/models/training_utils.py:31,277-279).
Its parameters live in ONE flat fp32 buffer (fp32 master weights; ``flat_b16`` bf16 operand copy;
``flat_grad``), laid out so that projections applied to the same input are adjacent and run as one
GEMM ([t2i.k | i2t.q | t2i.v] per block, [final.k | final.v]); ConvTranspose2d weights are stored as
[c_in][dy][dx][c_out] so the two upscaling convolutions are plain GEMMs whose outputs stay in a
"blocked" pixel order (see upmask.hip). The nn.Parameters HF code and checkpoints see are views of
that buffer (the ConvT ones permuted views), so state_dict keys/shapes are HF's.

Layer 0 shares the per-image tensors across the image's prompts (repeat_interleave at
hf:modeling_sam.py:499-501 is never materialised): keys/values/queries projected from
image_embeddings + dense are computed once per image; gradients of those projections are summed
over prompts (octsam_group_sum) before the weight-gradient GEMM.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch
import torch.nn as nn

from . import kernels as K
from ._lib import ACT_GELU, ACT_RELU
from .config import DecoderConfig

L_IMG = 4096  # 64 x 64 image tokens
C = 256
CI = 128


class Attention(nn.Module):
    def __init__(self, hidden=256, downsample=1):
        super().__init__()
        internal = hidden // downsample
        self.q_proj = nn.Linear(hidden, internal)
        self.k_proj = nn.Linear(hidden, internal)
        self.v_proj = nn.Linear(hidden, internal)
        self.out_proj = nn.Linear(internal, hidden)


class MLPBlock(nn.Module):
    def __init__(self, d, mlp):
        super().__init__()
        self.lin1 = nn.Linear(d, mlp)
        self.lin2 = nn.Linear(mlp, d)


class TwoWayBlock(nn.Module):
    def __init__(self, cfg: DecoderConfig):
        super().__init__()
        h = cfg.hidden_size
        self.self_attn = Attention(h, 1)
        self.layer_norm1 = nn.LayerNorm(h, eps=cfg.layer_norm_eps)
        self.cross_attn_token_to_image = Attention(h, cfg.attention_downsample_rate)
        self.layer_norm2 = nn.LayerNorm(h, eps=cfg.layer_norm_eps)
        self.mlp = MLPBlock(h, cfg.mlp_dim)
        self.layer_norm3 = nn.LayerNorm(h, eps=cfg.layer_norm_eps)
        self.layer_norm4 = nn.LayerNorm(h, eps=cfg.layer_norm_eps)
        self.cross_attn_image_to_token = Attention(h, cfg.attention_downsample_rate)


class TwoWayTransformer(nn.Module):
    def __init__(self, cfg: DecoderConfig):
        super().__init__()
        self.layers = nn.ModuleList([TwoWayBlock(cfg) for _ in range(cfg.num_hidden_layers)])
        self.final_attn_token_to_image = Attention(cfg.hidden_size, cfg.attention_downsample_rate)
        self.layer_norm_final_attn = nn.LayerNorm(cfg.hidden_size)  # eps 1e-5 (hf:modeling_sam.py:363)


class FeedForward(nn.Module):
    def __init__(self, din, dh, dout, num_layers):
        super().__init__()
        self.proj_in = nn.Linear(din, dh)
        self.proj_out = nn.Linear(dh, dout)
        self.layers = nn.ModuleList([nn.Linear(dh, dh) for _ in range(num_layers - 2)])


def _flat_order(nl: int, n_mask_tokens: int) -> list[str]:
    o = ["iou_token.weight", "mask_tokens.weight"]
    for l in range(nl):
        p = f"transformer.layers.{l}."
        sa, t2i, i2t = p + "self_attn.", p + "cross_attn_token_to_image.", p + "cross_attn_image_to_token."
        o += [sa + f"{n}_proj.weight" for n in ("q", "k", "v", "out")]
        o += [sa + f"{n}_proj.bias" for n in ("q", "k", "v", "out")]
        o += [t2i + "k_proj.weight", i2t + "q_proj.weight", t2i + "v_proj.weight"]  # GEMM group
        o += [t2i + "k_proj.bias", i2t + "q_proj.bias", t2i + "v_proj.bias"]
        o += [t2i + "q_proj.weight", t2i + "q_proj.bias", t2i + "out_proj.weight", t2i + "out_proj.bias"]
        o += [i2t + "k_proj.weight", i2t + "k_proj.bias", i2t + "v_proj.weight", i2t + "v_proj.bias",
              i2t + "out_proj.weight", i2t + "out_proj.bias"]
        o += [p + "mlp.lin1.weight", p + "mlp.lin1.bias", p + "mlp.lin2.weight", p + "mlp.lin2.bias"]
        o += [p + f"layer_norm{i}.{w}" for i in range(1, 5) for w in ("weight", "bias")]
    f = "transformer.final_attn_token_to_image."
    o += [f + "k_proj.weight", f + "v_proj.weight", f + "k_proj.bias", f + "v_proj.bias",
          f + "q_proj.weight", f + "q_proj.bias", f + "out_proj.weight", f + "out_proj.bias",
          "transformer.layer_norm_final_attn.weight", "transformer.layer_norm_final_attn.bias"]
    o += ["upscale_conv1.weight", "upscale_conv1.bias", "upscale_conv2.weight", "upscale_conv2.bias",
          "upscale_layer_norm.weight", "upscale_layer_norm.bias"]
    for i in range(n_mask_tokens):
        h = f"output_hypernetworks_mlps.{i}."
        o += [h + "proj_in.weight", h + "proj_in.bias", h + "layers.0.weight", h + "layers.0.bias",
              h + "proj_out.weight", h + "proj_out.bias"]
    o += ["iou_prediction_head.proj_in.weight", "iou_prediction_head.proj_in.bias",
          "iou_prediction_head.layers.0.weight", "iou_prediction_head.layers.0.bias",
          "iou_prediction_head.proj_out.weight", "iou_prediction_head.proj_out.bias"]
    return o


_CONVT = ("upscale_conv1.weight", "upscale_conv2.weight")


class MaskDecoder(nn.Module):
    """SamMaskDecoder parameters + HIP forward/backward."""

    def __init__(self, cfg: DecoderConfig):
        super().__init__()
        self.config = cfg
        h = cfg.hidden_size
        self.num_mask_tokens = cfg.num_multimask_outputs + 1
        self.iou_token = nn.Embedding(1, h)
        self.mask_tokens = nn.Embedding(self.num_mask_tokens, h)
        self.transformer = TwoWayTransformer(cfg)
        self.upscale_conv1 = nn.ConvTranspose2d(h, h // 4, kernel_size=2, stride=2)
        self.upscale_conv2 = nn.ConvTranspose2d(h // 4, h // 8, kernel_size=2, stride=2)
        self.upscale_layer_norm = nn.LayerNorm(h // 4, eps=1e-6)
        self.output_hypernetworks_mlps = nn.ModuleList(
            [FeedForward(h, h, h // 8, 3) for _ in range(self.num_mask_tokens)])
        self.iou_prediction_head = FeedForward(h, cfg.iou_head_hidden_dim, self.num_mask_tokens, cfg.iou_head_depth)
        self._order = _flat_order(cfg.num_hidden_layers, self.num_mask_tokens)
        self.flat = None
        self.flat_b16 = None
        self.flat_grad = None
        self.reflatten()

    # ------------------------------------------------------------------ flat parameter storage
    def _modules_params(self):
        named = dict(nn.Module.named_parameters(self))
        assert set(named) == set(self._order), sorted(set(named) ^ set(self._order))
        return named

    def reflatten(self):
        """(Re)build the flat buffer on the parameters' current device and re-point every parameter
        at a view of it. Called at construction and after .to()/.cuda()/.float()."""
        named = self._modules_params()
        dev = next(iter(named.values())).device
        regions = {}
        off = 0
        for name in self._order:
            p = named[name]
            n = p.numel()
            regions[name] = (off, n, tuple(p.shape))
            off += (n + 7) // 8 * 8
        flat = torch.zeros(off, device=dev, dtype=torch.float32)
        for name in self._order:
            o, n, shape = regions[name]
            src = named[name].detach().float()
            if name in _CONVT:  # [ci, co, 2, 2] -> storage [ci, 2, 2, co]
                src = src.permute(0, 2, 3, 1)
            flat[o:o + n].copy_(src.reshape(-1))
        self._regions = regions
        base = flat.detach()
        for name in self._order:
            mod_name, _, pname = name.rpartition(".")
            mod = self.get_submodule(mod_name)
            mod._parameters[pname] = nn.Parameter(self._param_view(base, name),
                                                  requires_grad=named[name].requires_grad)
        # the autograd leaf of the decoder: MaskDecoderFn returns the flat gradient for it
        self.flat = flat.requires_grad_(True)
        self.flat_grad = None
        self.flat_b16 = torch.empty(off, device=dev, dtype=torch.bfloat16)
        self.sync_bf16()

    def _param_view(self, flat, name):
        o, n, shape = self._regions[name]
        v = flat[o:o + n]
        if name in _CONVT:
            ci, co = shape[0], shape[1]
            return v.view(ci, 2, 2, co).permute(0, 3, 1, 2)
        return v.view(shape)

    @torch.no_grad()
    def sync_bf16(self):
        if self.flat is None:
            return
        if self.flat.is_cuda:
            K.cast_bf16(self.flat, self.flat_b16)
        else:
            self.flat_b16.copy_(self.flat.to(torch.bfloat16))

    def ensure_grad(self):
        if self.flat_grad is None or self.flat_grad.device != self.flat.device:
            self.flat_grad = torch.zeros_like(self.flat)
        return self.flat_grad

    def bind_param_grads(self):
        """Expose flat_grad slices as .grad of every parameter (so torch optimizers also work)."""
        g = self.ensure_grad()
        for name in self._order:
            mod_name, _, pname = name.rpartition(".")
            p = self.get_submodule(mod_name)._parameters[pname]
            if p.requires_grad:
                p.grad = self._param_view(g, name)

    def _storage(self, buf, name, rows=None):
        o, n, shape = self._regions[name]
        v = buf[o:o + n]
        if name in _CONVT:
            ci, co = shape[0], shape[1]
            return v.view(ci, 4 * co)
        if rows is not None:
            return v.view(rows, -1)
        return v.view(shape) if len(shape) != 1 else v

    def _group(self, buf, names, cols):
        o0 = self._regions[names[0]][0]
        n = sum(self._regions[nm][1] for nm in names)
        for a, b in zip(names, names[1:]):
            assert self._regions[a][0] + self._regions[a][1] == self._regions[b][0], (a, b)
        return buf[o0:o0 + n].view(-1, cols) if cols else buf[o0:o0 + n]

    def W(self, name):
        return self._storage(self.flat_b16, name)

    def Bf(self, name):
        return self._storage(self.flat, name)

    def G(self, name):
        return self._storage(self.flat_grad, name)

    def output_tokens_f32(self):
        return self._group(self.flat, ["iou_token.weight", "mask_tokens.weight"], 0)

    # ------------------------------------------------------------------ forward entry
    def run(self, emb, pe, tokens, no_mask_weight, multimask_output: bool, target_embedding=None,
            attention_similarity=None):
        """emb fp32 [B, 4096, 256]; pe fp32 [4096, 256]; tokens fp32 [B, N, T, 256] ->
        (pred_masks [B, N, k, 256, 256], iou_scores [B, N, k]). target_embedding: broadcastable to the tokens;
        attention_similarity: broadcastable to [B*N, 1, 1, 4096], added to the token->image logits of the two
        transformer layers (hf's PerSAM hooks; forward only)."""
        tgt = None if target_embedding is None else target_embedding.detach()
        sim = None if attention_similarity is None else attention_similarity.detach()
        return MaskDecoderFn.apply(self.flat, emb, pe, tokens, no_mask_weight.detach(), self, bool(multimask_output),
                                   tgt, sim)

    # ------------------------------------------------------------------ helpers
    def _lin(self, x, wname, bname, out, M, *, act=0, residual=None, r_remap=(0, 1), a_mode=0, A2=None,
             a2_rows=0, lda=None, ldc=None, pre_out=None, wgroup=None, bgroup=None):
        w = self.W(wname) if wgroup is None else self._group(self.flat_b16, wgroup, C)
        b = self.Bf(bname) if bgroup is None else self._group(self.flat, bgroup, 0)
        if a_mode == 4 and act == 0 and residual is None and pre_out is None:
            # (x + pe[m % L]) W^T + b = x W^T + P[m % L] with P = pe W^T + b (L x N, computed once): the
            # big product runs on the K-contiguous fast path, P enters as a periodic residual
            N = w.shape[0]
            P = torch.empty(a2_rows, N, device=out.device, dtype=torch.bfloat16)
            K.gemm(A2, w, M=a2_rows, N=N, K=w.shape[1], out=P, bias=b, lda=lda)
            K.gemm(x, w, M=M, N=N, K=w.shape[1], out=out, residual=P, ldr=N, r_remap=(a2_rows, max(1, M // a2_rows)),
                   lda=lda, ldc=ldc)
            return out
        K.gemm(x, w, M=M, N=w.shape[0], K=w.shape[1], out=out, bias=b, act=act, residual=residual, r_remap=r_remap,
               a_mode=a_mode, A2=A2, a2_rows=a2_rows, lda=lda, ldc=ldc, pre_out=pre_out)
        return out

    def _proj_pe(self, src_b, wnames, bnames, n_pe, out, M):
        """out = src @ W^T + b + [pe @ W[:n_pe]^T | 0] for the grouped weights W (rows [k | q' | v]): the
        keys + key-PE projections and the plain value projection of the same image-side input in ONE GEMM
        over the M (= P*4096) rows; the PE enters as a row-periodic residual P[m % 4096] (P's first n_pe
        columns = pe W^T + b, the rest = b), so the big product runs on the K-contiguous fast path."""
        w = self._group(self.flat_b16, wnames, C)
        b = self._group(self.flat, bnames, 0)
        N = w.shape[0]
        P = torch.empty(L_IMG, N, device=out.device, dtype=torch.bfloat16)
        K.gemm(self._pe_b, w[:n_pe], M=L_IMG, N=n_pe, K=C, out=P, bias=b[:n_pe], ldc=N)
        P[:, n_pe:].copy_(b[n_pe:].to(torch.bfloat16).expand(L_IMG, N - n_pe))
        K.gemm(src_b, w, M=M, N=N, K=C, out=out, residual=P, ldr=N, r_remap=(L_IMG, max(1, M // L_IMG)), ldc=N)
        return out

    # image-side weight gradients through octsam_wgrad (False: the split-K tile GEMM + reduction; A/B,
    # scripts/dw_ab.py / scripts/step_ab3.py)
    wide_wgrad = True
    # token-side weight + bias gradients through octsam_wgrad_tok (False: split-K tile GEMM + reduction + column-sum
    # kernel + reduction; A/B, scripts/step_ab3.py)
    tok_wgrad = True
    # the first block's attention backwards with the prompt sums of their image-shared operands' gradients fused in
    # (token->image K / V: octsam_dec_t2i_bwd_sum; image->token Q: octsam_dec_i2t_bwd_sum; False: per-prompt gradients
    # + octsam_group_sum; A/B, scripts/step_ab3.py)
    t2i_sum = True
    # the keys gradient of the mask head and the final attention as one product over [d up1pre | dK | dV] (True;
    # False: two products, the second read-modify-writing d keys2): 16.15 -> 16.09 ms per step (round 4). On the
    # sixteen-pair val-Dice protocol with the oracle-made warm start it is indistinguishable from the two-product form
    # (mean differences -0.0023 / +0.0077 / +0.0008 at steps 32 / 48 / 64 against -0.0019 / +0.0065 / -0.0012,
    # standard errors 0.001 / 0.004 / 0.003; profiles/r05/valdice_variants.log); A/B: scripts/step_ab3.py
    fuse_dkeys = True
    # LayerNorm2d + GELU backward of the upscaling fused into the mask-head backward (octsam_upmask_ln_bwd; False:
    # octsam_upmask_bwd writes d up1, octsam_layernorm_bwd reads it back; A/B, scripts/step_ab3.py)
    fused_ln_bwd = True

    # the backward's token-side weight gradients (octsam_wgrad_tok, ~18 us each, latency-bound, 29 per vit-b step)
    # deferred to the end of backward() and issued as grouped launches (octsam_wgrad_tok_group; False: one launch
    # each). A problem whose output overlaps a pending one's flushes the group first (the x_add / positional
    # accumulations), and so does an in-place write into a tensor a pending problem reads (_before_write: d s4, which
    # each block's projection backward accumulates into once its out_proj backward has read it).
    tok_group = True
    # flush the deferred group at the end of every two-way block as well (its operands still warm in L2 / MALL) instead
    # of only when a group is full or blocked: pipelined 15.85 -> 15.71 ms, sequential 18.08 -> 18.08
    # (scripts/step_ab3.py, profiles/r06/tok_flush_ab.log; one launch per weight instead: 15.77 / 18.17)
    tok_flush_block = True
    _tok_pending = None

    @staticmethod
    def _span(t):
        """Byte range a (possibly strided) view touches."""
        n = 1 + sum((d - 1) * st for d, st in zip(t.shape, t.stride())) if t.numel() else 0
        return t.data_ptr(), t.data_ptr() + n * t.element_size()

    def _defer_tok(self, prob):
        dy, x, out, db = prob[0], prob[1], prob[3], prob[7]
        spans = [self._span(out)] + ([self._span(db)] if db is not None else [])
        busy = self._tok_spans
        if any(a < d and c < b for a, b in spans for c, d in busy) or len(self._tok_pending) == K.TOK_GROUP_MAX:
            self._flush_tok()
        self._tok_pending.append(prob)
        self._tok_spans.extend(spans)
        self._tok_reads.extend([self._span(dy), self._span(x)])

    def _before_write(self, t):
        """t is about to be written in place: the deferred products that read it run first."""
        if self._tok_pending:
            a, b = self._span(t)
            if any(a < d and c < b for c, d in self._tok_reads):
                self._flush_tok()

    def _flush_tok(self):
        if self._tok_pending:
            K.wgrad_tok_group(self._tok_pending)
        self._tok_pending = [] if self._tok_pending is not None else None
        self._tok_spans, self._tok_reads = [], []

    @staticmethod
    def _pick_split(Mtok, O, I):
        """Split-K (splits, rows per split) for a weight gradient with Mtok reduction rows: enough (O x I tiles)
        x splits to fill the chip. Mtok % 64 == 0: splits divide Mtok into multiples of 64 rows. Ragged Mtok
        (token-side rows, e.g. P*7): 64-row multiples, the last split's tail zero-filled (k_total)."""
        tiles = -(-O // 256) * -(-I // 128)
        if Mtok % 64:
            want = max(1, min(-(-Mtok // 64), -(-128 // tiles)))
            ks = 64 * -(-Mtok // (64 * want))
            return -(-Mtok // ks), ks
        best = 1
        for s in range(1, 513):
            if Mtok % s:
                continue
            ch = Mtok // s
            if ch < 32:
                break
            if ch % 64:
                continue
            best = s
            if tiles * s >= 256:
                break
        return best, Mtok // best

    def _dw(self, dy, x, M, out, *, ldy=None, ldx=None, x_add=None, x_add_rows=0, split=None, accumulate=False,
            db=None, dbx=None, dbx_fold=1):
        """out[o, i] (+)= sum_m dy[m, o] * (x[m, i] (+ x_add[m % rows, i])) -> fp32 (deterministic split-K).
        The periodic addend (the image PE added to the keys) is folded as dy^T x + S^T x_add with
        S[p] = sum_j dy[j*rows + p], so the big product is a plain k-major GEMM.
        db (optional, fp32 [O]) = sum_m dy[m, o] and dbx (fp32 [I / dbx_fold]) = sum_m x[m, i] folded over
        dbx_fold column groups: the bias gradients, summed inside the GEMM's pass over dy / x (image-side
        weight gradients; both overwrite)."""
        O, I = out.shape
        ldy = O if ldy is None else ldy
        ldx = I if ldx is None else ldx
        if x_add is not None:
            rows = x_add_rows
            S = torch.empty(rows, O, device=out.device, dtype=torch.bfloat16)
            K.group_sum(dy, S, ld_in=ldy, cols=O, groups=1, nper=M // rows, rows_per=rows)
            self._dw(dy, x, M, out, ldy=ldy, ldx=ldx, accumulate=accumulate, db=db, dbx=dbx, dbx_fold=dbx_fold)
            self._dw(S, x_add, rows, out, ldy=O, ldx=ldx, accumulate=True)
            return out
        beta = 1.0 if accumulate else 0.0
        tok = (split is None and self.tok_wgrad and M < 65536 and dbx is None and O % 32 == 0 and I % 32 == 0
               and ldy % 8 == 0 and ldx % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0
               and out.is_contiguous())
        if not tok and self._tok_pending:
            # an immediate product must not overtake a deferred one into the same gradient
            spans = [self._span(t) for t in (out, db, dbx) if t is not None]
            if any(a < d and c < b for a, b in spans for c, d in self._tok_spans):
                self._flush_tok()
        if (split is None and self.wide_wgrad and M >= 65536 and K.wgrad_supported(M, O, I) and ldy % 8 == 0
                and ldx % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0 and out.is_contiguous()):
            # image side: one workgroup per CU holds the whole O x I output and streams its rows (octsam_wgrad)
            K.wgrad(dy, x, M, out, ldy=ldy, ldx=ldx, beta=beta, db=db, dbx=dbx, dbx_fold=dbx_fold)
            return out
        if tok:
            # token side (and image-side products over fewer rows): weight and bias gradient in one launch
            # (octsam_wgrad_tok); inside backward() deferred and issued in groups (octsam_wgrad_tok_group)
            if self._tok_pending is not None:
                self._defer_tok((dy, x, M, out, ldy, ldx, beta, db))
            else:
                K.wgrad_tok(dy, x, M, out, ldy=ldy, ldx=ldx, beta=beta, db=db)
            return out
        if split is None:
            split, Ks = self._pick_split(M, O, I)
        else:
            Ks = M // split
        dev = out.device
        if db is not None and M < 65536:  # (the small-problem tile kernel has no fused column sums)
            # (dy may be a column slice of a wider buffer, e.g. dKV_img[:, CI:] at ldy = 2*CI: address it by stride)
            K.colsum(dy if ldy == O else torch.as_strided(dy, (M, O), (ldy, 1)).contiguous(), M, O, db)
            db = None
        pa = torch.empty((split, O), device=dev, dtype=torch.float32) if db is not None else None
        pb = torch.empty((split, I), device=dev, dtype=torch.float32) if dbx is not None else None
        if split == 1 and Ks == M:
            K.gemm(dy, x, M=O, N=I, K=M, out=out, a_mode=1, b_mode=1, lda=ldy, ldb=ldx, beta=beta,
                   a_colsum=pa, b_colsum=pb)
        else:
            part = torch.empty((split, O, I), device=dev, dtype=torch.float32)
            K.gemm(dy, x, M=O, N=I, K=Ks, out=part, a_mode=1, b_mode=1, lda=ldy, ldb=ldx, batch=split,
                   stride_a=Ks * ldy, stride_b=Ks * ldx, stride_c=O * I, k_total=M if Ks * split != M else 0,
                   a_colsum=pa, b_colsum=pb)
            K.splitk_reduce(part.view(split, -1), out, split, beta=beta)
        if pa is not None:
            K.splitk_reduce(pa, db, split)
        if pb is not None:
            K.splitk_reduce(pb.view(split * dbx_fold, -1), dbx, split * dbx_fold)
        return out

    def _dw_pe(self, dy, x, M, out, n_pe, pe_b, db=None, ldy=None):
        """Weight gradient of _proj_pe: out[o, i] = sum_m dy[m, o] x[m, i] for every grouped row o (one
        k-major GEMM over the M rows), plus sum_p S[p, o] pe[p, i] for the first n_pe rows, S[p] = sum_j
        dy[j*4096 + p] (the PE term); db (optional) = sum_m dy[m, o], fused into the GEMM."""
        O = out.shape[0]
        ldy = O if ldy is None else ldy
        self._dw(dy, x, M, out, ldy=ldy, db=db)
        S = torch.empty(L_IMG, n_pe, device=out.device, dtype=torch.bfloat16)
        K.group_sum(dy, S, ld_in=ldy, cols=n_pe, groups=1, nper=M // L_IMG, rows_per=L_IMG)
        self._dw(S, pe_b, L_IMG, out[:n_pe], ldy=n_pe, accumulate=True)
        return out

    @staticmethod
    def _dx(dy_b, w, M, out, *, ldy=None, beta=0.0, ldc=None):
        """out (+)= dy @ w for w [O, I] bf16. Image-sized M: the NT fast path on a transposed copy of the
        (small) weight, the accumulation as an in-place residual; token-sized M: the k-major B path."""
        O, I = w.shape
        ldy = O if ldy is None else ldy
        if M >= 65536 and beta in (0.0, 1.0):
            ldc_ = I if ldc is None else ldc
            K.gemm(dy_b, w.t().contiguous(), M=M, N=I, K=O, out=out, lda=ldy, ldc=ldc_,
                   residual=out if beta == 1.0 else None, ldr=ldc_)
        else:
            K.gemm(dy_b, w, M=M, N=I, K=O, out=out, b_mode=1, lda=ldy, ldb=I, beta=beta, ldc=ldc)
        return out

    def _lin_bwd(self, dy_b, x_b, wname, bname, M, *, dx_out=None, dx_beta=0.0, ldy=None, ldx=None, x_add=None,
                 x_add_rows=0, wgroup=None, bgroup=None, ldc=None):
        """Backward of y = x W^T + b: dx (optional, accumulate with dx_beta), dW, db."""
        if wgroup is None:
            w = self.W(wname)
            gw = self.G(wname)
        else:
            w = self._group(self.flat_b16, wgroup, C)
            gw = self._group(self.flat_grad, wgroup, C)
        O, I = w.shape
        ldy = O if ldy is None else ldy
        if dx_out is not None:
            self._dx(dy_b, w, M, dx_out, ldy=ldy, beta=dx_beta, ldc=ldc)
        gb = self.G(bname) if bgroup is None else self._group(self.flat_grad, bgroup, 0)
        # the bias gradient rides on the weight gradient's pass over dy (image side: octsam_wgrad's column sums; token
        # side: octsam_wgrad_tok)
        self._dw(dy_b, x_b, M, gw, ldy=ldy, ldx=ldx, x_add=x_add, x_add_rows=x_add_rows, db=gb)

    def _ln(self, x, prefix, eps, rows, *, f32_out=True):
        w, b = self.Bf(prefix + ".weight"), self.Bf(prefix + ".bias")
        dev = x.device
        yb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16)
        yf = torch.empty(rows, C, device=dev, dtype=torch.float32) if f32_out else None
        mean = torch.empty(rows, device=dev, dtype=torch.float32)
        rstd = torch.empty(rows, device=dev, dtype=torch.float32)
        K.layernorm_fwd(x, w, b, eps, yb, out2_f32=yf, mean=mean, rstd=rstd)
        return yf, yb, (x, mean, rstd, prefix)

    def _ln_bwd(self, dy, saved, *, dx_f32=True, want_b16=True):
        x, mean, rstd, prefix = saved
        rows = mean.numel()
        dev = dy.device
        dx = torch.empty(rows, C, device=dev, dtype=torch.float32 if dx_f32 else torch.bfloat16)
        dxb = torch.empty(rows, C, device=dev, dtype=torch.bfloat16) if (want_b16 and dx_f32) else None
        K.layernorm_bwd(dy, x, mean, rstd, self.Bf(prefix + ".weight"), self.Bf(prefix + ".bias"), dx,
                        dx2_bf16=dxb, dw=self.G(prefix + ".weight"), db=self.G(prefix + ".bias"))
        return dx, (dxb if dx_f32 else dx)

    def _bf(self, x):
        out = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
        K.cast_bf16(x.contiguous(), out)
        return out

    def _add_b16(self, a, b):
        out = torch.empty(a.shape, device=a.device, dtype=torch.bfloat16)
        K.axpby(a, b, out)
        return out

    # ------------------------------------------------------------------ forward
    def forward_impl(self, emb, pe, tokens, no_mask, multimask, target=None, similarity=None):
        cfg = self.config
        B, N, T, _ = tokens.shape
        P, R = B * N, B * N * T
        L = L_IMG
        RL = P * L
        dev = emb.device
        eps = cfg.layer_norm_eps
        f32, b16 = torch.float32, torch.bfloat16
        s = SimpleNamespace(B=B, N=N, T=T, P=P, R=R, L=L, RL=RL, multimask=multimask)
        tr = "transformer."

        tok0 = tokens.reshape(R, C).contiguous()
        tgt = None
        if target is not None:
            # hf SamTwoWayTransformer: `queries += target_embedding` before every layer; the first add is in place
            # on point_embeddings itself, so the query positional embedding of every layer (and of the final
            # attention) is tokens + target as well
            tgt = target.to(device=dev, dtype=torch.float32).expand(B, N, T, C).reshape(R, C).contiguous()
            t0 = torch.empty_like(tok0)
            K.axpby(tok0, tgt, t0)
            tok0 = t0
        s.tok0 = tok0
        sbias = None
        if similarity is not None:
            sim = similarity.to(device=dev, dtype=torch.float32)
            if sim.dim() != 4 or sim.shape[1] != 1 or sim.shape[2] != 1 or sim.shape[3] != L or sim.shape[0] not in (1, P):
                raise ValueError(f"attention_similarity must broadcast as [B*N, 1, 1, {L}] (heads and tokens "
                                 f"shared), got {tuple(sim.shape)}")
            sbias = sim.reshape(-1, L).expand(P, L).contiguous()
        s.similarity = sbias is not None
        s.tok0_b = self._bf(tok0)
        imgd = torch.empty(B * L, C, device=dev, dtype=f32)
        imgd_b = torch.empty(B * L, C, device=dev, dtype=b16)
        # image_embeddings + dense: no_mask_embed [1, C] broadcast, or a mask prompt's embedding [B, L, C]
        dense = no_mask.float().contiguous()
        if dense.numel() not in (C, B * L * C):
            raise ValueError("dense prompt embedding must be [1, C] or [B, 4096, C]")
        K.axpby(emb, dense, imgd_b, b_period=C if dense.numel() == C else 0, out2_f32=imgd)
        s.imgd, s.imgd_b = imgd, imgd_b
        pe_b = self._bf(pe)
        s.pe_b = pe_b
        self._pe_b = pe_b
        s.layers = []
        queries, queries_b = None, None
        keys_b = None
        for li in range(cfg.num_hidden_layers):
            pre = tr + f"layers.{li}."
            sa, t2i, i2t = pre + "self_attn.", pre + "cross_attn_token_to_image.", pre + "cross_attn_image_to_token."
            ls = SimpleNamespace()
            if tgt is not None and li > 0:  # queries += target_embedding (layer 0: folded into tok0 above)
                qn, qb = torch.empty_like(queries), torch.empty(R, C, device=dev, dtype=b16)
                K.axpby(queries, tgt, qb, out2_f32=qn)
                queries, queries_b = qn, qb
            # ---- self attention (layer 0: skip_first_layer_pe -> no residual, no PE; :313-321)
            if li == 0:
                qin_b = s.tok0_b
                vin_b = s.tok0_b
            else:
                qin_b = self._add_b16(queries, tok0)
                vin_b = queries_b
            ls.sa_qin_b, ls.sa_vin_b = qin_b, vin_b
            q = self._lin(qin_b, sa + "q_proj.weight", sa + "q_proj.bias", torch.empty(R, C, device=dev, dtype=f32), R)
            k = self._lin(qin_b, sa + "k_proj.weight", sa + "k_proj.bias", torch.empty(R, C, device=dev, dtype=f32), R)
            v = self._lin(vin_b, sa + "v_proj.weight", sa + "v_proj.bias", torch.empty(R, C, device=dev, dtype=f32), R)
            so_b = torch.empty(R, C, device=dev, dtype=b16)
            probs = torch.empty(P, 8, T, T, device=dev, dtype=f32)
            K.tok_attn_fwd(q, k, v, P, T, so_b, probs)
            ls.sa_q, ls.sa_k, ls.sa_v, ls.sa_probs, ls.sa_o_b = q, k, v, probs, so_b
            s1 = self._lin(so_b, sa + "out_proj.weight", sa + "out_proj.bias", torch.empty(R, C, device=dev, dtype=f32),
                           R, residual=None if li == 0 else queries)
            queries, queries_b, ls.ln1 = self._ln(s1, pre + "layer_norm1", eps, R)
            # ---- cross attention token -> image (:323-333)
            qin_b = self._add_b16(queries, tok0)
            ls.t2i_qin_b = qin_b
            Q = self._lin(qin_b, t2i + "q_proj.weight", t2i + "q_proj.bias", torch.empty(R, CI, device=dev, dtype=f32),
                          R)
            if li == 0:
                src_b, M_kv, kv_rep = imgd_b, B * L, N
            else:
                src_b, M_kv, kv_rep = keys_b, RL, 1
            KQV = torch.empty(M_kv, 3 * CI, device=dev, dtype=b16)  # [K | Q' | V]
            self._proj_pe(src_b, [t2i + "k_proj.weight", i2t + "q_proj.weight", t2i + "v_proj.weight"],
                          [t2i + "k_proj.bias", i2t + "q_proj.bias", t2i + "v_proj.bias"], 2 * CI, KQV, M_kv)
            ls.KQV, ls.kv_src_b, ls.kv_rep = KQV, src_b, kv_rep
            to_b = torch.empty(R, CI, device=dev, dtype=b16)
            lse = torch.empty(P, 8, T, device=dev, dtype=f32)
            to_f = torch.empty(R, CI, device=dev, dtype=f32)  # unrounded O: the backward's delta = dO . O
            K.t2i_fwd(Q, KQV, KQV[:, 2 * CI:], 3 * CI, kv_rep, P, T, L, to_b, lse, score_bias=sbias, out_f32=to_f)
            ls.t2i_Q, ls.t2i_o_b, ls.t2i_o_f, ls.t2i_lse = Q, to_b, to_f, lse
            s2 = self._lin(to_b, t2i + "out_proj.weight", t2i + "out_proj.bias",
                           torch.empty(R, C, device=dev, dtype=f32), R, residual=queries)
            queries, queries_b, ls.ln2 = self._ln(s2, pre + "layer_norm2", eps, R)
            # ---- MLP (ReLU) (:335-339)
            ls.mlp_in_b = queries_b
            hb = self._lin(queries_b, pre + "mlp.lin1.weight", pre + "mlp.lin1.bias",
                           torch.empty(R, cfg.mlp_dim, device=dev, dtype=b16), R, act=ACT_RELU)
            ls.mlp_h_b = hb
            s3 = self._lin(hb, pre + "mlp.lin2.weight", pre + "mlp.lin2.bias", torch.empty(R, C, device=dev, dtype=f32),
                           R, residual=queries)
            queries, queries_b, ls.ln3 = self._ln(s3, pre + "layer_norm3", eps, R)
            # ---- cross attention image -> token (:341-346)
            ls.i2t_qin_b = self._add_b16(queries, tok0)
            ls.i2t_vin_b = queries_b
            Kt = self._lin(ls.i2t_qin_b, i2t + "k_proj.weight", i2t + "k_proj.bias",
                           torch.empty(R, CI, device=dev, dtype=f32), R)
            Vt = self._lin(queries_b, i2t + "v_proj.weight", i2t + "v_proj.bias",
                           torch.empty(R, CI, device=dev, dtype=f32), R)
            ls.i2t_K, ls.i2t_V = Kt, Vt
            io_b = torch.empty(RL, CI, device=dev, dtype=b16)
            K.i2t_fwd(KQV[:, CI:], 3 * CI, kv_rep, Kt, Vt, P, T, L, io_b, CI)
            ls.i2t_o_b = io_b
            s4 = torch.empty(RL, C, device=dev, dtype=b16)  # pre-LN4 keys stream: bf16 like keys_b (LN stats fp32)
            if li == 0:
                self._lin(io_b, i2t + "out_proj.weight", i2t + "out_proj.bias", s4, RL, residual=imgd, r_remap=(L, N))
            else:
                self._lin(io_b, i2t + "out_proj.weight", i2t + "out_proj.bias", s4, RL, residual=keys_b)
            _, keys_b, ls.ln4 = self._ln(s4, pre + "layer_norm4", eps, RL, f32_out=False)
            ls.keys_out_b = keys_b
            s.layers.append(ls)
        # ---- final token -> image attention (:392-404)
        f = tr + "final_attn_token_to_image."
        s.f_qin_b = self._add_b16(queries, tok0)
        s.f_Q = self._lin(s.f_qin_b, f + "q_proj.weight", f + "q_proj.bias", torch.empty(R, CI, device=dev, dtype=f32), R)
        KV = torch.empty(RL, 2 * CI, device=dev, dtype=b16)
        self._proj_pe(keys_b, [f + "k_proj.weight", f + "v_proj.weight"], [f + "k_proj.bias", f + "v_proj.bias"], CI,
                      KV, RL)
        s.f_KV = KV
        s.f_o_b = torch.empty(R, CI, device=dev, dtype=b16)
        s.f_lse = torch.empty(P, 8, T, device=dev, dtype=f32)
        s.f_o_f = torch.empty(R, CI, device=dev, dtype=f32)
        K.t2i_fwd(s.f_Q, KV, KV[:, CI:], 2 * CI, 1, P, T, L, s.f_o_b, s.f_lse, out_f32=s.f_o_f)
        sf = self._lin(s.f_o_b, f + "out_proj.weight", f + "out_proj.bias", torch.empty(R, C, device=dev, dtype=f32), R,
                       residual=queries)
        q7, q7_b, s.lnf = self._ln(sf, tr + "layer_norm_final_attn", 1e-5, R)
        s.q7_b = q7_b
        s.keys2_b = keys_b
        # ---- hypernetwork MLPs on the selected mask tokens (:523-531)
        sel = list(range(1, self.num_mask_tokens)) if multimask else [0]
        s.sel = sel
        nsel = len(sel)
        hyper = torch.empty(P, nsel, 32, device=dev, dtype=f32)
        q7v = q7_b.view(P, T, C)
        s.hyp = []
        for j, t in enumerate(sel):
            hp = f"output_hypernetworks_mlps.{t}."
            x_b = q7v[:, 1 + t]
            h1 = self._lin(x_b, hp + "proj_in.weight", hp + "proj_in.bias", torch.empty(P, C, device=dev, dtype=b16),
                           P, act=ACT_RELU, lda=T * C)
            h2 = self._lin(h1, hp + "layers.0.weight", hp + "layers.0.bias", torch.empty(P, C, device=dev, dtype=b16),
                           P, act=ACT_RELU)
            self._lin(h2, hp + "proj_out.weight", hp + "proj_out.bias", hyper[:, j], P, ldc=nsel * 32)
            s.hyp.append((t, x_b, h1, h2))
        s.hyper = hyper
        # ---- IoU head (forward only: the loss never uses iou_scores) (:534)
        ih = "iou_prediction_head."
        x_b = q7v[:, 0]
        h1 = self._lin(x_b, ih + "proj_in.weight", ih + "proj_in.bias", torch.empty(P, C, device=dev, dtype=b16), P,
                       act=ACT_RELU, lda=T * C)
        h2 = self._lin(h1, ih + "layers.0.weight", ih + "layers.0.bias", torch.empty(P, C, device=dev, dtype=b16), P,
                       act=ACT_RELU)
        iou = self._lin(h2, ih + "proj_out.weight", ih + "proj_out.bias",
                        torch.empty(P, self.num_mask_tokens, device=dev, dtype=f32), P)
        # ---- upscaling: ConvT(256->64) -> LN2d -> GELU -> ConvT(64->32) -> GELU (:519-521)
        b1 = self.Bf("upscale_conv1.bias").repeat(4)
        s.up_b1 = b1
        up1pre = torch.empty(RL, 4 * 64, device=dev, dtype=b16)
        K.gemm(keys_b, self.W("upscale_conv1.weight").t().contiguous(), M=RL, N=256, K=C, out=up1pre, bias=b1)
        up1 = torch.empty(RL * 4, 64, device=dev, dtype=b16)
        mean = torch.empty(RL * 4, device=dev, dtype=f32)
        rstd = torch.empty(RL * 4, device=dev, dtype=f32)
        K.layernorm_fwd(up1pre, self.Bf("upscale_layer_norm.weight"), self.Bf("upscale_layer_norm.bias"), 1e-6, up1,
                        act=ACT_GELU, mean=mean, rstd=rstd)
        s.up1pre, s.up1, s.up_mean, s.up_rstd = up1pre, up1, mean, rstd
        # ConvT2 -> GELU -> masks = hyper . up2, fused (csrc/upmask.hip): up2 is never stored
        masks = torch.empty(P, nsel, 256, 256, device=dev, dtype=f32)
        K.upmask_fwd(up1, self.W("upscale_conv2.weight"), self.Bf("upscale_conv2.bias"), hyper, P, nsel, masks)
        iou_sel = iou[:, sel[0]:sel[-1] + 1].contiguous()  # sel is a contiguous range (slice: capturable)
        return masks.view(B, N, nsel, 256, 256), iou_sel.view(B, N, nsel), s

    # ------------------------------------------------------------------ backward
    def backward_impl(self, s, dmasks):
        """The decoder backward (every parameter gradient into the flat buffer G); with tok_group the token-side
        weight gradients are deferred and issued in grouped launches before it returns."""
        self._tok_pending = [] if self.tok_group and self.tok_wgrad else None
        self._tok_spans, self._tok_reads = [], []
        try:
            G = self._backward_impl(s, dmasks)
            self._flush_tok()
        finally:
            self._tok_pending = None
        return G

    def _backward_impl(self, s, dmasks):
        cfg = self.config
        B, N, T, P, R, L, RL = s.B, s.N, s.T, s.P, s.R, s.L, s.RL
        dev = dmasks.device
        f32, b16 = torch.float32, torch.bfloat16
        tr = "transformer."
        G = self.ensure_grad()
        G.zero_()
        nsel = len(s.sel)
        dm = dmasks.reshape(P, nsel, 65536).contiguous().float()
        # ---- mask head + ConvT2 (+ GELU), fused: recomputes the ConvT2 product from up1; with fused_ln_bwd the
        # LayerNorm2d + GELU backward rides in the same pass (d up1 never reaches HBM)
        dhyper = torch.empty(P, nsel, 32, device=dev, dtype=f32)
        # joint: d up1pre is the left half of one [RL, 512] operand whose right half receives the final attention's
        # [dK | dV], so the keys gradient d keys2 = [d up1pre | dK | dV] @ [W1; Wk; Wv] is ONE product (no in-place
        # read-modify-write of d keys2 by a second one)
        joint = self.fuse_dkeys and self.fused_ln_bwd
        dup_ld = 512 if joint else 256
        dup1pre = torch.empty(RL, dup_ld, device=dev, dtype=b16)
        lnw, lnb = self.Bf("upscale_layer_norm.weight"), self.Bf("upscale_layer_norm.bias")
        glnw, glnb = self.G("upscale_layer_norm.weight"), self.G("upscale_layer_norm.bias")
        if self.fused_ln_bwd:
            K.upmask_bwd(s.up1, self.W("upscale_conv2.weight"), self.Bf("upscale_conv2.bias"), s.hyper, dm, P, nsel,
                         dup1pre, self.G("upscale_conv2.weight"), self.G("upscale_conv2.bias"), dhyper,
                         ln=(s.up1pre, s.up_mean, s.up_rstd, lnw, lnb, glnw, glnb), ldd=dup_ld)
        else:
            dup1 = torch.empty(RL * 4, 64, device=dev, dtype=b16)
            K.upmask_bwd(s.up1, self.W("upscale_conv2.weight"), self.Bf("upscale_conv2.bias"), s.hyper, dm, P, nsel,
                         dup1, self.G("upscale_conv2.weight"), self.G("upscale_conv2.bias"), dhyper)
            K.layernorm_bwd(dup1, s.up1pre, s.up_mean, s.up_rstd, lnw, lnb, dup1pre, act=ACT_GELU, dw=glnw, db=glnb)
        # ConvT1: y[RL, 256] = keys2[RL, 256] @ W1s[256, 256]
        # the image-side keys gradient stream is bf16 (as under the reference's bf16 autocast): it is written,
        # read-modify-written by each block's projection backward and read by LayerNorm4's backward per block
        dkeys = torch.empty(RL, C, device=dev, dtype=b16)
        if not joint:
            K.gemm(dup1pre, self.W("upscale_conv1.weight"), M=RL, N=C, K=256, out=dkeys, b_mode=0)
        # (bias: column sums of dup1pre's [RL, 4 x 64] view, folded over the 4 ConvT taps)
        self._dw(s.keys2_b, dup1pre, RL, self.G("upscale_conv1.weight"), ldy=C, ldx=dup_ld,
                 dbx=self.G("upscale_conv1.bias"), dbx_fold=4)
        # ---- hypernetwork MLP backward -> dq7
        dq7 = torch.zeros(R, C, device=dev, dtype=f32)
        dq7v = dq7.view(P, T, C)
        for j, (t, x_b, h1, h2) in enumerate(s.hyp):
            hp = f"output_hypernetworks_mlps.{t}."
            dh = self._bf(dhyper[:, j])
            dh2 = torch.empty(P, C, device=dev, dtype=f32)
            self._lin_bwd(dh, h2, hp + "proj_out.weight", hp + "proj_out.bias", P, dx_out=dh2)
            dh2b = torch.empty(P, C, device=dev, dtype=b16)
            K.relu_bwd(dh2, h2, dh2b, ldy=C, cols=C)
            dh1 = torch.empty(P, C, device=dev, dtype=f32)
            self._lin_bwd(dh2b, h1, hp + "layers.0.weight", hp + "layers.0.bias", P, dx_out=dh1)
            dh1b = torch.empty(P, C, device=dev, dtype=b16)
            K.relu_bwd(dh1, h1, dh1b, ldy=C, cols=C)
            self._lin_bwd(dh1b, x_b, hp + "proj_in.weight", hp + "proj_in.bias", P, dx_out=dq7v[:, 1 + t],
                          ldx=T * C, ldc=T * C)
        # ---- final attention
        f = tr + "final_attn_token_to_image."
        dsf, dsf_b = self._ln_bwd(dq7, s.lnf)
        dq = dsf  # d queries (q6) accumulator, fp32
        dtok = torch.zeros(R, C, device=dev, dtype=f32)
        dfo = torch.empty(R, CI, device=dev, dtype=f32)
        self._lin_bwd(dsf_b, s.f_o_b, f + "out_proj.weight", f + "out_proj.bias", R, dx_out=dfo)
        dQ = torch.empty(R, CI, device=dev, dtype=b16)
        if joint:
            dKV, lkv = dup1pre[:, 256:], 512
        else:
            dKV, lkv = torch.empty(RL, 2 * CI, device=dev, dtype=b16), 2 * CI
        K.t2i_bwd(s.f_Q, s.f_KV, s.f_KV[:, CI:], 2 * CI, 1, P, T, L, s.f_o_b, dfo, s.f_lse, dQ, dKV, dKV[:, CI:], lkv,
                  out_f32=s.f_o_f)
        self._qin_bwd(dQ, s.f_qin_b, f + "q_proj.weight", f + "q_proj.bias", R, dq, dtok)
        # d keys2 += [dK | dV] @ [Wk; Wv]
        wkv = self._group(self.flat_b16, [f + "k_proj.weight", f + "v_proj.weight"], C)
        if joint:  # d keys2 = [d up1pre | dK | dV] @ [W1; Wk; Wv], one product (B [C, 512]: B[n][k])
            bcat = torch.cat([self.W("upscale_conv1.weight"), wkv.t()], 1).contiguous()
            K.gemm(dup1pre, bcat, M=RL, N=C, K=512, out=dkeys, b_mode=0, lda=512)
        else:
            self._dx(dKV, wkv, RL, dkeys, beta=1.0)
        self._dw_pe(dKV, s.keys2_b, RL, self._group(self.flat_grad, [f + "k_proj.weight", f + "v_proj.weight"], C),
                    CI, s.pe_b, db=self._group(self.flat_grad, [f + "k_proj.bias", f + "v_proj.bias"], 0), ldy=lkv)
        # ---- two-way blocks in reverse
        for li in reversed(range(cfg.num_hidden_layers)):
            ls = s.layers[li]
            pre = tr + f"layers.{li}."
            sa, t2i, i2t = pre + "self_attn.", pre + "cross_attn_token_to_image.", pre + "cross_attn_image_to_token."
            # LN4 on keys
            x4, mean4, rstd4, _ = ls.ln4
            ds4_b = torch.empty(RL, C, device=dev, dtype=b16)
            K.layernorm_bwd(dkeys, x4, mean4, rstd4, self.Bf(pre + "layer_norm4.weight"),
                            self.Bf(pre + "layer_norm4.bias"), ds4_b,
                            dw=self.G(pre + "layer_norm4.weight"), db=self.G(pre + "layer_norm4.bias"))
            # d keys_in = d s4 (residual) + the block's image-side projection gradients, accumulated in place
            # once every reader of d s4 (out_proj backward) has run
            dkeys_in = ds4_b if li > 0 else None
            # s4 = keys_in + i2t_out @ Wo^T + bo
            dio_b = torch.empty(RL, CI, device=dev, dtype=b16)
            self._lin_bwd(ds4_b, ls.i2t_o_b, i2t + "out_proj.weight", i2t + "out_proj.bias", RL, dx_out=dio_b)
            # i2t attention
            KQV = ls.KQV
            dQ_img = None
            if li == 0 and self.t2i_sum and ls.kv_rep > 1 and L % 64 == 0:
                # queries shared by the image's prompts: their gradient summed over the prompts inside the kernel
                dQ_img = torch.empty(B * L, CI, device=dev, dtype=b16)
                dKt, dVt = K.i2t_bwd_sum(KQV[:, CI:], 3 * CI, ls.kv_rep, ls.i2t_K, ls.i2t_V, P, T, L, dio_b, CI,
                                         dQ_img, CI)
            elif li == 0:
                dQp = torch.empty(RL, CI, device=dev, dtype=b16)
                dKt, dVt = K.i2t_bwd(KQV[:, CI:], 3 * CI, ls.kv_rep, ls.i2t_K, ls.i2t_V, P, T, L, dio_b, CI, dQp, CI)
            else:
                dKQV = torch.empty(RL, 3 * CI, device=dev, dtype=b16)
                dKt, dVt = K.i2t_bwd(KQV[:, CI:], 3 * CI, 1, ls.i2t_K, ls.i2t_V, P, T, L, dio_b, CI, dKQV[:, CI:],
                                     3 * CI)
            dKt_b = self._bf(dKt.reshape(R, CI))
            dVt_b = self._bf(dVt.reshape(R, CI))
            self._qin_bwd(dKt_b, ls.i2t_qin_b, i2t + "k_proj.weight", i2t + "k_proj.bias", R, dq, dtok)
            self._lin_bwd(dVt_b, ls.i2t_vin_b, i2t + "v_proj.weight", i2t + "v_proj.bias", R, dx_out=dq, dx_beta=1.0)
            # LN3 / MLP
            dq, ds_b = self._ln_bwd(dq, ls.ln3)
            dh = torch.empty(R, cfg.mlp_dim, device=dev, dtype=f32)
            self._lin_bwd(ds_b, ls.mlp_h_b, pre + "mlp.lin2.weight", pre + "mlp.lin2.bias", R, dx_out=dh)
            dh_b = torch.empty(R, cfg.mlp_dim, device=dev, dtype=b16)
            K.relu_bwd(dh, ls.mlp_h_b, dh_b, ldy=cfg.mlp_dim, cols=cfg.mlp_dim)
            self._lin_bwd(dh_b, ls.mlp_in_b, pre + "mlp.lin1.weight", pre + "mlp.lin1.bias", R, dx_out=dq,
                          dx_beta=1.0)
            # LN2 / t2i
            dq, ds_b = self._ln_bwd(dq, ls.ln2)
            dto = torch.empty(R, CI, device=dev, dtype=f32)
            self._lin_bwd(ds_b, ls.t2i_o_b, t2i + "out_proj.weight", t2i + "out_proj.bias", R, dx_out=dto)
            dQ = torch.empty(R, CI, device=dev, dtype=b16)
            dKV_img = None
            if li == 0 and self.t2i_sum and ls.kv_rep > 1 and L % 64 == 0:
                # K / V shared by the image's prompts: their gradients summed over the prompts inside the kernel
                dKV_img = torch.empty(B * L, 2 * CI, device=dev, dtype=b16)
                K.t2i_bwd_sum(ls.t2i_Q, KQV, KQV[:, 2 * CI:], 3 * CI, ls.kv_rep, P, T, L, ls.t2i_o_b, dto, ls.t2i_lse,
                              dQ, dKV_img, dKV_img[:, CI:], 2 * CI, out_f32=ls.t2i_o_f)
            elif li == 0:
                dKV0 = torch.empty(RL, 2 * CI, device=dev, dtype=b16)
                K.t2i_bwd(ls.t2i_Q, KQV, KQV[:, 2 * CI:], 3 * CI, ls.kv_rep, P, T, L, ls.t2i_o_b, dto, ls.t2i_lse, dQ,
                          dKV0, dKV0[:, CI:], 2 * CI, out_f32=ls.t2i_o_f)
            else:
                K.t2i_bwd(ls.t2i_Q, KQV, KQV[:, 2 * CI:], 3 * CI, 1, P, T, L, ls.t2i_o_b, dto, ls.t2i_lse, dQ, dKQV,
                          dKQV[:, 2 * CI:], 3 * CI, out_f32=ls.t2i_o_f)
            self._qin_bwd(dQ, ls.t2i_qin_b, t2i + "q_proj.weight", t2i + "q_proj.bias", R, dq, dtok)
            # image-side projections of this block's input keys
            kq = [t2i + "k_proj.weight", i2t + "q_proj.weight"]
            if li == 0:
                # per-image tensors: sum the per-prompt gradients over the image's prompts first
                Mi = B * L
                ldkv = CI
                if dKV_img is not None:
                    dK_img, dV_img, ldkv = dKV_img, dKV_img[:, CI:], 2 * CI
                else:
                    dK_img = torch.empty(Mi, CI, device=dev, dtype=b16)
                    dV_img = torch.empty(Mi, CI, device=dev, dtype=b16)
                    K.group_sum(dKV0, dK_img, ld_in=2 * CI, cols=CI, groups=B, nper=N, rows_per=L)
                    K.group_sum(dKV0[:, CI:], dV_img, ld_in=2 * CI, cols=CI, groups=B, nper=N, rows_per=L)
                if dQ_img is None:
                    dQ_img = torch.empty(Mi, CI, device=dev, dtype=b16)
                    K.group_sum(dQp, dQ_img, ld_in=CI, cols=CI, groups=B, nper=N, rows_per=L)
                self._dw(dK_img, s.imgd_b, Mi, self.G(t2i + "k_proj.weight"), ldy=ldkv, x_add=s.pe_b, x_add_rows=L,
                         db=self.G(t2i + "k_proj.bias"))
                self._dw(dQ_img, s.imgd_b, Mi, self.G(i2t + "q_proj.weight"), x_add=s.pe_b, x_add_rows=L,
                         db=self.G(i2t + "q_proj.bias"))
                self._dw(dV_img, s.imgd_b, Mi, self.G(t2i + "v_proj.weight"), ldy=ldkv, db=self.G(t2i + "v_proj.bias"))
            else:
                wg = self._group(self.flat_b16, kq + [t2i + "v_proj.weight"], C)
                self._before_write(dkeys_in)  # (d s4, read by the deferred out_proj weight gradient at small RL)
                self._dx(dKQV, wg, RL, dkeys_in, beta=1.0)
                self._dw_pe(dKQV, ls.kv_src_b, RL, self._group(self.flat_grad, kq + [t2i + "v_proj.weight"], C),
                            2 * CI, s.pe_b, db=self._group(self.flat_grad, [t2i + "k_proj.bias", i2t + "q_proj.bias",
                                                                            t2i + "v_proj.bias"], 0))
                dkeys = dkeys_in
            # LN1 / self attention
            dq, ds_b = self._ln_bwd(dq, ls.ln1)
            if li == 0:
                dq = None  # queries = LN1(self_attn(tokens)) with no residual (skip_first_layer_pe)
            dso = torch.empty(R, C, device=dev, dtype=f32)
            self._lin_bwd(ds_b, ls.sa_o_b, sa + "out_proj.weight", sa + "out_proj.bias", R, dx_out=dso)
            dqs = torch.empty(R, C, device=dev, dtype=b16)
            dks = torch.empty(R, C, device=dev, dtype=b16)
            dvs = torch.empty(R, C, device=dev, dtype=b16)
            K.tok_attn_bwd(ls.sa_q, ls.sa_k, ls.sa_v, ls.sa_probs, dso, P, T, dqs, dks, dvs)
            if li == 0:
                # q = k = v = tokens (no PE); the tokens are the trainable iou/mask tokens (+ prompts)
                self._lin_bwd(dqs, ls.sa_qin_b, sa + "q_proj.weight", sa + "q_proj.bias", R, dx_out=dtok, dx_beta=1.0)
                self._lin_bwd(dks, ls.sa_qin_b, sa + "k_proj.weight", sa + "k_proj.bias", R, dx_out=dtok, dx_beta=1.0)
                self._lin_bwd(dvs, ls.sa_vin_b, sa + "v_proj.weight", sa + "v_proj.bias", R, dx_out=dtok, dx_beta=1.0)
            else:
                dqin = torch.empty(R, C, device=dev, dtype=f32)
                self._lin_bwd(dqs, ls.sa_qin_b, sa + "q_proj.weight", sa + "q_proj.bias", R, dx_out=dqin)
                self._lin_bwd(dks, ls.sa_qin_b, sa + "k_proj.weight", sa + "k_proj.bias", R, dx_out=dqin, dx_beta=1.0)
                K.axpby(dq, dqin, dq)
                K.axpby(dtok, dqin, dtok)
                self._lin_bwd(dvs, ls.sa_vin_b, sa + "v_proj.weight", sa + "v_proj.bias", R, dx_out=dq, dx_beta=1.0)
            if self.tok_flush_block and self._tok_pending:
                self._flush_tok()
        # ---- token embeddings: d[iou_token; mask_tokens] = sum over prompts of d tokens[:, 0:5]
        gtok = self._group(self.flat_grad, ["iou_token.weight", "mask_tokens.weight"], 0)
        part = torch.empty(T * C, device=dev, dtype=f32)
        K.colsum(dtok, P, T * C, part)
        gtok.copy_(part[: gtok.numel()])
        return G

    def _qin_bwd(self, dY_b, qin_b, wname, bname, R, dq, dtok):
        """y = (q + tok) W^T + b: dq += dY W, dtok += dY W, dW = dY^T (q+tok)_b, db."""
        dqin = torch.empty(R, C, device=dq.device, dtype=torch.float32)
        self._lin_bwd(dY_b, qin_b, wname, bname, R, dx_out=dqin)
        K.axpby(dq, dqin, dq)
        K.axpby(dtok, dqin, dtok)


class MaskDecoderFn(torch.autograd.Function):
    """autograd boundary: input = the decoder's flat fp32 parameter buffer (+ non-differentiable
    image/prompt tensors); grad = flat gradient buffer."""

    @staticmethod
    def forward(ctx, flat, emb, pe, tokens, no_mask, dec: MaskDecoder, multimask: bool, target=None, similarity=None):
        masks, iou, saved = dec.forward_impl(emb, pe, tokens, no_mask, multimask, target, similarity)
        ctx.saved = saved
        ctx.dec = dec
        ctx.mark_non_differentiable(iou)
        return masks, iou

    @staticmethod
    def backward(ctx, dmasks, diou):
        dec = ctx.dec
        if getattr(ctx.saved, "similarity", False):
            raise NotImplementedError("attention_similarity is a forward-only (inference) hook")
        g = dec.backward_impl(ctx.saved, dmasks)
        ctx.saved = None
        return g, None, None, None, None, None, None, None, None
