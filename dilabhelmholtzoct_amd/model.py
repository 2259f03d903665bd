"""Drop-in SamModel for the OCT-SAM training step, computed by liboctsam_hip.so.

Mirrors the transformers ``SamModel`` surface the reference uses (hf:modeling_sam.py:1193-1358;
ref:octsam/models/training_utils.py:55,273-280): same sub-module names (``vision_encoder``,
``prompt_encoder``, ``mask_decoder``, ``shared_image_embedding``), same parameter names and shapes
(state_dict keys interchange with HF checkpoints, 315 keys for vit-b), same forward signature and
output fields (``pred_masks`` [B,N,k,256,256], ``iou_scores`` [B,N,k]). The nn.Linear / nn.Conv2d /
nn.LayerNorm children are parameter containers only; every forward/backward FLOP runs in HIP kernels.

Precision: bf16 operands with fp32 accumulation on MFMA, fp32 LayerNorm/softmax statistics, fp32
residual streams in the encoder, fp32 master weights and Adam state for the mask decoder.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from . import kernels as K
from .config import SamConfig, config_for
from ._lib import ACT_GELU


# ----------------------------------------------------------------------------------- modules
class PositionalEmbedding(nn.Module):
    """SamPositionalEmbedding (hf:modeling_sam.py:546-566): random-Fourier features."""

    def __init__(self, cfg: SamConfig):
        super().__init__()
        self.scale = cfg.vision.scale
        self.positional_embedding = nn.Parameter(torch.zeros(2, cfg.vision.num_pos_feats))


class PatchEmbed(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.projection = nn.Conv2d(3, cfg.hidden_size, kernel_size=16, stride=16)


class VisionAttention(nn.Module):
    def __init__(self, cfg, window_size):
        super().__init__()
        side = window_size if window_size > 0 else cfg.image_size // cfg.patch_size
        self.window_size = window_size
        self.num_attention_heads = cfg.num_attention_heads
        self.qkv = nn.Linear(cfg.hidden_size, 3 * cfg.hidden_size)
        self.proj = nn.Linear(cfg.hidden_size, cfg.hidden_size)
        hd = cfg.hidden_size // cfg.num_attention_heads
        self.rel_pos_h = nn.Parameter(torch.zeros(2 * side - 1, hd))
        self.rel_pos_w = nn.Parameter(torch.zeros(2 * side - 1, hd))


class MLPBlock(nn.Module):
    def __init__(self, d, mlp):
        super().__init__()
        self.lin1 = nn.Linear(d, mlp)
        self.lin2 = nn.Linear(mlp, d)


class VisionLayer(nn.Module):
    def __init__(self, cfg, window_size):
        super().__init__()
        self.layer_norm1 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.attn = VisionAttention(cfg, window_size)
        self.layer_norm2 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.mlp = MLPBlock(cfg.hidden_size, cfg.mlp_dim)
        self.window_size = window_size


class VisionNeck(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.conv1 = nn.Conv2d(cfg.hidden_size, cfg.output_channels, kernel_size=1, bias=False)
        self.layer_norm1 = nn.LayerNorm(cfg.output_channels, eps=1e-6)
        self.conv2 = nn.Conv2d(cfg.output_channels, cfg.output_channels, kernel_size=3, padding=1, bias=False)
        self.layer_norm2 = nn.LayerNorm(cfg.output_channels, eps=1e-6)


class VisionEncoder(nn.Module):
    """SamVisionEncoder (hf:modeling_sam.py:1019-1072): patch-embed -> L ViT layers -> neck."""

    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.patch_embed = PatchEmbed(cfg)
        g = cfg.image_size // cfg.patch_size
        self.pos_embed = nn.Parameter(torch.zeros(1, g, g, cfg.hidden_size))
        self.layers = nn.ModuleList([
            VisionLayer(cfg, 0 if i in cfg.global_attn_indexes else cfg.window_size)
            for i in range(cfg.num_hidden_layers)])
        self.neck = VisionNeck(cfg)
        self._wcache: dict = {}
        # 16-bit operand type of the encoder's MFMA work: bf16 (BASELINE configs[1..3]) or fp16 (configs[4]);
        # the residual stream, LayerNorm statistics and accumulation stay fp32
        self.compute_dtype = torch.bfloat16

    # 16-bit operand cache, refreshed whenever a parameter is modified in place or moved
    def _w(self, key, p: torch.Tensor, fn=None):
        ent = self._wcache.get(key)
        tag = (p._version, p.data_ptr(), p.device, self.compute_dtype)
        if ent is None or ent[0] != tag:
            t = p.detach()
            t = fn(t) if fn is not None else t
            ent = (tag, t.to(self.compute_dtype).contiguous())
            self._wcache[key] = ent
        return ent[1]

    def _wf(self, key, p: torch.Tensor, fn=None):  # fp32 contiguous copy (biases, LN, pos-embed)
        ent = self._wcache.get(key)
        tag = (p._version, p.data_ptr(), p.device)
        if ent is None or ent[0] != tag:
            t = p.detach()
            t = fn(t) if fn is not None else t
            ent = (tag, t.float().contiguous())
            self._wcache[key] = ent
        return ent[1]

    @torch.no_grad()
    def forward_nhwc(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """pixel_values fp32 [B,3,1024,1024] -> image embeddings fp32 [B, 4096, 256] (NHWC)."""
        cfg = self.config
        if pixel_values.dim() != 4 or pixel_values.shape[1] != 3:
            raise ValueError("Make sure that the channel dimension of the pixel values match with the one set in "
                             "the configuration.")
        if pixel_values.shape[2] != cfg.image_size or pixel_values.shape[3] != cfg.image_size:
            raise ValueError(f"Input image size ({pixel_values.shape[2]}*{pixel_values.shape[3]}) doesn't match "
                             f"model ({cfg.image_size}*{cfg.image_size}).")
        px = pixel_values.float().contiguous()
        B = px.shape[0]
        D = cfg.hidden_size
        e16 = self.compute_dtype
        g = cfg.image_size // cfg.patch_size
        L = g * g
        M = B * L
        dev = px.device
        heads = cfg.num_attention_heads
        pe = self.patch_embed.projection
        x = torch.empty(M, D, device=dev, dtype=torch.float32)
        patches = K.patchify_bf16(px, torch.empty(M, 3 * 256, device=dev, dtype=e16))
        K.gemm(patches, self._w("patch.w", pe.weight, lambda t: t.reshape(D, -1)), M=M, N=D, K=3 * 256, out=x,
               bias=self._wf("patch.b", pe.bias), residual=self._wf("pos", self.pos_embed,
                                                                                   lambda t: t.reshape(L, D)),
               r_remap=(L, B))
        xn = torch.empty(M, D, device=dev, dtype=e16)
        mlp_h = torch.empty(M, cfg.mlp_dim, device=dev, dtype=e16)
        for li, layer in enumerate(self.layers):
            at = layer.attn
            ws = layer.window_size
            pre = f"l{li}."
            ln1w, ln1b = self._wf(pre + "ln1w", layer.layer_norm1.weight), self._wf(pre + "ln1b", layer.layer_norm1.bias)
            # windowed layers stay token-ordered: window_partition / window_unpartition (hf:modeling_sam.py:
            # 900-952, 960-966) happen inside the attention kernel's row addressing; the padding tokens' qkv
            # (Linear of a zero row = the bias) is one row, not 6432 computed ones
            K.layernorm_fwd(x, ln1w, ln1b, cfg.layer_norm_eps, xn)
            qkv = torch.empty(M, 3 * D, device=dev, dtype=e16)
            K.gemm(xn, self._w(pre + "qkv", at.qkv.weight), M=M, N=3 * D, K=D, out=qkv,
                   bias=self._wf(pre + "qkvb", at.qkv.bias))
            ao = torch.empty(M, D, device=dev, dtype=e16)
            rh, rw = self._wf(pre + "rh", at.rel_pos_h), self._wf(pre + "rw", at.rel_pos_w)
            if ws > 0:
                nw = (g + ws - 1) // ws
                K.vit_attention(qkv, ao, rh, rw, nseq=B * nw * nw, side=ws, heads=heads, grid=g,
                                pad_row=self._w(pre + "qkvpad", at.qkv.bias))
            else:
                K.vit_attention(qkv, ao, rh, rw, nseq=B, side=g, heads=heads)
            K.gemm(ao, self._w(pre + "proj", at.proj.weight), M=M, N=D, K=D, out=x,
                   bias=self._wf(pre + "projb", at.proj.bias), residual=x)
            del qkv, ao
            K.layernorm_fwd(x, self._wf(pre + "ln2w", layer.layer_norm2.weight),
                            self._wf(pre + "ln2b", layer.layer_norm2.bias), cfg.layer_norm_eps, xn)
            K.gemm(xn, self._w(pre + "fc1", layer.mlp.lin1.weight), M=M, N=cfg.mlp_dim, K=D, out=mlp_h,
                   bias=self._wf(pre + "fc1b", layer.mlp.lin1.bias), act=ACT_GELU)
            K.gemm(mlp_h, self._w(pre + "fc2", layer.mlp.lin2.weight), M=M, N=D, K=cfg.mlp_dim, out=x,
                   bias=self._wf(pre + "fc2b", layer.mlp.lin2.bias), residual=x)
        del mlp_h
        # neck: conv1x1 -> LN2d -> conv3x3 -> LN2d  (channels-last)
        K.cast_bf16(x, xn)
        C = cfg.output_channels
        nk = self.neck
        y = torch.empty(M, C, device=dev, dtype=torch.float32)
        K.gemm(xn, self._w("neck.c1", nk.conv1.weight, lambda t: t.reshape(C, D)), M=M, N=C, K=D, out=y)
        yb = torch.empty(M, C, device=dev, dtype=e16)
        K.layernorm_fwd(y, self._wf("neck.ln1w", nk.layer_norm1.weight), self._wf("neck.ln1b", nk.layer_norm1.bias),
                        1e-6, yb)
        K.gemm(yb, self._w("neck.c2", nk.conv2.weight, lambda t: t.permute(0, 2, 3, 1).reshape(C, 9 * C)), M=M,
               N=C, K=9 * C, out=y, a_mode=3, conv_c=C)
        emb = torch.empty(B, L, C, device=dev, dtype=torch.float32)
        K.layernorm_fwd(y, self._wf("neck.ln2w", nk.layer_norm2.weight), self._wf("neck.ln2b", nk.layer_norm2.bias),
                        1e-6, emb)
        return emb

    def forward(self, pixel_values):
        """HF-layout output: last_hidden_state [B, 256, 64, 64]."""
        emb = self.forward_nhwc(pixel_values)
        g = self.config.image_size // self.config.patch_size
        return emb.view(emb.shape[0], g, g, -1).permute(0, 3, 1, 2)


class MaskEmbedding(nn.Module):
    """SamMaskEmbedding (hf:modeling_sam.py:569-598): the dense prompt of input_masks, one HIP kernel
    (octsam_mask_embed). The reference never passes input_masks; this is the SamModel surface, forward only
    (the prompt encoder is frozen on the training path)."""

    def __init__(self, cfg):
        super().__init__()
        c = cfg.mask_input_channels
        self.conv1 = nn.Conv2d(1, c // 4, kernel_size=2, stride=2)
        self.conv2 = nn.Conv2d(c // 4, c, kernel_size=2, stride=2)
        self.conv3 = nn.Conv2d(c, cfg.hidden_size, kernel_size=1)
        self.layer_norm1 = nn.LayerNorm(c // 4, eps=1e-6)
        self.layer_norm2 = nn.LayerNorm(c, eps=1e-6)
        self.eps = cfg.layer_norm_eps

    @torch.no_grad()
    def packed(self) -> torch.Tensor:
        ps = [self.conv1.weight, self.conv1.bias, self.layer_norm1.weight, self.layer_norm1.bias, self.conv2.weight,
              self.conv2.bias, self.layer_norm2.weight, self.layer_norm2.bias, self.conv3.weight, self.conv3.bias]
        return torch.cat([p.detach().reshape(-1).float() for p in ps]).contiguous()

    @torch.no_grad()
    def forward_pixels(self, masks: torch.Tensor) -> torch.Tensor:
        """masks [B, 1, 256, 256] (or [B, 256, 256]) -> dense embeddings fp32 [B, 4096, 256] (pixel-major)."""
        if masks.dim() == 4 and masks.shape[1] == 1:
            masks = masks[:, 0]
        if masks.dim() != 3 or tuple(masks.shape[1:]) != (256, 256):
            raise ValueError(f"input_masks must be [batch_size, 1, 256, 256], got {tuple(masks.shape)}")
        if self.conv1.out_channels != 4 or self.conv2.out_channels != 16 or self.conv3.out_channels != 256:
            raise NotImplementedError("mask embedding kernel is built for mask_input_channels 16, hidden 256")
        m = masks.to(self.conv1.weight.device, torch.float32).contiguous()
        out = torch.empty(m.shape[0], 4096, 256, device=m.device, dtype=torch.float32)
        return K.mask_embed(m, self.packed(), self.eps, out)

    def forward(self, masks: torch.Tensor) -> torch.Tensor:
        """[B, 256, 64, 64] like hf SamMaskEmbedding.forward."""
        return self.forward_pixels(masks).view(-1, 64, 64, 256).permute(0, 3, 1, 2)


class PromptEncoder(nn.Module):
    """SamPromptEncoder (hf:modeling_sam.py:601-698)."""

    def __init__(self, cfg: SamConfig, shared: PositionalEmbedding):
        super().__init__()
        pc = cfg.prompt
        self.shared_embedding = shared
        self.mask_embed = MaskEmbedding(pc)
        self.no_mask_embed = nn.Embedding(1, pc.hidden_size)
        self.point_embed = nn.ModuleList([nn.Embedding(1, pc.hidden_size) for _ in range(pc.num_point_embeddings)])
        self.not_a_point_embed = nn.Embedding(1, pc.hidden_size)
        self.input_image_size = pc.image_size


# ----------------------------------------------------------------------------------- output
@dataclass
class SamImageSegmentationOutput:
    iou_scores: torch.Tensor = None
    pred_masks: torch.Tensor = None
    vision_hidden_states: tuple = None
    vision_attentions: tuple = None
    mask_decoder_attentions: tuple = None

    def __getitem__(self, k):
        return getattr(self, k) if isinstance(k, str) else (self.iou_scores, self.pred_masks)[k]


# ----------------------------------------------------------------------------------- model
class SamModel(nn.Module):
    """transformers.SamModel drop-in (training surface of ref:octsam/models/training_utils.py)."""

    def __init__(self, config: SamConfig | str = "facebook/sam-vit-base"):
        super().__init__()
        from .decoder import MaskDecoder  # local import: decoder imports model helpers
        cfg = config_for(config) if isinstance(config, str) else config
        self.config = cfg
        self.shared_image_embedding = PositionalEmbedding(cfg)
        self.vision_encoder = VisionEncoder(cfg.vision)
        self.prompt_encoder = PromptEncoder(cfg, self.shared_image_embedding)
        self.mask_decoder = MaskDecoder(cfg.decoder)

    # -- weights ----------------------------------------------------------------------
    @classmethod
    def from_pretrained(cls, name_or_path: str, **kw) -> "SamModel":
        """transformers' SamModel.from_pretrained(name) as the reference calls it (training_utils.py:274-275),
        offline. Weights, in order:
          1. ``state_dict_path=`` (a ``.pt`` / ``.safetensors`` state dict with HF keys), or a file path;
          2. a directory with ``model.safetensors`` / ``pytorch_model.bin`` (save_pretrained layout);
          3. a hub name found in the local HF cache (``$HF_HUB_CACHE`` or ``$HF_HOME/hub``:
             ``models--facebook--sam-vit-base/snapshots/*/model.safetensors``);
          4. otherwise the deterministic synthetic initialisation — silently only when ``seed=`` is given
             (an explicit opt-in to random weights); without it a warning names the paths searched."""
        import os
        import warnings
        cfg = kw.pop("config", None)
        seed = kw.pop("seed", None)
        path = kw.pop("state_dict_path", None)
        arch = name_or_path if name_or_path in _ALL_NAMES else os.path.basename(name_or_path.rstrip("/"))
        if cfg is None:
            try:
                cfg = config_for(arch)
            except ValueError:
                cfg = config_for("facebook/sam-vit-base") if path or os.path.exists(name_or_path) else None
                if cfg is None:
                    raise
        model = cls(cfg)
        searched = []
        if path is None:
            path = _find_weights(name_or_path, searched)
        if path:
            if path.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(path)
            else:
                sd = torch.load(path, map_location="cpu", weights_only=True)
            model.load_state_dict(sd)
            model.weights_path = path
        else:
            if seed is None:
                warnings.warn(f"SamModel.from_pretrained({name_or_path!r}): no local weights found (searched: "
                              f"{', '.join(searched) or 'nothing'}); the hub is unreachable offline, so the "
                              f"weights are the synthetic random initialisation (seed 0). Pass seed= to opt "
                              f"into random weights explicitly.", UserWarning, stacklevel=2)
                seed = 0
            model.init_weights(seed=seed)
            model.weights_path = None
        return model

    @torch.no_grad()
    def init_weights(self, seed: int = 0, std: float | None = None):
        """HF-style initialisation (SamPreTrainedModel._init_weights) with a fixed CPU generator:
        Linear/Conv/Embedding ~ N(0, 0.02), biases 0, LayerNorm (1, 0). Departures, so that the
        synthetic model exercises every path: pos_embed and rel_pos tables ~ N(0, 0.02) instead of
        zeros, and the random-Fourier matrix ~ N(0, 1) instead of N(0, hidden/2)."""
        std = self.config.initializer_range if std is None else std
        gen = torch.Generator().manual_seed(seed)
        for name, p in sorted(self.named_parameters(), key=lambda kv: kv[0]):
            if name.endswith("positional_embedding"):
                val = torch.randn(p.shape, generator=gen)
            elif ".layer_norm" in name or "upscale_layer_norm" in name:
                val = torch.ones(p.shape) if name.endswith("weight") else torch.zeros(p.shape)
            elif name.endswith("bias"):
                val = torch.zeros(p.shape)
            else:
                val = torch.randn(p.shape, generator=gen) * std
            p.copy_(val.to(p.dtype))
        self.mask_decoder.sync_bf16()

    def set_encoder_dtype(self, dtype) -> "SamModel":
        """Operand type of the frozen image encoder's GEMMs and attention: torch.bfloat16 (default) or
        torch.float16 (BASELINE configs[4]). The trainable mask decoder keeps fp32 master weights and bf16
        operands (bf16's fp32 exponent range needs no loss scaling for its gradients)."""
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("encoder dtype must be torch.bfloat16 or torch.float16")
        self.vision_encoder.compute_dtype = dtype
        return self

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=False)
        self.mask_decoder.sync_bf16()
        return res

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        self.mask_decoder.reflatten()
        return self

    # -- pieces -----------------------------------------------------------------------
    @torch.no_grad()
    def get_image_wide_positional_embeddings(self) -> torch.Tensor:
        """[1, 256, 64, 64] like hf:modeling_sam.py:1128-1139."""
        pe = self.image_pe()
        g = self.config.prompt.image_embedding_size
        return pe.view(g, g, -1).permute(2, 0, 1).unsqueeze(0)

    @torch.no_grad()
    def image_pe(self) -> torch.Tensor:
        G = self.shared_image_embedding.positional_embedding.detach().float().contiguous()
        g = self.config.prompt.image_embedding_size
        out = torch.empty(g * g, 256, device=G.device, dtype=torch.float32)
        K.image_pe(G, g, out)
        return out

    @torch.no_grad()
    def get_image_embeddings(self, pixel_values):
        return self.vision_encoder(pixel_values)

    @torch.no_grad()
    def prompt_tokens(self, input_points=None, input_labels=None, input_boxes=None) -> torch.Tensor:
        """[iou, mask x4, sparse...] tokens [B, N, T, 256] fp32 (decoder input point_embeddings)."""
        pe = self.prompt_encoder
        md = self.mask_decoder
        if input_boxes is not None:
            B, N = input_boxes.shape[:2]
        else:
            B, N = input_points.shape[:2]
        P = B * N
        dev = self.shared_image_embedding.positional_embedding.device
        boxes = input_boxes.reshape(P, 4).to(dev, torch.float32).contiguous() if input_boxes is not None else None
        pts = labels = None
        npts = 0
        if input_points is not None:
            npts = input_points.shape[2]
            pts = input_points.reshape(P, npts, 2).to(dev, torch.float32).contiguous()
            if input_labels is None:
                labels = torch.ones(P, npts, dtype=torch.int32, device=dev)
            else:
                labels = input_labels.reshape(P, npts).to(dev, torch.int32).contiguous()
        nsparse = (npts + (0 if boxes is not None else 1) if pts is not None else 0) + (2 if boxes is not None else 0)
        T = 5 + nsparse
        tokens = torch.empty(P, T, 256, device=dev, dtype=torch.float32)
        point_embed = torch.cat([e.weight.detach() for e in pe.point_embed], 0).float().contiguous()
        K.prompt_tokens(boxes, pts, labels, P, npts, self.shared_image_embedding.positional_embedding.detach().float()
                        .contiguous(), point_embed, pe.not_a_point_embed.weight.detach().float().contiguous(),
                        md.output_tokens_f32(), float(pe.input_image_size), tokens)
        return tokens.view(B, N, T, 256)

    # -- forward ----------------------------------------------------------------------
    def forward(self, pixel_values=None, input_points=None, input_labels=None, input_boxes=None, input_masks=None,
                image_embeddings=None, multimask_output: bool = True, attention_similarity=None,
                target_embedding=None, **kwargs) -> SamImageSegmentationOutput:
        """SamModel.forward (hf:modeling_sam.py:1193-1358); error messages follow HF."""
        if pixel_values is None and image_embeddings is None:
            raise ValueError("Either pixel_values or image_embeddings must be provided.")
        if pixel_values is not None and image_embeddings is not None:
            raise ValueError("Only one of pixel_values and image_embeddings can be provided.")
        if input_points is not None and len(input_points.shape) != 4:
            raise ValueError("The input_points must be a 4D tensor. Of shape `batch_size`, `point_batch_size`, "
                             f"`nb_points_per_image`, `2`. got {input_points.shape}.")
        if input_boxes is not None and len(input_boxes.shape) != 3:
            raise ValueError(f"The input_points must be a 3D tensor. Of shape `batch_size`, `nb_boxes`, `4`. got "
                             f"{input_boxes.shape}.")
        if input_points is not None and input_boxes is not None and input_points.shape[1] != input_boxes.shape[1]:
            raise ValueError("You should provide as many bounding boxes as input points per box. Got "
                             f"{input_points.shape[1]} and {input_boxes.shape[1]}.")
        if pixel_values is not None:
            emb = self.vision_encoder.forward_nhwc(pixel_values)
        else:
            B_, C_, H_, W_ = image_embeddings.shape
            emb = image_embeddings.permute(0, 2, 3, 1).reshape(B_, H_ * W_, C_).float().contiguous()
        if input_points is None and input_boxes is None:
            # prompt-free decoding (hf SamPromptEncoder: no sparse embeddings, SamMaskDecoder: the 5 output tokens
            # alone, point batch 1): every image gets the iou / mask tokens only
            md = self.mask_decoder
            tokens = md.output_tokens_f32().reshape(1, 1, 5, 256).expand(emb.shape[0], 1, 5, 256).contiguous()
        else:
            tokens = self.prompt_tokens(input_points, input_labels, input_boxes)
        B, N = tokens.shape[:2]
        if emb.shape[0] != B:
            raise ValueError("The batch size of the image embeddings and the input points must be the same. ")
        if input_masks is not None:
            dense = self.prompt_encoder.mask_embed.forward_pixels(input_masks)  # [B, 4096, 256]
            if dense.shape[0] != B:
                raise ValueError("input_masks must have one mask per image")
        else:
            dense = self.prompt_encoder.no_mask_embed.weight
        masks, iou = self.mask_decoder.run(emb, self.image_pe(), tokens, dense, multimask_output,
                                           target_embedding=target_embedding,
                                           attention_similarity=attention_similarity)
        return SamImageSegmentationOutput(iou_scores=iou, pred_masks=masks)


_ALL_NAMES = set()
_WEIGHT_FILES = ("model.safetensors", "pytorch_model.bin")


def _hf_cache_dirs():
    import os
    out = []
    for var in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE"):
        if os.environ.get(var):
            out.append(os.environ[var])
    home = os.environ.get("HF_HOME") or os.path.join(os.path.expanduser("~"), ".cache", "huggingface")
    out.append(os.path.join(home, "hub"))
    return list(dict.fromkeys(out))


def _find_weights(name_or_path: str, searched: list) -> str | None:
    """Local weight file for a path or hub name (see SamModel.from_pretrained), or None."""
    import glob
    import os
    if os.path.isfile(name_or_path):
        return name_or_path
    if os.path.isdir(name_or_path):
        for f in _WEIGHT_FILES:
            cand = os.path.join(name_or_path, f)
            searched.append(cand)
            if os.path.isfile(cand):
                return cand
        return None
    if "/" in name_or_path:
        repo = "models--" + name_or_path.replace("/", "--")
        for root in _hf_cache_dirs():
            for f in _WEIGHT_FILES:
                pat = os.path.join(root, repo, "snapshots", "*", f)
                searched.append(pat)
                hits = sorted(glob.glob(pat))
                if hits:
                    return hits[-1]
    return None


def _names():
    from .config import PRESETS
    _ALL_NAMES.update(PRESETS)


_names()
